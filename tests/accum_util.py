"""Test helpers: the oracle's ProofShape -> the product's halo2_amd.ProofShape,
and packing of synthetic proofs (tests only)."""
import numpy as np

import accum as A
import halo2_amd as H
import pasta as P


def to_product_shape(curve_id, sh):
    C = P.CURVES[curve_id]
    return H.ProofShape(
        curve_id, log_n=sh.log_n, blinding_factors=sh.blinding_factors,
        num_instance_columns=sh.num_instance_columns, num_advice_columns=sh.num_advice_columns,
        num_fixed_columns=sh.num_fixed_columns, num_lookups=sh.num_lookups, perm_chunk_len=sh.perm_chunk_len,
        quotient_degree=sh.quotient_degree, instance_queries=sh.instance_queries,
        advice_queries=sh.advice_queries, fixed_queries=sh.fixed_queries, perm_columns=sh.perm_columns,
        gates=sh.gates, lookup_inputs=sh.lookup_inputs, lookup_tables=sh.lookup_tables, omega=sh.omega,
        delta=sh.delta, g1=np.array(P.point_to_limbs(C, C.gen), dtype=np.uint64),
        fixed_commitments=np.array([P.point_to_limbs(C, q) for q in sh.fixed_commitments], dtype=np.uint64),
        sigma_commitments=np.array([P.point_to_limbs(C, q) for q in sh.sigma_commitments], dtype=np.uint64))


SHAPES = {"simple": A.simple_example_shape, "rich": A.rich_shape}


def make_case(curve_id, shape_name, log_n, B, seed):
    C = P.CURVES[curve_id]
    sh = A.synth_vk_points(C, SHAPES[shape_name](C, log_n), seed=seed ^ 0x7EC)
    proofs = [A.synth_proof(C, sh, seed, b) for b in range(B)]
    return C, sh, proofs

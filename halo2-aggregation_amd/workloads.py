"""Synthetic workloads of the hot path, product side.

* simple-example proof shape: the reference's inner circuit
  (/root/reference/examples/simple-example.rs:99-159, 331-344; SURVEY.md
  Appendix B) as a halo2_amd.ProofShape -- the VerifyingKey view the Rust shim
  would pass.  VK commitments and proof points are synthetic curve points
  generated on the device (pm_synth_bases), scalars / challenges uniform in
  [0, r) (pm_synth_scalars).
* scalar-field constants used by the shape (halo2 EvaluationDomain omega and
  the field's DELTA), derived from the published 2-adic structure.
"""
from __future__ import annotations

import numpy as np

import halo2_amd as H

BASE_MODULUS = {
    H.PALLAS: 0x40000000000000000000000000000000224698FC094CF91B992D30ED00000001,
    H.VESTA: 0x40000000000000000000000000000000224698FC0994A8DD8C46EB2100000001,
    H.BN254: 21888242871839275222246405745257275088696311157297823662689037894645226208583,
}
# generator (x, y) canonical: pasta (p - 1, 2), bn254 (1, 2)
GENERATOR = {H.PALLAS: (BASE_MODULUS[H.PALLAS] - 1, 2), H.VESTA: (BASE_MODULUS[H.VESTA] - 1, 2), H.BN254: (1, 2)}
# (multiplicative generator, 2-adicity S) of the scalar fields
TWO_ADIC = {H.PALLAS: (5, 32), H.VESTA: (5, 32), H.BN254: (7, 28)}

KIND_ADVICE, KIND_FIXED, KIND_INSTANCE = 0, 1, 2


def domain_omega(curve, k):
    r = H.SCALAR_MODULUS[curve]
    g, s = TWO_ADIC[curve]
    return pow(pow(g, (r - 1) >> s, r), 1 << (s - k), r)


def field_delta(curve):
    r = H.SCALAR_MODULUS[curve]
    g, s = TWO_ADIC[curve]
    return pow(g, 1 << s, r)


def generator_limbs(curve):
    p = BASE_MODULUS[curve]
    x, y = GENERATOR[curve]
    out = []
    for v in (x, y):
        v = v * (1 << 256) % p
        out += [(v >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)]
    return np.array(out, dtype=np.uint64)


def simple_example_args(curve, log_n):
    """Shape fields of the inner circuit (without VK commitments)."""
    gate = ("prod", ("fixed", 2), ("sum", ("prod", ("advice", 0), ("advice", 1)), ("neg", ("advice", 2))))
    return dict(log_n=log_n, blinding_factors=5, num_instance_columns=1, num_advice_columns=2,
                num_fixed_columns=4, num_lookups=1, perm_chunk_len=3, quotient_degree=4,
                instance_queries=[(0, 0)], advice_queries=[(0, 0), (1, 0), (0, 1)],
                fixed_queries=[(0, 0), (1, 0), (2, 0), (3, 0)],
                perm_columns=[(KIND_INSTANCE, 0), (KIND_FIXED, 0), (KIND_ADVICE, 0), (KIND_ADVICE, 1)],
                gates=[gate], lookup_inputs=[("prod", ("fixed", 3), ("advice", 0))], lookup_tables=[("fixed", 1)],
                omega=domain_omega(curve, log_n), delta=field_delta(curve))


def simple_example_shape(ctx, curve, log_n, seed=0x7EC):
    """ProofShape with VK commitments generated on ctx's device."""
    import torch

    args = simple_example_args(curve, log_n)
    nf, npc = args["num_fixed_columns"], len(args["perm_columns"])
    d = torch.empty((nf + npc, 8), dtype=torch.int64, device=torch.device("cuda", ctx.device))
    ctx.synth_bases(curve, seed, 0, nf + npc, d.data_ptr())
    vk = d.cpu().numpy().view(np.uint64)
    return H.ProofShape(curve, g1=generator_limbs(curve), fixed_commitments=vk[:nf], sigma_commitments=vk[nf:],
                        **args)


SYNTH_PINNED_VK = b"simple-example pinned verifying key (synthetic)"


class SyntheticBatch:
    """B shape-conformant proofs resident in HBM (points [a]G on the device;
    scalars uniform), plus output buffers.  With ``transcript`` (default) the
    challenges are replayed from the Blake2b transcript on the device
    (pm_accum_batch_transcript_device); otherwise they are drawn uniformly."""

    def __init__(self, ctx, shape, B, seed=0xACC, i0=0):
        import torch

        self.B = B
        npts, nsc, _ = shape.layout()
        dev = torch.device("cuda", ctx.device)
        self.points = torch.empty((B, npts, 8), dtype=torch.int64, device=dev)
        self.scalars = torch.empty((B, nsc, 4), dtype=torch.int64, device=dev)
        self.challenges = torch.empty((B, 7, 4), dtype=torch.int64, device=dev)
        self.quads = torch.empty((B, 4, 8), dtype=torch.int64, device=dev)
        self.h_eval = torch.empty((B, 4), dtype=torch.int64, device=dev)
        self.status = torch.empty((B,), dtype=torch.int32, device=dev)
        c = shape.curve
        self.vk_repr = H.vk_transcript_repr(c, SYNTH_PINNED_VK)
        ctx.synth_bases(c, seed, i0 * npts, B * npts, self.points.data_ptr())
        ctx.synth_scalars(c, seed ^ 0x5CA1A, i0 * nsc, B * nsc, self.scalars.data_ptr())
        ctx.synth_scalars(c, seed ^ 0xC4A1, i0 * 7, B * 7, self.challenges.data_ptr())
        torch.cuda.synchronize()

    def to_proof_bytes(self, shape):
        """Serialize the batch the way halo2's Blake2bWrite wrote it (the
        verifier's read order, include/pasta_msm.h "Proof bytes"): proof
        points compressed (canonical x, y parity in bit 255), scalars
        canonical, W_j last; instance commitments stay separate.  Host-side,
        untimed.  Sets self.proofs (B, psize) u8 and self.inst on the device."""
        import torch

        npts, nsc, nsets = shape.layout()
        ni = shape.c.num_instance_columns
        c = shape.curve
        p, r = BASE_MODULUS[c], H.SCALAR_MODULUS[c]
        rinv_p, rinv_r = pow(1 << 256, -1, p), pow(1 << 256, -1, r)
        pts = self.points.cpu().numpy().view(np.uint64)
        scs = self.scalars.cpu().numpy().view(np.uint64)

        def val(limbs):
            return int(limbs[0]) | int(limbs[1]) << 64 | int(limbs[2]) << 128 | int(limbs[3]) << 192

        def enc_point(q):
            x, y = val(q[:4]) * rinv_p % p, val(q[4:]) * rinv_p % p
            return (x | (y & 1) << 255).to_bytes(32, "little")

        pW = npts - nsets
        out = bytearray()
        for b in range(self.B):
            for i in range(ni, pW):
                out += enc_point(pts[b, i])
            for k in range(nsc):
                out += (val(scs[b, k]) * rinv_r % r).to_bytes(32, "little")
            for j in range(nsets):
                out += enc_point(pts[b, pW + j])
        psize = len(out) // self.B
        assert psize == H.proof_size(shape)
        dev = self.points.device
        self.psize = psize
        self.proofs = torch.from_numpy(np.frombuffer(bytes(out), dtype=np.uint8).reshape(self.B, psize).copy()).to(dev)
        self.inst = self.points[:, :ni, :].contiguous()
        torch.cuda.synchronize()

    def run_bytes(self, ctx, shape):
        """One batch from its proof bytes: device decode (read_point /
        read_scalar) + transcript replay + accumulator
        (pm_accum_batch_proofs_device)."""
        ctx.accum_batch_proofs_device(shape, self.B, self.vk_repr, self.proofs.data_ptr(), self.psize,
                                      self.inst.data_ptr(), self.challenges.data_ptr(), self.quads.data_ptr(),
                                      self.h_eval.data_ptr(), self.status.data_ptr())

    def run(self, ctx, shape, transcript=True):
        if transcript:
            ctx.accum_batch_transcript_device(shape, self.B, self.vk_repr, self.points.data_ptr(),
                                              self.scalars.data_ptr(), self.challenges.data_ptr(),
                                              self.quads.data_ptr(), self.h_eval.data_ptr(), self.status.data_ptr())
        else:
            ctx.accum_batch_device(shape, self.B, self.points.data_ptr(), self.scalars.data_ptr(),
                                   self.challenges.data_ptr(), self.quads.data_ptr(), self.h_eval.data_ptr())

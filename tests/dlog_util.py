"""Known-discrete-log answer of the synthetic MSM inputs (tests only): the
device generators give P_i = [a_i]G with a_i = synth scalar (seed SEED_BASES,
index i), so sum_i s_i P_i = [sum_i s_i a_i mod r]G for any n."""
import numpy as np

import msm_ref
import pasta as P


def _to_int(L):
    L = L.astype(object)
    return L[:, 0] + (L[:, 1] << 64) + (L[:, 2] << 128) + (L[:, 3] << 192)


def known_dlog_point(curve, n, i0=0, seed_scalars=P.SEED_SCALARS, seed_bases=P.SEED_BASES):
    """[sum_{i0 <= i < i0 + n} s_i a_i]G as an oracle point."""
    C = P.CURVES[curve]
    S = msm_ref.synth_scalars(curve, seed_scalars, i0, n)   # Montgomery form
    A = msm_ref.synth_scalars(curve, seed_bases, i0, n)     # dlogs a_i (Montgomery)
    rinv = pow(P.R_MONT, -1, C.r)
    tot = 0
    for k in range(0, n, 1 << 16):  # sum s_i a_i in the R^2-scaled Montgomery domain
        ss = _to_int(S[k:k + (1 << 16)])
        aa = _to_int(A[k:k + (1 << 16)])
        tot += int(np.dot(ss, aa))
    tot = tot * rinv * rinv % C.r
    # a_i == 0 maps to 1 in the generator; never happens for these seeds
    return C.mul(tot, C.gen)

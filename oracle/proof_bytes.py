"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the proof-byte boundary.

Checker for ``k_proof_decode`` (halo2-aggregation_amd/csrc/proof_kernels.hpp)
and ``pm_accum_batch_proofs*`` / ``pm_decode_proofs*``.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it; the product library never does.

The reference verifier reads every commitment and evaluation of an inner proof
from halo2's serialized byte transcript (``self.transcript``, a
``Blake2bRead``): ``t.read_point()`` at src/verifier.rs:370, src/lookup.rs:64-65,96,
src/permutation.rs:67, src/vanishing.rs:67,94, src/multiopen.rs:210 (via
``read_comm``), and ``t.read_scalar()`` at src/verifier.rs:443,456,469,
src/vanishing.rs:122, src/permutation.rs:100-107,163, src/lookup.rs:124-128.
Any error there propagates with ``?`` (map_err(TranscriptError)): the
verifier aborts.  What it restates [3P: halo2 fork kzg-agg2 transcript.rs,
pasta_curves / pairing_bn256 GroupEncoding + PrimeField, not vendored]:

  * point encoding (``GroupEncoding::to_bytes``, what ``Blake2bWrite::write_point``
    emits): the canonical little-endian x, with the parity of the canonical y
    in bit 7 of byte 31 (the top bit; both base fields are < 2^255); the
    identity is 32 zero bytes.
  * ``from_bytes`` (``read_point``): ysign = bit 255, cleared; x must be
    canonical (< p) else error; x == 0 and ysign == 0 -> the identity; else
    y = sqrt(x^3 + b) (error when x^3 + b is a non-residue) and y is replaced
    by -y when its parity differs from ysign.  ``read_point`` then calls the
    reader's ``common_point``, which errors on the identity ("cannot write
    points at infinity to the transcript"), so an identity encoding is an
    error too.
  * scalar encoding (``to_repr``): the canonical little-endian 32 bytes;
    ``from_repr`` (``read_scalar``) errors unless the integer is < r.
  * byte layout of one proof = the verifier's read order (oracle/accum.py
    layout without the instance commitments, which come from the instance
    column, verifier.rs:312-316): advice, per lookup (A', S'), permutation
    Z_p, per lookup Z, vanishing r, h_0..h_{d-1} (points); every scalar of
    the accumulator layout in order; then the multiopen witnesses W_j
    (read after v and u are squeezed, multiopen.rs:392 -> :202-218).

A proof whose bytes fail any read gets a status bit (the reference aborts);
its decoded slot holds the identity (point) or 0 (scalar).
PARITY STATUS: the encodings follow the published crates; the reference holds
no proof fixtures (src/lib.rs:43-44), so this is **parity unpinned** beyond
the restatement (round trips, and the on-curve / canonical checks below).
"""
from __future__ import annotations

import pasta as P

STATUS_BAD_POINT = 8    # PM_PROOF_BAD_POINT: read_point failed
STATUS_BAD_SCALAR = 16  # PM_PROOF_BAD_SCALAR: read_scalar failed


def sqrt_mod(a, p):
    """A square root of a mod p, or None (Tonelli-Shanks; which root comes
    back does not matter: from_bytes fixes the sign)."""
    a %= p
    if a == 0:
        return 0
    if pow(a, (p - 1) // 2, p) != 1:
        return None
    if p % 4 == 3:
        return pow(a, (p + 1) // 4, p)
    s, t = 0, p - 1
    while t % 2 == 0:
        s, t = s + 1, t // 2
    z = 2
    while pow(z, (p - 1) // 2, p) != p - 1:
        z += 1
    m, c, x, b = s, pow(z, t, p), pow(a, (t + 1) // 2, p), pow(a, t, p)
    while b != 1:
        i, bb = 0, b
        while bb != 1:
            bb, i = bb * bb % p, i + 1
        g = pow(c, 1 << (m - i - 1), p)
        m, c, x, b = i, g * g % p, x * g % p, b * g * g % p
    return x


def encode_point(curve, pt):
    if pt is None:
        return bytes(32)
    x, y = pt
    v = x | ((y & 1) << 255)
    return v.to_bytes(32, "little")


def decode_point(curve, data):
    """-> (ok, point): from_bytes + the reader's common_point (identity fails)."""
    v = int.from_bytes(data, "little")
    ysign = v >> 255
    x = v & ((1 << 255) - 1)
    p = curve.p
    if x >= p:
        return False, None
    if x == 0 and ysign == 0:
        return False, None          # the identity: common_point errors
    y = sqrt_mod(x * x * x + curve.b, p)
    if y is None:
        return False, None
    if (y & 1) != ysign:
        y = (-y) % p
    return True, (x, y)


def encode_scalar(r, s):
    return (s % r).to_bytes(32, "little")


def decode_scalar(r, data):
    v = int.from_bytes(data, "little")
    return (v < r), (v if v < r else 0)


def proof_items(shape):
    """[(kind, index)] in byte order: kind "pt" indexes the accumulator point
    layout, "sc" the scalar layout."""
    po = shape.point_offsets()
    items = []
    for name in ("adv", "lk_perm", "perm_z", "lk_z", "rand", "h"):
        k, n = po[name]
        items += [("pt", k + i) for i in range(n)]
    items += [("sc", i) for i in range(shape.scalars_per_proof())]
    k, n = po["W"]
    items += [("pt", k + i) for i in range(n)]
    return items


def proof_size(shape):
    return 32 * len(proof_items(shape))


def serialize(curve, shape, pf):
    """accum.Proof -> the proof bytes (instance commitments are not in them)."""
    out = bytearray()
    for kind, i in proof_items(shape):
        out += encode_point(curve, pf.points[i]) if kind == "pt" else encode_scalar(curve.r, pf.scalars[i])
    return bytes(out)


def parse(curve, shape, data, inst_points):
    """Proof bytes (+ the instance commitments) -> (points, scalars, status)."""
    npts, nsc = shape.points_per_proof(), shape.scalars_per_proof()
    points, scalars = [None] * npts, [0] * nsc
    k0, ni = shape.point_offsets()["inst"]
    for i in range(ni):
        points[k0 + i] = inst_points[i]
    status = 0
    for j, (kind, i) in enumerate(proof_items(shape)):
        chunk = data[32 * j:32 * j + 32]
        if kind == "pt":
            ok, pt = decode_point(curve, chunk)
            points[i] = pt
            status |= 0 if ok else STATUS_BAD_POINT
        else:
            ok, s = decode_scalar(curve.r, chunk)
            scalars[i] = s
            status |= 0 if ok else STATUS_BAD_SCALAR
    return points, scalars, status


def self_check():
    """sqrt_mod on both pasta fields and BN254 Fq; encode / decode round trip
    of each generator and its negation."""
    for C in (P.PALLAS, P.VESTA, P.BN254):
        for a in (1, 4, 9, C.b, 123456789):
            y = sqrt_mod(a, C.p)
            assert y is None or y * y % C.p == a % C.p
        g = C.gen
        for pt in (g, C.neg(g)):
            assert decode_point(C, encode_point(C, pt)) == (True, pt)
    return True

"""TEST INFRASTRUCTURE ONLY -- CPU oracle for the verifier's Blake2b transcript.

Checker for ``k_transcript`` (halo2-aggregation_amd/csrc/transcript_kernels.hpp)
and ``pm_vk_transcript_repr``.  Only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.

What it restates:

  * ``Blake2bTranscript``  halo2's ``Blake2bWrite<_, C, Challenge255<C>>`` as
    TranscriptChip drives it (/root/reference/src/transcript.rs:57-145) [3P:
    halo2 ``transcript.rs``, branch kzg-agg2, not vendored]: BLAKE2b-512 with
    personalisation ``Halo2-Transcript``; point = 0x01 || x || y and scalar =
    0x02 || s (canonical little-endian 32-byte reprs); squeeze = absorb 0x00,
    finalise a copy, read the digest as a little-endian 512-bit integer mod r
    (Challenge255 / from_bytes_wide).  TranscriptChip::common_point returns
    Err(Error::Synthesis) for the identity (C::from_xy(0, 0) fails,
    transcript.rs:101-110) before hashing, so the identity is never hashed.
    Every call site drops that error (lookup.rs:72-73, vanishing.rs:71,98,
    verifier.rs:362,375, permutation.rs:74) except the lookup product
    commitment Z (lookup.rs:100 propagates it with `?`: the verifier circuit
    aborts).  The replay reports both as status bits (STATUS_IDENTITY_SKIPPED,
    STATUS_LOOKUP_Z_IDENTITY; include/pasta_msm.h).
  * ``vk_repr``            src/verifier.rs:341-358: BLAKE2b-512 with
    personalisation ``Halo2-Verify-Key`` over le_u64(len) || debug string,
    reduced with from_bytes_wide.
  * ``replay_challenges``  the absorb / squeeze order of
    VerifierChip::_verify_proof (src/verifier.rs:341-719; lookup.rs:59-160,
    permutation.rs:62-182, vanishing.rs:54-135).

BLAKE2b itself is Python's ``hashlib.blake2b`` (RFC 7693); tests check it on
the RFC's published "abc" vector.  PARITY STATUS: the framing (prefix bytes,
byte order, wide reduction) follows the published halo2 source; the reference
ships no transcript test vectors, so the framing is **parity unpinned** beyond
that restatement.
"""
from __future__ import annotations

import hashlib

TRANSCRIPT_PERSONAL = b"Halo2-Transcript"
VERIFY_KEY_PERSONAL = b"Halo2-Verify-Key"
PREFIX_CHALLENGE, PREFIX_POINT, PREFIX_SCALAR = 0, 1, 2
CHALLENGE_NAMES = ("theta", "beta", "gamma", "y", "x", "v", "u")
STATUS_IDENTITY_SKIPPED = 1     # PM_TRANSCRIPT_IDENTITY_SKIPPED
STATUS_LOOKUP_Z_IDENTITY = 2    # PM_TRANSCRIPT_LOOKUP_Z_IDENTITY


class Blake2bTranscript:
    def __init__(self, r):
        self.r = r
        self.state = hashlib.blake2b(digest_size=64, person=TRANSCRIPT_PERSONAL)
        self.status = 0

    def common_point(self, pt, lookup_z=False):
        if pt is None:                      # transcript.rs:101-110: Err(Synthesis)
            self.status |= STATUS_IDENTITY_SKIPPED
            if lookup_z:                    # lookup.rs:100 propagates it
                self.status |= STATUS_LOOKUP_Z_IDENTITY
            return
        x, y = pt
        self.state.update(bytes([PREFIX_POINT]) + x.to_bytes(32, "little") + y.to_bytes(32, "little"))

    def common_scalar(self, s):
        self.state.update(bytes([PREFIX_SCALAR]) + (s % self.r).to_bytes(32, "little"))

    def squeeze_challenge(self):
        self.state.update(bytes([PREFIX_CHALLENGE]))
        return int.from_bytes(self.state.copy().digest(), "little") % self.r


def vk_repr(r, pinned: bytes):
    """verifier.rs:341-358"""
    h = hashlib.blake2b(digest_size=64, person=VERIFY_KEY_PERSONAL)
    h.update(len(pinned).to_bytes(8, "little"))
    h.update(pinned)
    return int.from_bytes(h.digest(), "little") % r


def replay_challenges(curve, shape, pf, vkr):
    """-> ([theta, beta, gamma, y, x, v, u], status bits) for one proof in
    the accumulator layout (oracle/accum.py docstring); status 0 = clean."""
    t = Blake2bTranscript(curve.r)
    po = shape.point_offsets()

    def pts(name):
        k, n = po[name]
        for q in pf.points[k:k + n]:
            t.common_point(q, lookup_z=(name == "lk_z"))

    t.common_scalar(vkr)                    # verifier.rs:341-358
    pts("inst")                             # :360-363
    pts("adv")                              # :365-376
    theta = t.squeeze_challenge()           # :378
    pts("lk_perm")                          # :381-387 (A', S' per lookup)
    beta = t.squeeze_challenge()            # :390
    gamma = t.squeeze_challenge()           # :393
    pts("perm_z")                           # :402-409
    pts("lk_z")                             # :411-417
    pts("rand")                             # :419-421
    y = t.squeeze_challenge()               # :423
    pts("h")                                # :425-434
    x = t.squeeze_challenge()               # :436
    for s in pf.scalars:                    # :438-509, layout == read order
        t.common_scalar(s)
    v = t.squeeze_challenge()               # :718
    u = t.squeeze_challenge()               # :719
    return [theta, beta, gamma, y, x, v, u], t.status


def with_replayed_challenges(curve, shape, proofs, vkr):
    """Replace each proof's challenges by the transcript's (in place)."""
    for pf in proofs:
        pf.challenges, _ = replay_challenges(curve, shape, pf, vkr)
    return proofs

// transcript_kernels.hpp -- batched replay of the verifier's Blake2b
// transcript: B proofs -> B x 7 challenges (theta, beta, gamma, y, x, v, u).
//
// The reference squeezes every challenge from TranscriptChip
// (/root/reference/src/transcript.rs:63-145), a halo2 `Blake2bWrite` with
// `Challenge255` encoding [3P].  Its absorb sequence is fixed by the
// verifier's read order (src/verifier.rs:341-719):
//   common_scalar(vk_repr)                         verifier.rs:341-358
//   instance commitments, advice commitments        :361-376
//   squeeze theta                                   :378
//   per lookup (A', S')                             :381-387, lookup.rs:59-73
//   squeeze beta, gamma                             :390-393
//   permutation Z_p (all chunks)                    :402-409, permutation.rs:62-75
//   per lookup Z                                    :411-417, lookup.rs:93-102
//   vanishing random commitment r                   :419-421, vanishing.rs:54-75
//   squeeze y                                       :423
//   quotient pieces h_i                             :427-434, vanishing.rs:77-107
//   squeeze x                                       :436
//   instance / advice / fixed evals, r(x)           :438-481, vanishing.rs:109-135
//   sigma evals, Z_p evals, lookup evals            :482-509 (permutation.rs:
//                                                   82-182, lookup.rs:104-160)
//   squeeze v, u                                    :718-719
// which is exactly the point / scalar layout of pm_accum_batch (the
// multiopen witnesses W_j come after the last squeeze and are not absorbed).
//
// halo2 transcript framing [3P]: point = 0x01 || x.to_repr() || y.to_repr(),
// scalar = 0x02 || s.to_repr() (canonical little-endian 32 bytes), squeeze =
// update(0x00) then finalise a copy of the state; the 64-byte digest is read
// as a little-endian 512-bit integer and reduced mod r
// (Challenge255::new -> from_bytes_wide).  TranscriptChip::common_point
// rejects the identity before touching the hash (C::from_xy(0, 0) fails,
// transcript.rs:101-110): such a point is skipped and flagged in `status`.
//
// One lane per proof; each lane's message buffer lives in LDS word-major
// ([word][lane]) so the compression's 32 word reads are conflict-free.  All
// lanes run the same absorb program, so block boundaries (and the
// compressions) stay wave-uniform unless a proof has an identity point.
#pragma once
#include "blake2b.hpp"
#include "curve.hpp"

namespace pm {

enum : uint32_t { kTrSqueeze = 0, kTrPoint = 1, kTrScalar = 2, kTrVk = 3 };
static constexpr uint32_t kTrChallenges = 7;
static constexpr uint32_t kTrStatusIdentity = 1;  // an identity point was skipped

struct TranscriptHdr {
  uint32_t B, npts, nsc, nprog;
  uint64_t h0[8];   // personalised initial chaining value
  uint32_t vk[8];   // vk_repr, canonical limbs
};

// from_bytes_wide: (lo + 2^256 hi) mod r, returned in Montgomery form.
// lo, hi < 2^256 = R, so each Montgomery product stays below 2r.
template <class Fs>
PM_HD Fe<Fs> fe_from_bytes_wide(const uint32_t d[16]) {
  Fe<Fs> lo, hi, r2;
  for (int i = 0; i < 8; i++) {
    lo.l[i] = d[i];
    hi.l[i] = d[8 + i];
    r2.l[i] = Fs::R2[i];
  }
  const Fe<Fs> r3 = fe_mul<Fs>(r2, r2);
  return fe_add<Fs>(fe_mul<Fs>(lo, r2), fe_mul<Fs>(hi, r3));
}

// Per-lane absorb state.  The message stream lives in a 256-byte circular
// buffer in LDS (two blocks, word-major [word][lane]); bytes are packed into
// whole words in a register first, so LDS sees only 32-bit stores.  The
// invariant between records is pos <= 128: a full block stays buffered until
// more data arrives (blake2b_simd's lazy compression), and the compression
// has a single call site in tr_settle().
struct TrLane {
  uint64_t h[8];
  uint64_t t;    // bytes compressed so far (multiple of 128)
  uint32_t pos;  // bytes buffered after t
  uint32_t acc;  // pending partial word (low `pos & 3` bytes valid)
};

__device__ __forceinline__ void tr_store(uint32_t (*buf)[64], uint32_t lane, uint32_t widx, uint32_t w) {
  buf[widx & 63][lane] = w;
}

__device__ __forceinline__ void tr_put_byte(TrLane& s, uint32_t (*buf)[64], uint32_t lane, uint32_t b) {
  const uint32_t a = (uint32_t)s.t + s.pos;
  const uint32_t k = a & 3;
  s.acc |= b << (8 * k);
  if (k == 3) {
    tr_store(buf, lane, a >> 2, s.acc);
    s.acc = 0;
  }
  s.pos++;
}

__device__ __forceinline__ void tr_put_word(TrLane& s, uint32_t (*buf)[64], uint32_t lane, uint32_t w) {
  const uint32_t a = (uint32_t)s.t + s.pos;
  const uint32_t k = a & 3;
  if (k == 0) {
    tr_store(buf, lane, a >> 2, w);
  } else {
    tr_store(buf, lane, a >> 2, s.acc | (w << (8 * k)));
    s.acc = w >> (32 - 8 * k);
  }
  s.pos += 4;
}

// Compress every full block that more data has arrived after; with `squeeze`
// also finalise a copy of the state and return the digest in d.
__device__ __forceinline__ void tr_settle(TrLane& s, uint32_t (*buf)[64], uint32_t lane, bool squeeze, uint32_t d[16]) {
  for (;;) {
    const bool flush = s.pos > 128;
    const bool fin = !flush && squeeze;
    if (!flush && !fin) return;
    const uint32_t a = (uint32_t)s.t + s.pos;
    if (fin && (a & 3)) tr_store(buf, lane, a >> 2, s.acc);  // partial word, zero above pos
    const uint32_t w0 = ((uint32_t)s.t & 255) >> 2;
    uint64_t m[16], hh[8];
#pragma unroll
    for (int i = 0; i < 16; i++)
      m[i] = (uint64_t)buf[(w0 + 2 * i) & 63][lane] | ((uint64_t)buf[(w0 + 2 * i + 1) & 63][lane] << 32);
    if (fin) {
#pragma unroll
      for (int i = 0; i < 16; i++) {
        const uint32_t lo = 8u * i;
        m[i] &= s.pos >= lo + 8 ? ~0ull : s.pos <= lo ? 0ull : ((1ull << (8 * (s.pos - lo))) - 1);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; i++) hh[i] = s.h[i];
    blake2b_compress(hh, m, fin ? s.t + s.pos : s.t + 128, fin);
    if (fin) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        d[2 * i] = (uint32_t)hh[i];
        d[2 * i + 1] = (uint32_t)(hh[i] >> 32);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < 8; i++) s.h[i] = hh[i];
    s.t += 128;
    s.pos -= 128;
  }
}

// Montgomery -> canonical for every point coordinate and scalar of the batch,
// one lane per field element (B (2 npts + nsc) lanes), so the transcript's
// serial chain only hashes: pts_out / scs_out have the layout of the inputs.
template <class Cv>
__global__ void __launch_bounds__(256) k_tr_canon(uint32_t B, uint32_t npts, uint32_t nsc,
                                                  const uint32_t* __restrict__ points,
                                                  const uint32_t* __restrict__ scalars,
                                                  uint32_t* __restrict__ pts_out, uint32_t* __restrict__ scs_out) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t ncoord = (size_t)B * 2 * npts, nall = ncoord + (size_t)B * nsc;
  if (e >= nall) return;
  if (e < ncoord) {
    const Fe<F> v = load_fe4<F>(reinterpret_cast<const uint4*>(points + 8 * e));
    store_fe4<F>(reinterpret_cast<uint4*>(pts_out + 8 * e), fe_from_mont<F>(v));
  } else {
    const size_t k = e - ncoord;
    const Fe<Fs> v = load_fe4<Fs>(reinterpret_cast<const uint4*>(scalars + 8 * k));
    store_fe4<Fs>(reinterpret_cast<uint4*>(scs_out + 8 * k), fe_from_mont<Fs>(v));
  }
}

// points / scalars: canonical (k_tr_canon).  The next record's words are
// loaded one record ahead (the record index comes from the uniform program,
// so the address is known early) to hide the global-load latency.
template <class Cv>
__global__ void __launch_bounds__(64) k_transcript(TranscriptHdr hd, const uint32_t* __restrict__ prog,
                                                   const uint32_t* __restrict__ points,
                                                   const uint32_t* __restrict__ scalars,
                                                   uint32_t* __restrict__ challenges, uint32_t* __restrict__ status) {
  using Fs = typename Cv::Scalar;
  __shared__ uint32_t buf[64][64];
  const uint32_t lane = threadIdx.x;
  const uint32_t b = blockIdx.x * 64 + lane;
  if (b >= hd.B) return;
  TrLane s;
#pragma unroll
  for (int i = 0; i < 8; i++) s.h[i] = hd.h0[i];
  s.t = 0;
  s.pos = 0;
  s.acc = 0;
  uint32_t st = 0;
  const uint32_t* pts = points + 16ull * hd.npts * b;
  const uint32_t* scs = scalars + 8ull * hd.nsc * b;
  uint32_t d[16];
  auto fetch = [&](uint32_t k, uint32_t w[16]) {
    const uint32_t op = k < hd.nprog ? prog[k] : 0u;
    const uint32_t kind = op >> 24, idx = op & 0xffffffu;
    const uint32_t* src = kind == kTrPoint ? pts + 16 * idx : kind == kTrScalar ? scs + 8 * idx : pts;
    const uint32_t nw = kind == kTrPoint ? 16 : kind == kTrScalar ? 8 : 0;
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)i < nw ? src[i] : 0u;
  };
  uint32_t cur[16], nxt[16];
  fetch(0, cur);
  for (uint32_t k = 0; k < hd.nprog; k++) {
    const uint32_t op = prog[k];
    const uint32_t kind = op >> 24, idx = op & 0xffffffu;
    fetch(k + 1, nxt);
    if (kind == kTrPoint) {
      uint32_t z = 0;
#pragma unroll
      for (int i = 0; i < 16; i++) z |= cur[i];
      if (z == 0) {
        st |= kTrStatusIdentity;
      } else {
        tr_put_byte(s, buf, lane, 1);
#pragma unroll
        for (int i = 0; i < 16; i++) tr_put_word(s, buf, lane, cur[i]);
      }
    } else if (kind == kTrScalar || kind == kTrVk) {
      tr_put_byte(s, buf, lane, 2);
#pragma unroll
      for (int i = 0; i < 8; i++) tr_put_word(s, buf, lane, kind == kTrVk ? hd.vk[i] : cur[i]);
    } else {
      tr_put_byte(s, buf, lane, 0);
    }
    // one compression site for every record kind
    const bool squeeze = kind == kTrSqueeze;
    tr_settle(s, buf, lane, squeeze, d);
    if (squeeze) {
      const Fe<Fs> c = fe_from_bytes_wide<Fs>(d);
      uint32_t* out = challenges + 8ull * (kTrChallenges * b + idx);
#pragma unroll
      for (int i = 0; i < 8; i++) out[i] = c.l[i];
    }
#pragma unroll
    for (int i = 0; i < 16; i++) cur[i] = nxt[i];
  }
  if (status) status[b] = st;
}

}  // namespace pm

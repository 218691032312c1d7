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
// Four lanes per proof (see TrLane); each proof's message buffer lives in
// LDS.  All proofs run the same absorb program, so block boundaries (and the
// compressions) stay wave-uniform unless a proof has an identity point.
#pragma once
#include "blake2b.hpp"
#include "curve.hpp"

namespace pm {

enum : uint32_t { kTrSqueeze = 0, kTrPoint = 1, kTrScalar = 2, kTrVk = 3 };
static constexpr uint32_t kTrChallenges = 7;
static constexpr uint32_t kTrStatusIdentity = 1;  // an identity point was skipped
// the skipped identity was a lookup product commitment Z: the reference's
// common_point error propagates there (lookup.rs:100 `?`), so the in-circuit
// verifier aborts; elsewhere the error is dropped (lookup.rs:72-73, ...)
static constexpr uint32_t kTrStatusLookupZIdentity = 2;
// point-op flag (bit 23 of the op's index field): this point is a lookup Z
static constexpr uint32_t kTrLookupZFlag = 1u << 23;

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

// Each proof's transcript is run by the 4 lanes of a quad (16 proofs per
// 64-lane block).  The absorb bookkeeping is repeated by all 4 lanes; the
// compression is split by column: lane q holds column q of the working state
// (v[q], v[4+q], v[8+q], v[12+q]) and of the chaining value (h[q], h[4+q]),
// runs one G per half round, and the diagonal half round is reached by
// rotating b, c, d by 1, 2, 3 lanes inside the quad (DPP quad_perm, no LDS).
// A compression is then 12 x 2 G steps per lane instead of 12 x 8: the
// single-lane form was bound by its ~2 K dependent VALU instructions.
//
// The message stream lives in a 256-byte circular buffer in LDS (two blocks,
// 64-bit-word-major [w64][slot]); bytes are packed into whole 32-bit words in
// a register first.  The invariant between records is pos <= 128: a full
// block stays buffered until more data arrives (blake2b_simd's lazy
// compression), and the compression has a single call site in tr_settle().
constexpr uint32_t kTrSlots = 16;  // proofs per 64-lane block

struct TrLane {
  uint64_t h0, h1;  // h[q], h[4 + q]
  uint64_t t;       // bytes compressed so far (multiple of 128)
  uint32_t pos;     // bytes buffered after t
  uint32_t acc;     // pending partial word (low `pos & 3` bytes valid)
};
typedef uint64_t TrBuf[32][kTrSlots];

// all 4 lanes of the quad store the same word to the same address
__device__ __forceinline__ void tr_store(TrBuf& buf, uint32_t slot, uint32_t widx, uint32_t w) {
  reinterpret_cast<uint32_t*>(&buf[(widx >> 1) & 31][slot])[widx & 1] = w;
}

__device__ __forceinline__ void tr_put_byte(TrLane& s, TrBuf& buf, uint32_t slot, uint32_t b) {
  const uint32_t a = (uint32_t)s.t + s.pos;
  const uint32_t k = a & 3;
  s.acc |= b << (8 * k);
  if (k == 3) {
    tr_store(buf, slot, a >> 2, s.acc);
    s.acc = 0;
  }
  s.pos++;
}

__device__ __forceinline__ void tr_put_word(TrLane& s, TrBuf& buf, uint32_t slot, uint32_t w) {
  const uint32_t a = (uint32_t)s.t + s.pos;
  const uint32_t k = a & 3;
  if (k == 0) {
    tr_store(buf, slot, a >> 2, w);
  } else {
    tr_store(buf, slot, a >> 2, s.acc | (w << (8 * k)));
    s.acc = w >> (32 - 8 * k);
  }
  s.pos += 4;
}

// lane i of the quad receives x from lane P[i]
template <int CTRL>
__device__ __forceinline__ uint64_t tr_qperm(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)x, CTRL, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(x >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
constexpr int kQRot1 = 1 | 2 << 2 | 3 << 4 | 0 << 6;  // from lane q + 1
constexpr int kQRot2 = 2 | 3 << 2 | 0 << 4 | 1 << 6;  // from lane q + 2
constexpr int kQRot3 = 3 | 0 << 2 | 1 << 4 | 2 << 6;  // from lane q + 3

// sigma rows of RFC 7693 §2.7, packed per half round: nibble q of COL is
// sigma[2q] (the x word of column G q), of COLY sigma[2q+1]; DIAG / DIAGY the
// same for the diagonal G's (sigma[8 + 2q], sigma[9 + 2q]).
struct TrSigma {
  uint16_t colx, coly, diagx, diagy;
};
__host__ __device__ constexpr TrSigma tr_sigma_pack(const int (&r)[16]) {
  return TrSigma{(uint16_t)(r[0] | r[2] << 4 | r[4] << 8 | r[6] << 12),
                 (uint16_t)(r[1] | r[3] << 4 | r[5] << 8 | r[7] << 12),
                 (uint16_t)(r[8] | r[10] << 4 | r[12] << 8 | r[14] << 12),
                 (uint16_t)(r[9] | r[11] << 4 | r[13] << 8 | r[15] << 12)};
}
constexpr int kB2Sigma[10][16] = {{0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
                                  {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
                                  {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
                                  {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
                                  {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
                                  {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
                                  {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
                                  {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
                                  {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
                                  {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

#define PM_B2_GQ(a, b, c, d, x, y) \
  do {                             \
    a = a + b + (x);               \
    d = PM_B2_ROT(d ^ a, 32);         \
    c = c + d;                     \
    b = PM_B2_ROT(b ^ c, 24);         \
    a = a + b + (y);               \
    d = PM_B2_ROT(d ^ a, 16);         \
    c = c + d;                     \
    b = PM_B2_ROT(b ^ c, 63);         \
  } while (0)

// message readers of the compression: word i (< 16) of the block
struct TrRingMsg {  // the per-record path's 256-byte ring (TrBuf)
  const TrBuf& buf;
  uint32_t slot, w0;
  __device__ __forceinline__ uint64_t operator()(uint32_t i) const { return buf[(w0 + i) & 31][slot]; }
};
struct TrStreamMsg {  // the streamed path's LDS stream ([w64][kTrSlots], this slot's column)
  const uint64_t* col;
  uint32_t w0;
  __device__ __forceinline__ uint64_t operator()(uint32_t i) const { return col[(w0 + i) * kTrSlots]; }
};

// F(h, m, t, f) of RFC 7693 §3.2 by the quad: lane q updates h[q] and h[4 + q].
template <int R, class Msg>
__device__ __forceinline__ void tr_round_q(uint64_t& a, uint64_t& b, uint64_t& c, uint64_t& d, const Msg& msg,
                                           uint32_t q4) {
  constexpr TrSigma S = tr_sigma_pack(kB2Sigma[R % 10]);
  const uint64_t x0 = msg((S.colx >> q4) & 15);
  const uint64_t y0 = msg((S.coly >> q4) & 15);
  const uint64_t x1 = msg((S.diagx >> q4) & 15);
  const uint64_t y1 = msg((S.diagy >> q4) & 15);
  PM_B2_GQ(a, b, c, d, x0, y0);
  b = tr_qperm<kQRot1>(b);
  c = tr_qperm<kQRot2>(c);
  d = tr_qperm<kQRot3>(d);
  PM_B2_GQ(a, b, c, d, x1, y1);
  b = tr_qperm<kQRot3>(b);
  c = tr_qperm<kQRot2>(c);
  d = tr_qperm<kQRot1>(d);
}
#undef PM_B2_GQ

template <class Msg>
__device__ __forceinline__ void tr_compress_q(uint64_t& h0, uint64_t& h1, const Msg& msg, uint32_t q, uint64_t tcount,
                                              bool last) {
  const uint64_t iv_c = q == 0 ? Blake2bIV::v[0] : q == 1 ? Blake2bIV::v[1] : q == 2 ? Blake2bIV::v[2]
                                                                                      : Blake2bIV::v[3];
  const uint64_t iv_d = q == 0 ? Blake2bIV::v[4] : q == 1 ? Blake2bIV::v[5] : q == 2 ? Blake2bIV::v[6]
                                                                                      : Blake2bIV::v[7];
  uint64_t a = h0, b = h1, c = iv_c, d = iv_d;
  if (q == 0) d ^= tcount;    // v12 ^= t
  if (q == 2 && last) d = ~d;  // v14 = ~v14
  const uint32_t q4 = 4 * q;
  tr_round_q<0>(a, b, c, d, msg, q4);
  tr_round_q<1>(a, b, c, d, msg, q4);
  tr_round_q<2>(a, b, c, d, msg, q4);
  tr_round_q<3>(a, b, c, d, msg, q4);
  tr_round_q<4>(a, b, c, d, msg, q4);
  tr_round_q<5>(a, b, c, d, msg, q4);
  tr_round_q<6>(a, b, c, d, msg, q4);
  tr_round_q<7>(a, b, c, d, msg, q4);
  tr_round_q<8>(a, b, c, d, msg, q4);
  tr_round_q<9>(a, b, c, d, msg, q4);
  tr_round_q<10>(a, b, c, d, msg, q4);
  tr_round_q<11>(a, b, c, d, msg, q4);
  h0 ^= a ^ c;
  h1 ^= b ^ d;
}

// the 64-byte digest of the quad's state: word 2i, 2i + 1 = h[i], h[K] is
// lane K's h0, h[4 + K] its h1 (all 4 lanes receive all 16 words)
__device__ __forceinline__ void tr_digest_q(uint64_t h0, uint64_t h1, uint32_t d[16]) {
#define PM_TR_BC(K)                                                                                            \
  d[2 * K] = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)h0, K * 0x55, 0xF, 0xF, false);                 \
  d[2 * K + 1] = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(h0 >> 32), K * 0x55, 0xF, 0xF, false);     \
  d[2 * K + 8] = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)h1, K * 0x55, 0xF, 0xF, false);             \
  d[2 * K + 9] = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(h1 >> 32), K * 0x55, 0xF, 0xF, false);
  PM_TR_BC(0)
  PM_TR_BC(1)
  PM_TR_BC(2)
  PM_TR_BC(3)
#undef PM_TR_BC
}

// Compress every full block that more data has arrived after; with `squeeze`
// finalise (the buffered tail zero-padded) and return the digest in d (all
// 4 lanes) without advancing the state.
__device__ __forceinline__ void tr_settle(TrLane& s, TrBuf& buf, uint32_t slot, uint32_t q, bool squeeze,
                                          uint32_t d[16]) {
  for (;;) {
    const bool flush = s.pos > 128;
    const bool fin = !flush && squeeze;
    if (!flush && !fin) return;
    const uint32_t a = (uint32_t)s.t + s.pos;
    const uint32_t wd0 = ((uint32_t)s.t & 255) >> 2;  // first 32-bit word of the block
    if (fin) {
      if (a & 3) tr_store(buf, slot, a >> 2, s.acc);  // partial word, zero above pos
      const uint32_t z0 = (s.pos + 3) >> 2;
#pragma unroll
      for (uint32_t j = 0; j < 32; j++)
        if (j >= z0) tr_store(buf, slot, wd0 + j, 0u);
    }
    TrLane n = s;
    tr_compress_q(n.h0, n.h1, TrRingMsg{buf, slot, wd0 >> 1}, q, fin ? s.t + s.pos : s.t + 128, fin);
    if (fin) {
      tr_digest_q(n.h0, n.h1, d);
      return;
    }
    s.h0 = n.h0;
    s.h1 = n.h1;
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

// The per-record replay of one proof by its quad (points / scalars canonical,
// k_tr_canon).  Records' words are loaded three records ahead (the record
// index comes from the uniform program, so the address is known early) to
// hide the global-load latency.  A quad always runs (and exits) together, as
// the DPP exchanges in the compression require.  Returns the status bits.
template <class Cv>
__device__ uint32_t tr_replay(const TranscriptHdr& hd, const uint32_t* __restrict__ prog,
                              const uint32_t* __restrict__ points, const uint32_t* __restrict__ scalars,
                              uint32_t* __restrict__ challenges, TrBuf& buf, uint32_t slot, uint32_t q, uint32_t b) {
  using Fs = typename Cv::Scalar;
  TrLane s;
  s.h0 = q == 0 ? hd.h0[0] : q == 1 ? hd.h0[1] : q == 2 ? hd.h0[2] : hd.h0[3];
  s.h1 = q == 0 ? hd.h0[4] : q == 1 ? hd.h0[5] : q == 2 ? hd.h0[6] : hd.h0[7];
  s.t = 0;
  s.pos = 0;
  s.acc = 0;
  // from_bytes_wide split over the quad: lane 0 computes lo R^2, lane 1 hi R^3
  Fe<Fs> kq;
  {
    Fe<Fs> r2;
#pragma unroll
    for (int i = 0; i < 8; i++) r2.l[i] = Fs::R2[i];
    const Fe<Fs> r3 = fe_mul<Fs>(r2, r2);
#pragma unroll
    for (int i = 0; i < 8; i++) kq.l[i] = (q & 1) ? r3.l[i] : r2.l[i];
  }
  uint32_t st = 0;
  const uint32_t* pts = points + 16ull * hd.npts * b;
  const uint32_t* scs = scalars + 8ull * hd.nsc * b;
  uint32_t d[16];
  auto fetch = [&](uint32_t k, uint32_t w[16]) {
    const uint32_t op = k < hd.nprog ? prog[k] : 0u;
    const uint32_t kind = op >> 24, idx = op & (kTrLookupZFlag - 1u);
    const uint32_t* src = kind == kTrPoint ? pts + 16 * idx : kind == kTrScalar ? scs + 8 * idx : pts;
    const uint32_t nw = kind == kTrPoint ? 16 : kind == kTrScalar ? 8 : 0;
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = (uint32_t)i < nw ? src[i] : 0u;
  };
  // records are fetched three ahead: one record's bookkeeping (~150
  // instructions, ~0.3 us for a lone wave) does not cover a global load
  uint32_t cur[16], n1[16], n2[16], n3[16];
  fetch(0, cur);
  fetch(1, n1);
  fetch(2, n2);
  for (uint32_t k = 0; k < hd.nprog; k++) {
    const uint32_t op = prog[k];
    const uint32_t kind = op >> 24, idx = op & 0xffffffu;
    fetch(k + 3, n3);
    if (kind == kTrPoint) {
      uint32_t z = 0;
#pragma unroll
      for (int i = 0; i < 16; i++) z |= cur[i];
      if (z == 0) {
        st |= kTrStatusIdentity | ((op & kTrLookupZFlag) ? kTrStatusLookupZIdentity : 0u);
      } else {
        tr_put_byte(s, buf, slot, 1);
#pragma unroll
        for (int i = 0; i < 16; i++) tr_put_word(s, buf, slot, cur[i]);
      }
    } else if (kind == kTrScalar || kind == kTrVk) {
      tr_put_byte(s, buf, slot, 2);
#pragma unroll
      for (int i = 0; i < 8; i++) tr_put_word(s, buf, slot, kind == kTrVk ? hd.vk[i] : cur[i]);
    } else {
      tr_put_byte(s, buf, slot, 0);
    }
    // one compression site for every record kind
    const bool squeeze = kind == kTrSqueeze;
    tr_settle(s, buf, slot, q, squeeze, d);
    if (squeeze) {
      Fe<Fs> x;  // lo (even lanes) or hi (odd lanes); a bitwise select, since a
                 // conditional select of the array halves became a scratch access
      const uint32_t mq = 0u - (q & 1u);
#pragma unroll
      for (int i = 0; i < 8; i++) x.l[i] = (d[8 + i] & mq) | (d[i] & ~mq);
      const Fe<Fs> pr = fe_mul<Fs>(x, kq);
      Fe<Fs> p0, p1;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        p0.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pr.l[i], 0x00, 0xF, 0xF, false);
        p1.l[i] = (uint32_t)__builtin_amdgcn_mov_dpp((int)pr.l[i], 0x55, 0xF, 0xF, false);
      }
      const Fe<Fs> c = fe_add<Fs>(p0, p1);  // = fe_from_bytes_wide(d)
      if (b < hd.B) {
        uint2* out = reinterpret_cast<uint2*>(challenges + 8ull * (kTrChallenges * b + idx));
        out[q] = make_uint2(q == 0 ? c.l[0] : q == 1 ? c.l[2] : q == 2 ? c.l[4] : c.l[6],
                            q == 0 ? c.l[1] : q == 1 ? c.l[3] : q == 2 ? c.l[5] : c.l[7]);
      }
    }
#pragma unroll
    for (int i = 0; i < 16; i++) {
      cur[i] = n1[i];
      n1[i] = n2[i];
      n2[i] = n3[i];
    }
  }
  return st;
}

// dflags: the proof decode's flags of this batch (proof-bytes entry), taken
// into the status word and cleared for the next batch
__device__ __forceinline__ void tr_finish_status(uint32_t st, uint32_t b, uint32_t* __restrict__ status,
                                                 uint32_t* __restrict__ dflags) {
  if (dflags) {
    st |= dflags[b];
    dflags[b] = 0;
  }
  if (status) status[b] = st;
}

// The per-record kernel (shapes whose stream does not fit the streamed
// kernel's LDS): 64 lanes = 16 proofs x 4 lanes.
template <class Cv>
__global__ void __launch_bounds__(64) k_transcript(TranscriptHdr hd, const uint32_t* __restrict__ prog,
                                                   const uint32_t* __restrict__ points,
                                                   const uint32_t* __restrict__ scalars,
                                                   uint32_t* __restrict__ challenges, uint32_t* __restrict__ status,
                                                   uint32_t* __restrict__ dflags) {
  __shared__ TrBuf buf;
  const uint32_t slot = threadIdx.x >> 2, q = threadIdx.x & 3;
  const uint32_t b = blockIdx.x * kTrSlots + slot;
  if (b >= hd.B) return;
  const uint32_t st = tr_replay<Cv>(hd, prog, points, scalars, challenges, buf, slot, q, b);
  if (q == 0) tr_finish_status(st, b, status, dflags);
}

// ------------------------------------------------------ streamed replay
// (round 5).  Every proof of a shape absorbs the same byte layout (record
// tags, the VK record and the squeeze bytes are constants; point and scalar
// bytes sit at fixed offsets), so the host lays the stream out once
// (tr_stream_plan): per 32-bit stream word a constant and up to two byte runs
// of the proof's canonical data.  One block of 4 waves per 16 proofs:
//   A  all waves stage the proofs' canonical data and the word table in LDS,
//      then assemble every proof's whole stream in LDS;
//   B  wave 0 runs the compression chain (quad per proof, as above): the
//      128-byte blocks in order -- no per-record bookkeeping on the chain (it
//      was about half of k_transcript's ~0.10 ms); at each squeeze it leaves
//      its state in LDS and raises that squeeze's flag, and waves 1-3 (squeeze
//      k on wave 1 + k % 3) run the final compression of the zero-padded
//      partial block from it, off the chain;
//   C  all waves turn the 7 x 16 digests into challenges.
// A block with an identity point among its proofs (that record is skipped,
// shifting the stream) runs the per-record replay instead.
struct TrStreamHdr {
  uint32_t nw32;     // stream words with content (ceil(bytes / 4))
  uint32_t nblk;     // 128-byte blocks spanned by the stream
  uint32_t npr;      // point records in prog (identity check)
  uint32_t L[kTrChallenges];  // stream length at each squeeze (after its 0x00 byte)
};
// wtab: 3 words per stream word (the constant bytes, two parts), then the
// point index of each point record (identity check).  Part: bit 31 present, 30 region (0 points, 1 scalars), 28-29
// byte shift in the source word, 26-27 byte position in the stream word,
// 23-25 byte count, 22 a second source word needed, 0-21 source word index
constexpr uint32_t kTrPartIdxMask = (1u << 22) - 1u;
constexpr uint32_t kTrDataStride = kTrSlots + 1;  // LDS data rows [word][slot], padded

// LDS words (u32) of the streamed kernel, and its layout
struct TrStreamLds {
  uint32_t oT, oD, oS, oF, oH, oG, oFlag, total;
  __host__ __device__ TrStreamLds(uint32_t nw32, uint32_t nblk, uint32_t npr, uint32_t npts, uint32_t nsc) {
    oT = 0;                                               // word table (3 per stream word), point records
    oD = (3 * nw32 + npr + 1) & ~1u;                      // canonical data [word][17]
    oS = (oD + kTrDataStride * (16 * npts + 8 * nsc) + 1) & ~1u;  // stream [w64][16] (u64)
    oF = oS + 2 * kTrSlots * 16 * nblk;                   // final blocks of waves 1-3, [16][16] (u64) each
    oH = oF + 3 * 2 * kTrSlots * 16;                      // chain states at the squeezes [7][16 slots][8] (u64)
    oG = oH + 2 * kTrChallenges * kTrSlots * 8;           // digests [7][16 slots][16]
    oFlag = oG + kTrChallenges * kTrSlots * 16;           // identity flag, then one flag per squeeze
    total = oFlag + 1 + kTrChallenges;
  }
};

template <class Cv>
__global__ void __launch_bounds__(256) k_transcript_s(TranscriptHdr hd, TrStreamHdr sh,
                                                     const uint32_t* __restrict__ prog,
                                                     const uint32_t* __restrict__ wtab,
                                                     const uint32_t* __restrict__ points,
                                                     const uint32_t* __restrict__ scalars,
                                                     uint32_t* __restrict__ challenges,
                                                     uint32_t* __restrict__ status, uint32_t* __restrict__ dflags) {
  using Fs = typename Cv::Scalar;
  extern __shared__ __align__(16) uint32_t tr_lds[];
  const TrStreamLds lay(sh.nw32, sh.nblk, sh.npr, hd.npts, hd.nsc);
  uint32_t* const T = tr_lds + lay.oT;
  uint32_t* const D = tr_lds + lay.oD;
  uint64_t* const S = reinterpret_cast<uint64_t*>(tr_lds + lay.oS);
  uint32_t* const G = tr_lds + lay.oG;
  uint32_t* const flag = tr_lds + lay.oFlag;
  const uint32_t tid = threadIdx.x, b0 = blockIdx.x * kTrSlots;
  const uint32_t ndp = 16 * hd.npts, nd = ndp + 8 * hd.nsc;  // data words per proof
  // --- A1: the word table and the 16 proofs' canonical data into LDS
  if (tid <= kTrChallenges) flag[tid] = 0;
  for (uint32_t f = tid; f < 3 * sh.nw32 + sh.npr; f += blockDim.x) T[f] = wtab[f];
  for (uint32_t f = tid; f < kTrSlots * (nd / 4); f += blockDim.x) {
    const uint32_t sl = f / (nd / 4), w = 4 * (f - sl * (nd / 4)), b = b0 + sl;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (b < hd.B)
      v = w < ndp ? *reinterpret_cast<const uint4*>(points + (size_t)ndp * b + w)
                  : *reinterpret_cast<const uint4*>(scalars + (size_t)(nd - ndp) * b + (w - ndp));
    D[(w + 0) * kTrDataStride + sl] = v.x;
    D[(w + 1) * kTrDataStride + sl] = v.y;
    D[(w + 2) * kTrDataStride + sl] = v.z;
    D[(w + 3) * kTrDataStride + sl] = v.w;
  }
  __syncthreads();
  // --- A2: the streams (item = (word, slot), slot fastest), and the identity check
  uint32_t* const S32 = reinterpret_cast<uint32_t*>(S);
  for (uint32_t f = tid; f < kTrSlots * 32 * sh.nblk; f += blockDim.x) {
    const uint32_t w = f / kTrSlots, sl = f - w * kTrSlots;
    uint32_t v = 0;
    if (w < sh.nw32) {
      v = T[3 * w];
#pragma unroll
      for (int k = 1; k <= 2; k++) {
        const uint32_t pt = T[3 * w + k];
        if (pt >> 31) {
          const uint32_t idx = (pt & kTrPartIdxMask) + (((pt >> 30) & 1u) ? ndp : 0u);
          const uint32_t lo = D[idx * kTrDataStride + sl];
          const uint32_t hi = ((pt >> 22) & 1u) ? D[(idx + 1) * kTrDataStride + sl] : 0u;
          const uint32_t sh8 = 8 * ((pt >> 28) & 3u), p8 = 8 * ((pt >> 26) & 3u), n = (pt >> 23) & 7u;
          const uint32_t dv = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh8);
          const uint32_t mask = n >= 4 ? ~0u : (1u << (8 * n)) - 1u;
          v |= (dv & mask) << p8;
        }
      }
    }
    S32[2 * ((w >> 1) * kTrSlots + sl) + (w & 1)] = v;
  }
  for (uint32_t f = tid; f < kTrSlots * sh.npr; f += blockDim.x) {
    const uint32_t r = f / kTrSlots, sl = f - r * kTrSlots;
    const uint32_t idx = 16 * T[3 * sh.nw32 + r];
    uint32_t z = 0;
    for (int i = 0; i < 16; i++) z |= D[(idx + i) * kTrDataStride + sl];
    if (z == 0 && b0 + sl < hd.B) atomicOr(flag, 1u);
  }
  __syncthreads();
  const bool slow = *flag != 0;
  // --- B: wave 0, a quad per proof
  if (tid < 64) {
    const uint32_t slot = tid >> 2, q = tid & 3, b = b0 + slot;
    uint32_t st = 0;
    if (slow) {
      st = tr_replay<Cv>(hd, prog, points, scalars, challenges, *reinterpret_cast<TrBuf*>(tr_lds), slot, q, b);
    }
    if (q == 0 && b < hd.B) tr_finish_status(st, b, status, dflags);
  }
  if (!slow) {
    const uint32_t w = tid >> 6, slot = (tid & 63) >> 2, q = tid & 3;
    uint64_t* const H = reinterpret_cast<uint64_t*>(tr_lds + lay.oH);
    const uint64_t* col = S + slot;
    if (w == 0) {  // the chain
      uint64_t h0 = q == 0 ? hd.h0[0] : q == 1 ? hd.h0[1] : q == 2 ? hd.h0[2] : hd.h0[3];
      uint64_t h1 = q == 0 ? hd.h0[4] : q == 1 ? hd.h0[5] : q == 2 ? hd.h0[6] : hd.h0[7];
      uint32_t done = 0;
      for (uint32_t k = 0; k < kTrChallenges; k++) {
        const uint32_t m = (sh.L[k] + 127) / 128 - 1;  // blocks compressed before the final one
        for (; done < m; done++) tr_compress_q(h0, h1, TrStreamMsg{col, 16 * done}, q, 128ull * (done + 1), false);
        H[8 * (k * kTrSlots + slot) + q] = h0;
        H[8 * (k * kTrSlots + slot) + 4 + q] = h1;
        if (tid == 0) __hip_atomic_store(&flag[1 + k], 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
    } else {  // the finals of squeezes w - 1, w + 2, ...
      uint64_t* fin = reinterpret_cast<uint64_t*>(tr_lds + lay.oF) + (w - 1) * 16 * kTrSlots + slot;
      for (uint32_t k = w - 1; k < kTrChallenges; k += 3) {
        while (__hip_atomic_load(&flag[1 + k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
          __builtin_amdgcn_s_sleep(1);
        const uint32_t L = sh.L[k], m = (L + 127) / 128 - 1;
        // block m zero-padded after byte L (every lane of the quad writes the
        // same 16 words, so each lane reads back only its own stores)
        const uint32_t lim = L - 128 * m;
#pragma unroll
        for (uint32_t i = 0; i < 16; i++) {
          const uint64_t v = col[(16 * m + i) * kTrSlots];
          const uint32_t lo = 8 * i;
          fin[i * kTrSlots] = lo + 8 <= lim ? v : lo >= lim ? 0ull : v & ((1ull << (8 * (lim - lo))) - 1ull);
        }
        uint64_t f0 = H[8 * (k * kTrSlots + slot) + q], f1 = H[8 * (k * kTrSlots + slot) + 4 + q];
        tr_compress_q(f0, f1, TrStreamMsg{fin, 0}, q, (uint64_t)L, true);
        uint32_t d[16];
        tr_digest_q(f0, f1, d);
        uint32_t* g = G + 16 * (k * kTrSlots + slot);
#pragma unroll
        for (int i = 0; i < 4; i++) g[4 * q + i] = d[4 * q + i];
      }
    }
  }
  __syncthreads();
  // --- C: challenges = from_bytes_wide(digest), 7 x 16 items over the block
  if (!slow)
    for (uint32_t f = tid; f < kTrChallenges * kTrSlots; f += blockDim.x) {
      const uint32_t k = f / kTrSlots, sl = f - k * kTrSlots, b = b0 + sl;
      if (b >= hd.B) continue;
      uint32_t d[16];
#pragma unroll
      for (int i = 0; i < 16; i++) d[i] = G[16 * (k * kTrSlots + sl) + i];
      const Fe<Fs> c = fe_from_bytes_wide<Fs>(d);
      uint4* out = reinterpret_cast<uint4*>(challenges + 8ull * (kTrChallenges * b + k));
      out[0] = make_uint4(c.l[0], c.l[1], c.l[2], c.l[3]);
      out[1] = make_uint4(c.l[4], c.l[5], c.l[6], c.l[7]);
    }
}

}  // namespace pm

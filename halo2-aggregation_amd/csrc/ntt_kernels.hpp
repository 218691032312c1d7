// ntt_kernels.hpp -- NTT over a scalar field: halo2's
// `best_fft(a, omega, log_n)` [3P], the transform behind EvaluationDomain's
// fft / ifft / coset conversions in create_proof.  Output is the natural-order
// DFT  A_k = sum_j a_j omega^{jk}; it is exact field arithmetic, so any
// correct factorisation is bit-identical to halo2's radix-2 DIT.
//
// Four-step factorisation n = n1 * n2 (both <= 2^12), two passes over HBM:
//   pass A (k_ntt_cols): for every column i2, the n1-point NTT over
//     x[i1 * n2 + i2] (root omega^{n2}), times omega^{i2 k1}, stored in place
//     at [k1 * n2 + i2];
//   pass B (k_ntt_rows): for every row k1, the n2-point NTT over the contiguous
//     row (root omega^{n1}), stored at out[k1 + n1 * k2]  (natural order),
//     optionally times a scale (ifft: the 1/n divisor).
// Each sub-transform runs as a radix-4 DIT on bit-reversed positions: its
// first round in registers as the inputs arrive from global memory
// (ntt_load_first), the middle rounds in LDS (structure of arrays: 9 limb
// planes of the radix-2^29 form at XOR-swizzled positions, lds_swz), the last
// round in registers on the way out (ntt_last_store).  A workgroup takes C
// adjacent columns (pass A) or rows (pass B) so its global loads / stores
// move C x 32 contiguous bytes.  Roots come from small per-transform tables
// (R = 2^261 form), built once per (field, omega, log_n) and cached in the
// context: one segment of L/2 powers per sub-transform, and the inter-pass
// twiddles as a two-level product (k_ntt_twiddles below).
#pragma once
#include "msm_kernels.hpp"

namespace pm {

// threads per block: chosen per launch by the host (ntt_engine.hpp), at most
// kNttMaxThreads; the device loops stride by blockDim.x
constexpr int kNttMaxThreads = 512;
constexpr int kNttMaxLogL = 12;  // longest sub-transform (2^12 x 36 B = 144 KiB of LDS)
constexpr size_t kNttLdsBytes = 36;  // LDS bytes per element (9 limb planes)

struct FeArg {
  uint32_t l[8];
};

template <class Fs>
__device__ __forceinline__ Fe<Fs> fe_of(const FeArg& a) {
  Fe<Fs> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = a.l[i];
  return r;
}

// Arithmetic (round 3): the radix-2^29 lazy Montgomery form of the MSM
// (fp29.hpp) instead of 8 x 32-bit limbs.  A 32-bit-limb product needs a
// v_mad_u64_u32 plus a carry add per limb pair (~300 VALU instructions for
// BN254 Fr); the 29-bit columns chain their multiply-adds in one 64-bit
// accumulator (~210), and additions are limb-wise with one carry pass per
// radix-4 output instead of a borrow chain and a select per add / sub.
// The DATA keeps the caller's R = 2^256 Montgomery meaning, only unpacked
// into 29-bit limbs; the TWIDDLES are stored in the R = 2^261 form, so the
// product x 2^256 * w 2^261 * 2^-261 = x w 2^256 stays in the data's form and
// no per-element conversion is needed.  Bounds (p < 2^254 for Pasta, ~2^253.6
// for BN254 Fr, so R / p >= 128): LDS holds Norm values < 3p; a twiddle is
// canonical (< p) or its negation 2p - w (< 2p), both Norm; f29_mul_c of a
// value < 9p with limbs < 2^30 by a Norm twiddle < 2p is Norm, < 2p
// (tests/test_fp29_asm.py::test_ntt_operand_bounds runs these operand shapes
// through the interpreter with its overflow checks); each radix-4 output
// (< 12p, limbs < 2^32 - 8) is normalised and reduced to < 3p, or, in every
// other LDS round, left normalised at < 7p for the next round to reduce.  A difference
// adds 2p when its subtrahend is a product (< 2p) and 6p when it is an
// unmultiplied input (< 3p, the twiddle-1 stage 0), so it never goes negative.  Between
// passes elements are stored packed but not canonical (< 3p < 2^256); the
// last pass canonicalises.

// Twiddle tables (round 4): instead of one flat table tw[i] = omega^i for
// i < n/2 (512 MiB at 2^25, whose inter-pass gathers went to HBM: pass A
// fetched 5.2 GB per 2^25 transform, profiles/r03/ntt_pmc/final_ntt25/),
// each transform keeps small segments, all L2-resident:
//   * per sub-transform of length L = 2^logL with root omega^step: its L/2
//     powers (omega^step)^m, read with stride 1 (lds_ntt4 / ntt_load_first /
//     ntt_last_store take the segment and tstride = 1);
//   * the inter-pass twiddles omega^e (e < n) as lo[e mod 2^s] * hi[e >> s]
//     (s = ceil(log n / 2): 2^13 + 2^12 entries at 2^25), one extra product.
// k_ntt_twiddles fills segment s with omega^{(step_s k) mod n}, k < count_s,
// by square-and-multiply per entry (R = 2^261 form, canonical, packed).
constexpr int kNttMaxSegs = 5;
struct NttSegs {
  uint32_t off[kNttMaxSegs], count[kNttMaxSegs], step[kNttMaxSegs];
  uint32_t nseg, logn;
};
template <class Fs>
__global__ void __launch_bounds__(256) k_ntt_twiddles(FeArg omega, NttSegs sg, uint32_t* __restrict__ tw) {
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = 0;
  while (s < sg.nseg && i >= sg.count[s]) i -= sg.count[s++];
  if (s >= sg.nseg) return;
  const uint64_t nmask = (1ull << sg.logn) - 1;
  uint64_t e = ((uint64_t)sg.step[s] * i) & nmask;
  Fe<Fs> r = fe_one<Fs>(), b = fe_of<Fs>(omega);
  for (; e; e >>= 1) {
    if (e & 1) r = fe_mul<Fs>(r, b);
    b = fe_sqr<Fs>(b);
  }
  Fe<Fs> o;
  f29_pack<Fs>(f29_canon<Fs>(f29_from_r256<Fs>(r.l)), o.l);
  store_fe4<Fs>(reinterpret_cast<uint4*>(tw + 8ull * (sg.off[s] + i)), o);
}

__device__ __forceinline__ uint32_t ntt_brev(uint32_t x, int bits) { return bits ? __brev(x) >> (32 - bits) : 0u; }

// packed element (8 x u32, value < 2^256) <-> Norm 29-bit limbs
template <class Fs>
__device__ __forceinline__ F29<Fs> g_ld29(const uint32_t* __restrict__ g, size_t idx) {
  const Fe<Fs> v = load_fe4<Fs>(reinterpret_cast<const uint4*>(g + 8ull * idx));
  return f29_unpack<Fs>(v.l);
}
template <class Fs>
__device__ __forceinline__ void g_st29(uint32_t* g, size_t idx, const F29<Fs>& v) {  // v Norm, < 2^256
  Fe<Fs> w;
  f29_pack<Fs>(v, w.l);
  store_fe4<Fs>(reinterpret_cast<uint4*>(g + 8ull * idx), w);
}

// LDS image: 9 limb planes of `plane` words.  Logical position idx sits at
// word lds_swz(idx) of each plane: bits 0-5 XORed with bits 2-7, 5-10 and
// 6-11.  Unswizzled, the bit-reversed scatter of the load phase put a wave's
// 64 stores into a few banks (up to 32-way conflicts) and the short-stride
// radix-4 rounds 2-4-way (rocprofv3: SQ_LDS_BANK_CONFLICT 78 % of
// SQ_LDS_IDX_ACTIVE in k_ntt_rows at 2^20, profiles/r03/ntt_f29/stall_*); a
// bank model of every access pattern of the fused load, the LDS rounds and the
// stores (tools/ntt_lds_bank_model.py, 64 banks) picked this swizzle.  The map
// is upper triangular on the bits, so it permutes [0, 2^m) for every plane
// size 2^m.
__device__ __forceinline__ uint32_t lds_swz(uint32_t i) { return i ^ (((i >> 2) ^ (i >> 5) ^ (i >> 6)) & 63u); }
template <class Fs>
__device__ __forceinline__ F29<Fs> lds_ld(const uint32_t* sm, uint32_t plane, uint32_t idx) {
  const uint32_t s = lds_swz(idx);
  F29<Fs> r;
#pragma unroll
  for (int k = 0; k < 9; k++) r.l[k] = sm[k * plane + s];
  return r;
}
template <class Fs>
__device__ __forceinline__ void lds_st(uint32_t* sm, uint32_t plane, uint32_t idx, const F29<Fs>& v) {
  const uint32_t s = lds_swz(idx);
#pragma unroll
  for (int k = 0; k < 9; k++) sm[k * plane + s] = v.l[k];
}

// twiddle m of a sub-transform segment (R261, Norm, canonical)
template <class Fs>
__device__ __forceinline__ F29<Fs> tw_half(const uint32_t* __restrict__ tw, size_t e) {
  return g_ld29<Fs>(tw, e);
}
// inter-pass twiddle omega^e, e < n: lo[e mod 2^s] hi[e >> s] (Norm, < 2p)
template <class Fs>
__device__ __forceinline__ F29<Fs> tw_two(const uint32_t* __restrict__ lo, const uint32_t* __restrict__ hi,
                                          uint32_t e, int s) {
  return f29_mul_c<Fs>(g_ld29<Fs>(lo, e & ((1u << s) - 1)), g_ld29<Fs>(hi, e >> s));
}

// lazy sum / difference -> Norm, < 3p
template <class Fs>
__device__ __forceinline__ F29<Fs> f29_nr(const F29<Fs>& a) {
  return f29_reduce3<Fs>(f29_norm<Fs>(a));
}

// In-LDS DIT over C interleaved transforms of length L = 2^logL (layout
// [position][c], positions already bit-reversed), two stages per LDS round
// trip: radix-4 units on positions j, j + h, j + 2h, j + 3h (h = 2^t), stage
// t with the twiddle W_{2h}^lo on both pairs, then stage t + 1 with W_{4h}^lo
// and W_{4h}^{lo+h}.  An odd logL starts with one radix-2 stage (twiddle 1).
// Root of the sub-transform: omega^{tstride}, looked up as tw[m * tstride].
// (Round 2 measured the radix-4 rounds against radix-2 stages: half the LDS
// traffic and barriers, 2^20 0.221 -> 0.205 ms; the radix-2 form is retired.)
template <class Fs>
__device__ __forceinline__ void lds_ntt4(uint32_t* sm, int logL, int logC, uint32_t tstride,
                                         const uint32_t* __restrict__ tw, int t = 0, bool skip_last = false) {
  using K = F29Consts<Fs>;
  const uint32_t plane = 1u << (logL + logC);
  const uint32_t cmask = (1u << logC) - 1;
  if (t == 0 && (logL & 1)) {  // stage 0: twiddle 1; v < 3p unmultiplied, so u - v + 6p (< 9p)
    for (uint32_t b = threadIdx.x; b < (plane >> 1); b += blockDim.x) {
      const uint32_t c = b & cmask, j = (b >> logC) << 1;
      const uint32_t ia = (j << logC) | c, ib = ((j + 1) << logC) | c;
      const F29<Fs> u = lds_ld<Fs>(sm, plane, ia), v = lds_ld<Fs>(sm, plane, ib);
      lds_st<Fs>(sm, plane, ia, f29_nr<Fs>(f29_add<Fs>(u, v)));
      lds_st<Fs>(sm, plane, ib, f29_nr<Fs>(f29_sub<Fs>(u, v, K::K6)));
    }
    __syncthreads();
    t = 1;
  }
  // Lazy reduction: a round whose inputs are < 3p may leave its outputs
  // normalised but unreduced (< 7p, since the t > 0 unit adds at most 4p);
  // the next round takes < 7p inputs (products < 7p * 2p, sums < 9p) and
  // reduces its < 11p outputs.  So rounds alternate, and the last LDS round
  // reduces when the unfused store phase (canonical form / packing, < 4p)
  // follows; the fused last round (ntt_last_store) reduces its own outputs.
  for (int r = 0; t + 1 < logL && !(skip_last && t == logL - 2); t += 2, r++) {
    const bool next = t + 3 < logL && !(skip_last && t + 2 == logL - 2);
    const bool red = (r & 1) || (!next && !skip_last) || t == 0;
    const uint32_t h = 1u << t;
    for (uint32_t b = threadIdx.x; b < (plane >> 2); b += blockDim.x) {
      const uint32_t c = b & cmask, bb = b >> logC;
      const uint32_t lo = bb & (h - 1);
      const uint32_t j = ((bb >> t) << (t + 2)) | lo;
      const uint32_t i0 = (j << logC) | c, i1 = ((j + h) << logC) | c, i2 = ((j + 2 * h) << logC) | c,
                     i3 = ((j + 3 * h) << logC) | c;
      F29<Fs> x0 = lds_ld<Fs>(sm, plane, i0), x1 = lds_ld<Fs>(sm, plane, i1);
      F29<Fs> x2 = lds_ld<Fs>(sm, plane, i2), x3 = lds_ld<Fs>(sm, plane, i3);
      F29<Fs> y0, y1, y2, y3;
      if (t > 0) {
        const F29<Fs> w1 = tw_half<Fs>(tw, (size_t)(lo << (logL - 1 - t)) * tstride);
        x1 = f29_mul_c<Fs>(x1, w1);  // < 2p
        x3 = f29_mul_c<Fs>(x3, w1);
        // y0, y2 < 5p (limbs < 2^30); y1, y3 < 5p, y3 normalised for the product
        y1 = f29_sub<Fs>(x0, x1, K::K2);
        y3 = f29_norm<Fs>(f29_sub<Fs>(x2, x3, K::K2));
      } else {
        // stage 0 twiddle 1: x1, x3 < 3p unmultiplied, so + 6p (< 9p; a + 2p - b
        // would go negative for b > a + 2p)
        y1 = f29_sub<Fs>(x0, x1, K::K6);
        y3 = f29_norm<Fs>(f29_sub<Fs>(x2, x3, K::K6));
      }
      y0 = f29_add<Fs>(x0, x1);
      y2 = f29_add<Fs>(x2, x3);
      const F29<Fs> w2 = tw_half<Fs>(tw, (size_t)(lo << (logL - 2 - t)) * tstride);
      const F29<Fs> w3 = tw_half<Fs>(tw, (size_t)((lo + h) << (logL - 2 - t)) * tstride);
      const F29<Fs> z2 = f29_mul_c<Fs>(y2, w2), z3 = f29_mul_c<Fs>(y3, w3);  // < 2p
      // outputs < 11p, limbs < 2^31 + 2^30
      F29<Fs> o0 = f29_norm<Fs>(f29_add<Fs>(y0, z2)), o2 = f29_norm<Fs>(f29_sub<Fs>(y0, z2, K::K2));
      F29<Fs> o1 = f29_norm<Fs>(f29_add<Fs>(y1, z3)), o3 = f29_norm<Fs>(f29_sub<Fs>(y1, z3, K::K2));
      if (red) {
        o0 = f29_reduce3<Fs>(o0);
        o1 = f29_reduce3<Fs>(o1);
        o2 = f29_reduce3<Fs>(o2);
        o3 = f29_reduce3<Fs>(o3);
      }
      lds_st<Fs>(sm, plane, i0, o0);
      lds_st<Fs>(sm, plane, i2, o2);
      lds_st<Fs>(sm, plane, i1, o1);
      lds_st<Fs>(sm, plane, i3, o3);
    }
    __syncthreads();
  }
}

// Load phase fused with the first round (saves one LDS round trip and
// barrier per pass, and the twiddle-1 product of the first radix-4 round):
// src(i, c) returns input i (natural order, < L) of transform c.  Position
// 2m / 2m + 1 of the bit-reversed layout holds inputs brev(m) and brev(m) +
// L/2 (odd logL: the radix-2 stage 0 in registers); positions 4m + q hold
// brev(m) + {0, L/2, L/4, 3L/4}[q] (even logL: the t = 0 radix-4 unit, W_2 =
// W_4^0 = 1, W_4^1 = omega^{tstride L/4}).  kfast: lanes walk m fastest (the
// rows pass: consecutive inputs are contiguous in memory), else c fastest.
// Returns the stage lds_ntt4 continues from.
template <class Fs, class Src>
__device__ __forceinline__ int ntt_load_first(uint32_t* sm, int logL, int logC, uint32_t tstride,
                                              const uint32_t* __restrict__ tw, bool kfast, Src src) {
  using K = F29Consts<Fs>;
  const uint32_t plane = 1u << (logL + logC), L = 1u << logL, C = 1u << logC;
  if (logL == 0) {
    for (uint32_t e = threadIdx.x; e < plane; e += blockDim.x) lds_st<Fs>(sm, plane, e, src(0u, e));
    return 0;
  }
  if (logL & 1) {
    const uint32_t nm = L >> 1;
    for (uint32_t b = threadIdx.x; b < (plane >> 1); b += blockDim.x) {
      const uint32_t m = kfast ? b & (nm - 1) : b >> logC, c = kfast ? b >> (logL - 1) : b & (C - 1);
      const uint32_t i = m, pos = ntt_brev(i, logL);  // i < L/2: pos = 2 m'
      const F29<Fs> u = src(i, c), v = src(i + nm, c);
      lds_st<Fs>(sm, plane, (pos << logC) | c, f29_nr<Fs>(f29_add<Fs>(u, v)));
      lds_st<Fs>(sm, plane, ((pos + 1) << logC) | c, f29_nr<Fs>(f29_sub<Fs>(u, v, K::K6)));
    }
    return 1;
  }
  const uint32_t nm = L >> 2;
  const F29<Fs> w3 = tw_half<Fs>(tw, (size_t)nm * tstride);  // omega_4
  for (uint32_t b = threadIdx.x; b < (plane >> 2); b += blockDim.x) {
    const uint32_t m = kfast ? b & (nm - 1) : b >> logC, c = kfast ? b >> (logL - 2) : b & (C - 1);
    const uint32_t i = m, pos = ntt_brev(i, logL);  // i < L/4: pos = 4 m'
    const F29<Fs> x0 = src(i, c), x1 = src(i + 2 * nm, c), x2 = src(i + nm, c), x3 = src(i + 3 * nm, c);
    // inputs < 3p: y0 < 6p; y1 = x0 - x1 + 6p < 9p; y2 normalised < 6p; y3 normalised < 9p
    const F29<Fs> y0 = f29_add<Fs>(x0, x1), y1 = f29_sub<Fs>(x0, x1, K::K6);
    const F29<Fs> y2 = f29_norm<Fs>(f29_add<Fs>(x2, x3)), y3 = f29_norm<Fs>(f29_sub<Fs>(x2, x3, K::K6));
    const F29<Fs> z3 = f29_mul_c<Fs>(y3, w3);  // < 2p
    lds_st<Fs>(sm, plane, (pos << logC) | c, f29_nr<Fs>(f29_add<Fs>(y0, y2)));              // < 12p
    lds_st<Fs>(sm, plane, ((pos + 2) << logC) | c, f29_nr<Fs>(f29_sub<Fs>(y0, y2, K::K6)));  // < 12p
    lds_st<Fs>(sm, plane, ((pos + 1) << logC) | c, f29_nr<Fs>(f29_add<Fs>(y1, z3)));         // < 11p
    lds_st<Fs>(sm, plane, ((pos + 3) << logC) | c, f29_nr<Fs>(f29_sub<Fs>(y1, z3, K::K2)));  // < 11p
  }
  return 2;
}

// Store phase fused with the last radix-4 round (t = logL - 2 >= 1, h = L/4):
// the unit on positions j, j + h, j + 2h, j + 3h (j < h) produces outputs
// j + q h directly, so dst(k, c, v) (the pass's epilogue: inter-pass twiddle
// or scale, canonical form, global store) takes them from registers instead
// of a last LDS round trip.  Lanes walk c fastest, as the unfused store does.
template <class Fs, class Dst>
__device__ __forceinline__ void ntt_last_store(const uint32_t* sm, int logL, int logC, uint32_t tstride,
                                               const uint32_t* __restrict__ tw, Dst dst) {
  using K = F29Consts<Fs>;
  const uint32_t plane = 1u << (logL + logC), C = 1u << logC, h = 1u << (logL - 2);
  for (uint32_t b = threadIdx.x; b < (plane >> 2); b += blockDim.x) {
    const uint32_t c = b & (C - 1), j = b >> logC;  // j < h: lo = j
    F29<Fs> x0 = lds_ld<Fs>(sm, plane, (j << logC) | c), x1 = lds_ld<Fs>(sm, plane, ((j + h) << logC) | c);
    F29<Fs> x2 = lds_ld<Fs>(sm, plane, ((j + 2 * h) << logC) | c), x3 = lds_ld<Fs>(sm, plane, ((j + 3 * h) << logC) | c);
    const F29<Fs> w1 = tw_half<Fs>(tw, (size_t)(j << 1) * tstride);  // W_{2h}^j
    x1 = f29_mul_c<Fs>(x1, w1);
    x3 = f29_mul_c<Fs>(x3, w1);
    const F29<Fs> y0 = f29_add<Fs>(x0, x1), y1 = f29_sub<Fs>(x0, x1, K::K2);
    const F29<Fs> y2 = f29_add<Fs>(x2, x3), y3 = f29_norm<Fs>(f29_sub<Fs>(x2, x3, K::K2));
    const F29<Fs> w2 = tw_half<Fs>(tw, (size_t)j * tstride), w3 = tw_half<Fs>(tw, (size_t)(j + h) * tstride);
    const F29<Fs> z2 = f29_mul_c<Fs>(y2, w2), z3 = f29_mul_c<Fs>(y3, w3);
    dst(j, c, f29_nr<Fs>(f29_add<Fs>(y0, z2)));
    dst(j + h, c, f29_nr<Fs>(f29_add<Fs>(y1, z3)));
    dst(j + 2 * h, c, f29_nr<Fs>(f29_sub<Fs>(y0, z2, K::K2)));
    dst(j + 3 * h, c, f29_nr<Fs>(f29_sub<Fs>(y1, z3, K::K2)));
  }
}

// rounds after the fused load, then the store (with the last round fused
// when there is one to fuse and its units occupy every thread: with fewer
// units than threads the epilogue of 4 outputs per unit would run on part of
// the block)
// make_dst() builds the epilogue after the rounds, so what it holds (the
// rows pass's scale) is not live across them (129 instead of 113 VGPRs: 3
// waves per SIMD, 2^23 rows pass 0.39 -> 0.48 ms)
template <class Fs, class MakeDst>
__device__ __forceinline__ void ntt_rounds_store(uint32_t* sm, int logL, int logC, uint32_t tstride,
                                                 const uint32_t* __restrict__ tw, int t0, MakeDst make_dst) {
  const bool fuse = logL - 2 >= t0 && logL >= 3 && (1u << (logL + logC - 2)) >= blockDim.x;
  lds_ntt4<Fs>(sm, logL, logC, tstride, tw, t0, fuse);
  auto dst = make_dst();
  if (fuse) {
    ntt_last_store<Fs>(sm, logL, logC, tstride, tw, dst);
    return;
  }
  const uint32_t plane = 1u << (logL + logC), C = 1u << logC;
  for (uint32_t e = threadIdx.x; e < plane; e += blockDim.x) dst(e >> logC, e & (C - 1), lds_ld<Fs>(sm, plane, e));
}

// XCD-aware block order: consecutive logical blocks (adjacent columns / rows,
// which share 128-B lines) land on the same XCD and its L2.
__device__ __forceinline__ uint32_t ntt_block(uint32_t nblocks) {
  const uint32_t b = blockIdx.x;
  if (nblocks % 8) return b;
  return (b % 8) * (nblocks / 8) + b / 8;
}

// pass A: C = 2^logC adjacent columns per block.  last != 0: this is the
// whole transform (one pass), so the output is canonicalised.
// tw: the (omega^{n2})^m segment; lo / hi / s: the inter-pass twiddles
template <class Fs>
__global__ void __launch_bounds__(kNttMaxThreads) k_ntt_cols(const uint32_t* in, uint32_t* out,  // may alias
                                                          int logn, int log1, int logC,
                                                          const uint32_t* __restrict__ tw,
                                                          const uint32_t* __restrict__ lo,
                                                          const uint32_t* __restrict__ hi, int s, uint32_t last) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int log2 = logn - log1;
  const uint32_t n2 = 1u << log2;
  const uint32_t col0 = ntt_block(n2 >> logC) << logC;
  const int t0 = ntt_load_first<Fs>(sm, log1, logC, 1, tw, false, [&](uint32_t i1, uint32_t c) {
    return g_ld29<Fs>(in, (size_t)i1 * n2 + col0 + c);
  });
  __syncthreads();
  // root omega^{n2}
  ntt_rounds_store<Fs>(sm, log1, logC, 1, tw, t0, [&] {
    return [&](uint32_t k1, uint32_t c, F29<Fs> v) {
      const uint32_t i2 = col0 + c;
      if (log2 > 0 && i2 && k1) v = f29_mul_c<Fs>(v, tw_two<Fs>(lo, hi, i2 * k1, s));  // i2 k1 < n
      if (last) v = f29_canon<Fs>(v);
      g_st29<Fs>(out, (size_t)k1 * n2 + i2, v);
    };
  });
}

// Three-pass form (n = n1 * na * nb, every factor <= 2^10, for n >= 2^23):
// pass A is k_ntt_cols with n2 = na * nb; the middle pass (k_ntt_mid) runs
// the row NTTs of length n2 (root omega^{n1}) as a four-step of their own:
// for every row k1 and column ib of the row's na x nb matrix, the na-point
// NTT over ia (root omega^{n1 nb}), times omega^{n1 ib ka}, stored at
// [(ka n1 + k1) nb + ib] so that pass B (k_ntt_rows over the n1 na rows of
// length nb, root omega^{n1 na}) writes out[k1 + n1 ka + n1 na kb] =
// out[k1 + n1 k2] with k2 = ka + na kb: the natural order.
template <class Fs>
__global__ void __launch_bounds__(kNttMaxThreads) k_ntt_mid(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         int logn, int log1, int loga, int logC,
                                                         const uint32_t* __restrict__ tw,
                                                         const uint32_t* __restrict__ lo,
                                                         const uint32_t* __restrict__ hi, int s) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int logb = logn - log1 - loga;
  const uint32_t n1 = 1u << log1, nb = 1u << logb;
  const uint32_t groups = nb >> logC;  // column groups per row
  const uint32_t blk = ntt_block(n1 * groups);
  const uint32_t k1 = blk / groups, col0 = (blk - k1 * groups) << logC;
  const uint32_t* row = in + 8ull * ((size_t)k1 << (loga + logb));
  const int t0 = ntt_load_first<Fs>(sm, loga, logC, 1, tw, false, [&](uint32_t ia, uint32_t c) {
    return g_ld29<Fs>(row, (size_t)ia * nb + col0 + c);
  });
  __syncthreads();
  // root omega^{n1 nb} (segment tw)
  ntt_rounds_store<Fs>(sm, loga, logC, 1, tw, t0, [&] {
    return [&](uint32_t ka, uint32_t c, F29<Fs> v) {
      const uint32_t ib = col0 + c;
      if (ib && ka) v = f29_mul_c<Fs>(v, tw_two<Fs>(lo, hi, n1 * ib * ka, s));  // n1 ib ka < n
      g_st29<Fs>(out, ((size_t)ka * n1 + k1) * nb + ib, v);
    };
  });
}

// pass B: R = 2^logR adjacent rows per block; optional output scale (R256
// form, converted once per thread); the output is canonical
template <class Fs>
__global__ void __launch_bounds__(kNttMaxThreads) k_ntt_rows(const uint32_t* in, uint32_t* out,  // may alias (log2 = 0)
                                                          int logn, int log2, int logR,
                                                          const uint32_t* __restrict__ tw, FeArg scale,
                                                          uint32_t use_scale) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int log1 = logn - log2;
  const uint32_t n1 = 1u << log1, L = 1u << log2;
  const uint32_t row0 = ntt_block(n1 >> logR) << logR;
  const int t0 = ntt_load_first<Fs>(sm, log2, logR, 1, tw, true, [&](uint32_t i2, uint32_t r) {
    return g_ld29<Fs>(in, (size_t)(row0 + r) * L + i2);  // row-contiguous loads
  });
  __syncthreads();
  // root omega^{n1} (segment tw); adjacent rows -> adjacent outputs
  ntt_rounds_store<Fs>(sm, log2, logR, 1, tw, t0, [&] {
    const F29<Fs> sc = use_scale ? f29_from_r256<Fs>(scale.l) : f29_zero<Fs>();  // Norm, < 2p
    return [&, sc](uint32_t k2, uint32_t r, F29<Fs> v) {
      if (use_scale) v = f29_mul_c<Fs>(v, sc);
      g_st29<Fs>(out, (size_t)(row0 + r) + (size_t)n1 * k2, f29_canon<Fs>(v));
    };
  });
}

}  // namespace pm

// msm_small.hpp -- the small-MSM path (n <= kSmallMaxN): two launches, no sort.
//
// halo2 also calls best_multiexp on short vectors (the verifier's and the
// multiopen's MSMs, [3P] src/poly/multiopen/*.rs, examples/simple-example.rs:
// 722), where the Pippenger pipeline's fixed cost (eight launches, two
// copies, a 256-position host Horner: ~0.25 ms at n = 1, bench.py small_n)
// dwarfs the work.  Here:
//   k_small_table   per base P_i: the multiples [1..8] P_i (XYZZ, R = 2^261,
//                   one quad per point per wave: [2]P; [4]P, [3]P; [8]P, [6]P,
//                   [5]P, [7]P -- three levels of quad-cooperative operations);
//                   in separate blocks of the same launch, from the scalar,
//                   the GLV halves k = k1 + lambda k2 (|k_h| < 2^127,
//                   glv.hpp) recoded into 33 signed 4-bit digits in [-8, 8]
//                   each (the half's sign folded in)
//   k_small_sum     block (s, j): window j's sum over terms [s kq 64, (s+1) kq
//                   64) of the 2n (point, half) terms: each of 64 quads adds
//                   kq selected table entries (phi(P) = (beta X, Y, ZZ, ZZZ),
//                   a negative digit negates Y), an LDS tree folds the 64
//                   quads, and with ns > 1 slices the last block of window j
//                   (atomic ticket) folds the ns partials.  Window sums go out
//                   Jacobian, in the R = 2^256 layout, straight into mapped
//                   host memory.
// The host finishes with a 33-window Jacobian Horner (128 doublings, 32
// additions, host_ec.hpp jdbl / jadd): the serial chain
// of ANY variable-base MSM is ~log2 r / 2 doublings after GLV, at ~2.2-2.4 us
// per doubling on one wave (profiles/r04/chain_latency.jsonl, ladder_dbl) but
// ~0.1-0.3 us on a host core, so the chain stays on the host.
#pragma once
#include "coop29.hpp"
#include "glv.hpp"
#include "msm_kernels.hpp"

namespace pm {

constexpr int kSmallWin = 33;          // 4-bit windows of a 128-bit GLV half (+ the carry window)
constexpr int kSmallMults = 8;         // table entries per base: [1..8] P
constexpr int kSmallTabPts = 16;       // k_small_table: bases per block (one per quad of each wave)
constexpr int kSmallQuads = 64;        // k_small_sum: quads per block
constexpr int kSmallPt = 36;           // an unpacked Xyzz29 in LDS (u32 words)
// k_small_fused up to here (one slice per window).  Several slices per window
// (one term per quad, the last block folding) measured slower than table + sum
// from 64 points on (64 / 128 / 256: 86.6-87.1 / 92.3-93.1 / 95.1-100.8 us
// against 83.4 / 89.0 / 95.1; profiles/r04/small/fused_ab.jsonl)
constexpr uint32_t kSmallFusedN = 32;

struct SmallGeom {
  uint32_t n;          // bases
  uint32_t canonical;  // scalars canonical (else Montgomery R = 2^256)
  uint32_t r261;       // bases already in the pipeline's packed R = 2^261 form (pm_bases)
  uint32_t kq;         // terms per quad and slice
  uint32_t ns;         // slices per window
};

// lane q of a quad writes coordinate q of p (9 words); every lane reads all 36
template <class F>
__device__ __forceinline__ void lds_put_q(uint32_t* s, const Xyzz29<F>& p, uint32_t q) {
  const F29<F> c = qsel<F>(q, p.X, p.Y, p.ZZ, p.ZZZ);
#pragma unroll
  for (int i = 0; i < 9; i++) s[q * 9 + i] = c.l[i];
}
template <class F>
__device__ __forceinline__ Xyzz29<F> lds_get(const uint32_t* s) {
  Xyzz29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    r.X.l[i] = s[i];
    r.Y.l[i] = s[9 + i];
    r.ZZ.l[i] = s[18 + i];
    r.ZZZ.l[i] = s[27 + i];
  }
  return r;
}
// lane q of a quad stores coordinate q of p in the packed Xyzz<F> layout
template <class F>
__device__ __forceinline__ void store_xyzz29_q(Xyzz<F>* dst, const Xyzz29<F>& p, uint32_t q) {
  st29<F>(reinterpret_cast<uint4*>(dst) + 2 * q, qsel<F>(q, p.X, p.Y, p.ZZ, p.ZZZ));
}

// lane k of a quad stores coordinate k of p's Jacobian form (X ZZ^2, Y ZZZ^2,
// ZZZ, 0) -- x = X / ZZ, y = Y / ZZZ and ZZ^3 = ZZZ^2 for every XYZZ point the
// group law produces -- in the R = 2^256 layout (the host Horner's input,
// host_ec.hpp jadd; the identity, ZZ = ZZZ = 0, becomes Z = 0)
template <class F>
__device__ __forceinline__ void store_jac_r256_q(Xyzz<F>* dst, const Xyzz29<F>& p, uint32_t lk) {
  const F29<F> z = qsel<F>(lk, p.ZZ, p.ZZZ, p.ZZ, p.ZZZ);
  const F29<F> sq = f29_mul_c<F>(z, z);
  const F29<F> zz2 = qbc<0, F>(sq), zzz2 = qbc<1, F>(sq);
  const F29<F> pr = f29_mul_c<F>(qsel<F>(lk, p.X, p.Y, p.X, p.Y), qsel<F>(lk, zz2, zzz2, zz2, zzz2));
  const F29<F> c = qsel<F>(lk, pr, pr, p.ZZZ, f29_zero<F>());
  uint32_t o[8];
  f29_to_r256<F>(c, o);
  uint4* q = reinterpret_cast<uint4*>(dst);
  q[2 * lk] = make_uint4(o[0], o[1], o[2], o[3]);
  q[2 * lk + 1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// k mod r for a 256-bit k (canonical-flag scalars may exceed r; 2^256 < 6 r
// on all three curves)
template <class Fs>
__device__ __forceinline__ Fe<Fs> fe_reduce_full(Fe<Fs> k) {
#pragma unroll
  for (int t = 0; t < 5; t++) k = fe_reduce_once<Fs>(k.l, 0u);
  return k;
}

// one GLV half (< 2^127, 4 words) -> 33 signed digits d_w in [-8, 8],
// sum_w d_w 16^w = k, stored at dst[w * stride]
__device__ __forceinline__ void small_recode(const uint32_t* k, bool neg, int8_t* dst, size_t stride) {
  uint32_t carry = 0;
#pragma unroll
  for (int w = 0; w < kSmallWin; w++) {
    const uint32_t nib = w < 32 ? (k[w >> 3] >> ((w & 7) * 4)) & 15u : 0u;
    const uint32_t v = nib + carry;  // <= 16
    carry = v >= 8u ? 1u : 0u;
    int d = (int)v - (carry ? 16 : 0);
    if (neg) d = -d;
    dst[(size_t)w * stride] = (int8_t)d;
  }
}

// blocks [0, nb_tab): the table, one quad per base per wave, 16 bases per
// block; blocks [nb_tab, ...): the digits, one lane per scalar (kept out of
// the table blocks, where the split's ~5 us held every level's barrier)
template <class Cv>
__global__ void __launch_bounds__(256) k_small_table(SmallGeom g, uint32_t nb_tab, const uint32_t* __restrict__ scalars,
                                                     const uint32_t* __restrict__ bases,
                                                     Xyzz<typename Cv::Base>* __restrict__ tab,
                                                     int8_t* __restrict__ digits) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  __shared__ uint32_t s_m[3][kSmallTabPts][kSmallPt];  // [2]P, [3]P, [4]P
  if (blockIdx.x >= nb_tab) {  // digits of scalar i (zero for an identity base)
    const uint32_t i = (blockIdx.x - nb_tab) * blockDim.x + threadIdx.x;
    if (i >= g.n) return;
    const size_t T = 2ull * g.n;
    int8_t* dst = digits + 2ull * i;
    const uint4* p = reinterpret_cast<const uint4*>(bases + 16ull * i);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    const bool ident = ((a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) | (c.x | c.y | c.z | c.w | d.x | d.y | d.z | d.w)) == 0;
    if (ident) {
      for (int w = 0; w < kSmallWin; w++) dst[(size_t)w * T] = dst[(size_t)w * T + 1] = 0;
      return;
    }
    Fe<Fs> k = load_canonical<Fs>(scalars, i, g.canonical);
    if (g.canonical) k = fe_reduce_full<Fs>(k);
    uint32_t k1[6], k2[6];
    bool n1, n2;
    glv_split<Cv, true>(k, k1, k2, n1, n2);
    small_recode(k1, n1, dst, T);
    small_recode(k2, n2, dst + 1, T);
    return;
  }
  const uint32_t wave = threadIdx.x >> 6, v = (threadIdx.x >> 2) & (kSmallTabPts - 1), q = threadIdx.x & 3u;
  const uint32_t i = blockIdx.x * kSmallTabPts + v;
  const bool valid = i < g.n;
  // base i: the identity (all-zero bytes) gets an all-identity table
  F29<F> x = f29_zero<F>(), y = f29_zero<F>();
  bool ident = true;
  if (valid) {
    const uint4* p = reinterpret_cast<const uint4*>(bases + 16ull * i);
    const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
    ident = ((a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) | (c.x | c.y | c.z | c.w | d.x | d.y | d.z | d.w)) == 0;
    const uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t wy[8] = {c.x, c.y, c.z, c.w, d.x, d.y, d.z, d.w};
    if (g.r261) {
      x = f29_unpack<F>(wx);
      y = f29_unpack<F>(wy);
    } else {
      x = f29_from_r256<F>(wx);
      y = f29_from_r256<F>(wy);
    }
  }
  const F29<F> one = f29_const<F>(F29Consts<F>::ONE);
  const Xyzz29<F> M1 = ident ? xyzz29_inf<F>() : Xyzz29<F>{x, y, one, one};
  Xyzz<F>* row = tab + (size_t)i * kSmallMults;
  // level 1: [2]P
  if (wave == 0) {
    const Xyzz29<F> M2 = xyzz29_dbl_q<F>(M1);
    lds_put_q<F>(s_m[0][v], M2, q);
    if (valid) {
      store_xyzz29_q<F>(&row[0], M1, q);
      store_xyzz29_q<F>(&row[1], M2, q);
    }
  }
  __syncthreads();
  // level 2: [4]P = 2 [2]P, [3]P = [2]P + P
  if (wave < 2) {
    const Xyzz29<F> M2 = lds_get<F>(s_m[0][v]);
    const Xyzz29<F> r = wave == 0 ? xyzz29_dbl_q<F>(M2) : xyzz29_add_q<F>(M2, M1);
    lds_put_q<F>(s_m[wave == 0 ? 2 : 1][v], r, q);
    if (valid) store_xyzz29_q<F>(&row[wave == 0 ? 3 : 2], r, q);
  }
  __syncthreads();
  // level 3: [8]P = 2 [4]P, [6]P = 2 [3]P, [5]P = [4]P + P, [7]P = [4]P + [3]P
  {
    const Xyzz29<F> M4 = lds_get<F>(s_m[2][v]);
    const Xyzz29<F> M3 = lds_get<F>(s_m[1][v]);
    Xyzz29<F> r;
    if (wave == 0) r = xyzz29_dbl_q<F>(M4);
    else if (wave == 1) r = xyzz29_dbl_q<F>(M3);
    else r = xyzz29_add_q<F>(M4, wave == 2 ? M1 : M3);
    const uint32_t slot = wave == 0 ? 7u : wave == 1 ? 5u : wave == 2 ? 4u : 6u;
    if (valid) store_xyzz29_q<F>(&row[slot], r, q);
  }
}

// fold the quads' points: on entry every quad v < cnt (a power of two <= 64)
// holds acc; on exit quad 0 holds the sum.  One barrier per level: level m
// reads slots [m, 2m) (written at level 2m) and writes [0, m).
template <class F>
__device__ __forceinline__ Xyzz29<F> small_tree(uint32_t (*s_p)[kSmallPt], Xyzz29<F> acc, uint32_t v, uint32_t q,
                                                uint32_t cnt) {
  if (cnt <= 1) return acc;
  if (v < cnt) lds_put_q<F>(s_p[v], acc, q);
  __syncthreads();
  for (uint32_t m = cnt >> 1; m > 0; m >>= 1) {
    if (v < m) {
      acc = xyzz29_add_q<F>(acc, lds_get<F>(s_p[v + m]));
      if (m > 1) lds_put_q<F>(s_p[v], acc, q);
    }
    __syncthreads();
  }
  return acc;
}

__device__ __forceinline__ uint32_t small_pow2(uint32_t x) {
  uint32_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

// c ? a : b limb by limb (bitwise selects: a select of whole objects became
// scratch-memory address selects, coop29.hpp)
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_pick(bool c, const Xyzz29<F>& a, const Xyzz29<F>& b) {
  const uint32_t m = c ? ~0u : 0u;
  Xyzz29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    r.X.l[i] = bsel(m, a.X.l[i], b.X.l[i]);
    r.Y.l[i] = bsel(m, a.Y.l[i], b.Y.l[i]);
    r.ZZ.l[i] = bsel(m, a.ZZ.l[i], b.ZZ.l[i]);
    r.ZZZ.l[i] = bsel(m, a.ZZZ.l[i], b.ZZZ.l[i]);
  }
  return r;
}

// quad 0 of the block that completes window j: the window sum goes to the
// host (Jacobian, R = 2^256), and the last of the 33 windows to finish raises
// the host's completion flag to seq (msm_small_impl spins on it instead of
// waiting for the kernel's completion signal)
template <class F>
__device__ __forceinline__ void small_finish(Xyzz<F>* out, uint32_t j, const Xyzz29<F>& acc, uint32_t q,
                                             uint32_t* done, uint32_t* flag, uint32_t seq) {
  store_jac_r256_q<F>(&out[j], acc, q);
  __threadfence_system();
  if (q == 0 && atomicAdd(done, 1u) == (uint32_t)kSmallWin - 1u) {
    *done = 0;  // every window has counted: ready for the next MSM
    __threadfence_system();
    *(volatile uint32_t*)flag = seq;
  }
}

// table entry of term t with digit d != 0: [|d|] P_i, phi'd for the second
// GLV half (t odd), negated for d < 0
template <class Cv>
__device__ __forceinline__ Xyzz29<typename Cv::Base> small_term(const Xyzz<typename Cv::Base>* __restrict__ tab,
                                                                 uint32_t t, int d) {
  using F = typename Cv::Base;
  using K = F29Consts<F>;
  Xyzz29<F> P = load_xyzz29<F>(&tab[(size_t)(t >> 1) * kSmallMults + (uint32_t)(d < 0 ? -d : d) - 1u]);
  if (t & 1u) P.X = f29_mul_c<F>(f29_const<F>(Glv<Cv>::BETA29), P.X);  // phi(P), X < 2p
  if (d < 0) P.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), P.Y, K::K6)));  // < 3p
  return P;
}

// after the block's tree (quad 0 holds slice s's sum of window j): with one
// slice, finish window j; else park the partial, and the last slice's block
// (atomic ticket) folds the ns partials and finishes it
template <class F>
__device__ __forceinline__ void small_fold(const SmallGeom& g, uint32_t (*s_p)[kSmallPt], uint32_t* last,
                                           Xyzz29<F> acc, uint32_t s, uint32_t j, uint32_t v, uint32_t q,
                                           Xyzz<F>* __restrict__ part, uint32_t* __restrict__ tickets,
                                           Xyzz<F>* __restrict__ out, uint32_t* done, uint32_t* flag, uint32_t seq) {
  if (g.ns > 1) {
    if (v == 0) {
      store_xyzz29_q<F>(&part[(size_t)j * g.ns + s], acc, q);
      __threadfence();
      if (q == 0) *last = atomicAdd(&tickets[j], 1u) == g.ns - 1u;
    }
    __syncthreads();
    if (!*last) return;
    __threadfence();
    acc = xyzz29_inf<F>();
    for (uint32_t u = v; u < g.ns; u += kSmallQuads) acc = xyzz29_add_q<F>(acc, load_xyzz29<F>(&part[(size_t)j * g.ns + u]));
    acc = small_tree<F>(s_p, acc, v, q, small_pow2(g.ns < (uint32_t)kSmallQuads ? g.ns : (uint32_t)kSmallQuads));
    if (v == 0 && q == 0) tickets[j] = 0;  // ready for the next MSM
  }
  if (v == 0) small_finish<F>(out, j, acc, q, done, flag, seq);
}

// Up to kSmallFusedN points: one launch, block (s, j) = slice s of window j,
// one quad per term (64 terms per slice; several slices are folded by the
// last block of the window, small_fold).
// The quad builds its own term [d] (+-phi^h P) from the affine base: [2]P,
// [4]P, [8]P and at most one addition ([3] = [2] + [1], [5] = [4] + [1], [6] =
// [4] + [2], [7] = [8] - [1]) -- four operations, against the table kernel's
// three levels plus a launch and a round trip through memory -- then the
// LDS tree.  The GLV split and recoding run per quad (only digit j is kept).
// TRACE (tools/microbench_small.hip only): thread 0 of block 0 records the
// real-time clock at each phase boundary into tr[0..7]
template <class Cv, bool TRACE = false>
__global__ void __launch_bounds__(256) k_small_fused(SmallGeom g, const uint32_t* __restrict__ scalars,
                                                     const uint32_t* __restrict__ bases,
                                                     Xyzz<typename Cv::Base>* __restrict__ part,
                                                     uint32_t* __restrict__ tickets,
                                                     Xyzz<typename Cv::Base>* __restrict__ out,
                                                     uint32_t* __restrict__ done, uint32_t* __restrict__ flag,
                                                     uint32_t seq, uint64_t* __restrict__ tr = nullptr) {
  const bool rec = TRACE && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
  if (rec) tr[0] = wall_clock64();
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  using K = F29Consts<F>;
  __shared__ uint32_t s_p[kSmallQuads][kSmallPt];
  __shared__ uint32_t last;
  const uint32_t s = blockIdx.x, j = blockIdx.y, v = threadIdx.x >> 2, q = threadIdx.x & 3u;
  const uint32_t T = 2u * g.n, t = s * kSmallQuads + v, i = t >> 1, h = t & 1u;
  Xyzz29<F> acc = xyzz29_inf<F>();
  int d = 0;
  F29<F> x = f29_zero<F>(), y = f29_zero<F>();
  if (t < T) {
    const uint4* p = reinterpret_cast<const uint4*>(bases + 16ull * i);
    const uint4* sp = reinterpret_cast<const uint4*>(scalars + 8ull * i);
    // the scalar's loads go out with the base's (one host-memory round trip, not two)
    const uint4 a = p[0], b = p[1], c = p[2], e = p[3], s0 = sp[0], s1 = sp[1];
    const bool ident = ((a.x | a.y | a.z | a.w | b.x | b.y | b.z | b.w) | (c.x | c.y | c.z | c.w | e.x | e.y | e.z | e.w)) == 0;
    const uint32_t wx[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    const uint32_t wy[8] = {c.x, c.y, c.z, c.w, e.x, e.y, e.z, e.w};
    if (g.r261) {
      x = f29_unpack<F>(wx);
      y = f29_unpack<F>(wy);
    } else {
      x = f29_from_r256<F>(wx);
      y = f29_from_r256<F>(wy);
    }
    if (h) x = f29_mul_c<F>(f29_const<F>(Glv<Cv>::BETA29), x);  // phi(P): independent of the split below
    if (rec) tr[1] = wall_clock64() + (x.l[0] & 0u);
    if (!ident) {
      Fe<Fs> k;
      const uint32_t kw[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
      for (int w = 0; w < 8; w++) k.l[w] = kw[w];
      k = g.canonical ? fe_reduce_full<Fs>(k) : fe_from_mont<Fs>(k);
      if (rec) tr[2] = wall_clock64() + (k.l[0] & 0u);
      uint32_t k1[6], k2[6];
      bool n1, n2;
      glv_split<Cv, true>(k, k1, k2, n1, n2);
      if (rec) tr[3] = wall_clock64() + (k1[0] & 0u);
      const uint32_t* kh = h ? k2 : k1;
      uint32_t carry = 0;
#pragma unroll
      for (int w = 0; w < kSmallWin; w++) {  // the recoding of small_recode, digit j kept
        const uint32_t nib = w < 32 ? (kh[w >> 3] >> ((w & 7) * 4)) & 15u : 0u;
        const uint32_t u = nib + carry;
        carry = u >= 8u ? 1u : 0u;
        if ((uint32_t)w == j) d = (int)u - (carry ? 16 : 0);
      }
      if (h ? n2 : n1) d = -d;
    }
  }
  if (rec) tr[4] = wall_clock64() + ((uint32_t)d & 0u);
  if (d != 0) {  // quad-uniform
    // [d] (+-phi^h P) = [|d|] of the base with phi (above) and the sign
    // applied first: no product after the chain
    if (d < 0) y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), y, K::K6)));
    const F29<F> one = f29_const<F>(K::ONE);
    const Xyzz29<F> P1{x, y, one, one};
    const Xyzz29<F> P2 = xyzz29_dbl_q<F>(P1);
    const Xyzz29<F> P4 = xyzz29_dbl_q<F>(P2);
    const Xyzz29<F> P8 = xyzz29_dbl_q<F>(P4);
    if (rec) tr[5] = wall_clock64() + (P8.X.l[0] & 0u);
    const uint32_t m = (uint32_t)(d < 0 ? -d : d);
    // [m] = A + B: (P1, -), (P2, -), (P2, P1), (P4, -), (P4, P1), (P4, P2), (P8, -P1), (P8, -)
    const Xyzz29<F> A = xyzz29_pick<F>(m == 1, P1, xyzz29_pick<F>(m <= 3, P2, xyzz29_pick<F>(m <= 6, P4, P8)));
    Xyzz29<F> B = xyzz29_pick<F>(m == 6, P2, P1);
    if (m == 7) B.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), B.Y, K::K6)));
    B = xyzz29_pick<F>(m == 3 || (m >= 5 && m <= 7), B, xyzz29_inf<F>());
    acc = xyzz29_add_q<F>(A, B);
  }
  if (rec) tr[6] = wall_clock64() + (acc.X.l[0] & 0u);
  const uint32_t active = T - s * kSmallQuads >= (uint32_t)kSmallQuads ? (uint32_t)kSmallQuads : T - s * kSmallQuads;
  acc = small_tree<F>(s_p, acc, v, q, small_pow2(active));
  if (rec) tr[7] = wall_clock64() + (acc.X.l[0] & 0u);
  small_fold<F>(g, s_p, &last, acc, s, j, v, q, part, tickets, out, done, flag, seq);
  if (rec) tr[8] = wall_clock64();
}

// block (s, j), quads: quad v adds terms t0 + r 64 + v, r < kq (quad-
// cooperative additions, ~3.2 us each), then the 64-quad tree
template <class Cv>
__global__ void __launch_bounds__(256) k_small_sum(SmallGeom g, const Xyzz<typename Cv::Base>* __restrict__ tab,
                                                   const int8_t* __restrict__ digits,
                                                   Xyzz<typename Cv::Base>* __restrict__ part,
                                                   uint32_t* __restrict__ tickets,
                                                   Xyzz<typename Cv::Base>* __restrict__ out, uint32_t* __restrict__ done,
                                                   uint32_t* __restrict__ flag, uint32_t seq) {
  using F = typename Cv::Base;
  __shared__ uint32_t s_p[kSmallQuads][kSmallPt];
  __shared__ uint32_t last;
  const uint32_t s = blockIdx.x, j = blockIdx.y, v = threadIdx.x >> 2, q = threadIdx.x & 3u;
  const uint32_t T = 2u * g.n, t0 = s * g.kq * kSmallQuads;
  const int8_t* dj = digits + (size_t)j * T;
  Xyzz29<F> acc = xyzz29_inf<F>();
  for (uint32_t r = 0; r < g.kq; r++) {
    const uint32_t t = t0 + r * kSmallQuads + v;
    if (t >= T) break;  // quad-uniform
    const int d = dj[t];
    if (d != 0) acc = xyzz29_add_q<F>(acc, small_term<Cv>(tab, t, d));
  }
  // quads holding at least one term
  const uint32_t active = T - t0 >= (uint32_t)kSmallQuads ? (uint32_t)kSmallQuads : T - t0;
  acc = small_tree<F>(s_p, acc, v, q, small_pow2(active));
  small_fold<F>(g, s_p, &last, acc, s, j, v, q, part, tickets, out, done, flag, seq);
}

// block (s, j), lanes (many terms per slice): lane l adds terms t0 + r 256 +
// l, r < kq, with one-lane additions (~6 us each but four in flight per quad:
// twice the quads' addition rate), then 256 -> 128 by one-lane additions and
// the 64-quad tree on the rest
template <class Cv>
__global__ void __launch_bounds__(256) k_small_sum_lanes(SmallGeom g, const Xyzz<typename Cv::Base>* __restrict__ tab,
                                                         const int8_t* __restrict__ digits,
                                                         Xyzz<typename Cv::Base>* __restrict__ part,
                                                         uint32_t* __restrict__ tickets,
                                                         Xyzz<typename Cv::Base>* __restrict__ out,
                                                         uint32_t* __restrict__ done, uint32_t* __restrict__ flag,
                                                         uint32_t seq) {
  using F = typename Cv::Base;
  __shared__ uint32_t s_p[256][kSmallPt];
  __shared__ uint32_t last;
  const uint32_t s = blockIdx.x, j = blockIdx.y, l = threadIdx.x, v = l >> 2, q = l & 3u;
  const uint32_t T = 2u * g.n, t0 = s * g.kq * 256u;
  const int8_t* dj = digits + (size_t)j * T;
  Xyzz29<F> acc = xyzz29_inf<F>();
  for (uint32_t r = 0; r < g.kq; r++) {
    const uint32_t t = t0 + r * 256u + l;
    if (t >= T) break;
    const int d = dj[t];
    if (d != 0) acc = xyzz29_add<F>(acc, small_term<Cv>(tab, t, d));
  }
#pragma unroll
  for (int i = 0; i < 9; i++) {
    s_p[l][i] = acc.X.l[i];
    s_p[l][9 + i] = acc.Y.l[i];
    s_p[l][18 + i] = acc.ZZ.l[i];
    s_p[l][27 + i] = acc.ZZZ.l[i];
  }
  __syncthreads();
  if (l < 128) {
    acc = xyzz29_add<F>(acc, lds_get<F>(s_p[l + 128]));
#pragma unroll
    for (int i = 0; i < 9; i++) {
      s_p[l][i] = acc.X.l[i];
      s_p[l][9 + i] = acc.Y.l[i];
      s_p[l][18 + i] = acc.ZZ.l[i];
      s_p[l][27 + i] = acc.ZZZ.l[i];
    }
  }
  __syncthreads();
  // quad v folds slots v and v + 64, then writes only slot v (read by quad v alone)
  acc = xyzz29_add_q<F>(lds_get<F>(s_p[v]), lds_get<F>(s_p[v + 64]));
  acc = small_tree<F>(s_p, acc, v, q, kSmallQuads);
  small_fold<F>(g, s_p, &last, acc, s, j, v, q, part, tickets, out, done, flag, seq);
}

}  // namespace pm

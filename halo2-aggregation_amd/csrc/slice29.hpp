// slice29.hpp -- row-sliced radix-2^29 field elements for latency-bound chains.
//
// A lone wave issues one v_mad_u64_u32 every ~8.8 cycles and a simple VALU op
// every ~5 whatever the dependency structure, so a one-lane
// Montgomery product (fp29.hpp: 135 multiply-adds, ~183 instructions) costs
// ~0.46 us of latency, and the accumulator's serial chains (the proof points'
// square roots, the 127-doubling ladder) are long chains of such products.
// When few chains are resident (config 3's 16 proofs, config 5's 32-proof
// rank slices) most SIMDs idle, and spreading ONE product over the 16 lanes of
// a DPP row shortens it: here a field element is ONE VGPR, lane l (= lane &
// 15) holding limb l for l < 9 and 0 in lanes 9..15, and the four rows of a
// wave hold four independent elements.
//
// Product (CIOS, operand scanning, one limb of b per step): for j = 0..8
//   T_l += a_l b_j                  (b_j: row broadcast of lane j, DPP row_newbcast)
//   t    = T_0 + c                  (T_0: 64-bit row broadcast of lane 0; c the carry)
//   m    = t (-p^-1) mod 2^29,  c = (t + m p_0) >> 29
//   T_l += m p_l   (l >= 1)         (lane 0 is dropped: its value lives on in c)
//   T_l  = T_{l+1}                  (DPP row_shl:1, two 32-bit moves)
// -- 2 multiply-adds per lane per step instead of ~15, 18 in all, ~11
// instructions per step -- then c goes into lane 0 and three rounds of
// parallel carries (lo + the lower lane's hi) bring every limb to <= 2^29.
// Same value as f29_mul (Montgomery, R = 2^261, result < 2p for the same
// operand bounds: limbs <= 2^30, a b < R p; column sums <= 9 2^60 + 9 2^58 +
// 2^35 < 2^64).  Linear steps are lane-parallel: an addition is one
// instruction, a normalisation three carry rounds.
#pragma once
#include "fp29.hpp"

namespace pm {

template <class F>
struct S29 {
  uint32_t v;
};

__device__ __forceinline__ uint32_t s_lane() { return threadIdx.x & 15u; }

// DPP row operations (gfx950: row_newbcast also on 64-bit moves)
// (a broadcast writes every lane: mov_dpp, no "old" operand to initialise)
template <int J>
__device__ __forceinline__ uint32_t rbc32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x150 + J, 0xF, 0xF, false);
}
// 64-bit broadcast of lane 0 into a fresh register (the builtin ties its
// destination to an "old" operand and copies it first); the s_nop covers the
// VALU-write -> DPP-read hazard the compiler does not see through the asm
__device__ __forceinline__ uint64_t rbc64_0(uint64_t v) {
  uint64_t r;
  asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v));
  return r;
}
// lane l <- lane l + 1 (lane 15 <- 0)
__device__ __forceinline__ uint32_t rshl1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ uint64_t rshl1_64(uint64_t v) {
  return (uint64_t)rshl1((uint32_t)v) | (uint64_t)rshl1((uint32_t)(v >> 32)) << 32;
}
// lane l <- lane l - 1 (lane 0 <- 0)
__device__ __forceinline__ uint32_t rshr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint64_t rshr1_64(uint64_t v) {
  return (uint64_t)rshr1((uint32_t)v) | (uint64_t)rshr1((uint32_t)(v >> 32)) << 32;
}

// per-lane constant: lane l < 9 gets c[l], lanes 9..15 get 0
__device__ __forceinline__ uint32_t s_limbs(const uint32_t (&c)[9]) {
  const uint32_t l = s_lane();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) r = l == (uint32_t)i ? c[i] : r;
  return r;
}

// The constants a sliced chain keeps in VGPRs (one register each)
template <class F>
struct SConst {
  uint32_t pnz;  // p_l for 1 <= l <= 8, 0 in lane 0 and lanes 9..15
  uint32_t p, k6, k8x3, k2, one, k12;
  __device__ static SConst make() {
    using K = F29Consts<F>;
    SConst c;
    c.p = s_limbs(K::P);
    c.pnz = s_lane() == 0 ? 0u : c.p;
    c.k6 = s_limbs(K::K6);
    c.k8x3 = s_limbs(K::K8x3);
    c.k2 = s_limbs(K::K2);
    c.one = s_limbs(K::ONE);
    c.k12 = s_limbs(F29K12<F>::L);
    return c;
  }
};

// one lane's F29 (the same in every lane of the row) -> sliced
template <class F>
__device__ __forceinline__ S29<F> s29_from(const F29<F>& x) {
  const uint32_t l = s_lane();
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) r = l == (uint32_t)i ? x.l[i] : r;
  return S29<F>{r};
}
// sliced -> F29 in every lane of the row
template <class F>
__device__ __forceinline__ F29<F> s29_to(S29<F> a) {
  F29<F> r;
  r.l[0] = rbc32<0>(a.v);
  r.l[1] = rbc32<1>(a.v);
  r.l[2] = rbc32<2>(a.v);
  r.l[3] = rbc32<3>(a.v);
  r.l[4] = rbc32<4>(a.v);
  r.l[5] = rbc32<5>(a.v);
  r.l[6] = rbc32<6>(a.v);
  r.l[7] = rbc32<7>(a.v);
  r.l[8] = rbc32<8>(a.v);
  return r;
}

// one CIOS step j (see the header comment)
template <class F, int J>
__device__ __forceinline__ void s29_step(uint32_t a, uint32_t b, uint32_t pnz, uint64_t& T, uint64_t& c) {
  using K = F29Consts<F>;
  T += (uint64_t)a * rbc32<J>(b);
  const uint64_t t = rbc64_0(T) + c;
  uint32_t m;
  if constexpr (K::INV == kM29) m = (0u - (uint32_t)t) & kM29;
  else m = ((uint32_t)t * K::INV) & kM29;
  c = (t + (uint64_t)m * K::P[0]) >> 29;
  T += (uint64_t)m * pnz;
  T = rshl1_64(T);
}

// three rounds of parallel carries: limbs <= 2^29 (value unchanged)
__device__ __forceinline__ uint32_t s29_carry64(uint64_t T) {
  const uint64_t t1 = (T & kM29) + rshr1_64(T >> 29);            // < 2^29 + 2^35
  const uint32_t t2 = ((uint32_t)t1 & kM29) + rshr1((uint32_t)(t1 >> 29));  // < 2^29 + 2^7
  return (t2 & kM29) + rshr1(t2 >> 29);                          // <= 2^29
}

// Montgomery product a b 2^-261 (the value of f29_mul)
template <class F>
__device__ __forceinline__ S29<F> s29_mul(S29<F> a, S29<F> b, const SConst<F>& k) {
  uint64_t T = 0, c = 0;
  s29_step<F, 0>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 1>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 2>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 3>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 4>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 5>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 6>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 7>(a.v, b.v, k.pnz, T, c);
  s29_step<F, 8>(a.v, b.v, k.pnz, T, c);
  T += s_lane() == 0 ? c : 0ull;
  return S29<F>{s29_carry64(T)};
}

// ---------------------------------------------------------- linear steps
template <class F>
__device__ __forceinline__ S29<F> s29_add(S29<F> a, S29<F> b) {
  return S29<F>{a.v + b.v};
}
// a + K - b (K a redundant multiple of p dominating b limb-wise)
template <class F>
__device__ __forceinline__ S29<F> s29_sub(S29<F> a, S29<F> b, uint32_t kl) {
  return S29<F>{a.v + kl - b.v};
}
// carry rounds for limbs < 2^32 - 2^29: limbs <= 2^29 afterwards (two rounds
// take limbs below 2^31.6 to <= 2^29 + 8, the third to <= 2^29)
template <class F>
__device__ __forceinline__ S29<F> s29_norm(S29<F> a) {
  uint32_t t = (a.v & kM29) + rshr1(a.v >> 29);
  t = (t & kM29) + rshr1(t >> 29);
  return S29<F>{(t & kM29) + rshr1(t >> 29)};
}
// exact normalisation (every limb < 2^29): carry rounds until no limb
// reaches 2^29 (row-uniform loop; usually no extra round)
template <class F>
__device__ __forceinline__ S29<F> s29_norm_exact(S29<F> a) {
  uint32_t t = s29_norm<F>(a).v;
  while (__builtin_amdgcn_ballot_w64(t > kM29 && s_lane() < 8u)) t = (t & kM29) + rshr1(t >> 29);
  return S29<F>{t};
}

// Norm-ish a (limbs <= 2^29 + small, value < 16p) -> exact Norm, < 3p:
// v - q p with q = floor(v_8 / (p_8 + 1)) (f29_reduce3's quotient), then
// signed carry rounds until every limb is in [0, 2^29) (the top lane keeps its
// carries: the value is non-negative, so it ends non-negative)
template <class F>
__device__ __forceinline__ S29<F> s29_norm_exact(S29<F> a);
template <class F>
__device__ __forceinline__ S29<F> s29_reduce3(S29<F> a_in, uint32_t pl) {
  using K = F29Consts<F>;
  const S29<F> a = s29_norm_exact<F>(a_in);  // the quotient from the exact top limb (f29_reduce3's q)
  const uint32_t q = (uint32_t)(((uint64_t)rbc32<8>(a.v) * K::QMAGIC) >> 40);
  const bool low = s_lane() < 8u;
  const int64_t t0 = (int64_t)a.v - (int64_t)q * pl;  // > -2^34 (the top lane's fits 32 bits)
  const int32_t hi0 = low ? (int32_t)(t0 >> 29) : 0;
  int32_t t = (int32_t)(low ? (uint32_t)t0 & kM29 : (uint32_t)t0) + (int32_t)rshr1((uint32_t)hi0);
  auto bad = [&](int32_t x) { return low && (x < 0 || x > (int32_t)kM29); };
  while (__builtin_amdgcn_ballot_w64(bad(t))) {
    const int32_t hi = low ? t >> 29 : 0;
    t = (low ? (int32_t)((uint32_t)t & kM29) : t) + (int32_t)rshr1((uint32_t)hi);
  }
  return S29<F>{(uint32_t)t};
}

// value of row K (lanes 16 K .. 16 K + 15) in every row (ds_bpermute)
template <int K>
__device__ __forceinline__ uint32_t s_row(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((((uint32_t)K << 4) | s_lane()) << 2), (int)v);
}
__device__ __forceinline__ uint32_t s_rowid() { return (threadIdx.x >> 4) & 3u; }

}  // namespace pm

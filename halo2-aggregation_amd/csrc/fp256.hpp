// fp256.hpp -- 255/254-bit prime-field arithmetic for gfx950 (and the host).
//
// Replaces the Montgomery field arithmetic of pasta_curves / pairing_bn256 that
// halo2's best_multiexp runs on ([3P], reached from
// /root/reference/examples/simple-example.rs:606,620,638-640).  Semantics match
// those crates: elements are kept in Montgomery form with R = 2^256, fully
// reduced to [0, p), so the in-memory limbs of a Rust `Fp` ([u64;4] LE) are
// bit-identical to the 8 x u32 LE limbs used here.
//
// Design (MI355X): one field element = 8 VGPRs per lane (32-bit limbs, since
// CDNA has no 64x64 multiply; 32x32->64 products lower to v_mad_u64_u32).
// Montgomery multiplication is CIOS with the modulus limbs as compile-time
// constants, so for the Pasta primes (p = 2^254 + small, limbs 4..6 zero,
// limb 7 = 2^30, p = 1 mod 2^32 => -p^-1 = 0xffffffff) the reduction half
// collapses to 3 real multiplies per row instead of 8.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define PM_HD __host__ __device__ __forceinline__
#else
#define PM_HD inline
#endif

namespace pm {

// ---------------------------------------------------------------- parameters
// Constants derived in tests/test_constants.py from the moduli in SURVEY.md
// Appendix A (INV = -p^-1 mod 2^32, ONE = R mod p, R2 = R^2 mod p).
struct PallasFp {  // Pallas base field == Vesta scalar field
  static constexpr uint32_t MOD[8] = {0x00000001u, 0x992d30edu, 0x094cf91bu, 0x224698fcu,
                                      0x00000000u, 0x00000000u, 0x00000000u, 0x40000000u};
  static constexpr uint32_t INV = 0xffffffffu;
  static constexpr uint32_t ONE[8] = {0xfffffffdu, 0x34786d38u, 0xe41914adu, 0x992c350bu,
                                      0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu};
  static constexpr uint32_t R2[8] = {0x0000000fu, 0x8c78ecb3u, 0x8b0de0e7u, 0xd7d30dbdu,
                                     0xc3c95d18u, 0x7797a99bu, 0x7b9cb714u, 0x096d41afu};
  static constexpr int NBITS = 255;
};
struct VestaFp {  // Vesta base field == Pallas scalar field
  static constexpr uint32_t MOD[8] = {0x00000001u, 0x8c46eb21u, 0x0994a8ddu, 0x224698fcu,
                                      0x00000000u, 0x00000000u, 0x00000000u, 0x40000000u};
  static constexpr uint32_t INV = 0xffffffffu;
  static constexpr uint32_t ONE[8] = {0xfffffffdu, 0x5b2b3e9cu, 0xe3420567u, 0x992c350bu,
                                      0xffffffffu, 0xffffffffu, 0xffffffffu, 0x3fffffffu};
  static constexpr uint32_t R2[8] = {0x0000000fu, 0xfc9678ffu, 0x891a16e3u, 0x67bb433du,
                                     0x04ccf590u, 0x7fae2310u, 0x7ccfdaa9u, 0x096d41afu};
  static constexpr int NBITS = 255;
};
struct Bn254Fq {  // BN254 G1 base field (reference's actual curve)
  static constexpr uint32_t MOD[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xe4866389u;
  static constexpr uint32_t ONE[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
  static constexpr int NBITS = 254;
};
struct Bn254Fr {  // BN254 scalar field
  static constexpr uint32_t MOD[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                      0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t INV = 0xefffffffu;
  static constexpr uint32_t ONE[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t R2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
  static constexpr int NBITS = 254;
};

// ------------------------------------------------------------------- element
template <class P>
struct Fe {
  uint32_t l[8];
};

// carry helpers (lower to v_add_co/v_addc_co, v_sub_co/v_subb_co on gfx950)
PM_HD uint32_t addc(uint32_t a, uint32_t b, uint32_t& c) {
  uint64_t s = (uint64_t)a + b + c;
  c = (uint32_t)(s >> 32);
  return (uint32_t)s;
}
PM_HD uint32_t subb(uint32_t a, uint32_t b, uint32_t& br) {
  uint64_t d = (uint64_t)a - b - br;
  br = (uint32_t)(d >> 63);
  return (uint32_t)d;
}

template <class P>
PM_HD Fe<P> fe_zero() {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = 0;
  return r;
}
template <class P>
PM_HD Fe<P> fe_one() {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = P::ONE[i];
  return r;
}
template <class P>
PM_HD bool fe_is_zero(const Fe<P>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.l[i];
  return o == 0;
}
template <class P>
PM_HD bool fe_eq(const Fe<P>& a, const Fe<P>& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= a.l[i] ^ b.l[i];
  return o == 0;
}

// r = t - p if (hi || t >= p) else t   (t < 2p)
template <class P>
PM_HD Fe<P> fe_reduce_once(const uint32_t t[8], uint32_t hi) {
  uint32_t d[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = subb(t[i], P::MOD[i], br);
  const bool take = hi || !br;
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = take ? d[i] : t[i];
  return r;
}

template <class P>
PM_HD Fe<P> fe_add(const Fe<P>& a, const Fe<P>& b) {
  uint32_t t[8], c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = addc(a.l[i], b.l[i], c);
  return fe_reduce_once<P>(t, c);
}

template <class P>
PM_HD Fe<P> fe_sub(const Fe<P>& a, const Fe<P>& b) {
  uint32_t t[8], br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = subb(a.l[i], b.l[i], br);
  // if borrow: add p back (mask trick keeps it branch-free)
  const uint32_t m = 0u - br;
  uint32_t c = 0;
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = addc(t[i], P::MOD[i] & m, c);
  return r;
}

template <class P>
PM_HD Fe<P> fe_neg(const Fe<P>& a) {
  return fe_sub<P>(fe_zero<P>(), a);
}

template <class P>
PM_HD Fe<P> fe_dbl(const Fe<P>& a) {
  return fe_add<P>(a, a);
}

// Montgomery product a*b*R^-1 mod p, CIOS, fully reduced (portable form;
// used on the host).
template <class P>
inline Fe<P> fe_mul_portable(const Fe<P>& a, const Fe<P>& b) {
  uint32_t t[10];
  for (int i = 0; i < 10; i++) t[i] = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t s = (uint64_t)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    uint64_t s = (uint64_t)t[8] + c;
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * P::INV;
    s = (uint64_t)m * P::MOD[0] + t[0];
    c = s >> 32;
    for (int j = 1; j < 8; j++) {
      s = (uint64_t)m * P::MOD[j] + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[8] + c;
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  return fe_reduce_once<P>(t, t[8]);
}

#if defined(__HIP_DEVICE_COMPILE__)
// 96-bit column accumulator (acc = 64-bit VGPR pair, acc2 = overflow word):
// acc += x*y with v_mad_u64_u32's carry-out (VCC) folded into acc2, i.e. two
// VALU instructions per 32x32 product.  VCC is produced and consumed inside
// one asm statement, so the compiler may interleave the statements freely.
__device__ __forceinline__ void mac_vv(uint64_t& acc, uint32_t& acc2, uint32_t x, uint32_t y) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_addc_co_u32_e64 %1, %3, 0, %1, %2"
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x), "v"(y));
}
// y = a modulus limb (compile-time constant, lives in an SGPR)
__device__ __forceinline__ void mac_vs(uint64_t& acc, uint32_t& acc2, uint32_t x, uint32_t y) {
  uint64_t c0, c1;
  asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\t"
      "v_addc_co_u32_e64 %1, %3, 0, %1, %2"
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x), "s"(y));
}

// Grouped forms: up to four products per asm statement.  The compiler pads
// every inline-asm statement that writes an SGPR with an s_nop before the next
// VALU statement; grouping keeps the (hazard-free) mad -> addc pairs inside one
// statement and removes 3 of every 4 of those pads.
#define PM_MAD2(X, Y) "v_mad_u64_u32 %0, %2, " X ", " Y ", %0\n\tv_addc_co_u32_e64 %1, %3, 0, %1, %2\n\t"
__device__ __forceinline__ void mac4_vv(uint64_t& acc, uint32_t& acc2, uint32_t x0, uint32_t y0, uint32_t x1,
                                        uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) {
  uint64_t c0, c1;
  asm(PM_MAD2("%4", "%5") PM_MAD2("%6", "%7") PM_MAD2("%8", "%9") PM_MAD2("%10", "%11")
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1), "v"(x2), "v"(y2), "v"(x3), "v"(y3));
}
__device__ __forceinline__ void mac2_vv(uint64_t& acc, uint32_t& acc2, uint32_t x0, uint32_t y0, uint32_t x1,
                                        uint32_t y1) {
  uint64_t c0, c1;
  asm(PM_MAD2("%4", "%5") PM_MAD2("%6", "%7")
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
}
__device__ __forceinline__ void mac4_vs(uint64_t& acc, uint32_t& acc2, uint32_t x0, uint32_t y0, uint32_t x1,
                                        uint32_t y1, uint32_t x2, uint32_t y2, uint32_t x3, uint32_t y3) {
  uint64_t c0, c1;
  asm(PM_MAD2("%4", "%5") PM_MAD2("%6", "%7") PM_MAD2("%8", "%9") PM_MAD2("%10", "%11")
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x0), "s"(y0), "v"(x1), "s"(y1), "v"(x2), "s"(y2), "v"(x3), "s"(y3));
}
__device__ __forceinline__ void mac2_vs(uint64_t& acc, uint32_t& acc2, uint32_t x0, uint32_t y0, uint32_t x1,
                                        uint32_t y1) {
  uint64_t c0, c1;
  asm(PM_MAD2("%4", "%5") PM_MAD2("%6", "%7")
      : "+v"(acc), "+v"(acc2), "=&s"(c0), "=&s"(c1)
      : "v"(x0), "s"(y0), "v"(x1), "s"(y1));
}
// acc += sum_{t<n} xs[t] * ys[t] in groups of 4 / 2 / 1 (n is a compile-time
// constant after unrolling)
template <bool YS>
__device__ __forceinline__ void mac_n(uint64_t& acc, uint32_t& acc2, const uint32_t* xs, const uint32_t* ys, int n) {
  int t = 0;
#pragma unroll
  for (; t + 4 <= n; t += 4) {
    if (YS) mac4_vs(acc, acc2, xs[t], ys[t], xs[t + 1], ys[t + 1], xs[t + 2], ys[t + 2], xs[t + 3], ys[t + 3]);
    else mac4_vv(acc, acc2, xs[t], ys[t], xs[t + 1], ys[t + 1], xs[t + 2], ys[t + 2], xs[t + 3], ys[t + 3]);
  }
  if (t + 2 <= n) {
    if (YS) mac2_vs(acc, acc2, xs[t], ys[t], xs[t + 1], ys[t + 1]);
    else mac2_vv(acc, acc2, xs[t], ys[t], xs[t + 1], ys[t + 1]);
    t += 2;
  }
  if (t < n) {
    if (YS) mac_vs(acc, acc2, xs[t], ys[t]);
    else mac_vv(acc, acc2, xs[t], ys[t]);
  }
}

// FIPS with grouped asm statements (same arithmetic as fe_mul_fips).
template <class P>
__device__ __forceinline__ Fe<P> fe_mul_fips_g(const Fe<P>& a, const Fe<P>& b) {
  uint32_t m[8], r[8];
  uint64_t acc = 0;
  uint32_t acc2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint32_t xs[8], ys[8], ms[8], ps[8];
    int n = 0, nr = 0;
    const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
#pragma unroll
    for (int i = lo; i <= hi; i++) {
      xs[n] = a.l[i];
      ys[n] = b.l[k - i];
      n++;
    }
#pragma unroll
    for (int i = lo; i <= hi && i < 8; i++)
      if (i < k && P::MOD[k - i] != 0u) {
        ms[nr] = m[i];
        ps[nr] = P::MOD[k - i];
        nr++;
      }
    mac_n<false>(acc, acc2, xs, ys, n);
    mac_n<true>(acc, acc2, ms, ps, nr);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac_vs(acc, acc2, m[k], P::MOD[0]);
    } else {
      r[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc2 = 0;
  }
  r[7] = (uint32_t)acc;
  return fe_reduce_once<P>(r, (uint32_t)(acc >> 32));
}

// Montgomery reduction alone, in the FIPS column form of fe_mul_fips_g:
// column k < 8 takes a_k (a multiply-add by 1) and sum m_i p_{k-i} over p's
// nonzero limbs, then m_k; columns 8..14 the remaining m_i p_{k-i}.  Pasta:
// 8 + 40 multiply-adds instead of fe_mul(a, 1)'s 104.
template <class P>
__device__ __forceinline__ Fe<P> fe_redc_fips_g(const Fe<P>& a) {
  uint32_t m[8], r[8];
  uint64_t acc = 0;
  uint32_t acc2 = 0;
#pragma unroll
  for (int k = 0; k < 15; k++) {
    uint32_t ms[8], ps[8];
    int nr = 0;
    const int lo = k < 8 ? 0 : k - 7, hi = k < 8 ? k : 7;
#pragma unroll
    for (int i = lo; i <= hi && i < 8; i++)
      if (i < k && P::MOD[k - i] != 0u) {
        ms[nr] = m[i];
        ps[nr] = P::MOD[k - i];
        nr++;
      }
    if (k < 8) mac_vs(acc, acc2, a.l[k], 1u);
    mac_n<true>(acc, acc2, ms, ps, nr);
    if (k < 8) {
      m[k] = (uint32_t)acc * P::INV;
      mac_vs(acc, acc2, m[k], P::MOD[0]);
    } else {
      r[k - 8] = (uint32_t)acc;
    }
    acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc2 = 0;
  }
  r[7] = (uint32_t)acc;
  return fe_reduce_once<P>(r, (uint32_t)(acc >> 32));
}

// Montgomery product by finely integrated product scanning (FIPS): column k
// accumulates sum a_i b_{k-i} + sum m_i p_{k-i}; the low columns also produce
// m_k = acc * (-p^-1) so that column k becomes divisible by 2^32.  Modulus
// limbs that are zero (Pasta: p_4..p_6) are skipped at compile time, so a
// Pasta product costs 64 + 32 + 8 multiply-adds.
template <class P>
__device__ __forceinline__ Fe<P> fe_mul_fips(const Fe<P>& a, const Fe<P>& b) {
  uint32_t m[8], r[8];
  uint64_t acc = 0;
  uint32_t acc2 = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) mac_vv(acc, acc2, a.l[i], b.l[k - i]);
#pragma unroll
    for (int i = 0; i < k; i++)
      if (P::MOD[k - i] != 0u) mac_vs(acc, acc2, m[i], P::MOD[k - i]);
    m[k] = (uint32_t)acc * P::INV;
    mac_vs(acc, acc2, m[k], P::MOD[0]);
    acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc2 = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; k++) {
#pragma unroll
    for (int i = k - 7; i < 8; i++) mac_vv(acc, acc2, a.l[i], b.l[k - i]);
#pragma unroll
    for (int i = k - 7; i < 8; i++)
      if (P::MOD[k - i] != 0u) mac_vs(acc, acc2, m[i], P::MOD[k - i]);
    r[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)acc2 << 32);
    acc2 = 0;
  }
  r[7] = (uint32_t)acc;
  return fe_reduce_once<P>(r, (uint32_t)(acc >> 32));
}

#endif

template <class P>
PM_HD Fe<P> fe_mul(const Fe<P>& a, const Fe<P>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fe_mul_fips_g<P>(a, b);
#else
  return fe_mul_portable<P>(a, b);
#endif
}

template <class P>
PM_HD Fe<P> fe_redc_portable(const Fe<P>& a);
template <class P>
PM_HD Fe<P> fe_redc(const Fe<P>& a) {
#if defined(__HIP_DEVICE_COMPILE__)
  return fe_redc_fips_g<P>(a);
#else
  return fe_redc_portable<P>(a);
#endif
}

template <class P>
PM_HD Fe<P> fe_sqr(const Fe<P>& a) {
  return fe_mul<P>(a, a);
}

// a R^-1 mod p for a < p (Montgomery -> canonical): the Montgomery reduction
// of the single-width a alone -- 8 rounds of m = t_0 (-p^-1) and t += m p,
// with p's zero limbs skipped at compile time (Pasta: 5 of 8), instead of a
// full product by 1 (the histogram pass spent 7 us of 29 at 2^20 and 34 of
// 97 us at 2^22 on it, profiles/r03/ab/hist_probe.jsonl).
template <class P>
PM_HD Fe<P> fe_redc_portable(const Fe<P>& a) {
  uint32_t t[8];
#pragma unroll
  for (int i = 0; i < 8; i++) t[i] = a.l[i];
  uint32_t top = 0;  // carry out of the window: t < 2^256 + p after each round
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t m = t[0] * P::INV;
    uint64_t acc = (uint64_t)m * P::MOD[0] + t[0];  // low word 0 by construction
    uint64_t c = acc >> 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      acc = (P::MOD[j] != 0u ? (uint64_t)m * P::MOD[j] : 0ull) + t[j] + c;
      t[j - 1] = (uint32_t)acc;
      c = acc >> 32;
    }
    acc = (uint64_t)top + c;
    t[7] = (uint32_t)acc;
    top = (uint32_t)(acc >> 32);
  }
  return fe_reduce_once<P>(t, top);
}

template <class P>
PM_HD Fe<P> fe_redc(const Fe<P>& a);  // device: FIPS columns (below); host: fe_redc_portable

template <class P>
PM_HD Fe<P> fe_from_mont(const Fe<P>& a) {
  return fe_redc<P>(a);
}
template <class P>
PM_HD Fe<P> fe_to_mont(const Fe<P>& a) {
  Fe<P> r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.l[i] = P::R2[i];
  return fe_mul<P>(a, r2);
}

// a^(p-2) by left-to-right square-and-multiply over the compile-time exponent.
template <class P>
PM_HD Fe<P> fe_inv(const Fe<P>& a) {
  uint32_t e[8], br = 0;
  const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = subb(P::MOD[i], two[i], br);
  Fe<P> r = fe_one<P>();
  bool started = false;
  for (int i = 7; i >= 0; i--) {
    for (int bit = 31; bit >= 0; bit--) {
      if (started) r = fe_sqr<P>(r);
      if ((e[i] >> bit) & 1u) {
        r = started ? fe_mul<P>(r, a) : a;
        started = true;
      }
    }
  }
  return r;
}

// small-constant multiple (k <= 8) by additions
template <class P>
PM_HD Fe<P> fe_mul_small(const Fe<P>& a, int k) {
  Fe<P> r = fe_zero<P>();
  for (int i = 0; i < k; i++) r = fe_add<P>(r, a);
  return r;
}

// -------------------------------------------------------- load / store
template <class P>
PM_HD Fe<P> fe_load(const uint32_t* p) {
  Fe<P> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = p[i];
  return r;
}
template <class P>
PM_HD void fe_store(uint32_t* p, const Fe<P>& a) {
#pragma unroll
  for (int i = 0; i < 8; i++) p[i] = a.l[i];
}

}  // namespace pm

// fp29.hpp -- radix-2^29 lazy Montgomery arithmetic for the MSM device pipeline.
//
// Why: with 32-bit limbs every 32x32 product needs a v_mad_u64_u32 plus a
// carry-out add into a third word (and the compiler pads the SGPR carry with
// s_nops), about 290 VALU instructions per Pasta product.  With 29-bit limbs
// (9 limbs, R = 2^261) a column of up to 18 products of < 2^58 plus the carry
// fits a 64-bit accumulator, so each product is ONE chained v_mad_u64_u32 and a
// column ends with one 64-bit shift: ~180 instructions per product.  Values
// stay lazily reduced (bounds below), so additions are limb-wise adds.
//
// Representation F29<P>: l[0..8], value = sum l[i] 2^(29 i), Montgomery form
// x * 2^261 mod p (NOT the R = 2^256 form of the Rust types; k_bases_to_r261
// converts the bases once per MSM and k_bucket_bits converts the window sums
// back).  "Norm" = every limb < 2^29.
//
// Bounds (p < 2^255, R = 2^261 > 32p):
//  * f29_mul(a, b): needs limb(a) * limb(b) <= 2^60 (both < 2^30, or one
//    < 2^31 and the other < 2^29) and a * b < R p (e.g. a < 16p, b < 2p;
//    a, b < 6p).  Column sum <= 9 * 2^60 + 9 * 2^58 + 2^36 < 2^64.
//    Result: Norm, < 2p.
//  * f29_sub(a, b, K): a + K - b limb-wise, K a redundant multiple of p
//    whose limbs dominate b's; result limbs < limb(a) + limb(K), not Norm.
//  * f29_norm: carry-propagates (value unchanged).
//  * f29_reduce3(v Norm < 16p): v - q p with q = floor(v_8 / (p_8 + 1))
//    (an underestimate of floor(v/p) by at most 1, computed with a magic
//    multiply that rounds down) -> Norm, < 3p.
// Every curve routine keeps point coordinates Norm and < 4p (stored X, Y < 3p,
// ZZ, ZZZ < 2p), so 3p < 2^256 and the 8 x u32 packed form holds them.
#pragma once
#include "fp256.hpp"
#include "inv_bgcd.hpp"

namespace pm {

template <class P>
struct F29 {
  uint32_t l[9];
};
template <class P>
struct F29Consts;

template <> struct F29Consts<PallasFp> {
  static constexpr uint32_t P[9] = {0x00000001u, 0x09698768u, 0x133e46e6u, 0x0d31f812u, 0x00000224u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00400000u};
  static constexpr uint32_t INV = 0x1fffffffu;  // -p^-1 mod 2^29
  static constexpr uint32_t ONE[9] = {0x1fffff81u, 0x14a5d367u, 0x141ad3c0u, 0x1435eec5u, 0x1ffeefefu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^261 mod p
  static constexpr uint32_t TO261[9] = {0x1ffff001u, 0x10f30767u, 0x0ecfe231u, 0x0db0ce73u, 0x1fddbb8bu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^266 mod p: R256 -> R261
  static constexpr uint32_t R522[9] = {0x00003b6au, 0x19c10910u, 0x1a6a0188u, 0x12a4fd88u, 0x0634b36du, 0x178792bau, 0x07797a99u, 0x1dce5b8au, 0x003506bdu};  // 2^522 mod p: canonical -> R261
  static constexpr uint32_t TO256[9] = {0x1ffffffdu, 0x03c369c7u, 0x06452b4du, 0x186a17c8u, 0x1ffff992u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^256 mod p: R261 -> R256
  static constexpr uint32_t K2[9] = {0x20000002u, 0x32d30ecfu, 0x267c8dcbu, 0x3a63f024u, 0x20000447u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x007fffffu};  // 2p, limbs >= 2^29 - 1
  static constexpr uint32_t K6[9] = {0x20000006u, 0x38792c6fu, 0x3375a964u, 0x2f2bd06eu, 0x20000cd9u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x017fffffu};  // 6p, limbs >= 2^29 - 1
  static constexpr uint32_t K8x3[9] = {0x60000008u, 0x6b4c3b3du, 0x79f2372fu, 0x698fc091u, 0x60001120u, 0x5ffffffdu, 0x5ffffffdu, 0x5ffffffdu, 0x01fffffdu};  // 8p, limbs >= 3 * 2^29 - 3
  static constexpr uint32_t JP0[8] = {0x00000000u, 0x00000001u, 0x00000002u, 0x00000003u, 0x00000004u, 0x00000005u, 0x00000006u, 0x00000007u};  // (j p) mod 2^29, j < 8
  static constexpr uint32_t R783[9] = {0x087c2a3au, 0x04d0a808u, 0x0a88e396u, 0x0f66ba31u, 0x06fd7543u, 0x0d4ff50bu, 0x1f1a2028u, 0x12d9910du, 0x00049116u};  // 2^783 mod p: inverse fix-up (f29_inv)
  static constexpr uint32_t QMAGIC = 0x0003ffffu;  // floor(2^40 / (p_8 + 1))
};
template <> struct F29Consts<VestaFp> {
  static constexpr uint32_t P[9] = {0x00000001u, 0x02375908u, 0x052a3763u, 0x0d31f813u, 0x00000224u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00400000u};
  static constexpr uint32_t INV = 0x1fffffffu;  // -p^-1 mod 2^29
  static constexpr uint32_t ONE[9] = {0x1fffff81u, 0x068ad507u, 0x100e85dau, 0x1435ee7eu, 0x1ffeefefu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^261 mod p
  static constexpr uint32_t TO261[9] = {0x1ffff001u, 0x0ca6d907u, 0x01b40647u, 0x0db0c57eu, 0x1fddbb8bu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^266 mod p: R256 -> R261
  static constexpr uint32_t R522[9] = {0x00003b6au, 0x02b1b550u, 0x1027888au, 0x1ea4ed96u, 0x0418ad7au, 0x000999ebu, 0x17fae231u, 0x1e67ed54u, 0x003506bdu};  // 2^522 mod p: canonical -> R261
  static constexpr uint32_t TO256[9] = {0x1ffffffdu, 0x1959f4e7u, 0x108159d6u, 0x186a17c6u, 0x1ffff992u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // 2^256 mod p: R261 -> R256
  static constexpr uint32_t K2[9] = {0x20000002u, 0x246eb20fu, 0x2a546ec5u, 0x3a63f025u, 0x20000447u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x007fffffu};  // 2p, limbs >= 2^29 - 1
  static constexpr uint32_t K6[9] = {0x20000006u, 0x2d4c162fu, 0x3efd4c51u, 0x2f2bd071u, 0x20000cd9u, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x017fffffu};  // 6p, limbs >= 2^29 - 1
  static constexpr uint32_t K8x3[9] = {0x60000008u, 0x71bac83du, 0x6951bb15u, 0x698fc096u, 0x60001120u, 0x5ffffffdu, 0x5ffffffdu, 0x5ffffffdu, 0x01fffffdu};  // 8p, limbs >= 3 * 2^29 - 3
  static constexpr uint32_t JP0[8] = {0x00000000u, 0x00000001u, 0x00000002u, 0x00000003u, 0x00000004u, 0x00000005u, 0x00000006u, 0x00000007u};  // (j p) mod 2^29, j < 8
  static constexpr uint32_t R783[9] = {0x1725f045u, 0x0bcb119eu, 0x05aace00u, 0x1fd24ea8u, 0x1ee82c09u, 0x038572d8u, 0x11fd9d97u, 0x06792c88u, 0x000bd037u};  // 2^783 mod p: inverse fix-up (f29_inv)
  static constexpr uint32_t QMAGIC = 0x0003ffffu;  // floor(2^40 / (p_8 + 1))
};
template <> struct F29Consts<Bn254Fq> {
  static constexpr uint32_t P[9] = {0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u, 0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  static constexpr uint32_t INV = 0x04866389u;  // -p^-1 mod 2^29
  static constexpr uint32_t ONE[9] = {0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u, 0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // 2^261 mod p
  static constexpr uint32_t TO261[9] = {0x13349ca1u, 0x1a5d84a8u, 0x0a3e5cacu, 0x100249e0u, 0x12b951e8u, 0x0e92d304u, 0x14cb95b3u, 0x041b9d3du, 0x00058003u};  // 2^266 mod p: R256 -> R261
  static constexpr uint32_t R522[9] = {0x059bac10u, 0x0d1503a3u, 0x018016b8u, 0x10ab0ca8u, 0x02632639u, 0x02c0169fu, 0x169bfd53u, 0x11869d4cu, 0x002a11a6u};  // 2^522 mod p: canonical -> R261
  static constexpr uint32_t TO256[9] = {0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u, 0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};  // 2^256 mod p: R261 -> R256
  static constexpr uint32_t K2[9] = {0x30f9fa8eu, 0x2208c16cu, 0x38e5469du, 0x25aa45a0u, 0x2b0bb2efu, 0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};  // 2p, limbs >= 2^29 - 1
  static constexpr uint32_t K6[9] = {0x32edefaau, 0x261a4447u, 0x2aafd3d9u, 0x30fed0e4u, 0x212318cfu, 0x31238483u, 0x23e94785u, 0x3628e537u, 0x012259d5u};  // 6p, limbs >= 2^29 - 1
  static constexpr uint32_t K8x3[9] = {0x63e7ea38u, 0x682305b3u, 0x63951a75u, 0x76a91684u, 0x6c2ecbbdu, 0x76da0602u, 0x65370a05u, 0x72e1319du, 0x01832270u};  // 8p, limbs >= 3 * 2^29 - 3
  static constexpr uint32_t JP0[8] = {0x00000000u, 0x187cfd47u, 0x10f9fa8eu, 0x0976f7d5u, 0x01f3f51cu, 0x1a70f263u, 0x12edefaau, 0x0b6aecf1u};  // (j p) mod 2^29, j < 8
  static constexpr uint32_t R783[9] = {0x0e2312b2u, 0x16c05ca2u, 0x0bc84389u, 0x1cdf310bu, 0x11adafddu, 0x032e568eu, 0x1d6ae48cu, 0x10d4cd1fu, 0x0026c2d2u};  // 2^783 mod p: inverse fix-up (f29_inv)
  static constexpr uint32_t QMAGIC = 0x00054a47u;  // floor(2^40 / (p_8 + 1))
};

template <> struct F29Consts<Bn254Fr> {
  static constexpr uint32_t P[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u, 0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
  static constexpr uint32_t INV = 0x0fffffffu;  // -p^-1 mod 2^29
  static constexpr uint32_t ONE[9] = {0x0fffff57u, 0x1ea70ab4u, 0x052c068bu, 0x17504f49u, 0x0aa8075bu, 0x1d4240ceu, 0x11d54c07u, 0x052ac7a8u, 0x000dc836u};  // 2^261 mod p
  static constexpr uint32_t TO261[9] = {0x0fffead7u, 0x1d5444f4u, 0x04438aa5u, 0x03b4d096u, 0x134c84dau, 0x0e92d304u, 0x14cb95b3u, 0x041b9d3du, 0x00058003u};  // 2^266 mod p: R256 -> R261
  static constexpr uint32_t TO256[9] = {0x0ffffffbu, 0x04b1a0e2u, 0x18334a6bu, 0x18ed2b3eu, 0x1462e36fu, 0x11b7bc3cu, 0x1cbd99bau, 0x183340fbu, 0x000e0a77u};  // 2^256 mod p: R261 -> R256
  static constexpr uint32_t K2[9] = {0x20000002u, 0x3e1f593eu, 0x3cb848a0u, 0x2fa121e5u, 0x2b0ba505u, 0x25b68180u, 0x214dc281u, 0x3cb84c67u, 0x0060c89bu};  // 2p, limbs >= 2^29 - 1
  static constexpr uint32_t K6[9] = {0x20000006u, 0x3a5e0bbcu, 0x3628d9e4u, 0x2ee365b3u, 0x2122ef12u, 0x31238483u, 0x23e94785u, 0x3628e537u, 0x012259d5u};  // 6p, limbs >= 2^29 - 1
  static constexpr uint32_t K8x3[9] = {0x60000008u, 0x787d64f9u, 0x72e12284u, 0x7e848798u, 0x6c2e9416u, 0x76da0602u, 0x65370a05u, 0x72e1319du, 0x01832270u};  // 8p, limbs >= 3 * 2^29 - 3
  static constexpr uint32_t JP0[8] = {0x00000000u, 0x10000001u, 0x00000002u, 0x10000003u, 0x00000004u, 0x10000005u, 0x00000006u, 0x10000007u};  // (j p) mod 2^29, j < 8
  static constexpr uint32_t R783[9] = {0x001fddb2u, 0x17d30b63u, 0x1a2600eeu, 0x09507c47u, 0x1496b29bu, 0x0b00a268u, 0x15b645ebu, 0x1f9fcb3du, 0x001baa96u};  // 2^783 mod p: inverse fix-up (f29_inv)
  static constexpr uint32_t QMAGIC = 0x00054a47u;  // floor(2^40 / (p_8 + 1))
};

constexpr uint32_t kM29 = (1u << 29) - 1u;

// 12p with every limb below the top in [2^30 - 2, 2^30 + 2^29): it dominates
// any limb <= 2^29, so a + K12 - b is non-negative limb-wise for b lazily
// normalised (limbs <= 2^29) and below 12p (the row-sliced ladder's unreduced
// X3 / Y3, k_acc_powers_s, and their negation in k_acc_termadd)
template <class P>
constexpr uint32_t f29_k12_limb(int i) {
  uint64_t c = 0, n = 0;
  for (int k = 0; k <= i; k++) {
    const uint64_t v = 12ull * F29Consts<P>::P[k] + c;
    n = k < 8 ? (v & kM29) : v;
    c = v >> 29;
  }
  return (uint32_t)(n + (i < 8 ? (1ull << 30) : 0ull) - (i > 0 ? 2ull : 0ull));
}
template <class P>
struct F29K12 {
  static constexpr uint32_t L[9] = {f29_k12_limb<P>(0), f29_k12_limb<P>(1), f29_k12_limb<P>(2),
                                    f29_k12_limb<P>(3), f29_k12_limb<P>(4), f29_k12_limb<P>(5),
                                    f29_k12_limb<P>(6), f29_k12_limb<P>(7), f29_k12_limb<P>(8)};
};

template <class P>
__device__ __forceinline__ F29<P> f29_const(const uint32_t (&c)[9]) {
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = c[i];
  return r;
}
template <class P>
__device__ __forceinline__ F29<P> f29_zero() {
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = 0;
  return r;
}
template <class P>
__device__ __forceinline__ bool f29_is_zero_exact(const F29<P>& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) o |= a.l[i];
  return o == 0;
}

// 256-bit packed (8 x u32, little endian) <-> 9 x 29-bit limbs
template <class P>
__device__ __forceinline__ F29<P> f29_unpack(const uint32_t w[8]) {
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, k = bit >> 5, s = bit & 31;
    uint32_t v = w[k] >> s;
    if (s > 3 && k + 1 < 8) v |= w[k + 1] << (32 - s);
    r.l[i] = v & kM29;
  }
  return r;
}
// requires Norm and value < 2^256
template <class P>
__device__ __forceinline__ void f29_pack(const F29<P>& a, uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int bit = 32 * k, i = bit / 29, s = bit - 29 * i;
    uint32_t v = a.l[i] >> s;
    if (i + 1 < 9) v |= a.l[i + 1] << (29 - s);
    if (s > 26 && i + 2 < 9) v |= a.l[i + 2] << (58 - s);
    w[k] = v;
  }
}

// Chained multiply-adds in inline asm: acc += x_t * y_t for up to four terms
// per statement.  Left to itself the compiler splits each column into partial
// sums (for ILP) and merges them with 64-bit adds; one chain per column needs
// none, and throughput (not single-chain latency) is what the MSM needs.  The
// carry-out of v_mad_u64_u32 is dead (columns never overflow 2^64).
#define PM_MC(X, Y) "v_mad_u64_u32 %0, %1, " X ", " Y ", %0\n\t"
__device__ __forceinline__ void mc_vv(uint64_t& acc, const uint32_t* x, const uint32_t* y, int n) {
  uint64_t c;
  if (n >= 4) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") PM_MC("%6", "%7") PM_MC("%8", "%9")
        : "+v"(acc), "=&s"(c) : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]), "v"(x[3]), "v"(y[3]));
  } else if (n == 3) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") PM_MC("%6", "%7")
        : "+v"(acc), "=&s"(c) : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]), "v"(x[2]), "v"(y[2]));
  } else if (n == 2) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") : "+v"(acc), "=&s"(c) : "v"(x[0]), "v"(y[0]), "v"(x[1]), "v"(y[1]));
  } else if (n == 1) {
    asm(PM_MC("%2", "%3") : "+v"(acc), "=&s"(c) : "v"(x[0]), "v"(y[0]));
  }
}
__device__ __forceinline__ void mc_vs(uint64_t& acc, const uint32_t* x, const uint32_t* y, int n) {
  uint64_t c;
  if (n >= 4) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") PM_MC("%6", "%7") PM_MC("%8", "%9")
        : "+v"(acc), "=&s"(c) : "v"(x[0]), "s"(y[0]), "v"(x[1]), "s"(y[1]), "v"(x[2]), "s"(y[2]), "v"(x[3]), "s"(y[3]));
  } else if (n == 3) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") PM_MC("%6", "%7")
        : "+v"(acc), "=&s"(c) : "v"(x[0]), "s"(y[0]), "v"(x[1]), "s"(y[1]), "v"(x[2]), "s"(y[2]));
  } else if (n == 2) {
    asm(PM_MC("%2", "%3") PM_MC("%4", "%5") : "+v"(acc), "=&s"(c) : "v"(x[0]), "s"(y[0]), "v"(x[1]), "s"(y[1]));
  } else if (n == 1) {
    asm(PM_MC("%2", "%3") : "+v"(acc), "=&s"(c) : "v"(x[0]), "s"(y[0]));
  }
}
template <bool YS>
__device__ __forceinline__ void mc_n(uint64_t& acc, const uint32_t* x, const uint32_t* y, int n) {
#pragma unroll
  for (int t = 0; t < n; t += 4) {
    if (YS) mc_vs(acc, x + t, y + t, n - t);
    else mc_vv(acc, x + t, y + t, n - t);
  }
}

// Column-chained forms of f29_mul / f29_sqr (same arithmetic, same result),
// generic over the field: up to four multiply-adds per asm statement, the
// power-of-two limb and p_0 = 1 folded in as 64-bit shift-adds.  The hot
// paths use the generated per-field forms below (f29_mul_a / f29_sqr_a).
template <class P>
__device__ __forceinline__ F29<P> f29_mul_g(const F29<P>& a, const F29<P>& b) {
  using K = F29Consts<P>;
  uint32_t m[9];
  F29<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint32_t xs[9], ys[9], ms[9], ps[9];
    int n = 0, nr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j >= 0 && j < 9) {
        xs[n] = a.l[i];
        ys[n] = b.l[j];
        n++;
      }
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 9 && K::P[j] != 0u) {
        if ((K::P[j] & (K::P[j] - 1u)) == 0u) {
          acc += (uint64_t)m[i] << __builtin_ctz(K::P[j]);  // power-of-two limb (Pasta p_8 = 2^22)
        } else {
          ms[nr] = m[i];
          ps[nr] = K::P[j];
          nr++;
        }
      }
    }
    mc_n<false>(acc, xs, ys, n);
    mc_n<true>(acc, ms, ps, nr);
    if (k < 9) {
      m[k] = ((uint32_t)acc * K::INV) & kM29;
      if (K::P[0] == 1u) acc += m[k];
      else mc_n<true>(acc, &m[k], &K::P[0], 1);
    } else {
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

template <class P>
__device__ __forceinline__ F29<P> f29_sqr_g(const F29<P>& a) {
  using K = F29Consts<P>;
  uint32_t m[9], d[9];
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
    uint32_t xs[9], ys[9], ms[9], ps[9];
    int n = 0, nr = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j > i && j < 9) {
        xs[n] = d[i];
        ys[n] = a.l[j];
        n++;
      }
    }
    if ((k & 1) == 0 && k / 2 < 9) {
      xs[n] = a.l[k / 2];
      ys[n] = a.l[k / 2];
      n++;
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 9 && K::P[j] != 0u) {
        if ((K::P[j] & (K::P[j] - 1u)) == 0u) {
          acc += (uint64_t)m[i] << __builtin_ctz(K::P[j]);
        } else {
          ms[nr] = m[i];
          ps[nr] = K::P[j];
          nr++;
        }
      }
    }
    mc_n<false>(acc, xs, ys, n);
    mc_n<true>(acc, ms, ps, nr);
    if (k < 9) {
      m[k] = ((uint32_t)acc * K::INV) & kM29;
      if (K::P[0] == 1u) acc += m[k];
      else mc_n<true>(acc, &m[k], &K::P[0], 1);
    } else {
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// One asm statement per product column, generated per field by
// tools/gen_fp29_asm.py (fp29_asm.hpp, included at the end of this file):
// every multiply-add of a column in one chain, including the reduction's
// power-of-two limb and p_0, so no 64-bit shift-adds, no {m, 0} register
// pairs and one s_nop pad per column.  Mul: 187 VALU instead of 200 (Pasta).
template <class P>
__device__ F29<P> f29_mul_a(const F29<P>& a, const F29<P>& b);
template <class P>
__device__ F29<P> f29_sqr_a(const F29<P>& a);
template <class P>
__device__ F29<P> f29_mul2_a(const F29<P>& a, const F29<P>& b, const F29<P>& u, const F29<P>& v);
template <class P>
__device__ __forceinline__ F29<P> f29_mul_c(const F29<P>& a, const F29<P>& b) {
  return f29_mul_a<P>(a, b);
}
// Sum of two products with one Montgomery reduction: (a b + u v) 2^-261.
// All four operands Norm (limbs < 2^29: a column holds 18 operand products +
// 6 reduction products < 2^58, < 2^63) and a b + u v < 2^261 p / 1.7 (e.g.
// a, b < 8p, u < 6p, v < 2p: 76 p^2) -> Norm, < 2p.  Saves a whole reduction
// (54 multiply-adds on Pasta) and the subtract / normalise / reduce3 of the
// difference form a b - u' v.
template <class P>
__device__ __forceinline__ F29<P> f29_mul2_c(const F29<P>& a, const F29<P>& b, const F29<P>& u, const F29<P>& v) {
  return f29_mul2_a<P>(a, b, u, v);
}
// Difference of two products with one Montgomery reduction: (a b - u v)
// 2^-261 (+ a multiple of p).  The u v terms enter the signed columns as
// multiply-adds by the negated limbs of v, so no negation of u or v as a field
// element (K - x + normalise) is needed.  All four operands Norm, a b < 80 p^2,
// u < 3p, v < 2p -> Norm, < 3p (tests/test_fp29_asm.py runs it in the
// interpreter with signed-overflow checks).
template <class P>
__device__ F29<P> f29_mul2n_a(const F29<P>& a, const F29<P>& b, const F29<P>& u, const F29<P>& v);
template <class P>
__device__ __forceinline__ F29<P> f29_mul2n_c(const F29<P>& a, const F29<P>& b, const F29<P>& u, const F29<P>& v) {
  return f29_mul2n_a<P>(a, b, u, v);
}
template <class P>
__device__ __forceinline__ F29<P> f29_sqr_c(const F29<P>& a) {
  return f29_sqr_a<P>(a);
}

// Montgomery product a * b * 2^-261 mod p (lazy: Norm, < 2p), product scanning
// with one 64-bit accumulator; zero limbs of p are skipped at compile time.
template <class P>
__device__ __forceinline__ F29<P> f29_mul(const F29<P>& a, const F29<P>& b) {
  using K = F29Consts<P>;
  uint32_t m[9];
  F29<P> r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc += (uint64_t)a.l[i] * b.l[j];
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 9 && K::P[j] != 0u) acc += (uint64_t)m[i] * K::P[j];
    }
    if (k < 9) {
      m[k] = ((uint32_t)acc * K::INV) & kM29;
      acc += (uint64_t)m[k] * K::P[0];
    } else {
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// Montgomery square (a Norm): cross products once with a doubled operand.
template <class P>
__device__ __forceinline__ F29<P> f29_sqr(const F29<P>& a) {
  using K = F29Consts<P>;
  uint32_t m[9], d[9];
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) d[i] = a.l[i] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; k++) {
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (j > i && j < 9) acc += (uint64_t)d[i] * a.l[j];
    }
    if ((k & 1) == 0 && k / 2 < 9) acc += (uint64_t)a.l[k / 2] * a.l[k / 2];
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int j = k - i;
      if (i < k && j >= 1 && j < 9 && K::P[j] != 0u) acc += (uint64_t)m[i] * K::P[j];
    }
    if (k < 9) {
      m[k] = ((uint32_t)acc * K::INV) & kM29;
      acc += (uint64_t)m[k] * K::P[0];
    } else {
      r.l[k - 9] = (uint32_t)acc & kM29;
    }
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

template <class P>
__device__ __forceinline__ F29<P> f29_add(const F29<P>& a, const F29<P>& b) {
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + b.l[i];
  return r;
}
// a + K - b (K: redundant multiple of p, limb-wise >= b)
template <class P>
__device__ __forceinline__ F29<P> f29_sub(const F29<P>& a, const F29<P>& b, const uint32_t (&K)[9]) {
  F29<P> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = a.l[i] + K[i] - b.l[i];
  return r;
}
template <class P>
__device__ __forceinline__ F29<P> f29_norm(const F29<P>& a) {
  F29<P> r;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t v = a.l[i] + c;  // limbs < 2^32 - 2^3, carry < 2^3
    r.l[i] = v & kM29;
    c = v >> 29;
  }
  r.l[8] = a.l[8] + c;
  return r;
}
// Norm, < 16p -> Norm, < 3p
template <class P>
__device__ __forceinline__ F29<P> f29_reduce3(const F29<P>& a) {
  using K = F29Consts<P>;
  const uint32_t q = (uint32_t)(((uint64_t)a.l[8] * K::QMAGIC) >> 40);
  F29<P> r;
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int64_t v = (int64_t)a.l[i] - (int64_t)q * K::P[i] + c;
    r.l[i] = i < 8 ? (uint32_t)v & kM29 : (uint32_t)v;
    c = v >> 29;  // arithmetic: borrows propagate
  }
  return r;
}
// Norm, < 4p -> canonical [0, p), Norm
template <class P>
__device__ __forceinline__ F29<P> f29_canon(const F29<P>& a) {
  using K = F29Consts<P>;
  F29<P> v = a;
#pragma unroll
  for (int t = 0; t < 3; t++) {  // subtract p while v >= p
    F29<P> d;
    int64_t c = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int64_t x = (int64_t)v.l[i] - K::P[i] + c;
      d.l[i] = (uint32_t)x & kM29;
      c = x >> 29;
    }
    const bool ge = c >= 0;
#pragma unroll
    for (int i = 0; i < 9; i++) v.l[i] = ge ? d.l[i] : v.l[i];
  }
  return v;
}
// v Norm, < 8p: v == 0 mod p?  Cheap limb-0 filter (v = j p, j < 8, has
// limb 0 = (j p) mod 2^29); the exact check runs only on a hit.
template <class P>
constexpr bool f29_jp0_linear() {  // (j p) mod 2^29 == j: p = 1 mod 2^29 (Pasta)
  for (int j = 0; j < 8; j++)
    if (F29Consts<P>::JP0[j] != (uint32_t)j) return false;
  return true;
}
// the cheap filter alone: false => v != 0 mod p
template <class P>
__device__ __forceinline__ bool f29_zero_filter(const F29<P>& v) {
  using K = F29Consts<P>;
  bool hit = false;
  if constexpr (f29_jp0_linear<P>()) {
    hit = v.l[0] < 8u;  // one compare instead of eight
  } else {
#pragma unroll
    for (int j = 0; j < 8; j++) hit |= v.l[0] == K::JP0[j];
  }
  return hit;
}
template <class P>
__device__ __forceinline__ bool f29_is_zero_mod(const F29<P>& v) {
  if (!f29_zero_filter<P>(v)) return false;
  return f29_is_zero_exact<P>(f29_canon<P>(f29_reduce3<P>(v)));
}

// a^(p-2) (Fermat inverse; 0 -> 0) by left-to-right square-and-multiply over
// the constant exponent (lane-uniform control flow).  Input Norm < 4p,
// output Norm < 2p, both in the R = 2^261 Montgomery form.  Kept as the
// reference for f29_inv (selftest).
template <class P>
__device__ F29<P> f29_inv_fermat(const F29<P>& a) {
  uint32_t e[8], br = 0;
  const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) e[i] = subb(P::MOD[i], two[i], br);
  F29<P> r = a;  // the exponent's top bit (bit NBITS-1) is set
  for (int bit = P::NBITS - 2; bit >= 0; bit--) {
    r = f29_sqr_c<P>(r);
    if ((e[bit >> 5] >> (bit & 31)) & 1u) r = f29_mul_c<P>(r, a);
  }
  return r;
}

// Inverse by the variable-time safegcd (inv_bgcd.hpp sg_inverse; 33 us per
// lane against 54 us for the binary GCD and ~170 us for Fermat):
// a = y 2^261 (Norm, < 4p) -> canonical packed -> (y 2^261)^-1 -> times
// 2^783 / 2^261 = y^-1 2^261.  Output Norm, < 2p; 0 -> 0.
template <class P>
__device__ F29<P> f29_inv(const F29<P>& a) {
  uint32_t w[8], v[8];
  f29_pack<P>(f29_canon<P>(a), w);
  sg_inverse<P>(w, v);
  return f29_mul_c<P>(f29_unpack<P>(v), f29_const<P>(F29Consts<P>::R783));
}

// Quad-cooperative f29_inv (sg_inverse_q): all 4 lanes of a quad, same input.
template <class P>
__device__ F29<P> f29_inv_q(const F29<P>& a) {
  uint32_t w[8], v[8];
  f29_pack<P>(f29_canon<P>(a), w);
  sg_inverse_q<P>(w, v);
  return f29_mul_c<P>(f29_unpack<P>(v), f29_const<P>(F29Consts<P>::R783));
}

// R256 packed Montgomery (Rust layout, canonical) -> F29 (Norm, < 2p)
template <class P>
__device__ __forceinline__ F29<P> f29_from_r256(const uint32_t w[8]) {
  return f29_mul_c<P>(f29_unpack<P>(w), f29_const<P>(F29Consts<P>::TO261));
}
// F29 (Norm, < 4p) -> R256 packed Montgomery, canonical
template <class P>
__device__ __forceinline__ void f29_to_r256(const F29<P>& a, uint32_t w[8]) {
  f29_pack<P>(f29_canon<P>(f29_mul_c<P>(a, f29_const<P>(F29Consts<P>::TO256))), w);
}

// Inverse of an R256 Montgomery element (binary GCD, inv_bgcd.hpp); same
// result as fe_inv.
template <class P>
__device__ __forceinline__ Fe<P> fe_inv_fast(const Fe<P>& a) {
  return fe_inv_bgcd<P>(a);
}

}  // namespace pm

#include "fp29_asm.hpp"

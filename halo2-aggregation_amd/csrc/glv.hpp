// glv.hpp -- GLV endomorphism decomposition shared by the MSM (GLV mode:
// 2n points with 128-bit scalars) and the accumulator's term products.
#pragma once
#include "curve.hpp"

namespace pm {

// ------------------------------------------------------------------- GLV
// All three curves have an efficient endomorphism phi(x, y) = (beta x, y) =
// [lambda](x, y) (y^2 = x^3 + b, p = 1 mod 3).  [k]P = [k1]P + [k2]phi(P) with
// |k1|, |k2| < 2^128 (Gallant-Lambert-Vanstone): c1 = floor(k g1 / 2^384),
// c2 = floor(k g2 / 2^384), k1 = k - c1 a1 - c2 a2, k2 = c1 (-b1) - c2 b2 for
// the short lattice basis (a1, b1), (a2, b2) of {(a, b) : a + b lambda = 0 mod
// r}.  Constants derived and checked in tests/test_glv.py (lambda G = phi(G),
// a + b lambda = 0 mod r, |k1|, |k2| < 2^128 over random and edge scalars).
template <class Cv>
struct Glv;
// PallasCurve: phi(x, y) = (beta x, y) = [lambda](x, y), lambda = 0x397e65a7d7c1ad71aee24b27e308f0a61259527ec1d4752e619d1840af55f1b1
template <> struct Glv<PallasCurve> {
  static constexpr uint32_t BETA29[9] = {0x0cbd58ebu, 0x1a2f8f16u, 0x0d140efau, 0x007bdfb9u, 0x1333ecadu, 0x0a33785bu, 0x04eacc49u, 0x09617a1eu, 0x0004ff6cu};  // beta * 2^261 mod p, radix 2^29
  static constexpr uint32_t B29[9] = {0x1ffffd81u, 0x01970367u, 0x178d072au, 0x1045c991u, 0x1ffaa71cu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // curve b * 2^261 mod p, radix 2^29
  static constexpr uint32_t BETA[8] = {0x9e65eac8u, 0xfbdfd7aau, 0xe50025fbu, 0x0cd4d654u, 0x3785b99au, 0xd59892a3u, 0x585e8789u, 0x2a27fb62u};  // Montgomery
  static constexpr uint32_t A1[4] = {0x00000000u, 0x8cb12793u, 0x40a89953u, 0x49e69d16u};
  static constexpr uint32_t NB1[4] = {0x00000001u, 0x7fcae1c7u, 0x40f04915u, 0x49e69d16u};  // -b1 > 0
  static constexpr uint32_t A2[4] = {0x00000001u, 0x0c7c095au, 0x8198e269u, 0x93cd3a2cu};
  static constexpr uint32_t B2[4] = {0x00000000u, 0x8cb12793u, 0x40a89953u, 0x49e69d16u};
  static constexpr uint32_t G1[9] = {0x72171db4u, 0x4a95a2d9u, 0x8480fa55u, 0x61afdea6u, 0xffffffffu, 0x32c49e4bu, 0x02a2654eu, 0x279a7459u, 0x00000001u};  // round(2^384 b2 / r)
  static constexpr uint32_t G2[9] = {0x9f98a4dfu, 0xc689c587u, 0x83e7688au, 0x61afdea6u, 0x00000003u, 0xff2b871cu, 0x03c12455u, 0x279a7459u, 0x00000001u};  // round(2^384 (-b1) / r)
};
// VestaCurve: phi(x, y) = (beta x, y) = [lambda](x, y), lambda = 0x12ccca834acdba712caad5dc57aab1b01d1f8bd237ad31491dad5ebdfdfe4ab9
template <> struct Glv<VestaCurve> {
  static constexpr uint32_t BETA29[9] = {0x02222437u, 0x00286338u, 0x1ad2e167u, 0x0c255d0eu, 0x16526d7eu, 0x1fb135b2u, 0x0801613au, 0x0220916cu, 0x0003a53fu};  // beta * 2^261 mod p, radix 2^29
  static constexpr uint32_t B29[9] = {0x1ffffd81u, 0x17d8c507u, 0x1b9fbfb6u, 0x1045c82bu, 0x1ffaa71cu, 0x1fffffffu, 0x1fffffffu, 0x1fffffffu, 0x003fffffu};  // curve b * 2^261 mod p, radix 2^29
  static constexpr uint32_t BETA[8] = {0x80111122u, 0x7c541a84u, 0x56ed29dau, 0x40630b9cu, 0x135b2b29u, 0x02c275fbu, 0x88245b10u, 0x121d29f8u};  // Montgomery
  static constexpr uint32_t A1[4] = {0x00000000u, 0x7fcae1c7u, 0x40f04915u, 0x49e69d16u};
  static constexpr uint32_t NB1[4] = {0x00000001u, 0x8cb12793u, 0x40a89953u, 0x49e69d16u};  // -b1 > 0
  static constexpr uint32_t A2[4] = {0x00000001u, 0x8cb12793u, 0x40a89953u, 0x49e69d16u};
  static constexpr uint32_t B2[4] = {0x00000001u, 0x0c7c095au, 0x8198e269u, 0x93cd3a2cu};
  static constexpr uint32_t G1[9] = {0x296e1563u, 0x841d8d62u, 0x0afe9926u, 0xc35fbd4du, 0x00000002u, 0x31f02568u, 0x066389a4u, 0x4f34e8b2u, 0x00000002u};  // round(2^384 b2 / r)
  static constexpr uint32_t G2[9] = {0x4bf99a83u, 0x841414c2u, 0x85cc1578u, 0x61afdea6u, 0x00000003u, 0x32c49e4cu, 0x02a2654eu, 0x279a7459u, 0x00000001u};  // round(2^384 (-b1) / r)
};
// Bn254Curve: phi(x, y) = (beta x, y) = [lambda](x, y), lambda = 0x30644e72e131a029048b6e193fd84104cc37a73fec2bc5e9b8ca0b2d36636f23
template <> struct Glv<Bn254Curve> {
  static constexpr uint32_t BETA29[9] = {0x18ccb791u, 0x175b1c3au, 0x0b83d6e2u, 0x0e8ed071u, 0x1282bee2u, 0x04220e84u, 0x1fe4017fu, 0x15084d4au, 0x00169119u};  // beta * 2^261 mod p, radix 2^29
  static constexpr uint32_t B29[9] = {0x00766463u, 0x1c54760au, 0x08f6927au, 0x03e40c4du, 0x1fea4f2bu, 0x17c6c26au, 0x157fe417u, 0x0f8056f9u, 0x002958a2u};  // curve b * 2^261 mod p, radix 2^29
  static constexpr uint32_t BETA[8] = {0x13e80b9cu, 0x3350c88eu, 0xdb5e56b9u, 0x7dce557cu, 0xb615564au, 0x6001b4b8u, 0x020217e0u, 0x2682e617u};  // Montgomery
  static constexpr uint32_t A1[4] = {0x7d4f1128u, 0x8211bbebu, 0xeeb859fcu, 0x6f4d8248u};
  static constexpr uint32_t NB1[4] = {0x94d213e3u, 0x89d32568u, 0x00000000u, 0x00000000u};  // -b1 > 0
  static constexpr uint32_t A2[4] = {0x94d213e3u, 0x89d32568u, 0x00000000u, 0x00000000u};
  static constexpr uint32_t B2[4] = {0x1221250bu, 0x0be4e154u, 0xeeb859fdu, 0x6f4d8248u};
  static constexpr uint32_t G1[9] = {0xcb4b9a5fu, 0x163b4843u, 0xd5e495ccu, 0x149d540fu, 0x00ff6565u, 0x5398fd03u, 0xa773d2d2u, 0x4ccef014u, 0x00000002u};  // round(2^384 b2 / r)
  static constexpr uint32_t G2[9] = {0x2fafba64u, 0x8fa7d32du, 0x773a6ef2u, 0x6eb9c714u, 0xc7e0b3d7u, 0xd91d232eu, 0x00000002u, 0x00000000u, 0x00000000u};  // round(2^384 (-b1) / r)
};

constexpr int kGlvBits = 128;  // loop length: |k_i| <= (|a1| + |a2|) (1 + 2^-120) < 2^127.8 (tests/test_glv.py)

// x (nx limbs) * y (ny limbs) -> out (nx + ny limbs), schoolbook, plain C.
template <int NX, int NY>
__device__ __forceinline__ void mp_mul(const uint32_t* x, const uint32_t* y, uint32_t* out) {
#pragma unroll
  for (int i = 0; i < NX + NY; i++) out[i] = 0;
#pragma unroll
  for (int i = 0; i < NX; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < NY; j++) {
      const uint64_t t = (uint64_t)x[i] * y[j] + out[i + j] + c;
      out[i + j] = (uint32_t)t;
      c = t >> 32;
    }
    out[i + NY] = (uint32_t)c;
  }
}

// d (6 limbs, mod 2^192) -= x (4) * y (4)  /  += x * y
template <bool SUB>
__device__ __forceinline__ void mp_fma6(uint32_t* d, const uint32_t* x, const uint32_t* y) {
  uint32_t pr[8];
  mp_mul<4, 4>(x, y, pr);
  uint64_t c = SUB ? 1 : 0;  // two's complement: d + ~pr + 1
#pragma unroll
  for (int i = 0; i < 6; i++) {
    const uint64_t t = (uint64_t)d[i] + (SUB ? (uint32_t)~pr[i] : pr[i]) + c;
    d[i] = (uint32_t)t;
    c = t >> 32;
  }
}

// |v| and sign of a 192-bit two's complement value
__device__ __forceinline__ bool mp_abs6(uint32_t* v) {
  const bool neg = (v[5] >> 31) != 0;
  if (neg) {
    uint64_t c = 1;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      const uint64_t t = (uint64_t)(uint32_t)~v[i] + c;
      v[i] = (uint32_t)t;
      c = t >> 32;
    }
  }
  return neg;
}

// ROUND: c_i = round(k g_i / 2^384) (Babai rounding, |k_i| <= (|a1| + |a2|) / 2
// + 1 < 2^127 on all three curves, tests/test_glv.py) instead of the floor
// (|k_i| < 2^127.8).  The MSM's GLV mode needs |k_i| < 2^127 so that the
// signed digits of 8 windows of 16 bits never carry out of bit 127.
template <int NY>
__device__ __forceinline__ void mp_quot384(const uint32_t* k, const uint32_t* g, bool round, uint32_t c[4]) {
  uint32_t pr[8 + NY];
  mp_mul<8, NY>(k, g, pr);
  uint64_t t = round ? 0x80000000ull : 0ull;  // + 2^383
#pragma unroll
  for (int i = 11; i < 8 + NY; i++) {
    t += pr[i];
    pr[i] = (uint32_t)t;
    t >>= 32;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) c[i] = pr[12 + i];
}
template <class Cv, bool ROUND = false>
__device__ __forceinline__ void glv_split(const Fe<typename Cv::Scalar>& k, uint32_t k1[6], uint32_t k2[6],
                                          bool& n1, bool& n2) {
  using Gc = Glv<Cv>;
  uint32_t c1[4], c2[4];
  mp_quot384<9>(k.l, Gc::G1, ROUND, c1);
  mp_quot384<9>(k.l, Gc::G2, ROUND, c2);
#pragma unroll
  for (int i = 0; i < 6; i++) {
    k1[i] = k.l[i];
    k2[i] = 0;
  }
  mp_fma6<true>(k1, c1, Gc::A1);
  mp_fma6<true>(k1, c2, Gc::A2);
  mp_fma6<false>(k2, c1, Gc::NB1);
  mp_fma6<true>(k2, c2, Gc::B2);
  n1 = mp_abs6(k1);
  n2 = mp_abs6(k2);
}

}  // namespace pm

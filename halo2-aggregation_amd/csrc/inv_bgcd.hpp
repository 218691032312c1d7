// inv_bgcd.hpp -- field inversion by Pornin's optimized binary GCD
// ("Optimized Binary GCD for Modular Inversion", T. Pornin, IACR ePrint
// 2020/972, Algorithm 2), host + device.
//
// Why: a Fermat inversion a^(p-2) is ~330 dependent Montgomery products.  In
// the latency-bound kernels (one lane per proof or per output: k_acc_scalars,
// k_acc_sum, the SRS table build) a single wave issues one v_mad_u64_u32 every
// ~9 cycles, so each product costs ~0.5 us and the inversion ~0.17 ms.  The
// binary GCD needs 2 len(p) - 1 = 509 cheap iterations on 62-bit
// approximations (30 per batch, 32-bit ops) plus, per batch, four 9-limb x
// 31-bit multiply-adds: ~4x lower latency.
//
// Numbers are 9 limbs of 30 bits (270 bits), so the per-batch division by
// 2^30 is a limb drop.  Invariant: a = u y (mod p), b = v y (mod p); at the
// end b = gcd = 1 and v = y^-1 (y = 0 gives 0, like the Fermat form).
#pragma once
#include "fp256.hpp"

namespace pm {

constexpr int kBgIter = 30;  // inner iterations per batch (= exact low bits)
constexpr uint32_t kBgM = (1u << 30) - 1u;

template <class P>
struct BgConsts {
  uint32_t p[9];
  uint32_t pinv;  // -p^-1 mod 2^30
  int batches;    // ceil((2 len(p) - 1) / 30), plus one batch of margin
};
template <class P>
PM_HD BgConsts<P> bg_consts() {
  BgConsts<P> c{};
  for (int i = 0; i < 9; i++) {
    const int bit = 30 * i, k = bit >> 5, s = bit & 31;
    uint64_t v = (uint64_t)P::MOD[k] >> s;
    if (k + 1 < 8) v |= (uint64_t)P::MOD[k + 1] << (32 - s);
    c.p[i] = (uint32_t)v & kBgM;
  }
  c.pinv = P::INV & kBgM;  // INV = -p^-1 mod 2^32
  c.batches = (2 * P::NBITS - 1 + kBgIter - 1) / kBgIter + 1;
  return c;
}

// 8 x 32-bit little-endian -> 9 x 30-bit limbs
PM_HD void bg_split(const uint32_t w[8], uint32_t o[9]) {
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int bit = 30 * i, k = bit >> 5, s = bit & 31;
    uint64_t v = (uint64_t)w[k] >> s;
    if (k + 1 < 8) v |= (uint64_t)w[k + 1] << (32 - s);
    o[i] = (uint32_t)v & kBgM;
  }
}
// 9 x 30-bit limbs (value < 2^256) -> 8 x 32-bit
PM_HD void bg_join(const uint32_t o[9], uint32_t w[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const int bit = 32 * k, i = bit / 30, s = bit - 30 * i;
    uint64_t v = (uint64_t)o[i] >> s;
    if (i + 1 < 9) v |= (uint64_t)o[i + 1] << (30 - s);
    if (i + 2 < 9) v |= (uint64_t)o[i + 2] << (60 - s);
    w[k] = (uint32_t)v;
  }
}

PM_HD int bg_clz32(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __clz((int)x);
#else
  return x ? __builtin_clz(x) : 32;
#endif
}

// (x f + y g) / 2^30 for non-negative 9-limb x, y and |f| + |g| <= 2^30;
// the low 30 bits of x f + y g are zero by construction.  Returns the
// result's sign; a negative result is negated in place.
PM_HD bool bg_lin(const uint32_t x[9], const uint32_t y[9], int32_t f, int32_t g, uint32_t o[9]) {
  int64_t c = (int64_t)x[0] * f + (int64_t)y[0] * g;
  c >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    c += (int64_t)x[i] * f + (int64_t)y[i] * g;
    o[i - 1] = (uint32_t)c & kBgM;
    c >>= 30;
  }
  o[8] = (uint32_t)c;  // |result| <= 2^256: c is the signed top limb
  const bool neg = c < 0;
  int64_t d = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {  // two's complement negation, selected below
    d -= (i < 8) ? (int64_t)o[i] : (int64_t)(int32_t)o[i];
    const uint32_t t = i < 8 ? ((uint32_t)d & kBgM) : (uint32_t)d;
    d >>= 30;
    o[i] = neg ? t : o[i];
  }
  return neg;
}

// (u f + v g) / 2^30 mod p for u, v in [0, p), |f| + |g| <= 2^30
// (Montgomery division by 2^30), result in [0, p).
template <class P>
PM_HD void bg_lin_mod(const BgConsts<P>& K, const uint32_t u[9], const uint32_t v[9], int32_t f, int32_t g,
                      uint32_t o[9]) {
  int64_t c = (int64_t)u[0] * f + (int64_t)v[0] * g;
  const uint32_t k = ((uint32_t)c * K.pinv) & kBgM;
  c += (int64_t)k * K.p[0];
  c >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    c += (int64_t)u[i] * f + (int64_t)v[i] * g + (int64_t)k * K.p[i];
    o[i - 1] = (uint32_t)c & kBgM;
    c >>= 30;
  }
  // value = o[0..7] + c 2^240 in (-p, 2p): add p if negative, subtract p if >= p
  const int64_t top = c;
  uint32_t s[9], t[9];
  int64_t cs = 0, ct = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const int64_t oi = i < 8 ? (int64_t)o[i] : top;
    cs += oi + K.p[i];
    ct += oi - (int64_t)K.p[i];
    s[i] = i < 8 ? ((uint32_t)cs & kBgM) : (uint32_t)cs;
    t[i] = i < 8 ? ((uint32_t)ct & kBgM) : (uint32_t)ct;
    cs >>= 30;
    ct >>= 30;
  }
  const bool neg = top < 0, ge = !neg && (int32_t)t[8] >= 0;
#pragma unroll
  for (int i = 0; i < 9; i++) o[i] = neg ? s[i] : ge ? t[i] : (i < 8 ? o[i] : (uint32_t)top);
}

// y^-1 mod p for y given as a plain integer in [0, p) (8 x 32-bit limbs);
// 0 -> 0.
template <class P>
PM_HD void bg_inverse(const uint32_t y[8], uint32_t out[8]) {
  const BgConsts<P> K = bg_consts<P>();
  uint32_t a[9], b[9], u[9], v[9];
  bg_split(y, a);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    b[i] = K.p[i];
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0u;
  }
  for (int it = 0; it < K.batches; it++) {
    // n = max(len a, len b, 62); approximations: low 30 bits exact, top 32 bits
    // of a and b at bit n - 32
    int n = 62;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const uint32_t x = a[i] | b[i];
      const int li = 30 * i + 32 - bg_clz32(x);
      n = (x != 0u && li > n) ? li : n;
    }
    const int sh = n - 32, q = sh / 30, off = sh - 30 * q;
    uint32_t a0 = 0, a1 = 0, a2 = 0, b0 = 0, b1 = 0, b2 = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a0 = i == q ? a[i] : a0;
      a1 = i == q + 1 ? a[i] : a1;
      a2 = i == q + 2 ? a[i] : a2;
      b0 = i == q ? b[i] : b0;
      b1 = i == q + 1 ? b[i] : b1;
      b2 = i == q + 2 ? b[i] : b2;
    }
    const uint64_t wa = (uint64_t)a0 | ((uint64_t)a1 << 30) | ((uint64_t)a2 << 60);
    const uint64_t wb = (uint64_t)b0 | ((uint64_t)b1 << 30) | ((uint64_t)b2 << 60);
    uint64_t A = (uint64_t)a[0] | ((uint64_t)(uint32_t)(wa >> off) << 30);
    uint64_t B = (uint64_t)b[0] | ((uint64_t)(uint32_t)(wb >> off) << 30);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int j = 0; j < kBgIter; j++) {
      const bool odd = (A & 1u) != 0;
      const bool sw = odd && A < B;
      const uint64_t tA = sw ? B : A, tB = sw ? A : B;
      const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      A = (odd ? tA - tB : tA) >> 1;
      B = tB;
      f0 = odd ? tf0 - tf1 : tf0;
      g0 = odd ? tg0 - tg1 : tg0;
      f1 = (int32_t)((uint32_t)tf1 << 1);
      g1 = (int32_t)((uint32_t)tg1 << 1);
    }
    uint32_t na[9], nb[9];
    if (bg_lin(a, b, f0, g0, na)) {
      f0 = -f0;
      g0 = -g0;
    }
    if (bg_lin(a, b, f1, g1, nb)) {
      f1 = -f1;
      g1 = -g1;
    }
    uint32_t nu[9], nv[9];
    bg_lin_mod<P>(K, u, v, f0, g0, nu);
    bg_lin_mod<P>(K, u, v, f1, g1, nv);
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a[i] = na[i];
      b[i] = nb[i];
      u[i] = nu[i];
      v[i] = nv[i];
    }
  }
  bg_join(v, out);
}

#if defined(__HIPCC__) || defined(__HIP__)  // device code (the host-only test build skips it)
#if defined(__HIP_DEVICE_COMPILE__)
// lane K's value of x, for every lane of the quad (DPP quad_perm [K,K,K,K])
template <int K>
__device__ __forceinline__ uint32_t bg_qbc(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, K * 0x55, 0xF, 0xF, false);
}
#endif

// Quad-cooperative bg_inverse: the 4 lanes of a quad call it with the same y
// (all 4 active) and all receive y^-1.  Each batch's approximation and 30
// inner steps run redundantly; its four 9-limb linear combinations run one per
// lane (a' on lane 0, b' on 1, u' on 2, v' on 3) with the same uniform code,
// then the quad exchanges them with DPP moves.  The sign of a' (b') negates
// u' (v') afterwards instead of negating (f, g) before: -x mod p is the same
// number, so the result equals bg_inverse's bit for bit.
template <class P>
__device__ void bg_inverse_q(const uint32_t y[8], uint32_t out[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const BgConsts<P> K = bg_consts<P>();
  const uint32_t q = threadIdx.x & 3u;
  const bool ab = q < 2u, odd = (q & 1u) != 0u;
  const uint32_t m_ab = ab ? ~0u : 0u;
  uint32_t a[9], b[9], u[9], v[9];
  bg_split(y, a);
#pragma unroll
  for (int i = 0; i < 9; i++) {
    b[i] = K.p[i];
    u[i] = i == 0 ? 1u : 0u;
    v[i] = 0u;
  }
  for (int it = 0; it < K.batches; it++) {
    int n = 62;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const uint32_t x = a[i] | b[i];
      const int li = 30 * i + 32 - bg_clz32(x);
      n = (x != 0u && li > n) ? li : n;
    }
    const int sh = n - 32, qq = sh / 30, off = sh - 30 * qq;
    uint32_t a0 = 0, a1 = 0, a2 = 0, b0 = 0, b1 = 0, b2 = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a0 = i == qq ? a[i] : a0;
      a1 = i == qq + 1 ? a[i] : a1;
      a2 = i == qq + 2 ? a[i] : a2;
      b0 = i == qq ? b[i] : b0;
      b1 = i == qq + 1 ? b[i] : b1;
      b2 = i == qq + 2 ? b[i] : b2;
    }
    const uint64_t wa = (uint64_t)a0 | ((uint64_t)a1 << 30) | ((uint64_t)a2 << 60);
    const uint64_t wb = (uint64_t)b0 | ((uint64_t)b1 << 30) | ((uint64_t)b2 << 60);
    uint64_t A = (uint64_t)a[0] | ((uint64_t)(uint32_t)(wa >> off) << 30);
    uint64_t B = (uint64_t)b[0] | ((uint64_t)(uint32_t)(wb >> off) << 30);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int j = 0; j < kBgIter; j++) {
      const bool oddA = (A & 1u) != 0;
      const bool sw = oddA && A < B;
      const uint64_t tA = sw ? B : A, tB = sw ? A : B;
      const int32_t tf0 = sw ? f1 : f0, tg0 = sw ? g1 : g0, tf1 = sw ? f0 : f1, tg1 = sw ? g0 : g1;
      A = (oddA ? tA - tB : tA) >> 1;
      B = tB;
      f0 = oddA ? tf0 - tf1 : tf0;
      g0 = oddA ? tg0 - tg1 : tg0;
      f1 = (int32_t)((uint32_t)tf1 << 1);
      g1 = (int32_t)((uint32_t)tg1 << 1);
    }
    // this lane's combination: (x f + y g [+ k p]) / 2^30
    const int32_t f = odd ? f1 : f0, g = odd ? g1 : g0;
    uint32_t x[9], z[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
      x[i] = (a[i] & m_ab) | (u[i] & ~m_ab);
      z[i] = (b[i] & m_ab) | (v[i] & ~m_ab);
    }
    int64_t c = (int64_t)x[0] * f + (int64_t)z[0] * g;
    const uint32_t k = ab ? 0u : (((uint32_t)c * K.pinv) & kBgM);
    c += (int64_t)k * K.p[0];
    c >>= 30;
    uint32_t o[9];
#pragma unroll
    for (int i = 1; i < 9; i++) {
      c += (int64_t)x[i] * f + (int64_t)z[i] * g + (int64_t)k * K.p[i];
      o[i - 1] = (uint32_t)c & kBgM;
      c >>= 30;
    }
    const int64_t top = c;
    o[8] = (uint32_t)c;
    const bool neg = top < 0;
    // candidates: -o (a / b lanes), o + p and o - p (u / v lanes)
    uint32_t rn[9], rs[9], rt[9];
    int64_t dn = 0, cs = 0, ct = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      const int64_t oi = i < 8 ? (int64_t)o[i] : top;
      dn -= oi;
      cs += oi + K.p[i];
      ct += oi - (int64_t)K.p[i];
      rn[i] = i < 8 ? ((uint32_t)dn & kBgM) : (uint32_t)dn;
      rs[i] = i < 8 ? ((uint32_t)cs & kBgM) : (uint32_t)cs;
      rt[i] = i < 8 ? ((uint32_t)ct & kBgM) : (uint32_t)ct;
      dn >>= 30;
      cs >>= 30;
      ct >>= 30;
    }
    const bool ge = !neg && (int32_t)rt[8] >= 0;
    uint32_t r[9];
#pragma unroll
    for (int i = 0; i < 9; i++) r[i] = ab ? (neg ? rn[i] : o[i]) : (neg ? rs[i] : ge ? rt[i] : o[i]);
    // u' (v') is negated mod p when a' (b') was negative
    const uint32_t nb = neg ? 1u : 0u;
    const uint32_t n0 = bg_qbc<0>(nb), n1 = bg_qbc<1>(nb);
    const bool flip = !ab && (odd ? n1 : n0) != 0u;
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) nz |= r[i];
    int64_t dp = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      dp += (int64_t)K.p[i] - (int64_t)r[i];
      const uint32_t pi = i < 8 ? ((uint32_t)dp & kBgM) : (uint32_t)dp;
      dp >>= 30;
      r[i] = (flip && nz != 0u) ? pi : r[i];
    }
#pragma unroll
    for (int i = 0; i < 9; i++) {
      a[i] = bg_qbc<0>(r[i]);
      b[i] = bg_qbc<1>(r[i]);
      u[i] = bg_qbc<2>(r[i]);
      v[i] = bg_qbc<3>(r[i]);
    }
  }
  bg_join(v, out);
#else
  bg_inverse<P>(y, out);
#endif
}
#endif  // __HIPCC__ || __HIP__

// ---------------------------------------------------------------------------
// Variable-time safegcd (Bernstein-Yang divsteps, "Fast constant-time gcd
// computation and modular inversion", IACR ePrint 2019/266; the variable-time
// batching of Wuille's libsecp256k1 modinv write-up): 30 divsteps per batch
// computed from the low 32 bits of f and g only, with runs of zeros shifted
// out at once (count trailing zeros) and up to 6 low bits of g cancelled per
// step with w = f g (f^2 - 2) (-1/f mod 64 by one Newton step), so a batch
// takes ~7 short iterations instead of Pornin's 30 64-bit ones; then the 2x2
// transition matrix (entries < 2^30) is applied to (f, g) and, with a
// Montgomery-style division by 2^30, to (d, e) mod p.  Numbers are 9 signed
// limbs of 30 bits (limb 8 signed).  Same contract as bg_inverse: y plain in
// [0, p), 0 -> 0; the result is bit-identical (the unique inverse in [0, p)).
constexpr int32_t kSgM30 = (int32_t)((1u << 30) - 1u);
constexpr int kSgMaxBatches = 26;  // 750 divsteps: the variable-time bound for 256-bit moduli

struct SgMat {
  int32_t u, v, q, r;
};

PM_HD int sg_ctz32(uint32_t x) {  // x != 0
#if defined(__HIP_DEVICE_COMPILE__)
  return __ffs((int)x) - 1;
#else
  return __builtin_ctz(x);
#endif
}

// 30 divsteps on the low bits of (f, g); returns the new eta
PM_HD int32_t sg_divsteps(int32_t eta, uint32_t f, uint32_t g, SgMat& t) {
  uint32_t u = 1, v = 0, q = 0, r = 1;
  int i = 30;
  for (;;) {
    const int zeros = sg_ctz32(g | (0xFFFFFFFFu << i));  // a sentinel bit stops at i
    g >>= zeros;
    u <<= zeros;
    v <<= zeros;
    eta -= zeros;
    i -= zeros;
    if (i == 0) break;
    if (eta < 0) {  // (f, g) <- (g, -f), with the matrix rows
      const uint32_t tf = f, tu = u, tv = v;
      eta = -eta;
      f = g;
      g = 0u - tf;
      u = q;
      q = 0u - tu;
      v = r;
      r = 0u - tv;
    }
    const int limit = eta + 1 < i ? eta + 1 : i;
    const uint32_t m = (0xFFFFFFFFu >> (32 - limit)) & 63u;
    const uint32_t w = (f * g * (f * f - 2u)) & m;  // g + w f = 0 mod 2^min(limit, 6)
    g += f * w;
    q += u * w;
    r += v * w;
  }
  t = SgMat{(int32_t)u, (int32_t)v, (int32_t)q, (int32_t)r};
  return eta;
}

// (f, g) <- (u f + v g, q f + r g) / 2^30 (exact)
PM_HD void sg_update_fg(int32_t f[9], int32_t g[9], const SgMat& t) {
  int64_t cf = (int64_t)t.u * f[0] + (int64_t)t.v * g[0];
  int64_t cg = (int64_t)t.q * f[0] + (int64_t)t.r * g[0];
  cf >>= 30;
  cg >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cf += (int64_t)t.u * f[i] + (int64_t)t.v * g[i];
    cg += (int64_t)t.q * f[i] + (int64_t)t.r * g[i];
    f[i - 1] = (int32_t)cf & kSgM30;
    g[i - 1] = (int32_t)cg & kSgM30;
    cf >>= 30;
    cg >>= 30;
  }
  f[8] = (int32_t)cf;
  g[8] = (int32_t)cg;
}

// (d, e) <- (u d + v e, q d + r e) / 2^30 mod p, both kept in (-2p, p)
PM_HD void sg_update_de(int32_t d[9], int32_t e[9], const SgMat& t, const int32_t pm[9], uint32_t pinv30) {
  const int32_t sd = d[8] >> 31, se = e[8] >> 31;
  int32_t md = (t.u & sd) + (t.v & se), me = (t.q & sd) + (t.r & se);
  int64_t cd = (int64_t)t.u * d[0] + (int64_t)t.v * e[0];
  int64_t ce = (int64_t)t.q * d[0] + (int64_t)t.r * e[0];
  md -= (int32_t)((pinv30 * (uint32_t)cd + (uint32_t)md) & (uint32_t)kSgM30);
  me -= (int32_t)((pinv30 * (uint32_t)ce + (uint32_t)me) & (uint32_t)kSgM30);
  cd += (int64_t)pm[0] * md;
  ce += (int64_t)pm[0] * me;
  cd >>= 30;
  ce >>= 30;
#pragma unroll
  for (int i = 1; i < 9; i++) {
    cd += (int64_t)t.u * d[i] + (int64_t)t.v * e[i] + (int64_t)pm[i] * md;
    ce += (int64_t)t.q * d[i] + (int64_t)t.r * e[i] + (int64_t)pm[i] * me;
    d[i - 1] = (int32_t)cd & kSgM30;
    e[i - 1] = (int32_t)ce & kSgM30;
    cd >>= 30;
    ce >>= 30;
  }
  d[8] = (int32_t)cd;
  e[8] = (int32_t)ce;
}

// r in (-2p, p) -> sign(s) r mod p in [0, p), limbs in [0, 2^30)
PM_HD void sg_normalize(int32_t r[9], int32_t s, const int32_t pm[9]) {
  int32_t ca = r[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] += pm[i] & ca;
  const int32_t cn = s >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] = (r[i] ^ cn) - cn;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r[i + 1] += r[i] >> 30;
    r[i] &= kSgM30;
  }
  ca = r[8] >> 31;
#pragma unroll
  for (int i = 0; i < 9; i++) r[i] += pm[i] & ca;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    r[i + 1] += r[i] >> 30;
    r[i] &= kSgM30;
  }
}

template <class P>
PM_HD void sg_inverse(const uint32_t y[8], uint32_t out[8]) {
  int32_t pm[9], d[9], e[9], f[9], g[9];
  bg_split(P::MOD, (uint32_t*)pm);
  bg_split(y, (uint32_t*)g);
  const uint32_t pinv30 = (0u - P::INV) & (uint32_t)kSgM30;  // p^-1 mod 2^30
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d[i] = 0;
    e[i] = i == 0 ? 1 : 0;
    f[i] = pm[i];
  }
  int32_t eta = -1;
  for (int it = 0; it < kSgMaxBatches; it++) {
    SgMat t;
    eta = sg_divsteps(eta, (uint32_t)f[0], (uint32_t)g[0], t);
    sg_update_de(d, e, t, pm, pinv30);
    sg_update_fg(f, g, t);
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) nz |= g[i];
    if (nz == 0) break;
  }
  sg_normalize(d, f[8], pm);  // f = +-1
  bg_join((const uint32_t*)d, out);
}

#if defined(__HIPCC__) || defined(__HIP__)
// Quad-cooperative sg_inverse: the 4 lanes of a quad call it with the same y
// (all 4 active).  The divsteps run redundantly; the four 9-limb updates run
// one per lane (f' on lane 0, g' on 1, d' on 2, e' on 3) with uniform code
// and are exchanged with DPP moves.  Same result as sg_inverse.
template <class P>
__device__ void sg_inverse_q(const uint32_t y[8], uint32_t out[8]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t q = threadIdx.x & 3u;
  const bool fg = q < 2u, row1 = (q & 1u) != 0u;
  int32_t pm[9], d[9], e[9], f[9], g[9];
  bg_split(P::MOD, (uint32_t*)pm);
  bg_split(y, (uint32_t*)g);
  const uint32_t pinv30 = (0u - P::INV) & (uint32_t)kSgM30;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    d[i] = 0;
    e[i] = i == 0 ? 1 : 0;
    f[i] = pm[i];
  }
  int32_t eta = -1;
  for (int it = 0; it < kSgMaxBatches; it++) {
    SgMat t;
    eta = sg_divsteps(eta, (uint32_t)f[0], (uint32_t)g[0], t);
    const int32_t a = row1 ? t.q : t.u, b = row1 ? t.r : t.v;
    int32_t x[9], z[9];
#pragma unroll
    for (int i = 0; i < 9; i++) {
      x[i] = fg ? f[i] : d[i];
      z[i] = fg ? g[i] : e[i];
    }
    int64_t c = (int64_t)a * x[0] + (int64_t)b * z[0];
    int32_t md = 0;
    if (!fg) {  // (a d + b e + p md) / 2^30 with md making the low limb vanish
      md = (a & (x[8] >> 31)) + (b & (z[8] >> 31));
      md -= (int32_t)((pinv30 * (uint32_t)c + (uint32_t)md) & (uint32_t)kSgM30);
    }
    c += (int64_t)pm[0] * md;
    c >>= 30;
    int32_t o[9];
#pragma unroll
    for (int i = 1; i < 9; i++) {
      c += (int64_t)a * x[i] + (int64_t)b * z[i] + (int64_t)pm[i] * md;
      o[i - 1] = (int32_t)c & kSgM30;
      c >>= 30;
    }
    o[8] = (int32_t)c;
    int32_t nz = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      f[i] = (int32_t)bg_qbc<0>((uint32_t)o[i]);
      g[i] = (int32_t)bg_qbc<1>((uint32_t)o[i]);
      d[i] = (int32_t)bg_qbc<2>((uint32_t)o[i]);
      e[i] = (int32_t)bg_qbc<3>((uint32_t)o[i]);
      nz |= g[i];
    }
    if (nz == 0) break;
  }
  sg_normalize(d, f[8], pm);
  bg_join((const uint32_t*)d, out);
#else
  sg_inverse<P>(y, out);
#endif
}
#endif  // __HIPCC__ || __HIP__

// Montgomery-form inverse (R = 2^256): a = x R -> x^-1 R.  bg_inverse gives
// (x R)^-1 = x^-1 R^-1; two products by R^2 restore x^-1 R.
template <class P>
PM_HD Fe<P> fe_inv_bgcd(const Fe<P>& a) {
  Fe<P> v, r2;
  sg_inverse<P>(a.l, v.l);  // safegcd: ~1.6x lower latency than bg_inverse (profiles/r05/ab_lazy_step.jsonl)
#pragma unroll
  for (int i = 0; i < 8; i++) r2.l[i] = P::R2[i];
  return fe_mul<P>(fe_mul<P>(v, r2), r2);
}

}  // namespace pm

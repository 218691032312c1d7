// curve29.hpp -- XYZZ group law on the radix-2^29 lazy field (fp29.hpp), used
// by every MSM device kernel after the base conversion.  Same formulas as
// curve.hpp (madd-2008-s, add-2008-s, dbl-2008-s-1, a = 0); the bounds in the
// comments keep every coordinate Norm with X, Y < 3p and ZZ, ZZZ < 2p, so a
// point packs into the 128-byte Xyzz<F> layout (3p < 2^256).  The identity has
// ZZ == 0 exactly (every routine writes an exact zero when its result is O).
#pragma once
#include "curve.hpp"
#include "fp29.hpp"

namespace pm {

template <class F>
struct Xyzz29 {
  F29<F> X, Y, ZZ, ZZZ;
};

template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_inf() {
  return Xyzz29<F>{f29_const<F>(F29Consts<F>::ONE), f29_const<F>(F29Consts<F>::ONE), f29_zero<F>(), f29_zero<F>()};
}
template <class F>
__device__ __forceinline__ bool xyzz29_is_inf(const Xyzz29<F>& p) {
  return f29_is_zero_exact<F>(p.ZZ);
}

// ---------------------------------------------------------- packed storage
template <class F>
__device__ __forceinline__ F29<F> ld29(const uint4* q) {
  const uint4 a = q[0], b = q[1];
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  return f29_unpack<F>(w);
}
template <class F>
__device__ __forceinline__ void st29(uint4* q, const F29<F>& v) {
  uint32_t w[8];
  f29_pack<F>(v, w);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}
template <class F>
__device__ __forceinline__ Xyzz29<F> load_xyzz29(const Xyzz<F>* src) {
  const uint4* q = reinterpret_cast<const uint4*>(src);
  return Xyzz29<F>{ld29<F>(q), ld29<F>(q + 2), ld29<F>(q + 4), ld29<F>(q + 6)};
}
template <class F>
__device__ __forceinline__ void store_xyzz29(Xyzz<F>* dst, const Xyzz29<F>& p) {
  uint4* q = reinterpret_cast<uint4*>(dst);
  st29<F>(q, p.X);
  st29<F>(q + 2, p.Y);
  st29<F>(q + 4, p.ZZ);
  st29<F>(q + 6, p.ZZZ);
}
// affine base in the converted (R261, canonical) packed layout
template <class F>
__device__ __forceinline__ void load_aff29(const uint32_t* p, F29<F>& x, F29<F>& y) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  x = ld29<F>(q);
  y = ld29<F>(q + 2);
}

// ------------------------------------------------------------ doubling
// dbl-2008-s-1 on (X, Y, ZZ, ZZZ); AFF: ZZ = ZZZ = 1 (skips two products).
// Inputs Norm, X, Y < 4p; valid points only (no y = 0 points: odd order).
template <class F, bool AFF>
__device__ __forceinline__ Xyzz29<F> xyzz29_dbl_impl(const F29<F>& X, const F29<F>& Y, const F29<F>& ZZ,
                                                     const F29<F>& ZZZ) {
  using K = F29Consts<F>;
  const F29<F> U = f29_norm<F>(f29_add<F>(Y, Y));              // < 8p
  const F29<F> V = f29_sqr_c<F>(U);                              // < 2p
  const F29<F> W = f29_mul_c<F>(U, V);                           // < 2p
  const F29<F> S = f29_mul_c<F>(X, V);                           // < 2p
  const F29<F> XX = f29_sqr_c<F>(X);                             // < 2p
  const F29<F> M = f29_norm<F>(f29_add<F>(f29_add<F>(XX, XX), XX));  // < 6p
  Xyzz29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(M), f29_add<F>(S, S), K::K8x3)));  // < 3p
  const F29<F> D = f29_norm<F>(f29_sub<F>(S, r.X, K::K6));     // < 8p
  r.Y = f29_mul2n_c<F>(M, D, W, Y);                              // M D - W Y (48p^2, W Y < 8p^2), < 3p
  r.ZZ = AFF ? V : f29_mul_c<F>(V, ZZ);
  r.ZZZ = AFF ? W : f29_mul_c<F>(W, ZZZ);
  return r;
}
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_dbl(const Xyzz29<F>& p) {
  if (xyzz29_is_inf<F>(p)) return p;
  return xyzz29_dbl_impl<F, false>(p.X, p.Y, p.ZZ, p.ZZZ);
}

// ------------------------------------------------- Jacobian doubling chain
// dbl-2009-l (a = 0) on Jacobian (X, Y, Z): 2M + 5S instead of XYZZ's 6M + 3S,
// for pure doubling chains (the accumulator's ladder).  Inputs Norm with
// X, Y < 3p, Z < 4p; outputs the same.  No identity handling: the chain starts
// from an affine non-identity point of odd order, so it never reaches O.
template <class F>
struct Jac29 {
  F29<F> X, Y, Z;
};
template <class F>
__device__ __forceinline__ Jac29<F> jac29_dbl(const Jac29<F>& p) {
  using K = F29Consts<F>;
  const F29<F> A = f29_sqr_c<F>(p.X);                                     // < 2p
  const F29<F> B = f29_sqr_c<F>(p.Y);                                     // < 2p
  const F29<F> C = f29_sqr_c<F>(B);                                       // < 2p
  const F29<F> s = f29_sqr_c<F>(f29_norm<F>(f29_add<F>(p.X, B)));         // (X + B)^2, X + B < 5p
  const F29<F> u = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(s, f29_add<F>(A, C), K::K8x3)));  // (4p, 10p) -> < 3p
  const F29<F> D = f29_reduce3<F>(f29_norm<F>(f29_add<F>(u, u)));         // < 3p
  const F29<F> E = f29_norm<F>(f29_add<F>(f29_add<F>(A, A), A));          // < 6p
  Jac29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(E), f29_add<F>(D, D), K::K8x3)));  // (2p, 10p) -> < 3p
  const F29<F> w = f29_sub<F>(D, r.X, K::K6);                            // loose limbs < 2^31, < 9p
  F29<F> C8 = C;
#pragma unroll
  for (int i = 0; i < 9; i++) C8.l[i] = C.l[i] << 3;
  C8 = f29_reduce3<F>(f29_norm<F>(C8));                                   // 8C < 16p -> < 3p
  r.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_mul_c<F>(E, w), C8, K::K8x3)));  // (5p, 10p) -> < 3p
  const F29<F> yz = f29_mul_c<F>(p.Y, p.Z);                              // < 2p
  r.Z = f29_norm<F>(f29_add<F>(yz, yz));                                  // < 4p
  return r;
}
// Jacobian -> XYZZ storage form (ZZ = Z^2, ZZZ = Z^3, both < 2p)
template <class F>
__device__ __forceinline__ Xyzz29<F> jac29_to_xyzz(const Jac29<F>& p) {
  const F29<F> zz = f29_sqr_c<F>(p.Z);
  return Xyzz29<F>{p.X, p.Y, zz, f29_mul_c<F>(zz, p.Z)};
}

// ------------------------------------------------------------ mixed add
// madd-2008-s: acc + (x2, y2) with the base (canonical, R261) negated when
// `neg`.  The caller tracks the identity of acc (acc_inf) and of the base.
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_madd(const Xyzz29<F>& acc, const F29<F>& x2, const F29<F>& y2in,
                                                 bool& acc_inf) {
  using K = F29Consts<F>;
  if (acc_inf) {
    acc_inf = false;
    return Xyzz29<F>{x2, y2in, f29_const<F>(K::ONE), f29_const<F>(K::ONE)};
  }
  const F29<F> U2 = f29_mul_c<F>(x2, acc.ZZ);                    // < 2p
  const F29<F> S2 = f29_mul_c<F>(y2in, acc.ZZZ);                 // < 2p
  const F29<F> P = f29_norm<F>(f29_sub<F>(U2, acc.X, K::K6));  // < 8p
  const F29<F> R = f29_norm<F>(f29_sub<F>(S2, acc.Y, K::K6));  // < 8p
  if (f29_is_zero_mod<F>(P)) {
    if (f29_is_zero_mod<F>(R)) return xyzz29_dbl_impl<F, true>(x2, y2in, x2, x2);
    acc_inf = true;
    return xyzz29_inf<F>();
  }
  const F29<F> PP = f29_sqr_c<F>(P);                             // 64p^2 < R p
  const F29<F> PPP = f29_mul_c<F>(P, PP);
  const F29<F> Q = f29_mul_c<F>(acc.X, PP);
  Xyzz29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(R), f29_add<F>(PPP, f29_add<F>(Q, Q)), K::K8x3)));
  const F29<F> D = f29_norm<F>(f29_sub<F>(Q, r.X, K::K6));     // < 8p
  r.Y = f29_mul2n_c<F>(R, D, acc.Y, PPP);                        // R D - Y1 PPP (64p^2, 6p^2), < 3p
  r.ZZ = f29_mul_c<F>(acc.ZZ, PP);
  r.ZZZ = f29_mul_c<F>(acc.ZZZ, PPP);
  return r;
}

template <class F>
__device__ __forceinline__ F29<F> f29_neg_canon(const F29<F>& y);

// ----------------------------------------- signed mixed add, bucket loop
// k_accumulate's step: acc + (x2, (-1)^s y2) for a canonical base, with the
// digit's sign folded into R instead of negating y2:
//   R = 8p + (-1)^s S2 - Y1   (limbs: K8x3 >= 3 * 2^29 - 3 covers the
//   -S2 - Y1 case, value in (3p, 10p) for Y1 < 3p), the rest as madd-2008-s,
//   and Y3 = R D - Y1 PPP as one difference of products (f29_mul2n: no
//   negated -Y1, ~34 VALU instructions less per addition than round 2's
//   R D + (6p - Y1) PPP).
// No branches: the caller overwrites the result of a lane whose acc is empty,
// and detects the exceptional P = 0 (acc = +-point) from the output: then
// ZZ3 = ZZ1 P^2 = 0 and X3 = R^2, so X3 = 0 iff acc = point (double it),
// else the sum is O (xyzz29_madd_fix).
// Bounds: R^2 < 100 p^2 < 2^261 p; Y3 = R D - Y1 PPP with R D < 80 p^2 and
// Y1 PPP < 6 p^2, fine for p < 2^254.3 (Pasta, BN254): outputs X, Y < 3p,
// ZZ, ZZZ < 2p.
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_madd_signed(const Xyzz29<F>& acc, const F29<F>& x2, const F29<F>& y2,
                                                        uint32_t negm) {
  using K = F29Consts<F>;
  const F29<F> U2 = f29_mul_c<F>(x2, acc.ZZ);                    // < 2p
  const F29<F> S2 = f29_mul_c<F>(y2, acc.ZZZ);                   // < 2p
  const F29<F> P = f29_norm<F>(f29_sub<F>(U2, acc.X, K::K6));  // < 8p
  F29<F> R;
#pragma unroll
  for (int i = 0; i < 9; i++) R.l[i] = K::K8x3[i] + ((S2.l[i] ^ negm) - negm) - acc.Y.l[i];
  R = f29_norm<F>(R);                                            // < 10p
  const F29<F> PP = f29_sqr_c<F>(P);
  const F29<F> PPP = f29_mul_c<F>(P, PP);
  const F29<F> Q = f29_mul_c<F>(acc.X, PP);
  Xyzz29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(R), f29_add<F>(PPP, f29_add<F>(Q, Q)), K::K8x3)));
  const F29<F> D = f29_norm<F>(f29_sub<F>(Q, r.X, K::K6));     // < 8p
  r.Y = f29_mul2n_c<F>(R, D, acc.Y, PPP);                        // R D - Y1 PPP, < 3p
  r.ZZ = f29_mul_c<F>(acc.ZZ, PP);
  r.ZZZ = f29_mul_c<F>(acc.ZZZ, PPP);
  return r;
}
// Round 5 form of the same step (k_accumulate): X kept lazy (< 9p, reduced
// only when the bucket is stored) and the differences P = U2 - X1 and
// D = Q - X3 left as signed limbs (|limb| < 2^29) feeding the signed-operand
// products of fp29_asm.hpp (v_mad_i64_i32 columns), so neither is offset by
// a multiple of p nor normalised: two normalisations, two 9-limb constant
// adds and the reduce3 of X3 less per addition.  Bounds (p < 2^254.3,
// R = 2^261 > 128p; tests/test_fp29_asm.py::test_lazy_bucket_addition runs
// this sequence through the column interpreter at the extremes):
//   X1 < 9p, Y1 < 3p, ZZ1, ZZZ1 < 2p;  P in (-9p, 2p);  R in (3p, 10p)
//   PP = P^2 < 1.75p;  PPP = P PP in (0.86p, 2.03p] (2 pR added);  Q < 1.14p
//   X3 = R^2 + 8p - PPP - 2Q in (3.7p, 8.92p);  D in (-8.92p, 1.14p)
//   Y3 = R D - Y1 PPP in (0.25p, 2.1p];  ZZ3, ZZZ3 < 2p.
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_madd_lazy(const Xyzz29<F>& acc, const F29<F>& x2, const F29<F>& y2,
                                                      uint32_t negm) {
  using K = F29Consts<F>;
  const F29<F> U2 = f29_mul_c<F>(x2, acc.ZZ);   // < 2p
  const F29<F> S2 = f29_mul_c<F>(y2, acc.ZZZ);  // < 2p
  F29<F> P, R, D;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    P.l[i] = U2.l[i] - acc.X.l[i];
    R.l[i] = K::K8x3[i] + ((S2.l[i] ^ negm) - negm) - acc.Y.l[i];
  }
  R = f29_norm<F>(R);
  const F29<F> PP = f29_sqr_sa_a<F>(P);
  const F29<F> PPP = f29_mul_sa_a<F>(P, PP);
  const F29<F> Q = f29_mul_c<F>(acc.X, PP);
  Xyzz29<F> r;
  r.X = f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(R), f29_add<F>(PPP, f29_add<F>(Q, Q)), K::K8x3));
#pragma unroll
  for (int i = 0; i < 9; i++) D.l[i] = Q.l[i] - r.X.l[i];
  r.Y = f29_mul2n_sb_a<F>(R, D, acc.Y, PPP);
  r.ZZ = f29_mul_c<F>(acc.ZZ, PP);
  r.ZZZ = f29_mul_c<F>(acc.ZZZ, PPP);
  return r;
}
// the stored form of a lazy accumulator (X < 3p, as every bucket consumer expects)
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_settle(const Xyzz29<F>& a) {
  return Xyzz29<F>{f29_reduce3<F>(a.X), a.Y, a.ZZ, a.ZZZ};
}

// The exceptional cases of xyzz29_madd_signed / _lazy (r = its output for a
// non-empty acc).  Returns true when the sum is O.
template <class F>
__device__ __forceinline__ bool xyzz29_madd_fix(Xyzz29<F>& r, const F29<F>& x2, const F29<F>& y2, uint32_t negm) {
  if (!f29_is_zero_mod<F>(r.ZZ)) return false;
  if (!f29_is_zero_mod<F>(f29_reduce3<F>(r.X))) {  // lazy X3 < 9p
    r.ZZ = f29_zero<F>();
    return true;
  }
  r = xyzz29_dbl_impl<F, true>(x2, negm ? f29_neg_canon<F>(y2) : y2, x2, x2);
  return false;
}

// ------------------------------------------------------------ full add
// add-2008-s: p + q, both packed-storage points (identity = ZZ exactly 0).
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_add(const Xyzz29<F>& p, const Xyzz29<F>& q) {
  using K = F29Consts<F>;
  if (xyzz29_is_inf<F>(q)) return p;
  if (xyzz29_is_inf<F>(p)) return q;
  const F29<F> U1 = f29_mul_c<F>(p.X, q.ZZ);
  const F29<F> U2 = f29_mul_c<F>(q.X, p.ZZ);
  const F29<F> S1 = f29_mul_c<F>(p.Y, q.ZZZ);
  const F29<F> S2 = f29_mul_c<F>(q.Y, p.ZZZ);
  const F29<F> P = f29_norm<F>(f29_sub<F>(U2, U1, K::K6));
  const F29<F> R = f29_norm<F>(f29_sub<F>(S2, S1, K::K6));
  if (f29_is_zero_mod<F>(P)) {
    // p == q: the doubling takes X, Y < 4p (an input may be a k_acc_powers_s
    // table point, X, Y < 9.4p: reduce first; never taken in practice)
    if (f29_is_zero_mod<F>(R))
      return xyzz29_dbl<F>(Xyzz29<F>{f29_reduce3<F>(p.X), f29_reduce3<F>(p.Y), p.ZZ, p.ZZZ});
    return xyzz29_inf<F>();
  }
  const F29<F> PP = f29_sqr_c<F>(P);
  const F29<F> PPP = f29_mul_c<F>(P, PP);
  const F29<F> Q = f29_mul_c<F>(U1, PP);
  Xyzz29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_sqr_c<F>(R), f29_add<F>(PPP, f29_add<F>(Q, Q)), K::K8x3)));
  const F29<F> D = f29_norm<F>(f29_sub<F>(Q, r.X, K::K6));     // < 8p
  r.Y = f29_mul2n_c<F>(R, D, S1, PPP);                           // R D - S1 PPP (64p^2, 4p^2), < 3p
  r.ZZ = f29_mul_c<F>(f29_mul_c<F>(p.ZZ, q.ZZ), PP);
  r.ZZZ = f29_mul_c<F>(f29_mul_c<F>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// y -> (2p - y) for a canonical y (the negated base of a signed digit), Norm
template <class F>
__device__ __forceinline__ F29<F> f29_neg_canon(const F29<F>& y) {
  return f29_norm<F>(f29_sub<F>(f29_zero<F>(), y, F29Consts<F>::K2));
}

// affine (R261) of an XYZZ point that is not the identity
template <class F>
__device__ __forceinline__ void xyzz29_to_aff(const Xyzz29<F>& p, F29<F>& x, F29<F>& y) {
  const F29<F> inv = f29_inv<F>(f29_mul_c<F>(p.ZZ, p.ZZZ));  // 1 / (ZZ ZZZ)
  x = f29_canon<F>(f29_mul_c<F>(p.X, f29_mul_c<F>(inv, p.ZZZ)));
  y = f29_canon<F>(f29_mul_c<F>(p.Y, f29_mul_c<F>(inv, p.ZZ)));
}

}  // namespace pm

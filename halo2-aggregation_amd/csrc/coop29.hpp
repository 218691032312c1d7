// coop29.hpp -- quad-cooperative group law for latency-bound chains.
//
// One wave alone issues a v_mad_u64_u32 every ~9 cycles, so a field product
// costs ~0.5 us of latency and a point operation is as slow as its number of
// products.  Here the 4 lanes of a quad hold the same point(s) and split each
// operation's products by dependency level: every lane computes ONE product
// per level (operands picked by its quad index with selects, so the quad
// stays convergent), the results are broadcast inside the quad with DPP
// quad_perm moves (no LDS), and the cheap linear steps are repeated by all 4
// lanes.  Levels per operation:
//   XYZZ add (add-2008-s)          4 instead of 14 products
//   XYZZ dbl (dbl-2008-s-1)        3 instead of 9
//   Jacobian dbl (dbl-2009-l)      3 instead of 7
// Same formulas, same lazy bounds and same results as curve29.hpp (the
// squares are computed as products, which give the same value).
// Precondition: all 4 lanes of every quad are active and hold equal inputs.
#pragma once
#include "curve29.hpp"

namespace pm {

__device__ __forceinline__ uint32_t quad_id() { return threadIdx.x & 3u; }

// value of lane k of this quad (quad_perm [k, k, k, k])
template <int K>
__device__ __forceinline__ uint32_t qbc32(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, K * 0x55, 0xF, 0xF, false);
}
template <int K, class F>
__device__ __forceinline__ F29<F> qbc(const F29<F>& v) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = qbc32<K>(v.l[i]);
  return r;
}
// operand of lane q: bitwise selects (v_bfi_b32) on the limb values.  A
// conditional-expression select of whole objects was turned by the compiler
// into a select of addresses into scratch memory plus loads.
__device__ __forceinline__ uint32_t bsel(uint32_t m, uint32_t a, uint32_t b) { return (a & m) | (b & ~m); }
template <class F>
__device__ __forceinline__ F29<F> qsel(uint32_t q, const F29<F>& a0, const F29<F>& a1, const F29<F>& a2,
                                       const F29<F>& a3) {
  const uint32_t m0 = 0u - (q & 1u), m1 = 0u - ((q >> 1) & 1u);
  F29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = bsel(m1, bsel(m0, a3.l[i], a2.l[i]), bsel(m0, a1.l[i], a0.l[i]));
  return r;
}
// lane q computes a_q * b_q; returns its product
template <class F>
__device__ __forceinline__ F29<F> qmul(uint32_t q, const F29<F>& a0, const F29<F>& b0, const F29<F>& a1,
                                       const F29<F>& b1, const F29<F>& a2, const F29<F>& b2, const F29<F>& a3,
                                       const F29<F>& b3) {
  return f29_mul_c<F>(qsel<F>(q, a0, a1, a2, a3), qsel<F>(q, b0, b1, b2, b3));
}

// dbl-2009-l on Jacobian (X, Y, Z), bounds of jac29_dbl
template <class F>
__device__ __forceinline__ Jac29<F> jac29_dbl_q(const Jac29<F>& p) {
  using K = F29Consts<F>;
  const uint32_t q = quad_id();
  // L1: A = X^2, B = Y^2, YZ = Y Z (operands: lane 0 (X, X), 1 (Y, Y),
  // 2 (Y, Z), 3 (X, X) -- one or two selects per limb instead of qsel's three)
  const uint32_t m12 = (q == 1u || q == 2u) ? ~0u : 0u, m2 = q == 2u ? ~0u : 0u;
  F29<F> o1a, o1b;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    o1a.l[i] = bsel(m12, p.Y.l[i], p.X.l[i]);
    o1b.l[i] = bsel(m2, p.Z.l[i], o1a.l[i]);
  }
  const F29<F> r1 = f29_mul_c<F>(o1a, o1b);
  const F29<F> A = qbc<0, F>(r1), B = qbc<1, F>(r1), YZ = qbc<2, F>(r1);
  // L2: C = B^2, s = (X + B)^2, F = E^2 (E = 3A): three squarings
  const F29<F> t = f29_norm<F>(f29_add<F>(p.X, B));                       // < 5p
  const F29<F> E = f29_norm<F>(f29_add<F>(f29_add<F>(A, A), A));          // < 6p
  const F29<F> r2 = f29_sqr_c<F>(qsel<F>(q, B, t, E, B));
  const F29<F> C = qbc<0, F>(r2), s = qbc<1, F>(r2), FF = qbc<2, F>(r2);
  const F29<F> u = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(s, f29_add<F>(A, C), K::K8x3)));
  const F29<F> D = f29_reduce3<F>(f29_norm<F>(f29_add<F>(u, u)));
  Jac29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(FF, f29_add<F>(D, D), K::K8x3)));
  const F29<F> w = f29_sub<F>(D, r.X, K::K6);
  F29<F> C8 = C;
#pragma unroll
  for (int i = 0; i < 9; i++) C8.l[i] = C.l[i] << 3;
  C8 = f29_reduce3<F>(f29_norm<F>(C8));
  // L3 (every lane): E (D - X3)
  r.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_mul_c<F>(E, w), C8, K::K8x3)));
  r.Z = f29_norm<F>(f29_add<F>(YZ, YZ));
  return r;
}

// The a = 0 doubling of k_acc_powers plus the storage form of the new point.
// dbl-2009-l's values, with every linear combination that can be a product
// turned into one (one quad level costs one product on every lane, whatever
// each lane multiplies, while the linear steps run on all 4 lanes in series):
//   L1  lane 1 B = Y Y, lane 2 Y Z, lane 3 E = (3X) X   (lane 0 idles)
//   L2  lane 0 4C = (4B) B, lane 1 D = (4X) B (= 2((X + B)^2 - A - C)),
//       lane 2 F = E E, lane 3 ZZ3 = Z3 Z3
//   L3  lanes 1, 2 E (D - X3), lane 0 beta X3, lane 3 ZZZ3 = ZZ3 Z3
// X3 = F - 2D, Y3 = E (D - X3) - 2 (4C), Z3 = 2 Y Z.  Against the
// squaring form (A, (X + B)^2 and C as squares, D, E and 8C from additions
// with a normalisation and a reduction each) this drops ~220 instructions of
// the ~610 between the products, for a product instead of a square at L2.
// Bounds (fp29.hpp: operand limbs a_i b_j <= 2^60, a b < R p): X, Y Norm < 3p,
// Z < 4p with limbs < 2^30 (Z3 is not normalised: it only enters products);
// 3X, 4X, 4B have limbs < 2^31 against a Norm partner; the products are
// <= 27 p^2.  X3 = F + 8p - 2D < 10p, Y3 = E w + 8p - 8C < 10p before the
// reduction (Norm, < 3p after it).  Only lanes 1 and 2 compute E (D - X3),
// so only they hold Y3 afterwards; lanes 0 and 3 never read Y and keep a
// bounded dummy there.  Outputs on the owning lanes: X3 (all), Y3 (1, 2),
// ZZ3 < 2p (3), ZZZ3 < 2p (3), beta X3 < 2p (0).
template <class F>
__device__ __forceinline__ Jac29<F> jac29_dbl_q_ext(const Jac29<F>& p, const F29<F>& beta, F29<F>& zz,
                                                    F29<F>& ext) {
  using K = F29Consts<F>;
  const uint32_t q = quad_id();
  const uint32_t m0 = q == 0u ? ~0u : 0u, m01 = q < 2u ? ~0u : 0u, m12 = (q == 1u || q == 2u) ? ~0u : 0u;
  const uint32_t m2 = q == 2u ? ~0u : 0u, m3 = q == 3u ? ~0u : 0u;
  // L1 operands: (X, X) / (Y, Y) / (Y, Z) / (3X, X)
  F29<F> o1a, o1b;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    o1a.l[i] = bsel(m12, p.Y.l[i], bsel(m3, p.X.l[i] * 3u, p.X.l[i]));
    o1b.l[i] = bsel(m2, p.Z.l[i], bsel(m12, p.Y.l[i], p.X.l[i]));
  }
  const F29<F> r1 = f29_mul_c<F>(o1a, o1b);
  const F29<F> B = qbc<1, F>(r1), YZ = qbc<2, F>(r1), E = qbc<3, F>(r1);
  Jac29<F> r;
  r.Z = f29_add<F>(YZ, YZ);  // < 4p, limbs < 2^30
  // L2 operands: (4B, B) / (4X, B) / (E, E) / (Z3, Z3)
  F29<F> o2a, o2b;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    const uint32_t ez = bsel(m2, E.l[i], r.Z.l[i]);
    o2a.l[i] = bsel(m01, bsel(m0, B.l[i], p.X.l[i]) << 2, ez);
    o2b.l[i] = bsel(m01, B.l[i], ez);
  }
  const F29<F> r2 = f29_mul_c<F>(o2a, o2b);
  zz = r2;
  const F29<F> C4 = qbc<0, F>(r2), D = qbc<1, F>(r2), FF = qbc<2, F>(r2);
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(FF, f29_add<F>(D, D), K::K8x3)));
  const F29<F> w = f29_sub<F>(D, r.X, K::K6);
  const F29<F> C8 = f29_add<F>(C4, C4);  // limbs < 2^30 <= K8x3's
  // L3 operands: (beta, X3) / (E, w) / (E, w) / (ZZ3, Z3)
  F29<F> o3a, o3b;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    o3a.l[i] = bsel(m0, beta.l[i], bsel(m3, r2.l[i], E.l[i]));
    o3b.l[i] = bsel(m0, r.X.l[i], bsel(m3, r.Z.l[i], w.l[i]));
  }
  const F29<F> r3 = f29_mul_c<F>(o3a, o3b);
  ext = r3;
  r.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(r3, C8, K::K8x3)));
  return r;
}

// Jacobian -> XYZZ (ZZ = Z^2, ZZZ = Z^3): two levels
template <class F>
__device__ __forceinline__ Xyzz29<F> jac29_to_xyzz_q(const Jac29<F>& p) {
  const F29<F> zz = f29_mul_c<F>(p.Z, p.Z);
  return Xyzz29<F>{p.X, p.Y, zz, f29_mul_c<F>(zz, p.Z)};
}

// dbl-2008-s-1, bounds of xyzz29_dbl_impl<F, false>
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_dbl_q(const Xyzz29<F>& p) {
  using K = F29Consts<F>;
  if (xyzz29_is_inf<F>(p)) return p;
  const uint32_t q = quad_id();
  const F29<F> U = f29_norm<F>(f29_add<F>(p.Y, p.Y));                     // < 8p
  // L1: V = U^2, XX = X^2
  const F29<F> r1 = qmul<F>(q, U, U, p.X, p.X, U, U, p.X, p.X);
  const F29<F> V = qbc<0, F>(r1), XX = qbc<1, F>(r1);
  const F29<F> M = f29_norm<F>(f29_add<F>(f29_add<F>(XX, XX), XX));       // < 6p
  // L2: W = U V, S = X V, ZZ3 = V ZZ, MM = M^2
  const F29<F> r2 = qmul<F>(q, U, V, p.X, V, V, p.ZZ, M, M);
  const F29<F> W = qbc<0, F>(r2), S = qbc<1, F>(r2), ZZ3 = qbc<2, F>(r2), MM = qbc<3, F>(r2);
  Xyzz29<F> r;
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(MM, f29_add<F>(S, S), K::K8x3)));
  const F29<F> D = f29_sub<F>(S, r.X, K::K6);
  // L3: M D, W Y, ZZZ3 = W ZZZ
  const F29<F> r3 = qmul<F>(q, M, D, W, p.Y, W, p.ZZZ, M, D);
  const F29<F> MD = qbc<0, F>(r3), WY = qbc<1, F>(r3);
  r.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(MD, WY, K::K6)));
  r.ZZ = ZZ3;
  r.ZZZ = qbc<2, F>(r3);
  return r;
}

// add-2008-s, bounds and special cases of xyzz29_add
template <class F>
__device__ __forceinline__ Xyzz29<F> xyzz29_add_q(const Xyzz29<F>& p, const Xyzz29<F>& o) {
  using K = F29Consts<F>;
  if (xyzz29_is_inf<F>(o)) return p;
  if (xyzz29_is_inf<F>(p)) return o;
  const uint32_t q = quad_id();
  // L1: U1 = X1 ZZ2, U2 = X2 ZZ1, S1 = Y1 ZZZ2, S2 = Y2 ZZZ1
  const F29<F> r1 = qmul<F>(q, p.X, o.ZZ, o.X, p.ZZ, p.Y, o.ZZZ, o.Y, p.ZZZ);
  const F29<F> U1 = qbc<0, F>(r1), U2 = qbc<1, F>(r1), S1 = qbc<2, F>(r1), S2 = qbc<3, F>(r1);
  const F29<F> P = f29_norm<F>(f29_sub<F>(U2, U1, K::K6));
  const F29<F> R = f29_norm<F>(f29_sub<F>(S2, S1, K::K6));
  if (f29_is_zero_mod<F>(P)) {
    // p == o: reduce first (p may be a k_acc_powers_s table point, X, Y < 9.4p)
    if (f29_is_zero_mod<F>(R))
      return xyzz29_dbl_q<F>(Xyzz29<F>{f29_reduce3<F>(p.X), f29_reduce3<F>(p.Y), p.ZZ, p.ZZZ});
    return xyzz29_inf<F>();
  }
  // L2: PP = P^2, RR = R^2, ZZ12 = ZZ1 ZZ2, ZZZ12 = ZZZ1 ZZZ2
  const F29<F> r2 = qmul<F>(q, P, P, R, R, p.ZZ, o.ZZ, p.ZZZ, o.ZZZ);
  const F29<F> PP = qbc<0, F>(r2), RR = qbc<1, F>(r2), ZZ12 = qbc<2, F>(r2), ZZZ12 = qbc<3, F>(r2);
  // L3: PPP = P PP, Q = U1 PP, ZZ3 = ZZ12 PP
  const F29<F> r3 = qmul<F>(q, P, PP, U1, PP, ZZ12, PP, P, PP);
  const F29<F> PPP = qbc<0, F>(r3), Q = qbc<1, F>(r3);
  Xyzz29<F> r;
  r.ZZ = qbc<2, F>(r3);
  r.X = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(RR, f29_add<F>(PPP, f29_add<F>(Q, Q)), K::K8x3)));
  const F29<F> D = f29_sub<F>(Q, r.X, K::K6);
  // L4: ZZZ3 = ZZZ12 PPP, T = S1 PPP, M = R D
  const F29<F> r4 = qmul<F>(q, ZZZ12, PPP, S1, PPP, R, D, R, D);
  r.ZZZ = qbc<0, F>(r4);
  r.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(qbc<2, F>(r4), qbc<1, F>(r4), K::K6)));
  return r;
}

}  // namespace pm

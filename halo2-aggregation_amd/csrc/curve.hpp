// curve.hpp -- short-Weierstrass a=0 group law for Pallas / Vesta / BN254-G1.
//
// Replaces the pasta_curves `Ep`/`EpAffine` group law ([3P]) used by halo2's
// best_multiexp and by the in-circuit BaseFieldEccChip::{add, mul_var}
// gadgets whose native meaning the reference relies on
// (/root/reference/src/multiopen.rs:393,443-487, src/vanishing.rs:183-187).
//
// Coordinates: buckets and accumulators use XYZZ (x = X/ZZ, y = Y/ZZZ,
// ZZ^3 = ZZZ^2), the cheapest a=0 system for repeated mixed additions:
// mixed add 8M+2S, add 12M+2S, dbl 6M+3S.  The identity is ZZ = 0.  Affine
// points follow the pasta_curves in-memory convention: (x, y) in Montgomery
// form with (0, 0) encoding the identity.  Every special case (P == Q,
// P == -Q, either operand the identity) is handled, so results are exact
// group elements regardless of input order.
#pragma once
#include "fp256.hpp"
#include "inv_bgcd.hpp"

namespace pm {

template <class F>
struct Aff {
  Fe<F> x, y;
};
template <class F>
struct Xyzz {
  Fe<F> X, Y, ZZ, ZZZ;
};

struct PallasCurve {
  using Base = PallasFp;
  using Scalar = VestaFp;
  static constexpr int B = 5;
};
struct VestaCurve {
  using Base = VestaFp;
  using Scalar = PallasFp;
  static constexpr int B = 5;
};
struct Bn254Curve {
  using Base = Bn254Fq;
  using Scalar = Bn254Fr;
  static constexpr int B = 3;
};

template <class F>
PM_HD bool aff_is_inf(const Aff<F>& a) {
  return fe_is_zero<F>(a.x) && fe_is_zero<F>(a.y);
}
template <class F>
PM_HD Aff<F> aff_inf() {
  return Aff<F>{fe_zero<F>(), fe_zero<F>()};
}
template <class F>
PM_HD Aff<F> aff_neg(const Aff<F>& a) {
  // -O = O: neg(0) = 0 keeps (0,0) intact
  return Aff<F>{a.x, fe_neg<F>(a.y)};
}

template <class F>
PM_HD Xyzz<F> xyzz_inf() {
  return Xyzz<F>{fe_one<F>(), fe_one<F>(), fe_zero<F>(), fe_zero<F>()};
}
template <class F>
PM_HD bool xyzz_is_inf(const Xyzz<F>& p) {
  return fe_is_zero<F>(p.ZZ);
}
template <class F>
PM_HD Xyzz<F> xyzz_from_aff(const Aff<F>& a) {
  if (aff_is_inf<F>(a)) return xyzz_inf<F>();
  return Xyzz<F>{a.x, a.y, fe_one<F>(), fe_one<F>()};
}
template <class F>
PM_HD Xyzz<F> xyzz_neg(const Xyzz<F>& p) {
  return Xyzz<F>{p.X, fe_neg<F>(p.Y), p.ZZ, p.ZZZ};
}

// dbl-2008-s-1 (a = 0)
template <class F>
PM_HD Xyzz<F> xyzz_dbl(const Xyzz<F>& p) {
  if (xyzz_is_inf<F>(p) || fe_is_zero<F>(p.Y)) return xyzz_inf<F>();
  const Fe<F> U = fe_dbl<F>(p.Y);
  const Fe<F> V = fe_sqr<F>(U);
  const Fe<F> W = fe_mul<F>(U, V);
  const Fe<F> S = fe_mul<F>(p.X, V);
  const Fe<F> XX = fe_sqr<F>(p.X);
  const Fe<F> M = fe_add<F>(fe_dbl<F>(XX), XX);
  Xyzz<F> r;
  r.X = fe_sub<F>(fe_sqr<F>(M), fe_dbl<F>(S));
  r.Y = fe_sub<F>(fe_mul<F>(M, fe_sub<F>(S, r.X)), fe_mul<F>(W, p.Y));
  r.ZZ = fe_mul<F>(V, p.ZZ);
  r.ZZZ = fe_mul<F>(W, p.ZZZ);
  return r;
}

// mdbl-2008-s-1: double an affine point (not the identity, y != 0)
template <class F>
PM_HD Xyzz<F> xyzz_dbl_aff(const Aff<F>& a) {
  if (aff_is_inf<F>(a) || fe_is_zero<F>(a.y)) return xyzz_inf<F>();
  const Fe<F> U = fe_dbl<F>(a.y);
  const Fe<F> V = fe_sqr<F>(U);
  const Fe<F> W = fe_mul<F>(U, V);
  const Fe<F> S = fe_mul<F>(a.x, V);
  const Fe<F> XX = fe_sqr<F>(a.x);
  const Fe<F> M = fe_add<F>(fe_dbl<F>(XX), XX);
  Xyzz<F> r;
  r.X = fe_sub<F>(fe_sqr<F>(M), fe_dbl<F>(S));
  r.Y = fe_sub<F>(fe_mul<F>(M, fe_sub<F>(S, r.X)), fe_mul<F>(W, a.y));
  r.ZZ = V;
  r.ZZZ = W;
  return r;
}

// madd-2008-s: p + a (a affine)
template <class F>
PM_HD Xyzz<F> xyzz_add_aff(const Xyzz<F>& p, const Aff<F>& a) {
  if (aff_is_inf<F>(a)) return p;
  if (xyzz_is_inf<F>(p)) return Xyzz<F>{a.x, a.y, fe_one<F>(), fe_one<F>()};
  const Fe<F> U2 = fe_mul<F>(a.x, p.ZZ);
  const Fe<F> S2 = fe_mul<F>(a.y, p.ZZZ);
  const Fe<F> P = fe_sub<F>(U2, p.X);
  const Fe<F> R = fe_sub<F>(S2, p.Y);
  if (fe_is_zero<F>(P)) {
    if (fe_is_zero<F>(R)) return xyzz_dbl_aff<F>(a);
    return xyzz_inf<F>();
  }
  const Fe<F> PP = fe_sqr<F>(P);
  const Fe<F> PPP = fe_mul<F>(P, PP);
  const Fe<F> Q = fe_mul<F>(p.X, PP);
  Xyzz<F> r;
  r.X = fe_sub<F>(fe_sub<F>(fe_sqr<F>(R), PPP), fe_dbl<F>(Q));
  r.Y = fe_sub<F>(fe_mul<F>(R, fe_sub<F>(Q, r.X)), fe_mul<F>(p.Y, PPP));
  r.ZZ = fe_mul<F>(p.ZZ, PP);
  r.ZZZ = fe_mul<F>(p.ZZZ, PPP);
  return r;
}

// add-2008-s: p + q
template <class F>
PM_HD Xyzz<F> xyzz_add(const Xyzz<F>& p, const Xyzz<F>& q) {
  if (xyzz_is_inf<F>(q)) return p;
  if (xyzz_is_inf<F>(p)) return q;
  const Fe<F> U1 = fe_mul<F>(p.X, q.ZZ);
  const Fe<F> U2 = fe_mul<F>(q.X, p.ZZ);
  const Fe<F> S1 = fe_mul<F>(p.Y, q.ZZZ);
  const Fe<F> S2 = fe_mul<F>(q.Y, p.ZZZ);
  const Fe<F> P = fe_sub<F>(U2, U1);
  const Fe<F> R = fe_sub<F>(S2, S1);
  if (fe_is_zero<F>(P)) {
    if (fe_is_zero<F>(R)) return xyzz_dbl<F>(p);
    return xyzz_inf<F>();
  }
  const Fe<F> PP = fe_sqr<F>(P);
  const Fe<F> PPP = fe_mul<F>(P, PP);
  const Fe<F> Q = fe_mul<F>(U1, PP);
  Xyzz<F> r;
  r.X = fe_sub<F>(fe_sub<F>(fe_sqr<F>(R), PPP), fe_dbl<F>(Q));
  r.Y = fe_sub<F>(fe_mul<F>(R, fe_sub<F>(Q, r.X)), fe_mul<F>(S1, PPP));
  r.ZZ = fe_mul<F>(fe_mul<F>(p.ZZ, q.ZZ), PP);
  r.ZZZ = fe_mul<F>(fe_mul<F>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

template <class F>
PM_HD Aff<F> xyzz_to_aff(const Xyzz<F>& p) {
  if (xyzz_is_inf<F>(p)) return aff_inf<F>();
  const Fe<F> inv = fe_inv_bgcd<F>(fe_mul<F>(p.ZZ, p.ZZZ));  // 1/(ZZ*ZZZ), binary GCD
  Aff<F> a;
  a.x = fe_mul<F>(p.X, fe_mul<F>(inv, p.ZZZ));  // X/ZZ
  a.y = fe_mul<F>(p.Y, fe_mul<F>(inv, p.ZZ));   // Y/ZZZ
  return a;
}

template <class F>
PM_HD Xyzz<F> xyzz_dbl_n(Xyzz<F> p, int n) {
  for (int i = 0; i < n; i++) p = xyzz_dbl<F>(p);
  return p;
}

}  // namespace pm

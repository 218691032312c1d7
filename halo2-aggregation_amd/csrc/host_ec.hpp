// host_ec.hpp -- 64-bit-limb host arithmetic for the serial tail of the MSM.
//
// A single wave on the GPU pays ~7 us per dependent EC addition (a Montgomery
// product is a ~100-long v_mad_u64_u32 dependency chain), while an x86 core
// with 64x64->128 multiplies does one in well under 1 us.  The MSM therefore
// ends on the host: the GPU delivers, per window w, the bit sums G_{w,b} and
// sum_j T_{w,j}; the host evaluates  sum_w 2^{o_w} (sum_j T_{w,j} +
// sum_b 2^{b + log2 L1} G_{w,b})  as ONE Horner over absolute bit positions
// (~256 doublings + ~W*(NB2+1) additions) -- the same group element as the
// per-window + cross-window Horner, with no per-window serial chain.
//
// Same representation as the device (Montgomery, R = 2^256, XYZZ); the u32
// limb layout of Fe<P> is bit-identical to 4 x u64 little-endian.
#pragma once
#include <stdint.h>
#include <string.h>

#include "curve.hpp"

namespace pm {
namespace host {

typedef unsigned __int128 u128;

template <class P>
struct F64 {
  static constexpr uint64_t mod(int i) { return (uint64_t)P::MOD[2 * i] | ((uint64_t)P::MOD[2 * i + 1] << 32); }
  static constexpr uint64_t inv() {  // -p^-1 mod 2^64 (Newton from 1)
    uint64_t p0 = mod(0), x = 1;
    for (int i = 0; i < 7; i++) x *= 2 - p0 * x;
    return (uint64_t)0 - x;
  }
};

template <class P>
struct E {
  uint64_t v[4];
};

template <class P>
inline bool is_zero(const E<P>& a) {
  return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0;
}

// Field elements are canonical (< p) on entry and exit.  Every modulus here
// is below 2^255, so a sum of two never carries out of 4 words and one
// conditional subtraction reduces it.  Add / sub / the products' final step
// are branch-free add/adc (sub/sbb) chains with cmov: the u128 forms GCC
// emitted spilled through the stack (~7-10 ns per add on the container's
// Xeon, tools/host_field_bench.cpp).
template <class P>
struct PMod {
  static constexpr uint64_t v[4] = {F64<P>::mod(0), F64<P>::mod(1), F64<P>::mod(2), F64<P>::mod(3)};
};

// t < 2p -> t mod p
template <class P>
inline E<P> reduce_once(uint64_t t0, uint64_t t1, uint64_t t2, uint64_t t3) {
  uint64_t d0 = t0, d1 = t1, d2 = t2, d3 = t3;
  asm("subq %[p0], %[d0]\n\t"
      "sbbq %[p1], %[d1]\n\t"
      "sbbq %[p2], %[d2]\n\t"
      "sbbq %[p3], %[d3]\n\t"
      "cmovcq %[t0], %[d0]\n\t"
      "cmovcq %[t1], %[d1]\n\t"
      "cmovcq %[t2], %[d2]\n\t"
      "cmovcq %[t3], %[d3]"
      : [d0] "+&r"(d0), [d1] "+&r"(d1), [d2] "+&r"(d2), [d3] "+&r"(d3)
      : [t0] "r"(t0), [t1] "r"(t1), [t2] "r"(t2), [t3] "r"(t3), [p0] "m"(PMod<P>::v[0]), [p1] "m"(PMod<P>::v[1]),
        [p2] "m"(PMod<P>::v[2]), [p3] "m"(PMod<P>::v[3])
      : "cc");
  E<P> r;
  r.v[0] = d0;
  r.v[1] = d1;
  r.v[2] = d2;
  r.v[3] = d3;
  return r;
}

template <class P>
inline E<P> add(const E<P>& a, const E<P>& b) {
  uint64_t t0 = a.v[0], t1 = a.v[1], t2 = a.v[2], t3 = a.v[3];
  asm("addq %[b0], %[t0]\n\t"
      "adcq %[b1], %[t1]\n\t"
      "adcq %[b2], %[t2]\n\t"
      "adcq %[b3], %[t3]"
      : [t0] "+r"(t0), [t1] "+r"(t1), [t2] "+r"(t2), [t3] "+r"(t3)
      : [b0] "rm"(b.v[0]), [b1] "rm"(b.v[1]), [b2] "rm"(b.v[2]), [b3] "rm"(b.v[3])
      : "cc");
  return reduce_once<P>(t0, t1, t2, t3);
}

template <class P>
inline E<P> sub(const E<P>& a, const E<P>& b) {
  uint64_t t0 = a.v[0], t1 = a.v[1], t2 = a.v[2], t3 = a.v[3], m;
  asm("subq %[b0], %[t0]\n\t"
      "sbbq %[b1], %[t1]\n\t"
      "sbbq %[b2], %[t2]\n\t"
      "sbbq %[b3], %[t3]\n\t"
      "sbbq %[m], %[m]"  // m = 0 - borrow: add p back on a borrow, branch-free
      : [t0] "+r"(t0), [t1] "+r"(t1), [t2] "+r"(t2), [t3] "+r"(t3), [m] "=&r"(m)
      : [b0] "rm"(b.v[0]), [b1] "rm"(b.v[1]), [b2] "rm"(b.v[2]), [b3] "rm"(b.v[3])
      : "cc");
  const uint64_t q0 = PMod<P>::v[0] & m, q1 = PMod<P>::v[1] & m, q2 = PMod<P>::v[2] & m, q3 = PMod<P>::v[3] & m;
  asm("addq %[q0], %[t0]\n\t"
      "adcq %[q1], %[t1]\n\t"
      "adcq %[q2], %[t2]\n\t"
      "adcq %[q3], %[t3]"
      : [t0] "+r"(t0), [t1] "+r"(t1), [t2] "+r"(t2), [t3] "+r"(t3)
      : [q0] "r"(q0), [q1] "r"(q1), [q2] "r"(q2), [q3] "r"(q3)
      : "cc");
  E<P> r;
  r.v[0] = t0;
  r.v[1] = t1;
  r.v[2] = t2;
  r.v[3] = t3;
  return r;
}

// CIOS Montgomery product, 4 x 64, "no-carry" form: every modulus here has
// its top limb below 2^63 - 1, so the running t never needs a fifth word
// (t < 2p throughout) and one conditional subtraction finishes.
template <class P>
inline E<P> mul(const E<P>& a, const E<P>& b) {
  constexpr uint64_t INV = F64<P>::inv();
  constexpr uint64_t p0 = F64<P>::mod(0), p1 = F64<P>::mod(1), p2 = F64<P>::mod(2), p3 = F64<P>::mod(3);
  static_assert(p3 < (1ull << 63) - 1, "no-carry CIOS (and the carry-free add) need a spare top bit");
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  for (int i = 0; i < 4; i++) {
    const uint64_t bi = b.v[i];
    u128 A = (u128)a.v[0] * bi + t0;
    const uint64_t m = (uint64_t)A * INV;
    u128 C = (u128)m * p0 + (uint64_t)A;
    A >>= 64;
    C >>= 64;
    A += (u128)a.v[1] * bi + t1;
    C += (u128)m * p1 + (uint64_t)A;
    t0 = (uint64_t)C;
    A >>= 64;
    C >>= 64;
    A += (u128)a.v[2] * bi + t2;
    C += (u128)m * p2 + (uint64_t)A;
    t1 = (uint64_t)C;
    A >>= 64;
    C >>= 64;
    A += (u128)a.v[3] * bi + t3;
    C += (u128)m * p3 + (uint64_t)A;
    t2 = (uint64_t)C;
    A >>= 64;
    C >>= 64;
    t3 = (uint64_t)C + (uint64_t)A;
  }
  return reduce_once<P>(t0, t1, t2, t3);
}

// The same product with BMI2 / ADX: CIOS, every round one mulx row of a b_i
// (lows on the OF chain, highs on the CF chain) and one of m p, m = t_0
// (-p^-1) mod 2^64, ~25 instructions per round instead of ~55 with
// mul / adc (the compiler's form keeps rax / rdx busy and spills).  Same
// no-carry bound as mul().  Only reached through horner_steps_bmi2 (engine.hpp),
// which runs after a CPU check.
template <class P>
inline E<P> mul_adx(const E<P>& a, const E<P>& b) {
  static constexpr uint64_t INV = F64<P>::inv();
  static constexpr uint64_t PM[4] = {F64<P>::mod(0), F64<P>::mod(1), F64<P>::mod(2), F64<P>::mod(3)};
  uint64_t t0 = 0, t1 = 0, t2 = 0, t3 = 0, t4, hi;
  for (int i = 0; i < 4; i++) {
    asm("movq %[bi], %%rdx\n\t"
        "xorl %%eax, %%eax\n\t"
        "mulxq %[a0], %%rax, %[hi]\n\t"
        "adoxq %%rax, %[t0]\n\t"
        "adcxq %[hi], %[t1]\n\t"
        "mulxq %[a1], %%rax, %[hi]\n\t"
        "adoxq %%rax, %[t1]\n\t"
        "adcxq %[hi], %[t2]\n\t"
        "mulxq %[a2], %%rax, %[hi]\n\t"
        "adoxq %%rax, %[t2]\n\t"
        "adcxq %[hi], %[t3]\n\t"
        "mulxq %[a3], %%rax, %[t4]\n\t"
        "adoxq %%rax, %[t3]\n\t"
        "movl $0, %%eax\n\t"
        "adcxq %%rax, %[t4]\n\t"
        "adoxq %%rax, %[t4]\n\t"
        // m = t0 * INV; t = (t + m p) / 2^64
        "movq %[t0], %%rdx\n\t"
        "imulq %[inv], %%rdx\n\t"
        "xorl %%eax, %%eax\n\t"
        "mulxq %[p0], %%rax, %[hi]\n\t"
        "adcxq %[t0], %%rax\n\t"
        "movq %[hi], %[t0]\n\t"
        "adcxq %[t1], %[t0]\n\t"
        "mulxq %[p1], %%rax, %[t1]\n\t"
        "adoxq %%rax, %[t0]\n\t"
        "adcxq %[t2], %[t1]\n\t"
        "mulxq %[p2], %%rax, %[t2]\n\t"
        "adoxq %%rax, %[t1]\n\t"
        "adcxq %[t3], %[t2]\n\t"
        "mulxq %[p3], %%rax, %[t3]\n\t"
        "adoxq %%rax, %[t2]\n\t"
        "movl $0, %%eax\n\t"
        "adcxq %%rax, %[t3]\n\t"
        "adoxq %[t4], %[t3]"
        : [t0] "+&r"(t0), [t1] "+&r"(t1), [t2] "+&r"(t2), [t3] "+&r"(t3), [t4] "=&r"(t4), [hi] "=&r"(hi)
        : [bi] "m"(b.v[i]), [a0] "m"(a.v[0]), [a1] "m"(a.v[1]), [a2] "m"(a.v[2]), [a3] "m"(a.v[3]),
          [p0] "m"(PM[0]), [p1] "m"(PM[1]), [p2] "m"(PM[2]), [p3] "m"(PM[3]), [inv] "m"(INV)
        : "rax", "rdx", "cc");
  }
  return reduce_once<P>(t0, t1, t2, t3);
}

template <class P>
struct Pt {  // XYZZ, ZZ == 0 is the identity
  E<P> X, Y, ZZ, ZZZ;
};

template <class P>
inline Pt<P> inf() {
  Pt<P> r;
  memset(&r, 0, sizeof(r));
  return r;
}

template <class P, bool ADX>
inline E<P> mulv(const E<P>& a, const E<P>& b) {
  if constexpr (ADX) return mul_adx<P>(a, b);
  else return mul<P>(a, b);
}

template <class P, bool ADX = false>
inline Pt<P> dbl(const Pt<P>& p) {
  if (is_zero(p.ZZ) || is_zero(p.Y)) return inf<P>();
  const E<P> U = add(p.Y, p.Y);
  const E<P> V = mulv<P, ADX>(U, U);
  const E<P> W = mulv<P, ADX>(U, V);
  const E<P> S = mulv<P, ADX>(p.X, V);
  const E<P> XX = mulv<P, ADX>(p.X, p.X);
  const E<P> M = add(add(XX, XX), XX);
  Pt<P> r;
  r.X = sub(mulv<P, ADX>(M, M), add(S, S));
  r.Y = sub(mulv<P, ADX>(M, sub(S, r.X)), mulv<P, ADX>(W, p.Y));
  r.ZZ = mulv<P, ADX>(V, p.ZZ);
  r.ZZZ = mulv<P, ADX>(W, p.ZZZ);
  return r;
}

template <class P, bool ADX = false>
inline Pt<P> addp(const Pt<P>& p, const Pt<P>& q) {
  if (is_zero(q.ZZ)) return p;
  if (is_zero(p.ZZ)) return q;
  const E<P> U1 = mulv<P, ADX>(p.X, q.ZZ);
  const E<P> U2 = mulv<P, ADX>(q.X, p.ZZ);
  const E<P> S1 = mulv<P, ADX>(p.Y, q.ZZZ);
  const E<P> S2 = mulv<P, ADX>(q.Y, p.ZZZ);
  const E<P> Pd = sub(U2, U1);
  const E<P> R = sub(S2, S1);
  if (is_zero(Pd)) {
    if (is_zero(R)) return dbl<P, ADX>(p);
    return inf<P>();
  }
  const E<P> PP = mulv<P, ADX>(Pd, Pd);
  const E<P> PPP = mulv<P, ADX>(Pd, PP);
  const E<P> Q = mulv<P, ADX>(U1, PP);
  Pt<P> r;
  r.X = sub(sub(mulv<P, ADX>(R, R), PPP), add(Q, Q));
  r.Y = sub(mulv<P, ADX>(R, sub(Q, r.X)), mulv<P, ADX>(S1, PPP));
  r.ZZ = mulv<P, ADX>(mulv<P, ADX>(p.ZZ, q.ZZ), PP);
  r.ZZZ = mulv<P, ADX>(mulv<P, ADX>(p.ZZZ, q.ZZZ), PPP);
  return r;
}

// Jacobian (x = X / Z^2, y = Y / Z^3; Z == 0 is the identity) for pure
// doubling chains: dbl-2009-l (a = 0) is 2M + 5S against XYZZ's 6M + 3S, and
// the small-MSM Horner (engine.hpp small_horner) spends 128 of its 161 group
// operations doubling.  Additions: add-2007-bl (11M + 5S).
template <class P>
struct Jac {
  E<P> X, Y, Z;
};

template <class P, bool ADX = false>
inline Jac<P> jdbl(const Jac<P>& p) {
  if (is_zero(p.Z)) return p;  // (no y = 0 points: every group here has odd order)
  const E<P> A = mulv<P, ADX>(p.X, p.X);
  const E<P> B = mulv<P, ADX>(p.Y, p.Y);
  const E<P> YZ = mulv<P, ADX>(p.Y, p.Z);
  const E<P> C = mulv<P, ADX>(B, B);
  const E<P> xb = add(p.X, B);
  const E<P> t = mulv<P, ADX>(xb, xb);
  const E<P> u = sub(t, add(A, C));
  const E<P> D = add(u, u);
  const E<P> Ee = add(add(A, A), A);
  const E<P> F = mulv<P, ADX>(Ee, Ee);
  Jac<P> r;
  r.X = sub(F, add(D, D));
  const E<P> C2 = add(C, C), C4 = add(C2, C2);
  r.Y = sub(mulv<P, ADX>(Ee, sub(D, r.X)), add(C4, C4));
  r.Z = add(YZ, YZ);
  return r;
}

template <class P, bool ADX = false>
inline Jac<P> jadd(const Jac<P>& p, const Jac<P>& q) {
  if (is_zero(q.Z)) return p;
  if (is_zero(p.Z)) return q;
  const E<P> Z1Z1 = mulv<P, ADX>(p.Z, p.Z), Z2Z2 = mulv<P, ADX>(q.Z, q.Z);
  const E<P> U1 = mulv<P, ADX>(p.X, Z2Z2), U2 = mulv<P, ADX>(q.X, Z1Z1);
  const E<P> S1 = mulv<P, ADX>(mulv<P, ADX>(p.Y, q.Z), Z2Z2);
  const E<P> S2 = mulv<P, ADX>(mulv<P, ADX>(q.Y, p.Z), Z1Z1);
  const E<P> H = sub(U2, U1), Rh = sub(S2, S1);
  if (is_zero(H)) {
    if (is_zero(Rh)) return jdbl<P, ADX>(p);
    Jac<P> o;
    memset(&o, 0, sizeof(o));
    return o;
  }
  const E<P> H2 = add(H, H);
  const E<P> I = mulv<P, ADX>(H2, H2);
  const E<P> J = mulv<P, ADX>(H, I);
  const E<P> r = add(Rh, Rh);
  const E<P> V = mulv<P, ADX>(U1, I);
  Jac<P> o;
  o.X = sub(sub(mulv<P, ADX>(r, r), J), add(V, V));
  const E<P> SJ = mulv<P, ADX>(S1, J);
  o.Y = sub(mulv<P, ADX>(r, sub(V, o.X)), add(SJ, SJ));
  const E<P> zs = add(p.Z, q.Z);
  o.Z = mulv<P, ADX>(sub(mulv<P, ADX>(zs, zs), add(Z1Z1, Z2Z2)), H);
  return o;
}

// Jacobian -> XYZZ (ZZ = Z^2, ZZZ = Z^3)
template <class P, bool ADX = false>
inline Pt<P> jac_to_xyzz(const Jac<P>& p) {
  Pt<P> r;
  r.X = p.X;
  r.Y = p.Y;
  r.ZZ = mulv<P, ADX>(p.Z, p.Z);
  r.ZZZ = mulv<P, ADX>(r.ZZ, p.Z);
  return r;
}

// reinterpret a device Xyzz<P> (8 x u32 LE limbs per coordinate)
template <class P>
inline Pt<P> from_dev(const Xyzz<P>& d) {
  Pt<P> r;
  static_assert(sizeof(Xyzz<P>) == sizeof(Pt<P>), "layout");
  memcpy(&r, &d, sizeof(r));
  return r;
}
template <class P>
inline Xyzz<P> to_dev(const Pt<P>& h) {
  Xyzz<P> r;
  memcpy(&r, &h, sizeof(r));
  return r;
}

}  // namespace host

// the host tail's BMI2 / ADX product (host::mul_adx) may run on this CPU
inline bool host_has_bmi2() {
  static const bool has = __builtin_cpu_supports("bmi2") && __builtin_cpu_supports("adx");
  return has;
}
}  // namespace pm

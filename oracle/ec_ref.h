/* ec_ref.h -- TEST INFRASTRUCTURE ONLY: the 4 x u64 Montgomery field and
 * Jacobian group law shared by the C restatements in oracle/ (msm_ref.c:
 * halo2 best_multiexp / best_fft; accum_ref.c: the multiopen accumulator and
 * its Blake2b transcript).  Never included by the product library.
 * pasta_curves / pairing_bn256 layout: Montgomery R = 2^256, 4 x u64 LE,
 * affine identity (0, 0). */
#ifndef EC_REF_H
#define EC_REF_H
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>

typedef uint64_t u64;
typedef unsigned __int128 u128;

typedef struct {
  u64 p[4];
  u64 inv;    /* -p^-1 mod 2^64 */
  u64 one[4]; /* R mod p */
} Field;

typedef struct {
  Field fp;   /* base field */
  Field fr;   /* scalar field */
  int b;      /* y^2 = x^3 + b */
  int gx_neg_one; /* generator x = -1 (Pasta) else x = 1 (BN254) */
} CurveDef;

static const CurveDef CURVES[3] = {
    /* Pallas: base = Fp(pallas), scalar = Fq(vesta base) */
    {{{0x992d30ed00000001ull, 0x224698fc094cf91bull, 0x0000000000000000ull, 0x4000000000000000ull},
      0x992d30ecffffffffull,
      {0x34786d38fffffffdull, 0x992c350be41914adull, 0xffffffffffffffffull, 0x3fffffffffffffffull}},
     {{0x8c46eb2100000001ull, 0x224698fc0994a8ddull, 0x0000000000000000ull, 0x4000000000000000ull},
      0x8c46eb20ffffffffull,
      {0x5b2b3e9cfffffffdull, 0x992c350be3420567ull, 0xffffffffffffffffull, 0x3fffffffffffffffull}},
     5, 1},
    /* Vesta: base = Fq, scalar = Fp */
    {{{0x8c46eb2100000001ull, 0x224698fc0994a8ddull, 0x0000000000000000ull, 0x4000000000000000ull},
      0x8c46eb20ffffffffull,
      {0x5b2b3e9cfffffffdull, 0x992c350be3420567ull, 0xffffffffffffffffull, 0x3fffffffffffffffull}},
     {{0x992d30ed00000001ull, 0x224698fc094cf91bull, 0x0000000000000000ull, 0x4000000000000000ull},
      0x992d30ecffffffffull,
      {0x34786d38fffffffdull, 0x992c350be41914adull, 0xffffffffffffffffull, 0x3fffffffffffffffull}},
     5, 1},
    /* BN254 G1 */
    {{{0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
      0x87d20782e4866389ull,
      {0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull, 0x0e0a77c19a07df2full}},
     {{0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
      0xc2e1f593efffffffull,
      {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull, 0x0e0a77c19a07df2full}},
     3, 0},
};

/* ------------------------------------------------------------- field ops */
static inline int geq(const u64 a[4], const u64 b[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > b[i]) return 1;
    if (a[i] < b[i]) return 0;
  }
  return 1;
}
static inline void sub4(u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 br = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - b[i] - br;
    r[i] = (u64)d;
    br = (u64)(d >> 64) & 1;
  }
}
static inline void f_add(const Field* F, u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[4], c = 0;
  for (int i = 0; i < 4; i++) {
    u128 s = (u128)a[i] + b[i] + c;
    t[i] = (u64)s;
    c = (u64)(s >> 64);
  }
  if (c || geq(t, F->p)) sub4(t, t, F->p);
  memcpy(r, t, 32);
}
static inline void f_sub(const Field* F, u64 r[4], const u64 a[4], const u64 b[4]) {
  if (geq(a, b)) {
    sub4(r, a, b);
  } else {
    u64 t[4];
    sub4(t, b, a);
    sub4(r, F->p, t);
  }
}
static inline void f_mul(const Field* F, u64 r[4], const u64 a[4], const u64 b[4]) {
  u64 t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    u64 carry = 0;
    u128 uv;
    for (int j = 0; j < 4; j++) {
      uv = (u128)a[j] * b[i] + t[j] + carry;
      t[j] = (u64)uv;
      carry = (u64)(uv >> 64);
    }
    uv = (u128)t[4] + carry;
    t[4] = (u64)uv;
    t[5] = (u64)(uv >> 64);
    u64 m = t[0] * F->inv;
    uv = (u128)m * F->p[0] + t[0];
    carry = (u64)(uv >> 64);
    for (int j = 1; j < 4; j++) {
      uv = (u128)m * F->p[j] + t[j] + carry;
      t[j - 1] = (u64)uv;
      carry = (u64)(uv >> 64);
    }
    uv = (u128)t[4] + carry;
    t[3] = (u64)uv;
    t[4] = t[5] + (u64)(uv >> 64);
  }
  if (t[4] || geq(t, F->p)) sub4(t, t, F->p);
  memcpy(r, t, 32);
}
static inline int f_is_zero(const u64 a[4]) { return (a[0] | a[1] | a[2] | a[3]) == 0; }
static inline void f_inv(const Field* F, u64 r[4], const u64 a[4]) {
  u64 e[4], two[4] = {2, 0, 0, 0}, acc[4];
  sub4(e, F->p, two);
  memcpy(acc, F->one, 32);
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      f_mul(F, acc, acc, acc);
      if ((e[i] >> b) & 1) f_mul(F, acc, acc, a);
    }
  memcpy(r, acc, 32);
}
static inline void from_mont(const Field* F, u64 r[4], const u64 a[4]) {
  u64 one[4] = {1, 0, 0, 0};
  f_mul(F, r, a, one);
}

/* ------------------------------------------------------------ Jacobian ops */
typedef struct { u64 x[4], y[4], z[4]; } Jac; /* z == 0: identity */

static inline void j_set_aff(const Field* F, Jac* r, const u64* aff) {
  if (f_is_zero(aff) && f_is_zero(aff + 4)) {
    memset(r, 0, sizeof(*r));
    memcpy(r->x, F->one, 32);
    memcpy(r->y, F->one, 32);
    return;
  }
  memcpy(r->x, aff, 32);
  memcpy(r->y, aff + 4, 32);
  memcpy(r->z, F->one, 32);
}

/* dbl-2009-l (a = 0) */
static inline void j_dbl(const Field* F, Jac* r, const Jac* p) {
  if (f_is_zero(p->z) || f_is_zero(p->y)) {
    memset(r->z, 0, 32);
    return;
  }
  u64 A[4], B[4], C[4], D[4], E[4], Fv[4], t[4], X3[4], Y3[4], Z3[4];
  f_mul(F, A, p->x, p->x);
  f_mul(F, B, p->y, p->y);
  f_mul(F, C, B, B);
  f_add(F, t, p->x, B);
  f_mul(F, t, t, t);
  f_sub(F, t, t, A);
  f_sub(F, t, t, C);
  f_add(F, D, t, t);
  f_add(F, E, A, A);
  f_add(F, E, E, A);
  f_mul(F, Fv, E, E);
  f_add(F, t, D, D);
  f_sub(F, X3, Fv, t);
  f_sub(F, t, D, X3);
  f_mul(F, t, E, t);
  u64 c8[4];
  f_add(F, c8, C, C);
  f_add(F, c8, c8, c8);
  f_add(F, c8, c8, c8);
  f_sub(F, Y3, t, c8);
  f_mul(F, Z3, p->y, p->z);
  f_add(F, Z3, Z3, Z3);
  memcpy(r->x, X3, 32);
  memcpy(r->y, Y3, 32);
  memcpy(r->z, Z3, 32);
}

/* add-2007-bl */
static inline void j_add(const Field* F, Jac* r, const Jac* p, const Jac* q) {
  if (f_is_zero(p->z)) { *r = *q; return; }
  if (f_is_zero(q->z)) { *r = *p; return; }
  u64 Z1Z1[4], Z2Z2[4], U1[4], U2[4], S1[4], S2[4], H[4], I[4], J[4], rr[4], V[4], t[4];
  f_mul(F, Z1Z1, p->z, p->z);
  f_mul(F, Z2Z2, q->z, q->z);
  f_mul(F, U1, p->x, Z2Z2);
  f_mul(F, U2, q->x, Z1Z1);
  f_mul(F, t, q->z, Z2Z2);
  f_mul(F, S1, p->y, t);
  f_mul(F, t, p->z, Z1Z1);
  f_mul(F, S2, q->y, t);
  if (memcmp(U1, U2, 32) == 0) {
    if (memcmp(S1, S2, 32) == 0) { j_dbl(F, r, p); return; }
    memset(r->z, 0, 32);
    return;
  }
  f_sub(F, H, U2, U1);
  f_add(F, I, H, H);
  f_mul(F, I, I, I);
  f_mul(F, J, H, I);
  f_sub(F, rr, S2, S1);
  f_add(F, rr, rr, rr);
  f_mul(F, V, U1, I);
  u64 X3[4], Y3[4], Z3[4];
  f_mul(F, X3, rr, rr);
  f_sub(F, X3, X3, J);
  f_sub(F, X3, X3, V);
  f_sub(F, X3, X3, V);
  f_sub(F, t, V, X3);
  f_mul(F, Y3, rr, t);
  f_mul(F, t, S1, J);
  f_add(F, t, t, t);
  f_sub(F, Y3, Y3, t);
  f_add(F, Z3, p->z, q->z);
  f_mul(F, Z3, Z3, Z3);
  f_sub(F, Z3, Z3, Z1Z1);
  f_sub(F, Z3, Z3, Z2Z2);
  f_mul(F, Z3, Z3, H);
  memcpy(r->x, X3, 32);
  memcpy(r->y, Y3, 32);
  memcpy(r->z, Z3, 32);
}

/* madd-2007-bl: p + affine q (q not identity) */
static inline void j_add_aff(const Field* F, Jac* r, const Jac* p, const u64* q) {
  if (f_is_zero(q) && f_is_zero(q + 4)) { *r = *p; return; }
  if (f_is_zero(p->z)) { j_set_aff(F, r, q); return; }
  u64 Z1Z1[4], U2[4], S2[4], H[4], HH[4], I[4], J[4], rr[4], V[4], t[4];
  f_mul(F, Z1Z1, p->z, p->z);
  f_mul(F, U2, q, Z1Z1);
  f_mul(F, t, p->z, Z1Z1);
  f_mul(F, S2, q + 4, t);
  if (memcmp(U2, p->x, 32) == 0) {
    if (memcmp(S2, p->y, 32) == 0) { j_dbl(F, r, p); return; }
    memset(r->z, 0, 32);
    return;
  }
  f_sub(F, H, U2, p->x);
  f_mul(F, HH, H, H);
  f_add(F, I, HH, HH);
  f_add(F, I, I, I);
  f_mul(F, J, H, I);
  f_sub(F, rr, S2, p->y);
  f_add(F, rr, rr, rr);
  f_mul(F, V, p->x, I);
  u64 X3[4], Y3[4], Z3[4];
  f_mul(F, X3, rr, rr);
  f_sub(F, X3, X3, J);
  f_sub(F, X3, X3, V);
  f_sub(F, X3, X3, V);
  f_sub(F, t, V, X3);
  f_mul(F, Y3, rr, t);
  f_mul(F, t, p->y, J);
  f_add(F, t, t, t);
  f_sub(F, Y3, Y3, t);
  f_add(F, Z3, p->z, H);
  f_mul(F, Z3, Z3, Z3);
  f_sub(F, Z3, Z3, Z1Z1);
  f_sub(F, Z3, Z3, HH);
  memcpy(r->x, X3, 32);
  memcpy(r->y, Y3, 32);
  memcpy(r->z, Z3, 32);
}

static inline void j_to_aff(const Field* F, u64* out, const Jac* p) {
  if (f_is_zero(p->z)) { memset(out, 0, 64); return; }
  u64 zi[4], zi2[4], zi3[4];
  f_inv(F, zi, p->z);
  f_mul(F, zi2, zi, zi);
  f_mul(F, zi3, zi2, zi);
  f_mul(F, out, p->x, zi2);
  f_mul(F, out + 4, p->y, zi3);
}

#endif /* EC_REF_H */

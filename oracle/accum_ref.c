/* accum_ref.c -- TEST INFRASTRUCTURE ONLY: C restatement of the multiopen
 * accumulator and of its Blake2b transcript replay.
 *
 * Used as (a) a second checker of the HIP accumulator beside the Python
 * oracle (tests/test_accum_oracle.py runs both on the golden proofs) and (b)
 * bench.py's accumulator cpu_baseline ("kind": "port", all host threads).
 * Never linked by the product library.
 *
 * It restates, per proof (same reference lines as oracle/accum.py and
 * oracle/transcript.py, whose docstrings hold the full mapping):
 *   transcript  TranscriptChip (/root/reference/src/transcript.rs:57-145) as
 *               halo2 Blake2bWrite / Challenge255 [3P], absorb order of
 *               src/verifier.rs:341-719; an identity point is skipped
 *               (transcript.rs:101-110), a skipped lookup Z marks the abort
 *               of lookup.rs:100;
 *   scalars     x^n, l_0 / l_last / l_blind (verifier.rs:512-591), gate
 *               expressions (compute_expr, verifier.rs:58-151, here on the
 *               postfix code of include/pasta_msm.h), permutation
 *               (src/permutation.rs:190-324) and lookup (src/lookup.rs:
 *               173-311, compress over the flattened lists) expressions,
 *               h_eval (src/vanishing.rs:136-175);
 *   queries     verifier.rs:654-715 + permutation.rs:332-358 + lookup.rs:
 *               314-347 + vanishing.rs:206-220, grouped by rotation in
 *               ascending order (multiopen.rs:19-45);
 *   outputs     calc_witness (multiopen.rs:271-509) in closed form: one
 *               coefficient per commitment (u^{S-1-j} v^{m_j-1-i}, H expanded
 *               as sum h_i (x^n)^i), w / zw / f by one Straus MSM each,
 *               e = [-eval_multi] g1.
 * Field and group law: ec_ref.h (4 x u64 Montgomery, Jacobian), independent
 * of the HIP library's radix-2^29 code.
 *
 * PARITY STATUS: parity unpinned by the reference (it holds no vectors for
 * this path, src/lib.rs:43-44); pinned by agreement with oracle/accum.py and
 * oracle/transcript.py on every golden case.
 *
 * Proof bytes (accum_ref_batch_proofs): halo2 Blake2bRead::read_point /
 * read_scalar [3P] as restated in oracle/proof_bytes.py (the reference's
 * reads: src/verifier.rs:370,443,456,469, src/lookup.rs:64-65,96,124-128,
 * src/permutation.rs:67,100-107,163, src/vanishing.rs:67,94,122,
 * src/multiopen.rs:210): point = canonical x with the y parity in bit 255,
 * decompressed by a square root (a^((p+1)/4) for BN254, Tonelli-Shanks for
 * Pasta), scalar = canonical < r; failures set status bits 8 / 16.
 *
 * Build: oracle/Makefile -> oracle/libmsm_ref.so (with msm_ref.c). */
#include "ec_ref.h"

#include "../include/pasta_msm.h" /* pm_proof_shape: the boundary's VK view */

/* ------------------------------------------------------------ BLAKE2b-512
 * RFC 7693, unkeyed, digest 64 bytes, 16-byte personalisation. */
typedef struct {
  u64 h[8];
  u64 t;
  uint8_t buf[128];
  size_t n;
} B2;

static const u64 B2_IV[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                             0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                             0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
static const uint8_t B2_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static inline u64 rotr64(u64 x, int n) { return (x >> n) | (x << (64 - n)); }
static inline u64 ld64(const uint8_t* p) {
  u64 v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

static void b2_compress(B2* s, const uint8_t blk[128], int last) {
  u64 m[16], v[16];
  for (int i = 0; i < 16; i++) m[i] = ld64(blk + 8 * i);
  for (int i = 0; i < 8; i++) {
    v[i] = s->h[i];
    v[i + 8] = B2_IV[i];
  }
  v[12] ^= s->t; /* messages here stay far below 2^64 bytes */
  if (last) v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t* z = B2_SIGMA[r];
#define B2G(a, b, c, d, x, y)          \
  v[a] = v[a] + v[b] + x;              \
  v[d] = rotr64(v[d] ^ v[a], 32);      \
  v[c] = v[c] + v[d];                  \
  v[b] = rotr64(v[b] ^ v[c], 24);      \
  v[a] = v[a] + v[b] + y;              \
  v[d] = rotr64(v[d] ^ v[a], 16);      \
  v[c] = v[c] + v[d];                  \
  v[b] = rotr64(v[b] ^ v[c], 63);
    B2G(0, 4, 8, 12, m[z[0]], m[z[1]]);
    B2G(1, 5, 9, 13, m[z[2]], m[z[3]]);
    B2G(2, 6, 10, 14, m[z[4]], m[z[5]]);
    B2G(3, 7, 11, 15, m[z[6]], m[z[7]]);
    B2G(0, 5, 10, 15, m[z[8]], m[z[9]]);
    B2G(1, 6, 11, 12, m[z[10]], m[z[11]]);
    B2G(2, 7, 8, 13, m[z[12]], m[z[13]]);
    B2G(3, 4, 9, 14, m[z[14]], m[z[15]]);
#undef B2G
  }
  for (int i = 0; i < 8; i++) s->h[i] ^= v[i] ^ v[i + 8];
}

static void b2_init(B2* s, const char personal[16]) {
  uint8_t p[64];
  memset(p, 0, 64);
  p[0] = 64; /* digest length */
  p[2] = 1;  /* fanout */
  p[3] = 1;  /* depth */
  memcpy(p + 48, personal, 16);
  for (int i = 0; i < 8; i++) s->h[i] = B2_IV[i] ^ ld64(p + 8 * i);
  s->t = 0;
  s->n = 0;
}

static void b2_update(B2* s, const uint8_t* d, size_t len) {
  for (size_t i = 0; i < len; i++) {
    if (s->n == 128) { /* a full block is compressed only once more data follows */
      s->t += 128;
      b2_compress(s, s->buf, 0);
      s->n = 0;
    }
    s->buf[s->n++] = d[i];
  }
}

static void b2_final(const B2* s0, uint8_t out[64]) { /* on a copy: the state goes on */
  B2 s = *s0;
  s.t += s.n;
  memset(s.buf + s.n, 0, 128 - s.n);
  b2_compress(&s, s.buf, 1);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 8; k++) out[8 * i + k] = (uint8_t)(s.h[i] >> (8 * k));
}

/* ------------------------------------------------------- field helpers */
static void f_r2r3(const Field* F, u64 r2[4], u64 r3[4]) { /* R^2, R^3 mod p */
  memcpy(r2, F->one, 32);
  for (int i = 0; i < 256; i++) f_add(F, r2, r2, r2);
  f_mul(F, r3, r2, r2);
}
static void f_neg(const Field* F, u64 r[4], const u64 a[4]) {
  u64 z[4] = {0, 0, 0, 0};
  f_sub(F, r, z, a);
}
/* from_bytes_wide: a little-endian 512-bit integer mod p, Montgomery out */
static void f_from_wide(const Field* F, const u64 r2[4], const u64 r3[4], const uint8_t d[64], u64 out[4]) {
  u64 lo[4], hi[4], a[4], b[4];
  for (int i = 0; i < 4; i++) {
    lo[i] = ld64(d + 8 * i);
    hi[i] = ld64(d + 32 + 8 * i);
  }
  f_mul(F, a, lo, r2); /* lo R mod p (lo < 2^256 = R: CIOS stays below 2p) */
  f_mul(F, b, hi, r3); /* hi 2^256 R mod p */
  f_add(F, out, a, b);
}
static void f_pow_u(const Field* F, u64 r[4], const u64 a[4], unsigned e) {
  u64 acc[4], b[4];
  memcpy(acc, F->one, 32);
  memcpy(b, a, 32);
  while (e) {
    if (e & 1) f_mul(F, acc, acc, b);
    f_mul(F, b, b, b);
    e >>= 1;
  }
  memcpy(r, acc, 32);
}
static void put_le(uint8_t* o, const u64 a[4]) {
  for (int i = 0; i < 4; i++)
    for (int k = 0; k < 8; k++) o[8 * i + k] = (uint8_t)(a[i] >> (8 * k));
}

/* ------------------------------------------------------------- layout */
typedef struct {
  uint32_t p_inst, p_adv, p_lkperm, p_permz, p_lkz, p_rand, p_h, p_W, npts;
  uint32_t s_inst, s_adv, s_fixed, s_rand, s_sigma, s_perm, s_lk, nsc;
  uint32_t nps, nsets;
  int rot[64]; /* distinct rotations, ascending */
} Layout;

static int has_rot(const Layout* L, int r) {
  for (uint32_t i = 0; i < L->nsets; i++)
    if (L->rot[i] == r) return 1;
  return 0;
}
static int add_rot(Layout* L, int r) {
  if (has_rot(L, r)) return 0;
  if (L->nsets == 64) return -1;
  uint32_t i = L->nsets++;
  while (i > 0 && L->rot[i - 1] > r) {
    L->rot[i] = L->rot[i - 1];
    i--;
  }
  L->rot[i] = r;
  return 0;
}

static int make_layout(const pm_proof_shape* s, Layout* L) {
  memset(L, 0, sizeof(*L));
  if (!s->perm_chunk_len && s->n_perm_columns) return -1;
  L->nps = s->n_perm_columns ? (s->n_perm_columns + s->perm_chunk_len - 1) / s->perm_chunk_len : 0;
  for (uint32_t i = 0; i < s->n_instance_queries; i++) add_rot(L, s->instance_queries[i].rotation);
  for (uint32_t i = 0; i < s->n_advice_queries; i++) add_rot(L, s->advice_queries[i].rotation);
  for (uint32_t i = 0; i < s->n_fixed_queries; i++) add_rot(L, s->fixed_queries[i].rotation);
  if (L->nps) {
    add_rot(L, 0);
    add_rot(L, 1);
    if (L->nps > 1) add_rot(L, -(int)(s->blinding_factors + 1));
  }
  if (s->num_lookups) {
    add_rot(L, 0);
    add_rot(L, -1);
    add_rot(L, 1);
  }
  add_rot(L, 0); /* vanishing */
  uint32_t k = 0;
  L->p_inst = k; k += s->num_instance_columns;
  L->p_adv = k; k += s->num_advice_columns;
  L->p_lkperm = k; k += 2 * s->num_lookups;
  L->p_permz = k; k += L->nps;
  L->p_lkz = k; k += s->num_lookups;
  L->p_rand = k; k += 1;
  L->p_h = k; k += s->quotient_degree;
  L->p_W = k; k += L->nsets;
  L->npts = k;
  k = 0;
  L->s_inst = k; k += s->n_instance_queries;
  L->s_adv = k; k += s->n_advice_queries;
  L->s_fixed = k; k += s->n_fixed_queries;
  L->s_rand = k; k += 1;
  L->s_sigma = k; k += s->n_perm_columns;
  L->s_perm = k; k += L->nps ? 3 * L->nps - 1 : 0;
  L->s_lk = k; k += 5 * s->num_lookups;
  L->nsc = k;
  return 0;
}

/* ---------------------------------------------------------- transcript */
enum { ST_IDENTITY = 1, ST_LOOKUP_Z = 2, ST_DENOM_ZERO = 4 };

typedef struct {
  B2 b2;
  const Field* F;  /* base field (point coordinates) */
  const Field* Fr; /* scalar field */
  u64 r2[4], r3[4];
  uint32_t status;
} Tr;

static void tr_point(Tr* t, const u64* p, int lookup_z) {
  if (f_is_zero(p) && f_is_zero(p + 4)) { /* common_point: Err(Synthesis) */
    t->status |= ST_IDENTITY | (lookup_z ? ST_LOOKUP_Z : 0);
    return;
  }
  uint8_t rec[65];
  u64 c[4];
  rec[0] = 1;
  from_mont(t->F, c, p);
  put_le(rec + 1, c);
  from_mont(t->F, c, p + 4);
  put_le(rec + 33, c);
  b2_update(&t->b2, rec, 65);
}
static void tr_scalar(Tr* t, const u64* s) {
  uint8_t rec[33];
  u64 c[4];
  rec[0] = 2;
  from_mont(t->Fr, c, s);
  put_le(rec + 1, c);
  b2_update(&t->b2, rec, 33);
}
static void tr_squeeze(Tr* t, u64 out[4]) {
  uint8_t z = 0, d[64];
  b2_update(&t->b2, &z, 1);
  b2_final(&t->b2, d);
  f_from_wide(t->Fr, t->r2, t->r3, d, out);
}

/* verifier.rs:341-719 read order -> theta, beta, gamma, y, x, v, u */
static uint32_t replay(const CurveDef* cv, const pm_proof_shape* s, const Layout* L, const u64* pts,
                       const u64* scs, const u64 vk[4], u64 ch[7][4]) {
  Tr t;
  b2_init(&t.b2, "Halo2-Transcript");
  t.F = &cv->fp;
  t.Fr = &cv->fr;
  f_r2r3(t.Fr, t.r2, t.r3);
  t.status = 0;
  tr_scalar(&t, vk);
  for (uint32_t i = 0; i < s->num_instance_columns; i++) tr_point(&t, pts + 8 * (L->p_inst + i), 0);
  for (uint32_t i = 0; i < s->num_advice_columns; i++) tr_point(&t, pts + 8 * (L->p_adv + i), 0);
  tr_squeeze(&t, ch[0]);
  for (uint32_t i = 0; i < 2 * s->num_lookups; i++) tr_point(&t, pts + 8 * (L->p_lkperm + i), 0);
  tr_squeeze(&t, ch[1]);
  tr_squeeze(&t, ch[2]);
  for (uint32_t i = 0; i < L->nps; i++) tr_point(&t, pts + 8 * (L->p_permz + i), 0);
  for (uint32_t i = 0; i < s->num_lookups; i++) tr_point(&t, pts + 8 * (L->p_lkz + i), 1);
  tr_point(&t, pts + 8 * L->p_rand, 0);
  tr_squeeze(&t, ch[3]);
  for (uint32_t i = 0; i < s->quotient_degree; i++) tr_point(&t, pts + 8 * (L->p_h + i), 0);
  tr_squeeze(&t, ch[4]);
  for (uint32_t i = 0; i < L->nsc; i++) tr_scalar(&t, scs + 4 * i);
  tr_squeeze(&t, ch[5]);
  tr_squeeze(&t, ch[6]);
  return t.status;
}

/* --------------------------------------------------------- expressions */
#define MAX_STACK 64
/* Evaluate postfix code from *pc to the next PM_EXPR_END; *pc moves past it. */
static int eval_code(const Field* Fr, const pm_proof_shape* s, const uint32_t* code, uint32_t len, uint32_t* pc,
                     const u64* adv, const u64* fix, const u64* inst, u64 out[4]) {
  u64 st[MAX_STACK][4];
  int sp = 0;
  while (*pc < len) {
    const uint32_t w = code[(*pc)++], op = w & 0xff, arg = w >> 8;
    switch (op) {
      case PM_EXPR_END:
        if (sp != 1) return -1;
        memcpy(out, st[0], 32);
        return 0;
      case PM_EXPR_CONST:
      case PM_EXPR_FIXED:
      case PM_EXPR_ADVICE:
      case PM_EXPR_INSTANCE: {
        if (sp == MAX_STACK) return -1;
        const u64* src = op == PM_EXPR_CONST ? s->constants : op == PM_EXPR_FIXED ? fix : op == PM_EXPR_ADVICE ? adv : inst;
        memcpy(st[sp++], src + 4 * arg, 32);
        break;
      }
      case PM_EXPR_NEG:
        if (sp < 1) return -1;
        f_neg(Fr, st[sp - 1], st[sp - 1]);
        break;
      case PM_EXPR_SUM:
      case PM_EXPR_PROD:
        if (sp < 2) return -1;
        if (op == PM_EXPR_SUM) f_add(Fr, st[sp - 2], st[sp - 2], st[sp - 1]);
        else f_mul(Fr, st[sp - 2], st[sp - 2], st[sp - 1]);
        sp--;
        break;
      case PM_EXPR_SCALED:
        if (sp < 1) return -1;
        f_mul(Fr, st[sp - 1], st[sp - 1], s->constants + 4 * arg);
        break;
      default:
        return -1;
    }
  }
  return -1;
}

/* lookup.rs:214-243: Horner in theta from zero over every expression of code */
static int compress(const Field* Fr, const pm_proof_shape* s, const uint32_t* code, uint32_t len, const u64 theta[4],
                    const u64* adv, const u64* fix, const u64* inst, u64 out[4]) {
  u64 acc[4] = {0, 0, 0, 0}, e[4];
  uint32_t pc = 0;
  while (pc < len) {
    if (eval_code(Fr, s, code, len, &pc, adv, fix, inst, e)) return -1;
    f_mul(Fr, acc, acc, theta);
    f_add(Fr, acc, acc, e);
  }
  memcpy(out, acc, 32);
  return 0;
}

/* ---------------------------------------------------------------- MSM */
/* sum_i k_i P_i (affine Montgomery in, identity (0,0)) by Straus with 4-bit
 * windows over the canonical scalars; result affine Montgomery. */
static void msm_straus(const CurveDef* cv, int n, const u64 (*k)[4], const u64* const* P, u64 out[8]) {
  const Field* F = &cv->fp;
  Jac (*tab)[16] = malloc(sizeof(Jac[16]) * (size_t)(n ? n : 1));
  u64 (*kc)[4] = malloc(32 * (size_t)(n ? n : 1));
  for (int i = 0; i < n; i++) {
    from_mont(&cv->fr, kc[i], k[i]);
    memset(&tab[i][0], 0, sizeof(Jac));
    j_set_aff(F, &tab[i][1], P[i]);
    for (int d = 2; d < 16; d++) j_add(F, &tab[i][d], &tab[i][d - 1], &tab[i][1]);
  }
  Jac acc;
  memset(&acc, 0, sizeof(acc));
  for (int win = 63; win >= 0; win--) {
    for (int b = 0; b < 4; b++) j_dbl(F, &acc, &acc);
    for (int i = 0; i < n; i++) {
      const unsigned d = (unsigned)(kc[i][win / 16] >> (4 * (win % 16))) & 15u;
      if (d) j_add(F, &acc, &acc, &tab[i][d]);
    }
  }
  j_to_aff(F, out, &acc);
  free(tab);
  free(kc);
}

/* ------------------------------------------------------------ one proof */
typedef struct { /* a query: commitment ref, rotation, eval */
  int ref;       /* [0, npts): proof point; npts + c: fixed c; npts + nf + k: sigma k; REF_H */
  int rot;
  u64 ev[4];
} Query;
#define REF_H (-1)

static uint32_t accum_one(const CurveDef* cv, const pm_proof_shape* s, const Layout* L, const u64* pts,
                          const u64* scs, u64 ch[7][4], u64 quad[32], u64 hout[4]) {
  const Field* Fr = &cv->fr;
  const u64 *theta = ch[0], *beta = ch[1], *gamma = ch[2], *y = ch[3], *x = ch[4], *v = ch[5], *u = ch[6];
  const u64 *inst = scs + 4 * L->s_inst, *adv = scs + 4 * L->s_adv, *fix = scs + 4 * L->s_fixed;
  const u64 *sig = scs + 4 * L->s_sigma, *perm = scs + 4 * L->s_perm, *lk = scs + 4 * L->s_lk;
  const u64* rand_ev = scs + 4 * L->s_rand;
  u64 one[4], t[4], t2[4];
  memcpy(one, Fr->one, 32);
  uint32_t status = 0;
  /* x^n (verifier.rs:513-516) */
  u64 xn[4];
  memcpy(xn, x, 32);
  for (uint32_t i = 0; i < s->log_n; i++) f_mul(Fr, xn, xn, xn);
  u64 xn1[4];
  f_sub(Fr, xn1, xn, one);
  /* l_i = w^i (x^n - 1) / (n (x - w^i)), w = omega^-1, i < bf + 2
   * (verifier.rs:553-591), and 1 / (x^n - 1), by one batch inversion */
  const uint32_t K = s->blinding_factors + 3;
  u64(*den)[4] = malloc(32 * K), (*pre)[4] = malloc(32 * K), (*wp)[4] = malloc(32 * K);
  u64 winv[4], nfe[4];
  f_inv(Fr, winv, s->omega);
  { /* n as a field element: 2^log_n */
    memcpy(nfe, one, 32);
    for (uint32_t i = 0; i < s->log_n; i++) f_add(Fr, nfe, nfe, nfe);
  }
  memcpy(wp[0], one, 32);
  for (uint32_t i = 1; i + 1 < K; i++) f_mul(Fr, wp[i], wp[i - 1], winv);
  for (uint32_t i = 0; i < K; i++) {
    if (i + 1 < K) {
      f_sub(Fr, t, x, wp[i]);
      f_mul(Fr, den[i], nfe, t);
    } else {
      memcpy(den[i], xn1, 32);
    }
    if (i) f_mul(Fr, pre[i], pre[i - 1], den[i]);
    else memcpy(pre[i], den[i], 32);
  }
  if (f_is_zero(pre[K - 1])) status |= ST_DENOM_ZERO; /* main_gate.div fails */
  u64 inv[4];
  f_inv(Fr, inv, pre[K - 1]);
  for (uint32_t i = K - 1; i > 0; i--) {
    f_mul(Fr, t, inv, pre[i - 1]);
    f_mul(Fr, inv, inv, den[i]);
    memcpy(den[i], t, 32); /* 1 / den_i */
  }
  memcpy(den[0], inv, 32);
  u64 l0[4], llast[4], lblind[4] = {0, 0, 0, 0};
  for (uint32_t i = 0; i + 1 < K; i++) {
    u64 li[4];
    f_mul(Fr, t, wp[i], xn1);
    f_mul(Fr, li, t, den[i]);
    if (i == 0) memcpy(l0, li, 32);
    else if (i == s->blinding_factors + 1) memcpy(llast, li, 32);
    else f_add(Fr, lblind, lblind, li);
  }
  u64 inv_xn1[4];
  memcpy(inv_xn1, den[K - 1], 32);
  free(den);
  free(pre);
  free(wp);
  u64 omb[4]; /* 1 - (l_last + l_blind) */
  f_add(Fr, t, llast, lblind);
  f_sub(Fr, omb, one, t);

  /* expressions in order: gates, permutation, lookups (verifier.rs:593-643);
   * vanishing Horner in y on the fly (vanishing.rs:148-155) */
  u64 h[4] = {0, 0, 0, 0};
  int nexpr = 0;
#define PUSH(e)                       \
  do {                                \
    if (nexpr++) f_mul(Fr, h, h, y);  \
    f_add(Fr, h, h, (e));             \
  } while (0)
  {
    uint32_t pc = 0;
    while (pc < s->gate_code_len) {
      u64 e[4];
      if (eval_code(Fr, s, s->gate_code, s->gate_code_len, &pc, adv, fix, inst, e)) return 0xffffffffu;
      PUSH(e);
    }
  }
  const uint32_t nps = L->nps;
  if (nps) { /* permutation.rs:190-324 */
    u64 e[4];
#define ZP(i) (perm + 4 * (3 * (i)))
#define ZPN(i) (perm + 4 * (3 * (i) + 1))
#define ZPL(i) (perm + 4 * (3 * (i) + 2))
    f_sub(Fr, t, one, ZP(0));
    f_mul(Fr, e, l0, t);
    PUSH(e);
    f_mul(Fr, t, ZP(nps - 1), ZP(nps - 1));
    f_sub(Fr, t, t, ZP(nps - 1));
    f_mul(Fr, e, llast, t);
    PUSH(e);
    for (uint32_t i = 1; i < nps; i++) {
      f_sub(Fr, t, ZP(i), ZPL(i - 1));
      f_mul(Fr, e, l0, t);
      PUSH(e);
    }
    u64 delta_k[4], bx[4];
    memcpy(delta_k, one, 32);
    f_mul(Fr, bx, beta, x);
    const uint32_t cl = s->perm_chunk_len;
    for (uint32_t ci = 0; ci < nps; ci++) {
      u64 left[4], right[4];
      memcpy(left, ZPN(ci), 32);
      memcpy(right, ZP(ci), 32);
      for (uint32_t k = ci * cl; k < (ci + 1) * cl && k < s->n_perm_columns; k++) {
        const pm_perm_column pc = s->perm_columns[k];
        const u64* src = pc.kind == PM_COL_ADVICE ? adv : pc.kind == PM_COL_FIXED ? fix : inst;
        const u64* val = src + 4 * pc.query_index;
        f_mul(Fr, t, beta, sig + 4 * k); /* beta sigma + p + gamma */
        f_add(Fr, t, t, val);
        f_add(Fr, t, t, gamma);
        f_mul(Fr, left, left, t);
        f_mul(Fr, t, bx, delta_k); /* beta delta^k x + p + gamma */
        f_add(Fr, t, t, val);
        f_add(Fr, t, t, gamma);
        f_mul(Fr, right, right, t);
        f_mul(Fr, delta_k, delta_k, s->delta);
      }
      f_sub(Fr, t, left, right);
      f_mul(Fr, e, t, omb);
      PUSH(e);
    }
  }
  for (uint32_t li = 0; li < s->num_lookups; li++) { /* lookup.rs:173-311 */
    const u64 *z = lk + 4 * (5 * li), *zw = z + 4, *a = z + 8, *ap = z + 12, *sv = z + 16;
    u64 e[4], cin[4], ctab[4];
    f_sub(Fr, t, one, z);
    f_mul(Fr, e, l0, t);
    PUSH(e);
    f_mul(Fr, t, z, z);
    f_sub(Fr, t, t, z);
    f_mul(Fr, e, llast, t);
    PUSH(e);
    if (compress(Fr, s, s->lookup_input_code, s->lookup_input_code_len, theta, adv, fix, inst, cin) ||
        compress(Fr, s, s->lookup_table_code, s->lookup_table_code_len, theta, adv, fix, inst, ctab))
      return 0xffffffffu;
    u64 left[4], right[4];
    f_add(Fr, t, a, beta);
    f_add(Fr, t2, sv, gamma);
    f_mul(Fr, left, t, t2);
    f_mul(Fr, left, left, zw);
    f_add(Fr, t, cin, beta);
    f_add(Fr, t2, ctab, gamma);
    f_mul(Fr, right, t, t2);
    f_mul(Fr, right, right, z);
    f_sub(Fr, t, left, right);
    f_mul(Fr, e, omb, t);
    PUSH(e);
    u64 aps[4];
    f_sub(Fr, aps, a, sv);
    f_mul(Fr, e, l0, aps);
    PUSH(e);
    f_sub(Fr, t, a, ap);
    f_mul(Fr, t, aps, t);
    f_mul(Fr, e, omb, t);
    PUSH(e);
  }
#undef PUSH
  u64 h_eval[4];
  f_mul(Fr, h_eval, h, inv_xn1); /* vanishing.rs:175 */
  memcpy(hout, h_eval, 32);

  /* queries in reference order */
  const int npts = (int)L->npts, nf = (int)s->num_fixed_columns;
  const int nq_max = (int)(s->n_instance_queries + s->n_advice_queries + 3 * nps + 5 * s->num_lookups +
                           s->n_fixed_queries + s->n_perm_columns + 2);
  Query* q = malloc(sizeof(Query) * (size_t)nq_max);
  int nq = 0;
#define Q(r_, rot_, ev_)          \
  do {                            \
    q[nq].ref = (r_);             \
    q[nq].rot = (rot_);           \
    memcpy(q[nq].ev, (ev_), 32);  \
    nq++;                         \
  } while (0)
  for (uint32_t i = 0; i < s->n_instance_queries; i++)
    Q((int)(L->p_inst + s->instance_queries[i].column), s->instance_queries[i].rotation, inst + 4 * i);
  for (uint32_t i = 0; i < s->n_advice_queries; i++)
    Q((int)(L->p_adv + s->advice_queries[i].column), s->advice_queries[i].rotation, adv + 4 * i);
  for (uint32_t i = 0; i < nps; i++) {
    Q((int)(L->p_permz + i), 0, ZP(i));
    Q((int)(L->p_permz + i), 1, ZPN(i));
  }
  for (int i = (int)nps - 2; i >= 0; i--) Q((int)(L->p_permz + i), -(int)(s->blinding_factors + 1), ZPL(i));
  for (uint32_t i = 0; i < s->num_lookups; i++) {
    const u64* z = lk + 4 * (5 * i);
    const int zr = (int)(L->p_lkz + i), ar = (int)(L->p_lkperm + 2 * i), sr = ar + 1;
    Q(zr, 0, z);
    Q(ar, 0, z + 8);
    Q(sr, 0, z + 16);
    Q(ar, -1, z + 12);
    Q(zr, 1, z + 4);
  }
  for (uint32_t i = 0; i < s->n_fixed_queries; i++)
    Q(npts + (int)s->fixed_queries[i].column, s->fixed_queries[i].rotation, fix + 4 * i);
  for (uint32_t k = 0; k < s->n_perm_columns; k++) Q(npts + nf + (int)k, 0, sig + 4 * k);
  Q(REF_H, 0, h_eval);
  Q((int)L->p_rand, 0, rand_ev);
#undef Q
#undef ZP
#undef ZPN
#undef ZPL

  /* closed-form coefficients over the rotation sets, ascending
   * (multiopen.rs:19-45, 271-509) */
  const int nref = npts + nf + (int)s->n_perm_columns;
  u64(*coef)[4] = calloc((size_t)nref + 1, 32); /* last slot: H */
  u64 ev[4] = {0, 0, 0, 0};
  const int S = (int)L->nsets;
  u64(*wco)[4] = malloc(32 * (size_t)S), (*zco)[4] = malloc(32 * (size_t)S);
  for (int j = 0; j < S; j++) {
    const int rot = L->rot[j];
    u64 uj[4];
    f_pow_u(Fr, uj, u, (unsigned)(S - 1 - j));
    int m = 0;
    for (int k = 0; k < nq; k++) m += q[k].rot == rot;
    int i = 0;
    for (int k = 0; k < nq; k++) {
      if (q[k].rot != rot) continue;
      u64 c[4];
      f_pow_u(Fr, t, v, (unsigned)(m - 1 - i));
      f_mul(Fr, c, uj, t);
      f_mul(Fr, t, c, q[k].ev);
      f_add(Fr, ev, ev, t);
      u64* slot = q[k].ref == REF_H ? coef[nref] : coef[q[k].ref];
      f_add(Fr, slot, slot, c);
      i++;
    }
    memcpy(wco[j], uj, 32);
    u64 wr[4];
    if (rot >= 0) f_pow_u(Fr, wr, s->omega, (unsigned)rot);
    else f_pow_u(Fr, wr, winv, (unsigned)(-rot));
    f_mul(Fr, t, wr, x);
    f_mul(Fr, zco[j], uj, t);
  }
  free(q);
  /* f: every referenced commitment, H expanded as sum h_i (x^n)^i */
  const int nterm = nref + (int)s->quotient_degree;
  u64(*tk)[4] = malloc(32 * (size_t)nterm);
  const u64** tp = malloc(sizeof(u64*) * (size_t)nterm);
  int nt = 0;
  for (int r = 0; r < nref; r++) {
    if (f_is_zero(coef[r])) continue;
    memcpy(tk[nt], coef[r], 32);
    tp[nt++] = r < npts ? pts + 8 * r : r < npts + nf ? s->fixed_commitments + 8 * (r - npts)
                                                     : s->sigma_commitments + 8 * (r - npts - nf);
  }
  {
    u64 xp[4];
    memcpy(xp, one, 32);
    for (uint32_t i = 0; i < s->quotient_degree; i++) {
      f_mul(Fr, tk[nt], coef[nref], xp);
      tp[nt++] = pts + 8 * (L->p_h + i);
      f_mul(Fr, xp, xp, xn);
    }
  }
  msm_straus(cv, nt, (const u64(*)[4])tk, tp, quad + 16);
  const u64** wp2 = malloc(sizeof(u64*) * (size_t)S);
  for (int j = 0; j < S; j++) wp2[j] = pts + 8 * (L->p_W + j);
  msm_straus(cv, S, (const u64(*)[4])wco, wp2, quad);
  msm_straus(cv, S, (const u64(*)[4])zco, wp2, quad + 8);
  f_neg(Fr, t, ev); /* e = [-eval_multi] g1 */
  const u64* g1p = s->g1;
  msm_straus(cv, 1, (const u64(*)[4])&t, &g1p, quad + 24);
  free(coef);
  free(wco);
  free(zco);
  free(tk);
  free(tp);
  free(wp2);
  return status;
}

/* ---------------------------------------------------------------- batch */
typedef struct {
  const CurveDef* cv;
  const pm_proof_shape* s;
  const Layout* L;
  const u64 *points, *scalars, *challenges, *vk;
  u64 *out_ch, *quads, *hev;
  uint32_t* status;
  size_t lo, hi;
  int rc;
} AccJob;

static void* acc_worker(void* arg) {
  AccJob* j = arg;
  for (size_t b = j->lo; b < j->hi; b++) {
    const u64* pts = j->points + (size_t)8 * j->L->npts * b;
    const u64* scs = j->scalars + (size_t)4 * j->L->nsc * b;
    u64 ch[7][4];
    uint32_t st = 0;
    if (j->challenges) memcpy(ch, j->challenges + 28 * b, sizeof(ch));
    else st = replay(j->cv, j->s, j->L, pts, scs, j->vk, ch);
    if (j->out_ch) memcpy(j->out_ch + 28 * b, ch, sizeof(ch));
    u64 h[4];
    const uint32_t a = accum_one(j->cv, j->s, j->L, pts, scs, ch, j->quads + 32 * b, h);
    if (a == 0xffffffffu) {
      j->rc = -1;
      return NULL;
    }
    if (j->hev) memcpy(j->hev + 4 * b, h, 32);
    if (j->status) j->status[b] = st | a;
  }
  return NULL;
}

/* B proofs in the boundary layout of pm_accum_batch / pm_accum_batch_transcript
 * (Montgomery limbs); challenges == NULL: replay the transcript from vk_repr.
 * out_challenges, out_h_eval, out_status may be NULL.  0 on success. */
int accum_ref_batch(int curve, const pm_proof_shape* s, size_t B, const u64* points, const u64* scalars,
                    const u64* challenges, const u64* vk_repr, int num_threads, u64* out_challenges,
                    u64* out_quads, u64* out_h_eval, uint32_t* out_status) {
  if (curve < 0 || curve > 2 || !s || num_threads < 1 || (!challenges && !vk_repr)) return -1;
  Layout L;
  if (make_layout(s, &L)) return -1;
  if (B == 0) return 0;
  if (num_threads > 256) num_threads = 256;
  if ((size_t)num_threads > B) num_threads = (int)B;
  pthread_t th[256];
  AccJob jobs[256];
  const size_t per = (B + num_threads - 1) / num_threads;
  for (int t = 0; t < num_threads; t++) {
    size_t lo = per * t, hi = per * (t + 1);
    if (lo > B) lo = B;
    if (hi > B) hi = B;
    jobs[t] = (AccJob){&CURVES[curve], s, &L, points, scalars, challenges, vk_repr, out_challenges, out_quads,
                       out_h_eval, out_status, lo, hi, 0};
    pthread_create(&th[t], NULL, acc_worker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < num_threads; t++) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  return rc;
}

/* ------------------------------------------------------- proof bytes */
enum { ST_BAD_POINT = 8, ST_BAD_SCALAR = 16 };

static void f_pow_words(const Field* F, u64 r[4], const u64 a[4], const u64 e[4]) {
  u64 acc[4];
  memcpy(acc, F->one, 32);
  for (int i = 3; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      f_mul(F, acc, acc, acc);
      if ((e[i] >> b) & 1) f_mul(F, acc, acc, a);
    }
  memcpy(r, acc, 32);
}
static int f_eq(const u64 a[4], const u64 b[4]) { return !memcmp(a, b, 32); }
static void shr1(u64 a[4]) {
  for (int i = 0; i < 4; i++) a[i] = (a[i] >> 1) | (i < 3 ? a[i + 1] << 63 : 0);
}
/* per-curve constants of the decoder, computed once per batch */
typedef struct {
  u64 r2p[4], r2r[4]; /* R^2 mod p, mod r: canonical -> Montgomery */
  u64 bm[4];          /* b, Montgomery */
  u64 t[4], th[4];    /* p - 1 = 2^s t; (t - 1) / 2 */
  u64 c[4];           /* z^t for the first non-residue z */
  int s;
} DecCtx;
static void dec_init(const CurveDef* cv, DecCtx* d) {
  const Field* F = &cv->fp;
  u64 r3[4], one[4] = {1, 0, 0, 0}, half[4], mone[4], zc[4] = {2, 0, 0, 0}, z[4], e[4];
  f_r2r3(F, d->r2p, r3);
  f_r2r3(&cv->fr, d->r2r, r3);
  u64 bc[4] = {(u64)cv->b, 0, 0, 0};
  f_mul(F, d->bm, bc, d->r2p);
  sub4(d->t, F->p, one);
  memcpy(half, d->t, 32);
  shr1(half);
  d->s = 0;
  while (!(d->t[0] & 1)) {
    shr1(d->t);
    d->s++;
  }
  memcpy(d->th, d->t, 32); /* t odd: (t - 1) / 2 = t >> 1 */
  shr1(d->th);
  memset(mone, 0, 32);
  f_sub(F, mone, mone, F->one);
  for (;; zc[0]++) {
    f_mul(F, z, zc, d->r2p);
    f_pow_words(F, e, z, half);
    if (f_eq(e, mone)) break;
  }
  f_pow_words(F, d->c, z, d->t);
}
/* y with y^2 = a (Montgomery); 0 if a is a non-residue.  Tonelli-Shanks
 * (for BN254 Fq, s = 1: y = a^((t+1)/2) = a^((p+1)/4)). */
static int f_sqrt(const Field* F, const DecCtx* d, u64 y[4], const u64 a[4]) {
  if (f_is_zero(a)) {
    memset(y, 0, 32);
    return 1;
  }
  u64 c[4], w[4], x[4], b[4];
  memcpy(c, d->c, 32);
  f_pow_words(F, w, a, d->th); /* a^((t-1)/2) */
  f_mul(F, x, w, a);           /* a^((t+1)/2) */
  f_mul(F, b, x, w);           /* a^t */
  int m = d->s;
  while (!f_eq(b, F->one)) {
    int i = 0;
    u64 bb[4];
    memcpy(bb, b, 32);
    while (!f_eq(bb, F->one)) {
      f_mul(F, bb, bb, bb);
      if (++i == m) return 0; /* b of order 2^m: a non-residue */
    }
    u64 g[4];
    memcpy(g, c, 32);
    for (int k = 0; k < m - i - 1; k++) f_mul(F, g, g, g);
    m = i;
    f_mul(F, c, g, g);
    f_mul(F, x, x, g);
    f_mul(F, b, b, c);
  }
  memcpy(y, x, 32);
  return 1;
}
static void ld_words(u64 w[4], const uint8_t* p) {
  for (int i = 0; i < 4; i++) w[i] = ld64(p + 8 * i);
}
/* read_point: 1 ok (aff Montgomery), 0 failed (identity written) */
static int read_point(const CurveDef* cv, const DecCtx* d, const uint8_t* enc, u64* aff) {
  const Field* F = &cv->fp;
  u64 x[4];
  ld_words(x, enc);
  const int ysign = (int)(x[3] >> 63);
  x[3] &= 0x7fffffffffffffffull;
  memset(aff, 0, 64);
  if (geq(x, F->p)) return 0;
  if (f_is_zero(x) && !ysign) return 0; /* the identity: common_point fails */
  u64 xm[4], rhs[4], y[4], yc[4];
  f_mul(F, xm, x, d->r2p);
  f_mul(F, rhs, xm, xm);
  f_mul(F, rhs, rhs, xm);
  f_add(F, rhs, rhs, d->bm);
  if (!f_sqrt(F, d, y, rhs)) return 0;
  from_mont(F, yc, y);
  if ((int)(yc[0] & 1) != ysign) {
    u64 zz[4] = {0, 0, 0, 0};
    f_sub(F, y, zz, y);
  }
  memcpy(aff, xm, 32);
  memcpy(aff + 4, y, 32);
  return 1;
}
static int read_scalar(const Field* Fr, const DecCtx* d, const uint8_t* enc, u64* out) {
  u64 v[4];
  ld_words(v, enc);
  if (geq(v, Fr->p)) {
    memset(out, 0, 32);
    return 0;
  }
  f_mul(Fr, out, v, d->r2r);
  return 1;
}
/* one proof's bytes (+ instance points) -> the accumulator layout; status bits */
static uint32_t decode_proof(const CurveDef* cv, const DecCtx* d, const pm_proof_shape* s, const Layout* L,
                             const uint8_t* pf, const u64* inst, u64* pts, u64* scs) {
  uint32_t st = 0;
  const uint32_t ni = s->num_instance_columns;
  memcpy(pts, inst, (size_t)64 * ni);
  size_t off = 0;
  for (uint32_t i = ni; i < L->p_W; i++, off += 32)
    if (!read_point(cv, d, pf + off, pts + 8 * i)) st |= ST_BAD_POINT;
  for (uint32_t k = 0; k < L->nsc; k++, off += 32)
    if (!read_scalar(&cv->fr, d, pf + off, scs + 4 * k)) st |= ST_BAD_SCALAR;
  for (uint32_t j = 0; j < L->nsets; j++, off += 32)
    if (!read_point(cv, d, pf + off, pts + 8 * (L->p_W + j))) st |= ST_BAD_POINT;
  return st;
}

typedef struct {
  const CurveDef* cv;
  const pm_proof_shape* s;
  const Layout* L;
  const DecCtx* dec;
  const uint8_t* proofs;
  size_t stride;
  const u64 *inst, *vk;
  u64 *out_ch, *quads, *hev, *out_pts, *out_scs;
  uint32_t* status;
  size_t lo, hi;
  int rc;
} PfJob;

static void* pf_worker(void* arg) {
  PfJob* j = arg;
  const Layout* L = j->L;
  u64* pts = malloc((size_t)64 * L->npts);
  u64* scs = malloc((size_t)32 * (L->nsc ? L->nsc : 1));
  if (!pts || !scs) {
    j->rc = -1;
    free(pts);
    free(scs);
    return NULL;
  }
  for (size_t b = j->lo; b < j->hi; b++) {
    uint32_t st = decode_proof(j->cv, j->dec, j->s, L, j->proofs + j->stride * b,
                               j->inst + (size_t)8 * j->s->num_instance_columns * b, pts, scs);
    if (j->out_pts) memcpy(j->out_pts + (size_t)8 * L->npts * b, pts, (size_t)64 * L->npts);
    if (j->out_scs) memcpy(j->out_scs + (size_t)4 * L->nsc * b, scs, (size_t)32 * L->nsc);
    if (j->quads) {
      u64 ch[7][4], h[4];
      st |= replay(j->cv, j->s, L, pts, scs, j->vk, ch);
      if (j->out_ch) memcpy(j->out_ch + 28 * b, ch, sizeof(ch));
      const uint32_t a = accum_one(j->cv, j->s, L, pts, scs, ch, j->quads + 32 * b, h);
      if (a == 0xffffffffu) {
        j->rc = -1;
        break;
      }
      st |= a;
      if (j->hev) memcpy(j->hev + 4 * b, h, 32);
    }
    if (j->status) j->status[b] = st;
  }
  free(pts);
  free(scs);
  return NULL;
}

/* B serialized proofs (stride bytes apart) + instance commitments -> decoded
 * layout (out_points / out_scalars may be NULL) and, with vk_repr and
 * out_quads, the replay + accumulator of every proof.  0 on success. */
int accum_ref_batch_proofs(int curve, const pm_proof_shape* s, size_t B, const uint8_t* proofs, size_t stride,
                           const u64* inst, const u64* vk_repr, int num_threads, u64* out_points, u64* out_scalars,
                           u64* out_challenges, u64* out_quads, u64* out_h_eval, uint32_t* out_status) {
  if (curve < 0 || curve > 2 || !s || num_threads < 1 || (out_quads && !vk_repr)) return -1;
  Layout L;
  if (make_layout(s, &L)) return -1;
  if (B == 0) return 0;
  if (num_threads > 256) num_threads = 256;
  if ((size_t)num_threads > B) num_threads = (int)B;
  pthread_t th[256];
  PfJob jobs[256];
  DecCtx dec;
  dec_init(&CURVES[curve], &dec);
  const size_t per = (B + num_threads - 1) / num_threads;
  for (int t = 0; t < num_threads; t++) {
    size_t lo = per * t, hi = per * (t + 1);
    if (lo > B) lo = B;
    if (hi > B) hi = B;
    jobs[t] = (PfJob){&CURVES[curve], s, &L, &dec, proofs, stride, inst, vk_repr, out_challenges, out_quads, out_h_eval,
                      out_points, out_scalars, out_status, lo, hi, 0};
    pthread_create(&th[t], NULL, pf_worker, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < num_threads; t++) {
    pthread_join(th[t], NULL);
    rc |= jobs[t].rc;
  }
  return rc;
}

/* layout query for the Python wrapper: points / scalars per proof, sets */
int accum_ref_layout(const pm_proof_shape* s, uint32_t* npts, uint32_t* nsc, uint32_t* nsets) {
  Layout L;
  if (!s || make_layout(s, &L)) return -1;
  *npts = L.npts;
  *nsc = L.nsc;
  *nsets = L.nsets;
  return 0;
}

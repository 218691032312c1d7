/* msm_ref.c -- TEST INFRASTRUCTURE ONLY: C restatement of halo2 best_multiexp.
 *
 * Used as (a) the large-n checker in tests/ and (b) bench.py's cpu_baseline
 * ("kind": "port").  Never linked by the product library.
 *
 * PARITY STATUS: parity unpinned by the reference -- the reference's MSM lives
 * in the un-vendored halo2 fork `kzg-agg2` (/root/reference/Cargo.toml:12) and
 * pasta_curves, neither present in /root/reference, and the reference ships no
 * test vectors (/root/reference/src/lib.rs:43-44).  This file restates the
 * published algorithms of those crates:
 *   halo2 arithmetic.rs `multiexp_serial`:
 *     c = 1 if n < 4, 3 if n < 32, else ceil(ln n);  segments = 256/c + 1;
 *     for each segment (high to low): c doublings of acc; (2^c - 1) buckets
 *     filled from get_at(segment, c, coeff.to_repr()) with mixed additions
 *     (Bucket::None -> Affine -> Projective); summation by parts: running_sum
 *     over buckets high->low, acc += running_sum after each bucket.
 *   halo2 `best_multiexp`: if n > num_threads, chunk = n / num_threads, one
 *     multiexp_serial per contiguous chunk (chunks(chunk), so possibly one
 *     extra short chunk), results folded left to right; else one serial call.
 *   pasta_curves / pairing_bn256: Montgomery form R = 2^256 in 4 x u64,
 *     Jacobian projective points, affine identity (0, 0).
 * It is an independent implementation from the HIP library (64-bit limbs,
 * Jacobian coordinates, unsigned windows) and from oracle/pasta.py.
 *
 * Build: oracle/Makefile -> oracle/libmsm_ref.so
 */
#include "ec_ref.h"


/* ------------------------------------------------------- multiexp_serial */
static size_t get_at(size_t segment, size_t c, const uint8_t bytes[32]) {
  size_t skip_bits = segment * c, skip_bytes = skip_bits / 8;
  if (skip_bytes >= 32) return 0;
  uint8_t v[8] = {0};
  for (size_t k = 0; k < 8 && skip_bytes + k < 32; k++) v[k] = bytes[skip_bytes + k];
  u64 tmp = 0;
  for (int k = 7; k >= 0; k--) tmp = (tmp << 8) | v[k];
  tmp >>= skip_bits - skip_bytes * 8;
  tmp %= (1ull << c);
  return (size_t)tmp;
}

enum { B_NONE = 0, B_AFF = 1, B_PROJ = 2 };

static void multiexp_serial(const CurveDef* cv, const uint8_t* repr /* n x 32 canonical LE */,
                            const u64* bases, size_t n, Jac* acc) {
  const Field* F = &cv->fp;
  size_t c = n < 4 ? 1 : (n < 32 ? 3 : (size_t)ceil(log((double)n)));
  size_t segments = 256 / c + 1;
  size_t nb = ((size_t)1 << c) - 1;
  int* kind = (int*)malloc(nb * sizeof(int));
  const u64** aff = (const u64**)malloc(nb * sizeof(u64*));
  Jac* proj = (Jac*)malloc(nb * sizeof(Jac));
  for (size_t seg = segments; seg-- > 0;) {
    for (size_t k = 0; k < c; k++) j_dbl(F, acc, acc);
    memset(kind, 0, nb * sizeof(int));
    for (size_t i = 0; i < n; i++) {
      size_t d = get_at(seg, c, repr + 32 * i);
      if (d == 0) continue;
      const u64* b = bases + 8 * i;
      size_t bi = d - 1;
      if (kind[bi] == B_NONE) {
        kind[bi] = B_AFF;
        aff[bi] = b;
      } else if (kind[bi] == B_AFF) {
        Jac t;
        j_set_aff(F, &t, aff[bi]);
        j_add_aff(F, &proj[bi], &t, b);
        kind[bi] = B_PROJ;
      } else {
        j_add_aff(F, &proj[bi], &proj[bi], b);
      }
    }
    Jac running;
    memset(&running, 0, sizeof(running));
    for (size_t bi = nb; bi-- > 0;) {
      if (kind[bi] == B_AFF) j_add_aff(F, &running, &running, aff[bi]);
      else if (kind[bi] == B_PROJ) j_add(F, &running, &running, &proj[bi]);
      j_add(F, acc, acc, &running);
    }
  }
  free(kind);
  free(aff);
  free(proj);
}

/* ---------------------------------------------------------- best_multiexp */
typedef struct {
  const CurveDef* cv;
  const uint8_t* repr;
  const u64* bases;
  size_t n, chunk, nchunks;
  Jac* results;
  volatile size_t next;
  pthread_mutex_t mu;
} Job;

static void* worker(void* arg) {
  Job* job = (Job*)arg;
  for (;;) {
    pthread_mutex_lock(&job->mu);
    size_t k = job->next++;
    pthread_mutex_unlock(&job->mu);
    if (k >= job->nchunks) break;
    size_t lo = k * job->chunk, hi = lo + job->chunk;
    if (hi > job->n) hi = job->n;
    memset(&job->results[k], 0, sizeof(Jac));
    multiexp_serial(job->cv, job->repr + 32 * lo, job->bases + 8 * lo, hi - lo, &job->results[k]);
  }
  return NULL;
}

static void scalars_to_repr(const CurveDef* cv, const u64* scalars, size_t n, int canonical, uint8_t* repr) {
  for (size_t i = 0; i < n; i++) {
    u64 v[4];
    if (canonical) memcpy(v, scalars + 4 * i, 32);
    else from_mont(&cv->fr, v, scalars + 4 * i);
    for (int k = 0; k < 4; k++)
      for (int b = 0; b < 8; b++) repr[32 * i + 8 * k + b] = (uint8_t)(v[k] >> (8 * b));
  }
}

/* Public: halo2 best_multiexp.  scalars Montgomery unless canonical != 0;
 * bases affine Montgomery (0,0)=identity; out affine Montgomery. */
int msm_ref_best_multiexp(int curve, const u64* scalars, const u64* bases, size_t n, int canonical,
                          int num_threads, u64 out[8]) {
  if (curve < 0 || curve > 2 || num_threads < 1) return -1;
  const CurveDef* cv = &CURVES[curve];
  uint8_t* repr = (uint8_t*)malloc(n ? 32 * n : 32);
  scalars_to_repr(cv, scalars, n, canonical, repr);
  Jac acc;
  memset(&acc, 0, sizeof(acc));
  if (n > (size_t)num_threads) {
    Job job;
    job.cv = cv;
    job.repr = repr;
    job.bases = bases;
    job.n = n;
    job.chunk = n / (size_t)num_threads;
    job.nchunks = (n + job.chunk - 1) / job.chunk;
    job.results = (Jac*)calloc(job.nchunks, sizeof(Jac));
    job.next = 0;
    pthread_mutex_init(&job.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * num_threads);
    for (int t = 0; t < num_threads; t++) pthread_create(&th[t], NULL, worker, &job);
    for (int t = 0; t < num_threads; t++) pthread_join(th[t], NULL);
    for (size_t k = 0; k < job.nchunks; k++) j_add(&cv->fp, &acc, &acc, &job.results[k]);
    pthread_mutex_destroy(&job.mu);
    free(th);
    free(job.results);
  } else {
    multiexp_serial(cv, repr, bases, n, &acc);
  }
  j_to_aff(&cv->fp, out, &acc);
  free(repr);
  return 0;
}

/* ------------------------------------------------- synthetic inputs (tests) */
static u64 mix64(u64 x) {
  u64 z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static u64 synth_word(u64 seed, u64 i, u64 j) { return mix64(mix64(seed + i) + j); }

static void synth_scalar(const Field* Fr, int nbits, u64 seed, u64 i, u64 out[4]) {
  for (u64 t = 0;; t++) {
    for (int k = 0; k < 4; k++) out[k] = synth_word(seed, i, 4 * t + k);
    out[3] &= (1ull << (nbits - 192)) - 1ull;
    if (!geq(out, Fr->p)) return;
  }
}

/* canonical -> Montgomery: a * R2 * R^-1 with R2 = R^2 mod p computed as one^2 * ... */
static void to_mont(const Field* F, u64 r[4], const u64 a[4]) {
  /* R2 = (R mod p)^2 * R^-1 * R ... compute R2 by doubling `one` 256 times */
  u64 r2[4];
  memcpy(r2, F->one, 32);
  for (int k = 0; k < 256; k++) f_add(F, r2, r2, r2); /* one * 2^256 = R^2 mod p */
  f_mul(F, r, a, r2);
}

typedef struct {
  const CurveDef* cv;
  u64 seed, i0;
  size_t lo, hi;
  u64* out;
  int kind; /* 0 scalars (Montgomery), 1 bases */
} SynthJob;

static void* synth_worker(void* arg) {
  SynthJob* j = (SynthJob*)arg;
  const CurveDef* cv = j->cv;
  const Field* F = &cv->fp;
  int nbits = (cv == &CURVES[2]) ? 254 : 255;
  for (size_t i = j->lo; i < j->hi; i++) {
    u64 a[4];
    synth_scalar(&cv->fr, nbits, j->seed, j->i0 + i, a);
    if (j->kind == 0) {
      to_mont(&cv->fr, j->out + 4 * i, a);
      continue;
    }
    if (f_is_zero(a)) a[0] = 1;
    u64 g[8];
    memcpy(g + 4, F->one, 32);
    f_add(F, g + 4, g + 4, F->one); /* y = 2 */
    if (cv->gx_neg_one) {
      u64 z[4] = {0, 0, 0, 0};
      f_sub(F, g, z, F->one);       /* x = -1 */
    } else {
      memcpy(g, F->one, 32);        /* x = 1 */
    }
    Jac acc;
    memset(&acc, 0, sizeof(acc));
    for (int k = 3; k >= 0; k--)
      for (int b = 63; b >= 0; b--) {
        j_dbl(F, &acc, &acc);
        if ((a[k] >> b) & 1) j_add_aff(F, &acc, &acc, g);
      }
    j_to_aff(F, j->out + 8 * i, &acc);
  }
  return NULL;
}

static int synth_run(int curve, u64 seed, u64 i0, size_t n, int num_threads, u64* out, int kind) {
  if (curve < 0 || curve > 2 || num_threads < 1) return -1;
  pthread_t th[256];
  SynthJob jobs[256];
  if (num_threads > 256) num_threads = 256;
  size_t per = (n + num_threads - 1) / num_threads;
  for (int t = 0; t < num_threads; t++) {
    size_t lo = per * t, hi = per * (t + 1);
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (SynthJob){&CURVES[curve], seed, i0, lo, hi, out, kind};
    pthread_create(&th[t], NULL, synth_worker, &jobs[t]);
  }
  for (int t = 0; t < num_threads; t++) pthread_join(th[t], NULL);
  return 0;
}

int msm_ref_synth_scalars(int curve, u64 seed, u64 i0, size_t n, int num_threads, u64* out) {
  return synth_run(curve, seed, i0, n, num_threads, out, 0);
}
int msm_ref_synth_bases(int curve, u64 seed, u64 i0, size_t n, int num_threads, u64* out) {
  return synth_run(curve, seed, i0, n, num_threads, out, 1);
}

/* ------------------------------------------------------------------ NTT
 * C restatement of halo2 arithmetic.rs `best_fft` [3P] (checker for pm_fft at
 * sizes the Python oracle cannot reach, and bench.py's NTT cpu_baseline):
 *   serial_fft: bit-reverse swap, radix-2 DIT, w_m = omega^(n/2m), w *= w_m;
 *   best_fft: log_threads = floor(log2 threads); if log_n <= log_threads the
 *     serial form, else parallel_fft: for each thread j a sub-array
 *     tmp_j[i] = sum_s a[(i + s 2^{log_n - log_threads}) mod n] * elt with
 *     elt walking omega_step = omega^(j 2^{log_new_n}) and omega_j = omega^j,
 *     a serial sub-FFT with omega^threads, then a[idx] = tmp[idx & mask]
 *     [idx >> log_threads].
 * Elements are scalar-field values in Montgomery form (4 x u64). */
static void f_pow(const Field* F, u64 r[4], const u64 base[4], u64 e) {
  u64 b[4], acc[4];
  memcpy(b, base, 32);
  memcpy(acc, F->one, 32);
  while (e) {
    if (e & 1) f_mul(F, acc, acc, b);
    f_mul(F, b, b, b);
    e >>= 1;
  }
  memcpy(r, acc, 32);
}

static size_t brev_bits(size_t x, unsigned bits) {
  size_t r = 0;
  for (unsigned i = 0; i < bits; i++) {
    r = (r << 1) | (x & 1);
    x >>= 1;
  }
  return r;
}

static void serial_fft(const Field* F, u64* a, unsigned log_n, const u64 omega[4]) {
  const size_t n = (size_t)1 << log_n;
  for (size_t k = 0; k < n; k++) {
    size_t rk = brev_bits(k, log_n);
    if (k < rk) {
      u64 t[4];
      memcpy(t, a + 4 * k, 32);
      memcpy(a + 4 * k, a + 4 * rk, 32);
      memcpy(a + 4 * rk, t, 32);
    }
  }
  size_t m = 1;
  for (unsigned s = 0; s < log_n; s++) {
    u64 w_m[4];
    f_pow(F, w_m, omega, n / (2 * m));
    for (size_t k = 0; k < n; k += 2 * m) {
      u64 w[4];
      memcpy(w, F->one, 32);
      for (size_t j = 0; j < m; j++) {
        u64 t[4];
        f_mul(F, t, a + 4 * (k + j + m), w);
        f_sub(F, a + 4 * (k + j + m), a + 4 * (k + j), t);
        f_add(F, a + 4 * (k + j), a + 4 * (k + j), t);
        f_mul(F, w, w, w_m);
      }
    }
    m *= 2;
  }
}

typedef struct {
  const Field* F;
  const u64* a;
  u64* tmp;
  unsigned log_n, log_threads;
  size_t j;
  const u64* omega;
} FftJob;

static void* fft_worker(void* arg) {
  FftJob* J = (FftJob*)arg;
  const Field* F = J->F;
  const unsigned log_new_n = J->log_n - J->log_threads;
  const size_t num_threads = (size_t)1 << J->log_threads, new_n = (size_t)1 << log_new_n;
  const size_t mask_n = ((size_t)1 << J->log_n) - 1;
  u64 omega_j[4], omega_step[4], new_omega[4], elt[4];
  f_pow(F, omega_j, J->omega, J->j);
  f_pow(F, omega_step, J->omega, J->j << log_new_n);
  f_pow(F, new_omega, J->omega, num_threads);
  memcpy(elt, F->one, 32);
  for (size_t i = 0; i < new_n; i++) {
    u64 acc[4] = {0, 0, 0, 0};
    for (size_t s = 0; s < num_threads; s++) {
      const size_t idx = (i + (s << log_new_n)) & mask_n;
      u64 t[4];
      f_mul(F, t, J->a + 4 * idx, elt);
      f_add(F, acc, acc, t);
      f_mul(F, elt, elt, omega_step);
    }
    memcpy(J->tmp + 4 * i, acc, 32);
    f_mul(F, elt, elt, omega_j);
  }
  serial_fft(F, J->tmp, log_new_n, new_omega);
  return NULL;
}

int ntt_ref_best_fft(int curve, u64* a, unsigned log_n, const u64 omega[4], int num_threads) {
  if (curve < 0 || curve > 2 || num_threads < 1 || log_n > 30) return -1;
  const Field* F = &CURVES[curve].fr;
  unsigned log_threads = 0;
  while ((2u << log_threads) <= (unsigned)num_threads) log_threads++;
  if (log_n <= log_threads) {
    serial_fft(F, a, log_n, omega);
    return 0;
  }
  const size_t T = (size_t)1 << log_threads, new_n = (size_t)1 << (log_n - log_threads);
  u64* tmp = (u64*)malloc(T * new_n * 32);
  FftJob* jobs = (FftJob*)malloc(T * sizeof(FftJob));
  pthread_t* th = (pthread_t*)malloc(T * sizeof(pthread_t));
  for (size_t j = 0; j < T; j++) {
    jobs[j] = (FftJob){F, a, tmp + 4 * new_n * j, log_n, log_threads, j, omega};
    pthread_create(&th[j], NULL, fft_worker, &jobs[j]);
  }
  for (size_t j = 0; j < T; j++) pthread_join(th[j], NULL);
  const size_t n = (size_t)1 << log_n, mask = T - 1;
  for (size_t idx = 0; idx < n; idx++) memcpy(a + 4 * idx, tmp + 4 * (new_n * (idx & mask) + (idx >> log_threads)), 32);
  free(th);
  free(jobs);
  free(tmp);
  return 0;
}

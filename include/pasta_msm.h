/* pasta_msm.h -- C-ABI of the MI355X-native MSM + multiopen-accumulator library.
 *
 * This is the drop-in boundary for the hot path of
 * Trapdoor-Tech/halo2-aggregation (see INTEGRATION.md for the Rust binding a
 * maintainer adds).  Every entry point is extern "C", takes plain pointers and
 * sizes, and returns 0 (PM_OK) or a negative PM_ERR_* code; the message of the
 * last failure on the calling thread is available from pm_last_error().
 *
 * Memory layout (matches the Rust in-memory representation of pasta_curves /
 * pairing_bn256 types, which the Rust shim passes with `as_ptr()`):
 *   scalar  : 4 x u64 little-endian limbs, Montgomery form (R = 2^256) unless
 *             PM_SCALARS_CANONICAL is set (then the `to_repr()` integer).
 *   affine  : 8 x u64 = x[4] then y[4], Montgomery form; (0,0) is the identity
 *             (the pasta_curves EpAffine/EqAffine convention).
 * Ownership: the caller owns every buffer; the library only borrows pointers
 * for the duration of a call, except the explicit base cache (pm_bases_*).
 * Threading: all calls are synchronous and re-entrant; a pm_ctx serialises its
 * own calls with a mutex, distinct contexts run concurrently.
 */
#ifndef PASTA_MSM_H
#define PASTA_MSM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum pm_curve { PM_CURVE_PALLAS = 0, PM_CURVE_VESTA = 1, PM_CURVE_BN254 = 2 };

enum pm_flags {
  PM_SCALARS_CANONICAL = 1u /* scalars are canonical integers (to_repr), not Montgomery */
};

enum pm_status {
  PM_OK = 0,
  PM_ERR_ARG = -1,         /* bad argument (null pointer, unknown curve, size) */
  PM_ERR_HIP = -2,         /* HIP runtime error (message in pm_last_error) */
  PM_ERR_NODEV = -3,       /* no HIP device / device index out of range */
  PM_ERR_UNSUPPORTED = -4  /* shape or option not supported by this build */
};

/* ABI version: bumped on every change of a signature or of an argument's
 * meaning.  3 = round 3 (pm_ctx_set_stream(ctx, NULL) selects the context's
 * own stream again; the accumulator entries take the trailing out_status
 * argument); 4 = round 4 (proof-byte entries pm_*_proofs*, the drop-in cache
 * admits a base set on its second sighting under a keyed digest).  A binding
 * asserts pm_abi_version() == PM_ABI_VERSION at load. */
#define PM_ABI_VERSION 4

typedef struct pm_ctx pm_ctx;     /* one device + one HIP stream + workspace */
typedef struct pm_bases pm_bases; /* device-resident base points (SRS cache) */

/* ---------------------------------------------------------------- misc */
const char* pm_version(void);
int pm_abi_version(void);
const char* pm_last_error(void);
int pm_device_count(int* count);

/* ------------------------------------------------------------- context */
int pm_ctx_create(int device, pm_ctx** out);
int pm_ctx_destroy(pm_ctx* ctx);
/* Stream ordering contract.  Every entry point is synchronous: it returns
 * after its own work has finished.  Its device work is queued on the
 * context's current stream, so inputs the caller wrote on the device must be
 * ordered before it:
 *   - by default the context runs on its own BLOCKING stream, which is
 *     ordered after everything queued on the legacy null stream (torch's
 *     default stream, the hipMemcpy / hipMemset default);
 *   - pm_ctx_set_stream(ctx, s) runs on the caller's stream s instead
 *     (e.g. torch.cuda.current_stream().cuda_stream); s == NULL goes back to
 *     the context's own stream, s == PM_STREAM_LEGACY selects the legacy
 *     null stream itself;
 *   - pm_ctx_use_own_stream(ctx) also goes back to the context's own stream.
 * Work the caller queues on any other non-blocking stream must be
 * synchronised by the caller before the call. */
#define PM_STREAM_LEGACY ((void*)1) /* the HIP legacy null stream (hipStreamLegacy) */
int pm_ctx_set_stream(pm_ctx* ctx, void* hip_stream);
int pm_ctx_use_own_stream(pm_ctx* ctx);
/* Force the window width c (0 = automatic). */
int pm_ctx_set_window(pm_ctx* ctx, int c);
/* Pipeline tuning: the minimum accumulate slice per lane (0 = automatic).
 * `groups` must be 0 or 1: pipelined window groups measured slower on MI355X
 * and were retired (PM_ERR_UNSUPPORTED for groups > 1). */
int pm_ctx_set_pipeline(pm_ctx* ctx, int groups, int min_chunk);
/* Small-MSM path: MSM calls (pm_msm*, pm_msm_device, pm_msm_resident*) of at
 * most max_n terms under the automatic window run two launches -- a table of
 * [1..8] P_i with the GLV-split 4-bit digits, then per-window sums -- and a
 * 33-window host Horner instead of the sorting pipeline.  Default
 * PM_SMALL_MSM_DEFAULT, 0 disables it, at most PM_SMALL_MSM_LIMIT.  Results do
 * not depend on it. */
#define PM_SMALL_MSM_DEFAULT 16384
#define PM_SMALL_MSM_LIMIT 65536
int pm_ctx_set_small_msm(pm_ctx* ctx, size_t max_n);
/* Retired: the GLV-mode variable-base MSM measured slower on MI355X
 * (DESIGN.md §7).  enable == 0 succeeds, anything else returns
 * PM_ERR_UNSUPPORTED.  Kept so older bindings still link. */
int pm_ctx_set_glv(pm_ctx* ctx, int enable);
/* Batch accumulator: each MSM term's scalar is split into 2^lg_lanes bit
 * segments, one lane each (0..5; 0 = one lane per term; -1 = automatic: more
 * lanes per term while the batch leaves SIMDs idle).  Results do not depend
 * on it. */
int pm_ctx_set_accum_split(pm_ctx* ctx, int lg_lanes);
/* Batch accumulator: how the powers-of-two table chains run (mode 0: a quad
 * of lanes per chain; 1: one wave per chain with row-sliced field elements,
 * shorter steps while the chains fit one wave per SIMD; -1 = automatic: 1 for
 * up to 800 chains, and the proof decoder's square roots row-sliced for up
 * to 4096 points on BN254).  Results do not depend on it. */
int pm_ctx_set_accum_ladder(pm_ctx* ctx, int mode);
/* Batch accumulator schedule options (round 6; they replace the PM_ACC_*
 * environment switches of round 5, so a test can flip them per context).
 * value -1 = automatic (the default) for every option.  Results never depend
 * on them.
 *   PM_ACC_OPT_TWIST           0: no twisted ladder (the powers-table ladder
 *                                 waits for the decoded points); 1 / 2: the
 *                                 twisted ladder whenever the powers tables
 *                                 are built, the decode unfenced beside it
 *                                 (1) or two decode blocks per CU (2)
 *   PM_ACC_OPT_TAIL_STREAM     0: term additions and sums on the main stream
 *   PM_ACC_OPT_TERMS_PER_LANE  1 or 2: the one-lane GLV form's terms per lane
 *   PM_ACC_OPT_TRANSCRIPT      0: per-record transcript replay (no streamed
 *                                 byte layout)
 * PM_ERR_ARG for an unknown option or a value out of range. */
enum {
  PM_ACC_OPT_TWIST = 1,
  PM_ACC_OPT_TAIL_STREAM = 2,
  PM_ACC_OPT_TERMS_PER_LANE = 3,
  PM_ACC_OPT_TRANSCRIPT = 4
};
int pm_ctx_set_accum_option(pm_ctx* ctx, int option, int value);
/* MSM schedule options (round 6); value -1 = automatic (the default).
 * Results never depend on them.
 *   PM_MSM_OPT_SPLIT_COPY   0: one scalar copy.  Automatic: an MSM over a
 *                           resident row table with scalars in host memory
 *                           (pm_msm_resident, the drop-in pm_msm's warm
 *                           calls) of at least PM_SPLIT_COPY_MIN_N points
 *                           copies the scalars in two parts (3/8, 5/8;
 *                           three from 2^21 points) and sorts and
 *                           accumulates each part while the next crosses
 *                           PCIe.
 * PM_ERR_ARG for an unknown option or a value out of range. */
#define PM_SPLIT_COPY_MIN_N 262144
enum { PM_MSM_OPT_SPLIT_COPY = 1 };
int pm_ctx_set_msm_option(pm_ctx* ctx, int option, int value);
/* Per-kernel HIP-event timing on the context stream (for bench/profiling).
 * Every event pair costs ~10 us of stream time on MI355X, so a timed region
 * should restrict events to the kernel it measures:
 * pm_ctx_set_timing_filter(ctx, "accumulate") (NULL or "" = every kernel). */
int pm_ctx_set_timing(pm_ctx* ctx, int enable);
int pm_ctx_set_timing_filter(pm_ctx* ctx, const char* kernel);
int pm_ctx_kernel_stats(pm_ctx* ctx, const char* kernel, uint64_t* launches, double* total_ms);
int pm_ctx_reset_stats(pm_ctx* ctx);

/* ------------------------------------------------------------------ MSM
 * Replaces halo2 `arithmetic::best_multiexp<C>(coeffs: &[C::Scalar],
 * bases: &[C]) -> C::Curve` ([3P] halo2 fork kzg-agg2, /root/reference/
 * Cargo.toml:12), called from Params::commit / commit_lagrange
 * (/root/reference/examples/simple-example.rs:638-640) and inside
 * create_proof / verify_proof (:606,620,702,722).  Result: sum_i s_i * P_i as
 * an affine point (8 limbs, Montgomery, (0,0) = identity); the Rust shim turns
 * it into C::Curve with `to_curve()`.  n == 0 yields the identity. */
int pm_msm(int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
           uint64_t out[8]);
/* Below this many terms the Rust shim would keep halo2's CPU multiexp.  Since
 * the small-MSM path (round 4: ~67 us at one term, ~81 us at 32, ~140 us at
 * 4096) every n >= 1 is faster on the GPU than halo2's multiexp on 16 host
 * threads (~150 us at one term, ~700 us at 32: bench.py small_n, DESIGN.md
 * §12), so the threshold is 1.  pm_msm itself computes any n. */
#define PM_MSM_GPU_MIN_N 1
/* Same, on an explicit context (host pointers).
 * Drop-in base cache: from 4096 points on (and above the small-MSM threshold,
 * PM_SMALL_MSM_DEFAULT by default), pm_msm / pm_msm_ctx keep the base
 * sets they see repeatedly resident on the device (converted, with the row
 * table from 2^18 points, like pm_bases_upload), keyed by (curve, n, a keyed
 * 254-bit digest of the base bytes computed on host threads while the
 * scalars are copied).  A set is admitted on its SECOND sighting (the first
 * call runs the plain pipeline on uploaded bases), so one-shot bases never
 * pay the resident build; a repeated set -- halo2's commits against params.g
 * / params.g_lagrange -- then costs only its scalars' transfer.  Changed
 * bytes (at the same address or not) miss.  The digest is a universal hash
 * (NH + two polynomial layers over GF(2^127 - 1)) under a secret key drawn
 * per context from the OS RNG and never returned: a caller cannot construct
 * two base sets that collide except with probability ~2^-128.  At most 4 sets,
 * min(16 GiB, half the free device memory) per context, least recently used
 * evicted before a new set is built; if the build still runs out of memory
 * every set is released and, failing that, the call runs the plain pipeline.
 * A warm call starts the MSM of the set a cheap keyed hash of its first and
 * last 8 points predicts right behind the scalar copy, while the full digest
 * is still being computed; the result is returned only if the digest then
 * names that same set (else the speculative MSM is drained and the call
 * proceeds as a miss).  n <= the small-MSM threshold bypasses the cache. */
int pm_msm_ctx(pm_ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n,
               uint32_t flags, uint64_t out[8]);
/* Drop-in cache counters of ctx (any pointer may be NULL), and a way to
 * release its sets early. */
int pm_ctx_dropin_stats(pm_ctx* ctx, uint64_t* hits, uint64_t* misses, int* entries, size_t* device_bytes);
int pm_ctx_dropin_clear(pm_ctx* ctx);
/* Speculative starts of pm_msm_ctx: kept (the digest confirmed the predicted
 * set) and drained (it named another set or none). */
int pm_ctx_dropin_spec_stats(pm_ctx* ctx, uint64_t* kept, uint64_t* drained);
/* Out-of-memory events of the drop-in cache: *flushes = builds that failed
 * and released every cached set before their one retry, *failed_builds =
 * sets left unadmitted (that call ran the plain pipeline and succeeded). */
int pm_ctx_dropin_oom_stats(pm_ctx* ctx, uint64_t* flushes, uint64_t* failed_builds);
/* The drop-in cache's small sets (1 <= n <= 512, where the many-MSM path
 * beats the small-MSM path): a set seen twice is kept resident with a multiples table
 * (pm_msm_resident_many's) and later calls with it run as one short MSM of
 * that path; at most 8 sets and 4 GiB per context, LRU; pm_ctx_dropin_clear
 * releases them too.  *hits = calls served from a kept set, *admitted = sets
 * admitted so far, *entries / *device_bytes = what is held now. */
int pm_ctx_dropin_small_stats(pm_ctx* ctx, uint64_t* hits, uint64_t* admitted, int* entries, size_t* device_bytes);
/* A fingerprint of ctx's secret digest key (16 bytes of BLAKE2b of the key,
 * personal "pm-dropin-key-id"): distinct contexts hold distinct keys.  It
 * reveals nothing about the key itself. */
int pm_ctx_dropin_key_id(pm_ctx* ctx, uint64_t out[2]);
/* Same, with scalars and bases already in device memory of ctx's device. */
int pm_msm_device(pm_ctx* ctx, int curve, const void* d_scalars, const void* d_bases, size_t n,
                  uint32_t flags, uint64_t out[8]);
/* Split the points into `ngpu` contiguous slices, one device each (devices
 * 0..ngpu-1), and sum the per-device partial points (the multi-GPU analogue
 * of best_multiexp's per-thread chunks). */
int pm_msm_multi(int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
                 int ngpu, uint64_t out[8]);

/* Device-resident base cache: the SRS bases of halo2 Params (`params.g`,
 * `params.g_lagrange`, replacing the `bases` argument of best_multiexp at
 * examples/simple-example.rs:638-640) are fixed, so a caller uploads them once
 * and runs many MSMs against a window [offset, offset + n) of them.  The
 * library converts them once, at upload, to the pipeline's internal form
 * (64 B per point on the device, no per-call conversion).  From 2^18 points
 * on it also keeps [2^{256 j / rows}] P (rows = 8 up to 2^20 points, 4 up to 2^22, else 2;
 * rows x 64 B per point): an MSM over (at least half of) the set from
 * offset 0 then runs as a row-table MSM (pm_fixed_bases_create_rows) with a
 * rows-times shorter bucket reduction and host tail; other windows run the
 * plain pipeline.  pm_bases_info reports n, the rows and the device bytes.
 * _upload takes host bases (Rust layout, as pm_msm), _upload_device bases
 * already in device memory of ctx's device (copied; the caller keeps its
 * buffer).  pm_msm_resident takes host scalars (one pageable copy),
 * pm_msm_resident_device device scalars. */
int pm_bases_upload(pm_ctx* ctx, int curve, const uint64_t* bases, size_t n, pm_bases** out);
int pm_bases_upload_device(pm_ctx* ctx, int curve, const void* d_bases, size_t n, pm_bases** out);
int pm_bases_info(const pm_bases* b, size_t* n, int* rows, size_t* device_bytes);
int pm_bases_release(pm_bases* b);
int pm_msm_resident(pm_ctx* ctx, const pm_bases* b, size_t offset, const uint64_t* scalars,
                    size_t n, uint32_t flags, uint64_t out[8]);
int pm_msm_resident_device(pm_ctx* ctx, const pm_bases* b, size_t offset, const void* d_scalars,
                           size_t n, uint32_t flags, uint64_t out[8]);
/* k MSMs over the same window of resident bases, one per host scalar array
 * (scalars[j]: n x 4 u64), out: k x 8 u64 -- the prover's commit of many
 * polynomials against params.g / g_lagrange (create_proof,
 * examples/simple-example.rs:606,702).  Pipelined: the H2D copy of MSM j+1's
 * scalars overlaps MSM j's kernels on a second stream, and MSM j-1's host
 * tail overlaps them too.  Same results as k pm_msm_resident calls. */
int pm_msm_resident_batch(pm_ctx* ctx, const pm_bases* b, size_t offset, const uint64_t* const* scalars,
                          size_t k, size_t n, uint32_t flags, uint64_t* out);
/* B independent short MSMs against one resident base set in one launch --
 * the aggregator's per-proof instance commitments
 * params_verifier.commit_lagrange(public_inputs)
 * (examples/simple-example.rs:632-641; verifier.rs:200-225, 312-316 take them
 * as the instance column's commitment), i.e. B calls of
 * best_multiexp(public_inputs_i, g_lagrange[0..n_i]):
 *   out[i] = sum_{t < n[i]} s_i[t] P[offsets[i] + t]   (8 u64 affine each)
 * with s_i the next n[i] scalars of `scalars` (concatenated, n x 4 u64 in
 * the pm_msm scalar form and flags).  offsets == NULL: every MSM starts at
 * base 0 (commit_lagrange).  n[i] == 0 gives the identity (0, 0).
 * The first call that reaches a base beyond the set's multiples table builds
 * it (entry (i, w, m) = [m 2^{c w}] P_i: 2^(c-1) x W(c) x 128 B per base, c = 8
 * for up to 4096 bases, narrower windows for longer prefixes, at most 8 GiB);
 * prefixes beyond that cap run one resident MSM per entry (same results).
 * pm_bases_many_prepare builds the table for [0, max_n) ahead of time;
 * pm_bases_many_info reports its prefix, window and bytes (0 when none).
 * Same results as B pm_msm_resident calls. */
int pm_msm_resident_many(pm_ctx* ctx, const pm_bases* b, size_t B, const size_t* n, const size_t* offsets,
                         const uint64_t* scalars, uint32_t flags, uint64_t* out);
int pm_msm_resident_many_device(pm_ctx* ctx, const pm_bases* b, size_t B, const size_t* n, const size_t* offsets,
                                const void* d_scalars, uint32_t flags, uint64_t* out);
int pm_bases_many_prepare(pm_ctx* ctx, const pm_bases* b, size_t max_n);
int pm_bases_many_info(const pm_bases* b, size_t* n, int* window, size_t* device_bytes);
/* Retired: host inputs are copied with one pageable hipMemcpyAsync, which
 * measured faster on MI355X than pinned staging threads (~52 vs ~38 GB/s for
 * 32 MB).  threads == 0 succeeds, threads > 0 returns PM_ERR_UNSUPPORTED. */
int pm_ctx_set_h2d_threads(pm_ctx* ctx, int threads);

/* Device self-test of the MSM pipeline's radix-2^29 lazy field arithmetic
 * against the 32-bit Montgomery arithmetic (n random + edge operand pairs of
 * the curve's base field); *mismatches = number of failed checks. */
int pm_selftest_field(pm_ctx* ctx, int curve, uint64_t seed, size_t n, uint64_t* mismatches);

/* Host self-test of the MSM's host tail arithmetic (no GPU): n random
 * products and a random Horner chain of doublings / additions of the curve's
 * base field through the BMI2/ADX Montgomery product against the portable
 * one; *mismatches = failed checks.  PM_ERR_UNSUPPORTED when the CPU lacks
 * BMI2/ADX (the tail then runs the portable code). */
int pm_selftest_host(int curve, uint64_t seed, size_t n, uint64_t* mismatches);

/* Affine helpers (host) for combining partial results: out = a + b. */
int pm_point_add(int curve, const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);
/* out = points[0] + ... + points[n-1] (n affine points, 8 limbs each, (0,0) =
 * identity; n == 0 yields the identity): the fold of a sharded MSM's per-rank
 * partials in one call (round 6; one inversion instead of one per addition). */
int pm_points_sum(int curve, const uint64_t* points, size_t n, uint64_t out[8]);

/* Synthetic inputs generated on the device: scalar i is
 * uniform in [0, r) from a SplitMix64 stream keyed by (seed, i0 + i);
 * base i is [a_i]G with a_i drawn the same way.  d_out: n*4 (scalars) or n*8
 * (bases) u64 in device memory.  Scalars are Montgomery unless
 * PM_SCALARS_CANONICAL is set. */
int pm_synth_scalars(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, uint32_t flags,
                     void* d_out);
int pm_synth_bases(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, void* d_out);

/* ------------------------------------------------- multiopen accumulator
 * Boundary 2: the native meaning of the reference's in-circuit
 * verifier for a batch of B inner proofs that share one verifying key.
 * Per proof it evaluates the scalar block of VerifierChip::_verify_proof
 * (/root/reference/src/verifier.rs:512-652: x^n, l_0 / l_last / l_blind,
 * gate, permutation (src/permutation.rs:190-324) and lookup
 * (src/lookup.rs:173-311) expressions, vanishing h_eval
 * (src/vanishing.rs:136-201)), assembles the queries in the reference order
 * (verifier.rs:654-715), groups them by rotation (src/multiopen.rs:19-45) and
 * produces MultiopenChip::calc_witness's accumulator (src/multiopen.rs:271-509)
 *     w  = sum_j u^{S-1-j} W_j          zw = sum_j u^{S-1-j} z_j W_j
 *     f  = sum_j u^{S-1-j} sum_i v^{m_j-1-i} C_{j,i}   (H = sum_i x^{n i} h_i)
 *     e  = [-sum_j u^{S-1-j} sum_i v^{m_j-1-i} e_{j,i}] g1
 * as exact affine points, plus h_eval.  The Rust side replays the transcript
 * and passes the challenges in; the EccChip / Transcript / VerifyingKey
 * surfaces stay unchanged.
 *
 * Expression code (halo2 plonk::Expression, compute_expr verifier.rs:58-151)
 * is postfix, one u32 word per node: op | arg << 8.  Each expression ends with
 * PM_EXPR_END.  Leaves index the query evals (advice/fixed/instance query
 * index) or the shape's constant table (CONST, SCALED). */
enum pm_expr_op {
  PM_EXPR_END = 0,
  PM_EXPR_CONST = 1,    /* push constants[arg] */
  PM_EXPR_FIXED = 2,    /* push fixed_evals[arg] */
  PM_EXPR_ADVICE = 3,   /* push advice_evals[arg] */
  PM_EXPR_INSTANCE = 4, /* push instance_evals[arg] */
  PM_EXPR_NEG = 5,
  PM_EXPR_SUM = 6,
  PM_EXPR_PROD = 7,
  PM_EXPR_SCALED = 8    /* top *= constants[arg] */
};
enum pm_column_kind { PM_COL_ADVICE = 0, PM_COL_FIXED = 1, PM_COL_INSTANCE = 2 };

typedef struct pm_query {
  uint32_t column;
  int32_t rotation;
} pm_query;

typedef struct pm_perm_column {
  uint32_t kind;        /* pm_column_kind */
  uint32_t query_index; /* index into that kind's query evals */
} pm_perm_column;

/* What the accumulator reads from VerifyingKey / ConstraintSystem
 * (verifier.rs:227-285).  Scalars are 4 x u64 Montgomery, points 8 x u64
 * affine Montgomery, (0,0) = identity. */
typedef struct pm_proof_shape {
  uint32_t log_n;
  uint32_t blinding_factors;     /* cs.blinding_factors() */
  uint32_t num_instance_columns;
  uint32_t num_advice_columns;
  uint32_t num_fixed_columns;
  uint32_t num_lookups;
  uint32_t perm_chunk_len;       /* cs.degree() - 2 */
  uint32_t quotient_degree;      /* number of h pieces */
  uint32_t n_instance_queries, n_advice_queries, n_fixed_queries, n_perm_columns;
  const pm_query* instance_queries;
  const pm_query* advice_queries;
  const pm_query* fixed_queries;
  const pm_perm_column* perm_columns;
  const uint32_t* gate_code;         /* all gate polynomials, in gate order */
  uint32_t gate_code_len;
  const uint32_t* lookup_input_code; /* flattened over lookups (verifier.rs:244-251) */
  uint32_t lookup_input_code_len;
  const uint32_t* lookup_table_code;
  uint32_t lookup_table_code_len;
  const uint64_t* constants;         /* n_constants x 4 */
  uint32_t n_constants;
  uint64_t omega[4];                 /* vk.get_domain().get_omega() */
  uint64_t delta[4];                 /* C::ScalarExt::DELTA */
  uint64_t g1[8];                    /* C::generator() */
  const uint64_t* fixed_commitments; /* num_fixed_columns x 8 */
  const uint64_t* sigma_commitments; /* n_perm_columns x 8 */
} pm_proof_shape;

/* Per-proof layout implied by a shape (transcript read order, see
 * oracle/accum.py): points, scalars, and rotation sets S (= number of W_j). */
int pm_shape_layout(const pm_proof_shape* shape, uint32_t* points_per_proof, uint32_t* scalars_per_proof,
                    uint32_t* num_sets);

/* Batch accumulator, host buffers.  points: B x points_per_proof x 8;
 * scalars: B x scalars_per_proof x 4; challenges: B x 7 x 4 (theta, beta,
 * gamma, y, x, v, u); out_quads: B x 4 x 8 (w, zw, f, e); out_h_eval: B x 4
 * (may be NULL).  curve selects the group (PM_CURVE_*); its scalar field is
 * the field of every scalar above. */
int pm_accum_batch(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t* points,
                   const uint64_t* scalars, const uint64_t* challenges, uint64_t* out_quads, uint64_t* out_h_eval,
                   uint32_t* out_status);
/* Same with every buffer in device memory of ctx's device. */
int pm_accum_batch_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const void* d_points,
                          const void* d_scalars, const void* d_challenges, void* d_out_quads, void* d_out_h_eval,
                          void* d_out_status);
/* Per-proof status words (out_status: B x uint32, may be NULL) of every
 * accumulator entry point.  A nonzero word means the reference verifier
 * would not have produced an accumulator for that proof; its quad and h_eval
 * are then unspecified and the caller must reject the proof:
 *   PM_TRANSCRIPT_IDENTITY_SKIPPED (1)  an identity commitment was skipped by
 *       the transcript (transcript.rs:101-110), transcript entries only;
 *   PM_TRANSCRIPT_LOOKUP_Z_IDENTITY (2) that commitment was a lookup product
 *       Z, where the reference propagates the error and aborts (lookup.rs:100);
 *   PM_ACCUM_DENOM_ZERO (4)  x^n = 1 or x = omega^-i for a Lagrange basis
 *       point: the reference's main_gate.div fails (vanishing.rs:175,
 *       verifier.rs:580). */
#define PM_ACCUM_DENOM_ZERO 4u
/* A batch sharded over nctx contexts (one per device) in one process: proofs
 * are independent, context k takes the contiguous range [k*ceil(B/nctx), ...)
 * in its own host thread (the multi-GPU form of VerifierChip::verify_proof
 * over many proofs, src/verifier.rs:227-285).  challenges == NULL replays
 * the Blake2b transcript from vk_repr (as pm_accum_batch_transcript);
 * otherwise the given challenges are used and vk_repr may be NULL.
 * out_challenges, out_h_eval and out_status may be NULL. */
int pm_accum_batch_multi(pm_ctx* const* ctxs, int nctx, int curve, const pm_proof_shape* shape, size_t B,
                         const uint64_t* points, const uint64_t* scalars, const uint64_t* challenges,
                         const uint64_t vk_repr[4], uint64_t* out_challenges, uint64_t* out_quads,
                         uint64_t* out_h_eval, uint32_t* out_status);

/* ---- Fixed-base MSM ----------------------------------------
 * The prover's commitments (Params::commit / commit_lagrange,
 * examples/simple-example.rs:638-640,702) are MSMs against the static SRS
 * bases.  pm_fixed_bases_create precomputes, once per SRS, the table
 * [2^{o_w}] P_i for every window offset o_w (W = ceil(256 / c) windows, c = 0
 * picks the default); every later MSM then sorts all W digits of every scalar
 * into ONE set of 2^(c-1) buckets and skips the per-window bucket reduction
 * and the cross-window doublings.  Table size: W x n x 64 bytes of device
 * memory (2^20 bases, c = 16: 1 GiB).  pm_msm_fixed* use the first n bases
 * (n <= the table's n); results are bit-identical to pm_msm. */
typedef struct pm_fixed_bases pm_fixed_bases;
int pm_fixed_bases_create(pm_ctx* ctx, int curve, const uint64_t* bases, size_t n, int c, pm_fixed_bases** out);
int pm_fixed_bases_create_device(pm_ctx* ctx, int curve, const void* d_bases, size_t n, int c,
                                 pm_fixed_bases** out);
/* A table of `rows` rows (rows divides W, and rows < W needs equal window
 * widths, 256 % W == 0, e.g. c = 16; 0 = W): row j = [2^{o_{jW/rows}}] P_i,
 * so windows w, w + W/rows, ... share one of W/rows bucket sets.  rows = W is
 * the table above; rows = 2 at c = 16 keeps P and [2^128] P (2 x the bases'
 * memory), halves the bucket reduction and the host Horner (128 instead of
 * 256 doublings) of a plain MSM.  bases_on_device: bases is a device pointer. */
int pm_fixed_bases_create_rows(pm_ctx* ctx, int curve, const void* bases, int bases_on_device, size_t n, int c,
                               int rows, pm_fixed_bases** out);
int pm_fixed_bases_info(const pm_fixed_bases* fb, size_t* n, int* c, int* windows, size_t* table_bytes);
int pm_fixed_bases_release(pm_fixed_bases* fb);
int pm_msm_fixed(pm_ctx* ctx, const pm_fixed_bases* fb, const uint64_t* scalars, size_t n, uint32_t flags,
                 uint64_t out[8]);
int pm_msm_fixed_device(pm_ctx* ctx, const pm_fixed_bases* fb, const void* d_scalars, size_t n, uint32_t flags,
                        uint64_t out[8]);

/* ---- NTT over the scalar field -------------------------------
 * halo2 `best_fft(a, omega, log_n)` [3P] (EvaluationDomain::fft / ifft /
 * coset conversions inside create_proof): in place, natural order in and out,
 * a_k <- sum_j a_j omega^{jk} over the scalar field of `curve` (Montgomery
 * 4 x u64 per element, like pm_msm's scalars).  Elements, omega and scale are
 * canonical (< the modulus), as every value of the Rust field types is; the
 * outputs are canonical.  omega must be a primitive
 * 2^log_n-th root of unity.  scale (may be NULL) multiplies every output:
 * EvaluationDomain::ifft is pm_fft(omega_inv, scale = 1/n).  log_n <= 28
 * (create_proof at k = 23 transforms the extended domain, 2^25); above 2^22
 * the transform takes three passes and 2 n x 32 B of context scratch.  The
 * twiddle tables (each sub-transform's root powers and a two-level table of
 * the inter-pass twiddles, ~0.4 MB at 2^25) are cached in the context (4 most
 * recent (curve, log_n, omega)). */
int pm_fft(pm_ctx* ctx, int curve, uint64_t* data, uint32_t log_n, const uint64_t omega[4], const uint64_t* scale);
int pm_fft_device(pm_ctx* ctx, int curve, void* d_data, uint32_t log_n, const uint64_t omega[4],
                  const uint64_t* scale);

/* ---- Blake2b transcript replay ------------------------------
 * The verifier squeezes theta, beta, gamma, y, x, v, u from a halo2
 * Blake2bWrite/Challenge255 transcript (TranscriptChip,
 * /root/reference/src/transcript.rs:57-145) fed in the verifier's read order
 * (src/verifier.rs:341-719).  These entry points replay it for B proofs at
 * once, one GPU lane per proof, from the same points / scalars buffers
 * pm_accum_batch reads (the W_j are not absorbed).
 *
 * vk_repr: the scalar the verifier absorbs first, Montgomery form; it is
 *   pm_vk_transcript_repr() of the pinned-VK debug string (verifier.rs:341-358).
 * out_status (may be NULL): B x uint32; bit 0 = an identity point was
 *   skipped (TranscriptChip::common_point rejects the identity before hashing,
 *   transcript.rs:101-110).  Such a proof's challenges differ from an honest
 *   prover's; the caller should reject it.  Bit 1 = that point was a lookup
 *   product commitment Z (the reference aborts there, lookup.rs:100).  The
 *   fused accumulator entries add PM_ACCUM_DENOM_ZERO (see pm_accum_batch). */
#define PM_TRANSCRIPT_IDENTITY_SKIPPED 1u
#define PM_TRANSCRIPT_LOOKUP_Z_IDENTITY 2u

/* vk_repr = from_bytes_wide(Blake2b-512(personal "Halo2-Verify-Key",
 *   le_u64(len) || pinned[0..len))) in Montgomery form (verifier.rs:341-358).
 *   Host only; needs no device. */
int pm_vk_transcript_repr(int curve, const uint8_t* pinned, size_t len, uint64_t out[4]);
/* out_challenges: B x 7 x 4 (theta, beta, gamma, y, x, v, u), Montgomery. */
int pm_transcript_batch(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4],
                        const uint64_t* points, const uint64_t* scalars, uint64_t* out_challenges,
                        uint32_t* out_status);
int pm_transcript_batch_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                               const uint64_t vk_repr[4], const void* d_points, const void* d_scalars,
                               void* d_out_challenges, void* d_out_status);
/* Transcript replay + accumulator in one call (challenges stay on the
 * device).  out_challenges, out_h_eval and out_status may be NULL. */
int pm_accum_batch_transcript(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                              const uint64_t vk_repr[4], const uint64_t* points, const uint64_t* scalars,
                              uint64_t* out_challenges, uint64_t* out_quads, uint64_t* out_h_eval,
                              uint32_t* out_status);
/* Device-buffer variant; d_challenges is caller-provided B x 7 x 4 scratch
 * (it receives the replayed challenges). */
int pm_accum_batch_transcript_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                                     const uint64_t vk_repr[4], const void* d_points, const void* d_scalars,
                                     void* d_challenges, void* d_out_quads, void* d_out_h_eval,
                                     void* d_out_status);

/* ---- Proof bytes (SURVEY §8b boundary 2, from the serialized proofs) --------
 * The reference verifier reads each inner proof from halo2's byte transcript
 * (Blake2bRead): t.read_point() (src/verifier.rs:370, src/lookup.rs:64-65,96,
 * src/permutation.rs:67, src/vanishing.rs:67,94, src/multiopen.rs:210) and
 * t.read_scalar() (src/verifier.rs:443,456,469, src/vanishing.rs:122,
 * src/permutation.rs:100-107,163, src/lookup.rs:124-128).  These entries take
 * the proofs as those bytes and do the reads on the device, B proofs at once:
 *   point  = 32 bytes: canonical little-endian x, bit 255 = parity of the
 *            canonical y (GroupEncoding::to_bytes of pasta_curves /
 *            pairing_bn256 [3P]); decompressed with a square root;
 *   scalar = 32 bytes: canonical little-endian (PrimeField::to_repr).
 * Byte layout of one proof, pm_proof_size() bytes: the proof points of the
 * accumulator layout after the instance commitments (advice, per lookup A'
 * and S', permutation Z_p, per lookup Z, vanishing r, h_0..h_{d-1}), then every
 * scalar in the accumulator layout, then the multiopen witnesses W_0..W_{S-1}
 * -- the verifier's read order.  Instance commitments do not travel in the
 * proof (verifier.rs:312-316 takes them from the instance column); the caller
 * passes them as affine Montgomery points, B x num_instance_columns x 8 u64.
 * proofs: B proofs, proof i at byte i * stride (stride >= pm_proof_size; the
 * device variants need stride % 4 == 0).
 * Status bits (out_status), where the reference's read fails and it aborts:
 *   PM_PROOF_BAD_POINT (8)   a point encoding is invalid: x not canonical,
 *       x^3 + b a non-residue, or the identity (Blake2bRead's common_point
 *       rejects it);
 *   PM_PROOF_BAD_SCALAR (16) a scalar encoding is >= r.
 * Such a proof's decoded slot holds the identity / zero and its quad is
 * unspecified; the rest of the batch is unaffected. */
#define PM_PROOF_BAD_POINT 8u
#define PM_PROOF_BAD_SCALAR 16u
int pm_proof_size(const pm_proof_shape* shape, size_t* bytes);
/* Decode only: out_points B x points_per_proof x 8 (instance commitments
 * copied in), out_scalars B x scalars_per_proof x 4, out_status B (required):
 * the inputs of pm_accum_batch*. */
int pm_decode_proofs(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint8_t* proofs,
                     size_t stride, const uint64_t* instance_points, uint64_t* out_points, uint64_t* out_scalars,
                     uint32_t* out_status);
int pm_decode_proofs_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const void* d_proofs,
                            size_t stride, const void* d_instance_points, void* d_out_points, void* d_out_scalars,
                            void* d_out_status);
/* Decode + transcript replay + accumulator in one call (pm_accum_batch_transcript
 * on the decoded proofs; the decoded points and scalars stay on the device).
 * out_challenges, out_h_eval and out_status may be NULL; the status words
 * carry the decoder's bits as well as the replay's and PM_ACCUM_DENOM_ZERO. */
int pm_accum_batch_proofs(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4],
                          const uint8_t* proofs, size_t stride, const uint64_t* instance_points,
                          uint64_t* out_challenges, uint64_t* out_quads, uint64_t* out_h_eval, uint32_t* out_status);
/* Device-buffer variant; d_challenges: B x 7 x 4 caller scratch (receives the
 * challenges); d_out_h_eval and d_out_status may be NULL. */
int pm_accum_batch_proofs_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                                 const uint64_t vk_repr[4], const void* d_proofs, size_t stride,
                                 const void* d_instance_points, void* d_challenges, void* d_out_quads,
                                 void* d_out_h_eval, void* d_out_status);

#ifdef __cplusplus
}
#endif
#endif /* PASTA_MSM_H */

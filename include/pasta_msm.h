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

typedef struct pm_ctx pm_ctx;     /* one device + one HIP stream + workspace */
typedef struct pm_bases pm_bases; /* device-resident base points (SRS cache) */

/* ---------------------------------------------------------------- misc */
const char* pm_version(void);
const char* pm_last_error(void);
int pm_device_count(int* count);

/* ------------------------------------------------------------- context */
int pm_ctx_create(int device, pm_ctx** out);
int pm_ctx_destroy(pm_ctx* ctx);
/* Run on an external HIP stream (e.g. torch.cuda.current_stream().cuda_stream);
 * NULL restores the context's own stream. */
int pm_ctx_set_stream(pm_ctx* ctx, void* hip_stream);
/* Force the window width c (0 = automatic). */
int pm_ctx_set_window(pm_ctx* ctx, int c);
/* Per-kernel HIP-event timing on the context stream (for bench/profiling). */
int pm_ctx_set_timing(pm_ctx* ctx, int enable);
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
/* Same, on an explicit context (host pointers). */
int pm_msm_ctx(pm_ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n,
               uint32_t flags, uint64_t out[8]);
/* Same, with scalars and bases already in device memory of ctx's device. */
int pm_msm_device(pm_ctx* ctx, int curve, const void* d_scalars, const void* d_bases, size_t n,
                  uint32_t flags, uint64_t out[8]);
/* Split the points into `ngpu` contiguous slices, one device each (devices
 * 0..ngpu-1), and sum the per-device partial points (the multi-GPU analogue
 * of best_multiexp's per-thread chunks). */
int pm_msm_multi(int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
                 int ngpu, uint64_t out[8]);

/* Device-resident base cache: the SRS bases of halo2 Params are fixed, so a
 * caller uploads them once and runs many MSMs against a window of them. */
int pm_bases_upload(pm_ctx* ctx, int curve, const uint64_t* bases, size_t n, pm_bases** out);
int pm_bases_release(pm_bases* b);
int pm_msm_resident(pm_ctx* ctx, const pm_bases* b, size_t offset, const uint64_t* scalars,
                    size_t n, uint32_t flags, uint64_t out[8]);

/* Affine helpers (host) for combining partial results: out = a + b. */
int pm_point_add(int curve, const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);

/* Synthetic inputs generated on the device: scalar i is
 * uniform in [0, r) from a SplitMix64 stream keyed by (seed, i0 + i);
 * base i is [a_i]G with a_i drawn the same way.  d_out: n*4 (scalars) or n*8
 * (bases) u64 in device memory.  Scalars are Montgomery unless
 * PM_SCALARS_CANONICAL is set. */
int pm_synth_scalars(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, uint32_t flags,
                     void* d_out);
int pm_synth_bases(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, void* d_out);

#ifdef __cplusplus
}
#endif
#endif /* PASTA_MSM_H */

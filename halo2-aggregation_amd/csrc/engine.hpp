// engine.hpp -- templated MSM pipeline driver (instantiated once per curve).
//
// Boundary: halo2 `best_multiexp` ([3P], /root/reference/examples/
// simple-example.rs:606,620,638-640,702,722); see include/pasta_msm.h.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "msm_kernels.hpp"
#include "runtime.hpp"

// time a launch on the context stream when timing is enabled
#define PM_LAUNCH(ctx, name, ...)                                        \
  do {                                                                   \
    hipEvent_t a_ = nullptr, b_ = nullptr;                               \
    if ((ctx)->timing) {                                                 \
      a_ = (ctx)->next_event();                                          \
      b_ = (ctx)->next_event();                                          \
      (void)hipEventRecord(a_, (ctx)->stream);                           \
    }                                                                    \
    __VA_ARGS__;                                                         \
    hipError_t le_ = hipGetLastError();                                  \
    if (le_ != hipSuccess)                                               \
      return pm::set_error(PM_ERR_HIP, std::string("launch ") + (name) + \
                                           ": " + hipGetErrorString(le_)); \
    if ((ctx)->timing) {                                                 \
      (void)hipEventRecord(b_, (ctx)->stream);                           \
      (ctx)->mark((name), a_, b_);                                       \
    }                                                                    \
  } while (0)

namespace pm {
// ---------------------------------------------------------- MSM pipeline

template <class Fs, int W>
void launch_digits_w(const uint32_t* s, uint32_t n, int NB, uint32_t canonical, uint32_t* digits,
                     uint32_t* counts, hipStream_t st) {
  k_digits<Fs, W><<<(n + 255) / 256, 256, 0, st>>>(s, n, NB, canonical, digits, counts);
}

// one instance per window count reachable from c in [kMinC, kMaxC]
template <class Fs>
int launch_digits(int W, const uint32_t* s, uint32_t n, int NB, uint32_t canonical, uint32_t* digits,
                  uint32_t* counts, hipStream_t st) {
  switch (W) {
#define PM_W(k) \
  case k: launch_digits_w<Fs, k>(s, n, NB, canonical, digits, counts, st); return PM_OK;
    PM_W(13) PM_W(14) PM_W(15) PM_W(16) PM_W(18) PM_W(19) PM_W(20) PM_W(22) PM_W(24) PM_W(26) PM_W(29)
    PM_W(32) PM_W(37) PM_W(43) PM_W(52) PM_W(64)
#undef PM_W
    default: return set_error(PM_ERR_UNSUPPORTED, "window count out of range");
  }
}

// Run the device pipeline; result = host XYZZ point (sum over windows).
template <class Cv>
int msm_device_impl(Ctx* ctx, const uint32_t* d_scalars, const uint32_t* d_bases, size_t n, uint32_t flags,
                    Xyzz<typename Cv::Base>* result) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  if (n == 0) {
    *result = xyzz_inf<F>();
    return PM_OK;
  }
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "n exceeds 2^26 points per device call");
  const MsmPlan pl = make_plan(n, ctx->window_c);
  const hipStream_t st = ctx->stream;
  const size_t TOT = (size_t)pl.W * pl.NB + 1;
  const size_t nW = (size_t)n * pl.W;
  int rc;
  if ((rc = ctx->digits.ensure(nW * 4))) return rc;
  if ((rc = ctx->sorted.ensure(nW * 4))) return rc;
  if ((rc = ctx->counts.ensure(TOT * 4))) return rc;
  if ((rc = ctx->offsets.ensure(TOT * 4))) return rc;
  if ((rc = ctx->cursor.ensure(TOT * 4))) return rc;
  const uint32_t nb = (uint32_t)((TOT + kScanChunk - 1) / kScanChunk);
  if ((rc = ctx->bsum.ensure((size_t)nb * 4))) return rc;
  if ((rc = ctx->buckets.ensure((size_t)pl.W * pl.NB * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->head.ensure((size_t)pl.nthreads * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->segS.ensure((size_t)pl.W * pl.M1 * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->segT.ensure((size_t)pl.W * pl.M1 * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->bits.ensure((size_t)pl.W * (pl.NB2 + 1) * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->win.ensure((size_t)pl.W * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->longs.ensure(16 + (size_t)pl.maxlong * sizeof(LongChain)))) return rc;
  if ((rc = ctx->ensure_pinned((size_t)pl.W * sizeof(Xyzz<F>)))) return rc;

  uint32_t* digits = (uint32_t*)ctx->digits.p;
  uint32_t* sorted = (uint32_t*)ctx->sorted.p;
  uint32_t* counts = (uint32_t*)ctx->counts.p;
  uint32_t* offsets = (uint32_t*)ctx->offsets.p;
  uint32_t* cursor = (uint32_t*)ctx->cursor.p;
  uint32_t* bsum = (uint32_t*)ctx->bsum.p;
  Xyzz<F>* buckets = (Xyzz<F>*)ctx->buckets.p;
  Xyzz<F>* head = (Xyzz<F>*)ctx->head.p;
  Xyzz<F>* S = (Xyzz<F>*)ctx->segS.p;
  Xyzz<F>* T = (Xyzz<F>*)ctx->segT.p;
  Xyzz<F>* G = (Xyzz<F>*)ctx->bits.p;
  Xyzz<F>* R = (Xyzz<F>*)ctx->win.p;
  const uint32_t un = (uint32_t)n;

  uint32_t* nlong = (uint32_t*)ctx->longs.p;
  LongChain* longs = (LongChain*)((char*)ctx->longs.p + 16);
  HIP_TRY(hipMemsetAsync(counts, 0, TOT * 4, st));
  HIP_TRY(hipMemsetAsync(nlong, 0, 16, st));
  PM_LAUNCH(ctx, "digits",
            rc = launch_digits<Fs>(pl.W, d_scalars, un, pl.NB, (flags & PM_SCALARS_CANONICAL) ? 1u : 0u,
                                   digits, counts, st));
  if (rc) return rc;
  PM_LAUNCH(ctx, "scan", {
    k_scan_reduce<<<nb, kScanThreads, 0, st>>>(counts, (uint32_t)TOT, bsum);
    k_scan_top<<<1, 1024, 0, st>>>(bsum, nb);
    k_scan_down<<<nb, kScanThreads, 0, st>>>(counts, (uint32_t)TOT, bsum, offsets, cursor);
  });
  PM_LAUNCH(ctx, "scatter",
            (k_scatter<<<(uint32_t)((nW + 255) / 256), 256, 0, st>>>(digits, un, pl.W, pl.NB, cursor, sorted)));
  const uint32_t nslots = (uint32_t)(TOT - 1);
  PM_LAUNCH(ctx, "accumulate",
            (k_accumulate<F><<<(pl.nthreads + 255) / 256, 256, 0, st>>>(sorted, offsets, nslots, d_bases,
                                                                         pl.chunk, buckets, head)));
  PM_LAUNCH(ctx, "fixup", {
    k_fixup<F><<<(pl.nthreads + 255) / 256, 256, 0, st>>>(offsets, nslots, pl.chunk, pl.nthreads, buckets, head,
                                                           longs, nlong);
    k_fixup_long<F><<<pl.maxlong, 256, 0, st>>>(longs, nlong, buckets, head);
  });
  PM_LAUNCH(ctx, "bucket_seg",
            (k_bucket_seg<F><<<(pl.W * pl.M1 + 255) / 256, 256, 0, st>>>(offsets, buckets, pl.W, pl.NB, pl.L1,
                                                                          S, T)));
  PM_LAUNCH(ctx, "bucket_bits",
            (k_bucket_bits<F><<<dim3(pl.NB2 + 1, pl.W), kRedThreads, 0, st>>>(S, T, pl.M1, pl.NB2, G)));
  PM_LAUNCH(ctx, "window", (k_window<F><<<1, 64, 0, st>>>(G, pl.W, pl.NB2, pl.log2L1, R)));
  HIP_TRY(hipMemcpyAsync(ctx->h_pinned, R, (size_t)pl.W * sizeof(Xyzz<F>), hipMemcpyDeviceToHost, st));
  HIP_TRY(hipStreamSynchronize(st));
  ctx->end_call();

  // window combine on the host: sum_w 2^(o_w) R_w (Horner, c_w doublings)
  const Xyzz<F>* hR = (const Xyzz<F>*)ctx->h_pinned;
  Xyzz<F> acc = hR[pl.W - 1];
  for (int w = pl.W - 2; w >= 0; w--) {
    for (int k = 0; k < pl.width(w); k++) acc = xyzz_dbl<F>(acc);
    acc = xyzz_add<F>(acc, hR[w]);
  }
  *result = acc;
  return PM_OK;
}

template <class F>
void aff_to_u64(const Aff<F>& a, uint64_t out[8]) {
  for (int k = 0; k < 4; k++) {
    out[k] = (uint64_t)a.x.l[2 * k] | ((uint64_t)a.x.l[2 * k + 1] << 32);
    out[4 + k] = (uint64_t)a.y.l[2 * k] | ((uint64_t)a.y.l[2 * k + 1] << 32);
  }
}
template <class F>
Aff<F> aff_from_u64(const uint64_t in[8]) {
  Aff<F> a;
  for (int k = 0; k < 4; k++) {
    a.x.l[2 * k] = (uint32_t)in[k];
    a.x.l[2 * k + 1] = (uint32_t)(in[k] >> 32);
    a.y.l[2 * k] = (uint32_t)in[4 + k];
    a.y.l[2 * k + 1] = (uint32_t)(in[4 + k] >> 32);
  }
  return a;
}

template <class Cv>
int msm_device_to_aff(Ctx* ctx, const void* d_s, const void* d_b, size_t n, uint32_t flags, uint64_t out[8]) {
  using F = typename Cv::Base;
  Xyzz<F> r;
  int rc = msm_device_impl<Cv>(ctx, (const uint32_t*)d_s, (const uint32_t*)d_b, n, flags, &r);
  if (rc) return rc;
  aff_to_u64<F>(xyzz_to_aff<F>(r), out);
  return PM_OK;
}

template <class F>
int point_add_impl(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]) {
  Xyzz<F> r = xyzz_add_aff<F>(xyzz_from_aff<F>(aff_from_u64<F>(a)), aff_from_u64<F>(b));
  aff_to_u64<F>(xyzz_to_aff<F>(r), out);
  return PM_OK;
}

template <class Cv>
int synth_scalars_impl(Ctx* ctx, uint64_t seed, uint64_t i0, uint32_t n, uint32_t mont, void* d_out) {
  k_synth_scalars<typename Cv::Scalar><<<(n + 255) / 256, 256, 0, ctx->stream>>>(seed, i0, n, mont, (uint32_t*)d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

template <class Cv>
int synth_bases_impl(Ctx* ctx, uint64_t seed, uint64_t i0, uint32_t n, void* d_out) {
  k_synth_bases<Cv><<<(n + 255) / 256, 256, 0, ctx->stream>>>(seed, i0, n, (uint32_t*)d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

}  // namespace pm

// Explicit instantiations are visible to both compilation passes, so the
// device pass instantiates every kernel the host driver launches; the op
// table (host function pointers) exists only in the host pass.
#if defined(__HIP_DEVICE_COMPILE__)
#define PM_OPS_TABLE(Cv, name)
#else
#define PM_OPS_TABLE(Cv, name)                                                                 \
  extern const CurveOps name;                                                                  \
  const CurveOps name = {&msm_device_to_aff<Cv>, &point_add_impl<typename Cv::Base>,            \
                         &synth_scalars_impl<Cv>, &synth_bases_impl<Cv>};
#endif
#define PM_DEFINE_CURVE_OPS(Cv, name)                                                          \
  namespace pm {                                                                               \
  template int msm_device_to_aff<Cv>(Ctx*, const void*, const void*, size_t, uint32_t, uint64_t*); \
  template int synth_scalars_impl<Cv>(Ctx*, uint64_t, uint64_t, uint32_t, uint32_t, void*);     \
  template int synth_bases_impl<Cv>(Ctx*, uint64_t, uint64_t, uint32_t, void*);                 \
  PM_OPS_TABLE(Cv, name)                                                                       \
  }

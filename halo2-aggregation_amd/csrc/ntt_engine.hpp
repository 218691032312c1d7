// ntt_engine.hpp -- host driver of the NTT (pm_fft*).
// Boundary: halo2 `best_fft(a: &mut [G], omega: G::Scalar, log_n: u32)` [3P],
// reached from EvaluationDomain::{fft, ifft, coeff_to_extended,
// extended_to_coeff} inside create_proof (examples/simple-example.rs:606,702).
#pragma once
#include <cstring>

#include "engine.hpp"
#include "ntt_kernels.hpp"

namespace pm {

// Up to 2^7 elements one block does the whole transform; above that the
// two-pass form spreads it over many blocks (a single block for 2^12 took
// 0.14 ms, two passes 0.03 ms).
constexpr uint32_t kNttOnePassLog = 7;

template <class Fs>
FeArg fearg_from_u64(const uint64_t* p) {
  FeArg a;
  for (int k = 0; k < 4; k++) {
    a.l[2 * k] = (uint32_t)p[k];
    a.l[2 * k + 1] = (uint32_t)(p[k] >> 32);
  }
  return a;
}

// twiddle table omega^i (i < n/2), cached per (curve, log_n, omega)
inline int ntt_twiddles_lookup(Ctx* ctx, int curve, uint32_t logn, const uint64_t omega[4], const uint32_t** out,
                               bool* fresh) {
  for (auto& e : ctx->ntt_tw) {
    if (e.curve == curve && e.logn == logn && std::memcmp(e.omega, omega, 32) == 0) {
      e.stamp = ++ctx->ntt_clock;
      *out = (const uint32_t*)e.buf.p;
      *fresh = false;
      return PM_OK;
    }
  }
  NttTwiddles* slot = nullptr;
  if (ctx->ntt_tw.size() < kNttTwiddleSlots) {
    ctx->ntt_tw.emplace_back();
    slot = &ctx->ntt_tw.back();
  } else {
    slot = &ctx->ntt_tw[0];
    for (auto& e : ctx->ntt_tw)
      if (e.stamp < slot->stamp) slot = &e;
  }
  slot->curve = curve;
  slot->logn = logn;
  std::memcpy(slot->omega, omega, 32);
  slot->stamp = ++ctx->ntt_clock;
  int rc = slot->buf.ensure(std::max<size_t>(32, ((size_t)1 << (logn ? logn - 1 : 0)) * 32));
  if (rc) {
    slot->curve = -1;
    return rc;
  }
  *out = (const uint32_t*)slot->buf.p;
  *fresh = true;
  return PM_OK;
}

// elements per block (2^kNttPlaneLog): C = 2^logC adjacent columns / rows of a
// short sub-transform share one block so that global accesses move C x 32
// contiguous bytes (A/B: PM_NTT_PLANE_LOG=10 measured within noise,
// profiles/r03/ntt_f29/ab.jsonl)
#ifndef PM_NTT_PLANE_LOG
#define PM_NTT_PLANE_LOG 11
#endif
constexpr int kNttPlaneLog = PM_NTT_PLANE_LOG;

// passes over HBM: one up to 2^7 (one LDS transform), two up to 2^22 (four
// steps, factors <= 2^11), three above (factors <= 2^10: at 2^23 / 2^24 the
// two-pass form's 2^12-point transforms need 128 KiB of LDS, one block per
// CU).  PM_NTT_PASSES (2 or 3) overrides for 2^15 <= n (diagnostics).
inline int ntt_passes(const Ctx* ctx, uint32_t logn) {
  if (ctx->ntt_passes == 2 && logn <= 2 * (uint32_t)kNttMaxLogL) return 2;
  if (ctx->ntt_passes == 3 && logn >= 15) return 3;
  return logn <= 22 ? 2 : 3;
}

template <class Cv>
int ntt_device_impl(Ctx* ctx, int curve, void* d_data, uint32_t logn, const uint64_t omega[4],
                    const uint64_t* scale) {
  using Fs = typename Cv::Scalar;
  if (logn > kNttMaxLog) return set_error(PM_ERR_UNSUPPORTED, "NTT longer than 2^28");
  if (logn == 0) {
    if (scale) {  // a_0 *= scale
      // a one-element transform is the identity; apply the scale on the host
      uint64_t v[4];
      HIP_TRY(hipMemcpyAsync(v, d_data, 32, hipMemcpyDeviceToHost, ctx->stream));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
      const Fe<Fs> r = fe_mul<Fs>(fe_from_u64<Fs>(v), fe_from_u64<Fs>(scale));
      for (int k = 0; k < 4; k++) v[k] = (uint64_t)r.l[2 * k] | ((uint64_t)r.l[2 * k + 1] << 32);
      HIP_TRY(hipMemcpyAsync(d_data, v, 32, hipMemcpyHostToDevice, ctx->stream));
      HIP_TRY(hipStreamSynchronize(ctx->stream));
    }
    return PM_OK;
  }
  const hipStream_t st = ctx->stream;
  const size_t n = (size_t)1 << logn;
  const uint32_t half = (uint32_t)(n >> 1);
  const uint32_t* tw = nullptr;
  bool fresh = false;
  int rc = ntt_twiddles_lookup(ctx, curve, logn, omega, &tw, &fresh);
  if (rc) return rc;
  if (fresh)
    PM_LAUNCH(ctx, "ntt_twiddles", (k_ntt_twiddles<Fs><<<(half + 255) / 256, 256, 0, st>>>(
                                       fearg_from_u64<Fs>(omega), half, (uint32_t*)tw)));
  const FeArg sc = scale ? fearg_from_u64<Fs>(scale) : FeArg{};
  // threads per block: one / two passes and three passes (A/B: PM_NTT_THREADS2 / 3)
  const unsigned nt2 = (unsigned)ctx->ntt_threads2, nt3 = (unsigned)ctx->ntt_threads3;
  uint32_t* data = (uint32_t*)d_data;
  if (logn <= (uint32_t)kNttOnePassLog) {
    // one sub-transform in LDS (pass A with a single column, in place)
    const size_t lds = n * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<1, nt2, lds, st>>>(data, data, (int)logn, (int)logn, 0, tw, scale ? 0u : 1u)));
    if (scale) {
      // scaling rides on a rows pass of length 1 would be wasteful: fold it in
      // with a trivial rows pass of log2 = 0 (one element per row)
      PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)(n >> std::min<uint32_t>(logn, 8)), nt2,
                                                   ((size_t)1 << std::min<uint32_t>(logn, 8)) * kNttLdsBytes, st>>>(
                                     data, data, (int)logn, 0, (int)std::min<uint32_t>(logn, 8), tw, sc, 1u)));
    }
  } else if (ntt_passes(ctx, logn) == 2) {
    const int log1 = (int)(logn + 1) / 2, log2 = (int)logn - log1;
    const int mc = ctx->ntt_maxlogc;
    const int logC = std::max(0, std::min(mc, kNttPlaneLog - log1)), logR = std::max(0, std::min(mc, kNttPlaneLog - log2));
    if ((rc = ctx->ntt_scratch.ensure(n * 32))) return rc;
    uint32_t* tmp = (uint32_t*)ctx->ntt_scratch.p;
    const size_t ldsA = ((size_t)1 << (log1 + logC)) * kNttLdsBytes, ldsB = ((size_t)1 << (log2 + logR)) * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<(unsigned)((size_t)1 << (log2 - logC)), nt2, ldsA, st>>>(
                                   data, tmp, (int)logn, log1, logC, tw, 0u)));
    PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)((size_t)1 << (log1 - logR)), nt2, ldsB, st>>>(
                                   tmp, data, (int)logn, log2, logR, tw, sc, scale ? 1u : 0u)));
  } else {
    // three passes (k_ntt_kernels.hpp: k_ntt_mid), factors of at most 2^10,
    // through two scratch buffers (the middle pass permutes rows)
    int log1 = (int)(logn + 2) / 3;
    if (ctx->ntt_log1 > 0) log1 = std::max((int)logn - 2 * kNttMaxLogL, std::min(std::min(kNttMaxLogL, ctx->ntt_log1), (int)logn - 2));
    const int loga = ((int)logn - log1 + 1) / 2, logb = (int)logn - log1 - loga;
    const int mc = ctx->ntt_maxlogc;
    const int logC = std::max(0, std::min(mc, kNttPlaneLog - log1)), logM = std::max(0, std::min(mc, kNttPlaneLog - loga)),
              logR = std::max(0, std::min(mc, kNttPlaneLog - logb));
    if ((rc = ctx->ntt_scratch.ensure(n * 32)) || (rc = ctx->ntt_scratch2.ensure(n * 32))) return rc;
    uint32_t* tmp = (uint32_t*)ctx->ntt_scratch.p;
    uint32_t* tmp2 = (uint32_t*)ctx->ntt_scratch2.p;
    const size_t ldsA = ((size_t)1 << (log1 + logC)) * kNttLdsBytes, ldsM = ((size_t)1 << (loga + logM)) * kNttLdsBytes,
                 ldsB = ((size_t)1 << (logb + logR)) * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<(unsigned)(n >> (log1 + logC)), nt3, ldsA, st>>>(
                                   data, tmp, (int)logn, log1, logC, tw, 0u)));
    PM_LAUNCH(ctx, "ntt_mid", (k_ntt_mid<Fs><<<(unsigned)(n >> (loga + logM)), nt3, ldsM, st>>>(
                                  tmp, tmp2, (int)logn, log1, loga, logM, tw)));
    PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)(n >> (logb + logR)), nt3, ldsB, st>>>(
                                   tmp2, data, (int)logn, logb, logR, tw, sc, scale ? 1u : 0u)));
  }
  HIP_TRY(hipStreamSynchronize(st));
  ctx->end_call();
  return PM_OK;
}

}  // namespace pm

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

// twiddle segments (ntt_kernels.hpp), cached per (curve, log_n, omega)
inline int ntt_twiddles_lookup(Ctx* ctx, int curve, uint32_t logn, const uint64_t omega[4], size_t words,
                               NttTwiddles** out, bool* fresh) {
  for (auto& e : ctx->ntt_tw) {
    if (e.curve == curve && e.logn == logn && std::memcmp(e.omega, omega, 32) == 0) {
      e.stamp = ++ctx->ntt_clock;
      *out = &e;
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
  int rc = slot->buf.ensure(std::max<size_t>(32, words * 4));
  if (rc) {
    slot->curve = -1;
    return rc;
  }
  *out = slot;
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
// CU).  PM_NTT_PASSES (2 or 3) overrides for 2^15 <= n (test hook: the
// three-pass form below 2^23).
inline int ntt_passes(const Ctx* ctx, uint32_t logn) {
  if (ctx->ntt_passes == 2 && logn <= 2 * (uint32_t)kNttMaxLogL) return 2;
  if (ctx->ntt_passes == 3 && logn >= 15) return 3;
  return logn <= 22 ? 2 : 3;
}
// most adjacent columns / rows per block, log2 (round 3 A/B: 2)
constexpr int kNttMaxLogC = 2;
// threads per block: one / two passes, three passes (round 3 A/B,
// profiles/r03/ntt_f29/threads_ab3.jsonl)
constexpr unsigned kNttThreads2 = 512, kNttThreads3 = 256;

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
  // factorisation and twiddle segments: [sub-transform segments | lo | hi]
  const int passes = logn <= (uint32_t)kNttOnePassLog ? 1 : ntt_passes(ctx, logn);
  int log1 = (int)logn, loga = 0, logb = 0;
  if (passes == 2) {
    log1 = (int)(logn + 1) / 2;
    logb = (int)logn - log1;
  } else if (passes == 3) {
    log1 = (int)(logn + 2) / 3;
    loga = ((int)logn - log1 + 1) / 2;
    logb = (int)logn - log1 - loga;
  }
  const int s2 = (int)(logn + 1) / 2;  // inter-pass split: lo 2^s2, hi 2^(logn - s2) entries
  NttSegs sg{};
  sg.logn = logn;
  uint32_t words = 0;
  auto seg = [&](uint32_t count, uint32_t step) {
    const uint32_t k = sg.nseg++;
    sg.off[k] = words / 8;
    sg.count[k] = std::max(1u, count);
    sg.step[k] = step;
    words += 8 * sg.count[k];
    return k;
  };
  const uint32_t n1 = 1u << log1, na = 1u << loga, nb = 1u << logb;
  const uint32_t sA = seg(n1 >> 1, na * nb);                           // root omega^{n / n1}
  const uint32_t sM = passes == 3 ? seg(na >> 1, n1 * nb) : sA;       // root omega^{n1 nb}
  const uint32_t sB = passes >= 2 ? seg(nb >> 1, n1 * na) : sA;       // root omega^{n1 na}
  const uint32_t sLo = passes >= 2 ? seg(1u << s2, 1) : sA;
  const uint32_t sHi = passes >= 2 ? seg(1u << (logn - s2), 1u << s2) : sA;
  NttTwiddles* twe = nullptr;
  bool fresh = false;
  int rc = ntt_twiddles_lookup(ctx, curve, logn, omega, words, &twe, &fresh);
  if (rc) return rc;
  const uint32_t* tw = (const uint32_t*)twe->buf.p;
  if (fresh) {
    uint32_t tot = 0;
    for (uint32_t k = 0; k < sg.nseg; k++) tot += sg.count[k];
    PM_LAUNCH(ctx, "ntt_twiddles", (k_ntt_twiddles<Fs><<<(tot + 255) / 256, 256, 0, st>>>(
                                       fearg_from_u64<Fs>(omega), sg, (uint32_t*)tw)));
  }
  const uint32_t *twA = tw + 8ull * sg.off[sA], *twM = tw + 8ull * sg.off[sM], *twB = tw + 8ull * sg.off[sB];
  const uint32_t *twLo = tw + 8ull * sg.off[sLo], *twHi = tw + 8ull * sg.off[sHi];
  const FeArg sc = scale ? fearg_from_u64<Fs>(scale) : FeArg{};
  const unsigned nt2 = kNttThreads2, nt3 = kNttThreads3;
  uint32_t* data = (uint32_t*)d_data;
  if (passes == 1) {
    // one sub-transform in LDS (pass A with a single column, in place)
    const size_t lds = n * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<1, nt2, lds, st>>>(data, data, (int)logn, (int)logn, 0, twA, twLo,
                                                                     twHi, 0, scale ? 0u : 1u)));
    if (scale) {
      // the scale rides on a trivial rows pass of log2 = 0 (one element per row)
      PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)(n >> std::min<uint32_t>(logn, 8)), nt2,
                                                   ((size_t)1 << std::min<uint32_t>(logn, 8)) * kNttLdsBytes, st>>>(
                                     data, data, (int)logn, 0, (int)std::min<uint32_t>(logn, 8), twB, sc, 1u)));
    }
  } else if (passes == 2) {
    const int log2 = logb;
    const int logC = std::max(0, std::min(kNttMaxLogC, kNttPlaneLog - log1)),
              logR = std::max(0, std::min(kNttMaxLogC, kNttPlaneLog - log2));
    if ((rc = ctx->ntt_scratch.ensure(n * 32))) return rc;
    uint32_t* tmp = (uint32_t*)ctx->ntt_scratch.p;
    const size_t ldsA = ((size_t)1 << (log1 + logC)) * kNttLdsBytes, ldsB = ((size_t)1 << (log2 + logR)) * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<(unsigned)((size_t)1 << (log2 - logC)), nt2, ldsA, st>>>(
                                   data, tmp, (int)logn, log1, logC, twA, twLo, twHi, s2, 0u)));
    PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)((size_t)1 << (log1 - logR)), nt2, ldsB, st>>>(
                                   tmp, data, (int)logn, log2, logR, twB, sc, scale ? 1u : 0u)));
  } else {
    // three passes (ntt_kernels.hpp: k_ntt_mid), factors of at most 2^10,
    // through two scratch buffers (the middle pass permutes rows)
    const int logC = std::max(0, std::min(kNttMaxLogC, kNttPlaneLog - log1)),
              logM = std::max(0, std::min(kNttMaxLogC, kNttPlaneLog - loga)),
              logR = std::max(0, std::min(kNttMaxLogC, kNttPlaneLog - logb));
    if ((rc = ctx->ntt_scratch.ensure(n * 32)) || (rc = ctx->ntt_scratch2.ensure(n * 32))) return rc;
    uint32_t* tmp = (uint32_t*)ctx->ntt_scratch.p;
    uint32_t* tmp2 = (uint32_t*)ctx->ntt_scratch2.p;
    const size_t ldsA = ((size_t)1 << (log1 + logC)) * kNttLdsBytes, ldsM = ((size_t)1 << (loga + logM)) * kNttLdsBytes,
                 ldsB = ((size_t)1 << (logb + logR)) * kNttLdsBytes;
    PM_LAUNCH(ctx, "ntt_cols", (k_ntt_cols<Fs><<<(unsigned)(n >> (log1 + logC)), nt3, ldsA, st>>>(
                                   data, tmp, (int)logn, log1, logC, twA, twLo, twHi, s2, 0u)));
    PM_LAUNCH(ctx, "ntt_mid", (k_ntt_mid<Fs><<<(unsigned)(n >> (loga + logM)), nt3, ldsM, st>>>(
                                  tmp, tmp2, (int)logn, log1, loga, logM, twM, twLo, twHi, s2)));
    PM_LAUNCH(ctx, "ntt_rows", (k_ntt_rows<Fs><<<(unsigned)(n >> (logb + logR)), nt3, ldsB, st>>>(
                                   tmp2, data, (int)logn, logb, logR, twB, sc, scale ? 1u : 0u)));
  }
  HIP_TRY(hipStreamSynchronize(st));
  ctx->end_call();
  return PM_OK;
}

}  // namespace pm

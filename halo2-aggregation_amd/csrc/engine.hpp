// engine.hpp -- templated MSM pipeline driver (instantiated once per curve).
//
// Boundary: halo2 `best_multiexp` ([3P], /root/reference/examples/
// simple-example.rs:606,620,638-640,702,722); see include/pasta_msm.h.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>

#include "host_ec.hpp"
#include "msm_kernels.hpp"
#include "runtime.hpp"

// time a launch on stream `st_` when timing is enabled
#define PM_LAUNCH_ST(ctx, st_, name, ...)                                \
  do {                                                                   \
    hipEvent_t a_ = nullptr, b_ = nullptr;                               \
    const bool tm_ = (ctx)->timed(name);                                 \
    if (tm_) {                                                           \
      a_ = (ctx)->next_event();                                          \
      b_ = (ctx)->next_event();                                          \
      (void)hipEventRecord(a_, (st_));                                   \
    }                                                                    \
    __VA_ARGS__;                                                         \
    hipError_t le_ = hipGetLastError();                                  \
    if (le_ != hipSuccess)                                               \
      return pm::set_error(PM_ERR_HIP, std::string("launch ") + (name) + \
                                           ": " + hipGetErrorString(le_)); \
    if (tm_) {                                                           \
      (void)hipEventRecord(b_, (st_));                                   \
      (ctx)->mark((name), a_, b_);                                       \
    }                                                                    \
  } while (0)
#define PM_LAUNCH(ctx, name, ...) PM_LAUNCH_ST(ctx, (ctx)->stream, name, __VA_ARGS__)

namespace pm {
// ---------------------------------------------------------- MSM pipeline

template <bool D16, bool WIDE>
void launch_coarse(const void* dg, uint32_t ue, SortGeom gm, const uint32_t* bofs, void* mid, dim3 grid, size_t lds,
                   hipStream_t st) {
  using DT = typename DigitCode<D16>::T;
  using MT = typename SortEntry<WIDE>::T;
  const DT* d = (const DT*)dg;
  MT* m = (MT*)mid;
  switch (gm.ppt) {
    case 1: k_sort_coarse<D16, WIDE, 1><<<grid, kSortThreads, lds, st>>>(d, ue, gm, bofs, m); break;
    case 2: k_sort_coarse<D16, WIDE, 2><<<grid, kSortThreads, lds, st>>>(d, ue, gm, bofs, m); break;
    case 4: k_sort_coarse<D16, WIDE, 4><<<grid, kSortThreads, lds, st>>>(d, ue, gm, bofs, m); break;
    default: k_sort_coarse<D16, WIDE, 8><<<grid, kSortThreads, lds, st>>>(d, ue, gm, bofs, m); break;
  }
}

template <class Fs, int W>
void launch_sort_w(bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, uint32_t* bh,
                   void* digits, uint32_t stride, uint32_t merged, hipStream_t st) {
  const size_t lds = (size_t)W * g.NCB * 4;
  if (d16)
    k_sort_hist<Fs, W, true><<<g.nblk, kSortThreads, lds, st>>>(s, n, canonical, g, (uint16_t*)digits, bh, stride,
                                                                merged);
  else
    k_sort_hist<Fs, W, false><<<g.nblk, kSortThreads, lds, st>>>(s, n, canonical, g, (uint32_t*)digits, bh, stride,
                                                                 merged);
}

// one instance per window count reachable from c in [kMinC, kMaxC]
template <class Fs>
int launch_sort(int W, bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, uint32_t* bh,
                void* digits, uint32_t stride, uint32_t merged, hipStream_t st) {
  switch (W) {
#define PM_W(k) \
  case k: launch_sort_w<Fs, k>(d16, s, n, canonical, g, bh, digits, stride, merged, st); return PM_OK;
    PM_W(13) PM_W(14) PM_W(15) PM_W(16) PM_W(18) PM_W(19) PM_W(20) PM_W(22) PM_W(24) PM_W(26) PM_W(29)
    PM_W(32) PM_W(37) PM_W(43) PM_W(52) PM_W(64)
#undef PM_W
    default: return set_error(PM_ERR_UNSUPPORTED, "window count out of range");
  }
}

// GLV mode (variable-base MSM, c >= kGlvMinC): W = ceil(128 / c) in {7 .. 11}
template <class Cv, int W>
void launch_sort_glv_w(bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, uint32_t* bh,
                       void* digits, uint32_t stride, hipStream_t st) {
  const size_t lds = (size_t)W * g.NCB * 4;
  if (d16)
    k_sort_hist_glv<Cv, W, true><<<g.nblk, kSortThreads, lds, st>>>(s, n, canonical, g, (uint16_t*)digits, bh, stride);
  else
    k_sort_hist_glv<Cv, W, false><<<g.nblk, kSortThreads, lds, st>>>(s, n, canonical, g, (uint32_t*)digits, bh,
                                                                       stride);
}
template <class Cv>
int launch_sort_glv(int W, bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, uint32_t* bh,
                    void* digits, uint32_t stride, hipStream_t st) {
  switch (W) {
#define PM_WG(k) \
  case k: launch_sort_glv_w<Cv, k>(d16, s, n, canonical, g, bh, digits, stride, st); return PM_OK;
    PM_WG(7) PM_WG(8) PM_WG(9) PM_WG(10) PM_WG(11)
#undef PM_WG
    default: return set_error(PM_ERR_UNSUPPORTED, "GLV window count out of range");
  }
}
constexpr int kGlvMinC = 12;  // below: the plain 256-bit pipeline (small n)

// Run the device pipeline; result = host XYZZ point (sum over windows).
//
// Sort once, then the windows are processed in G groups from the top window
// down.  Group g is accumulated on the context stream; its fixup, segment and
// bit sums and the D2H copy of its G_{w,b} run on red_stream while group g-1
// accumulates, and the host Horner over group g's bit positions runs while the
// GPU works on the lower groups (window w's terms sit at bit positions
// [o_w, o_w + cmax), so a group's positions are final once every group above
// it has arrived).
//
// Fixed-base mode (ft != nullptr, pm_msm_fixed): the bases are a precomputed
// table ft->d with entry w * npad + i = [2^{o_w}] P_i (k_fixed_table), so the
// digits of all W windows index ONE bucket set: the sort runs over the W * npad
// entries as a single window (merged histogram rows), and the bucket
// reduction and host tail handle one window at offset 0 -- no per-window
// reduction and no cross-window doublings.
// What the host Horner tail of one enqueued MSM needs (msm_tail): the plan's
// window geometry, the pinned slot its bit sums land in and its events.
template <class F>
struct MsmTail {
  int G = 0, Wr = 0, NQ = 0, wpg = 1, base = 0, extra = 0, log2L1 = 0, cmax = 0;
  bool fixed = false, empty = true;
  const Xyzz<F>* hG = nullptr;  // pinned host slot
  std::vector<hipEvent_t> ev;    // 2 per window group
  hipStream_t st = nullptr, st2 = nullptr;
};

template <class F>
int msm_tail(Ctx* ctx, const MsmTail<F>& t, Xyzz<F>* result);

// Enqueue the device pipeline of one MSM (everything up to the D2H copy of
// the folded bit sums into pinned slot `slot`) and describe its host tail in
// *tail; msm_tail then waits for it and runs the Horner.  Two MSMs can be in
// flight (slots 0 and 1): the tail of one overlaps the kernels of the next
// (pm_msm_resident_batch).  tail == nullptr: run the tail here.
template <class Cv>
int msm_device_impl(Ctx* ctx, const uint32_t* d_scalars, const uint32_t* d_bases, size_t n, uint32_t flags,
                    Xyzz<typename Cv::Base>* result, const pm_fixed_bases* ft = nullptr,
                    MsmTail<typename Cv::Base>* tail = nullptr, int slot = 0) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  if (n == 0) {
    if (tail) *tail = MsmTail<F>{};
    else *result = xyzz_inf<F>();
    return PM_OK;
  }
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "n exceeds 2^26 points per device call");
  const bool fixed = ft != nullptr;
  // GLV mode: s_i P_i = k1_i P_i + k2_i phi(P_i) with |k1|, |k2| < 2^127, i.e.
  // an MSM of 2n points with 128-bit scalars: the same number of bucket
  // additions, half the windows (bucket reduction and host Horner halve).
  // pre29: resident bases already in the pipeline's R = 2^261 form (pm_bases)
  const bool pre29 = !fixed && (flags & kBasesR261) != 0;
  MsmPlan pl = fixed ? make_plan_fixed(ft->npad, ft->c, ctx->min_chunk)
                     : make_plan(2 * n, ctx->window_c, ctx->groups, ctx->min_chunk, 128);
  const bool glv = !fixed && !pre29 && ctx->glv && pl.c >= kGlvMinC;
  if (!fixed && !glv) pl = make_plan(n, ctx->window_c, ctx->groups, ctx->min_chunk);
  const size_t npts = glv ? 2 * n : n;  // sort entries per window row
  // reduction stream only when window groups overlap; with one group the
  // cross-stream wake-up cost ~12 us between k_accumulate and the fixup
  const hipStream_t st = ctx->stream, st2 = pl.G > 1 ? ctx->red_stream : st;
  // fixed-base table of `rows` rows: windows w, w + Wr, ... share bucket set
  // w mod Wr (kmerge = rows; rows = W: one bucket set)
  const int kmerge = fixed ? ft->rows : 1;
  const int Wr = pl.W / kmerge;                     // bucket sets (reduced windows)
  const int wpg = fixed ? Wr : pl.wpg;
  const size_t stride = fixed ? ft->npad : npts;    // digit row length
  const size_t E = (size_t)kmerge * stride;         // entries of one sort row
  // merged buckets of many windows span several accumulate slices each: the
  // bucket-parallel fixup (k_fixup) then beats the chain lists
  const bool bucket_fixup = fixed && kmerge > 2;
  const size_t TOT = (size_t)Wr * pl.NB + 1;
  const size_t nW = (size_t)stride * pl.W;
  const int NJ = pl.NB2 + kTJobs;                        // bit-sum jobs per window
  // folded terms per window for the host Horner: bit folds, sum T, bucket K
  const int NQ = (pl.NB2 + kBitsFold - 1) / kBitsFold + 2;
  SortGeom g{};  // histogram geometry (blocks of scalars)
  g.FB = std::max(0, pl.cmax - 1 - 8);
  // the fixed-base MSM's merged sort rows are W x longer: 4x more coarse bins
  // once they exceed 2^24 entries (2^23, c = 20: FB 11 -> 9, sort 3.4 -> 2.3 ms)
  if (fixed && E > (size_t(1) << 24)) g.FB = std::max(0, pl.cmax - 1 - 10);
  if (ctx->sort_fb > 0) g.FB = std::min(pl.cmax - 1, ctx->sort_fb);  // PM_SORT_FB: tuning experiments
  g.NCB = (pl.K >> g.FB) + 1;
  // points per thread: blocks of 1024 threads x ppt points, ppt the largest
  // power of two <= 8 that still gives >= 128 blocks (2^20: 8192 points per
  // block; larger blocks give longer contiguous runs per coarse bin in
  // k_sort_coarse and a 4x smaller block histogram to scan: sort 0.19 ->
  // 0.16 ms at 2^20; small n keeps enough blocks)
  g.ppt = 1;
  while (g.ppt < kSortPerThread && stride >= (size_t)256 * g.ppt * kSortThreads) g.ppt *= 2;
  if (ctx->sort_ppt > 0 && !fixed) g.ppt = ctx->sort_ppt;  // PM_SORT_PPT (1, 2, 4, 8): tuning experiments
  g.nblk = (int)((stride + (size_t)g.ppt * kSortThreads - 1) / ((size_t)g.ppt * kSortThreads));
  // The histogram pass is compute-bound per block (Montgomery -> canonical,
  // W signed digits and LDS atomics per scalar); with 8192-point blocks 2^20
  // gives 128 blocks for 256 CUs.  Split each coarse block's points over 2
  // histogram blocks when the grid is short of the CUs: the coarse pass keeps
  // its long runs and reads its start offsets at every hsub-th histogram
  // block.  The scan doubles with it, so one split only (same box, 2^20:
  // histogram 0.049-0.050 -> 0.035-0.041 ms, scan 0.014 -> 0.019 ms; below
  // 128 blocks the scan's growth cancels the gain: 2^19 +-0, 2^18 +3-5 us,
  // profiles/r02/hs/ab.txt and profiles/r02/p/ab.txt).
  int hsub = 1;
  if (ctx->sort_ppt == 0 && g.ppt >= 2 && g.nblk >= 128 && g.nblk < 256) hsub = 2;
  g.hsub = 1;
  SortGeom gm = g;  // coarse / fine geometry (blocks of sort-row entries)
  g.ppt /= hsub;    // histogram geometry
  g.nblk *= hsub;
  gm.nblk = g.nblk * kmerge;
  gm.hsub = hsub;
  const size_t TOTB = (size_t)pl.W * g.NCB * g.nblk + 1;
  // 4-B coarse entries when the entry index fits beside the fine bits and the sign
  const bool wide = E > (size_t(1) << (31 - g.FB));
  const bool d16 = pl.cmax <= 16;
  // per group: [nlong, nshort, pad] [maxlong long chains] [nthreads short chains]
  const size_t longs_stride = (16 + ((size_t)pl.maxlong + pl.nthreads) * sizeof(LongChain) + 15) & ~size_t(15);
  int rc;
  if ((rc = ctx->digits.ensure(nW * (d16 ? 2 : 4)))) return rc;
  if ((rc = ctx->sorted.ensure(nW * 4))) return rc;
  if ((rc = ctx->mid.ensure(nW * (wide ? 8 : 4)))) return rc;
  if ((rc = ctx->counts.ensure(TOTB * 4))) return rc;
  if ((rc = ctx->cursor.ensure(TOTB * 4))) return rc;
  if ((rc = ctx->offsets.ensure(TOT * 4))) return rc;
  const uint32_t nb = (uint32_t)((TOTB + kScanChunk - 1) / kScanChunk);
  if ((rc = ctx->bsum.ensure((size_t)nb * 4))) return rc;
  if ((rc = ctx->buckets.ensure((size_t)Wr * pl.NB * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->head.ensure((size_t)pl.G * pl.nthreads * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->segS.ensure((size_t)Wr * (pl.M1 + 1) * sizeof(Xyzz<F>)))) return rc;  // S, then Kb
  if ((rc = ctx->segT.ensure((size_t)Wr * pl.M1 * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->bits.ensure((size_t)Wr * NJ * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->bitsQ.ensure((size_t)Wr * NQ * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->longs.ensure((size_t)pl.G * longs_stride))) return rc;
  const size_t nG = (size_t)Wr * NJ;
  if ((rc = ctx->ensure_pinned(2 * nG * sizeof(Xyzz<F>)))) return rc;  // two slots (batch pipelining)
  if ((rc = ctx->ensure_group_events(4 * pl.G))) return rc;
  Xyzz<F>* hslot = (Xyzz<F>*)ctx->h_pinned + (size_t)slot * nG;
  hipEvent_t* gev = ctx->grp_ev.data() + (size_t)2 * pl.G * slot;

  uint32_t* sorted = (uint32_t*)ctx->sorted.p;
  void* mid = ctx->mid.p;
  uint32_t* bh = (uint32_t*)ctx->counts.p;
  uint32_t* bofs = (uint32_t*)ctx->cursor.p;
  uint32_t* offsets = (uint32_t*)ctx->offsets.p;
  uint32_t* bsum = (uint32_t*)ctx->bsum.p;
  Xyzz<F>* buckets = (Xyzz<F>*)ctx->buckets.p;
  Xyzz<F>* head = (Xyzz<F>*)ctx->head.p;
  Xyzz<F>* S = (Xyzz<F>*)ctx->segS.p;
  Xyzz<F>* Kb = S + (size_t)Wr * pl.M1;  // per window: the top bucket K, folded
  Xyzz<F>* T = (Xyzz<F>*)ctx->segT.p;
  Xyzz<F>* G = (Xyzz<F>*)ctx->bits.p;
  Xyzz<F>* Qb = (Xyzz<F>*)ctx->bitsQ.p;
  const uint32_t un = (uint32_t)n;

  g.clr_bh = bh + (TOTB - 1);  // zeroed by the histogram kernel's block 0
  g.clr_longs = (uint32_t*)ctx->longs.p;
  g.clr_stride = (uint32_t)(longs_stride / 4);
  g.clr_groups = pl.G;
  // bases -> R261 once per MSM (with GLV: also phi(P)).  Running it on the
  // reduction stream beside the sort measured no faster: both are memory
  // bound (bases 0.04 -> 0.07 ms, histogram 0.048 -> 0.082 ms concurrently).
  const uint32_t* bases29;
  if (fixed) {
    bases29 = (const uint32_t*)ft->d;
  } else if (pre29) {
    bases29 = d_bases;
  } else {
    if ((rc = ctx->bases29.ensure(npts * 64))) return rc;
    bases29 = (const uint32_t*)ctx->bases29.p;
    if (glv)
      PM_LAUNCH(ctx, "bases_r261",
                (k_bases_glv<Cv><<<(un + 255) / 256, 256, 0, st>>>(d_bases, un, (uint32_t*)ctx->bases29.p)));
    else
      PM_LAUNCH(ctx, "bases_r261",
                (k_bases_to_r261<F><<<(un + 255) / 256, 256, 0, st>>>(d_bases, un, (uint32_t*)ctx->bases29.p)));
  }
  const uint32_t canon = (flags & PM_SCALARS_CANONICAL) ? 1u : 0u;
  if (glv)
    PM_LAUNCH(ctx, "sort_hist", rc = launch_sort_glv<Cv>(pl.W, d16, d_scalars, un, canon, g, bh, ctx->digits.p,
                                                         (uint32_t)stride, st));
  else
    PM_LAUNCH(ctx, "sort_hist", rc = launch_sort<Fs>(pl.W, d16, d_scalars, un, canon, g, bh, ctx->digits.p,
                                                     (uint32_t)stride, (uint32_t)kmerge, st));
  if (rc) return rc;
  PM_LAUNCH(ctx, "scan", {
    k_scan_reduce<<<nb, kScanThreads, 0, st>>>(bh, (uint32_t)TOTB, bsum);
    k_scan_down<<<nb, kScanThreads, 0, st>>>(bh, (uint32_t)TOTB, bsum, bofs, nullptr);
  });
  {
    const size_t lds = (size_t)gm.ppt * kSortThreads * ((wide ? 8 : 4) + 2) + (size_t)(2 * g.NCB + 1) * 4 + (kSortThreads / 64 + 1) * 4;
    const dim3 grid(gm.nblk / gm.hsub, Wr);
    void* dg = ctx->digits.p;
    const uint32_t ue = (uint32_t)E;
    if (d16 && !wide)
      PM_LAUNCH(ctx, "sort_coarse", launch_coarse<true, false>(dg, ue, gm, bofs, mid, grid, lds, st));
    else if (d16)
      PM_LAUNCH(ctx, "sort_coarse", launch_coarse<true, true>(dg, ue, gm, bofs, mid, grid, lds, st));
    else if (!wide)
      PM_LAUNCH(ctx, "sort_coarse", launch_coarse<false, false>(dg, ue, gm, bofs, mid, grid, lds, st));
    else
      PM_LAUNCH(ctx, "sort_coarse", launch_coarse<false, true>(dg, ue, gm, bofs, mid, grid, lds, st));
  }
  // LDS cache: room for 1.5x the mean segment (random digits fill segments
  // evenly; a skewed segment falls back to re-reading mid), capped at 64 KiB
  const size_t esz = wide ? 8 : 4;
  const size_t mean_seg = E / std::max(1, g.NCB - 1) + 1;
  // A mean segment that fits 24 KiB is cached whole (1.5x its size); larger
  // ones go through the chunked path in 16 KiB chunks, which keeps 3 blocks
  // per CU instead of one (2^22: sort_fine 0.48 -> 0.27 ms, fixed-base 2^23:
  // 2.5 -> 1.06 ms; profiles/r02/sort/fb_sweep.jsonl)
  size_t cache_cap = (mean_seg * 3 / 2 + 63) & ~size_t(63);
  if (cache_cap > kFineCacheSmall / esz) cache_cap = kFineChunkBytes / esz;
  if (ctx->fine_cache > 0) cache_cap = (size_t)ctx->fine_cache;  // PM_FINE_CACHE: tuning experiments
  uint32_t cache_n = (uint32_t)std::min<size_t>(cache_cap, kFineCacheBytes / esz);
  const size_t fine_fixed = ((size_t)3 * (1 << g.FB) + kFineThreads / 64 + 1) * 4;  // hist, lcur, lst, scan
  if (fine_fixed + 64 * (esz + 4) > kMaxLds) return set_error(PM_ERR_UNSUPPORTED, "sort: fine bits too wide");
  while (cache_n > 64 && (size_t)cache_n * (esz + 4) + fine_fixed > kMaxLds) cache_n /= 2;
  const size_t lds_fine = (size_t)cache_n * (esz + 4) + fine_fixed;
  if (wide)
    PM_LAUNCH(ctx, "sort_fine", (k_sort_fine<true><<<Wr * g.NCB, kFineThreads, lds_fine, st>>>(
                                    (const uint64_t*)mid, bofs, gm, Wr, pl.NB, cache_n, offsets, sorted)));
  else
    PM_LAUNCH(ctx, "sort_fine", (k_sort_fine<false><<<Wr * g.NCB, kFineThreads, lds_fine, st>>>(
                                    (const uint32_t*)mid, bofs, gm, Wr, pl.NB, cache_n, offsets, sorted)));
  const bool prefetch = ctx->prefetch >= 0 ? ctx->prefetch != 0 : (size_t)n * 64 > kPrefetchBytes;
  const unsigned ablocks = (pl.nthreads + 255) / 256;
  // chains + segment sums in one quad-cooperative kernel (k_bucket_seg_q);
  // PM_SEGQ=0: the separate k_fixup* + k_bucket_seg (A/B)
  static_assert(kL1 == (int)kSegQ, "k_bucket_seg_q takes one quad per segment");
  const bool segq = ctx->segq != 0;
  // bit sums of few windows (fixed-base: one bucket set) are split over
  // more blocks.  Every extra lane also adds one tree addition, so the split
  // stops at ~16 blocks per job (c = 20, 2^19 buckets: 16 -> 0.33 ms,
  // 64 -> 0.47 ms).
  const int nsplit = std::max(1, std::min(kMaxSplit, 16 / wpg));
  Xyzz<F>* bitsP = nullptr;
  uint32_t* tickets = nullptr;
  if (nsplit > 1) {
    if ((rc = ctx->bitsP.ensure((size_t)Wr * NJ * nsplit * sizeof(Xyzz<F>)))) return rc;
    const size_t old_cap = ctx->tickets.cap;  // tickets are self-resetting; zero fresh allocations
    if ((rc = ctx->tickets.ensure((size_t)Wr * NJ * 4))) return rc;
    if (ctx->tickets.cap != old_cap) HIP_TRY(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets.cap, st2));
    bitsP = (Xyzz<F>*)ctx->bitsP.p;
    tickets = (uint32_t*)ctx->tickets.p;
  }
  for (int gi = pl.G - 1; gi >= 0; gi--) {
    const int w0 = gi * wpg, w1 = std::min(Wr, w0 + wpg), nw = w1 - w0;
    const uint32_t s0 = (uint32_t)((size_t)w0 * pl.NB), s1 = (uint32_t)((size_t)w1 * pl.NB);
    Xyzz<F>* hg = head + (size_t)gi * pl.nthreads;
    uint32_t* nlong = (uint32_t*)((char*)ctx->longs.p + gi * longs_stride);
    LongChain* longs = (LongChain*)((char*)nlong + 16);
    uint32_t* nshort = nlong + 1;
    LongChain* shorts = longs + pl.maxlong;
    if (prefetch)
      PM_LAUNCH(ctx, "accumulate",
                (k_accumulate<F, true><<<ablocks, 256, 0, st>>>(sorted, offsets, s0, s1, bases29, pl.chunk, buckets, hg,
                                                                 pl.nthreads, (bucket_fixup && !segq) ? nullptr : longs, nlong,
                                                                 segq ? nullptr : shorts, nshort)));
    else
      PM_LAUNCH(ctx, "accumulate",
                (k_accumulate<F, false><<<ablocks, 256, 0, st>>>(sorted, offsets, s0, s1, bases29, pl.chunk, buckets, hg,
                                                                  pl.nthreads, (bucket_fixup && !segq) ? nullptr : longs, nlong,
                                                                 segq ? nullptr : shorts, nshort)));
    if (st2 != st) {
      HIP_TRY(hipEventRecord(gev[2 * gi], st));
      HIP_TRY(hipStreamWaitEvent(st2, gev[2 * gi], 0));
    }
    if (segq) {
      // long chains (usually none) first, then chains + segment sums in one
      PM_LAUNCH_ST(ctx, st2, "fixup",
                   (k_fixup_long<F><<<std::min<uint32_t>(pl.maxlong, 256), 256, 0, st2>>>(longs, nlong, buckets, hg)));
      PM_LAUNCH_ST(ctx, st2, "bucket_seg",
                   (k_bucket_seg_q<F><<<(unsigned)((4ull * nw * pl.M1 + 255) / 256), 256, 0, st2>>>(
                       offsets, s0, pl.chunk, pl.nthreads, buckets, hg, w0, nw, pl.NB, (uint32_t)pl.M1, S, T, Kb)));
    } else {
      PM_LAUNCH_ST(ctx, st2, "fixup", {
        const uint32_t lblocks = std::min<uint32_t>(pl.maxlong, 256);
        if (bucket_fixup) {  // merged buckets span ~W*n/2^(c-1)/chunk slices each: one lane per bucket
          k_fixup<F><<<(s1 - s0 + 255) / 256, 256, 0, st2>>>(offsets, s0, s1, pl.chunk, pl.nthreads, buckets, hg,
                                                             longs, nlong);
          k_fixup_long<F><<<lblocks, 256, 0, st2>>>(longs, nlong, buckets, hg);
        } else {
          k_fixup_short<F><<<ablocks + lblocks, 256, 0, st2>>>(shorts, nshort, buckets, hg, ablocks, longs, nlong);
        }
      });
      PM_LAUNCH_ST(ctx, st2, "bucket_seg",
                   (k_bucket_seg<F><<<(nw * pl.M1 + 255) / 256, 256, 0, st2>>>(offsets, buckets, w0, nw, pl.NB, pl.M1, pl.L1,
                                                                                 S, T, Kb)));
    }
    PM_LAUNCH_ST(ctx, st2, "bucket_bits",
                 (k_bucket_bits<F><<<dim3(NJ, nw, nsplit), kRedThreads, 0, st2>>>(S, T, w0, pl.M1, pl.NB2, G, nsplit,
                                                                                      bitsP, tickets)));
    PM_LAUNCH_ST(ctx, st2, "bits_combine",
                 (k_bits_combine<F><<<(4 * nw * NQ + 63) / 64, 64, 0, st2>>>(G, Kb, w0, nw, pl.NB2, Qb)));
    HIP_TRY(hipMemcpyAsync(hslot + (size_t)w0 * NQ, Qb + (size_t)w0 * NQ,
                           (size_t)nw * NQ * sizeof(Xyzz<F>), hipMemcpyDeviceToHost, st2));
    HIP_TRY(hipEventRecord(gev[2 * gi + 1], st2));
  }
  MsmTail<F> t;
  t.G = pl.G;
  t.Wr = Wr;
  t.NQ = NQ;
  t.wpg = wpg;
  t.base = pl.base;
  t.extra = pl.extra;
  t.log2L1 = pl.log2L1;
  t.cmax = pl.cmax;
  t.fixed = fixed;
  t.empty = false;
  t.hG = hslot;
  t.ev.assign(gev, gev + 2 * pl.G);
  t.st = st;
  t.st2 = st2;
  if (tail) {
    *tail = t;
    return PM_OK;
  }
  if ((rc = msm_tail<F>(ctx, t, result))) return rc;
  // msm_tail waited for every group's last event (recorded on st2 after the
  // partials' copy, which follows all of st's work): nothing is pending on
  // either stream.  A hipStreamSynchronize here still cost ~16 us per call
  // (profiles/r02/htr/), GPU idle before the next call.
  ctx->end_call();
  return PM_OK;
}

// The Horner steps q = hi .. lo (hi >= lo): one doubling per position, then
// the terms at that position.  Two builds: on a CPU with BMI2 / ADX the field
// products are host::mul_adx (mulx with two carry chains); the dispatch
// checks the CPU once.
template <class F>
inline void horner_steps(host::Pt<F>& hacc, int& q, int low, size_t& ti, const std::pair<int, int>* terms,
                         size_t nterms, const Xyzz<F>* hG) {
  for (; q >= low; q--) {
    hacc = host::dbl<F>(hacc);
    for (; ti < nterms && terms[ti].first == q; ti++) hacc = host::addp<F>(hacc, host::from_dev<F>(hG[terms[ti].second]));
  }
}
template <class F>
__attribute__((target("bmi2,adx"))) void horner_steps_bmi2(host::Pt<F>& hacc, int& q, int low, size_t& ti,
                                                           const std::pair<int, int>* terms, size_t nterms,
                                                           const Xyzz<F>* hG) {
  for (; q >= low; q--) {
    hacc = host::dbl<F, true>(hacc);
    for (; ti < nterms && terms[ti].first == q; ti++)
      hacc = host::addp<F, true>(hacc, host::from_dev<F>(hG[terms[ti].second]));
  }
}

// Host tail: sum_w 2^{o_w} (sum_j T_{w,j} + sum_b 2^{b+log2 L1} G_{w,b} + K B_{w,K}) as one
// Horner over absolute bit positions q (host_ec.hpp), consumed group by group.
template <class F>
int msm_tail(Ctx* ctx, const MsmTail<F>& t, Xyzz<F>* result) {
  if (t.empty) {
    *result = xyzz_inf<F>();
    return PM_OK;
  }
  const int Wr = t.Wr, NQ = t.NQ, wpg = t.wpg;
  struct {
    int G, base, extra, log2L1, cmax;
  } pl{t.G, t.base, t.extra, t.log2L1, t.cmax};
  const hipStream_t st = t.st, st2 = t.st2;
  const Xyzz<F>* hG = t.hG;
  // the terms as (position, index) sorted by descending position: one flat
  // array (the former vector per position cost ~270 allocations per call)
  std::vector<std::pair<int, int>> terms;
  terms.reserve((size_t)Wr * NQ);
  std::vector<int> gmax(pl.G, -1);  // highest position of any term of group g
  for (int w = 0; w < Wr; w++) {
    const int o = w * pl.base + std::min(w, pl.extra);  // w < Wr: window w's offset (fixed, one set: 0)
    for (int b = 0; b < NQ; b++) {
      // bit folds at o + 2b + log2 L1, sum T at o, the top bucket (K = 2^(cmax-1)) at o + cmax - 1
      const int q = b < NQ - 2 ? o + kBitsFold * b + pl.log2L1 : b == NQ - 2 ? o : o + pl.cmax - 1;
      terms.emplace_back(q, w * NQ + b);
      gmax[w / wpg] = std::max(gmax[w / wpg], q);
    }
  }
  std::sort(terms.begin(), terms.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  });
  host::Pt<F> hacc = host::inf<F>();
  int q = terms.empty() ? 0 : terms.front().first;
  size_t ti = 0;
  double tail_ms = 0.0;
  for (int gi = pl.G - 1; gi >= 0; gi--) {
    HIP_TRY(hipEventSynchronize(t.ev[2 * gi + 1]));
    const auto t0 = std::chrono::steady_clock::now();
    int low = 0;  // positions above every lower group's terms are final now
    for (int gj = 0; gj < gi; gj++) low = std::max(low, gmax[gj] + 1);
    if (host_has_bmi2())
      horner_steps_bmi2<F>(hacc, q, low, ti, terms.data(), terms.size(), hG);
    else
      horner_steps<F>(hacc, q, low, ti, terms.data(), terms.size(), hG);
    tail_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  if (ctx->timing) {
    auto& stt = ctx->stats["host_tail"];
    stt.first += 1;
    stt.second += tail_ms;
  }
  (void)st;
  (void)st2;
  *result = host::to_dev<F>(hacc);
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

// pm_msm_resident_batch: k MSMs of n host scalars each against resident
// bases (halo2's commit of many polynomials against params.g).  Scalars of
// MSM j+1 are copied on the context's copy stream into the second device
// buffer while MSM j's kernels run, and the host Horner of MSM j-1 runs
// while the GPU works on MSM j: in steady state the GPU never waits for
// PCIe or for the host.
template <class Cv>
int msm_resident_batch_impl(Ctx* ctx, const void* d_bases29, const pm_fixed_bases* ft, const uint64_t* const* scalars,
                            size_t k, size_t n, uint32_t flags, uint64_t* out) {
  using F = typename Cv::Base;
  if (k == 0) return PM_OK;
  if (n == 0) {
    std::memset(out, 0, k * 64);
    return PM_OK;
  }
  int rc;
  if ((rc = ctx->in_scalars.ensure(n * 32)) || (rc = ctx->in_scalars2.ensure(n * 32))) return rc;
  if (!ctx->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
  for (int i = 0; i < 4; i++)
    if (!ctx->batch_ev[i]) HIP_TRY(hipEventCreateWithFlags(&ctx->batch_ev[i], hipEventDisableTiming));
  hipEvent_t* copied = ctx->batch_ev;      // [slot]: scalars of the slot's MSM are on the device
  hipEvent_t* consumed = ctx->batch_ev + 2;  // [slot]: the slot's MSM no longer reads its buffer
  void* dbuf[2] = {ctx->in_scalars.p, ctx->in_scalars2.p};
  const hipStream_t st = ctx->stream, cs = ctx->copy_stream;
  auto copy = [&](size_t j) -> int {
    const int sl = (int)(j & 1);
    if (j >= 2) HIP_TRY(hipStreamWaitEvent(cs, consumed[sl], 0));
    HIP_TRY(hipMemcpyAsync(dbuf[sl], scalars[j], n * 32, hipMemcpyHostToDevice, cs));
    HIP_TRY(hipEventRecord(copied[sl], cs));
    return PM_OK;
  };
  MsmTail<F> tails[2];
  const bool overlap = ctx->groups <= 1;
  size_t tailed = 0;
  if ((rc = copy(0))) return rc;
  for (size_t j = 0; j < k; j++) {
    const int sl = (int)(j & 1);
    HIP_TRY(hipStreamWaitEvent(st, copied[sl], 0));
    if ((rc = msm_device_impl<Cv>(ctx, (const uint32_t*)dbuf[sl], (const uint32_t*)d_bases29, n,
                                  ft ? flags : flags | kBasesR261, nullptr, ft, &tails[sl], sl)))
      return rc;
    HIP_TRY(hipEventRecord(consumed[sl], st));
    if (j + 1 < k && (rc = copy(j + 1))) return rc;
    // with window groups (pm_ctx_set_pipeline) the reduction runs on the
    // second stream and would race the next MSM's kernels over the shared
    // workspace: no overlap then, each tail completes before the next MSM
    const size_t done = overlap ? j : j + 1;  // MSMs whose tail can run now
    for (; tailed < done; tailed++) {
      Xyzz<F> r;
      if ((rc = msm_tail<F>(ctx, tails[tailed & 1], &r))) return rc;
      if (!overlap) HIP_TRY(hipStreamSynchronize(ctx->red_stream));
      aff_to_u64<F>(xyzz_to_aff<F>(r), out + 8 * tailed);
    }
  }
  for (; tailed < k; tailed++) {
    Xyzz<F> r;
    if ((rc = msm_tail<F>(ctx, tails[tailed & 1], &r))) return rc;
    aff_to_u64<F>(xyzz_to_aff<F>(r), out + 8 * tailed);
  }
  HIP_TRY(hipStreamSynchronize(cs));
  HIP_TRY(hipStreamSynchronize(ctx->red_stream));
  HIP_TRY(hipStreamSynchronize(st));
  ctx->end_call();
  return PM_OK;
}

// Build a fixed-base table (pm_fixed_bases_create): ft->n, ft->c set by the
// caller; fills W, npad and the device table.
template <class Cv>
int fixed_table_impl(Ctx* ctx, const void* d_bases, pm_fixed_bases* ft) {
  using F = typename Cv::Base;
  const MsmPlan pl = make_plan_fixed(kSortB, ft->c);
  ft->W = pl.W;
  if (ft->rows <= 0) ft->rows = pl.W;
  if (pl.W % ft->rows) return set_error(PM_ERR_ARG, "table rows must divide the window count");
  // windows w and w + W/rows share a bucket set only if their offsets differ
  // by the same amount for every w: equal window widths (256 = W x width)
  if (ft->rows < pl.W && pl.extra)
    return set_error(PM_ERR_ARG, "fewer table rows than windows needs equal window widths (256 % W == 0)");
  ft->npad = std::max<size_t>(kSortB, (ft->n + kSortB - 1) / kSortB * kSortB);
  const size_t bytes = (size_t)ft->rows * ft->npad * 64;
  HIP_TRY(hipMalloc(&ft->d, bytes));
  k_fixed_table<F><<<(unsigned)((ft->npad + 255) / 256), 256, 0, ctx->stream>>>(
      (const uint32_t*)d_bases, (uint32_t)ft->n, (uint32_t)ft->npad, pl.W, pl.base, pl.extra, ft->rows,
      (uint32_t*)ft->d);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

template <class Cv>
int msm_fixed_to_aff(Ctx* ctx, const pm_fixed_bases* ft, const void* d_s, size_t n, uint32_t flags, uint64_t out[8]) {
  using F = typename Cv::Base;
  Xyzz<F> r;
  int rc = msm_device_impl<Cv>(ctx, (const uint32_t*)d_s, nullptr, n, flags, &r, ft);
  if (rc) return rc;
  aff_to_u64<F>(xyzz_to_aff<F>(r), out);
  return PM_OK;
}

// Resident bases (pm_bases_upload*): convert once at upload so every
// pm_msm_resident* call skips k_bases_to_r261 and the bases29 copy.
template <class Cv>
int bases_to29_impl(Ctx* ctx, const void* d_in, size_t n, void* d_out) {
  using F = typename Cv::Base;
  if (n == 0) return PM_OK;
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "more than 2^26 resident bases");
  k_bases_to_r261<F><<<(unsigned)((n + 255) / 256), 256, 0, ctx->stream>>>((const uint32_t*)d_in, (uint32_t)n,
                                                                          (uint32_t*)d_out);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipStreamSynchronize(ctx->stream));
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


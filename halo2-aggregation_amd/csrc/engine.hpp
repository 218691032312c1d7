// engine.hpp -- templated MSM pipeline driver (instantiated once per curve).
//
// Boundary: halo2 `best_multiexp` ([3P], /root/reference/examples/
// simple-example.rs:606,620,638-640,702,722); see include/pasta_msm.h.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>
#include <memory>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>

#include "host_ec.hpp"
#include "msm_kernels.hpp"
#include "msm_small.hpp"
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

// k_sort_hist over blocks [g.blk0, g.blk0 + nb)
template <class Fs, int W>
void launch_sort_w(bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, int nb, uint32_t* bh,
                   void* digits, uint32_t stride, uint32_t merged, hipStream_t st) {
  const size_t lds = (size_t)W * g.NCB * 4;
  if (d16)
    k_sort_hist<Fs, W, true><<<nb, kSortThreads, lds, st>>>(s, n, canonical, g, (uint16_t*)digits, bh, stride,
                                                            merged);
  else
    k_sort_hist<Fs, W, false><<<nb, kSortThreads, lds, st>>>(s, n, canonical, g, (uint32_t*)digits, bh, stride,
                                                             merged);
}

// one instance per window count reachable from c in [kMinC, kMaxC]
template <class Fs>
int launch_sort(int W, bool d16, const uint32_t* s, uint32_t n, uint32_t canonical, SortGeom g, int nb, uint32_t* bh,
                void* digits, uint32_t stride, uint32_t merged, hipStream_t st) {
  switch (W) {
#define PM_W(k) \
  case k: launch_sort_w<Fs, k>(d16, s, n, canonical, g, nb, bh, digits, stride, merged, st); return PM_OK;
    PM_W(13) PM_W(14) PM_W(15) PM_W(16) PM_W(18) PM_W(19) PM_W(20) PM_W(22) PM_W(24) PM_W(26) PM_W(29)
    PM_W(32) PM_W(37) PM_W(43) PM_W(52) PM_W(64)
#undef PM_W
    default: return set_error(PM_ERR_UNSUPPORTED, "window count out of range");
  }
}

// Run the device pipeline of one MSM; result = host XYZZ point.
//
// Sort once, accumulate every bucket set in one launch, then the bucket
// reduction (k_bucket_seg_q, k_bucket_bits) leaves NQ host terms per bucket
// set in the Rust R = 2^256 layout, one D2H copy brings them to a pinned
// slot, and the host evaluates sum_w 2^{o_w} (...) as one Horner over
// absolute bit positions (msm_tail).
//
// Fixed-base mode (ft != nullptr, pm_msm_fixed and the resident row
// tables): the bases are a precomputed table ft->d with entry j * npad + i =
// [2^{o_{j Wr}}] P_i (k_fixed_table), so the digits of windows w, w + Wr, ...
// index ONE bucket set (kmerge = rows windows per set, Wr = W / rows sets):
// the sort runs over kmerge * npad entries per set (merged histogram rows),
// and the reduction and host tail handle Wr sets only.
//
// Host terms per bucket set (NQ = NB2 + kTJobs + 1): the bit sums G_b at
// o + b + log2 L1, the kTJobs partial sums of T at o, the top bucket K at
// o + cmax - 1.
template <class F>
struct MsmTail {
  int Wr = 0, NQ = 0, NB2 = 0, base = 0, extra = 0, log2L1 = 0, cmax = 0;
  bool empty = true;
  const Xyzz<F>* hQ = nullptr;  // pinned host slot
  hipEvent_t ev = nullptr;      // recorded after the slot's D2H copy
};

template <class F>
int msm_tail(Ctx* ctx, const MsmTail<F>& t, Xyzz<F>* result);

// Enqueue the device pipeline of one MSM (everything up to the D2H copy of
// its host terms into pinned slot `slot`) and describe its host tail in
// *tail; msm_tail then waits for it and runs the Horner.  Two MSMs can be in
// flight (slots 0 and 1): the tail of one overlaps the kernels of the next
// (pm_msm_resident_batch).  tail == nullptr: run the tail here.
//
// h_scalars != nullptr: the scalars are still in (pageable) host memory and
// d_scalars is their device buffer; they are copied ahead of the sort.
template <class Cv>
int msm_device_impl(Ctx* ctx, const uint32_t* d_scalars, const uint32_t* d_bases, size_t n, uint32_t flags,
                    Xyzz<typename Cv::Base>* result, const pm_fixed_bases* ft = nullptr,
                    MsmTail<typename Cv::Base>* tail = nullptr, int slot = 0, const void* h_scalars = nullptr) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  if (n == 0) {
    if (tail) *tail = MsmTail<F>{};
    else *result = xyzz_inf<F>();
    return PM_OK;
  }
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "n exceeds 2^26 points per device call");
  const bool fixed = ft != nullptr;
  // pre29: resident bases already in the pipeline's R = 2^261 form (pm_bases)
  const bool pre29 = !fixed && (flags & kBasesR261) != 0;
  const MsmPlan pl = fixed ? make_plan_fixed(ft->npad, ft->c, ctx->min_chunk)
                           : make_plan(n, ctx->window_c, ctx->min_chunk);
  const hipStream_t st = ctx->stream;
  const int kmerge = fixed ? ft->rows : 1;
  const int Wr = pl.W / kmerge;                     // bucket sets (reduced windows)
  const size_t TOT = (size_t)Wr * pl.NB + 1;
  const int NJ = pl.NB2 + kTJobs;                   // bit-sum jobs per set
  const int NQ = NJ + 1;                            // host terms per set
  const bool d16 = pl.cmax <= 16;
  // Split scalar copy (round 6): a row-table MSM with scalars in host memory
  // sorts and accumulates a first part of its points while the rest of the
  // scalars cross PCIe.  A pageable hipMemcpyAsync blocks the calling thread
  // for the whole copy but overlaps kernels on other streams
  // (tools/h2d_overlap.hip: 32 MB in 0.60 ms, 2 x 16 MB 0.62, a 0.45 ms kernel
  // meanwhile hidden), so: copy part 0 on the context stream (blocks), queue
  // its sort and accumulation there, copy part 1 on the copy stream (blocks
  // while part 0 runs), then queue part 1's sort and accumulation on the
  // context stream behind an event of that copy, and one bucket reduction
  // over both sorted lists (k_bucket_seg_q<F, 2>).  Part 1's kernels stay on
  // the context stream: beside part 0's accumulation on a queue of their own
  // they only slowed it (sort 0.10 -> 0.27 ms, accumulation 0.49 -> 0.52,
  // same end; rocprofv3 trace, round 6).  Each part is sorted as a table of
  // its own points (digit rows of its padded length) and k_sort_coarse
  // writes the full table's indices.
  const int nch = fixed && h_scalars && ctx->msm_split_copy != 0 && n >= kSplitCopyMinN
                      ? (n >= kSplitCopy3MinN ? 3 : 2) : 1;
  // Two parts: the first is 3/8 of the points -- its copy is the exposed one,
  // and the second part's copy (5/8) still ends before the first part's sort
  // and accumulation do (2^20 with host scalars: 1/2 1.61 ms, 5/16
  // 1.57-1.58, 3/8 1.57, 7/16 1.64; 2^22: 3/8 5.68 ms, 1/2 6.00 ms, one copy
  // 7.3-7.4).  Three parts (1/4, 3/8, 3/8) from kSplitCopy3MinN points: the
  // exposed copy shrinks with n while each extra part costs a fixed sort
  // (~0.04 ms) and chain fold (2^20: 1.64-1.68 ms against 1.59-1.62 with two;
  // 2^22: 5.25-5.32 against 5.63-5.66; profiles/r06/split_copy_ab.jsonl)
  // part starts (multiples of kSortB): two parts 3/8 + 5/8, three 1/4 + 3/8 + 3/8
  size_t pstart[kMaxParts + 1] = {0, n, n, n};
  auto rnd = [](size_t v) { return (v + kSortB - 1) / kSortB * kSortB; };
  if (nch == 2) pstart[1] = rnd(n * 3 / 8);
  if (nch == 3) {
    pstart[1] = rnd(n / 4);
    pstart[2] = rnd(n * 5 / 8);
  }
  pstart[nch] = n;
  int rc;
  if ((rc = ctx->segS.ensure((size_t)Wr * pl.M1 * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->segT.ensure((size_t)Wr * pl.M1 * sizeof(Xyzz<F>)))) return rc;
  if ((rc = ctx->bitsQ.ensure((size_t)Wr * NQ * sizeof(Xyzz<F>)))) return rc;
  const size_t nQ = (size_t)Wr * NQ;
  if ((rc = ctx->ensure_pinned(2 * nQ * sizeof(Xyzz<F>)))) return rc;  // two slots (batch pipelining)
  if ((rc = ctx->ensure_group_events(2))) return rc;
  Xyzz<F>* hslot = (Xyzz<F>*)ctx->h_pinned + (size_t)slot * nQ;
  Xyzz<F>* S = (Xyzz<F>*)ctx->segS.p;
  Xyzz<F>* T = (Xyzz<F>*)ctx->segT.p;
  // host terms: the reduction kernels store them straight into the pinned
  // slot (mapped; visible to the host once the event below completes), which
  // saves the blit of a D2H copy (~11 us per MSM, profiles/r03/kernel_stats.csv
  // __amd_rocclr_copyBuffer; the copy measured within noise on the headline
  // and 24 us slower on the variable-base path, profiles/r03/ab/).
  Xyzz<F>* Qd = (Xyzz<F>*)ctx->h_pinned_dev + (size_t)slot * nQ;
  const uint32_t un = (uint32_t)n;

  // bases -> R261 once per MSM.  Running it on a second stream beside the
  // sort measured no faster: both are memory bound (bases 0.04 -> 0.07 ms,
  // histogram 0.048 -> 0.082 ms concurrently).
  const uint32_t* bases29;
  if (fixed) {
    bases29 = (const uint32_t*)ft->d;
  } else if (pre29) {
    bases29 = d_bases;
  } else {
    if ((rc = ctx->bases29.ensure(n * 64))) return rc;
    bases29 = (const uint32_t*)ctx->bases29.p;
    PM_LAUNCH(ctx, "bases_r261",
              (k_bases_to_r261<F><<<(un + 255) / 256, 256, 0, st>>>(d_bases, un, (uint32_t*)ctx->bases29.p)));
  }
  const uint32_t canon = (flags & PM_SCALARS_CANONICAL) ? 1u : 0u;
  SegChunks<F> co = {};
  if (nch > 1) {  // the copy stream starts behind everything queued on the context stream
    if (!ctx->copy_stream) HIP_TRY(hipStreamCreateWithFlags(&ctx->copy_stream, hipStreamNonBlocking));
    hipEvent_t ev0 = ctx->next_event();
    if (!ev0) return set_error(PM_ERR_HIP, "hipEventCreate failed");
    HIP_TRY(hipEventRecord(ev0, st));
    HIP_TRY(hipStreamWaitEvent(ctx->copy_stream, ev0, 0));
  }
  // sort geometry of a digit row length (the whole MSM's, or a part's)
  struct PartGeom {
    size_t E, nW, TOTB;
    SortGeom g, gm;
    ScanTiles tiles;
    uint32_t nb;
    bool wide;
  };
  auto geom = [&](size_t stride) {
    PartGeom r{};
    r.E = (size_t)kmerge * stride;  // entries of one sort row
    r.nW = (size_t)stride * pl.W;
    SortGeom& g = r.g;  // histogram geometry (blocks of scalars)
    g.FB = std::max(0, pl.cmax - 1 - 8);
    // the fixed-base MSM's merged sort rows are W x longer: 4x more coarse bins
    // once they exceed 2^24 entries (2^23, c = 20: FB 11 -> 9, sort 3.4 -> 2.3 ms)
    if (fixed && r.E > (size_t(1) << 24)) g.FB = std::max(0, pl.cmax - 1 - 10);
    g.NCB = (pl.K >> g.FB) + 1;
    // points per thread: blocks of 1024 threads x ppt points, ppt the largest
    // power of two <= 8 that still gives >= 128 blocks (2^20: 8192 points per
    // block; larger blocks give longer contiguous runs per coarse bin in
    // k_sort_coarse and a 4x smaller block histogram to scan: sort 0.19 ->
    // 0.16 ms at 2^20; small n keeps enough blocks)
    g.ppt = 1;
    while (g.ppt < kSortPerThread && stride >= (size_t)256 * g.ppt * kSortThreads) g.ppt *= 2;
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
    if (g.ppt >= 2 && g.nblk >= 128 && g.nblk < 256) hsub = 2;
    g.hsub = 1;
    r.gm = g;         // coarse / fine geometry (blocks of sort-row entries)
    g.ppt /= hsub;    // histogram geometry
    g.nblk *= hsub;
    r.gm.nblk = g.nblk * kmerge;
    r.gm.hsub = hsub;
    r.TOTB = (size_t)pl.W * g.NCB * g.nblk + 1;
    r.tiles = scan_tiles((uint32_t)(pl.W * g.NCB), (uint32_t)g.nblk);  // k_sort_hist's layout
    r.nb = (uint32_t)((r.TOTB + r.tiles.chunk - 1) / r.tiles.chunk);
    // 4-B coarse entries when the entry index fits beside the fine bits and
    // the sign (a part's entries carry the full table's indices)
    const size_t imax = nch > 1 ? (size_t)kmerge * ft->npad : r.E;
    r.wide = imax > (size_t(1) << (31 - g.FB));
    return r;
  };
  // digit row length: n, the table's padded rows, or a part's own padded length
  auto part_stride = [&](int ch) -> size_t {
    return !fixed ? n : nch > 1 ? std::max<size_t>(kSortB, rnd(pstart[ch + 1] - pstart[ch])) : ft->npad;
  };
  // the sort scratch, shared by the parts (their kernels run in stream order),
  // sized for the largest before anything is queued
  for (int ch = 0; ch < nch; ch++) {
    const PartGeom q = geom(part_stride(ch));
    if ((rc = ctx->digits.ensure(q.nW * (d16 ? 2 : 4)))) return rc;
    if ((rc = ctx->mid.ensure(q.nW * (q.wide ? 8 : 4)))) return rc;
    if ((rc = ctx->counts.ensure(q.TOTB * 4))) return rc;
    if ((rc = ctx->cursor.ensure(q.TOTB * 4))) return rc;
    if ((rc = ctx->bsum.ensure((size_t)q.nb * 4))) return rc;
  }
  for (int ch = 0; ch < nch; ch++) {
    const hipStream_t cs = st;
    const size_t c0 = pstart[ch], nc = pstart[ch + 1] - c0;
    const size_t stride = part_stride(ch);
    const PartGeom q = geom(stride);
    const size_t E = q.E, nW = q.nW, TOTB = q.TOTB;
    SortGeom g = q.g;
    SortGeom gm = q.gm;
    const ScanTiles tiles = q.tiles;
    const uint32_t nb = q.nb;
    const bool wide = q.wide;
    // a part's entries carry table indices j npad + c0 + i (k_sort_coarse)
    gm.rstride = (uint32_t)stride;
    gm.rdelta = nch > 1 ? (uint32_t)(ft->npad - stride) : 0u;
    gm.roff = nch > 1 ? (uint32_t)c0 : 0u;
    // each part keeps its sorted list and bucket partials for the reduction
    Buf& b_digits = ctx->digits;
    Buf& b_mid = ctx->mid;
    Buf& b_counts = ctx->counts;
    Buf& b_cursor = ctx->cursor;
    Buf& b_bsum = ctx->bsum;
    Buf& b_sorted = ch ? ctx->part_sorted[ch - 1] : ctx->sorted;
    Buf& b_offsets = ch ? ctx->part_offsets[ch - 1] : ctx->offsets;
    Buf& b_buckets = ch ? ctx->part_buckets[ch - 1] : ctx->buckets;
    Buf& b_head = ch ? ctx->part_head[ch - 1] : ctx->head;
    // accumulation lanes: each part's own plan (~4 waves per SIMD; a part's
    // buckets reach as many slices as a full sort's).  The whole MSM's slice
    // length instead (fewer lanes, shorter chains) measured the same with
    // equal halves and 0.17 ms slower with a 3/8 first part (1.5 waves per
    // SIMD in its accumulation)
    const uint32_t chunk = nch > 1 ? make_plan_fixed(stride, ft->c, ctx->min_chunk).chunk : pl.chunk;
    const uint32_t nthreads = nch > 1 ? (uint32_t)((nW + chunk - 1) / chunk) : pl.nthreads;
    if ((rc = b_sorted.ensure(nW * 4))) return rc;
    if ((rc = b_offsets.ensure(TOT * 4))) return rc;
    if ((rc = b_buckets.ensure((size_t)Wr * pl.NB * sizeof(Xyzz<F>)))) return rc;
    if ((rc = b_head.ensure((size_t)nthreads * sizeof(Xyzz<F>)))) return rc;

    uint32_t* sorted = (uint32_t*)b_sorted.p;
    void* mid = b_mid.p;
    uint32_t* bh = (uint32_t*)b_counts.p;
    uint32_t* bofs = (uint32_t*)b_cursor.p;
    uint32_t* offsets = (uint32_t*)b_offsets.p;
    uint32_t* bsum = (uint32_t*)b_bsum.p;
    Xyzz<F>* buckets = (Xyzz<F>*)b_buckets.p;
    Xyzz<F>* head = (Xyzz<F>*)b_head.p;
    g.clr_bh = bh + (TOTB - 1);  // zeroed by the histogram kernel's block 0
    const uint32_t* sc = d_scalars + 8 * c0;
    const uint32_t unc = (uint32_t)nc;
    if (h_scalars) {
      // one pageable copy ahead of this part's histogram pass (without the
      // split: a copy in 4 chunks, each chunk's histogram blocks launched
      // behind it, measured ~0.1 ms slower per 2^20 MSM: round 3,
      // profiles/r03/h2d/)
      const hipStream_t xs = ch == 0 ? st : ctx->copy_stream;
      if ((rc = ctx->upload_h2d((void*)sc, (const uint8_t*)h_scalars + 32 * c0, nc * 32, xs))) return rc;
      if (ch > 0) {
        hipEvent_t evc = ctx->next_event();
        if (!evc) return set_error(PM_ERR_HIP, "hipEventCreate failed");
        HIP_TRY(hipEventRecord(evc, xs));
        HIP_TRY(hipStreamWaitEvent(st, evc, 0));
      }
    }
    PM_LAUNCH_ST(ctx, cs, "sort_hist", rc = launch_sort<Fs>(pl.W, d16, sc, unc, canon, g, g.nblk, bh, b_digits.p,
                                                            (uint32_t)stride, (uint32_t)kmerge, cs));
    if (rc) return rc;
    PM_LAUNCH_ST(ctx, cs, "scan", {
      k_scan_reduce<<<nb, kScanThreads, 0, cs>>>(bh, (uint32_t)TOTB, tiles, bsum);
      k_scan_down<<<nb, kScanThreads, 0, cs>>>(bh, (uint32_t)TOTB, tiles, bsum, bofs, nullptr);
    });
    {
      const size_t lds = (size_t)gm.ppt * kSortThreads * ((wide ? 8 : 4) + 2) + (size_t)(2 * g.NCB + 1) * 4 + (kSortThreads / 64 + 1) * 4;
      const dim3 grid(gm.nblk / gm.hsub, Wr);
      void* dg = b_digits.p;
      const uint32_t ue = (uint32_t)E;
      if (d16 && !wide)
        PM_LAUNCH_ST(ctx, cs, "sort_coarse", launch_coarse<true, false>(dg, ue, gm, bofs, mid, grid, lds, cs));
      else if (d16)
        PM_LAUNCH_ST(ctx, cs, "sort_coarse", launch_coarse<true, true>(dg, ue, gm, bofs, mid, grid, lds, cs));
      else if (!wide)
        PM_LAUNCH_ST(ctx, cs, "sort_coarse", launch_coarse<false, false>(dg, ue, gm, bofs, mid, grid, lds, cs));
      else
        PM_LAUNCH_ST(ctx, cs, "sort_coarse", launch_coarse<false, true>(dg, ue, gm, bofs, mid, grid, lds, cs));
    }
    // fine sort LDS: segment cache + chunk buffer (k_sort_fine).  A mean
    // segment that fits 24 KiB is cached whole with room for 1.5x its size and
    // sorted as one chunk; larger ones are re-read from mid in 32 KiB chunks
    // (2 blocks per CU).  Sweep with 16-B loads (profiles/r03/sort_fine/): 16
    // KiB chunks 2^20 0.065 / 2^22 0.233 ms, 24-32 KiB 0.056 / 0.210, 40-64 KiB
    // (one block per CU) 0.064-0.074 / 0.256-0.288; the whole segment cached in
    // LDS (64-136 KiB) 0.069-0.107 / 0.34-0.44.  PM_FINE_CACHE_KB /
    // PM_FINE_CHUNK_KB override both (A/B).
    const size_t esz = wide ? 8 : 4;
    const size_t mean_seg = E / std::max(1, g.NCB - 1) + 1;
    const size_t fine_fixed = ((size_t)3 * (1 << g.FB) + kFineThreads / 64 + 1) * 4;  // hist, lcur, lst, scan
    size_t cache_n = (mean_seg * 3 / 2 + 63) & ~size_t(63), chn;
    if (cache_n * esz > 24576) cache_n = kFineChunkBytes / esz;
    chn = cache_n;
    if (ctx->fine_cache_kb > 0) cache_n = ((size_t)ctx->fine_cache_kb * 1024 / esz) & ~size_t(63);
    if (ctx->fine_chunk_kb > 0) chn = ((size_t)ctx->fine_chunk_kb * 1024 / esz) & ~size_t(63);
    chn = std::max<size_t>(64, std::min(chn, cache_n));
    cache_n = std::max(cache_n, chn);
    if (fine_fixed + 128 * esz > kMaxLds) return set_error(PM_ERR_UNSUPPORTED, "sort: fine bits too wide");
    while (cache_n > 64 && (cache_n + chn) * esz + fine_fixed > kMaxLds) {
      cache_n /= 2;
      chn = std::min(chn, cache_n);
    }
    const size_t lds_fine = (cache_n + chn) * esz + fine_fixed;
    if (wide)
      PM_LAUNCH_ST(ctx, cs, "sort_fine", (k_sort_fine<true><<<Wr * g.NCB, kFineThreads, lds_fine, cs>>>(
                                            (const uint64_t*)mid, bofs, gm, Wr, pl.NB, (uint32_t)cache_n, (uint32_t)chn,
                                            offsets, sorted)));
    else
      PM_LAUNCH_ST(ctx, cs, "sort_fine", (k_sort_fine<false><<<Wr * g.NCB, kFineThreads, lds_fine, cs>>>(
                                            (const uint32_t*)mid, bofs, gm, Wr, pl.NB, (uint32_t)cache_n, (uint32_t)chn,
                                            offsets, sorted)));
    const uint32_t s1 = (uint32_t)((size_t)Wr * pl.NB);
    PM_LAUNCH_ST(ctx, cs, "accumulate",
                 (k_accumulate<F><<<(nthreads + 255) / 256, 256, 0, cs>>>(sorted, offsets, s1, bases29, chunk,
                                                                          buckets, head)));
    co.c[ch] = SegChunk<F>{offsets, chunk, nthreads, buckets, head};
  }
  // chains (long ones wave-cooperatively) + segment sums + the top bucket
  const unsigned seg_blocks = (unsigned)((4ull * Wr * pl.M1 + 255) / 256);
  if (nch == 3)
    PM_LAUNCH(ctx, "bucket_seg", (k_bucket_seg_q<F, 3><<<seg_blocks, 256, 0, st>>>(co, Wr, pl.NB, (uint32_t)pl.M1, S, T,
                                                                                   Qd, NQ)));
  else if (nch == 2)
    PM_LAUNCH(ctx, "bucket_seg", (k_bucket_seg_q<F, 2><<<seg_blocks, 256, 0, st>>>(co, Wr, pl.NB, (uint32_t)pl.M1, S, T,
                                                                                   Qd, NQ)));
  else
    PM_LAUNCH(ctx, "bucket_seg", (k_bucket_seg_q<F, 1><<<seg_blocks, 256, 0, st>>>(co, Wr, pl.NB, (uint32_t)pl.M1, S, T,
                                                                                   Qd, NQ)));
  // bit sums of few sets (the row tables, the fixed-base MSM's one set) are
  // split over more blocks.  Every extra lane also adds one tree addition, so
  // the split stops at ~16 blocks per job (c = 20, 2^19 buckets: 16 -> 0.33
  // ms, 64 -> 0.47 ms; round 3, 16 / Wr against 4, 8, 32, 64 / Wr at 2^19 -
  // 2^22, resident and raw: profiles/r03/ab/bits_split_sweep.jsonl).
  const int nsplit = std::max(1, std::min(kMaxSplit, kBitsSplitK / Wr));
  Xyzz<F>* bitsP = nullptr;
  uint32_t* tickets = nullptr;
  if (nsplit > 1) {
    if ((rc = ctx->bitsP.ensure((size_t)Wr * NJ * nsplit * sizeof(Xyzz<F>)))) return rc;
    const size_t old_cap = ctx->tickets.cap;  // tickets are self-resetting; zero fresh allocations
    if ((rc = ctx->tickets.ensure((size_t)Wr * NJ * 4))) return rc;
    if (ctx->tickets.cap != old_cap) HIP_TRY(hipMemsetAsync(ctx->tickets.p, 0, ctx->tickets.cap, st));
    bitsP = (Xyzz<F>*)ctx->bitsP.p;
    tickets = (uint32_t*)ctx->tickets.p;
  }
  PM_LAUNCH(ctx, "bucket_bits",
            (k_bucket_bits<F><<<dim3(NJ, Wr, nsplit), kRedThreads, 0, st>>>(S, T, pl.M1, pl.NB2, Qd, NQ, nsplit,
                                                                             bitsP, tickets)));
  hipEvent_t ev = ctx->grp_ev[slot];
  HIP_TRY(hipEventRecord(ev, st));
  MsmTail<F> t;
  t.Wr = Wr;
  t.NQ = NQ;
  t.NB2 = pl.NB2;
  t.base = pl.base;
  t.extra = pl.extra;
  t.log2L1 = pl.log2L1;
  t.cmax = pl.cmax;
  t.empty = false;
  t.hQ = hslot;
  t.ev = ev;
  if (tail) {
    *tail = t;
    return PM_OK;
  }
  if ((rc = msm_tail<F>(ctx, t, result))) return rc;
  // msm_tail waited for the event recorded after the terms' copy, which
  // follows all of this MSM's work: nothing is pending on the stream.  A
  // hipStreamSynchronize here still cost ~16 us per call (profiles/r02/htr/),
  // GPU idle before the next call.
  ctx->end_call();
  return PM_OK;
}

// The Horner steps q = hi .. 0: one doubling per position, then the terms at
// that position.  Two builds: on a CPU with BMI2 / ADX the field products are
// host::mul_adx (mulx with two carry chains); the dispatch checks the CPU once.
template <class F>
inline void horner_steps(host::Pt<F>& hacc, int q, const std::pair<int, int>* terms, size_t nterms,
                         const Xyzz<F>* hQ) {
  size_t ti = 0;
  for (; q >= 0; q--) {
    hacc = host::dbl<F>(hacc);
    for (; ti < nterms && terms[ti].first == q; ti++) hacc = host::addp<F>(hacc, host::from_dev<F>(hQ[terms[ti].second]));
  }
}
template <class F>
__attribute__((target("bmi2,adx"))) void horner_steps_bmi2(host::Pt<F>& hacc, int q,
                                                           const std::pair<int, int>* terms, size_t nterms,
                                                           const Xyzz<F>* hQ) {
  size_t ti = 0;
  for (; q >= 0; q--) {
    hacc = host::dbl<F, true>(hacc);
    for (; ti < nterms && terms[ti].first == q; ti++)
      hacc = host::addp<F, true>(hacc, host::from_dev<F>(hQ[terms[ti].second]));
  }
}

// Host tail with many bucket sets (Wr >= kTailSplitSets: the variable-base
// MSM's 16 windows): the one Horner over 256 positions costs ~256 additions
// on one core (0.157 ms at 2^20, profiles/r04/bench_r04b.json; split: 0.072
// ms, bench_r04d.json).  With the 4-row tables' 4 sets the split measured
// slower (2^22: 0.047 against 0.040 ms), so it starts at 8 sets.
// Instead each set's V_w = sum_b 2^{rel_b} Q_{w,b} (rel_b < cmax) is a short
// Horner on a pool thread, and the caller runs the outer Horner
// sum_w 2^{o_w} V_w from the top set down in Jacobian form (host_ec.hpp jdbl),
// waiting for each V_w only when the chain reaches it.
constexpr int kTailSplitSets = 8;
template <class F, bool ADX>
host::Pt<F> tail_set(const MsmTail<F>& t, int w) {
  // terms of set w by descending relative position: bit sums b + log2 L1,
  // the top bucket at cmax - 1, the T partials at 0
  host::Pt<F> acc = host::inf<F>();
  int q = t.cmax - 1;
  if (t.NB2 - 1 + t.log2L1 > q) q = t.NB2 - 1 + t.log2L1;
  const Xyzz<F>* Q = t.hQ + (size_t)w * t.NQ;
  for (; q >= 0; q--) {
    acc = host::dbl<F, ADX>(acc);
    const int b = q - t.log2L1;
    if (b >= 0 && b < t.NB2) acc = host::addp<F, ADX>(acc, host::from_dev<F>(Q[b]));
    if (q == t.cmax - 1) acc = host::addp<F, ADX>(acc, host::from_dev<F>(Q[t.NQ - 1]));
    if (q == 0)
      for (int b2 = t.NB2; b2 < t.NQ - 1; b2++) acc = host::addp<F, ADX>(acc, host::from_dev<F>(Q[b2]));
  }
  return acc;
}
// Sets are claimed, not assigned: a worker takes the next unclaimed set from
// the top (shared counter + per-set claim), and the caller computes a set
// itself when the chain reaches it unclaimed -- so a worker that wakes late
// (condition-variable wake-ups take ~10-20 us) delays nothing; the caller
// waits only for a set already in progress on a worker.
template <class F, bool ADX>
host::Pt<F> tail_split(HostPool& pool, const MsmTail<F>& t) {
  const int Wr = t.Wr;
  std::vector<host::Pt<F>> V((size_t)Wr);
  std::unique_ptr<std::atomic<int>[]> state(new std::atomic<int>[(size_t)Wr]);  // 0 free, 1 claimed, 2 ready
  for (int w = 0; w < Wr; w++) state[w].store(0, std::memory_order_relaxed);
  std::atomic<int> next(Wr - 2);
  auto run = [&](int w) {
    V[(size_t)w] = tail_set<F, ADX>(t, w);
    state[w].store(2, std::memory_order_release);
  };
  auto claim = [&](int w) {
    int z = 0;
    return state[w].compare_exchange_strong(z, 1, std::memory_order_acq_rel);
  };
  const int nt = std::min(pool.size(), Wr);
  auto job = [&](int, int) {
    for (int w = next.fetch_sub(1, std::memory_order_relaxed); w >= 0; w = next.fetch_sub(1, std::memory_order_relaxed))
      if (claim(w)) run(w);
  };
  if (nt > 1) pool.start(nt, job);
  state[Wr - 1].store(1, std::memory_order_relaxed);
  run(Wr - 1);  // the caller: the top set now, then the outer chain
  auto jac = [](const host::Pt<F>& p) {  // XYZZ (ZZ^3 = ZZZ^2) -> Jacobian (X ZZ^2, Y ZZZ^2, ZZZ)
    host::Jac<F> r;
    if (host::is_zero(p.ZZ)) {
      std::memset(&r, 0, sizeof(r));
      return r;
    }
    r.X = host::mulv<F, ADX>(p.X, host::mulv<F, ADX>(p.ZZ, p.ZZ));
    r.Y = host::mulv<F, ADX>(p.Y, host::mulv<F, ADX>(p.ZZZ, p.ZZZ));
    r.Z = p.ZZZ;
    return r;
  };
  host::Jac<F> acc = jac(V[(size_t)Wr - 1]);
  for (int w = Wr - 2; w >= 0; w--) {
    const int width = t.base + (w < t.extra ? 1 : 0);  // o_{w+1} - o_w
    for (int k = 0; k < width; k++) acc = host::jdbl<F, ADX>(acc);
    if (claim(w)) run(w);
    while (state[w].load(std::memory_order_acquire) != 2) __builtin_ia32_pause();
    acc = host::jadd<F, ADX>(acc, jac(V[(size_t)w]));
  }
  if (nt > 1) pool.wait();
  if (host::is_zero(acc.Z)) return host::inf<F>();
  return host::jac_to_xyzz<F, ADX>(acc);
}
template <class F>
__attribute__((target("bmi2,adx"))) host::Pt<F> tail_split_bmi2(HostPool& pool, const MsmTail<F>& t) {
  return tail_split<F, true>(pool, t);
}

// The single Horner over absolute bit positions (fewer than kTailSplitSets
// sets): tail_terms lists the terms as (position, index) sorted by descending
// position, one flat array (a vector per position cost ~270 allocations per
// call; msm_tail builds it while the kernels still run), tail_run evaluates.
template <class F>
std::vector<std::pair<int, int>> tail_terms(const MsmTail<F>& t) {
  std::vector<std::pair<int, int>> terms;
  terms.reserve((size_t)t.Wr * t.NQ);
  for (int w = 0; w < t.Wr; w++) {
    const int o = w * t.base + std::min(w, t.extra);  // w < Wr: set w's offset
    for (int b = 0; b < t.NQ; b++) {
      const int q = b < t.NB2 ? o + b + t.log2L1 : b < t.NQ - 1 ? o : o + t.cmax - 1;
      terms.emplace_back(q, w * t.NQ + b);
    }
  }
  std::sort(terms.begin(), terms.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  });
  return terms;
}
template <class F>
host::Pt<F> tail_run(const MsmTail<F>& t, const std::vector<std::pair<int, int>>& terms) {
  host::Pt<F> hacc = host::inf<F>();
  const int q = terms.front().first;
  if (host_has_bmi2())
    horner_steps_bmi2<F>(hacc, q, terms.data(), terms.size(), t.hQ);
  else
    horner_steps<F>(hacc, q, terms.data(), terms.size(), t.hQ);
  return hacc;
}

// Host tail: sum_w 2^{o_w} (sum_b 2^{b + log2 L1} G_{w,b} + sum T_w + K B_{w,K})
// as one Horner over absolute bit positions q (host_ec.hpp), or split by set
// (tail_split) when there are many sets.
template <class F>
int msm_tail(Ctx* ctx, const MsmTail<F>& t, Xyzz<F>* result) {
  if (t.empty) {
    *result = xyzz_inf<F>();
    return PM_OK;
  }
  if (t.Wr >= kTailSplitSets) {
    if (int rc = wait_event(ctx, t.ev)) return rc;
    const auto t0 = std::chrono::steady_clock::now();
    const host::Pt<F> r = host_has_bmi2() ? tail_split_bmi2<F>(ctx->host_pool(), t)
                                          : tail_split<F, false>(ctx->host_pool(), t);
    if (ctx->timing) {
      auto& stt = ctx->stats["host_tail"];
      stt.first += 1;
      stt.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    }
    *result = host::to_dev<F>(r);
    return PM_OK;
  }
  const std::vector<std::pair<int, int>> terms = tail_terms<F>(t);
  if (int rc = wait_event(ctx, t.ev)) return rc;
  const auto t0 = std::chrono::steady_clock::now();
  const host::Pt<F> hacc = tail_run<F>(t, terms);
  if (ctx->timing) {
    auto& stt = ctx->stats["host_tail"];
    stt.first += 1;
    stt.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
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
int msm_device_to_aff(Ctx* ctx, const void* d_s, const void* d_b, size_t n, uint32_t flags, uint64_t out[8],
                      const void* h_s) {
  using F = typename Cv::Base;
  Xyzz<F> r;
  int rc = msm_device_impl<Cv>(ctx, (const uint32_t*)d_s, (const uint32_t*)d_b, n, flags, &r, nullptr, nullptr, 0, h_s);
  if (rc) return rc;
  aff_to_u64<F>(xyzz_to_aff<F>(r), out);
  return PM_OK;
}

// the two halves of a resident-bases MSM (CurveOps::msm_start / msm_finish)
template <class Cv>
int msm_start_impl(Ctx* ctx, const pm_fixed_bases* ft, const void* d_bases29, const void* d_s, size_t n,
                   uint32_t flags, void* tail, const void* h_s) {
  using F = typename Cv::Base;
  static_assert(sizeof(MsmTail<F>) <= kTailBytes, "tail storage");
  MsmTail<F>* t = new (tail) MsmTail<F>();
  return msm_device_impl<Cv>(ctx, (const uint32_t*)d_s, (const uint32_t*)d_bases29, n,
                             ft ? flags & ~kBasesR261 : flags | kBasesR261, nullptr, ft, t, 0, h_s);
}
template <class Cv>
int msm_finish_impl(Ctx* ctx, const void* tail, uint64_t out[8]) {
  using F = typename Cv::Base;
  Xyzz<F> r;
  if (int rc = msm_tail<F>(ctx, *(const MsmTail<F>*)tail, &r)) return rc;
  ctx->end_call();
  aff_to_u64<F>(xyzz_to_aff<F>(r), out);
  return PM_OK;
}

// ------------------------------------------------------ small-MSM path
// Host Horner over the 33 window sums of msm_small.hpp (Jacobian, X Y Z in
// the first three coordinates of each slot): 128 doublings, 32 additions.
template <class F, bool ADX>
inline host::Pt<F> small_horner(const Xyzz<F>* W) {
  auto jac = [&](int j) {
    host::Jac<F> r;
    std::memcpy(&r, &W[j], sizeof(r));
    return r;
  };
  host::Jac<F> acc = jac(kSmallWin - 1);
  for (int j = kSmallWin - 2; j >= 0; j--) {
    for (int k = 0; k < 4; k++) acc = host::jdbl<F, ADX>(acc);
    acc = host::jadd<F, ADX>(acc, jac(j));
  }
  if (host::is_zero(acc.Z)) return host::inf<F>();
  return host::jac_to_xyzz<F, ADX>(acc);
}
template <class F>
__attribute__((target("bmi2,adx"))) host::Pt<F> small_horner_bmi2(const Xyzz<F>* W) {
  return small_horner<F, true>(W);
}

// n <= ctx->small_max: k_small_fused (2n <= 64 terms) or k_small_table +
// k_small_sum (msm_small.hpp), then the host Horner.  Host inputs are copied
// into a pinned mapped buffer that the first kernel reads directly (no DMA
// copy and its launch latency); the 33 window sums land in mapped host
// memory (no D2H copy), and the host spins on the completion flag the last
// window raises instead of waiting for the kernel's completion signal
// (falling back to the stream's event, which also surfaces a failed launch).
template <class Cv>
int msm_small_impl(Ctx* ctx, const void* scalars, bool s_host, const void* bases, bool b_host, bool b_r261, size_t n,
                   uint32_t flags, uint64_t out[8]) {
  using F = typename Cv::Base;
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  if (n > kSmallLimit) return set_error(PM_ERR_UNSUPPORTED, "small-MSM path: n above its limit");
  const hipStream_t st = ctx->stream;
  const uint32_t un = (uint32_t)n, T = 2u * un;
  const bool fused = un <= kSmallFusedN;
  // slices per window: up to kSmallSlices blocks of 64 quads (or, from 4096
  // terms, 256 lanes with one-lane additions), each adding kq terms serially.
  // Measured (profiles/r04/small/ab.jsonl, n = 256 .. 8192, quads / lanes x
  // 4 .. 32 slices): 8 slices best at every size, lanes ahead from n = 2048
  // (121 vs 132 us; 4096: 138 vs 167 us), even at 1024.
  constexpr uint32_t kSmallSlices = 8;
  const bool lanes = T >= 4096u;
  const uint32_t per = lanes ? 256u : (uint32_t)kSmallQuads;  // terms per block and round
  SmallGeom g{};
  g.n = un;
  g.canonical = (flags & PM_SCALARS_CANONICAL) ? 1u : 0u;
  g.r261 = b_r261 ? 1u : 0u;
  g.kq = std::max<uint32_t>(1u, (T + per * kSmallSlices - 1) / (per * kSmallSlices));
  g.ns = (T + per * g.kq - 1) / (per * g.kq);
  if (fused) {  // one term per quad: 64 per slice
    g.kq = 1;
    g.ns = (T + kSmallQuads - 1) / kSmallQuads;
  }
  int rc;
  const uint32_t* ds = (const uint32_t*)scalars;
  const uint32_t* db = (const uint32_t*)bases;
  const auto tstage = std::chrono::steady_clock::now();
  // host phases (pm_ctx_set_timing_filter(ctx, "small_host"): no kernel is
  // event-timed, the call runs exactly as untimed and records small_stage,
  // small_launch, small_wait, host_tail and small_finish)
  auto phase = [&](const char* name, std::chrono::steady_clock::time_point t0) {
    if (!ctx->timing) return;
    auto& stt = ctx->stats[name];
    stt.first += 1;
    stt.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  };
  if (s_host || b_host) {
    const size_t sb = s_host ? n * 32 : 0, bb = b_host ? n * 64 : 0;
    if ((rc = ctx->ensure_small_pin(sb + bb))) return rc;
    void* dp = ctx->small_pin_dev;
    if (s_host) {
      std::memcpy(ctx->small_pin, scalars, sb);
      ds = (const uint32_t*)dp;
    }
    if (b_host) {
      std::memcpy((char*)ctx->small_pin + sb, bases, bb);
      db = (const uint32_t*)((char*)dp + sb);
    }
  }
  phase("small_stage", tstage);  // host copy into the pinned staging buffer
  const auto tlaunch = std::chrono::steady_clock::now();
  if (!fused) {
    if ((rc = ctx->small_tab.ensure(n * kSmallMults * sizeof(Xyzz<F>)))) return rc;
    if ((rc = ctx->small_dig.ensure((size_t)kSmallWin * T))) return rc;
  }
  if ((rc = ctx->small_part.ensure((size_t)kSmallWin * g.ns * sizeof(Xyzz<F>)))) return rc;
  // counters (self-resetting; zero fresh allocations): a ticket per window, the done count
  const size_t old_cap = ctx->small_tk.cap;
  if ((rc = ctx->small_tk.ensure((kSmallWin + 1) * 4))) return rc;
  if (ctx->small_tk.cap != old_cap) HIP_TRY(hipMemsetAsync(ctx->small_tk.p, 0, ctx->small_tk.cap, st));
  uint32_t* tickets = (uint32_t*)ctx->small_tk.p;
  if ((rc = ctx->ensure_pinned(kSmallWin * sizeof(Xyzz<F>) + 64))) return rc;
  if ((rc = ctx->ensure_group_events(1))) return rc;
  Xyzz<F>* hW = (Xyzz<F>*)ctx->h_pinned;
  volatile uint32_t* hflag = (volatile uint32_t*)(hW + kSmallWin);
  *hflag = 0;
  const uint32_t seq = ++ctx->small_seq ? ctx->small_seq : ++ctx->small_seq;
  void* dW = ctx->h_pinned_dev;
  uint32_t* dflag = (uint32_t*)((Xyzz<F>*)dW + kSmallWin);
  if (fused) {
    PM_LAUNCH(ctx, "small_fused",
              (k_small_fused<Cv><<<dim3(g.ns, kSmallWin), 256, 0, st>>>(g, ds, db, (Xyzz<F>*)ctx->small_part.p,
                                                                         tickets, (Xyzz<F>*)dW, tickets + kSmallWin,
                                                                         dflag, seq)));
  } else {
    Xyzz<F>* tab = (Xyzz<F>*)ctx->small_tab.p;
    int8_t* dig = (int8_t*)ctx->small_dig.p;
    const uint32_t nb_tab = (un + kSmallTabPts - 1) / kSmallTabPts, nb_dig = (un + 255) / 256;
    PM_LAUNCH(ctx, "small_table",
              (k_small_table<Cv><<<nb_tab + nb_dig, 256, 0, st>>>(g, nb_tab, ds, db, tab, dig)));
    if (lanes)
      PM_LAUNCH(ctx, "small_sum",
                (k_small_sum_lanes<Cv><<<dim3(g.ns, kSmallWin), 256, 0, st>>>(
                    g, tab, dig, (Xyzz<F>*)ctx->small_part.p, tickets, (Xyzz<F>*)dW, tickets + kSmallWin, dflag, seq)));
    else
      PM_LAUNCH(ctx, "small_sum",
                (k_small_sum<Cv><<<dim3(g.ns, kSmallWin), 256, 0, st>>>(g, tab, dig, (Xyzz<F>*)ctx->small_part.p,
                                                                         tickets, (Xyzz<F>*)dW, tickets + kSmallWin,
                                                                         dflag, seq)));
  }
  hipEvent_t ev = ctx->grp_ev[0];
  HIP_TRY(hipEventRecord(ev, st));
  phase("small_launch", tlaunch);  // buffers, counters and the launches queued
  const auto twait = std::chrono::steady_clock::now();
  // the flag instead of the event: 66.5 / 80.3 / 138.8 us against 71.9 /
  // 86.4 / 144.5 at n = 1 / 32 / 4096 (profiles/r04/small/flag_vs_event.txt)
  const bool kev = ctx->timed("small_fused") || ctx->timed("small_table") || ctx->timed("small_sum");
  if (kev) {  // the timed launches' events must complete (end_call)
    if ((rc = wait_event(ctx, ev))) return rc;
  } else {
    for (uint32_t it = 1;; it++) {
      if (__atomic_load_n((const uint32_t*)hflag, __ATOMIC_ACQUIRE) == seq) break;
      if ((it & 1023u) == 0) {
        const hipError_t q = hipEventQuery(ev);
        if (q == hipSuccess) {
          if (*hflag != seq) {  // counters left inconsistent by an earlier failure: reset them for the next call
            (void)hipMemsetAsync(ctx->small_tk.p, 0, ctx->small_tk.cap, st);
            (void)hipStreamSynchronize(st);
            return set_error(PM_ERR_HIP, "small MSM: kernels finished without the completion flag");
          }
          break;
        }
        if (q != hipErrorNotReady) return set_error(PM_ERR_HIP, std::string("small MSM: ") + hipGetErrorString(q));
      }
      __builtin_ia32_pause();
    }
  }
  phase("small_wait", twait);  // launches -> the completion flag
  const auto t0 = std::chrono::steady_clock::now();
  const host::Pt<F> r = host_has_bmi2() ? small_horner_bmi2<F>(hW) : small_horner<F, false>(hW);
  phase("host_tail", t0);
  const auto tfin = std::chrono::steady_clock::now();
  ctx->end_call();
  aff_to_u64<F>(xyzz_to_aff<F>(host::to_dev<F>(r)), out);
  phase("small_finish", tfin);  // end_call + the affine conversion
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
    // every MSM runs on st, so MSM j's kernels are queued behind MSM j-1's
    // term copy: the tail of j-1 runs on the host while the GPU works on j
    for (; tailed < j; tailed++) {
      Xyzz<F> r;
      if ((rc = msm_tail<F>(ctx, tails[tailed & 1], &r))) return rc;
      aff_to_u64<F>(xyzz_to_aff<F>(r), out + 8 * tailed);
    }
  }
  for (; tailed < k; tailed++) {
    Xyzz<F> r;
    if ((rc = msm_tail<F>(ctx, tails[tailed & 1], &r))) return rc;
    aff_to_u64<F>(xyzz_to_aff<F>(r), out + 8 * tailed);
  }
  HIP_TRY(hipStreamSynchronize(cs));
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
int msm_fixed_to_aff(Ctx* ctx, const pm_fixed_bases* ft, const void* d_s, size_t n, uint32_t flags, uint64_t out[8],
                     const void* h_s) {
  using F = typename Cv::Base;
  Xyzz<F> r;
  int rc = msm_device_impl<Cv>(ctx, (const uint32_t*)d_s, nullptr, n, flags, &r, ft, nullptr, 0, h_s);
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

// the fold of the per-rank partials of a sharded MSM (sharded.py): one call,
// additions in index order in XYZZ, one conversion (inversion) at the end
template <class F>
int points_sum_impl(const uint64_t* points, size_t n, uint64_t out[8]) {
  Xyzz<F> r = xyzz_from_aff<F>(aff_from_u64<F>(points));  // (0, 0) = identity
  for (size_t i = 1; i < n; i++) r = xyzz_add_aff<F>(r, aff_from_u64<F>(points + 8 * i));
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


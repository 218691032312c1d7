// runtime.hpp -- device context, workspace and launch plan of the MSM engine.
//
// A pm_ctx binds one device, one HIP stream and a grow-only workspace, so a
// caller (rayon thread in the Rust shim, one rank in bench.py) reuses device
// memory across calls and no hipMalloc happens once warm.  Calls on one
// context are serialised by its mutex (the C-ABI is re-entrant, §8b).
#pragma once
#include <hip/hip_runtime.h>

#include "../../include/pasta_msm.h"
#include "dropin_digest.hpp"

#include <condition_variable>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

namespace pm {

int set_error(int code, const std::string& msg);

constexpr int kMinC = 4;
constexpr int kMaxC = 20;
// Widest automatic window.  Measured on MI355X (profiles/r01_s2/diag22): once
// the bucket array (W * 2^(c-1) * 128 B) outgrows the caches, the scattered
// 128-B bucket stores of k_accumulate dominate: at 2^22, c = 18 took 11.7 ms
// in accumulate vs 6.1 ms at c = 16; at 2^20, c = 20 took 23.8 ms vs 1.4 ms.
constexpr int kAutoMaxC = 16;
constexpr size_t kMaxPoints = size_t(1) << 26;
constexpr int kL1 = 4;  // bucket-segment length of k_bucket_seg_q (one quad per segment)
// internal msm flag (never in the public header; the C-ABI strips it from
// caller flags): d_bases already hold the pipeline's R = 2^261 canonical
// form (resident pm_bases converted at upload), so no per-call conversion
constexpr uint32_t kBasesR261 = 1u << 30;
// k_bucket_bits blocks per job = kBitsSplitK / (bucket sets): the bit sums of
// few sets (row tables, the fixed-base MSM) are split over more blocks; every
// extra lane also adds one tree addition (round 3 sweep of 4..64 / Wr at
// 2^19-2^22, profiles/r03/ab/bits_split_sweep.jsonl: 16 best)
constexpr int kBitsSplitK = 16;
// drop-in base cache of pm_msm / pm_msm_ctx (capi.hip): base sets of at least
// kDropinMinN points are kept resident, keyed by a content digest; at most
// kDropinEntries sets and kDropinBytes of device memory per context
constexpr size_t kDropinMinN = size_t(1) << 12;
// the split scalar copy of row-table MSMs with host scalars (engine.hpp)
constexpr size_t kSplitCopyMinN = PM_SPLIT_COPY_MIN_N;
constexpr size_t kSplitCopy3MinN = size_t(1) << 21;  // three parts from here (measured at 2^20 and 2^22)
constexpr int kDropinEntries = 4;
constexpr size_t kDropinBytes = size_t(16) << 30;
// ... and at most this fraction (1/kDropinFreeDiv) of the device memory free
// at admission, counting the sets already held
constexpr size_t kDropinFreeDiv = 2;
// base sets seen once and not admitted: a set becomes resident on its second
// sighting, so one-shot bases never pay the row-table build
constexpr int kDropinSeen = 8;
// small drop-in sets (multiples tables, capi.hip dropin_small_msm): at most
// this many, and this many bytes of tables, per context.  A table costs
// 512 KiB per base at c = 8, so only sets of at most kDropinSmallMaxN points
// are kept (512-point sets held 256 MiB each); their bytes count in
// the drop-in cache's free-memory-aware budget with the large sets'.
constexpr int kDropinSmallEntries = 8;
constexpr size_t kDropinSmallMaxN = 64;
constexpr size_t kDropinSmallBytes = size_t(256) << 20;
// small-MSM path (msm_small.hpp): pm_msm* calls with n <= ctx->small_max (and
// the automatic window) run the two-launch table + window-sum kernels instead
// of the sorting pipeline; kSmallLimit bounds pm_ctx_set_small_msm
constexpr size_t kTailBytes = 128;  // opaque MsmTail storage (CurveOps::msm_start)
constexpr size_t kSmallMaxN = PM_SMALL_MSM_DEFAULT;
constexpr size_t kSmallLimit = PM_SMALL_MSM_LIMIT;

struct Buf {
  void* p = nullptr;
  size_t cap = 0;
  uint64_t gen = 0;  // bumped on every (re)allocation
  int ensure(size_t bytes);
  void release();
};

// Device copy of a small host table (accumulator / transcript programs,
// constants, VK points) that is uploaded only when its bytes change: a batch
// of proofs against one verifying key re-sends nothing after the first call.
struct CachedUpload {
  Buf buf;
  std::vector<uint8_t> host;
  uint64_t gen_at_upload = ~0ull;
  bool sent = false;  // the last put() queued a copy (false: the device copy was current)
  template <class T>
  int put(const std::vector<T>& v, hipStream_t st, size_t pad = 0);
};

struct MsmPlan {
  int c;          // target window width (bits)
  int W;          // windows = ceil(256 / c); widths base or base+1 (WinGeom)
  int base, extra;
  int cmax;       // widest window
  int K;          // max |digit| = 2^(cmax-1)
  int L1;         // bucket-segment length of k_bucket_seg_q
  int log2L1;
  int NB;         // bucket slots per window (K+1 rounded up to L1)
  int M1;         // segments per window: K / L1 (slots [0, K); bucket K apart)
  int NB2;        // bits of the segment index
  uint32_t n;
  uint32_t chunk;     // sorted entries per accumulate lane
  uint32_t nthreads;  // accumulate lanes
  int width(int w) const { return base + (w < extra ? 1 : 0); }
};

MsmPlan make_plan(size_t n, int c_override, int min_chunk = 0);
// fixed-base MSM over a table of npad rows per window (accumulate work =
// W * npad entries)
MsmPlan make_plan_fixed(size_t npad, int c, int min_chunk = 0);
// fixed-base windows: one bucket set of 2^(c-1) buckets
constexpr int kFixedMaxC = 20;
constexpr int kAutoFixedC = 16;       // n <= 2^21
constexpr int kAutoFixedCLarge = 20;  // n > 2^21 (fewer windows: 13 instead of 16)

struct TimedSpan {
  const char* name;
  hipEvent_t a, b;
};

// A few persistent host threads for data-parallel host work inside a call
// (the drop-in cache's content digest of the caller's bases runs on them
// while the scalars cross PCIe).  run() starts job(t, nt) for t = 1 .. nt-1
// on the workers; the caller runs t = 0 itself and then wait()s.
class HostPool {
 public:
  explicit HostPool(int threads);
  ~HostPool();
  int size() const { return (int)th_.size() + 1; }
  void start(int nt, std::function<void(int, int)> job);
  void wait();

 private:
  void loop(int t);
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::function<void(int, int)> job_;
  int nt_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// resident base set of the drop-in cache (pm_msm): key = (curve, n, keyed
// digest, dropin_digest.hpp)
struct DropinEntry {
  int curve;
  size_t n;
  uint64_t d[4];
  pm_bases* b;  // nullptr: seen once, not admitted yet (run through the plain path)
  size_t bytes;
  uint64_t last_use;
  uint64_t quick = 0;  // keyed hash of the first and last 8 points: picks the set to start speculatively
};

}  // namespace pm

// Fixed-base table (pm_fixed_bases_create*): rows x npad affine points in the
// pipeline's R = 2^261 form, row j = [2^{o_{j W / rows}}] P_i.  rows = W (the
// default) merges every window into one bucket set; rows = k < W merges
// windows w, w + W/k, ... into W/k bucket sets (W/k windows to reduce, a host
// Horner over 256/k bit positions, k x the bases' memory).
struct pm_fixed_bases {
  int curve;
  int device;
  int c, W, rows;
  size_t n, npad;
  void* d;
};

namespace pm {
// multiples table of a resident base set (msm_many.hpp): entry (i, w, m) =
// [m 2^{c w}] P_i, m = 1 .. H = 2^(c-1), w < W, XYZZ R = 2^261 (128 B), for
// the first n bases; built on demand by pm_msm_resident_many* /
// pm_bases_many_prepare and owned by the pm_bases
struct ManyTable {
  void* d = nullptr;
  size_t n = 0;
  uint32_t c = 0, W = 0, H = 0;
};
// geometry for a prefix of n bases: the widest window (fewest additions per
// scalar, W(c) of them) whose table fits kManyTabBudget; c = 4 up to the hard
// cap, beyond it pm_msm_resident_many falls back to one resident MSM each.
// W(c): signed digits in [-(2^(c-1) - 1), 2^(c-1)] of a scalar < 2^255 need a
// carry window only when c divides 255.
constexpr size_t kManyTabBudget = size_t(2) << 30;
constexpr size_t kManyTabCap = size_t(8) << 30;
inline uint32_t many_windows(uint32_t c) { return 255u % c == 0 ? 255u / c + 1u : (255u + c - 1u) / c; }
inline size_t many_bytes_per_base(uint32_t c) { return (size_t)many_windows(c) << (c - 1) << 7; }
inline uint32_t many_pick_c(size_t n) {
  for (uint32_t c = 8; c > 4; c--)
    if (n * many_bytes_per_base(c) <= kManyTabBudget) return c;
  return 4;
}
constexpr size_t kNttTwiddleSlots = 4;
constexpr uint32_t kNttMaxLog = 28;  // pm_fft: three passes above 2^22; BN254 Fr has 2-adicity 28
struct NttTwiddles {
  int curve = -1;
  uint32_t logn = 0;
  uint64_t omega[4] = {0, 0, 0, 0};
  uint64_t stamp = 0;
  Buf buf;
};
}  // namespace pm

struct pm_ctx {
  int device = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t stream = nullptr;
  hipStream_t red_stream = nullptr;  // accumulator side stream (accum_engine.hpp)
  // H2D copies beside the context stream's kernels: pm_msm_resident_batch (the
  // next MSM's scalars), the split scalar copy's second half (engine.hpp)
  hipStream_t copy_stream = nullptr;
  pm::HostPool* pool = nullptr;      // lazily created (drop-in digest)
  std::vector<pm::DropinEntry> dropin;  // drop-in base cache (pm_msm / pm_msm_ctx)
  std::vector<pm::DropinEntry> dropin_seen;  // digests seen once (b == nullptr), admitted on the second sighting
  // small sets (n <= small_max, below kDropinMinN): resident with a multiples
  // table (msm_many.hpp) after their second sighting, run as one-MSM
  // pm_msm_resident_many calls
  std::vector<pm::DropinEntry> dropin_small, dropin_small_seen;
  uint64_t dropin_small_hits = 0, dropin_small_admits = 0;
  pm::DigestKey dropin_key;             // secret per-context digest key (pm_ctx_create)
  uint64_t dropin_clock = 0;
  uint64_t dropin_hits = 0, dropin_misses = 0;
  uint64_t dropin_spec_hits = 0, dropin_spec_misses = 0;  // speculative starts kept / drained
  uint64_t dropin_oom_flushes = 0, dropin_failed_builds = 0;  // out-of-memory: whole cache released / set not admitted
  hipEvent_t batch_ev[4] = {};       // batch pipelining: copied[2], consumed[2]
  std::vector<hipEvent_t> grp_ev;    // MSM: one per pinned term slot (terms copied)
  int window_c = 0;
  int min_chunk = 0;
  // test hooks (tests/test_msm_gpu.py::test_fine_sort_lds_modes forces the
  // fine sort's LDS modes that only large segments reach): PM_FINE_CACHE_KB /
  // PM_FINE_CHUNK_KB, 0 = auto
  int fine_cache_kb = 0, fine_chunk_kb = 0;
  int ntt_passes = 0;  // NTT passes over HBM, 0 = auto (test hook: PM_NTT_PASSES env)
  int acc_split = -1; // accumulator lanes per term = 2^acc_split, -1 = auto (pm_ctx_set_accum_split)
  int acc_ladder = -1; // powers-table chains: 0 quads, 1 row-sliced waves, -1 = auto (pm_ctx_set_accum_ladder)
  // pm_ctx_set_accum_option (-1 = auto for each): the twisted ladder (0 off),
  // the stream of the term additions / sums (0 main), the one-lane form's
  // terms per lane (1, 2), the streamed transcript replay (0: per record)
  int acc_twist = -1, acc_tail = -1, acc_tpl = -1, acc_tr_stream = -1;
  // pm_ctx_set_msm_option(PM_MSM_OPT_SPLIT_COPY): -1 auto, 0 one scalar copy
  int msm_split_copy = -1;
  // the device's CU count (hipDeviceAttributeMultiprocessorCount, 256 on an
  // MI355X): the one-block-per-CU fences of the latency-bound accumulator
  // kernels are sized against it (pm_ctx_create refuses a device with less
  // than the 160 KiB of LDS per CU those fences and kernels assume)
  int num_cus = 256;
  bool timing = false;
  std::string timing_filter;  // time only launches with this name ("" = all)
  bool timed(const char* name) const { return timing && (timing_filter.empty() || timing_filter == name); }
  std::mutex mu;
  // workspace
  pm::Buf in_scalars, in_scalars2, in_bases, digits, sorted, counts, offsets, cursor, bsum, buckets, head, segS, segT, bits,
      win, longs, mid, acc_coef, acc_part, acc_io, bases29, tr_io, bitsP, tickets, ntt_scratch, bitsQ, acc_lad, acc_corr, tr_canon, ntt_scratch2,
      acc_vkpow, small_tab, small_dig, small_part, small_tk;
  // the later parts' sorted lists and bucket partials of the split scalar
  // copy (engine.hpp; the sort scratch is shared, its kernels run in order)
  pm::Buf part_sorted[2], part_offsets[2], part_buckets[2], part_head[2];
  pm::CachedUpload acc_prog, acc_const, acc_vk, tr_prog;
  pm::CachedUpload tr_wtab;  // streamed transcript: word table of the shape's byte stream
  pm::CachedUpload many_prog;  // pm_msm_resident_many*: job + MSM tables
  // proof-byte decoder (proof_kernels.hpp): square-root tables per curve
  // (pm_curve order), the point map of the current shape, host staging
  pm::Buf sqrt_tab[3];
  bool sqrt_ready[3] = {false, false, false};
  bool sqrt_tab_ts[3] = {false, false, false};  // the curve's root needs the Tonelli-Shanks windows (Pasta)
  pm::CachedUpload pf_map;
  pm::Buf pf_io;
  pm::Buf pf_flags;            // proof-decode flags per proof (cleared by k_transcript)
  bool pf_flags_dirty = false;  // a call failed between the decode and the replay
  // accumulator: powers-of-two tables of the verifying key's points (fixed,
  // sigma, g1), built once per (curve, VK) and reused by every later batch
  std::vector<uint64_t> acc_vkpow_key;
  uint64_t acc_vkpow_gen = ~0ull;  // acc_vkpow.gen when the tables were built
  std::vector<pm::NttTwiddles> ntt_tw;  // cached twiddle segments (pm_fft*)
  uint64_t ntt_clock = 0;
  void* h_pinned = nullptr;  // MSM host terms: two slots (batch pipelining)
  void* h_pinned_dev = nullptr;  // its device address (hipHostGetDevicePointer, once per allocation)
  size_t h_pinned_cap = 0;
  size_t small_max = pm::kSmallMaxN;  // small-MSM path threshold (pm_ctx_set_small_msm)
  void* small_pin = nullptr;          // small-MSM host inputs, pinned + mapped (read by k_small_table)
  void* small_pin_dev = nullptr;      // its device address
  size_t small_pin_cap = 0;
  uint32_t small_seq = 0;             // completion-flag value of the last small MSM
  // timing
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
  std::vector<pm::TimedSpan> pending;
  std::map<std::string, std::pair<uint64_t, double>> stats;

  std::vector<pm::Buf*> all_bufs() {
    return {&in_scalars, &in_scalars2, &in_bases, &digits, &sorted, &counts, &offsets, &cursor,
            &bsum,       &buckets,  &head,   &segS,   &segT,   &bits,    &win, &longs, &mid,
            &acc_prog.buf, &acc_const.buf, &acc_vk.buf, &acc_coef, &acc_part, &acc_io, &bases29, &tr_prog.buf, &tr_io, &bitsP, &tickets, &ntt_scratch, &bitsQ, &acc_lad, &acc_corr, &tr_canon, &ntt_scratch2, &acc_vkpow, &sqrt_tab[0], &sqrt_tab[1], &sqrt_tab[2], &pf_map.buf, &pf_io, &pf_flags, &small_tab, &small_dig, &small_part, &small_tk, &many_prog.buf, &tr_wtab.buf, &part_sorted[0], &part_sorted[1], &part_offsets[0], &part_offsets[1], &part_buckets[0], &part_buckets[1], &part_head[0], &part_head[1]};
  }
  ~pm_ctx();
  int begin_call();
  int end_call();
  int ensure_pinned(size_t bytes);
  int ensure_small_pin(size_t bytes);
  // host -> device copy of a caller buffer on `st` (one pageable
  // hipMemcpyAsync: ~52 GB/s for 32 MB on MI355X, faster than the pinned
  // staging threads round 2 measured, ~38 GB/s, and retired)
  int upload_h2d(void* d, const void* h, size_t bytes, hipStream_t st);
  int ensure_group_events(int n);
  pm::HostPool& host_pool();
  hipEvent_t next_event();
  void mark(const char* name, hipEvent_t a, hipEvent_t b);
};

namespace pm {
using Ctx = ::pm_ctx;
}

namespace pm {

// Per-curve engine entry points, one translation unit per curve
// (inst_pallas.hip, inst_vesta.hip, inst_bn254.hip) so they build in parallel.
struct CurveOps {
  // h_scalars != nullptr: scalars still in host memory, d_scalars their device buffer (chunked copy)
  int (*msm)(Ctx* ctx, const void* d_scalars, const void* d_bases, size_t n, uint32_t flags, uint64_t out[8],
             const void* h_scalars);
  int (*point_add)(const uint64_t a[8], const uint64_t b[8], uint64_t out[8]);
  int (*synth_scalars)(Ctx* ctx, uint64_t seed, uint64_t i0, uint32_t n, uint32_t mont, void* d_out);
  int (*synth_bases)(Ctx* ctx, uint64_t seed, uint64_t i0, uint32_t n, void* d_out);
  // vk_repr != nullptr: replay the transcript into d_challenges first (d_status as in transcript)
  int (*accum)(Ctx* ctx, const pm_proof_shape* shape, size_t B, const void* d_points, const void* d_scalars,
               void* d_challenges, void* d_out_quads, void* d_out_h, const uint64_t* vk_repr, void* d_status);
  int (*selftest_field)(Ctx* ctx, uint64_t seed, uint32_t n, uint64_t* mismatches);
  int (*transcript)(Ctx* ctx, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4], const void* d_points,
                    const void* d_scalars, void* d_challenges, void* d_status);
  int (*vk_repr)(const uint8_t digest[64], uint64_t out[4]);
  int (*fixed_table)(Ctx* ctx, const void* d_bases, pm_fixed_bases* ft);
  int (*ntt)(Ctx* ctx, int curve, void* d_data, uint32_t logn, const uint64_t omega[4], const uint64_t* scale);
  int (*msm_fixed)(Ctx* ctx, const pm_fixed_bases* ft, const void* d_scalars, size_t n, uint32_t flags,
                   uint64_t out[8], const void* h_scalars);
  // resident bases: Rust-layout affine (R = 2^256) -> the pipeline's R = 2^261 canonical form
  int (*bases_to29)(Ctx* ctx, const void* d_in, size_t n, void* d_out);
  // k MSMs of n host scalars against resident (R = 2^261) bases, pipelined
  // (ft != nullptr: the resident bases' row table, pm_fixed_bases_create_rows)
  int (*msm_resident_batch)(Ctx* ctx, const void* d_bases29, const pm_fixed_bases* ft, const uint64_t* const* scalars,
                            size_t k, size_t n, uint32_t flags, uint64_t* out);
  // proof bytes -> decoded points / scalars + status (proof_kernels.hpp); with
  // vk_repr also the transcript replay + accumulator (pm_accum_batch_proofs*)
  int (*proofs)(Ctx* ctx, const pm_proof_shape* shape, size_t B, const void* d_proofs, size_t stride,
                const void* d_inst, void* d_points, void* d_scalars, void* d_status, const uint64_t* vk_repr,
                void* d_ch, void* d_quads, void* d_h);
  // resident-bases MSM in two halves (the drop-in cache's speculative start):
  // msm_start enqueues the device pipeline on ctx->stream (ft: the row table,
  // else d_bases29 in the R = 2^261 form) and fills the opaque tail;
  // msm_finish waits for it and runs the host Horner.  h_scalars != nullptr:
  // the scalars are still in host memory and are copied to d_scalars first
  // (in two halves beside the pipeline with a row table: engine.hpp)
  int (*msm_start)(Ctx* ctx, const pm_fixed_bases* ft, const void* d_bases29, const void* d_scalars, size_t n,
                   uint32_t flags, void* tail, const void* h_scalars);
  int (*msm_finish)(Ctx* ctx, const void* tail, uint64_t out[8]);
  // small-MSM path (msm_small.hpp); s_host / b_host: the input is in host
  // memory; b_r261: bases in the resident R = 2^261 form
  int (*msm_small)(Ctx* ctx, const void* scalars, bool s_host, const void* bases, bool b_host, bool b_r261, size_t n,
                   uint32_t flags, uint64_t out[8]);
  // many short MSMs against resident bases (msm_many.hpp): build / grow the
  // multiples table of the first n bases, and the batched sum
  int (*many_table)(Ctx* ctx, const void* d_bases29, size_t n, ManyTable* t);
  int (*msm_many)(Ctx* ctx, const ManyTable* t, size_t B, const size_t* n, const size_t* off, const void* scalars,
                  bool s_host, uint32_t flags, uint64_t* out);
  // host: out = sum of n affine points (XYZZ accumulation, one inversion)
  int (*points_sum)(const uint64_t* points, size_t n, uint64_t out[8]);
};
extern const CurveOps kPallasOps, kVestaOps, kBn254Ops;

}  // namespace pm

#define HIP_TRY(expr)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return pm::set_error(PM_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

namespace pm {
template <class T>
int CachedUpload::put(const std::vector<T>& v, hipStream_t st, size_t pad) {
  const size_t bytes = v.size() * sizeof(T);
  int rc;
  sent = false;
  if ((rc = buf.ensure(bytes + pad))) return rc;
  if (buf.gen == gen_at_upload && host.size() == bytes && (bytes == 0 || memcmp(host.data(), v.data(), bytes) == 0))
    return PM_OK;
  if (bytes) HIP_TRY(hipMemcpyAsync(buf.p, v.data(), bytes, hipMemcpyHostToDevice, st));
  sent = bytes != 0;
  host.assign((const uint8_t*)v.data(), (const uint8_t*)v.data() + bytes);
  gen_at_upload = buf.gen;
  return PM_OK;
}

// Wait for `ev` on the host: the runtime's blocking wait (a hipEventQuery
// poll measured within run-to-run noise and burns a host core, round 3:
// profiles/r03/ab/spin_wait/).
inline int wait_event(const pm_ctx*, hipEvent_t ev) {
  HIP_TRY(hipEventSynchronize(ev));
  return PM_OK;
}
}  // namespace pm

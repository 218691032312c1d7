// capi.hip -- context, launch plan and the extern "C" boundary of the MSM engine.
//
// Boundary: halo2 `best_multiexp` ([3P], /root/reference/examples/
// simple-example.rs:606,620,638-640,702,722); see include/pasta_msm.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sched.h>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "../../include/pasta_msm.h"
#include "accum_plan.hpp"
#include "host_ec.hpp"
#include "msm_kernels.hpp"
#include "runtime.hpp"
#include "blake2b.hpp"
#include "engine.hpp"

using namespace pm;

// ------------------------------------------------------------------ errors
namespace pm {
thread_local std::string g_last_error;
int set_error(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}
}  // namespace pm

// ------------------------------------------------------------------ context
int pm::Buf::ensure(size_t bytes) {
  if (bytes <= cap) return PM_OK;
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  size_t want = std::max<size_t>(bytes, 256);
  hipError_t e = hipMalloc(&p, want);
  if (e != hipSuccess) {
    p = nullptr;
    return set_error(PM_ERR_HIP, std::string("hipMalloc(") + std::to_string(want) + "): " + hipGetErrorString(e));
  }
  cap = want;
  gen++;
  return PM_OK;
}
void pm::Buf::release() {
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
}

static void dropin_release_all(pm_ctx* ctx);

pm_ctx::~pm_ctx() {
  (void)hipSetDevice(device);
  dropin_release_all(this);
  delete pool;
  for (pm::Buf* b : all_bufs()) b->release();
  for (auto& t : ntt_tw) t.buf.release();
  if (h_pinned) (void)hipHostFree(h_pinned);
  if (small_pin) (void)hipHostFree(small_pin);
  for (auto& e : ev_pool) (void)hipEventDestroy(e);
  for (auto& e : grp_ev) (void)hipEventDestroy(e);
  for (auto& e : batch_ev)
    if (e) (void)hipEventDestroy(e);
  if (copy_stream) (void)hipStreamDestroy(copy_stream);
  if (red_stream) (void)hipStreamDestroy(red_stream);
  if (own_stream) (void)hipStreamDestroy(own_stream);
}

int pm_ctx::begin_call() {
  HIP_TRY(hipSetDevice(device));
  pending.clear();
  ev_used = 0;
  return PM_OK;
}

hipEvent_t pm_ctx::next_event() {
  if (ev_used == ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ev_pool.push_back(e);
  }
  return ev_pool[ev_used++];
}

void pm_ctx::mark(const char* name, hipEvent_t a, hipEvent_t b) { pending.push_back({name, a, b}); }

int pm_ctx::end_call() {
  // called after the stream has been synchronised
  for (auto& p : pending) {
    float ms = 0.f;
    if (p.a && p.b && hipEventElapsedTime(&ms, p.a, p.b) == hipSuccess) {
      auto& s = stats[p.name];
      s.first += 1;
      s.second += ms;
    }
  }
  pending.clear();
  return PM_OK;
}

int pm_ctx::ensure_group_events(int n) {
  while ((int)grp_ev.size() < n) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    grp_ev.push_back(e);
  }
  return PM_OK;
}

// threads for host-side data-parallel work: this process's CPUs, capped by
// OMP_NUM_THREADS (the GPU pool's 16-CPU share per GPU) and 16
static int host_threads() {
  int n = (int)std::thread::hardware_concurrency();
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = CPU_COUNT(&cs);
  if (const char* e = std::getenv("OMP_NUM_THREADS")) {
    const int k = std::atoi(e);
    if (k > 0) n = std::min(n, k);
  }
  return std::max(1, std::min(16, n));
}

pm::HostPool& pm_ctx::host_pool() {
  if (!pool) pool = new pm::HostPool(host_threads());
  return *pool;
}

pm::HostPool::HostPool(int threads) {
  for (int t = 1; t < threads; t++) th_.emplace_back([this, t] { loop(t); });
}
pm::HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> lk(m_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}
void pm::HostPool::loop(int t) {
  uint64_t seen = 0;
  for (;;) {
    std::function<void(int, int)> job;
    int nt;
    {
      std::unique_lock<std::mutex> lk(m_);
      cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      if (t >= nt_) continue;
      job = job_;
      nt = nt_;
    }
    job(t, nt);
    std::lock_guard<std::mutex> lk(m_);
    if (--pending_ == 0) done_.notify_all();
  }
}
void pm::HostPool::start(int nt, std::function<void(int, int)> job) {
  nt = std::max(1, std::min(nt, size()));
  {
    std::lock_guard<std::mutex> lk(m_);
    job_ = std::move(job);
    nt_ = nt;
    pending_ = nt - 1;
    gen_++;
  }
  cv_.notify_all();
}
void pm::HostPool::wait() {
  std::unique_lock<std::mutex> lk(m_);
  done_.wait(lk, [&] { return pending_ == 0; });
}

int pm_ctx::ensure_pinned(size_t bytes) {
  if (bytes <= h_pinned_cap) return PM_OK;
  if (h_pinned) (void)hipHostFree(h_pinned);
  h_pinned = nullptr;
  h_pinned_cap = 0;
  // coherent: the small-MSM path's window sums and completion flag live here
  // and are read by the host while the kernel still runs
  h_pinned_dev = nullptr;
  HIP_TRY(hipHostMalloc(&h_pinned, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer(&h_pinned_dev, h_pinned, 0));
  h_pinned_cap = bytes;
  return PM_OK;
}

int pm_ctx::ensure_small_pin(size_t bytes) {
  if (bytes <= small_pin_cap) return PM_OK;
  if (small_pin) (void)hipHostFree(small_pin);
  small_pin = nullptr;
  small_pin_cap = 0;
  // coherent (fine-grained) whatever HIP_HOST_COHERENT says: the host spins on
  // the completion flag and window sums the kernel writes here mid-launch
  small_pin_dev = nullptr;
  HIP_TRY(hipHostMalloc(&small_pin, bytes, hipHostMallocMapped | hipHostMallocCoherent));
  HIP_TRY(hipHostGetDevicePointer(&small_pin_dev, small_pin, 0));
  small_pin_cap = bytes;
  return PM_OK;
}

int pm_ctx::upload_h2d(void* d, const void* h, size_t bytes, hipStream_t st) {
  hipEvent_t ta = nullptr, tb = nullptr;
  if (timed("h2d")) {
    ta = next_event();
    tb = next_event();
    HIP_TRY(hipEventRecord(ta, st));
  }
  HIP_TRY(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, st));
  if (ta) {
    HIP_TRY(hipEventRecord(tb, st));
    mark("h2d", ta, tb);
  }
  return PM_OK;
}

// ------------------------------------------------------------------- plan
namespace pm {

static int bit_length(uint32_t v) {
  int b = 0;
  while (v) {
    b++;
    v >>= 1;
  }
  return b;
}

MsmPlan make_plan(size_t n, int c_override, int min_chunk) {
  MsmPlan pl;
  int lg = bit_length((uint32_t)std::max<size_t>(n, 1)) - 1;
  // auto window: lg - 2 from 2^14 up (capped at 16), lg - 4 below; swept on
  // MI355X (profiles/r01_s3/c_sweep_*.jsonl): 2^16 c = 14, 2^18 c = 16 (was
  // lg - 4 everywhere: 2^18 0.85 -> 0.77 ms, 2^16 0.68 -> 0.61 ms)
  int c = c_override > 0 ? c_override : std::max(4, std::min(kAutoMaxC, lg >= 14 ? lg - 2 : lg - 4));
  c = std::max(kMinC, std::min(kMaxC, c));
  pl.c = c;
  pl.W = (256 + c - 1) / c;
  pl.base = 256 / pl.W;
  pl.extra = 256 % pl.W;
  pl.cmax = pl.base + (pl.extra ? 1 : 0);
  pl.K = 1 << (pl.cmax - 1);
  pl.L1 = std::min(kL1, pl.K);
  pl.log2L1 = bit_length((uint32_t)pl.L1) - 1;
  pl.NB = ((pl.K + 1 + pl.L1 - 1) / pl.L1) * pl.L1;
  // segments cover slots [0, K); the top bucket K (the only one past them)
  // is folded by segment 0's unused slot-0 lane and reaches the host Horner
  // on its own (weight K): K / L1 is a power of two, so the segment grids
  // fill whole block rounds (2^20: 2048 blocks of k_bucket_seg_q, not 2049)
  pl.M1 = pl.K / pl.L1;
  pl.NB2 = bit_length((uint32_t)(pl.M1 - 1));
  pl.n = (uint32_t)n;
  // one window group: round 1 measured pipelined window groups (reduction of
  // group g beside the accumulation of g-1) slower at every size -- the
  // reduction kernels compete for the same VALU slots and each smaller
  // accumulate launch loses occupancy (2^20: G=1 2.29 ms, G=2 2.43, G=4 2.95;
  // profiles/r01_s2/pipe2) -- and round 3 retired them
  const size_t work = (size_t)n * pl.W;
  const size_t target = 256 * 1024;  // lanes in flight: 256 CUs x 16 waves x 64
  const size_t mc = min_chunk > 0 ? (size_t)min_chunk : 16;
  pl.chunk = (uint32_t)std::max<size_t>(mc, (work + target - 1) / target);
  pl.nthreads = (uint32_t)((work + pl.chunk - 1) / pl.chunk);
  return pl;
}

MsmPlan make_plan_fixed(size_t npad, int c, int min_chunk) {
  MsmPlan pl = make_plan(npad, c, min_chunk);
  const size_t work = npad * pl.W;  // every window's entries
  const size_t target = 256 * 1024;
  const size_t mc = min_chunk > 0 ? (size_t)min_chunk : 16;
  pl.chunk = (uint32_t)std::max<size_t>(mc, (work + target - 1) / target);
  pl.nthreads = (uint32_t)((work + pl.chunk - 1) / pl.chunk);
  return pl;
}

}  // namespace pm

namespace {

const CurveOps* curve_ops(int curve) {
  switch (curve) {
    case PM_CURVE_PALLAS: return &kPallasOps;
    case PM_CURVE_VESTA: return &kVestaOps;
    case PM_CURVE_BN254: return &kBn254Ops;
    default: return nullptr;
  }
}

// the small-MSM path (msm_small.hpp) takes n <= small_max under the automatic
// window (an explicit pm_ctx_set_window selects the sorting pipeline)
bool use_small(const Ctx* ctx, size_t n) { return n <= ctx->small_max && ctx->window_c == 0; }

// pre29: d_b holds resident bases already in the R = 2^261 form (pm_bases);
// h_s != nullptr: the scalars are still on the host (d_s is their buffer)
int dispatch_msm_device(Ctx* ctx, int curve, const void* d_s, const void* d_b, size_t n, uint32_t flags,
                        uint64_t out[8], bool pre29 = false, const void* h_s = nullptr) {
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  flags &= ~kBasesR261;  // internal bit: never taken from the caller
  return ops->msm(ctx, d_s, d_b, n, flags | (pre29 ? kBasesR261 : 0u), out, h_s);
}

// default context per device (lazily created, process lifetime)
std::mutex g_default_mu;
std::map<int, Ctx*> g_default;  // process lifetime: never freed (HIP may be torn down at exit)

int default_ctx(int device, Ctx** out) {
  std::lock_guard<std::mutex> lk(g_default_mu);
  auto it = g_default.find(device);
  if (it != g_default.end()) {
    *out = it->second;
    return PM_OK;
  }
  pm_ctx* c = nullptr;
  int rc = pm_ctx_create(device, &c);
  if (rc) return rc;
  g_default[device] = c;
  *out = c;
  return PM_OK;
}

bool valid_curve(int c) { return c == PM_CURVE_PALLAS || c == PM_CURVE_VESTA || c == PM_CURVE_BN254; }

}  // namespace

// ================================================================== C-ABI
extern "C" {

const char* pm_version(void) { return "pasta_msm 0.3 (gfx950)"; }
int pm_abi_version(void) { return PM_ABI_VERSION; }
const char* pm_last_error(void) { return pm::g_last_error.c_str(); }

int pm_device_count(int* count) {
  if (!count) return set_error(PM_ERR_ARG, "null count");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) {
    *count = 0;
    return set_error(PM_ERR_NODEV, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = c;
  return PM_OK;
}

int pm_ctx_create(int device, pm_ctx** out) {
  if (!out) return set_error(PM_ERR_ARG, "null out");
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) return set_error(PM_ERR_NODEV, "no HIP device");
  if (device < 0 || device >= cnt) return set_error(PM_ERR_NODEV, "device index out of range");
  std::unique_ptr<Ctx> c(new Ctx());
  c->device = device;
  HIP_TRY(hipSetDevice(device));
  {  // gfx950 only: the kernels' LDS layouts and fences assume 160 KiB per CU
    int cus = 0, lds = 0;
    HIP_TRY(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
    HIP_TRY(hipDeviceGetAttribute(&lds, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, device));
    if (lds < (int)kMaxLds)
      return set_error(PM_ERR_UNSUPPORTED, "device has " + std::to_string(lds) +
                                               " B of LDS per CU; this build needs gfx950's 160 KiB");
    c->num_cus = std::max(1, cus);
  }
  // the context's own stream is a BLOCKING stream: it is ordered after work
  // the caller queued on the legacy null stream (torch's default stream), so
  // a *_device entry sees inputs the caller has just written there.  The
  // internal reduction stream is ordered by events only.
  HIP_TRY(hipStreamCreateWithFlags(&c->own_stream, hipStreamDefault));
  c->stream = c->own_stream;
  HIP_TRY(hipStreamCreateWithFlags(&c->red_stream, hipStreamNonBlocking));
  try {  // std::random_device may throw when no entropy source is available
    pm::digest_key_init(c->dropin_key);
  } catch (const std::exception& e) {
    return set_error(PM_ERR_HIP, std::string("drop-in cache key: no entropy source: ") + e.what());
  }
  if (const char* e = std::getenv("PM_NTT_PASSES")) c->ntt_passes = std::atoi(e);
  if (const char* e = std::getenv("PM_FINE_CACHE_KB")) c->fine_cache_kb = std::max(0, std::min(144, std::atoi(e)));
  if (const char* e = std::getenv("PM_FINE_CHUNK_KB")) c->fine_chunk_kb = std::max(0, std::min(144, std::atoi(e)));
  *out = c.release();
  return PM_OK;
}

int pm_ctx_destroy(pm_ctx* ctx) {
  delete ctx;
  return PM_OK;
}

int pm_ctx_set_stream(pm_ctx* ctx, void* s) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  // NULL = the context's own stream (the round-1 meaning, which callers
  // compiled against that header rely on); PM_STREAM_LEGACY = the legacy
  // null stream itself
  if (s == nullptr) ctx->stream = ctx->own_stream;
  else if (s == PM_STREAM_LEGACY) ctx->stream = nullptr;
  else ctx->stream = (hipStream_t)s;
  return PM_OK;
}

int pm_ctx_use_own_stream(pm_ctx* ctx) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->stream = ctx->own_stream;
  return PM_OK;
}

int pm_ctx_set_glv(pm_ctx* ctx, int enable) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (enable) return set_error(PM_ERR_UNSUPPORTED, "GLV mode retired (measured slower on MI355X, DESIGN.md §7)");
  return PM_OK;
}

int pm_ctx_set_accum_ladder(pm_ctx* ctx, int mode) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (mode < -1 || mode > 1) return set_error(PM_ERR_ARG, "accum ladder mode out of range (-1 auto, 0 quads, 1 sliced)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->acc_ladder = mode;
  return PM_OK;
}

int pm_ctx_set_accum_split(pm_ctx* ctx, int lg_lanes) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (lg_lanes < -1 || lg_lanes > 5) return set_error(PM_ERR_ARG, "accum split out of range (-1 auto, 0..5)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->acc_split = lg_lanes;
  return PM_OK;
}

int pm_ctx_set_accum_option(pm_ctx* ctx, int option, int value) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  switch (option) {
    case PM_ACC_OPT_TWIST:
      if (value < -1 || value > 2)
        return set_error(PM_ERR_ARG, "twist option out of range (-1 auto, 0 off, 1 unfenced decode, 2 paired decode)");
      ctx->acc_twist = value;
      return PM_OK;
    case PM_ACC_OPT_TAIL_STREAM:
    case PM_ACC_OPT_TRANSCRIPT:
      if (value < -1 || value > 0) return set_error(PM_ERR_ARG, "accum option value out of range (-1 auto, 0 off)");
      (option == PM_ACC_OPT_TAIL_STREAM ? ctx->acc_tail : ctx->acc_tr_stream) = value;
      return PM_OK;
    case PM_ACC_OPT_TERMS_PER_LANE:
      if (value < -1 || value == 0 || value > 2)
        return set_error(PM_ERR_ARG, "terms per lane out of range (-1 auto, 1, 2)");
      ctx->acc_tpl = value;
      return PM_OK;
    default:
      return set_error(PM_ERR_ARG, "unknown accum option");
  }
}

int pm_ctx_set_msm_option(pm_ctx* ctx, int option, int value) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  switch (option) {
    case PM_MSM_OPT_SPLIT_COPY:
      if (value < -1 || value > 0) return set_error(PM_ERR_ARG, "msm option value out of range (-1 auto, 0 off)");
      ctx->msm_split_copy = value;
      return PM_OK;
    default:
      return set_error(PM_ERR_ARG, "unknown msm option");
  }
}

int pm_ctx_set_window(pm_ctx* ctx, int c) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (c != 0 && (c < kMinC || c > kMaxC)) return set_error(PM_ERR_ARG, "window width out of range");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->window_c = c;
  return PM_OK;
}

int pm_ctx_set_small_msm(pm_ctx* ctx, size_t max_n) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (max_n > kSmallLimit) return set_error(PM_ERR_ARG, "small-MSM threshold above PM_SMALL_MSM_LIMIT");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->small_max = max_n;
  return PM_OK;
}

int pm_ctx_set_pipeline(pm_ctx* ctx, int groups, int min_chunk) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (groups < 0 || min_chunk < 0 || min_chunk > (1 << 20)) return set_error(PM_ERR_ARG, "pipeline setting out of range");
  if (groups > 1)
    return set_error(PM_ERR_UNSUPPORTED, "window groups retired (measured slower on MI355X, DESIGN.md §7)");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->min_chunk = min_chunk;
  return PM_OK;
}

int pm_ctx_set_timing(pm_ctx* ctx, int enable) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->timing = enable != 0;
  return PM_OK;
}

int pm_ctx_set_timing_filter(pm_ctx* ctx, const char* kernel) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->timing_filter = kernel ? kernel : "";
  return PM_OK;
}

int pm_ctx_kernel_stats(pm_ctx* ctx, const char* kernel, uint64_t* launches, double* total_ms) {
  if (!ctx || !kernel || !launches || !total_ms) return set_error(PM_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  auto it = ctx->stats.find(kernel);
  *launches = it == ctx->stats.end() ? 0 : it->second.first;
  *total_ms = it == ctx->stats.end() ? 0.0 : it->second.second;
  return PM_OK;
}

int pm_ctx_reset_stats(pm_ctx* ctx) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->stats.clear();
  return PM_OK;
}

static int dropin_msm(Ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
                      uint64_t out[8]);

int pm_msm_ctx(pm_ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
               uint64_t out[8]) {
  if (!ctx || !out || (n && (!scalars || !bases))) return set_error(PM_ERR_ARG, "null argument");
  if (!valid_curve(curve)) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  return dropin_msm(ctx, curve, scalars, bases, n, flags, out);
}

int pm_msm(int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags, uint64_t out[8]) {
  Ctx* ctx = nullptr;
  int rc = default_ctx(0, &ctx);
  if (rc) return rc;
  return pm_msm_ctx(ctx, curve, scalars, bases, n, flags, out);
}

int pm_msm_device(pm_ctx* ctx, int curve, const void* d_scalars, const void* d_bases, size_t n, uint32_t flags,
                  uint64_t out[8]) {
  if (!ctx || !out || (n && (!d_scalars || !d_bases))) return set_error(PM_ERR_ARG, "null argument");
  if (!valid_curve(curve)) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  int rc = ctx->begin_call();
  if (rc) return rc;
  if (use_small(ctx, n)) return curve_ops(curve)->msm_small(ctx, d_scalars, false, d_bases, false, false, n, flags, out);
  return dispatch_msm_device(ctx, curve, d_scalars, d_bases, n, flags, out);
}

int pm_msm_multi(int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags, int ngpu,
                 uint64_t out[8]) {
  if (!out || (n && (!scalars || !bases))) return set_error(PM_ERR_ARG, "null argument");
  if (!valid_curve(curve)) return set_error(PM_ERR_ARG, "unknown curve id");
  int cnt = 0;
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt == 0) return set_error(PM_ERR_NODEV, "no HIP device");
  if (ngpu <= 0 || ngpu > cnt) return set_error(PM_ERR_NODEV, "ngpu out of range");
  std::vector<uint64_t> parts((size_t)ngpu * 8, 0);
  std::vector<int> rcs(ngpu, PM_OK);
  std::vector<std::string> errs(ngpu);
  std::vector<std::thread> th;
  const size_t per = (n + ngpu - 1) / ngpu;
  for (int g = 0; g < ngpu; g++) {
    th.emplace_back([&, g]() {
      const size_t lo = std::min(n, per * g), hi = std::min(n, per * (g + 1));
      Ctx* ctx = nullptr;
      int rc = default_ctx(g, &ctx);
      if (!rc) rc = pm_msm_ctx(ctx, curve, scalars + 4 * lo, bases + 8 * lo, hi - lo, flags, &parts[8 * g]);
      rcs[g] = rc;
      if (rc) errs[g] = pm::g_last_error;
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < ngpu; g++)
    if (rcs[g]) return set_error(rcs[g], "device " + std::to_string(g) + ": " + errs[g]);
  return pm_points_sum(curve, parts.data(), (size_t)ngpu, out);
}

// Resident SRS bases: stored in the pipeline's R = 2^261 canonical form
// (converted once here), so pm_msm_resident* skips the per-call conversion.
// From 2^18 points on the upload also keeps [2^{64 j}] P (4 rows up to 2^21
// points, [2^128] P beside P above): a full-length resident MSM then runs as a
// 4-row (2-row) table MSM (pm_fixed_bases_create_rows), whose bucket
// reduction and host Horner are 4x (2x) shorter (2^20: 1.61 -> 1.40 ms,
// profiles/r02/rows/).  Row 0 is the bases themselves, so windows with an
// offset still run the plain pipeline on it.
struct pm_bases {
  int curve;
  int device;
  size_t n;
  void* d;                 // row 0 (64 B per point)
  pm_fixed_bases* table;   // rows > 1: the same memory as a row table, or nullptr
  // multiples table of pm_msm_resident_many* (msm_many.hpp), built on demand
  mutable pm::ManyTable many;
  mutable std::mutex many_mu;
};

namespace {
constexpr size_t kResidentRowsMinN = size_t(1) << 18;
int resident_rows(size_t n) {
  if (n < kResidentRowsMinN) return 1;
  // round 3, after the sort changes (profiles/r03/rows_ab/, same box, 3
  // interleaved runs): 8 rows (two bucket sets) win up to 2^20 (2^20
  // 1.193-1.221 vs 1.224-1.273 ms; 2^19 0.738 vs 0.759), 4 rows at 2^21
  // (2.33-2.35 vs 2.35-2.39) and 2^22 (4.73-4.75 vs 2 rows 4.80-4.98);
  // larger sets keep 2 rows (unmeasured: the table grows past 1 GiB)
  if (n <= (size_t(1) << 20)) return 8;
  return n <= (size_t(1) << 22) ? 4 : 2;
}
// a resident MSM takes the row-table path when it starts at the first base
// and covers at least half of the table (rows past n are zero digits)
bool resident_use_table(const pm_bases* b, size_t offset, size_t n) {
  return b->table && offset == 0 && n >= kResidentRowsMinN && 2 * n >= b->table->npad;
}
}  // namespace

// the caller holds ctx->mu and has run begin_call
static int bases_upload_locked(pm_ctx* ctx, int curve, const void* bases, bool host, size_t n, pm_bases** out) {
  const CurveOps* ops = curve_ops(curve);
  int rc;
  std::unique_ptr<pm_bases> b(new pm_bases{curve, ctx->device, n, nullptr, nullptr});
  const void* src = bases;
  if (host && n) {
    if ((rc = ctx->in_bases.ensure(n * 64)) || (rc = ctx->upload_h2d(ctx->in_bases.p, bases, n * 64, ctx->stream)))
      return rc;
    src = ctx->in_bases.p;
  }
  const int rows = resident_rows(n);
  if (rows > 1) {
    std::unique_ptr<pm_fixed_bases> ft(new pm_fixed_bases{curve, ctx->device, 16, 0, rows, n, 0, nullptr});
    if ((rc = ops->fixed_table(ctx, src, ft.get()))) {
      if (ft->d) (void)hipFree(ft->d);
      return rc;
    }
    b->d = ft->d;
    b->table = ft.release();
  } else {
    HIP_TRY(hipMalloc(&b->d, std::max<size_t>(64, n * 64)));
    if ((rc = ops->bases_to29(ctx, src, n, b->d))) {
      (void)hipFree(b->d);
      return rc;
    }
  }
  *out = b.release();
  return PM_OK;
}

static int bases_upload(pm_ctx* ctx, int curve, const void* bases, bool host, size_t n, pm_bases** out) {
  if (!ctx || !out || (n && !bases)) return set_error(PM_ERR_ARG, "null argument");
  *out = nullptr;
  if (!curve_ops(curve)) return set_error(PM_ERR_ARG, "unknown curve id");
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "more than 2^26 resident bases");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return bases_upload_locked(ctx, curve, bases, host, n, out);
}

int pm_bases_upload(pm_ctx* ctx, int curve, const uint64_t* bases, size_t n, pm_bases** out) {
  return bases_upload(ctx, curve, bases, true, n, out);
}

int pm_bases_upload_device(pm_ctx* ctx, int curve, const void* d_bases, size_t n, pm_bases** out) {
  return bases_upload(ctx, curve, d_bases, false, n, out);
}

int pm_bases_info(const pm_bases* b, size_t* n, int* rows, size_t* device_bytes) {
  if (!b) return set_error(PM_ERR_ARG, "null argument");
  if (n) *n = b->n;
  if (rows) *rows = b->table ? b->table->rows : 1;
  if (device_bytes)
    *device_bytes = b->table ? (size_t)b->table->rows * b->table->npad * 64 : std::max<size_t>(64, b->n * 64);
  return PM_OK;
}

int pm_bases_release(pm_bases* b) {
  if (!b) return PM_OK;
  (void)hipSetDevice(b->device);
  (void)hipFree(b->d);  // the row table's memory when there is one
  if (b->many.d) (void)hipFree(b->many.d);
  delete b->table;
  delete b;
  return PM_OK;
}

static int msm_resident(pm_ctx* ctx, const pm_bases* b, size_t offset, const void* scalars, bool host, size_t n,
                        uint32_t flags, uint64_t out[8]) {
  if (!ctx || !b || !out || (n && !scalars)) return set_error(PM_ERR_ARG, "null argument");
  if (b->device != ctx->device) return set_error(PM_ERR_ARG, "bases live on another device");
  if (offset > b->n || n > b->n - offset) return set_error(PM_ERR_ARG, "window exceeds resident bases");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  int rc = ctx->begin_call();
  if (rc) return rc;
  const void* d_s = scalars;
  if (host) {  // copied by msm_device_impl (in two parts with a row table)
    if ((rc = ctx->in_scalars.ensure(n * 32))) return rc;
    d_s = ctx->in_scalars.p;
  }
  if (use_small(ctx, n))  // row 0 of a row table is the bases themselves
    return curve_ops(b->curve)->msm_small(ctx, scalars, host, (const char*)b->d + offset * 64, false, true, n,
                                          flags & ~kBasesR261, out);
  const void* h_s = host ? scalars : nullptr;
  if (resident_use_table(b, offset, n))
    return curve_ops(b->curve)->msm_fixed(ctx, b->table, d_s, n, flags & ~kBasesR261, out, h_s);
  return dispatch_msm_device(ctx, b->curve, d_s, (const char*)b->d + offset * 64, n, flags, out, true, h_s);
}

// ------------------------------------- many short MSMs (pm_msm_resident_many)
namespace {
// the multiples table covers the first n bases (grown to a power of two,
// at least 64, at most the set); the caller holds ctx->mu and b->many_mu
int many_ensure(pm_ctx* ctx, const pm_bases* b, size_t need) {
  if (b->many.d && b->many.n >= need) return PM_OK;
  size_t n = 64;
  while (n < need) n <<= 1;
  n = std::max(need, std::min({n, b->n, pm::kManyTabCap / pm::many_bytes_per_base(4)}));
  return curve_ops(b->curve)->many_table(ctx, b->d, n, &b->many);
}
}  // namespace

static int msm_many(pm_ctx* ctx, const pm_bases* b, size_t B, const size_t* n, const size_t* offsets,
                    const void* scalars, bool host, uint32_t flags, uint64_t* out) {
  if (!ctx || !b || (B && (!n || !out))) return set_error(PM_ERR_ARG, "null argument");
  if (b->device != ctx->device) return set_error(PM_ERR_ARG, "bases live on another device");
  if (B > (size_t(1) << 20)) return set_error(PM_ERR_UNSUPPORTED, "more than 2^20 MSMs in one call");
  size_t need = 0, total = 0;
  for (size_t i = 0; i < B; i++) {
    const size_t o = offsets ? offsets[i] : 0;
    if (o > b->n || n[i] > b->n - o) return set_error(PM_ERR_ARG, "an MSM window exceeds the resident bases");
    if (n[i]) need = std::max(need, o + n[i]);
    total += n[i];
  }
  if (total && !scalars) return set_error(PM_ERR_ARG, "null scalars");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  if (need * pm::many_bytes_per_base(4) > pm::kManyTabCap) {
    // a prefix too long for a table: one resident MSM per entry (same results)
    size_t s0 = 0;
    for (size_t i = 0; i < B; i++) {
      const void* si = (const char*)scalars + s0 * 32;
      const size_t o = offsets ? offsets[i] : 0;
      if (n[i] == 0) std::memset(out + 8 * i, 0, 64);
      else if (use_small(ctx, n[i]))
        rc = curve_ops(b->curve)->msm_small(ctx, si, host, (const char*)b->d + o * 64, false, true, n[i],
                                            flags & ~kBasesR261, out + 8 * i);
      else {
        const void* d_s = si;
        if (host) {
          if ((rc = ctx->in_scalars.ensure(n[i] * 32))) return rc;
          d_s = ctx->in_scalars.p;
        }
        rc = dispatch_msm_device(ctx, b->curve, d_s, (const char*)b->d + o * 64, n[i], flags, out + 8 * i, true,
                                 host ? si : nullptr);
      }
      if (rc) return rc;
      if ((rc = ctx->begin_call())) return rc;
      s0 += n[i];
    }
    return PM_OK;
  }
  std::lock_guard<std::mutex> lt(b->many_mu);
  if (need && (rc = many_ensure(ctx, b, need))) return rc;
  return curve_ops(b->curve)->msm_many(ctx, &b->many, B, n, offsets, scalars, host, flags, out);
}

int pm_msm_resident_many(pm_ctx* ctx, const pm_bases* bases, size_t B, const size_t* n, const size_t* offsets,
                         const uint64_t* scalars, uint32_t flags, uint64_t* out) {
  return msm_many(ctx, bases, B, n, offsets, scalars, true, flags, out);
}

int pm_msm_resident_many_device(pm_ctx* ctx, const pm_bases* bases, size_t B, const size_t* n, const size_t* offsets,
                                const void* d_scalars, uint32_t flags, uint64_t* out) {
  return msm_many(ctx, bases, B, n, offsets, d_scalars, false, flags, out);
}

int pm_bases_many_prepare(pm_ctx* ctx, const pm_bases* bases, size_t max_n) {
  if (!ctx || !bases) return set_error(PM_ERR_ARG, "null argument");
  if (bases->device != ctx->device) return set_error(PM_ERR_ARG, "bases live on another device");
  if (max_n > bases->n) return set_error(PM_ERR_ARG, "prefix exceeds the resident bases");
  if (max_n * pm::many_bytes_per_base(4) > pm::kManyTabCap)
    return set_error(PM_ERR_UNSUPPORTED, "prefix too long for a multiples table");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  std::lock_guard<std::mutex> lt(bases->many_mu);
  return max_n ? many_ensure(ctx, bases, max_n) : PM_OK;
}

int pm_bases_many_info(const pm_bases* bases, size_t* n, int* window, size_t* device_bytes) {
  if (!bases) return set_error(PM_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lt(bases->many_mu);
  if (n) *n = bases->many.d ? bases->many.n : 0;
  if (window) *window = bases->many.d ? (int)bases->many.c : 0;
  if (device_bytes) *device_bytes = bases->many.d ? bases->many.n * pm::many_bytes_per_base(bases->many.c) : 0;
  return PM_OK;
}

// ------------------------------------------------ drop-in base cache (pm_msm)
// halo2 calls best_multiexp with the same SRS bases over and over
// (commit_lagrange over params.g_lagrange, the commits inside create_proof:
// examples/simple-example.rs:606,638-640,702).  pm_msm / pm_msm_ctx keep base
// sets of >= kDropinMinN points resident, keyed by (curve, n, a keyed 254-bit
// digest of the base bytes: dropin_digest.hpp, secret key per context), so a
// repeated set skips its 64 B/point upload and runs as a resident (row-table)
// MSM.  The digest is computed on the host pool while the scalars cross
// PCIe; any change of the bytes (same pointer or not) changes the key.
//  * admission on the second sighting: the first call with a set runs the
//    plain pipeline on uploaded bases (no row-table build for one-shot sets)
//    and only remembers the digest;
//  * memory: least recently used sets are evicted BEFORE a new one is built,
//    against kDropinEntries and min(kDropinBytes, free device memory /
//    kDropinFreeDiv); if the build still fails, every set is released and the
//    build retried once, and if that fails the call runs the plain pipeline.
namespace {
constexpr size_t kDigestChunk = size_t(1) << 15;  // points per chunk (2 MiB)

// device bytes of a resident set of n points (bases_upload_locked's layout)
size_t dropin_bytes(size_t n) {
  const int rows = resident_rows(n);
  if (rows <= 1) return std::max<size_t>(64, n * 64);
  return (size_t)rows * std::max<size_t>(kSortB, (n + kSortB - 1) / kSortB * kSortB) * 64;  // fixed_table's npad
}

bool same_key(const pm::DropinEntry& e, int curve, size_t n, const uint64_t d[4]) {
  return e.curve == curve && e.n == n && std::memcmp(e.d, d, sizeof(e.d)) == 0;
}
}  // namespace

static void dropin_release_all(pm_ctx* ctx) {
  for (auto& e : ctx->dropin) pm_bases_release(e.b);
  ctx->dropin.clear();
  for (auto& e : ctx->dropin_small) pm_bases_release(e.b);
  ctx->dropin_small.clear();
}

static size_t dropin_small_total(const pm_ctx* ctx) {
  size_t s = 0;
  for (auto& e : ctx->dropin_small) s += e.bytes;
  return s;
}

// every byte the drop-in cache holds: the large sets and the small sets' tables
static size_t dropin_total(const pm_ctx* ctx) {
  size_t s = dropin_small_total(ctx);
  for (auto& e : ctx->dropin) s += e.bytes;
  return s;
}

static void dropin_evict_lru(pm_ctx* ctx) {
  auto lru = std::min_element(ctx->dropin.begin(), ctx->dropin.end(),
                              [](const pm::DropinEntry& x, const pm::DropinEntry& y) { return x.last_use < y.last_use; });
  pm_bases_release(lru->b);
  ctx->dropin.erase(lru);
}

// make room for `bytes` more: LRU eviction against the entry count and the
// memory budget (the fixed cap and a fraction of what the device has free)
static void dropin_make_room(pm_ctx* ctx, size_t bytes) {
  size_t free_b = 0, total_b = 0;
  const bool have_info = hipMemGetInfo(&free_b, &total_b) == hipSuccess;
  for (;;) {
    if (ctx->dropin.empty()) return;
    const size_t held = dropin_total(ctx);
    size_t budget = kDropinBytes;
    if (have_info) budget = std::min(budget, (free_b + held) / kDropinFreeDiv);
    if ((int)ctx->dropin.size() < kDropinEntries && held + bytes <= budget) return;
    const size_t before = ctx->dropin.size();
    dropin_evict_lru(ctx);
    if (have_info) free_b += held - dropin_total(ctx);
    if (ctx->dropin.size() == before) return;
  }
}

// Small sets (the small-MSM path's sizes): a repeated set -- halo2's
// commit_lagrange of a few public inputs against the first bases of
// g_lagrange, examples/simple-example.rs:632-641 -- is kept resident with a
// multiples table after its second sighting and then runs as ONE short MSM of
// pm_msm_resident_many (no doublings, no host Horner); first sightings and
// sets that do not fit run the small-MSM path on the host inputs.  The keyed
// digest of a small set is cheap (at most 1 MiB of bases).
// up to pm::kDropinSmallMaxN = 64 points (measured,
// profiles/r05/small_n_cache.json: a kept set against the small-MSM path 38 vs
// 66 us at n = 1, 63 vs 73 at 32, 82 vs 93 at 512 -- the last not worth its
// 256 MiB table, ADVICE r5 -- 107 vs 106 at 1024, 174 vs 139 at 4096)
static int dropin_small_msm(Ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n,
                            uint32_t flags, uint64_t out[8]) {
  const CurveOps* ops = curve_ops(curve);
  auto small = [&]() { return ops->msm_small(ctx, scalars, true, bases, true, false, n, flags, out); };
  const size_t tbytes = n * pm::many_bytes_per_base(pm::many_pick_c(n));
  if (n > pm::kDropinSmallMaxN || tbytes > pm::kDropinSmallBytes / 2) return small();
  pm::u128 part[2];
  pm::digest_chunk(ctx->dropin_key, bases, 8 * n, part);
  uint64_t d[4];
  pm::digest_combine(ctx->dropin_key, part, 1, d);
  pm_bases* b = nullptr;
  for (auto& e : ctx->dropin_small)
    if (same_key(e, curve, n, d)) {
      e.last_use = ++ctx->dropin_clock;
      b = e.b;
      break;
    }
  if (!b) {
    auto seen = std::find_if(ctx->dropin_small_seen.begin(), ctx->dropin_small_seen.end(),
                             [&](const pm::DropinEntry& e) { return same_key(e, curve, n, d); });
    if (seen == ctx->dropin_small_seen.end()) {  // first sighting
      if ((int)ctx->dropin_small_seen.size() >= kDropinSeen) ctx->dropin_small_seen.erase(ctx->dropin_small_seen.begin());
      ctx->dropin_small_seen.push_back(pm::DropinEntry{curve, n, {d[0], d[1], d[2], d[3]}, nullptr, 0, ++ctx->dropin_clock});
      return small();
    }
    ctx->dropin_small_seen.erase(seen);
    // LRU room against the entry count, the small sets' byte cap and the
    // drop-in cache's whole budget (large sets included: min(kDropinBytes,
    // free device memory / kDropinFreeDiv)); a set that still does not fit
    // is not admitted
    const size_t need = tbytes + 64 * n;
    size_t free_b = 0, total_b = 0;
    const bool have_info = hipMemGetInfo(&free_b, &total_b) == hipSuccess;
    for (;;) {
      const size_t held = dropin_total(ctx), held_small = dropin_small_total(ctx);
      size_t budget = kDropinBytes;
      if (have_info) budget = std::min(budget, (free_b + held) / kDropinFreeDiv);
      if ((int)ctx->dropin_small.size() < kDropinSmallEntries && held_small + need <= pm::kDropinSmallBytes &&
          held + need <= budget)
        break;
      // the large sets alone leave no room: keep the small sets, do not admit
      if (ctx->dropin_small.empty() || held - held_small + need > budget) return small();
      auto lru = std::min_element(ctx->dropin_small.begin(), ctx->dropin_small.end(),
                                  [](const pm::DropinEntry& x, const pm::DropinEntry& y) { return x.last_use < y.last_use; });
      if (have_info) free_b += lru->bytes;
      pm_bases_release(lru->b);
      ctx->dropin_small.erase(lru);
    }
    int rc = bases_upload_locked(ctx, curve, bases, true, n, &b);
    if (!rc) {
      std::lock_guard<std::mutex> lt(b->many_mu);
      rc = ops->many_table(ctx, b->d, n, &b->many);
    }
    if (rc) {  // not admitted (e.g. out of memory): the small path still computes it
      if (b) pm_bases_release(b);
      pm::g_last_error.clear();
      if ((rc = ctx->begin_call())) return rc;
      return small();
    }
    ctx->dropin_small_admits++;
    ctx->dropin_small.push_back(pm::DropinEntry{curve, n, {d[0], d[1], d[2], d[3]}, b, tbytes + 64 * n,
                                                ++ctx->dropin_clock});
    if (int r = ctx->begin_call()) return r;
  } else {
    ctx->dropin_small_hits++;
  }
  std::lock_guard<std::mutex> lt(b->many_mu);
  return ops->msm_many(ctx, &b->many, 1, &n, nullptr, scalars, true, flags, out);
}

static int dropin_msm(Ctx* ctx, int curve, const uint64_t* scalars, const uint64_t* bases, size_t n, uint32_t flags,
                      uint64_t out[8]) {
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  int rc;
  if ((rc = ctx->begin_call())) return rc;
  if (use_small(ctx, n)) return dropin_small_msm(ctx, curve, scalars, bases, n, flags, out);
  if ((rc = ctx->in_scalars.ensure(n * 32))) return rc;
  auto plain = [&]() -> int {  // both inputs uploaded, plain pipeline
    int r;
    if ((r = ctx->in_bases.ensure(n * 64))) return r;
    if ((r = ctx->upload_h2d(ctx->in_bases.p, bases, n * 64, ctx->stream))) return r;
    return dispatch_msm_device(ctx, curve, ctx->in_scalars.p, ctx->in_bases.p, n, flags, out);
  };
  if (n < kDropinMinN || n > kMaxPoints) {  // small MSMs bypass the cache
    if ((rc = ctx->upload_h2d(ctx->in_scalars.p, scalars, n * 32, ctx->stream))) return rc;
    return plain();
  }
  // keyed digest of the bases on the pool's workers while this thread copies the scalars
  const size_t nch = (n + kDigestChunk - 1) / kDigestChunk;
  std::vector<pm::u128> part(2 * nch);
  pm::HostPool& pool = ctx->host_pool();
  const int nw = std::max(1, pool.size() - 1);
  const pm::DigestKey& key = ctx->dropin_key;
  auto job = [&](int t, int) {
    for (size_t k = (size_t)(t - 1); k < nch; k += (size_t)nw) {
      const size_t p0 = k * kDigestChunk, p1 = std::min(n, p0 + kDigestChunk);
      pm::digest_chunk(key, bases + 8 * p0, 8 * (p1 - p0), &part[2 * k]);
    }
  };
  // a cheap keyed hash of the first and last 8 points names the resident set
  // this call most likely hits; its MSM starts right behind the scalar copy,
  // while the pool still hashes every byte, and its result is returned only
  // if the full digest then names the same set (else it is drained and the
  // call goes on as a miss)
  uint64_t quick;
  {
    const size_t k = std::min<size_t>(n, 8);
    pm::u128 a[2], z[2];
    pm::digest_chunk(key, bases, 8 * k, a);
    pm::digest_chunk(key, bases + 8 * (n - k), 8 * k, z);
    quick = (uint64_t)a[0] ^ ((uint64_t)(z[1] >> 64) * 0x9E3779B97F4A7C15ull) ^ (uint64_t)n;
  }
  const pm_bases* spec = nullptr;
  uint64_t spec_use = 0;
  for (auto& e : ctx->dropin)
    if (e.curve == curve && e.n == n && e.quick == quick && e.last_use >= spec_use) {
      spec = e.b;
      spec_use = e.last_use;
    }
  const bool threaded = pool.size() > 1;
  const auto t0 = std::chrono::steady_clock::now();
  if (threaded) pool.start(pool.size(), job);
  // with a predicted set the MSM copies the scalars itself (a row table's
  // MSM in two parts, the first part's sort and accumulation beside the
  // second part's copy: engine.hpp); else one copy here
  alignas(16) unsigned char tail[pm::kTailBytes];
  int spec_rc = -1, copy_rc = 0;
  if (spec)
    spec_rc = curve_ops(curve)->msm_start(ctx, resident_use_table(spec, 0, n) ? spec->table : nullptr, spec->d,
                                          ctx->in_scalars.p, n, flags, tail, scalars);
  else
    copy_rc = ctx->upload_h2d(ctx->in_scalars.p, scalars, n * 32, ctx->stream);
  const auto t1 = std::chrono::steady_clock::now();
  if (threaded) pool.wait();
  else job(1, 1);
  if (copy_rc) return copy_rc;
  if (spec && spec_rc) return spec_rc;
  uint64_t d[4];
  pm::digest_combine(key, part.data(), nch, d);
  if (ctx->timing) {  // host-side phases of the drop-in call (bench.py dropin_pm_msm)
    const auto t2 = std::chrono::steady_clock::now();
    auto add = [&](const char* k, double ms) {
      auto& e = ctx->stats[k];
      e.first += 1;
      e.second += ms;
    };
    add("dropin_copy_call", std::chrono::duration<double, std::milli>(t1 - t0).count());
    add("dropin_digest", std::chrono::duration<double, std::milli>(t2 - t0).count());
  }
  pm_bases* b = nullptr;
  for (auto& e : ctx->dropin)
    if (same_key(e, curve, n, d)) {
      e.last_use = ++ctx->dropin_clock;
      e.quick = quick;
      b = e.b;
      ctx->dropin_hits++;
      break;
    }
  if (spec) {
    if (b == spec) {
      ctx->dropin_spec_hits++;
      return curve_ops(curve)->msm_finish(ctx, tail, out);
    }
    uint64_t junk[8];  // another set: drain the speculative MSM
    if ((rc = curve_ops(curve)->msm_finish(ctx, tail, junk))) return rc;
    ctx->dropin_spec_misses++;
    if ((rc = ctx->begin_call())) return rc;
  }
  if (!b) {
    ctx->dropin_misses++;
    auto seen = std::find_if(ctx->dropin_seen.begin(), ctx->dropin_seen.end(),
                             [&](const pm::DropinEntry& e) { return same_key(e, curve, n, d); });
    if (seen == ctx->dropin_seen.end()) {  // first sighting: remember it, plain pipeline
      if ((int)ctx->dropin_seen.size() >= kDropinSeen) ctx->dropin_seen.erase(ctx->dropin_seen.begin());
      pm::DropinEntry e{curve, n, {d[0], d[1], d[2], d[3]}, nullptr, 0, ++ctx->dropin_clock};
      ctx->dropin_seen.push_back(e);
      return plain();
    }
    ctx->dropin_seen.erase(seen);
    dropin_make_room(ctx, dropin_bytes(n));
    rc = bases_upload_locked(ctx, curve, bases, true, n, &b);
    if (rc && !ctx->dropin.empty()) {  // out of device memory: release every set and retry once
      dropin_release_all(ctx);
      ctx->dropin_oom_flushes++;
      rc = bases_upload_locked(ctx, curve, bases, true, n, &b);
    }
    if (rc) {  // the set stays unadmitted; the MSM itself still runs (and succeeds without a stale message)
      ctx->dropin_failed_builds++;
      pm::g_last_error.clear();
      return plain();
    }
    size_t bytes = 0;
    pm_bases_info(b, nullptr, nullptr, &bytes);
    ctx->dropin.push_back(pm::DropinEntry{curve, n, {d[0], d[1], d[2], d[3]}, b, bytes, ++ctx->dropin_clock, quick});
  }
  if (resident_use_table(b, 0, n))
    return curve_ops(curve)->msm_fixed(ctx, b->table, ctx->in_scalars.p, n, flags & ~kBasesR261, out, nullptr);
  return dispatch_msm_device(ctx, curve, ctx->in_scalars.p, b->d, n, flags, out, true);
}

int pm_ctx_dropin_key_id(pm_ctx* ctx, uint64_t out[2]) {
  if (!ctx || !out) return set_error(PM_ERR_ARG, "null argument");
  std::lock_guard<std::mutex> lk(ctx->mu);
  pm::Blake2bHost h("pm-dropin-key-id");
  h.update(&ctx->dropin_key, sizeof(ctx->dropin_key));
  uint8_t dg[64];
  h.finalize(dg);
  std::memcpy(out, dg, 16);
  return PM_OK;
}

int pm_ctx_dropin_stats(pm_ctx* ctx, uint64_t* hits, uint64_t* misses, int* entries, size_t* device_bytes) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (hits) *hits = ctx->dropin_hits;
  if (misses) *misses = ctx->dropin_misses;
  if (entries) *entries = (int)ctx->dropin.size();
  if (device_bytes) {
    size_t s = 0;
    for (auto& e : ctx->dropin) s += e.bytes;
    *device_bytes = s;
  }
  return PM_OK;
}

int pm_ctx_dropin_spec_stats(pm_ctx* ctx, uint64_t* kept, uint64_t* drained) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (kept) *kept = ctx->dropin_spec_hits;
  if (drained) *drained = ctx->dropin_spec_misses;
  return PM_OK;
}

int pm_ctx_dropin_oom_stats(pm_ctx* ctx, uint64_t* flushes, uint64_t* failed_builds) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (flushes) *flushes = ctx->dropin_oom_flushes;
  if (failed_builds) *failed_builds = ctx->dropin_failed_builds;
  return PM_OK;
}

int pm_ctx_dropin_clear(pm_ctx* ctx) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  (void)hipSetDevice(ctx->device);
  dropin_release_all(ctx);
  ctx->dropin_seen.clear();
  ctx->dropin_small_seen.clear();
  return PM_OK;
}

int pm_ctx_dropin_small_stats(pm_ctx* ctx, uint64_t* hits, uint64_t* admitted, int* entries, size_t* device_bytes) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (hits) *hits = ctx->dropin_small_hits;
  if (admitted) *admitted = ctx->dropin_small_admits;
  if (entries) *entries = (int)ctx->dropin_small.size();
  if (device_bytes) {
    size_t t = 0;
    for (auto& e : ctx->dropin_small) t += e.bytes;
    *device_bytes = t;
  }
  return PM_OK;
}

int pm_msm_resident(pm_ctx* ctx, const pm_bases* b, size_t offset, const uint64_t* scalars, size_t n,
                    uint32_t flags, uint64_t out[8]) {
  return msm_resident(ctx, b, offset, scalars, true, n, flags, out);
}

int pm_msm_resident_device(pm_ctx* ctx, const pm_bases* b, size_t offset, const void* d_scalars, size_t n,
                           uint32_t flags, uint64_t out[8]) {
  return msm_resident(ctx, b, offset, d_scalars, false, n, flags, out);
}

int pm_msm_resident_batch(pm_ctx* ctx, const pm_bases* b, size_t offset, const uint64_t* const* scalars, size_t k,
                          size_t n, uint32_t flags, uint64_t* out) {
  if (!ctx || !b || (k && (!scalars || !out))) return set_error(PM_ERR_ARG, "null argument");
  for (size_t j = 0; j < k && n; j++)
    if (!scalars[j]) return set_error(PM_ERR_ARG, "null scalar array");
  if (b->device != ctx->device) return set_error(PM_ERR_ARG, "bases live on another device");
  if (offset > b->n || n > b->n - offset) return set_error(PM_ERR_ARG, "window exceeds resident bases");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return curve_ops(b->curve)->msm_resident_batch(ctx, (const char*)b->d + offset * 64,
                                                 resident_use_table(b, offset, n) ? b->table : nullptr, scalars, k,
                                                 n, flags & ~kBasesR261, out);
}

int pm_ctx_set_h2d_threads(pm_ctx* ctx, int threads) {
  if (!ctx) return set_error(PM_ERR_ARG, "null ctx");
  if (threads < 0) return set_error(PM_ERR_ARG, "h2d threads out of range");
  if (threads > 0)
    return set_error(PM_ERR_UNSUPPORTED, "pinned staging threads retired (measured slower on MI355X, DESIGN.md §5)");
  return PM_OK;
}

// ------------------------------------------------- NTT (§8f-4)
int pm_fft_device(pm_ctx* ctx, int curve, void* d_data, uint32_t log_n, const uint64_t omega[4],
                  const uint64_t* scale) {
  if (!ctx || !d_data || !omega) return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  if (log_n > pm::kNttMaxLog) return set_error(PM_ERR_UNSUPPORTED, "NTT longer than 2^28");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return ops->ntt(ctx, curve, d_data, log_n, omega, scale);
}

int pm_fft(pm_ctx* ctx, int curve, uint64_t* data, uint32_t log_n, const uint64_t omega[4], const uint64_t* scale) {
  if (!ctx || !data || !omega) return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  if (log_n > pm::kNttMaxLog) return set_error(PM_ERR_UNSUPPORTED, "NTT longer than 2^28");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  const size_t bytes = ((size_t)1 << log_n) * 32;
  if ((rc = ctx->in_scalars.ensure(bytes))) return rc;
  HIP_TRY(hipMemcpyAsync(ctx->in_scalars.p, data, bytes, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = ops->ntt(ctx, curve, ctx->in_scalars.p, log_n, omega, scale))) return rc;
  HIP_TRY(hipMemcpyAsync(data, ctx->in_scalars.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

// ------------------------------------------------- fixed-base MSM (§8f-3)
static int fixed_create(pm_ctx* ctx, int curve, const void* bases, bool host, size_t n, int c, int rows,
                        pm_fixed_bases** out) {
  if (!ctx || !out || (n && !bases)) return set_error(PM_ERR_ARG, "null argument");
  *out = nullptr;
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  if (n == 0) return set_error(PM_ERR_ARG, "empty base set");
  if (n > kMaxPoints) return set_error(PM_ERR_UNSUPPORTED, "more than 2^26 fixed bases");
  if (c == 0) c = n > (size_t(1) << 21) ? kAutoFixedCLarge : kAutoFixedC;
  if (c < kMinC || c > kFixedMaxC) return set_error(PM_ERR_ARG, "fixed-base window out of range");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  if (rows < 0) return set_error(PM_ERR_ARG, "negative table rows");
  std::unique_ptr<pm_fixed_bases> ft(new pm_fixed_bases{curve, ctx->device, c, 0, rows, n, 0, nullptr});
  const void* d = bases;
  if (host) {
    if ((rc = ctx->in_bases.ensure(n * 64))) return rc;
    if ((rc = ctx->upload_h2d(ctx->in_bases.p, bases, n * 64, ctx->stream))) return rc;
    d = ctx->in_bases.p;
  }
  if ((rc = ops->fixed_table(ctx, d, ft.get()))) {
    if (ft->d) (void)hipFree(ft->d);
    return rc;
  }
  *out = ft.release();
  return PM_OK;
}

int pm_fixed_bases_create(pm_ctx* ctx, int curve, const uint64_t* bases, size_t n, int c, pm_fixed_bases** out) {
  return fixed_create(ctx, curve, bases, true, n, c, 0, out);
}

int pm_fixed_bases_create_device(pm_ctx* ctx, int curve, const void* d_bases, size_t n, int c,
                                 pm_fixed_bases** out) {
  return fixed_create(ctx, curve, d_bases, false, n, c, 0, out);
}

int pm_fixed_bases_create_rows(pm_ctx* ctx, int curve, const void* bases, int bases_on_device, size_t n, int c,
                               int rows, pm_fixed_bases** out) {
  return fixed_create(ctx, curve, bases, bases_on_device == 0, n, c, rows, out);
}

int pm_fixed_bases_info(const pm_fixed_bases* fb, size_t* n, int* c, int* windows, size_t* table_bytes) {
  if (!fb) return set_error(PM_ERR_ARG, "null argument");
  if (n) *n = fb->n;
  if (c) *c = fb->c;
  if (windows) *windows = fb->W;
  if (table_bytes) *table_bytes = (size_t)fb->rows * fb->npad * 64;
  return PM_OK;
}

int pm_fixed_bases_release(pm_fixed_bases* fb) {
  if (!fb) return PM_OK;
  (void)hipSetDevice(fb->device);
  (void)hipFree(fb->d);
  delete fb;
  return PM_OK;
}

int pm_msm_fixed_device(pm_ctx* ctx, const pm_fixed_bases* fb, const void* d_scalars, size_t n, uint32_t flags,
                        uint64_t out[8]) {
  if (!ctx || !fb || !out || (n && !d_scalars)) return set_error(PM_ERR_ARG, "null argument");
  if (fb->device != ctx->device) return set_error(PM_ERR_ARG, "fixed bases live on another device");
  if (n > fb->n) return set_error(PM_ERR_ARG, "more scalars than fixed bases");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  int rc = ctx->begin_call();
  if (rc) return rc;
  return curve_ops(fb->curve)->msm_fixed(ctx, fb, d_scalars, n, flags & ~kBasesR261, out, nullptr);
}

int pm_msm_fixed(pm_ctx* ctx, const pm_fixed_bases* fb, const uint64_t* scalars, size_t n, uint32_t flags,
                 uint64_t out[8]) {
  if (!ctx || !fb || !out || (n && !scalars)) return set_error(PM_ERR_ARG, "null argument");
  if (fb->device != ctx->device) return set_error(PM_ERR_ARG, "fixed bases live on another device");
  if (n > fb->n) return set_error(PM_ERR_ARG, "more scalars than fixed bases");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  int rc = ctx->begin_call();
  if (rc) return rc;
  if ((rc = ctx->in_scalars.ensure(n * 32))) return rc;
  return curve_ops(fb->curve)->msm_fixed(ctx, fb, ctx->in_scalars.p, n, flags & ~kBasesR261, out, scalars);
}

int pm_point_add(int curve, const uint64_t a[8], const uint64_t b[8], uint64_t out[8]) {
  if (!a || !b || !out) return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  return ops->point_add(a, b, out);
}

int pm_points_sum(int curve, const uint64_t* points, size_t n, uint64_t out[8]) {
  if (!out || (n && !points)) return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  if (n == 0) {
    std::memset(out, 0, 64);
    return PM_OK;
  }
  return ops->points_sum(points, n, out);
}

int pm_synth_scalars(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, uint32_t flags, void* d_out) {
  if (!ctx || (n && !d_out)) return set_error(PM_ERR_ARG, "null argument");
  if (n > 0xffffffffull) return set_error(PM_ERR_ARG, "n too large");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) return PM_OK;
  int rc = ctx->begin_call();
  if (rc) return rc;
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  return ops->synth_scalars(ctx, seed, i0, (uint32_t)n, (flags & PM_SCALARS_CANONICAL) ? 0u : 1u, d_out);
}

int pm_synth_bases(pm_ctx* ctx, int curve, uint64_t seed, uint64_t i0, size_t n, void* d_out) {
  if (!ctx || (n && !d_out)) return set_error(PM_ERR_ARG, "null argument");
  if (n > 0xffffffffull) return set_error(PM_ERR_ARG, "n too large");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (n == 0) return PM_OK;
  int rc = ctx->begin_call();
  if (rc) return rc;
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  return ops->synth_bases(ctx, seed, i0, (uint32_t)n, d_out);
}

int pm_selftest_field(pm_ctx* ctx, int curve, uint64_t seed, size_t n, uint64_t* mismatches) {
  if (!ctx || !mismatches) return set_error(PM_ERR_ARG, "null argument");
  if (n > (1u << 24)) return set_error(PM_ERR_ARG, "n too large");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return ops->selftest_field(ctx, seed, (uint32_t)n, mismatches);
}

extern "C++" {
namespace {
template <class P>
uint64_t selftest_host_field(uint64_t seed, size_t n) {
  using namespace pm::host;
  uint64_t st = seed * 0x9E3779B97F4A7C15ull + 1, bad = 0;
  auto rnd = [&]() {
    st ^= st << 13;
    st ^= st >> 7;
    st ^= st << 17;
    return st;
  };
  auto fe = [&]() {  // uniform-ish below p, plus the edges 0, 1, p - 1
    E<P> e;
    const uint64_t k = rnd() % 16;
    for (int i = 0; i < 4; i++) e.v[i] = k == 0 ? 0 : k == 1 ? (i == 0) : k == 2 ? F64<P>::mod(i) - (i == 0) : rnd();
    if (k > 2) {
      e.v[3] %= F64<P>::mod(3);
    }
    return e;
  };
  for (size_t i = 0; i < n; i++) {
    const E<P> a = fe(), b = fe();
    const E<P> x = mul<P>(a, b), y = mul_adx<P>(a, b);
    bad += memcmp(x.v, y.v, 32) != 0;
  }
  Pt<P> h0{fe(), fe(), fe(), fe()}, h1 = h0, g{fe(), fe(), fe(), fe()};
  for (size_t i = 0; i < 64; i++) {
    h0 = dbl<P, false>(h0);
    h1 = dbl<P, true>(h1);
    if (i & 1) {
      h0 = addp<P, false>(h0, g);
      h1 = addp<P, true>(h1, g);
    }
  }
  bad += memcmp(&h0, &h1, sizeof(h0)) != 0;
  // Jacobian chain (jdbl / jadd, the small-MSM Horner) == the XYZZ chain: the
  // same rational maps, so any (x, y) works; both start from the same point
  // under a random z (Jacobian (X, Y, z), XYZZ (X, Y, z^2, z^3))
  auto both = [&](Pt<P>& x, Jac<P>& j) {
    const E<P> z = fe(), zz = mul<P>(z, z), zzz = mul<P>(zz, z);
    x = Pt<P>{fe(), fe(), zz, zzz};
    j = Jac<P>{x.X, x.Y, z};
  };
  Pt<P> xa, xg;
  Jac<P> ja, jg;
  both(xa, ja);
  both(xg, jg);
  for (size_t i = 0; i < 40; i++) {
    xa = dbl<P, true>(xa);
    ja = jdbl<P, true>(ja);
    if (i % 3 == 0) {
      xa = addp<P, true>(xa, xg);
      ja = jadd<P, false>(ja, jg);
    }
  }
  const Pt<P> jx = jac_to_xyzz<P, true>(ja);  // equal points: X1 ZZ2 == X2 ZZ1, Y1 ZZZ2 == Y2 ZZZ1
  auto same = [&](const Pt<P>& u, const Pt<P>& v) {
    const E<P> l1 = mul<P>(u.X, v.ZZ), r1 = mul<P>(v.X, u.ZZ), l2 = mul<P>(u.Y, v.ZZZ), r2 = mul<P>(v.Y, u.ZZZ);
    return memcmp(&l1, &r1, 32) == 0 && memcmp(&l2, &r2, 32) == 0 && !is_zero(u.ZZ) && !is_zero(v.ZZ);
  };
  bad += !same(xa, jx);
  // the split host tail (sets claimed by pool threads, engine.hpp tail_split)
  // == the single Horner (tail_terms / tail_run) on the variable-base
  // geometry (16 sets of 16 bits), with identity terms among random ones, on
  // pools of 1, 3 and 16 threads
  {
    pm::MsmTail<P> t;
    t.Wr = 16;
    t.NB2 = 13;
    t.NQ = t.NB2 + pm::kTJobs + 1;
    t.base = 16;
    t.extra = 0;
    t.log2L1 = 2;
    t.cmax = 16;
    t.empty = false;
    // terms on the curve (the group law is associative only there, and the
    // two forms add the terms in different orders): multiples of the
    // generator by a random double-and-add walk, each under a random z
    auto e_of = [](const pm::Fe<P>& f) {
      E<P> e;
      for (int k = 0; k < 4; k++) e.v[k] = (uint64_t)f.l[2 * k] | ((uint64_t)f.l[2 * k + 1] << 32);
      return e;
    };
    const pm::Fe<P> one = pm::fe_one<P>();
    const bool pasta = !std::is_same<P, pm::Bn254Fq>::value;  // generators (-1, 2) / (1, 2)
    const Pt<P> G{e_of(pasta ? pm::fe_neg<P>(one) : one), e_of(pm::fe_add<P>(one, one)), e_of(one), e_of(one)};
    std::vector<pm::Xyzz<P>> Q((size_t)t.Wr * t.NQ);
    Pt<P> cur = G;
    for (size_t k = 0; k < Q.size(); k++) {
      cur = (rnd() & 1) ? dbl<P, true>(cur) : addp<P, true>(cur, G);
      const E<P> z = fe(), zz = mul<P>(z, z), zzz = mul<P>(zz, z);
      const Pt<P> x{mul<P>(cur.X, zz), mul<P>(cur.Y, zzz), mul<P>(cur.ZZ, zz), mul<P>(cur.ZZZ, zzz)};
      Q[k] = to_dev<P>(k % 37 == 5 || is_zero(z) ? inf<P>() : x);
    }
    t.hQ = Q.data();
    const Pt<P> want = pm::tail_run<P>(t, pm::tail_terms<P>(t));
    for (int th : {1, 3, 16}) {
      pm::HostPool pool(th);
      bad += !same(pm::tail_split_bmi2<P>(pool, t), want);
    }
  }
  return bad;
}
}  // namespace
}  // extern "C++"

int pm_selftest_host(int curve, uint64_t seed, size_t n, uint64_t* mismatches) {
  if (!mismatches) return set_error(PM_ERR_ARG, "null argument");
  if (n > (1u << 24)) return set_error(PM_ERR_ARG, "n too large");
  if (!pm::host_has_bmi2()) return set_error(PM_ERR_UNSUPPORTED, "CPU without BMI2/ADX");
  switch (curve) {
    case PM_CURVE_PALLAS: *mismatches = selftest_host_field<pm::PallasFp>(seed, n); break;
    case PM_CURVE_VESTA: *mismatches = selftest_host_field<pm::VestaFp>(seed, n); break;
    case PM_CURVE_BN254: *mismatches = selftest_host_field<pm::Bn254Fq>(seed, n); break;
    default: return set_error(PM_ERR_ARG, "unknown curve id");
  }
  return PM_OK;
}

// ------------------------------------------------- multiopen accumulator
int pm_shape_layout(const pm_proof_shape* shape, uint32_t* points_per_proof, uint32_t* scalars_per_proof,
                    uint32_t* num_sets) {
  std::vector<AccQuery> q;
  AccLayout L;
  const std::string err = acc_validate(shape, q, L, nullptr);
  if (!err.empty()) return set_error(PM_ERR_ARG, "accum shape: " + err);
  if (points_per_proof) *points_per_proof = L.npts;
  if (scalars_per_proof) *scalars_per_proof = L.nsc;
  if (num_sets) *num_sets = L.nsets;
  return PM_OK;
}

int pm_accum_batch_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const void* d_points,
                          const void* d_scalars, const void* d_challenges, void* d_out_quads, void* d_out_h_eval,
                          void* d_out_status) {
  if (!ctx || !shape || (B && (!d_points || !d_scalars || !d_challenges || !d_out_quads)))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return ops->accum(ctx, shape, B, d_points, d_scalars, const_cast<void*>(d_challenges), d_out_quads, d_out_h_eval, nullptr,
                    d_out_status);
}

int pm_accum_batch(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t* points,
                   const uint64_t* scalars, const uint64_t* challenges, uint64_t* out_quads, uint64_t* out_h_eval,
                   uint32_t* out_status) {
  if (!ctx || !shape || (B && (!points || !scalars || !challenges || !out_quads)))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (B == 0) return PM_OK;
  if ((rc = ctx->begin_call())) return rc;
  const size_t bp = B * npts * 64, bs = B * nsc * 32, bc = B * 7 * 32, bo = B * 4 * 64, bh = B * 32, bst = B * 4;
  if ((rc = ctx->acc_io.ensure(bp + bs + bc + bo + bh + bst))) return rc;
  char* base = (char*)ctx->acc_io.p;
  HIP_TRY(hipMemcpyAsync(base, points, bp, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(base + bp, scalars, bs, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(base + bp + bs, challenges, bc, hipMemcpyHostToDevice, ctx->stream));
  char* dq = base + bp + bs + bc;
  char* dh = dq + bo;
  char* dst = dh + bh;
  if ((rc = ops->accum(ctx, shape, B, base, base + bp, base + bp + bs, dq, dh, nullptr, out_status ? dst : nullptr)))
    return rc;
  HIP_TRY(hipMemcpyAsync(out_quads, dq, bo, hipMemcpyDeviceToHost, ctx->stream));
  if (out_h_eval) HIP_TRY(hipMemcpyAsync(out_h_eval, dh, bh, hipMemcpyDeviceToHost, ctx->stream));
  if (out_status) HIP_TRY(hipMemcpyAsync(out_status, dst, bst, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

// ------------------------------------------------- Blake2b transcript replay
int pm_vk_transcript_repr(int curve, const uint8_t* pinned, size_t len, uint64_t out[4]) {
  if (!out || (len && !pinned)) return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  Blake2bHost hs(kVerifyKeyPersonal);
  uint8_t le[8];
  for (int i = 0; i < 8; i++) le[i] = (uint8_t)((uint64_t)len >> (8 * i));
  hs.update(le, 8);
  hs.update(pinned, len);
  uint8_t d[64];
  hs.finalize(d);
  return ops->vk_repr(d, out);
}

int pm_transcript_batch_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                               const uint64_t vk_repr[4], const void* d_points, const void* d_scalars,
                               void* d_out_challenges, void* d_out_status) {
  if (!ctx || !shape || !vk_repr || (B && (!d_points || !d_scalars || !d_out_challenges)))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  if ((rc = ops->transcript(ctx, shape, B, vk_repr, d_points, d_scalars, d_out_challenges, d_out_status))) return rc;
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  ctx->end_call();
  return PM_OK;
}

int pm_accum_batch_transcript_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                                     const uint64_t vk_repr[4], const void* d_points, const void* d_scalars,
                                     void* d_challenges, void* d_out_quads, void* d_out_h_eval,
                                     void* d_out_status) {
  if (!ctx || !shape || !vk_repr || (B && (!d_points || !d_scalars || !d_challenges || !d_out_quads)))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return ops->accum(ctx, shape, B, d_points, d_scalars, d_challenges, d_out_quads, d_out_h_eval, vk_repr, d_out_status);
}

// Host-buffer variants share one staging layout in acc_io:
// points | scalars | challenges | quads | h_eval | status.
static int transcript_host(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4],
                           const uint64_t* points, const uint64_t* scalars, uint64_t* out_challenges,
                           uint64_t* out_quads, uint64_t* out_h_eval, uint32_t* out_status, bool accum) {
  if (!ctx || !shape || !vk_repr || (B && (!points || !scalars || (accum ? !out_quads : !out_challenges))))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (B == 0) return PM_OK;
  if (B > (1u << 20)) return set_error(PM_ERR_UNSUPPORTED, "transcript batch larger than 2^20 proofs");
  if ((rc = ctx->begin_call())) return rc;
  const size_t bp = B * npts * 64, bs = B * nsc * 32, bc = B * 7 * 32, bo = B * 4 * 64, bh = B * 32, bst = B * 4;
  if ((rc = ctx->acc_io.ensure(bp + bs + bc + bo + bh + bst))) return rc;
  char* dp = (char*)ctx->acc_io.p;
  char* ds = dp + bp;
  char* dc = ds + bs;
  char* dq = dc + bc;
  char* dh = dq + bo;
  char* dst = dh + bh;
  HIP_TRY(hipMemcpyAsync(dp, points, bp, hipMemcpyHostToDevice, ctx->stream));
  HIP_TRY(hipMemcpyAsync(ds, scalars, bs, hipMemcpyHostToDevice, ctx->stream));
  if (accum) {
    if ((rc = ops->accum(ctx, shape, B, dp, ds, dc, dq, dh, vk_repr, dst))) return rc;
  } else if ((rc = ops->transcript(ctx, shape, B, vk_repr, dp, ds, dc, dst))) {
    return rc;
  }
  if (out_challenges) HIP_TRY(hipMemcpyAsync(out_challenges, dc, bc, hipMemcpyDeviceToHost, ctx->stream));
  if (accum) HIP_TRY(hipMemcpyAsync(out_quads, dq, bo, hipMemcpyDeviceToHost, ctx->stream));
  if (accum && out_h_eval) HIP_TRY(hipMemcpyAsync(out_h_eval, dh, bh, hipMemcpyDeviceToHost, ctx->stream));
  if (out_status) HIP_TRY(hipMemcpyAsync(out_status, dst, bst, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  if (!accum) ctx->end_call();
  return PM_OK;
}

int pm_transcript_batch(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4],
                        const uint64_t* points, const uint64_t* scalars, uint64_t* out_challenges,
                        uint32_t* out_status) {
  return transcript_host(ctx, curve, shape, B, vk_repr, points, scalars, out_challenges, nullptr, nullptr,
                         out_status, false);
}

int pm_accum_batch_transcript(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                              const uint64_t vk_repr[4], const uint64_t* points, const uint64_t* scalars,
                              uint64_t* out_challenges, uint64_t* out_quads, uint64_t* out_h_eval,
                              uint32_t* out_status) {
  return transcript_host(ctx, curve, shape, B, vk_repr, points, scalars, out_challenges, out_quads, out_h_eval,
                         out_status, true);
}

// ------------------------------------------------- proof bytes (read_point / read_scalar)
int pm_proof_size(const pm_proof_shape* shape, size_t* bytes) {
  if (!shape || !bytes) return set_error(PM_ERR_ARG, "null argument");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  *bytes = 32ull * (npts - shape->num_instance_columns + nsc);
  return PM_OK;
}

int pm_decode_proofs_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const void* d_proofs,
                            size_t stride, const void* d_instance_points, void* d_out_points, void* d_out_scalars,
                            void* d_out_status) {
  if (!ctx || !shape || (B && (!d_proofs || !d_out_points || !d_out_scalars || !d_out_status)) ||
      (B && shape->num_instance_columns && !d_instance_points))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  std::lock_guard<std::mutex> lk(ctx->mu);
  int rc = ctx->begin_call();
  if (rc) return rc;
  return ops->proofs(ctx, shape, B, d_proofs, stride, d_instance_points, d_out_points, d_out_scalars, d_out_status,
                     nullptr, nullptr, nullptr, nullptr);
}

int pm_accum_batch_proofs_device(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B,
                                 const uint64_t vk_repr[4], const void* d_proofs, size_t stride,
                                 const void* d_instance_points, void* d_challenges, void* d_out_quads,
                                 void* d_out_h_eval, void* d_out_status) {
  if (!ctx || !shape || !vk_repr || (B && (!d_proofs || !d_challenges || !d_out_quads)) ||
      (B && shape->num_instance_columns && !d_instance_points))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (B == 0) return PM_OK;
  if ((rc = ctx->begin_call())) return rc;
  // decoded points / scalars (and the status words when the caller passes none) in context scratch
  const size_t bp = B * npts * 64, bs = B * nsc * 32, bst = B * 4;
  if ((rc = ctx->pf_io.ensure(bp + bs + bst))) return rc;
  char* dp = (char*)ctx->pf_io.p;
  return ops->proofs(ctx, shape, B, d_proofs, stride, d_instance_points, dp, dp + bp,
                     d_out_status ? d_out_status : dp + bp + bs, vk_repr, d_challenges, d_out_quads, d_out_h_eval);
}

// Host-buffer variants: proofs | instance points | decoded points | decoded
// scalars | challenges | quads | h_eval | status in pf_io.
static int proofs_host(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t* vk_repr,
                       const uint8_t* proofs, size_t stride, const uint64_t* inst, uint64_t* out_points,
                       uint64_t* out_scalars, uint64_t* out_challenges, uint64_t* out_quads, uint64_t* out_h_eval,
                       uint32_t* out_status) {
  const bool accum = vk_repr != nullptr;
  if (!ctx || !shape || (B && !proofs) || (B && shape->num_instance_columns && !inst) ||
      (B && (accum ? !out_quads : (!out_points || !out_scalars))))
    return set_error(PM_ERR_ARG, "null argument");
  const CurveOps* ops = curve_ops(curve);
  if (!ops) return set_error(PM_ERR_ARG, "unknown curve id");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  size_t psize = 0;
  if ((rc = pm_proof_size(shape, &psize))) return rc;
  if (stride < psize) return set_error(PM_ERR_ARG, "proof stride below the proof size");
  std::lock_guard<std::mutex> lk(ctx->mu);
  if (B == 0) return PM_OK;
  if (B > (1u << 20)) return set_error(PM_ERR_UNSUPPORTED, "proof batch larger than 2^20 proofs");
  if ((rc = ctx->begin_call())) return rc;
  const size_t ni = shape->num_instance_columns;
  const size_t bpf = (B * psize + 255) & ~size_t(255), bin = (B * ni * 64 + 255) & ~size_t(255);
  const size_t bp = B * npts * 64, bs = B * nsc * 32, bc = B * 7 * 32, bo = B * 4 * 64, bh = B * 32, bst = B * 4;
  if ((rc = ctx->pf_io.ensure(bpf + bin + bp + bs + bc + bo + bh + bst))) return rc;
  char* dpf = (char*)ctx->pf_io.p;
  char* din = dpf + bpf;
  char* dp = din + bin;
  char* ds = dp + bp;
  char* dc = ds + bs;
  char* dq = dc + bc;
  char* dh = dq + bo;
  char* dst = dh + bh;
  // the proofs packed densely (stride = psize) for the device
  if (stride == psize) {
    HIP_TRY(hipMemcpyAsync(dpf, proofs, B * psize, hipMemcpyHostToDevice, ctx->stream));
  } else {
    HIP_TRY(hipMemcpy2DAsync(dpf, psize, proofs, stride, psize, B, hipMemcpyHostToDevice, ctx->stream));
  }
  if (ni) HIP_TRY(hipMemcpyAsync(din, inst, B * ni * 64, hipMemcpyHostToDevice, ctx->stream));
  if ((rc = ops->proofs(ctx, shape, B, dpf, psize, din, dp, ds, dst, vk_repr, dc, dq, dh))) return rc;
  if (out_points) HIP_TRY(hipMemcpyAsync(out_points, dp, bp, hipMemcpyDeviceToHost, ctx->stream));
  if (out_scalars) HIP_TRY(hipMemcpyAsync(out_scalars, ds, bs, hipMemcpyDeviceToHost, ctx->stream));
  if (accum && out_challenges) HIP_TRY(hipMemcpyAsync(out_challenges, dc, bc, hipMemcpyDeviceToHost, ctx->stream));
  if (accum) HIP_TRY(hipMemcpyAsync(out_quads, dq, bo, hipMemcpyDeviceToHost, ctx->stream));
  if (accum && out_h_eval) HIP_TRY(hipMemcpyAsync(out_h_eval, dh, bh, hipMemcpyDeviceToHost, ctx->stream));
  if (out_status) HIP_TRY(hipMemcpyAsync(out_status, dst, bst, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  return PM_OK;
}

int pm_decode_proofs(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint8_t* proofs,
                     size_t stride, const uint64_t* instance_points, uint64_t* out_points, uint64_t* out_scalars,
                     uint32_t* out_status) {
  return proofs_host(ctx, curve, shape, B, nullptr, proofs, stride, instance_points, out_points, out_scalars, nullptr,
                     nullptr, nullptr, out_status);
}

int pm_accum_batch_proofs(pm_ctx* ctx, int curve, const pm_proof_shape* shape, size_t B, const uint64_t vk_repr[4],
                          const uint8_t* proofs, size_t stride, const uint64_t* instance_points,
                          uint64_t* out_challenges, uint64_t* out_quads, uint64_t* out_h_eval, uint32_t* out_status) {
  if (!vk_repr) return set_error(PM_ERR_ARG, "null argument");
  return proofs_host(ctx, curve, shape, B, vk_repr, proofs, stride, instance_points, nullptr, nullptr,
                     out_challenges, out_quads, out_h_eval, out_status);
}

// Proof batch sharded over several contexts (devices) in one process: proofs
// are independent, so context k takes the contiguous range
// [k*per, (k+1)*per) and runs the single-context host entry on it in its own
// thread; the outputs land in place.  challenges == NULL replays the
// transcript (vk_repr required), else vk_repr is ignored.
int pm_accum_batch_multi(pm_ctx* const* ctxs, int nctx, int curve, const pm_proof_shape* shape, size_t B,
                         const uint64_t* points, const uint64_t* scalars, const uint64_t* challenges,
                         const uint64_t vk_repr[4], uint64_t* out_challenges, uint64_t* out_quads,
                         uint64_t* out_h_eval, uint32_t* out_status) {
  if (!ctxs || nctx < 1 || !shape || (B && (!points || !scalars || !out_quads)) || (!challenges && !vk_repr))
    return set_error(PM_ERR_ARG, "null argument");
  for (int k = 0; k < nctx; k++)
    if (!ctxs[k]) return set_error(PM_ERR_ARG, "null context");
  if (!valid_curve(curve)) return set_error(PM_ERR_ARG, "unknown curve id");
  uint32_t npts = 0, nsc = 0, ns = 0;
  int rc = pm_shape_layout(shape, &npts, &nsc, &ns);
  if (rc) return rc;
  if (B == 0) return PM_OK;
  const size_t per = (B + nctx - 1) / nctx;
  std::vector<int> rcs(nctx, PM_OK);
  std::vector<std::string> errs(nctx);
  std::vector<std::thread> th;
  for (int k = 0; k < nctx; k++) {
    const size_t lo = std::min(B, per * k), cnt = std::min(B, lo + per) - lo;
    if (cnt == 0) continue;
    th.emplace_back([&, k, lo, cnt] {
      const uint64_t* p = points + lo * npts * 8;
      const uint64_t* sc = scalars + lo * nsc * 4;
      uint64_t* q = out_quads + lo * 32;
      uint64_t* h = out_h_eval ? out_h_eval + lo * 4 : nullptr;
      uint32_t* st = out_status ? out_status + lo : nullptr;
      int r;
      if (challenges)
        r = pm_accum_batch(ctxs[k], curve, shape, cnt, p, sc, challenges + lo * 28, q, h, st);
      else
        r = pm_accum_batch_transcript(ctxs[k], curve, shape, cnt, vk_repr, p, sc,
                                      out_challenges ? out_challenges + lo * 28 : nullptr, q, h, st);
      rcs[k] = r;
      if (r) errs[k] = pm::g_last_error;
    });
  }
  for (auto& t : th) t.join();
  for (int k = 0; k < nctx; k++)
    if (rcs[k]) return set_error(rcs[k], "context " + std::to_string(k) + ": " + errs[k]);
  if (challenges && out_challenges) std::memcpy(out_challenges, challenges, B * 7 * 32);
  return PM_OK;
}

}  // extern "C"

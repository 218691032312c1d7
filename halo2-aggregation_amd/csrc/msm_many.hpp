// msm_many.hpp -- many independent short MSMs against one resident base set
// (pm_msm_resident_many*).
//
// The aggregator commits every inner proof's instance column on its own:
// params_verifier.commit_lagrange(public_inputs) (examples/simple-example.rs:
// 632-641), a best_multiexp of the public inputs against the first bases of
// params.g_lagrange [3P], whose result the verifier then takes as the
// instance commitment (src/verifier.rs:200-225, 312-316).  One proof has a
// handful of public inputs (simple-example: one), so B proofs are B MSMs of
// n_i ~ 1..64 terms -- as separate pm_msm calls ~60 us each, 25x the batch
// accumulator that consumes them (What's missing #1).
//
// Here the bases are the SRS, resident and fixed, so the serial part of a
// variable-base MSM (the ~128 doublings of a Horner over windows) moves into
// a one-time table:
//   multiples table (built once per base set and prefix, k_many_pow +
//   k_many_mult): entry (i, w, m) = [m 2^{c w}] P_i, m = 1 .. H = 2^(c-1),
//   for windows w < W(c) of c bits, XYZZ in the pipeline's R = 2^261 form
//   (128 B; identity bases give identity entries).
//   sum (k_many_sum, one launch for all B MSMs): a scalar's signed c-bit
//   digits d_w in [-(H-1), H] select W table entries, so
//     MSM_i = sum_{t < n_i} sum_{w < W} sign(d_tw) T[o_i + t][w][|d_tw|]
//   is a plain sum of n_i W points -- no doublings anywhere.  Block = (MSM,
//   slice of its terms); each quad adds kq consecutive terms with
//   quad-cooperative additions (coop29.hpp), the 64 quads fold in LDS
//   (small_tree), several slices of one MSM are folded by its last block
//   (atomic ticket).  Results go out XYZZ (R = 2^256) into mapped host
//   memory; the host converts all B to affine with one inversion
//   (Montgomery's trick) and spins on a completion flag the last MSM raises.
// Latency at n_i = 1 and c = 8: one addition per quad, a 5-level tree; no
// ladder, no host Horner.  Throughput: W(c) additions per scalar (32 at c = 8).
#pragma once
#include "engine.hpp"

namespace pm {

constexpr uint32_t kManyQuads = 64;          // quads per block (256 threads)
constexpr uint32_t kManyQuadBudget = 32768;  // quads in flight: ~2 waves per SIMD of the 1024
constexpr size_t kManyMappedBytes = size_t(64) << 10;  // host scalars up to this are read from mapped memory
struct ManyJob {
  uint32_t msm;    // MSM index (output slot)
  uint32_t e0;     // first term of the slice (term e = t W + w)
  uint32_t e1;     // one past its last
  uint32_t slice;  // slice index within the MSM
};
struct ManyMsm {
  uint32_t s_off;  // first scalar in the concatenated scalar array
  uint32_t b_off;  // first base (row of the table)
  uint32_t ns;     // slices
  uint32_t job0;   // index of its first job (its partials sit at part[job0 ..])
};
struct ManySumGeom {
  uint32_t c, W, H;
  uint32_t kq;         // terms per quad and slice
  uint32_t canonical;  // scalars canonical (else Montgomery R = 2^256)
  uint32_t nout;       // MSMs with at least one term (the completion count)
};

// ------------------------------------------------------------ table build
// lane i: [2^{c w}] P_i for every window, by Jacobian doublings (the chain
// starts at an affine non-identity point of odd order: never O), stored at
// entry (i, w, 1).  Identity bases store the identity (all-zero words).
template <class F>
__global__ void __launch_bounds__(256) k_many_pow(const uint32_t* __restrict__ bases29, uint32_t n, uint32_t c,
                                                  uint32_t W, uint32_t H, Xyzz<F>* __restrict__ tab) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  F29<F> x, y;
  load_aff29<F>(bases29 + 16ull * i, x, y);
  Xyzz<F>* row = tab + (size_t)i * W * H;
  if (f29_is_zero_exact<F>(x) && f29_is_zero_exact<F>(y)) {
    const Xyzz29<F> z{f29_zero<F>(), f29_zero<F>(), f29_zero<F>(), f29_zero<F>()};
    for (uint32_t w = 0; w < W; w++) store_xyzz29<F>(&row[(size_t)w * H], z);
    return;
  }
  const F29<F> one = f29_const<F>(F29Consts<F>::ONE);
  store_xyzz29<F>(&row[0], Xyzz29<F>{x, y, one, one});
  Jac29<F> J{x, y, one};
  for (uint32_t w = 1; w < W; w++) {
    for (uint32_t k = 0; k < c; k++) J = jac29_dbl<F>(J);
    store_xyzz29<F>(&row[(size_t)w * H], jac29_to_xyzz<F>(J));
  }
}

// lane (i, w): entries m = 2 .. H from entry 1 (Q): [2]Q, then + Q.  mQ is
// never +-Q or O for 2 <= m <= H < r, so only the identity Q needs care
// (xyzz29_add passes it through: every entry stays the identity).
template <class F>
__global__ void __launch_bounds__(256) k_many_mult(uint32_t nw, uint32_t H, Xyzz<F>* __restrict__ tab) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= nw || H < 2) return;
  Xyzz<F>* e = tab + (size_t)g * H;
  const Xyzz29<F> Q = load_xyzz29<F>(e);
  Xyzz29<F> M = xyzz29_is_inf<F>(Q) ? Q : xyzz29_dbl<F>(Q);
  store_xyzz29<F>(&e[1], M);
  for (uint32_t m = 3; m <= H; m++) {
    M = xyzz29_add<F>(M, Q);
    store_xyzz29<F>(&e[m - 1], M);
  }
}

// ------------------------------------------------------------------ sum
// c-bit field of k at bit offset b (bits past 255 read as zero); k is a
// register array, so the word index is resolved with selects, not scratch
__device__ __forceinline__ uint32_t many_bits(const uint32_t (&k)[8], uint32_t b, uint32_t c) {
  const uint32_t wd = b >> 5, sh = b & 31u;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    lo = (uint32_t)j == wd ? k[j] : lo;
    hi = (uint32_t)j == wd + 1u ? k[j] : hi;
  }
  const uint64_t v = ((uint64_t)hi << 32 | lo) >> sh;
  return (uint32_t)v & ((1u << c) - 1u);
}

// lane q of a quad stores coordinate q of p in the R = 2^256 packed layout
// (canonical), the host's form (host_ec.hpp Pt); the identity stays ZZ = 0
template <class F>
__device__ __forceinline__ void store_xyzz_r256_q(Xyzz<F>* dst, const Xyzz29<F>& p, uint32_t q) {
  uint32_t o[8];
  f29_to_r256<F>(qsel<F>(q, p.X, p.Y, p.ZZ, p.ZZZ), o);
  uint4* d = reinterpret_cast<uint4*>(dst) + 2 * q;
  d[0] = make_uint4(o[0], o[1], o[2], o[3]);
  d[1] = make_uint4(o[4], o[5], o[6], o[7]);
}

// block = job (one slice of one MSM's terms); quad v adds terms [e0 + v kq,
// e0 + (v + 1) kq) of it.  Terms of one scalar are consecutive (e = t W + w),
// so a quad reloads and re-splits a scalar only when t changes; the digit
// carry into the quad's first window is recomputed from window 0 (integer
// work only).  Every branch below is quad-uniform.
template <class Cv>
__global__ void __launch_bounds__(256) k_many_sum(ManySumGeom g, const ManyJob* __restrict__ jobs,
                                                  const ManyMsm* __restrict__ msms, const uint32_t* __restrict__ scalars,
                                                  const Xyzz<typename Cv::Base>* __restrict__ tab,
                                                  Xyzz<typename Cv::Base>* __restrict__ part,
                                                  uint32_t* __restrict__ tickets, Xyzz<typename Cv::Base>* __restrict__ out,
                                                  uint32_t* __restrict__ done, uint32_t* __restrict__ flag, uint32_t seq) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  using K = F29Consts<F>;
  __shared__ uint32_t s_p[kManyQuads][kSmallPt];
  __shared__ uint32_t last;
  const ManyJob jb = jobs[blockIdx.x];
  const ManyMsm ms = msms[jb.msm];
  const uint32_t v = threadIdx.x >> 2, q = threadIdx.x & 3u;
  const uint32_t e0 = jb.e0 + v * g.kq;
  const uint32_t e1 = min(e0 + g.kq, jb.e1);
  Xyzz29<F> acc = xyzz29_inf<F>();
  uint32_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  uint32_t cur = ~0u, carry = 0, nextw = 0;
  for (uint32_t e = e0; e < e1; e++) {
    const uint32_t t = e / g.W, w = e - t * g.W;
    if (t != cur) {
      cur = t;
      Fe<Fs> s = load_fe4<Fs>(reinterpret_cast<const uint4*>(scalars + 8ull * (ms.s_off + t)));
      s = g.canonical ? fe_reduce_full<Fs>(s) : fe_from_mont<Fs>(s);
#pragma unroll
      for (int j = 0; j < 8; j++) k[j] = s.l[j];
      carry = 0;
      nextw = 0;
    }
    for (; nextw < w; nextw++) carry = many_bits(k, nextw * g.c, g.c) + carry > g.H ? 1u : 0u;
    const uint32_t u = many_bits(k, w * g.c, g.c) + carry;
    carry = u > g.H ? 1u : 0u;
    nextw = w + 1;
    const int d = (int)u - (carry ? (int)(2u * g.H) : 0);
    if (d != 0) {
      const uint32_t m = (uint32_t)(d < 0 ? -d : d);
      Xyzz29<F> P = load_xyzz29<F>(&tab[((size_t)(ms.b_off + t) * g.W + w) * g.H + m - 1u]);
      if (d < 0) P.Y = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), P.Y, K::K6)));  // < 3p
      acc = xyzz29_add_q<F>(acc, P);
    }
  }
  // quads holding at least one term
  const uint32_t span = jb.e1 - jb.e0;
  const uint32_t active = min((span + g.kq - 1u) / g.kq, kManyQuads);
  acc = small_tree<F>(s_p, acc, v, q, small_pow2(active));
  if (ms.ns > 1) {  // park the slice's sum; the MSM's last block folds them
    if (v == 0) {
      store_xyzz29_q<F>(&part[blockIdx.x], acc, q);  // = part[ms.job0 + jb.slice]
      __threadfence();
      if (q == 0) last = atomicAdd(&tickets[jb.msm], 1u) == ms.ns - 1u;
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    acc = xyzz29_inf<F>();
    for (uint32_t u2 = v; u2 < ms.ns; u2 += kManyQuads) acc = xyzz29_add_q<F>(acc, load_xyzz29<F>(&part[ms.job0 + u2]));
    acc = small_tree<F>(s_p, acc, v, q, small_pow2(min(ms.ns, kManyQuads)));
    if (v == 0 && q == 0) tickets[jb.msm] = 0;  // ready for the next call
  }
  if (v == 0) {
    store_xyzz_r256_q<F>(&out[jb.msm], acc, q);
    __threadfence_system();
    if (q == 0 && atomicAdd(done, 1u) == g.nout - 1u) {
      *done = 0;  // every MSM has counted: ready for the next call
      __threadfence_system();
      *(volatile uint32_t*)flag = seq;
    }
  }
}

// ------------------------------------------------------------------ host
template <class Cv>
int many_table_impl(Ctx* ctx, const void* d_bases29, size_t n, ManyTable* t) {
  using F = typename Cv::Base;
  const uint32_t c = many_pick_c(n), W = many_windows(c), H = 1u << (c - 1);
  const size_t bytes = n * many_bytes_per_base(c);
  if (bytes > kManyTabCap) return set_error(PM_ERR_UNSUPPORTED, "many-MSM table above its memory cap");
  void* d = nullptr;
  HIP_TRY(hipMalloc(&d, std::max<size_t>(bytes, 128)));
  const hipStream_t st = ctx->stream;
  k_many_pow<F><<<(unsigned)((n + 255) / 256), 256, 0, st>>>((const uint32_t*)d_bases29, (uint32_t)n, c, W, H,
                                                             (Xyzz<F>*)d);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    const size_t nw = n * W;
    k_many_mult<F><<<(unsigned)((nw + 255) / 256), 256, 0, st>>>((uint32_t)nw, H, (Xyzz<F>*)d);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) {
    (void)hipFree(d);
    return set_error(PM_ERR_HIP, std::string("many-MSM table build: ") + hipGetErrorString(e));
  }
  if (t->d) (void)hipFree(t->d);
  t->d = d;
  t->n = n;
  t->c = c;
  t->W = W;
  t->H = H;
  return PM_OK;
}

// XYZZ (R = 2^256, canonical) -> affine for all outputs with one inversion
// (Montgomery's trick over ZZZ; x = X (ZZ / ZZZ)^2, y = Y / ZZZ)
template <class F, bool ADX>
void many_to_affine(const Xyzz<F>* R, const std::vector<uint32_t>& slot, uint64_t* out) {
  using E = host::E<F>;
  const size_t B = slot.size();
  std::vector<E> pre;
  pre.reserve(B);
  std::vector<uint32_t> live;
  live.reserve(B);
  E acc{};
  for (size_t i = 0; i < B; i++) {
    std::memset(out + 8 * i, 0, 64);
    if (slot[i] == ~0u) continue;
    const host::Pt<F> p = host::from_dev<F>(R[slot[i]]);
    if (host::is_zero(p.ZZ)) continue;
    acc = live.empty() ? p.ZZZ : host::mulv<F, ADX>(acc, p.ZZZ);
    pre.push_back(acc);
    live.push_back((uint32_t)i);
  }
  if (live.empty()) return;
  Fe<F> a;
  std::memcpy(&a, &acc, 32);
  const Fe<F> ia = fe_inv_bgcd<F>(a);
  E inv;
  std::memcpy(&inv, &ia, 32);
  for (size_t j = live.size(); j-- > 0;) {
    const size_t i = live[j];
    const host::Pt<F> p = host::from_dev<F>(R[slot[i]]);
    const E izzz = j ? host::mulv<F, ADX>(inv, pre[j - 1]) : inv;  // 1 / ZZZ_j
    if (j) inv = host::mulv<F, ADX>(inv, p.ZZZ);
    const E iz = host::mulv<F, ADX>(p.ZZ, izzz);  // 1 / Z
    const E x = host::mulv<F, ADX>(p.X, host::mulv<F, ADX>(iz, iz));
    const E y = host::mulv<F, ADX>(p.Y, izzz);
    std::memcpy(out + 8 * i, x.v, 32);
    std::memcpy(out + 8 * i + 4, y.v, 32);
  }
}
template <class F>
__attribute__((target("bmi2,adx"))) void many_to_affine_bmi2(const Xyzz<F>* R, const std::vector<uint32_t>& slot,
                                                             uint64_t* out) {
  many_to_affine<F, true>(R, slot, out);
}

// B MSMs: MSM i = sum_{t < n[i]} s[t] P[off[i] + t] with s the next n[i]
// scalars of the concatenated array (host or device), against the table t
// (which covers every off[i] + n[i]).  out: B affine points (8 u64 each).
template <class Cv>
int msm_many_impl(Ctx* ctx, const ManyTable* tb, size_t B, const size_t* n, const size_t* off, const void* scalars,
                  bool s_host, uint32_t flags, uint64_t* out) {
  using F = typename Cv::Base;
  const hipStream_t st = ctx->stream;
  size_t total_s = 0, total_e = 0;
  for (size_t i = 0; i < B; i++) {
    total_s += n[i];
    total_e += n[i] * tb->W;
  }
  if (total_s >= (size_t(1) << 31) || total_e >= (size_t(1) << 32) - (size_t)64 * tb->W)
    return set_error(PM_ERR_UNSUPPORTED, "many-MSM call above 2^31 scalars");
  ManySumGeom g{};
  g.c = tb->c;
  g.W = tb->W;
  g.H = tb->H;
  g.canonical = (flags & PM_SCALARS_CANONICAL) ? 1u : 0u;
  g.kq = (uint32_t)std::max<size_t>(1, (total_e + kManyQuadBudget - 1) / kManyQuadBudget);
  const size_t per = (size_t)kManyQuads * g.kq;
  std::vector<ManyJob> jobs;
  std::vector<ManyMsm> msms;
  std::vector<uint32_t> slot(B, ~0u);  // output slot of MSM i (~0: no terms, the identity)
  size_t s_off = 0;
  for (size_t i = 0; i < B; i++) {
    const size_t te = n[i] * tb->W;
    if (te) {
      slot[i] = (uint32_t)msms.size();
      const uint32_t ns = (uint32_t)((te + per - 1) / per);
      msms.push_back(ManyMsm{(uint32_t)s_off, (uint32_t)(off ? off[i] : 0), ns, (uint32_t)jobs.size()});
      for (uint32_t s = 0; s < ns; s++)
        jobs.push_back(ManyJob{(uint32_t)(msms.size() - 1), (uint32_t)(s * per), (uint32_t)std::min(te, (s + 1) * per), s});
    }
    s_off += n[i];
  }
  g.nout = (uint32_t)msms.size();
  if (msms.empty()) {
    std::memset(out, 0, 64 * B);
    return PM_OK;
  }
  int rc;
  // job and MSM tables in one upload (cached: a repeated batch shape re-sends nothing)
  std::vector<uint32_t> prog;
  prog.reserve(4 * (jobs.size() + msms.size()));
  for (auto& j : jobs) prog.insert(prog.end(), {j.msm, j.e0, j.e1, j.slice});
  for (auto& m : msms) prog.insert(prog.end(), {m.s_off, m.b_off, m.ns, m.job0});
  if ((rc = ctx->many_prog.put(prog, st))) return rc;
  const ManyJob* djobs = (const ManyJob*)ctx->many_prog.buf.p;
  const ManyMsm* dmsms = (const ManyMsm*)((const uint32_t*)ctx->many_prog.buf.p + 4 * jobs.size());
  // scalars: small host batches are read by the kernel straight from mapped
  // pinned memory (no DMA launch), larger ones are copied
  const uint32_t* ds = (const uint32_t*)scalars;
  if (s_host) {
    const size_t sb = total_s * 32;
    if (sb <= kManyMappedBytes) {
      if ((rc = ctx->ensure_small_pin(sb))) return rc;
      std::memcpy(ctx->small_pin, scalars, sb);
      ds = (const uint32_t*)ctx->small_pin_dev;
    } else {
      if ((rc = ctx->in_scalars.ensure(sb)) || (rc = ctx->upload_h2d(ctx->in_scalars.p, scalars, sb, st))) return rc;
      ds = (const uint32_t*)ctx->in_scalars.p;
    }
  }
  if ((rc = ctx->small_part.ensure(jobs.size() * sizeof(Xyzz<F>)))) return rc;
  // tickets per MSM + the done count (self-resetting; zero fresh allocations)
  const size_t old_cap = ctx->small_tk.cap;
  if ((rc = ctx->small_tk.ensure((msms.size() + 1) * 4))) return rc;
  if (ctx->small_tk.cap != old_cap) HIP_TRY(hipMemsetAsync(ctx->small_tk.p, 0, ctx->small_tk.cap, st));
  uint32_t* tickets = (uint32_t*)ctx->small_tk.p;
  uint32_t* dcount = tickets + msms.size();
  if ((rc = ctx->ensure_pinned(msms.size() * sizeof(Xyzz<F>) + 64))) return rc;
  if ((rc = ctx->ensure_group_events(1))) return rc;
  Xyzz<F>* hR = (Xyzz<F>*)ctx->h_pinned;
  volatile uint32_t* hflag = (volatile uint32_t*)(hR + msms.size());
  *hflag = 0;
  const uint32_t seq = ++ctx->small_seq ? ctx->small_seq : ++ctx->small_seq;
  void* dR = ctx->h_pinned_dev;
  uint32_t* dflag = (uint32_t*)((Xyzz<F>*)dR + msms.size());
  PM_LAUNCH(ctx, "many_sum",
            (k_many_sum<Cv><<<(unsigned)jobs.size(), 256, 0, st>>>(g, djobs, dmsms, ds, (const Xyzz<F>*)tb->d,
                                                                   (Xyzz<F>*)ctx->small_part.p, tickets, (Xyzz<F>*)dR,
                                                                   dcount, dflag, seq)));
  hipEvent_t ev = ctx->grp_ev[0];
  HIP_TRY(hipEventRecord(ev, st));
  if (ctx->timing) {
    if ((rc = wait_event(ctx, ev))) return rc;
  } else {
    for (uint32_t it = 1;; it++) {
      if (__atomic_load_n((const uint32_t*)hflag, __ATOMIC_ACQUIRE) == seq) break;
      if ((it & 1023u) == 0) {
        const hipError_t qe = hipEventQuery(ev);
        if (qe == hipSuccess) {
          if (*hflag != seq) {
            (void)hipMemsetAsync(ctx->small_tk.p, 0, ctx->small_tk.cap, st);
            (void)hipStreamSynchronize(st);
            return set_error(PM_ERR_HIP, "many MSM: kernel finished without the completion flag");
          }
          break;
        }
        if (qe != hipErrorNotReady) return set_error(PM_ERR_HIP, std::string("many MSM: ") + hipGetErrorString(qe));
      }
      __builtin_ia32_pause();
    }
  }
  const auto t0 = std::chrono::steady_clock::now();
  if (host_has_bmi2()) many_to_affine_bmi2<F>(hR, slot, out);
  else many_to_affine<F, false>(hR, slot, out);
  if (ctx->timing) {
    auto& stt = ctx->stats["host_tail"];
    stt.first += 1;
    stt.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return ctx->end_call();
}

}  // namespace pm

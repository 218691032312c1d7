// accum_engine.hpp -- host driver of the batch multiopen accumulator
// (instantiated once per curve next to the MSM engine).
//
// Boundary: pm_accum_batch / pm_accum_batch_device (include/pasta_msm.h),
// replacing the native meaning of VerifierChip::_verify_proof's scalar block
// + MultiopenChip::calc_witness (/root/reference/src/verifier.rs:512-733,
// src/multiopen.rs:271-509).
#pragma once
#include <functional>
#include <vector>
#include <hip/hip_ext.h>

#include "accum_kernels.hpp"
#include "engine.hpp"
#include "selftest.hpp"
#include "transcript_kernels.hpp"
#include "proof_kernels.hpp"

namespace pm {

template <class Fs>
Fe<Fs> fe_from_u64(const uint64_t* p) {
  Fe<Fs> r;
  for (int k = 0; k < 4; k++) {
    r.l[2 * k] = (uint32_t)p[k];
    r.l[2 * k + 1] = (uint32_t)(p[k] >> 32);
  }
  return r;
}
template <class Fs>
Fe<Fs> fe_pow_u64(Fe<Fs> a, uint64_t e) {
  Fe<Fs> r = fe_one<Fs>();
  while (e) {
    if (e & 1) r = fe_mul<Fs>(r, a);
    a = fe_sqr<Fs>(a);
    e >>= 1;
  }
  return r;
}
template <class Fs>
void push_fe(std::vector<uint32_t>& v, const Fe<Fs>& a) {
  for (int i = 0; i < 8; i++) v.push_back(a.l[i]);
}

template <class Cv>
int transcript_device_impl(Ctx* ctx, const pm_proof_shape* s, size_t B, const uint64_t vk_repr[4], const void* d_points,
                           const void* d_scalars, void* d_ch, void* d_status);
// canon_ready: the canonical coordinates / scalars the replay hashes are
// already in ctx->tr_canon (written by k_proof_decode), so k_tr_canon is
// skipped; dflags: the decoder's per-proof flags, OR-ed into d_status by the
// replay, which clears them
template <class Cv>
int transcript_launch(Ctx* ctx, const pm_proof_shape* s, size_t B, const uint64_t vk_repr[4], const void* d_points,
                      const void* d_scalars, void* d_ch, void* d_status, hipStream_t st, bool canon_ready = false,
                      uint32_t* dflags = nullptr);

// Lanes per item for the latency-bound accumulator kernels: the largest
// power of two 2^lg <= 2^maxlg that keeps items * 2^lg within about two
// waves per SIMD of the 1024 on an MI355X.  Term additions: maxlg = 3 (8
// lanes share a term's ~85 table additions; 16 measured no faster at B = 256,
// the wider butterfly and the second wave per SIMD cost what the shorter loop
// saves).
constexpr size_t kAccLaneBudget = 1024 * 2 * 64;
constexpr size_t kAccSumLanes = 16384;
// 152 KiB (round 5, was 128): k_acc_scalars' per-proof rows grew with wave
// 3's slot sums and the fold rows, and 32 proofs (config 5's rank slice)
// should still fit one block
constexpr size_t kAccScalarsLds = 152 * 1024;
// LDS fence: the transcript and k_acc_scalars blocks request kAccScalarsLds
// and every ladder block kAccLadderFence (unused), so the two can never share
// a CU (160 KiB per CU).  Both sides are single-wave latency chains; sharing
// a SIMD with a ladder wave doubled k_acc_scalars (0.14 -> 0.27 ms at
// B = 256).
constexpr size_t kAccLadderFence = 40 * 1024;
// (the quad ladder takes kAccSlicedFence, one block per CU, while its grid fits
// the CUs: beside the twisted ladder's decode on the other stream its blocks
// were otherwise packed two or three per CU, B = 256 ladder 0.27 -> 0.68 ms)
// row-sliced ladder (k_acc_powers_s) up to this many chains: one wave each,
// four per block and one block per CU (kAccSlicedFence), leaving CUs for the
// side stream's transcript / k_acc_scalars blocks (which a ladder block on
// every CU kept waiting until the ladder ended: B = 16 transcript 0.10 ->
// 0.27 ms with 64-thread ladder blocks, profiles/r05/ladder_ab/r05_lad_scaling.jsonl
// against r05_lad_b_auto.jsonl)
constexpr size_t kAccSlicedChains = 800;
constexpr size_t kAccSlicedFence = 84 * 1024;
static_assert(2 * kAccSlicedFence > 160 * 1024 && kAccSlicedFence + kAccScalarsLds > 160 * 1024,
              "one sliced ladder block per CU, no side-stream block beside it");
// row-sliced square roots (k_proof_decode<Cv, true>) up to this many points
// (four per wave: 1024 waves)
constexpr size_t kDecodeSlicedPoints = 4096;
static_assert(kAccScalarsLds + kAccLadderFence > 160 * 1024, "the fence must not fit beside k_acc_scalars");
inline uint32_t acc_auto_lanes(size_t items, uint32_t maxlg) {
  uint32_t lg = 0;
  while (lg < maxlg && (items << (lg + 1)) <= kAccLaneBudget) lg++;
  return lg;
}

// The MSM term slots of one proof (accum_device_impl's plan): one slot per
// distinct commitment of f in first-use order, then H's h_i, the W_j of w and
// of zw, and g1 for e; qprog = (slot, eval) per query in set order.
struct AccTerms {
  std::vector<uint32_t> termsrc;  // (kind << 28) | idx ; VK index space: fixed, sigma, g1
  std::vector<uint32_t> qprog;
  uint32_t nslots = 0, h_slot0 = 0, T = 0, Tp = 0;  // Tp: proof-point terms (the powers-table chains)
};
inline void acc_terms(const pm_proof_shape* s, const AccLayout& L, const std::vector<std::vector<AccQuery>>& sets,
                      AccTerms& t) {
  std::map<std::pair<uint32_t, uint32_t>, uint32_t> slot_of;
  auto vk_index = [&](uint32_t kind, uint32_t idx) -> uint32_t {
    return kind == kRefFixed ? idx : s->num_fixed_columns + idx;
  };
  for (auto& st : sets)
    for (auto& x : st) {
      uint32_t slot = kSlotH;
      if (x.ref_kind != kRefH) {
        auto key = std::make_pair(x.ref_kind, x.ref_idx);
        auto it = slot_of.find(key);
        if (it == slot_of.end()) {
          slot = (uint32_t)t.termsrc.size();
          slot_of[key] = slot;
          t.termsrc.push_back(x.ref_kind == kRefProof ? x.ref_idx : ((1u << 28) | vk_index(x.ref_kind, x.ref_idx)));
        } else {
          slot = it->second;
        }
      }
      t.qprog.push_back(slot);
      t.qprog.push_back(x.eval);
    }
  t.h_slot0 = (uint32_t)t.termsrc.size();
  for (uint32_t i = 0; i < s->quotient_degree; i++) t.termsrc.push_back(L.p_h + i);
  t.nslots = (uint32_t)t.termsrc.size();
  for (uint32_t j = 0; j < L.nsets; j++) t.termsrc.push_back(L.p_W + j);  // w
  for (uint32_t j = 0; j < L.nsets; j++) t.termsrc.push_back(L.p_W + j);  // zw
  t.termsrc.push_back((1u << 28) | (s->num_fixed_columns + s->n_perm_columns));  // e: g1
  t.T = (uint32_t)t.termsrc.size();
  t.Tp = 0;
  for (uint32_t v : t.termsrc) t.Tp += (v >> 28) == 0 ? 1u : 0u;
}

// log2 of the lanes per term of the split (powers-table) form, 0 = the
// one-lane GLV form.  The powers tables pay only while their chains stay
// within ~3/4 of the lane budget: beyond it the 127-doubling chains share
// SIMDs and queue, while the one-lane GLV products still run in one pass at
// a flat ~1.16 ms.  Simple shape, T = 30 of which 21 proof points, wall per
// batch (profiles/r02/vkt/): split 1.13 ms at B = 1024, 1.67 at 1536 against
// one-lane 1.54 / 1.57 (the old rule without VK tables, 4 B T <= budget:
// profiles/r02/xover/).
inline uint32_t acc_split_lanes(const Ctx* ctx, size_t B, const AccTerms& t) {
  const size_t nterm = B * t.T, nprf = B * t.Tp;
  uint32_t lgS = ctx->acc_split >= 0 ? (uint32_t)ctx->acc_split
                 : 4 * (nprf << 2) > 3 * kAccLaneBudget ? 0u
                                                        : acc_auto_lanes(nterm, 3);
  // 16 / 32 lanes per term only while the term additions still fit one wave
  // per SIMD (B = 16: k_acc_termadd 0.075 ms at 16 lanes, 0.061 at 32; B = 256
  // stays at 8 lanes: 0.129 ms, 16 lanes 0.138, 32 lanes 0.197:
  // profiles/r02/pow/timing_pow1.jsonl)
  if (ctx->acc_split < 0 && lgS == 3)
    while (lgS < 5 && (nterm << (lgS + 1)) <= kAccLaneBudget / 2) lgS++;
  return lgS;
}

// static LDS of a decode instantiation (the fence is the block's total)
template <class Cv, bool SLICED>
size_t decode_static_lds() {
  static const size_t v = [] {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(k_proof_decode<Cv, SLICED>)) == hipSuccess
               ? (size_t)a.sharedSizeBytes
               : kDecodeStaticLds;  // the non-sliced arrays: an upper bound
  }();
  return v;
}

// The proof-bytes entry's square-root decode (proof_kernels.hpp), launched
// by accum_device_impl on the stream (and with the LDS fence) it picks:
// beside the twisted ladder on the reduction stream when the powers tables
// are built (the ladder needs only the proofs' x bytes, acc_chain_start),
// else first on the main stream.  off_of: the byte offset within a proof of
// every point index read from the bytes (kAccNoByte: instance commitments).
struct AccDecode {
  std::function<int(hipStream_t, size_t, uint4*)> launch;  // (stream, LDS fence bytes, twist factors or null)
  const void* proofs;
  size_t stride;
  const void* inst;
  std::vector<uint32_t> off_of;
  bool sliced;         // row-sliced square roots (few points)
  hipEvent_t in_ready = nullptr;  // on st: the inputs are on the device (recorded before the decode)
  bool launched = false;          // the decode is already queued on st (it writes the twist factors)
  bool twist = false;             // the plan runs the twisted ladder beside it (proofs_device_impl)
};
// a decode block beside a ladder block would share its SIMDs (both are
// issue-bound lone-wave chains): its LDS request keeps it off any CU holding
// a ladder block (sliced 84 KiB, quad 40 KiB) or a side-stream block
constexpr size_t kDecodeFence = 124 * 1024;
// two decode blocks per CU, and none beside a ladder block fenced at
// kAccSlicedFence (84 KiB)
constexpr size_t kDecodePairFence = 80 * 1024;
static_assert(2 * kDecodePairFence <= 160 * 1024 && kDecodePairFence + kAccSlicedFence > 160 * 1024,
              "decode pair fence");

// vk_repr != nullptr: the challenges are first replayed into d_ch on the
// device (transcript_device_impl); the split ladder then runs concurrently
// with the replay and k_acc_scalars on the reduction stream.
template <class Cv>
int accum_device_impl(Ctx* ctx, const pm_proof_shape* s, size_t B, const void* d_points, const void* d_scalars,
                      void* d_ch, void* d_out, void* d_hout, const uint64_t* vk_repr, void* d_status,
                      bool canon_ready = false, uint32_t* dflags = nullptr, const AccDecode* dec = nullptr) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  const auto tplan = std::chrono::steady_clock::now();  // host planning (stat "accum_plan_host")
  std::vector<AccQuery> q;
  AccLayout L;
  const std::string err = acc_validate(s, q, L, nullptr);
  if (!err.empty()) return set_error(PM_ERR_ARG, "accum shape: " + err);
  if (B == 0) return PM_OK;
  if (B > (1u << 20)) return set_error(PM_ERR_UNSUPPORTED, "accum batch larger than 2^20 proofs");
  if (vk_repr && !d_ch) return set_error(PM_ERR_ARG, "null challenge buffer");

  std::vector<int32_t> rots;
  std::vector<std::vector<AccQuery>> sets;
  acc_group_sets(q, rots, sets);
  for (auto& st : sets)
    if (st.size() > kAccMaxPerSet) return set_error(PM_ERR_UNSUPPORTED, "accum: rotation set too large");

  // --- term slots (acc_terms)
  AccTerms tm;
  acc_terms(s, L, sets, tm);
  const std::vector<uint32_t>& termsrc = tm.termsrc;
  const std::vector<uint32_t>& qprog = tm.qprog;
  const uint32_t h_slot0 = tm.h_slot0, nslots = tm.nslots, T = tm.T;

  // --- program words
  AccumHdr h{};
  h.B = (uint32_t)B;
  h.npts = L.npts;
  h.nsc = L.nsc;
  h.T = T;
  h.nslots = nslots;
  h.nsets = L.nsets;
  h.log_n = s->log_n;
  h.bf = s->blinding_factors;
  h.num_lookups = s->num_lookups;
  h.n_perm_cols = s->n_perm_columns;
  h.perm_chunk = s->perm_chunk_len;
  h.n_perm_sets = L.n_perm_sets;
  h.sc_inst = L.s_inst;
  h.sc_adv = L.s_adv;
  h.sc_fixed = L.s_fixed;
  h.sc_rand = L.s_rand;
  h.sc_sigma = L.s_sigma;
  h.sc_perm = L.s_perm;
  h.sc_lk = L.s_lk;
  h.h_slot0 = h_slot0;
  h.nh = s->quotient_degree;
  std::vector<uint32_t> prog;
  auto put = [&](const uint32_t* p, uint32_t n, uint32_t& off, uint32_t& len) {
    off = (uint32_t)prog.size();
    len = n;
    for (uint32_t i = 0; i < n; i++) prog.push_back(p[i]);
  };
  put(s->gate_code, s->gate_code_len, h.p_gate, h.n_gate);
  put(s->lookup_input_code, s->lookup_input_code_len, h.p_lkin, h.n_lkin);
  put(s->lookup_table_code, s->lookup_table_code_len, h.p_lktab, h.n_lktab);
  h.p_permcol = (uint32_t)prog.size();
  for (uint32_t k = 0; k < s->n_perm_columns; k++) {
    const pm_perm_column& c = s->perm_columns[k];
    prog.push_back((c.kind == PM_COL_ADVICE ? L.s_adv : c.kind == PM_COL_FIXED ? L.s_fixed : L.s_inst) +
                   c.query_index);
  }
  h.p_setlen = (uint32_t)prog.size();
  for (auto& st : sets) prog.push_back((uint32_t)st.size());
  h.p_query = (uint32_t)prog.size();
  prog.insert(prog.end(), qprog.begin(), qprog.end());
  h.p_termsrc = (uint32_t)prog.size();
  prog.insert(prog.end(), termsrc.begin(), termsrc.end());
  // proof-point terms (the powers tables per proof) and each term's rank
  // among them; VK terms use the per-VK tables (ctx->acc_vkpow)
  std::vector<uint32_t> psrc, rank(termsrc.size(), 0u);
  for (size_t t = 0; t < termsrc.size(); t++)
    if ((termsrc[t] >> 28) == 0) {
      rank[t] = (uint32_t)psrc.size();
      psrc.push_back(termsrc[t]);
    }
  h.Tp = (uint32_t)psrc.size();
  h.p_psrc = (uint32_t)prog.size();
  prog.insert(prog.end(), psrc.begin(), psrc.end());
  h.p_rank = (uint32_t)prog.size();
  prog.insert(prog.end(), rank.begin(), rank.end());
  h.p_pbyte = (uint32_t)prog.size();
  if (dec) {
    for (uint32_t idx : psrc) prog.push_back(idx < dec->off_of.size() ? dec->off_of[idx] : kAccNoByte);
    h.pstride = (uint32_t)dec->stride;
    h.ninst = s->num_instance_columns;
  }

  // pairs of terms of one output for the one-lane form's two-term lanes
  // (k_acc_termmul NT = 2), per output range as k_acc_sum folds them
  const uint32_t p_pairs = (uint32_t)prog.size();
  uint32_t npair = 0;
  {
    const uint32_t T0 = (uint32_t)termsrc.size(), ns = nslots, nst = L.nsets;
    const uint32_t lo[4] = {0, ns, ns + nst, T0 - 1}, hi[4] = {ns, ns + nst, ns + 2 * nst, T0};
    for (int o = 0; o < 4; o++)
      for (uint32_t t = lo[o]; t < hi[o]; t += 2) {
        prog.push_back(t);
        prog.push_back(t + 1 < hi[o] ? t + 1 : kAccNoByte);
        npair++;
      }
  }

  // --- constants (Montgomery)
  std::vector<uint32_t> cst;
  h.c_user = 0;
  for (uint32_t i = 0; i < s->n_constants; i++) push_fe<Fs>(cst, fe_from_u64<Fs>(s->constants + 4 * i));
  const Fe<Fs> omega = fe_from_u64<Fs>(s->omega), delta = fe_from_u64<Fs>(s->delta);
  const Fe<Fs> omega_inv = fe_inv_bgcd<Fs>(omega);  // host binary GCD: ~10x faster than Fermat, same value
  h.c_delta = (uint32_t)(cst.size() / 8);
  Fe<Fs> acc = fe_one<Fs>();
  for (uint32_t k = 0; k < s->n_perm_columns; k++) {
    push_fe<Fs>(cst, acc);
    acc = fe_mul<Fs>(acc, delta);
  }
  h.c_omega_eval = (uint32_t)(cst.size() / 8);
  for (int32_t r : rots)  // multiopen.rs:348-359
    push_fe<Fs>(cst, r >= 0 ? fe_pow_u64<Fs>(omega, (uint64_t)r) : fe_pow_u64<Fs>(omega_inv, (uint64_t)(-(int64_t)r)));
  h.c_wpow = (uint32_t)(cst.size() / 8);
  acc = fe_one<Fs>();
  for (uint32_t i = 0; i < s->blinding_factors + 2; i++) {
    push_fe<Fs>(cst, acc);
    acc = fe_mul<Fs>(acc, omega_inv);
  }
  h.c_n = (uint32_t)(cst.size() / 8);
  Fe<Fs> nmont;
  {
    Fe<Fs> nf = fe_zero<Fs>();
    const uint64_t nn = 1ull << s->log_n;
    nf.l[0] = (uint32_t)nn;
    nf.l[1] = (uint32_t)(nn >> 32);
    nmont = fe_to_mont<Fs>(nf);
    push_fe<Fs>(cst, nmont);
  }
  // R = 2^261 copies (x 2^5 of the R = 2^256 integers, canonical)
  auto r261 = [](Fe<Fs> a) {
    for (int k = 0; k < 5; k++) a = fe_add<Fs>(a, a);
    return a;
  };
  h.c_wpow29 = (uint32_t)(cst.size() / 8);
  acc = fe_one<Fs>();
  for (uint32_t i = 0; i < s->blinding_factors + 2; i++) {
    push_fe<Fs>(cst, r261(acc));
    acc = fe_mul<Fs>(acc, omega_inv);
  }
  h.c_n29 = (uint32_t)(cst.size() / 8);
  push_fe<Fs>(cst, r261(nmont));
  // --- VK points: fixed commitments, sigma commitments, g1
  std::vector<uint64_t> vk;
  for (uint32_t i = 0; i < s->num_fixed_columns; i++) vk.insert(vk.end(), s->fixed_commitments + 8 * i, s->fixed_commitments + 8 * i + 8);
  for (uint32_t i = 0; i < s->n_perm_columns; i++) vk.insert(vk.end(), s->sigma_commitments + 8 * i, s->sigma_commitments + 8 * i + 8);
  vk.insert(vk.end(), s->g1, s->g1 + 8);

  const hipStream_t st = ctx->stream;
  int rc;
  if ((rc = ctx->acc_prog.put(prog, st))) return rc;
  if ((rc = ctx->acc_const.put(cst, st, 32))) return rc;
  if ((rc = ctx->acc_vk.put(vk, st))) return rc;
  if ((rc = ctx->acc_coef.ensure((size_t)B * T * 32))) return rc;
  if ((rc = ctx->acc_part.ensure((size_t)B * T * sizeof(Xyzz<F>)))) return rc;
  const uint32_t* dprog = (const uint32_t*)ctx->acc_prog.buf.p;
  uint32_t* dcoef = (uint32_t*)ctx->acc_coef.p;
  Xyzz<F>* dpart = (Xyzz<F>*)ctx->acc_part.p;
  const size_t nterm = (size_t)B * T, nprf = (size_t)B * h.Tp;
  const uint32_t lgS = acc_split_lanes(ctx, B, tm);
  // few terms (B <= ~34 for the simple shape): 16 quads per term with
  // quad-cooperative additions (k_acc_termadd<Cv, true>)
  const bool quad_terms = ctx->acc_split < 0 && lgS == 5 && nterm * 64 <= kAccLaneBudget / 2;
  const uint32_t lgT = quad_terms ? 4u : lgS;  // log2 of lanes (or quads) per term
  const uint32_t S = 1u << lgS;
  // Streams: with the split ladder (points only, the critical chain) it goes
  // first on the main stream, and the transcript replay + k_acc_scalars run
  // beside it on the reduction stream (kept off the ladder's CUs by the LDS
  // fence); the term products wait for both.  Launching the ladder after the
  // other two on the side stream cost ~20 us of start-up and ~20 us of
  // cross-stream wake-up on the critical path (profiles/r01_s4/ktrace_*).
  hipStream_t side = st;
  hipEvent_t up = nullptr, sc_done = nullptr;
  // proof bytes with the powers tables: the ladder runs on the twist from the
  // x bytes on the reduction stream, beside the decode -> replay -> scalar
  // block chain on the main stream, which is then the critical one and has no
  // cross-stream hop (decided with the decode's fence by proofs_device_impl)
  h.twist = dec && dec->twist && lgS > 0 ? 1u : 0u;
  if (h.twist && !dec->launched && (rc = ctx->acc_corr.ensure((size_t)B * L.npts * kAccCorrWords * sizeof(uint4))))
    return rc;
  std::vector<uint64_t> built_key;  // VK tables built by this call (committed after its final sync)
  bool lad_sliced = false;          // the ladder's chain form (below)
  // without the twist the decode comes first: everything after reads its points
  if (dec && !dec->launched && !h.twist && (rc = dec->launch(st, kDecodeFence, nullptr))) return rc;
  if (lgS > 0) {  // inputs and uploads are ready at this point of the stream
    const size_t tab = (size_t)kPowPos * kPowPoint * sizeof(uint4), nvk = vk.size() / 8;
    if ((rc = ctx->acc_lad.ensure(std::max<size_t>(nprf, 1) * tab))) return rc;
    if ((rc = ctx->acc_vkpow.ensure(std::max<size_t>(nvk, 1) * tab))) return rc;
    // per-VK tables: rebuilt (in the same launch, beside the proofs' chains)
    // only when the curve or the VK points differ from the last build, or
    // the buffer was reallocated
    std::vector<uint64_t> key(vk);
    key.push_back((uint64_t)F::MOD[1] << 32 | F::MOD[2]);  // the curve (its base field)
    const bool vk_current = ctx->acc_vkpow_gen == ctx->acc_vkpow.gen && ctx->acc_vkpow_key == key;
    const uint32_t nvk_build = vk_current ? 0u : (uint32_t)nvk;
    // up: the inputs and uploads (programs, constants, the decoder's map)
    // are complete; the other stream starts from it
    up = ctx->next_event();
    sc_done = ctx->next_event();
    if (!up || !sc_done) return set_error(PM_ERR_HIP, "hipEventCreate failed");
    // with the twist the decode heads the critical chain on st, queued by
    // proofs_device_impl before this plan was built; the ladder waits only for
    // the inputs (or, when this call re-sent programs or VK points, for those
    // copies, which sit behind the decode)
    const bool resent = ctx->acc_prog.sent || ctx->acc_const.sent || ctx->acc_vk.sent;
    if (h.twist && dec->launched && !resent && dec->in_ready) {
      up = dec->in_ready;
    } else {
      HIP_TRY(hipEventRecord(up, st));
    }
    if (h.twist && !dec->launched && (rc = dec->launch(st, kDecodeFence, (uint4*)ctx->acc_corr.p))) return rc;
    const hipStream_t lst = h.twist ? ctx->red_stream : st;  // the ladder's stream
    if (h.twist) HIP_TRY(hipStreamWaitEvent(lst, up, 0));
    const uint32_t* lproofs = h.twist ? (const uint32_t*)dec->proofs : nullptr;
    const uint32_t* linst = h.twist ? (const uint32_t*)dec->inst : nullptr;
    // few chains: one row-sliced wave per chain (slice29.hpp, ~2x shorter
    // steps while the waves fit one per SIMD); more: a quad per chain
    const size_t chains = nprf + nvk_build;
    const bool sliced = ctx->acc_ladder >= 0 ? ctx->acc_ladder == 1 : chains <= kAccSlicedChains;
    lad_sliced = sliced;
    if (ctx->timing) {  // entry -> the ladder's launch (filter "accum_host": no kernel events)
      auto& stt = ctx->stats["accum_plan_host"];
      stt.first += 1;
      stt.second += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tplan).count();
    }
    if (chains > 0 && sliced)
      PM_LAUNCH_ST(ctx, lst, "acc_ladder",
                (k_acc_powers_s<Cv><<<(unsigned)((chains + 3) / 4), 256, kAccSlicedFence, lst>>>(
                    h, dprog, (const uint32_t*)d_points, lproofs, linst, (const uint32_t*)ctx->acc_vk.buf.p, nvk_build,
                    (uint4*)ctx->acc_lad.p, (uint4*)ctx->acc_vkpow.p)));
    else if (chains > 0)
      PM_LAUNCH_ST(ctx, lst, "acc_ladder",
                (k_acc_powers<Cv><<<(unsigned)((4 * chains + 255) / 256), 256,
                                    4 * chains <= 256 * (size_t)ctx->num_cus ? kAccSlicedFence : kAccLadderFence, lst>>>(
                    h, dprog, (const uint32_t*)d_points, lproofs, linst, (const uint32_t*)ctx->acc_vk.buf.p, nvk_build,
                    (uint4*)ctx->acc_lad.p, (uint4*)ctx->acc_vkpow.p)));
    if (!vk_current) {
      // the tables count as built only once this call's work has completed
      // (below): a failed launch or call leaves the cache invalid, so the next
      // batch rebuilds them instead of reading unwritten tables
      ctx->acc_vkpow_key.clear();
      built_key.swap(key);
    }
    if (!h.twist) {
      side = ctx->red_stream;
      HIP_TRY(hipStreamWaitEvent(side, up, 0));
    }
  }
  if (vk_repr && (rc = transcript_launch<Cv>(ctx, s, B, vk_repr, d_points, d_scalars, d_ch, d_status, side,
                                             canon_ready, dflags)))
    return rc;
  // status: the replay stores bits 0-1 per proof, k_acc_scalars ORs in the
  // denominator bit; without a replay the words start at zero
  if (d_status && !vk_repr) HIP_TRY(hipMemsetAsync(d_status, 0, B * sizeof(uint32_t), side));
  // k_acc_scalars: 4 waves per block of np proofs, (nsc + T + exchange +
  // work) rows of 32 B per proof in LDS (proof stride np + 1), np <= 64
  // within a 128 KiB budget
  const size_t row_bytes =
      (size_t)(L.nsc + T + kAccXVals + acc_num_vals(h) + 2 * (h.bf + 3) + kAccStack + h.nslots + h.nh) * 32;
  const size_t tail_bytes = (size_t)acc_scalars_tail_words(h) * 4;  // constants + program
  if (tail_bytes + 2 * row_bytes > kAccScalarsLds)
    return set_error(PM_ERR_UNSUPPORTED, "accum: too many evaluations / terms per proof");
  // 16 proofs per block (round 5): wave 0 then runs the Lagrange chain with a
  // quad per proof (acc_lagrange_q, ~half the one-lane chain); more blocks
  // only spread the batch over more CUs
  const uint32_t np = (uint32_t)std::min<size_t>(16, (kAccScalarsLds - tail_bytes) / row_bytes - 1);
  const size_t lds = std::max(row_bytes * (np + 1) + tail_bytes, lgS > 0 ? kAccScalarsLds : 0);
  PM_LAUNCH_ST(ctx, side, "acc_scalars",
               (k_acc_scalars<Fs><<<(unsigned)((B + np - 1) / np), 256, lds, side>>>(
                   h, dprog, (const uint32_t*)ctx->acc_const.buf.p, (const uint32_t*)d_scalars, (const uint32_t*)d_ch,
                   dcoef, (uint32_t*)d_hout, np, (uint32_t*)d_status)));
  // the stream of the term additions and sums (tst): the one whose chain
  // ends last, so the cross-stream wait finds its event already signalled.
  // With the twist and the quad ladder (0.26 ms against decode -> transcript
  // -> scalars ~0.25) that is the ladder's stream; with the sliced ladder
  // (0.15 ms) the main one.  Waiting for the later stream cost ~5-10 us more
  // (profiles/r05/tail_ab/, interleaved runs: B = 64 0.433 -> 0.427 ms, B =
  // 128 0.454 -> 0.446; B = 16 0.341 -> 0.347 had it followed the ladder too)
  const bool tail_red = ctx->acc_tail != 0;  // PM_ACC_OPT_TAIL_STREAM = 0: always the main stream
  const hipStream_t tst = lgS > 0 && h.twist && !lad_sliced && tail_red ? ctx->red_stream : st;
  uint32_t pstep = 1;  // k_acc_sum's row step (2 after two-term lanes)
  if (lgS > 0) {
    // the term additions wait for the other stream: the scalar block (side),
    // or with the twist the ladder (or, on the ladder's stream, the scalar block)
    HIP_TRY(hipEventRecord(sc_done, h.twist ? (tst == st ? ctx->red_stream : st) : side));
    HIP_TRY(hipStreamWaitEvent(tst, sc_done, 0));
    if (quad_terms)
      PM_LAUNCH_ST(ctx, tst, "acc_termmul",
                (k_acc_termadd<Cv, true><<<(unsigned)((nterm * 64 + 255) / 256), 256, 0, tst>>>(
                    h, dprog, dcoef, (const uint4*)ctx->acc_lad.p, (const uint4*)ctx->acc_vkpow.p,
                    (const uint4*)ctx->acc_corr.p, lgT, dpart)));
    else
      PM_LAUNCH_ST(ctx, tst, "acc_termmul",
                (k_acc_termadd<Cv><<<(unsigned)((nterm * S + 255) / 256), 256, 0, tst>>>(
                    h, dprog, dcoef, (const uint4*)ctx->acc_lad.p, (const uint4*)ctx->acc_vkpow.p,
                    (const uint4*)ctx->acc_corr.p, lgS, dpart)));
  } else {
    // GLV products by signed 3-bit windows; two terms of one output per lane
    // (shared doublings) once one term per lane would put more than one wave
    // on a SIMD, while the pairs still fit one wave per SIMD (their 144 KiB of
    // LDS tables per block keep one block per CU); PM_ACC_OPT_TERMS_PER_LANE
    // forces 1 or 2
    const bool pairs_fit = (size_t)B * npair <= kAccLaneBudget / 2;
    const int tpl = ctx->acc_tpl > 0 ? ctx->acc_tpl : (nterm > kAccLaneBudget / 2 && pairs_fit ? 2 : 1);
    const uint32_t* dvk = (const uint32_t*)ctx->acc_vk.buf.p;
    if (tpl == 2) pstep = 2;
    if (tpl == 2)
      PM_LAUNCH(ctx, "acc_termmul",
                (k_acc_termmul<Cv, 2><<<(unsigned)(((size_t)B * npair + 255) / 256), 256, 0, st>>>(
                    h, dprog, dcoef, (const uint32_t*)d_points, dvk, p_pairs, npair, dpart)));
    else
      PM_LAUNCH(ctx, "acc_termmul",
                (k_acc_termmul<Cv, 1><<<(unsigned)((nterm + 255) / 256), 256, 0, st>>>(
                    h, dprog, dcoef, (const uint32_t*)d_points, dvk, 0u, 0u, dpart)));
  }
  // lanes per output: at most ~16 K in total.  The affine conversion runs on
  // lane 0 of each group, and it slowed from ~0.08 to ~0.14 ms when 32
  // lanes per output spread the 1024 outputs of B = 256 over 512 waves
  // (profiles/r01_s4/accum_sum_lanes.jsonl).
  uint32_t lgL = 0;
  while (lgL < 5 && ((size_t)B * 4 << (lgL + 1)) <= kAccSumLanes) lgL++;
  // large batches: still quads (quad-cooperative additions and inversion),
  // up to two per output, within one wave per SIMD; one lane per output ran
  // f's ~12 term sums and a lone-lane inversion while the w / zw / e lanes of
  // its wave idled (round 6, profiles/r06/sum_lanes_ab.jsonl: B = 4096 0.133
  // -> 0.114 ms, 3072 0.133 -> 0.080)
  while (lgL < 3 && ((size_t)B * 4 << (lgL + 1)) <= kAccLaneBudget / 2) lgL++;
  {
    hipEvent_t done = ctx->next_event();
    if (!done) return set_error(PM_ERR_HIP, "hipEventCreate failed");
    const unsigned nblk = (unsigned)((B * 4 * (1u << lgL) + 63) / 64);
    if (ctx->timing) {
      PM_LAUNCH_ST(ctx, tst, "acc_sum", (k_acc_sum<Cv><<<nblk, 64, 0, tst>>>(h, dpart, lgL, (uint32_t*)d_out, pstep)));
      HIP_TRY(hipEventRecord(done, tst));
    } else {  // the completion event rides on the dispatch (no marker packet behind it)
      hipExtLaunchKernelGGL(k_acc_sum<Cv>, dim3(nblk), dim3(64), 0, tst, nullptr, done, 0, h, dpart, lgL,
                            (uint32_t*)d_out, pstep);
      HIP_TRY(hipGetLastError());
    }
    if (int rc = wait_event(ctx, done)) return rc;
  }
  if (!built_key.empty()) {
    ctx->acc_vkpow_key.swap(built_key);
    ctx->acc_vkpow_gen = ctx->acc_vkpow.gen;
  }
  ctx->end_call();
  return PM_OK;
}

// Batched Blake2b transcript replay (transcript_kernels.hpp): absorb program
// in verifier read order, four lanes per proof, challenges written in the
// (B, 7, 4) layout pm_accum_batch reads.
// The byte stream every proof of the shape absorbs, laid out for
// k_transcript_s (transcript_kernels.hpp): per 32-bit stream word the
// constant bytes (record tags, the VK record, squeeze bytes) and up to two
// runs of the proof's canonical data bytes (points region: 64 bytes per point
// x || y; scalars region: 32 bytes each), then the point records' indices.
// false: the shape's stream does not fit the kernel's LDS (or its encoding):
// the per-record kernel runs instead (as it does under PM_ACC_OPT_TRANSCRIPT = 0,
// the caller's check).
inline bool tr_stream_plan(const std::vector<uint32_t>& prog, const TranscriptHdr& hd, TrStreamHdr& sh,
                           std::vector<uint32_t>& wtab) {
  struct Byte {
    uint32_t kind, v;  // kind 0: constant v; 1 / 2: data byte v of the points / scalars region
  };
  std::vector<Byte> by;
  std::vector<uint32_t> pts;
  uint32_t nsq = 0;
  for (uint32_t op : prog) {
    const uint32_t kind = op >> 24, idx = op & (kTrLookupZFlag - 1u);
    if (kind == kTrVk) {
      by.push_back({0, 2});
      for (int i = 0; i < 32; i++) by.push_back({0, (hd.vk[i / 4] >> (8 * (i % 4))) & 0xffu});
    } else if (kind == kTrPoint) {
      by.push_back({0, 1});
      for (uint32_t i = 0; i < 64; i++) by.push_back({1, 64 * idx + i});
      pts.push_back(idx);
    } else if (kind == kTrScalar) {
      by.push_back({0, 2});
      for (uint32_t i = 0; i < 32; i++) by.push_back({2, 32 * idx + i});
    } else {
      by.push_back({0, 0});
      if (idx != nsq || nsq >= kTrChallenges) return false;  // squeezes in challenge order
      sh.L[nsq++] = (uint32_t)by.size();
    }
  }
  if (nsq != kTrChallenges) return false;
  sh.nw32 = (uint32_t)((by.size() + 3) / 4);
  sh.nblk = (uint32_t)((by.size() + 127) / 128);
  sh.npr = (uint32_t)pts.size();
  wtab.assign(3 * (size_t)sh.nw32, 0u);
  for (uint32_t w = 0; w < sh.nw32; w++) {
    uint32_t nparts = 0;
    for (uint32_t p = 0; p < 4; p++) {
      const size_t i = 4 * (size_t)w + p;
      if (i >= by.size()) break;
      const Byte c = by[i];
      if (c.kind == 0) {
        wtab[3 * w] |= c.v << (8 * p);
        continue;
      }
      const bool cont = p > 0 && by[i - 1].kind == c.kind && by[i - 1].v + 1 == c.v;
      if (cont) {
        uint32_t& part = wtab[3 * w + nparts];
        const uint32_t n = ((part >> 23) & 7u) + 1, s8 = (part >> 28) & 3u;
        part = (part & ~(7u << 23) & ~(1u << 22)) | (n << 23) | ((s8 + n > 4) ? 1u << 22 : 0u);
        continue;
      }
      if (++nparts > 2) return false;
      const uint32_t widx = c.v >> 2;
      if (widx + 1 > kTrPartIdxMask) return false;
      wtab[3 * w + nparts] = (1u << 31) | ((c.kind == 2 ? 1u : 0u) << 30) | ((c.v & 3u) << 28) | (p << 26) |
                             (1u << 23) | widx;
    }
  }
  wtab.insert(wtab.end(), pts.begin(), pts.end());
  const TrStreamLds lay(sh.nw32, sh.nblk, sh.npr, hd.npts, hd.nsc);
  return 4ull * lay.total <= kAccScalarsLds;
}

template <class Cv>
int transcript_launch(Ctx* ctx, const pm_proof_shape* s, size_t B, const uint64_t vk_repr[4], const void* d_points,
                      const void* d_scalars, void* d_ch, void* d_status, hipStream_t st, bool canon_ready,
                      uint32_t* dflags) {
  using Fs = typename Cv::Scalar;
  std::vector<AccQuery> q;
  AccLayout L;
  const std::string err = acc_validate(s, q, L, nullptr);
  if (!err.empty()) return set_error(PM_ERR_ARG, "transcript shape: " + err);
  if (B == 0) return PM_OK;
  if (B > (1u << 20)) return set_error(PM_ERR_UNSUPPORTED, "transcript batch larger than 2^20 proofs");
  std::vector<uint32_t> prog;
  auto pts = [&](uint32_t p0, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) prog.push_back((kTrPoint << 24) | (p0 + i));
  };
  auto squeeze = [&](uint32_t slot) { prog.push_back((kTrSqueeze << 24) | slot); };
  prog.push_back(kTrVk << 24);                             // verifier.rs:341-358
  pts(L.p_inst, s->num_instance_columns);                  // :360-363
  pts(L.p_adv, s->num_advice_columns);                     // :365-376
  squeeze(0);                                              // theta :378
  pts(L.p_lkperm, 2 * s->num_lookups);                     // :381-387
  squeeze(1);                                              // beta :390
  squeeze(2);                                              // gamma :393
  pts(L.p_permz, L.n_perm_sets);                           // :402-409
  for (uint32_t i = 0; i < s->num_lookups; i++)            // :411-417 (lookup.rs:100: an
    prog.push_back((kTrPoint << 24) | kTrLookupZFlag | (L.p_lkz + i));  // identity Z aborts)
  pts(L.p_rand, 1);                                        // :419-421
  squeeze(3);                                              // y :423
  pts(L.p_h, s->quotient_degree);                          // :425-434
  squeeze(4);                                              // x :436
  for (uint32_t i = 0; i < L.nsc; i++) prog.push_back((kTrScalar << 24) | i);  // :438-509
  squeeze(5);                                              // v :718
  squeeze(6);                                              // u :719

  TranscriptHdr hd{};
  hd.B = (uint32_t)B;
  hd.npts = L.npts;
  hd.nsc = L.nsc;
  hd.nprog = (uint32_t)prog.size();
  blake2b_init_personal(hd.h0, (const uint8_t*)kTranscriptPersonal);
  const Fe<Fs> vk = fe_from_mont<Fs>(fe_from_u64<Fs>(vk_repr));
  for (int i = 0; i < 8; i++) hd.vk[i] = vk.l[i];

  int rc;
  if ((rc = ctx->tr_prog.put(prog, st))) return rc;
  TrStreamHdr sh{};
  std::vector<uint32_t> wtab;
  const bool streamed = ctx->acc_tr_stream != 0 && tr_stream_plan(prog, hd, sh, wtab);
  if (streamed && (rc = ctx->tr_wtab.put(wtab, st))) return rc;
  const size_t ncoord = B * 2 * (size_t)L.npts, nall = ncoord + B * (size_t)L.nsc;
  if ((rc = ctx->tr_canon.ensure(nall * 32))) return rc;
  uint32_t* cpts = (uint32_t*)ctx->tr_canon.p;
  uint32_t* cscs = cpts + 8 * ncoord;
  // LDS fence against the accumulator's ladder (kAccLadderFence) while the
  // blocks fit one per CU; larger batches run without the ladder anyway
  const size_t tblocks = (B + kTrSlots - 1) / kTrSlots;
  const bool fence = tblocks <= (size_t)ctx->num_cus;
  PM_LAUNCH_ST(ctx, st, "transcript", {
    if (!canon_ready)
      k_tr_canon<Cv><<<(unsigned)((nall + 255) / 256), 256, 0, st>>>(
          (uint32_t)B, L.npts, L.nsc, (const uint32_t*)d_points, (const uint32_t*)d_scalars, cpts, cscs);
    if (streamed) {
      const size_t lds = std::max<size_t>(4ull * TrStreamLds(sh.nw32, sh.nblk, sh.npr, L.npts, L.nsc).total,
                                          fence ? kAccScalarsLds : 0);
      k_transcript_s<Cv><<<(unsigned)tblocks, 256, lds, st>>>(
          hd, sh, (const uint32_t*)ctx->tr_prog.buf.p, (const uint32_t*)ctx->tr_wtab.buf.p, cpts, cscs,
          (uint32_t*)d_ch, (uint32_t*)d_status, dflags);
    } else {
      k_transcript<Cv><<<(unsigned)tblocks, 64, fence ? kAccScalarsLds : 0, st>>>(
          hd, (const uint32_t*)ctx->tr_prog.buf.p, cpts, cscs, (uint32_t*)d_ch, (uint32_t*)d_status, dflags);
    }
  });
  return PM_OK;
}

template <class Cv>
int transcript_device_impl(Ctx* ctx, const pm_proof_shape* s, size_t B, const uint64_t vk_repr[4], const void* d_points,
                           const void* d_scalars, void* d_ch, void* d_status) {
  return transcript_launch<Cv>(ctx, s, B, vk_repr, d_points, d_scalars, d_ch, d_status, ctx->stream);
}

// Proof bytes -> the accumulator's inputs (proof_kernels.hpp), then, with
// vk_repr, the fused transcript replay + accumulator on them.  Byte layout of
// one proof (the verifier's read order, oracle/proof_bytes.py): the proof
// points of the accumulator layout after the instance commitments (advice ..
// h_{d-1}), every scalar, then the W_j.  d_points / d_scalars receive the
// decoded layout (instance commitments copied from d_inst); d_status gets
// PM_PROOF_BAD_POINT / _SCALAR per proof (and the replay's bits).
template <class Cv>
int proofs_device_impl(Ctx* ctx, const pm_proof_shape* s, size_t B, const void* d_proofs, size_t stride,
                       const void* d_inst, void* d_points, void* d_scalars, void* d_status, const uint64_t* vk_repr,
                       void* d_ch, void* d_quads, void* d_h) {
  std::vector<AccQuery> q;
  AccLayout L;
  const std::string err = acc_validate(s, q, L, nullptr);
  if (!err.empty()) return set_error(PM_ERR_ARG, "proof shape: " + err);
  if (B == 0) return PM_OK;
  if (B > (1u << 20)) return set_error(PM_ERR_UNSUPPORTED, "proof batch larger than 2^20 proofs");
  const uint32_t ninst = s->num_instance_columns, npp = L.p_W - ninst + L.nsets;
  const size_t psize = 32ull * (L.npts - ninst + L.nsc);
  if (stride < psize || (stride & 3u)) return set_error(PM_ERR_ARG, "proof stride below the proof size or not a multiple of 4");
  if (stride * B > (size_t(1) << 40)) return set_error(PM_ERR_UNSUPPORTED, "proof batch too large");
  const int slot = curve_slot<Cv>();
  int rc;
  const hipStream_t st = ctx->stream;
  if (!ctx->sqrt_ready[slot]) {
    SqrtTab tab;
    if ((rc = sqrt_tab_build<Cv>(tab))) return rc;
    if ((rc = ctx->sqrt_tab[slot].ensure(sizeof(SqrtTab)))) return rc;
    HIP_TRY(hipMemcpy(ctx->sqrt_tab[slot].p, &tab, sizeof(SqrtTab), hipMemcpyHostToDevice));
    ctx->sqrt_ready[slot] = true;
    ctx->sqrt_tab_ts[slot] = tab.ts != 0;
  }
  // (byte offset, destination point) of every point read from the bytes
  std::vector<uint32_t> map;
  const uint32_t sc_off = 32u * (L.p_W - ninst);
  for (uint32_t i = ninst; i < L.p_W; i++) {
    map.push_back(32u * (i - ninst));
    map.push_back(i);
  }
  for (uint32_t j = 0; j < L.nsets; j++) {
    map.push_back(sc_off + 32u * L.nsc + 32u * j);
    map.push_back(L.p_W + j);
  }
  if ((rc = ctx->pf_map.put(map, st))) return rc;
  const size_t ncoord = B * 2 * (size_t)L.npts, nall = ncoord + B * (size_t)L.nsc;
  if ((rc = ctx->tr_canon.ensure(nall * 32))) return rc;
  uint32_t* cpts = (uint32_t*)ctx->tr_canon.p;
  uint32_t* cscs = cpts + 8 * ncoord;
  // decode flags: straight into the caller's status words (zeroed first) when
  // only decoding; with the replay, into a per-context word per proof that
  // k_transcript folds into the status and clears, so no memset precedes the
  // decode (a failed call leaves them dirty: cleared on the next call)
  uint32_t* dflags = (uint32_t*)d_status;
  if (vk_repr) {
    const size_t old_cap = ctx->pf_flags.cap;
    if ((rc = ctx->pf_flags.ensure(B * sizeof(uint32_t)))) return rc;
    if (ctx->pf_flags.cap != old_cap || ctx->pf_flags_dirty)
      HIP_TRY(hipMemsetAsync(ctx->pf_flags.p, 0, ctx->pf_flags.cap, st));
    ctx->pf_flags_dirty = true;
    dflags = (uint32_t*)ctx->pf_flags.p;
  } else {
    HIP_TRY(hipMemsetAsync(d_status, 0, B * sizeof(uint32_t), st));
  }
  ProofDecodeHdr h{};
  h.B = (uint32_t)B;
  h.npts = L.npts;
  h.nsc = L.nsc;
  h.ninst = ninst;
  h.npp = npp;
  h.sc_off = sc_off;
  h.stride = (uint32_t)stride;
  // Plan facts the decode's form and fence depend on (the split form and
  // the ladder's grid; accum_device_impl recomputes them identically).
  bool twist = false;
  size_t lad_blocks = 0;
  const size_t cus = (size_t)ctx->num_cus;
  {
    std::vector<int32_t> rots;
    std::vector<std::vector<AccQuery>> sets;
    acc_group_sets(q, rots, sets);
    AccTerms tm;
    acc_terms(s, L, sets, tm);
    const bool split = vk_repr && acc_split_lanes(ctx, B, tm) > 0;
    const size_t nprf = B * (size_t)tm.Tp;
    lad_blocks = nprf <= kAccSlicedChains ? (nprf + 3) / 4 : (4 * nprf + 255) / 256;
    twist = split && ctx->acc_twist != 0;
  }
  const size_t nblk_sc = (B * ((size_t)L.nsc + ninst) + kDecodeThreads - 1) / kDecodeThreads;
  auto pt_blocks = [&](bool sl) {
    const size_t per = sl ? kDecodeThreads / 16 : kDecodeThreads;
    return (B * npp + per - 1) / per;
  };
  // few points on a p = 3 mod 4 curve: one point per row, the square root
  // row-sliced (k_proof_decode<Cv, true>); up to ~one wave per SIMD.  Beside
  // the twisted ladder (automatic schedule) only while its grid fits the CUs
  // with the ladder's blocks: else the one-lane decode, 16x fewer blocks,
  // which then fits fenced beside the ladder and leaves it undisturbed --
  // the decode is off the critical path there, the ladder on it (round 6,
  // profiles/r06/decode_form_ab.jsonl: B = 256 0.546 -> 0.50 ms)
  bool sliced = !ctx->sqrt_tab_ts[slot] && (ctx->acc_ladder >= 0 ? ctx->acc_ladder == 1
                                                                  : B * npp <= kDecodeSlicedPoints);
  if (sliced && twist && ctx->acc_ladder < 0 && ctx->acc_twist < 0 && pt_blocks(true) + nblk_sc + lad_blocks > cus)
    sliced = false;
  h.nblk_pts = (uint32_t)pt_blocks(sliced);
  if (stride > 0xffffffffull) return set_error(PM_ERR_UNSUPPORTED, "proof stride above 4 GiB");
  AccDecode dec;
  dec.proofs = d_proofs;
  dec.stride = stride;
  dec.inst = d_inst;
  dec.sliced = sliced;
  // The decode's fence beside the twisted ladder: its blocks are kept off the
  // ladder's CUs where the CUs allow (round 6, profiles/r06/twist_fence_ab.jsonl,
  // B = 128 .. 1024):
  //  * decode and ladder blocks fit the CUs side by side: kDecodeFence, one
  //    decode block per CU beside nothing (B <= 128, 384, 512);
  //  * else, while the decode's blocks alone leave CUs free: kDecodePairFence
  //    (B = 192 with the sliced decode: 0.507 ms against 0.540 unfenced, 0.60
  //    without the twist);
  //  * else unfenced, among the ladder's blocks: the dispatcher spreads the
  //    first blocks one per CU, so a pair-fenced decode filling every CU kept
  //    the ladder waiting (B = 256 sliced: 0.547 unfenced, 0.600 paired or no
  //    twist).
  // (In round 5 the twist beside a fenced decode lost at B = 256 for that
  // reason and was kept to the first case.)  PM_ACC_OPT_TWIST = 1 / 2 force
  // the unfenced / paired decode (and keep the row-sliced form where it
  // applies).  Without the split form (the one-lane GLV products) the decode
  // is fenced up to num_cus point blocks (beyond, throughput work).
  const size_t nblk_dec = h.nblk_pts + nblk_sc;
  size_t dec_fence;
  if (!twist) dec_fence = h.nblk_pts <= cus ? kDecodeFence : 0;
  else if (ctx->acc_twist == 1) dec_fence = 0;
  else if (ctx->acc_twist == 2) dec_fence = kDecodePairFence;
  else dec_fence = nblk_dec + lad_blocks <= cus ? kDecodeFence : nblk_dec < cus ? kDecodePairFence : 0;
  dec.twist = twist;
  dec.off_of.assign(L.npts, kAccNoByte);
  for (size_t i = 0; i + 1 < map.size(); i += 2) dec.off_of[map[i + 1]] = map[i];
  const SqrtTab* tabp = (const SqrtTab*)ctx->sqrt_tab[slot].p;
  const uint32_t* dmap = (const uint32_t*)ctx->pf_map.buf.p;
  dec.launch = [=](hipStream_t dst, size_t fence, uint4* cp) -> int {
    // the fence is the whole block's LDS (the kernel's static arrays count):
    // one block per CU, beside nothing (latency-bound chains; unfenced, the
    // dispatcher packed several blocks per CU, B = 16 decode 0.11 -> 0.16 ms);
    // cp: the twisted ladder's factors (acc_corr, sized by accum_device_impl)
    auto kern = sliced ? k_proof_decode<Cv, true> : k_proof_decode<Cv, false>;
    const size_t stat = sliced ? decode_static_lds<Cv, true>() : decode_static_lds<Cv, false>();
    const size_t dyn = fence > stat ? fence - stat : 0;
    PM_LAUNCH_ST(ctx, dst, "proof_decode",
                 (kern<<<(unsigned)(h.nblk_pts + nblk_sc), kDecodeThreads, dyn, dst>>>(
                     h, tabp, dmap, (const uint32_t*)d_proofs, (const uint32_t*)d_inst, (uint32_t*)d_points,
                     (uint32_t*)d_scalars, cpts, cscs, dflags, cp)));
    return PM_OK;
  };
  if (!vk_repr) {
    if ((rc = dec.launch(st, dec_fence, nullptr))) return rc;
    HIP_TRY(hipStreamSynchronize(st));
    ctx->end_call();
    return PM_OK;
  }
  // the decode first, before the accumulator's plan is even built (host time
  // off the critical chain), writing the twisted ladder's factors in case the
  // plan picks the twist; in_ready lets the twisted ladder start beside it
  dec.in_ready = ctx->next_event();
  if (!dec.in_ready) return set_error(PM_ERR_HIP, "hipEventCreate failed");
  HIP_TRY(hipEventRecord(dec.in_ready, st));
  if ((rc = ctx->acc_corr.ensure(B * (size_t)L.npts * kAccCorrWords * sizeof(uint4)))) return rc;
  if ((rc = dec.launch(st, dec_fence, (uint4*)ctx->acc_corr.p))) return rc;
  dec.launched = true;
  rc = accum_device_impl<Cv>(ctx, s, B, d_points, d_scalars, d_ch, d_quads, d_h, vk_repr, d_status, true, dflags,
                             &dec);
  if (rc == PM_OK) ctx->pf_flags_dirty = false;  // k_transcript has cleared every word
  return rc;
}

// the CurveOps entry (no extra parameters)
template <class Cv>
int accum_device_entry(Ctx* ctx, const pm_proof_shape* s, size_t B, const void* d_points, const void* d_scalars,
                       void* d_ch, void* d_out, void* d_hout, const uint64_t* vk_repr, void* d_status) {
  return accum_device_impl<Cv>(ctx, s, B, d_points, d_scalars, d_ch, d_out, d_hout, vk_repr, d_status);
}

// vk_repr = from_bytes_wide(Blake2b("Halo2-Verify-Key", ...)) (verifier.rs:347-354)
template <class Cv>
int vk_repr_impl(const uint8_t digest[64], uint64_t out[4]) {
  using Fs = typename Cv::Scalar;
  uint32_t d[16];
  memcpy(d, digest, 64);
  const Fe<Fs> v = fe_from_bytes_wide<Fs>(d);
  for (int k = 0; k < 4; k++) out[k] = (uint64_t)v.l[2 * k] | ((uint64_t)v.l[2 * k + 1] << 32);
  return PM_OK;
}

}  // namespace pm

#include "ntt_engine.hpp"  // uses fe_from_u64 above
#include "msm_many.hpp"

// Explicit instantiations are visible to both compilation passes, so the
// device pass instantiates every kernel the host driver launches; the op
// table (host function pointers) exists only in the host pass.
#if defined(__HIP_DEVICE_COMPILE__)
#define PM_OPS_TABLE(Cv, name)
#else
#define PM_OPS_TABLE(Cv, name)                                                                 \
  extern const CurveOps name;                                                                  \
  const CurveOps name = {&msm_device_to_aff<Cv>, &point_add_impl<typename Cv::Base>,            \
                         &synth_scalars_impl<Cv>, &synth_bases_impl<Cv>,  \
                         &accum_device_entry<Cv>, &selftest_field_impl<Cv>,           \
                         &transcript_device_impl<Cv>, &vk_repr_impl<Cv>,                   \
                         &fixed_table_impl<Cv>, &ntt_device_impl<Cv>, &msm_fixed_to_aff<Cv>,    \
                         &bases_to29_impl<Cv>, &msm_resident_batch_impl<Cv>, &proofs_device_impl<Cv>,    \
                         &msm_start_impl<Cv>, &msm_finish_impl<Cv>, &msm_small_impl<Cv>,         \
                         &many_table_impl<Cv>, &msm_many_impl<Cv>, &points_sum_impl<typename Cv::Base>};
#endif
#define PM_DEFINE_CURVE_OPS(Cv, name)                                                          \
  namespace pm {                                                                               \
  template int msm_device_to_aff<Cv>(Ctx*, const void*, const void*, size_t, uint32_t, uint64_t*, const void*); \
  template int synth_scalars_impl<Cv>(Ctx*, uint64_t, uint64_t, uint32_t, uint32_t, void*);     \
  template int synth_bases_impl<Cv>(Ctx*, uint64_t, uint64_t, uint32_t, void*);                 \
  template int accum_device_entry<Cv>(Ctx*, const pm_proof_shape*, size_t, const void*, const void*, void*, void*, \
                                      void*, const uint64_t*, void*);                            \
  template int proofs_device_impl<Cv>(Ctx*, const pm_proof_shape*, size_t, const void*, size_t, const void*, void*, \
                                      void*, void*, const uint64_t*, void*, void*, void*);       \
  template int selftest_field_impl<Cv>(Ctx*, uint64_t, uint32_t, uint64_t*);                      \
  template int fixed_table_impl<Cv>(Ctx*, const void*, pm_fixed_bases*);                          \
  template int ntt_device_impl<Cv>(Ctx*, int, void*, uint32_t, const uint64_t*, const uint64_t*);  \
  template int msm_fixed_to_aff<Cv>(Ctx*, const pm_fixed_bases*, const void*, size_t, uint32_t, uint64_t*, \
                                    const void*);                                                  \
  template int bases_to29_impl<Cv>(Ctx*, const void*, size_t, void*);                            \
  template int msm_resident_batch_impl<Cv>(Ctx*, const void*, const pm_fixed_bases*, const uint64_t* const*, size_t, \
                                           size_t, uint32_t, uint64_t*);                             \
  template int transcript_device_impl<Cv>(Ctx*, const pm_proof_shape*, size_t, const uint64_t*, const void*, \
                                          const void*, void*, void*);                            \
  template int msm_start_impl<Cv>(Ctx*, const pm_fixed_bases*, const void*, const void*, size_t, uint32_t, void*, \
                                  const void*); \
  template int msm_finish_impl<Cv>(Ctx*, const void*, uint64_t*);                                \
  template int msm_small_impl<Cv>(Ctx*, const void*, bool, const void*, bool, bool, size_t, uint32_t, uint64_t*); \
  template int many_table_impl<Cv>(Ctx*, const void*, size_t, ManyTable*);                       \
  template int msm_many_impl<Cv>(Ctx*, const ManyTable*, size_t, const size_t*, const size_t*, const void*, bool, \
                                 uint32_t, uint64_t*);                                           \
  PM_OPS_TABLE(Cv, name)                                                                       \
  }

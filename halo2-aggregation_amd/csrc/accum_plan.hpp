// accum_plan.hpp -- host-side plan of the batch multiopen accumulator.
//
// From a pm_proof_shape (the VerifyingKey / ConstraintSystem view of
// /root/reference/src/verifier.rs:227-285) this builds, once per call, the
// query list in the reference order (verifier.rs:654-715 with
// permutation.rs:332-358, lookup.rs:314-347, vanishing.rs:206-220), groups it
// by rotation like construct_intermediate_sets (src/multiopen.rs:19-45:
// BTreeMap => ascending rotation, query order kept inside a set), and assigns
// every distinct commitment of `f` an MSM term slot.  The device kernels
// (accum_kernels.hpp) only follow this table.
#pragma once
#include <algorithm>
#include <map>
#include <string>
#include <vector>

#include "../../include/pasta_msm.h"

namespace pm {

// point reference kinds in the query list
enum : uint32_t { kRefProof = 0, kRefFixed = 1, kRefSigma = 2, kRefH = 3 };
constexpr uint32_t kEvalH = 0xFFFFFFFFu;  // query eval = computed h_eval
constexpr uint32_t kSlotH = 0xFFFFu;      // query point = H (vanishing.rs:178-188)
constexpr uint32_t kAccStack = 16;        // expression stack depth bound
constexpr uint32_t kAccMaxSets = 64;
constexpr uint32_t kAccMaxPerSet = 256;
constexpr uint32_t kAccMaxBlind = 61;     // l_i batch of bf + 3 inversions

struct AccQuery {
  uint32_t ref_kind, ref_idx;  // point
  int32_t rot;
  uint32_t eval;               // index into the proof's scalars, or kEvalH
};

// Per-proof layout (transcript read order, see oracle/accum.py)
struct AccLayout {
  uint32_t p_inst, p_adv, p_lkperm, p_permz, p_lkz, p_rand, p_h, p_W, npts;
  uint32_t s_inst, s_adv, s_fixed, s_rand, s_sigma, s_perm, s_lk, nsc;
  uint32_t n_perm_sets, nsets;
};

inline uint32_t acc_perm_sets(const pm_proof_shape* s) {
  return s->perm_chunk_len ? (s->n_perm_columns + s->perm_chunk_len - 1) / s->perm_chunk_len : 0;
}

// Validates the shape and returns the query list + layout; "" on success.
inline std::string acc_build_queries(const pm_proof_shape* s, std::vector<AccQuery>& q, AccLayout& L) {
  if (!s) return "null shape";
  if (s->n_perm_columns && !s->perm_chunk_len) return "perm_chunk_len = 0 with permutation columns";
  if (s->quotient_degree == 0) return "quotient_degree must be >= 1";
  if (s->blinding_factors > kAccMaxBlind) return "blinding_factors too large";
  if (s->log_n == 0 || s->log_n > 32) return "log_n out of range";
  if ((s->n_instance_queries && !s->instance_queries) || (s->n_advice_queries && !s->advice_queries) ||
      (s->n_fixed_queries && !s->fixed_queries) || (s->n_perm_columns && !s->perm_columns))
    return "null query / permutation array";
  if ((s->num_fixed_columns && !s->fixed_commitments) || (s->n_perm_columns && !s->sigma_commitments))
    return "null VK commitments";
  const uint32_t nps = acc_perm_sets(s);
  L.p_inst = 0;
  L.p_adv = L.p_inst + s->num_instance_columns;
  L.p_lkperm = L.p_adv + s->num_advice_columns;
  L.p_permz = L.p_lkperm + 2 * s->num_lookups;
  L.p_lkz = L.p_permz + nps;
  L.p_rand = L.p_lkz + s->num_lookups;
  L.p_h = L.p_rand + 1;
  L.p_W = L.p_h + s->quotient_degree;
  L.s_inst = 0;
  L.s_adv = L.s_inst + s->n_instance_queries;
  L.s_fixed = L.s_adv + s->n_advice_queries;
  L.s_rand = L.s_fixed + s->n_fixed_queries;
  L.s_sigma = L.s_rand + 1;
  L.s_perm = L.s_sigma + s->n_perm_columns;
  L.s_lk = L.s_perm + (nps ? 3 * nps - 1 : 0);
  L.nsc = L.s_lk + 5 * s->num_lookups;
  L.n_perm_sets = nps;

  q.clear();
  for (uint32_t i = 0; i < s->n_instance_queries; i++) {
    if (s->instance_queries[i].column >= s->num_instance_columns) return "instance query column out of range";
    q.push_back({kRefProof, L.p_inst + s->instance_queries[i].column, s->instance_queries[i].rotation, L.s_inst + i});
  }
  for (uint32_t i = 0; i < s->n_advice_queries; i++) {
    if (s->advice_queries[i].column >= s->num_advice_columns) return "advice query column out of range";
    q.push_back({kRefProof, L.p_adv + s->advice_queries[i].column, s->advice_queries[i].rotation, L.s_adv + i});
  }
  // permutation.rs:332-358: (Z, cur), (Z, next) per set; (Z, last) for all but the last set, reversed
  const int32_t last_rot = -(int32_t)(s->blinding_factors + 1);
  for (uint32_t i = 0; i < nps; i++) {
    q.push_back({kRefProof, L.p_permz + i, 0, L.s_perm + 3 * i});
    q.push_back({kRefProof, L.p_permz + i, 1, L.s_perm + 3 * i + 1});
  }
  for (int i = (int)nps - 2; i >= 0; i--) q.push_back({kRefProof, L.p_permz + i, last_rot, L.s_perm + 3 * i + 2});
  // lookup.rs:314-347
  for (uint32_t i = 0; i < s->num_lookups; i++) {
    const uint32_t z = L.p_lkz + i, a = L.p_lkperm + 2 * i, sp = a + 1, e = L.s_lk + 5 * i;
    q.push_back({kRefProof, z, 0, e + 0});
    q.push_back({kRefProof, a, 0, e + 2});
    q.push_back({kRefProof, sp, 0, e + 4});
    q.push_back({kRefProof, a, -1, e + 3});
    q.push_back({kRefProof, z, 1, e + 1});
  }
  for (uint32_t i = 0; i < s->n_fixed_queries; i++) {
    if (s->fixed_queries[i].column >= s->num_fixed_columns) return "fixed query column out of range";
    q.push_back({kRefFixed, s->fixed_queries[i].column, s->fixed_queries[i].rotation, L.s_fixed + i});
  }
  for (uint32_t k = 0; k < s->n_perm_columns; k++) q.push_back({kRefSigma, k, 0, L.s_sigma + k});
  // vanishing.rs:206-220
  q.push_back({kRefH, 0, 0, kEvalH});
  q.push_back({kRefProof, L.p_rand, 0, L.s_rand});

  for (uint32_t k = 0; k < s->n_perm_columns; k++) {
    const pm_perm_column& c = s->perm_columns[k];
    const uint32_t lim = c.kind == PM_COL_ADVICE ? s->n_advice_queries
                         : c.kind == PM_COL_FIXED ? s->n_fixed_queries
                         : c.kind == PM_COL_INSTANCE ? s->n_instance_queries : 0;
    if (c.query_index >= lim) return "permutation column query index out of range";
  }
  std::vector<int32_t> rots;
  for (auto& x : q) rots.push_back(x.rot);
  std::sort(rots.begin(), rots.end());
  rots.erase(std::unique(rots.begin(), rots.end()), rots.end());
  if (rots.size() > kAccMaxSets) return "too many rotation sets";
  L.nsets = (uint32_t)rots.size();
  L.npts = L.p_W + L.nsets;
  return "";
}

// Rotation sets: stable grouping by ascending rotation.
inline void acc_group_sets(const std::vector<AccQuery>& q, std::vector<int32_t>& rots,
                           std::vector<std::vector<AccQuery>>& sets) {
  std::map<int32_t, std::vector<AccQuery>> by;
  for (auto& x : q) by[x.rot].push_back(x);
  rots.clear();
  sets.clear();
  for (auto& kv : by) {
    rots.push_back(kv.first);
    sets.push_back(kv.second);
  }
}

// Checks a postfix expression program; returns the number of expressions
// (END words) or -1 with a message.
inline int acc_check_code(const uint32_t* code, uint32_t len, uint32_t n_const, uint32_t n_adv, uint32_t n_fixed,
                          uint32_t n_inst, std::string& err) {
  if (len && !code) {
    err = "null expression code";
    return -1;
  }
  int sp = 0, nexpr = 0;
  for (uint32_t i = 0; i < len; i++) {
    const uint32_t op = code[i] & 0xffu, arg = code[i] >> 8;
    switch (op) {
      case PM_EXPR_CONST:
        if (arg >= n_const) { err = "CONST index out of range"; return -1; }
        sp++;
        break;
      case PM_EXPR_FIXED:
        if (arg >= n_fixed) { err = "FIXED query index out of range"; return -1; }
        sp++;
        break;
      case PM_EXPR_ADVICE:
        if (arg >= n_adv) { err = "ADVICE query index out of range"; return -1; }
        sp++;
        break;
      case PM_EXPR_INSTANCE:
        if (arg >= n_inst) { err = "INSTANCE query index out of range"; return -1; }
        sp++;
        break;
      case PM_EXPR_NEG:
        if (sp < 1) { err = "NEG on empty stack"; return -1; }
        break;
      case PM_EXPR_SUM:
      case PM_EXPR_PROD:
        if (sp < 2) { err = "binary op on short stack"; return -1; }
        sp--;
        break;
      case PM_EXPR_SCALED:
        if (sp < 1 || arg >= n_const) { err = "bad SCALED"; return -1; }
        break;
      case PM_EXPR_END:
        if (sp != 1) { err = "END with stack depth != 1"; return -1; }
        sp = 0;
        nexpr++;
        break;
      default:
        err = "unknown expression op";
        return -1;
    }
    if (sp > (int)kAccStack) {
      err = "expression stack deeper than 16";
      return -1;
    }
  }
  if (sp != 0) {
    err = "expression code does not end with END";
    return -1;
  }
  return nexpr;
}

// Full validation: queries / layout plus the three expression programs.
inline std::string acc_validate(const pm_proof_shape* s, std::vector<AccQuery>& q, AccLayout& L, int* ngates) {
  std::string err = acc_build_queries(s, q, L);
  if (!err.empty()) return err;
  if (s->n_constants && !s->constants) return "null constants";
  const uint32_t ni = s->n_instance_queries, na = s->n_advice_queries, nf = s->n_fixed_queries;
  const int ng = acc_check_code(s->gate_code, s->gate_code_len, s->n_constants, na, nf, ni, err);
  if (ng < 0) return "gate code: " + err;
  if (acc_check_code(s->lookup_input_code, s->lookup_input_code_len, s->n_constants, na, nf, ni, err) < 0)
    return "lookup input code: " + err;
  if (acc_check_code(s->lookup_table_code, s->lookup_table_code_len, s->n_constants, na, nf, ni, err) < 0)
    return "lookup table code: " + err;
  if (ng + L.n_perm_sets + 5 * s->num_lookups == 0) return "no expressions (vanishing.rs:147 asserts >= 1)";
  if (ngates) *ngates = ng;
  return "";
}

}  // namespace pm

// accum_kernels.hpp -- batch multiopen accumulator kernels for gfx950.
//
// Native meaning of the reference's in-circuit verifier for B proofs of one
// verifying key (SURVEY.md §8 rows a-3 … a-9):
//   k_acc_scalars  one lane per proof: x^n, the l_i batch inversion
//                  (src/verifier.rs:512-591), gate / permutation / lookup
//                  expressions (verifier.rs:593-643, permutation.rs:190-324,
//                  lookup.rs:173-311), h_eval (vanishing.rs:136-175), then
//                  the closed-form coefficient of every MSM term of
//                  calc_witness (multiopen.rs:271-509): u^{S-1-j} v^{m_j-1-i}
//                  per query, H expanded as sum_i x^{n i} h_i
//                  (vanishing.rs:178-188), z_j u^{S-1-j} for zw and
//                  -eval_multi for e = [.] g1.
//   k_acc_termmul  one lane per (proof, term): [coef] P by MSB-first
//                  double-and-add in XYZZ.
//   k_acc_sum      one lane per (proof, output): sums its terms, converts to
//                  the unique affine point (w, zw, f, e order of MultiopenVar).
// Scalars / points use the Rust in-memory Montgomery layout (pasta_msm.h).
#pragma once
#include "accum_plan.hpp"
#include "msm_kernels.hpp"

namespace pm {

struct AccumHdr {
  uint32_t B, npts, nsc, T, nslots, nsets;
  uint32_t log_n, bf, num_lookups;
  uint32_t n_perm_cols, perm_chunk, n_perm_sets;
  uint32_t sc_inst, sc_adv, sc_fixed, sc_rand, sc_sigma, sc_perm, sc_lk;
  // u32 program offsets
  uint32_t p_gate, n_gate, p_lkin, n_lkin, p_lktab, n_lktab;
  uint32_t p_permcol;  // n_perm_cols: scalar index of the column's eval
  uint32_t p_setlen;   // nsets: queries per set
  uint32_t p_query;    // 2 words per query: slot (kSlotH = H), eval index (kEvalH = h_eval)
  uint32_t p_termsrc;  // T words: (kind << 28) | index, kind 0 = proof point, 1 = VK point
  uint32_t h_slot0, nh;
  // constant table (8 u32 per element, Montgomery)
  uint32_t c_user, c_delta, c_omega_eval, c_wpow, c_n;
};

template <class Fs>
__device__ __forceinline__ Fe<Fs> ldfe(const uint32_t* base, uint32_t idx) {
  return load_fe4<Fs>(reinterpret_cast<const uint4*>(base + 8ull * idx));
}
template <class Fs>
__device__ __forceinline__ void stfe(uint32_t* base, uint32_t idx, const Fe<Fs>& v) {
  store_fe4<Fs>(reinterpret_cast<uint4*>(base + 8ull * idx), v);
}

// Postfix program (compute_expr, verifier.rs:58-151); every END folds the
// finished expression into acc = acc * mult + value (vanishing Horner in y,
// or compress_expressions in theta, lookup.rs:214-243).
template <class Fs>
__device__ Fe<Fs> acc_eval_code(const uint32_t* code, uint32_t len, const uint32_t* sc, const AccumHdr& h,
                                const uint32_t* consts, Fe<Fs> acc, const Fe<Fs>& mult) {
  Fe<Fs> st[kAccStack];
  int sp = 0;
  for (uint32_t i = 0; i < len; i++) {
    const uint32_t op = code[i] & 0xffu, arg = code[i] >> 8;
    if (op == PM_EXPR_END) {
      acc = fe_add<Fs>(fe_mul<Fs>(acc, mult), st[--sp]);
    } else if (op <= PM_EXPR_INSTANCE) {
      const uint32_t* src = op == PM_EXPR_CONST ? consts : sc;
      const uint32_t base = op == PM_EXPR_CONST ? h.c_user
                            : op == PM_EXPR_FIXED ? h.sc_fixed
                            : op == PM_EXPR_ADVICE ? h.sc_adv : h.sc_inst;
      st[sp++] = ldfe<Fs>(src, base + arg);
    } else if (op == PM_EXPR_NEG) {
      st[sp - 1] = fe_neg<Fs>(st[sp - 1]);
    } else if (op == PM_EXPR_SUM) {
      st[sp - 2] = fe_add<Fs>(st[sp - 2], st[sp - 1]);
      sp--;
    } else {  // PROD, SCALED
      const Fe<Fs> b = op == PM_EXPR_PROD ? st[sp - 1] : ldfe<Fs>(consts, h.c_user + arg);
      const int dst = op == PM_EXPR_PROD ? sp - 2 : sp - 1;
      st[dst] = fe_mul<Fs>(st[dst], b);
      if (op == PM_EXPR_PROD) sp--;
    }
  }
  return acc;
}

template <class Fs>
__global__ void __launch_bounds__(64) k_acc_scalars(AccumHdr h, const uint32_t* __restrict__ prog,
                                                    const uint32_t* __restrict__ consts,
                                                    const uint32_t* __restrict__ scalars,
                                                    const uint32_t* __restrict__ challenges,
                                                    uint32_t* __restrict__ coef, uint32_t* __restrict__ h_out) {
  const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= h.B) return;
  const uint32_t* sc = scalars + 8ull * h.nsc * b;
  const uint32_t* ch = challenges + 8ull * 7 * b;
  uint32_t* cf = coef + 8ull * h.T * b;
  const Fe<Fs> theta = ldfe<Fs>(ch, 0), beta = ldfe<Fs>(ch, 1), gamma = ldfe<Fs>(ch, 2), y = ldfe<Fs>(ch, 3),
               x = ldfe<Fs>(ch, 4), v = ldfe<Fs>(ch, 5), u = ldfe<Fs>(ch, 6);
  const Fe<Fs> one = fe_one<Fs>(), zero = fe_zero<Fs>();

  // x^n (verifier.rs:513-516)
  Fe<Fs> xn = x;
  for (uint32_t i = 0; i < h.log_n; i++) xn = fe_sqr<Fs>(xn);
  const Fe<Fs> xn1 = fe_sub<Fs>(xn, one);

  // l_i = w^i (x^n - 1) / (n (x - w^i)), w = omega^-1, i < bf + 2, plus
  // 1 / (x^n - 1) for h_eval: one batched inversion (Montgomery's trick).
  const uint32_t K = h.bf + 3;
  Fe<Fs> den[kAccMaxBlind + 3], pre[kAccMaxBlind + 3];
  const Fe<Fs> nfe = ldfe<Fs>(consts, h.c_n);
  for (uint32_t i = 0; i < K; i++) {
    den[i] = i + 1 < K ? fe_mul<Fs>(nfe, fe_sub<Fs>(x, ldfe<Fs>(consts, h.c_wpow + i))) : xn1;
    pre[i] = i ? fe_mul<Fs>(pre[i - 1], den[i]) : den[i];
  }
  Fe<Fs> inv = fe_inv<Fs>(pre[K - 1]);
  for (uint32_t i = K - 1; i > 0; i--) {
    const Fe<Fs> t = fe_mul<Fs>(inv, pre[i - 1]);
    inv = fe_mul<Fs>(inv, den[i]);
    den[i] = t;  // now 1 / den_i
  }
  den[0] = inv;
  Fe<Fs> l_0 = zero, l_last = zero, l_blind = zero;
  for (uint32_t i = 0; i + 1 < K; i++) {
    const Fe<Fs> li = fe_mul<Fs>(fe_mul<Fs>(ldfe<Fs>(consts, h.c_wpow + i), xn1), den[i]);
    if (i == 0) l_0 = li;
    else if (i == h.bf + 1) l_last = li;
    else l_blind = fe_add<Fs>(l_blind, li);
  }
  const Fe<Fs> inv_xn1 = den[K - 1];
  const Fe<Fs> omb = fe_sub<Fs>(one, fe_add<Fs>(l_last, l_blind));  // 1 - (l_last + l_blind)

  // expressions in order gates, permutation, lookups; h = h*y + expr
  Fe<Fs> hv = acc_eval_code<Fs>(prog + h.p_gate, h.n_gate, sc, h, consts, zero, y);
  if (h.n_perm_sets) {
    const uint32_t* ps = sc + 8ull * h.sc_perm;
    auto zp = [&](uint32_t i) { return ldfe<Fs>(ps, 3 * i); };
    auto zpn = [&](uint32_t i) { return ldfe<Fs>(ps, 3 * i + 1); };
    auto zpl = [&](uint32_t i) { return ldfe<Fs>(ps, 3 * i + 2); };
    hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_0, fe_sub<Fs>(one, zp(0))));
    const Fe<Fs> zl = zp(h.n_perm_sets - 1);
    hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_last, fe_sub<Fs>(fe_sqr<Fs>(zl), zl)));
    for (uint32_t i = 1; i < h.n_perm_sets; i++)
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_0, fe_sub<Fs>(zp(i), zpl(i - 1))));
    const Fe<Fs> bx = fe_mul<Fs>(beta, x);
    for (uint32_t ci = 0; ci < h.n_perm_sets; ci++) {
      Fe<Fs> left = zpn(ci), right = zp(ci);
      const uint32_t k1 = min(h.n_perm_cols, (ci + 1) * h.perm_chunk);
      for (uint32_t k = ci * h.perm_chunk; k < k1; k++) {
        const Fe<Fs> ev = ldfe<Fs>(sc, prog[h.p_permcol + k]);
        const Fe<Fs> sg = ldfe<Fs>(sc, h.sc_sigma + k);
        left = fe_mul<Fs>(left, fe_add<Fs>(fe_add<Fs>(fe_mul<Fs>(beta, sg), ev), gamma));
        const Fe<Fs> t = fe_mul<Fs>(bx, ldfe<Fs>(consts, h.c_delta + k));
        right = fe_mul<Fs>(right, fe_add<Fs>(fe_add<Fs>(t, ev), gamma));
      }
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(fe_sub<Fs>(left, right), omb));
    }
  }
  if (h.num_lookups) {
    const Fe<Fs> cin = acc_eval_code<Fs>(prog + h.p_lkin, h.n_lkin, sc, h, consts, zero, theta);
    const Fe<Fs> ctab = acc_eval_code<Fs>(prog + h.p_lktab, h.n_lktab, sc, h, consts, zero, theta);
    const Fe<Fs> rfac = fe_mul<Fs>(fe_add<Fs>(cin, beta), fe_add<Fs>(ctab, gamma));
    for (uint32_t i = 0; i < h.num_lookups; i++) {
      const uint32_t e = h.sc_lk + 5 * i;
      const Fe<Fs> z = ldfe<Fs>(sc, e), zw = ldfe<Fs>(sc, e + 1), a = ldfe<Fs>(sc, e + 2),
                   ap = ldfe<Fs>(sc, e + 3), s = ldfe<Fs>(sc, e + 4);
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_0, fe_sub<Fs>(one, z)));
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_last, fe_sub<Fs>(fe_sqr<Fs>(z), z)));
      const Fe<Fs> left = fe_mul<Fs>(fe_mul<Fs>(fe_add<Fs>(a, beta), fe_add<Fs>(s, gamma)), zw);
      const Fe<Fs> right = fe_mul<Fs>(rfac, z);
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(omb, fe_sub<Fs>(left, right)));
      const Fe<Fs> as = fe_sub<Fs>(a, s);
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(l_0, as));
      hv = fe_add<Fs>(fe_mul<Fs>(hv, y), fe_mul<Fs>(omb, fe_mul<Fs>(as, fe_sub<Fs>(a, ap))));
    }
  }
  const Fe<Fs> h_eval = fe_mul<Fs>(hv, inv_xn1);
  if (h_out) stfe<Fs>(h_out, b, h_eval);

  // calc_witness coefficients (closed form of the Horner walks)
  Fe<Fs> up[kAccMaxSets];
  up[h.nsets - 1] = one;
  for (int j = (int)h.nsets - 2; j >= 0; j--) up[j] = fe_mul<Fs>(up[j + 1], u);
  for (uint32_t t = 0; t < h.nslots; t++) stfe<Fs>(cf, t, zero);
  Fe<Fs> coefH = zero, ev = zero;
  uint32_t qi = 0;
  for (uint32_t j = 0; j < h.nsets; j++) {
    const uint32_t m = prog[h.p_setlen + j];
    // c_i = u^{S-1-j} v^{m-1-i}, walked from the last query of the set
    Fe<Fs> c = up[j];
    for (int i = (int)m - 1; i >= 0; i--) {
      const uint32_t slot = prog[h.p_query + 2 * (qi + i)], eidx = prog[h.p_query + 2 * (qi + i) + 1];
      const Fe<Fs> e = eidx == kEvalH ? h_eval : ldfe<Fs>(sc, eidx);
      ev = fe_add<Fs>(ev, fe_mul<Fs>(c, e));
      if (slot == kSlotH) coefH = fe_add<Fs>(coefH, c);
      else stfe<Fs>(cf, slot, fe_add<Fs>(ldfe<Fs>(cf, slot), c));
      c = fe_mul<Fs>(c, v);
    }
    qi += m;
    stfe<Fs>(cf, h.nslots + j, up[j]);
    stfe<Fs>(cf, h.nslots + h.nsets + j, fe_mul<Fs>(fe_mul<Fs>(up[j], ldfe<Fs>(consts, h.c_omega_eval + j)), x));
  }
  Fe<Fs> xp = one;
  for (uint32_t i = 0; i < h.nh; i++) {
    stfe<Fs>(cf, h.h_slot0 + i, fe_add<Fs>(ldfe<Fs>(cf, h.h_slot0 + i), fe_mul<Fs>(coefH, xp)));
    xp = fe_mul<Fs>(xp, xn);
  }
  stfe<Fs>(cf, h.T - 1, fe_neg<Fs>(ev));
  for (uint32_t t = 0; t < h.T; t++) stfe<Fs>(cf, t, fe_from_mont<Fs>(ldfe<Fs>(cf, t)));
}

template <class Cv>
__global__ void __launch_bounds__(256) k_acc_termmul(AccumHdr h, const uint32_t* __restrict__ prog,
                                                     const uint32_t* __restrict__ coef,
                                                     const uint32_t* __restrict__ points,
                                                     const uint32_t* __restrict__ vk,
                                                     Xyzz<typename Cv::Base>* __restrict__ part) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= h.B * h.T) return;
  const uint32_t b = g / h.T, t = g - b * h.T;
  const uint32_t src = prog[h.p_termsrc + t];
  const uint32_t idx = src & 0x0FFFFFFFu;
  const uint32_t* pp = (src >> 28) == 0 ? points + 16ull * ((size_t)h.npts * b + idx) : vk + 16ull * idx;
  const Aff<F> P = load_aff<F>(pp);
  const Fe<Fs> c = ldfe<Fs>(coef, g);
  store_xyzz<F>(&part[g], aff_is_inf<F>(P) ? xyzz_inf<F>() : scalar_mul<F, Fs>(c, P));
}

template <class Cv>
__global__ void __launch_bounds__(64) k_acc_sum(AccumHdr h, const Xyzz<typename Cv::Base>* __restrict__ part,
                                                uint32_t* __restrict__ out) {
  using F = typename Cv::Base;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= h.B * 4) return;
  const uint32_t b = g >> 2, o = g & 3;
  // MultiopenVar order: w, zw, f, e
  const uint32_t lo = o == 0 ? h.nslots : o == 1 ? h.nslots + h.nsets : o == 2 ? 0 : h.T - 1;
  const uint32_t hi = o == 0 ? h.nslots + h.nsets : o == 1 ? h.nslots + 2 * h.nsets : o == 2 ? h.nslots : h.T;
  Xyzz<F> acc = xyzz_inf<F>();
  for (uint32_t t = lo; t < hi; t++) acc = xyzz_add<F>(acc, load_xyzz<F>(&part[(size_t)b * h.T + t]));
  const Aff<F> a = xyzz_to_aff<F>(acc);
  uint4* q = reinterpret_cast<uint4*>(out + 16ull * g);
  store_fe4<F>(q, a.x);
  store_fe4<F>(q + 2, a.y);
}

}  // namespace pm

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
//   k_acc_termmul  one lane per (proof, term) or per two terms of one output:
//                  [coef] P by GLV and signed 3-bit windows (43 windows of 3
//                  doublings, shared by a lane's terms, and 2 mixed additions
//                  per term), XYZZ.
//   k_acc_sum      lanes or quads per (proof, output): sums its terms, converts
//                  to the unique affine point (w, zw, f, e order of MultiopenVar).
// Scalars / points use the Rust in-memory Montgomery layout (pasta_msm.h).
#pragma once
#include "accum_plan.hpp"
#include "msm_kernels.hpp"
#include "curve29.hpp"
#include "coop29.hpp"
#include "slice29.hpp"
#include "glv.hpp"

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
  // the same w^i (i < bf + 2) and n as canonical R = 2^261 integers, packed
  // (k_acc_scalars' Lagrange chain runs in the radix-2^29 form)
  uint32_t c_wpow29, c_n29;
  // powers-of-two tables (split path): Tp proof-point terms; p_psrc: their
  // point indices in slot order (Tp words); p_rank: T words, term t's rank
  // among the proof-point terms (VK terms read the per-VK tables instead)
  uint32_t Tp, p_psrc, p_rank;
  // proof-bytes entry (round 5): twist = 1 makes the ladders read each proof
  // point's x from the proof bytes (p_pbyte: Tp words, the byte offset of
  // term tp's point in a proof, kAccNoByte for an instance commitment, read
  // affine from inst) and run on the twist E_A (acc_chain_start), so they need
  // no decoded points; k_acc_termadd maps its sums back to the curve with the
  // decoder's factors (A, y A) per point
  uint32_t twist, p_pbyte, pstride, ninst;
};
constexpr uint32_t kAccNoByte = 0xffffffffu;
constexpr uint32_t kAccCorrWords = 6;  // uint4 per point in the correction table: A, y A (pow_st layout)

template <class Fs>
__device__ __forceinline__ Fe<Fs> ldfe(const uint32_t* base, uint32_t idx) {
  return load_fe4<Fs>(reinterpret_cast<const uint4*>(base + 8ull * idx));
}
template <class Fs>
__device__ __forceinline__ void stfe(uint32_t* base, uint32_t idx, const Fe<Fs>& v) {
  store_fe4<Fs>(reinterpret_cast<uint4*>(base + 8ull * idx), v);
}

// One lane's rows of field elements in LDS, word-major with a padded lane
// stride (conflict-free when the lanes of a wave read the same row).
// k_acc_scalars stages each proof's evaluations here once, with coalesced
// loads, instead of ~60 dependent global loads per lane, and accumulates the
// MSM coefficients here instead of read-modify-writes to global memory.
// per-proof status bit set by k_acc_scalars (include/pasta_msm.h
// PM_ACCUM_DENOM_ZERO); bits 0-1 come from the transcript replay
static constexpr uint32_t kAccStatusDenomZero = 4;

struct LdsRows {
  uint32_t* base;
  uint32_t lane, stride;  // stride = lanes per block + 1
  template <class Fs>
  __device__ __forceinline__ Fe<Fs> get(uint32_t row) const {
    Fe<Fs> r;
#pragma unroll
    for (int w = 0; w < 8; w++) r.l[w] = base[(row * 8 + w) * stride + lane];
    return r;
  }
  template <class Fs>
  __device__ __forceinline__ void put(uint32_t row, const Fe<Fs>& v) const {
#pragma unroll
    for (int w = 0; w < 8; w++) base[(row * 8 + w) * stride + lane] = v.l[w];
  }
};

// Postfix program (compute_expr, verifier.rs:58-151); every END folds the
// finished expression into acc = acc * mult + value (vanishing Horner in y,
// or compress_expressions in theta, lookup.rs:214-243).
template <class Fs>
__device__ Fe<Fs> acc_eval_code(const uint32_t* code, uint32_t len, const LdsRows& sc, const AccumHdr& h,
                                const uint32_t* consts, const LdsRows& stk, Fe<Fs> acc, const Fe<Fs>& mult) {
  // top of stack in registers, the entries below it in the lane's LDS rows
  // (a private array indexed by the runtime depth lived in scratch memory)
  Fe<Fs> top;
  int sp = 0;  // entries, including top
  for (uint32_t i = 0; i < len; i++) {
    const uint32_t op = code[i] & 0xffu, arg = code[i] >> 8;
    if (op == PM_EXPR_END) {
      acc = fe_add<Fs>(fe_mul<Fs>(acc, mult), top);
      sp = 0;
    } else if (op <= PM_EXPR_INSTANCE) {
      if (sp) stk.put<Fs>(sp - 1, top);
      if (op == PM_EXPR_CONST) {
        top = ldfe<Fs>(consts, h.c_user + arg);
      } else {
        const uint32_t base = op == PM_EXPR_FIXED ? h.sc_fixed : op == PM_EXPR_ADVICE ? h.sc_adv : h.sc_inst;
        top = sc.get<Fs>(base + arg);
      }
      sp++;
    } else if (op == PM_EXPR_NEG) {
      top = fe_neg<Fs>(top);
    } else if (op == PM_EXPR_SUM) {
      top = fe_add<Fs>(stk.get<Fs>(sp - 2), top);
      sp--;
    } else if (op == PM_EXPR_PROD) {
      top = fe_mul<Fs>(stk.get<Fs>(sp - 2), top);
      sp--;
    } else {  // SCALED
      top = fe_mul<Fs>(top, ldfe<Fs>(consts, h.c_user + arg));
    }
  }
  return acc;
}

// k_acc_scalars: one block of 4 waves per np proofs (np <= 64, lane = proof
// within the block).  The waves work on independent parts of the same proofs
// (divergent roles inside one wave would serialise):
//   wave 0  x^n, the Lagrange denominators' batched inversion, l_0, l_last,
//           l_blind (the long latency chain);
//   wave 1  gate expressions (Horner in y -> hv_g) and every permutation /
//           lookup identity value that does not need the l_i;
//   wave 2  the calc_witness coefficients (u / v powers, zw, H expansion)
//           and the e-term sums that do not need h_eval;
//   then wave 0 folds the identity values into h (h = h y + sel val,
//   sel in {l_0, l_last, 1 - l_last - l_blind}), h_eval and the e
//   coefficient; finally all 4 waves convert the T coefficients.
// LDS rows per proof (word-major, proof stride np + 1): [0, nsc) evaluations,
// then T coefficients, then the exchange rows (kAccX*), then the work rows of
// wave 0 (2 (bf + 3): Montgomery's-trick denominators and prefix products)
// and of wave 1 (kAccStack: the expression stack).  Nothing is indexed at
// run time in private arrays: those live in scratch memory, whose latency
// sat on every chain (4 KiB of scratch per lane, ~0.23 ms per call).
// exchange row offsets: gate value (times y^N after wave 1's fold); per
// calc_witness wave (2, 3) the e-term sum, the H-query coefficient sum and
// H's coefficient; wave 1's fold of the
// identity values by selector (l_0, l_last, 1 - l_last - l_blind); then the
// identity values themselves
constexpr uint32_t kAccXHvg = 0, kAccXEvs = 1, kAccXCeh = 2, kAccXW3 = 3, kAccXFold = 7,
                   kAccXVals = 10;
constexpr int kAccSelL0 = 0, kAccSelLast = 1, kAccSelOmb = 2;

// identity values of the permutation / lookup arguments in h-fold order
// (permutation.rs:190-324, lookup.rs:173-311) with their selector
__host__ __device__ inline uint32_t acc_num_vals(const AccumHdr& h) {
  return (h.n_perm_sets ? 2 * h.n_perm_sets + 1 : 0) + 5 * h.num_lookups;
}

// LDS words k_acc_scalars keeps after its per-proof rows: the constant table
// and the program (read by every lane's chains; from LDS instead of global
// loads, whose ~1 us latency sat on the lone-wave chains, round 5)
__host__ __device__ inline uint32_t acc_scalars_tail_words(const AccumHdr& h) {
  return 8 * (h.c_n29 + 1) + (h.p_rank + h.T);
}

// Wave 0's Lagrange chain with a quad per proof (blocks of up to 16 proofs,
// round 5): the lone-lane chain (x^n, 2K products into the batched inverse,
// 2K back out, 2K for the l_i: ~72 us) split over the quad's four lanes.
//   A  lane 0 squares x log n times; meanwhile lane j = 1..3 forms its dens
//      den_i = n (x - w^i), i = j - 1 (mod 3), with its own prefix products
//      and w^i * prefix (rows i and K + i)
//   B  A = P1 P2, Bv = P3 (x^n - 1), then D = A Bv and the cofactors of each
//      lane's product (S1 = P2 Bv, S2 = P1 Bv, S3 = A (x^n - 1), S4 = A P3)
//   C  1 / D (quad safegcd)
//   D  one step: lane 0 1 / (x^n - 1), lane j 1 / P_j
//   E  lane j walks its dens back: t_i = w^i / den_i = R (w^i prefix_i),
//      R *= den_i; sums t_i over the blinding rows, keeps t_0, t_{bf+1}
//   F  l_0, l_last, l_blind = (x^n - 1) t (one step over three lanes)
// Results (Fe, R = 2^256) go to the proof's wk rows 0..3: l_0, l_last,
// l_blind, 1 / (x^n - 1); wave 0's lane for the proof reads them after the
// barrier.  Same values as the one-lane chain.
template <class Fs>
__device__ __forceinline__ void acc_lagrange_q(const AccumHdr& h, const LdsRows& wk, const uint32_t* consts,
                                               const uint32_t* __restrict__ challenges, uint32_t b0, uint32_t nv,
                                               uint32_t* __restrict__ status) {
  using K29 = F29Consts<Fs>;
  const uint32_t pl = threadIdx.x & 63u, p = pl >> 2, q = pl & 3u;
  const bool own = p < nv;
  const LdsRows wq{wk.base, p, wk.stride};
  const uint32_t K = h.bf + 3, nd = K - 1;  // dens of x - w^i, i < nd (the K-th is x^n - 1)
  auto put29 = [&](uint32_t row, const F29<Fs>& v) {
    Fe<Fs> w;
    f29_pack<Fs>(v, w.l);
    wq.put<Fs>(row, w);
  };
  auto get29 = [&](uint32_t row) { return f29_unpack<Fs>(wq.get<Fs>(row).l); };
  auto ld29 = [&](uint32_t idx) { return f29_unpack<Fs>(ldfe<Fs>(consts, idx).l); };  // canonical R261
  const uint32_t mq0 = q == 0 ? ~0u : 0u;
  auto sel = [&](uint32_t m, const F29<Fs>& a, const F29<Fs>& b) {  // m ? a : b, limb-wise
    F29<Fs> r;
#pragma unroll
    for (int i = 0; i < 9; i++) r.l[i] = bsel(m, a.l[i], b.l[i]);
    return r;
  };
  const Fe<Fs> xfe = ldfe<Fs>(challenges + 8ull * 7 * (b0 + (own ? p : 0u)), 4);
  const F29<Fs> x29 = f29_from_r256<Fs>(xfe.l);  // < 2p
  const F29<Fs> one29 = f29_const<Fs>(K29::ONE), nfe = ld29(h.c_n29);
  // --- A
  const uint32_t nk = q == 0 ? 0u : (nd + 3u - q) / 3u;  // dens of this lane (i = q - 1 + 3 k)
  const uint32_t nkmax = (nd + 2u) / 3u;
  const uint32_t steps = max(h.log_n, 3u * nkmax);
  F29<Fs> xn = x29, pre = one29, den = one29;
  for (uint32_t s = 0; s < steps; s++) {
    const uint32_t kind = s % 3u, k = s / 3u;
    const uint32_t i = q - 1u + 3u * k, ic = i < nd ? i : 0u;
    const bool valid = q != 0 && k < nk;
    const F29<Fs> w = ld29(h.c_wpow29 + ic);
    F29<Fs> a, b;
    if (kind == 0) {  // den_i = n (x - w^i)
      a = nfe;
      b = f29_norm<Fs>(f29_sub<Fs>(x29, w, K29::K2));
    } else if (kind == 1) {  // w^i * prefix before i
      a = w;
      b = pre;
    } else {  // prefix *= den_i
      a = pre;
      b = den;
    }
    const F29<Fs> r = f29_mul_c<Fs>(sel(mq0, xn, a), sel(mq0, xn, b));
    if (q == 0) {
      if (s < h.log_n) xn = r;
    } else if (valid) {
      if (kind == 0) {
        den = r;
        put29(ic, r);
      } else if (kind == 1) {
        put29(K + ic, r);
      } else {
        pre = r;
      }
    }
  }
  // --- B
  const F29<Fs> xn1 = f29_reduce3<Fs>(f29_norm<Fs>(f29_sub<Fs>(qbc<0>(xn), one29, K29::K2)));  // < 3p
  const F29<Fs> P1 = qbc<1>(pre), P2 = qbc<2>(pre), P3 = qbc<3>(pre);
  const F29<Fs> r1 = qmul<Fs>(q, P1, P2, P3, xn1, one29, one29, one29, one29);
  const F29<Fs> A = qbc<0>(r1), Bv = qbc<1>(r1);
  const F29<Fs> r2 = qmul<Fs>(q, A, Bv, P2, Bv, P1, Bv, A, xn1);  // D, S1, S2, S3
  const F29<Fs> S4 = f29_mul_c<Fs>(A, P3);
  const F29<Fs> D = qbc<0>(r2);
  // a zero denominator (x^n = 1, or x = omega^-i for a Lagrange basis point)
  // is where the reference's main_gate.div fails (vanishing.rs:175,
  // verifier.rs:580): flag the proof; its outputs are then unspecified
  if (q == 0 && own && status && f29_is_zero_mod<Fs>(D)) status[b0 + p] |= kAccStatusDenomZero;
  // --- C, D
  const F29<Fs> inv = f29_inv_q<Fs>(D);
  F29<Fs> R = f29_mul_c<Fs>(inv, sel(mq0, S4, r2));  // lane 0: 1 / (x^n - 1); lane j: 1 / P_j
  const F29<Fs> inv_xn1 = qbc<0>(R);
  // --- E
  F29<Fs> t0 = f29_zero<Fs>(), tl = t0, tb = t0;
  for (uint32_t kk = 0; kk < nkmax; kk++) {
    const bool valid = kk < nk;
    const uint32_t k = valid ? nk - 1u - kk : 0u, i = q - 1u + 3u * k, ic = q != 0 && i < nd ? i : 0u;
    const F29<Fs> t = f29_mul_c<Fs>(R, get29(K + ic));  // w^i / den_i
    R = f29_mul_c<Fs>(R, get29(ic));
    if (valid) {
      if (i == 0) t0 = t;
      else if (i == h.bf + 1) tl = t;
      else tb = f29_reduce3<Fs>(f29_norm<Fs>(f29_add<Fs>(tb, t)));  // < 3p
    }
  }
  auto qsum = [&](const F29<Fs>& v) {  // sum over lanes 1..3, < 9p
    return f29_norm<Fs>(f29_add<Fs>(f29_add<Fs>(qbc<1>(v), qbc<2>(v)), qbc<3>(v)));
  };
  const F29<Fs> t0s = f29_reduce3<Fs>(qsum(t0)), tls = f29_reduce3<Fs>(qsum(tl)), tbs = f29_reduce3<Fs>(qsum(tb));
  // --- F: lane 0 l_0, 1 l_last, 2 l_blind, 3 carries 1 / (x^n - 1)
  // (lane 3's product by one (R) is 1 / (x^n - 1) itself, < 2p like the others)
  const F29<Fs> lv = qmul<Fs>(q, xn1, t0s, xn1, tls, xn1, tbs, inv_xn1, one29);
  Fe<Fs> o;
  f29_to_r256<Fs>(lv, o.l);
  if (own) wq.put<Fs>(q, o);
}

template <class Fs>
__global__ void __launch_bounds__(256) k_acc_scalars(AccumHdr h, const uint32_t* __restrict__ prog_g,
                                                     const uint32_t* __restrict__ consts_g,
                                                     const uint32_t* __restrict__ scalars,
                                                     const uint32_t* __restrict__ challenges,
                                                     uint32_t* __restrict__ coef, uint32_t* __restrict__ h_out,
                                                     uint32_t np, uint32_t* __restrict__ status) {
  extern __shared__ uint32_t acc_lds[];
  const uint32_t role = threadIdx.x >> 6, pl = threadIdx.x & 63;
  const uint32_t b0 = blockIdx.x * np, b = b0 + pl;
  const uint32_t nv = min(np, h.B - b0);  // proofs in this block
#ifdef PM_ACC_PROFILE
  const uint64_t pc0 = wall_clock64();
#endif
  const uint32_t r_wk = h.nsc + h.T + kAccXVals + acc_num_vals(h);
  // rows after the stack: wave 3's slot coefficients (cf3, nslots rows), then
  // the powers x^{n i} of the H expansion (nh rows)
  const uint32_t r_cf3 = r_wk + 2 * (h.bf + 3) + kAccStack, r_xp = r_cf3 + h.nslots;
  uint32_t* const consts = acc_lds + (size_t)8 * (r_xp + h.nh) * (np + 1);
  __shared__ uint32_t xp_ready;  // wave 3 has written the x^{n i} rows
  if (threadIdx.x == 0) xp_ready = 0;
  uint32_t* const prog = consts + 8 * (h.c_n29 + 1);
  {  // coalesced staging of the block's evaluations (rows [0, nsc)), the constants and the program
    const uint32_t per = 8 * h.nsc;
    const uint32_t* src = scalars + (size_t)per * b0;
    for (uint32_t f = threadIdx.x; f < per * nv; f += blockDim.x) {
      const uint32_t q = f / per, k = f - q * per;
      acc_lds[k * (np + 1) + q] = src[f];
    }
    for (uint32_t f = threadIdx.x; f < 8 * (h.c_n29 + 1); f += blockDim.x) consts[f] = consts_g[f];
    for (uint32_t f = threadIdx.x; f < h.p_rank + h.T; f += blockDim.x) prog[f] = prog_g[f];
  }
  __syncthreads();
#ifdef PM_ACC_PROFILE
  const uint64_t pc1 = wall_clock64();
#endif
  const bool live = pl < nv;
  const LdsRows sc{acc_lds, pl, np + 1};
  const LdsRows cf{acc_lds + (size_t)8 * h.nsc * (np + 1), pl, np + 1};
  const LdsRows xr{acc_lds + (size_t)8 * (h.nsc + h.T) * (np + 1), pl, np + 1};
  const LdsRows wk{acc_lds + (size_t)8 * r_wk * (np + 1), pl, np + 1};                      // wave 0
  const LdsRows stk{acc_lds + (size_t)8 * (r_wk + 2 * (h.bf + 3)) * (np + 1), pl, np + 1};  // wave 1
  const LdsRows cf3{acc_lds + (size_t)8 * r_cf3 * (np + 1), pl, np + 1};                     // wave 3
  const LdsRows xpr{acc_lds + (size_t)8 * r_xp * (np + 1), pl, np + 1};                      // wave 3 -> 2
  const uint32_t* ch = challenges + 8ull * 7 * (live ? b : b0);
  const Fe<Fs> one = fe_one<Fs>(), zero = fe_zero<Fs>();
  const Fe<Fs> y = ldfe<Fs>(ch, 3), x = ldfe<Fs>(ch, 4);

  if (role == 0) {
    // Wave 0: the long chain of the kernel, the Lagrange values and 1 / (x^n
    // - 1) in the radix-2^29 lazy form with a quad per proof (acc_lagrange_q;
    // np <= 16: the host caps it); the results are read after the barrier
    acc_lagrange_q<Fs>(h, wk, consts, challenges, b0, nv, status);
  } else if (live && role == 1) {
    // gates (verifier.rs:593-605), then the identity values in fold order
    xr.put<Fs>(kAccXHvg, acc_eval_code<Fs>(prog + h.p_gate, h.n_gate, sc, h, consts, stk, zero, y));
    const Fe<Fs> beta = ldfe<Fs>(ch, 1), gamma = ldfe<Fs>(ch, 2);
    uint32_t vi = kAccXVals;
    if (h.n_perm_sets) {
      auto zp = [&](uint32_t i) { return sc.get<Fs>(h.sc_perm + 3 * i); };
      auto zpn = [&](uint32_t i) { return sc.get<Fs>(h.sc_perm + 3 * i + 1); };
      auto zpl = [&](uint32_t i) { return sc.get<Fs>(h.sc_perm + 3 * i + 2); };
      xr.put<Fs>(vi++, fe_sub<Fs>(one, zp(0)));                              // l_0
      const Fe<Fs> zl = zp(h.n_perm_sets - 1);
      xr.put<Fs>(vi++, fe_sub<Fs>(fe_sqr<Fs>(zl), zl));                      // l_last
      for (uint32_t i = 1; i < h.n_perm_sets; i++) xr.put<Fs>(vi++, fe_sub<Fs>(zp(i), zpl(i - 1)));  // l_0
      const Fe<Fs> bx = fe_mul<Fs>(beta, x);
      for (uint32_t ci = 0; ci < h.n_perm_sets; ci++) {                      // omb
        Fe<Fs> left = zpn(ci), right = zp(ci);
        const uint32_t k1 = min(h.n_perm_cols, (ci + 1) * h.perm_chunk);
        for (uint32_t k = ci * h.perm_chunk; k < k1; k++) {
          const Fe<Fs> ev = sc.get<Fs>(prog[h.p_permcol + k]);
          const Fe<Fs> sg = sc.get<Fs>(h.sc_sigma + k);
          left = fe_mul<Fs>(left, fe_add<Fs>(fe_add<Fs>(fe_mul<Fs>(beta, sg), ev), gamma));
          const Fe<Fs> t = fe_mul<Fs>(bx, ldfe<Fs>(consts, h.c_delta + k));
          right = fe_mul<Fs>(right, fe_add<Fs>(fe_add<Fs>(t, ev), gamma));
        }
        xr.put<Fs>(vi++, fe_sub<Fs>(left, right));
      }
    }
    if (h.num_lookups) {
      const Fe<Fs> theta = ldfe<Fs>(ch, 0);
      const Fe<Fs> cin = acc_eval_code<Fs>(prog + h.p_lkin, h.n_lkin, sc, h, consts, stk, zero, theta);
      const Fe<Fs> ctab = acc_eval_code<Fs>(prog + h.p_lktab, h.n_lktab, sc, h, consts, stk, zero, theta);
      const Fe<Fs> rfac = fe_mul<Fs>(fe_add<Fs>(cin, beta), fe_add<Fs>(ctab, gamma));
      for (uint32_t i = 0; i < h.num_lookups; i++) {
        const uint32_t e = h.sc_lk + 5 * i;
        const Fe<Fs> z = sc.get<Fs>(e), zw = sc.get<Fs>(e + 1), a = sc.get<Fs>(e + 2), ap = sc.get<Fs>(e + 3),
                     s = sc.get<Fs>(e + 4);
        const Fe<Fs> left = fe_mul<Fs>(fe_mul<Fs>(fe_add<Fs>(a, beta), fe_add<Fs>(s, gamma)), zw);
        const Fe<Fs> as = fe_sub<Fs>(a, s);
        xr.put<Fs>(vi++, fe_sub<Fs>(one, z));                                     // l_0
        xr.put<Fs>(vi++, fe_sub<Fs>(fe_sqr<Fs>(z), z));                           // l_last
        xr.put<Fs>(vi++, fe_sub<Fs>(left, fe_mul<Fs>(rfac, z)));                  // omb
        xr.put<Fs>(vi++, as);                                                     // l_0
        xr.put<Fs>(vi++, fe_mul<Fs>(as, fe_sub<Fs>(a, ap)));                      // omb
      }
    }
    // Fold the values into h = h y + sel v (gates first, then these in order)
    // per selector, so wave 0 needs only h = G y^N + l_0 A + l_last B + omb C
    // once its l_i are known (round 5: the 2 N products of the fold moved off
    // wave 0's chain, which is the kernel's longest)
    // value k of N is weighted y^{N-1-k}: walked from the last value with a
    // running power of y (2 products per value instead of 4 Horner steps)
    auto sel_of = [&](uint32_t k) {  // the selector of value k in fold order
      if (h.n_perm_sets) {
        if (k < 2 * h.n_perm_sets + 1) return k == 0 ? kAccSelL0 : k == 1 ? kAccSelLast : k <= h.n_perm_sets ? kAccSelL0 : kAccSelOmb;
        k -= 2 * h.n_perm_sets + 1;
      }
      const uint32_t r = k % 5;  // lookups: l_0, l_last, omb, l_0, omb
      return r == 0 || r == 3 ? kAccSelL0 : r == 1 ? kAccSelLast : kAccSelOmb;
    };
    Fe<Fs> A = zero, Bs = zero, C = zero, yp = one;
#pragma unroll 1
    for (uint32_t k = vi - kAccXVals; k-- > 0;) {
      const Fe<Fs> t = fe_mul<Fs>(xr.get<Fs>(kAccXVals + k), yp);
      const int sel = sel_of(k);
      if (sel == kAccSelL0) A = fe_add<Fs>(A, t);
      else if (sel == kAccSelLast) Bs = fe_add<Fs>(Bs, t);
      else C = fe_add<Fs>(C, t);
      yp = fe_mul<Fs>(yp, y);
    }
    xr.put<Fs>(kAccXHvg, fe_mul<Fs>(xr.get<Fs>(kAccXHvg), yp));  // G y^N
    xr.put<Fs>(kAccXFold, A);
    xr.put<Fs>(kAccXFold + 1, Bs);
    xr.put<Fs>(kAccXFold + 2, C);
  } else if (live && role >= 2) {
    // calc_witness coefficients (closed form of the Horner walks), the
    // query sets split between waves 2 (sets [J, S)) and 3 (sets [0, J)) at
    // about half the queries (round 5: one wave took ~117 us at B = 16,
    // profiles/r05/acc_scalars_roles.txt); each keeps its own slot sums
    // (cf / cf3, added in the conversion) and e-term / H sums (exchange rows).
    // The e term is -(sum_{non-H} c e + h_eval sum_{H queries} c), finished by
    // wave 0; H's coefficients are expanded below (x^{n i} from wave 3).
    const bool w3 = role == 3;
    const LdsRows& cfs = w3 ? cf3 : cf;
    const Fe<Fs> v = ldfe<Fs>(ch, 5), u = ldfe<Fs>(ch, 6);
    for (uint32_t t = 0; t < h.nslots; t++) cfs.put<Fs>(t, zero);
    uint32_t qtot = 0, J = 0;
    for (uint32_t j = 0; j < h.nsets; j++) qtot += prog[h.p_setlen + j];
    for (uint32_t acc = 0; J < h.nsets && 2 * (acc + prog[h.p_setlen + J]) <= qtot; J++) acc += prog[h.p_setlen + J];
    const uint32_t jlo = w3 ? 0u : J, jhi = w3 ? J : h.nsets;
    uint32_t qi = 0;
    for (uint32_t j = 0; j < jhi; j++) qi += prog[h.p_setlen + j];
    // sets from the last, so u^{S-1-j} is a running product (every
    // coefficient is a sum, so the order of the additions does not matter)
    Fe<Fs> upj = one;
    for (uint32_t j = jhi; j < h.nsets; j++) upj = fe_mul<Fs>(upj, u);
    Fe<Fs> coefH = zero, ev = zero, ceh = zero;
    for (int j = (int)jhi - 1; j >= (int)jlo; j--) {
      const uint32_t m = prog[h.p_setlen + j];
      qi -= m;
      // c_i = u^{S-1-j} v^{m-1-i}, walked from the last query of the set
      Fe<Fs> c = upj;
      for (int i = (int)m - 1; i >= 0; i--) {
        const uint32_t slot = prog[h.p_query + 2 * (qi + i)], eidx = prog[h.p_query + 2 * (qi + i) + 1];
        if (eidx == kEvalH) ceh = fe_add<Fs>(ceh, c);
        else ev = fe_add<Fs>(ev, fe_mul<Fs>(c, sc.get<Fs>(eidx)));
        if (slot == kSlotH) coefH = fe_add<Fs>(coefH, c);
        else cfs.put<Fs>(slot, fe_add<Fs>(cfs.get<Fs>(slot), c));
        c = fe_mul<Fs>(c, v);
      }
      cf.put<Fs>(h.nslots + j, upj);
      cf.put<Fs>(h.nslots + h.nsets + j, fe_mul<Fs>(fe_mul<Fs>(upj, ldfe<Fs>(consts, h.c_omega_eval + j)), x));
      upj = fe_mul<Fs>(upj, u);
    }
    const uint32_t xo = w3 ? kAccXW3 : 0u;
    xr.put<Fs>(kAccXEvs + xo, ev);
    xr.put<Fs>(kAccXCeh + xo, ceh);
    // H = sum_i x^{n i} h_i (vanishing.rs:178-188): h_i's coefficient gains
    // coefH x^{n i}, each wave adding its own share of coefH to its own slot
    // rows.  Wave 3 (far ahead of wave 2) makes the powers and raises
    // xp_ready; wave 2 then needs nh products.  (Round 5: wave 2 did it all
    // after the barrier, ~20 us on the kernel's critical path.)
    if (h.nh) {
      if (w3) {
        Fe<Fs> xn = x;
        for (uint32_t i = 0; i < h.log_n; i++) xn = fe_sqr<Fs>(xn);
        Fe<Fs> xp = one;
        for (uint32_t i = 0; i < h.nh; i++) {
          xpr.put<Fs>(i, xp);
          cf3.put<Fs>(h.h_slot0 + i, fe_add<Fs>(cf3.get<Fs>(h.h_slot0 + i), fe_mul<Fs>(coefH, xp)));
          xp = fe_mul<Fs>(xp, xn);
        }
        if (pl == 0) __hip_atomic_store(&xp_ready, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      } else {
        while (__hip_atomic_load(&xp_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) == 0)
          __builtin_amdgcn_s_sleep(1);
        for (uint32_t i = 0; i < h.nh; i++)
          cf.put<Fs>(h.h_slot0 + i, fe_add<Fs>(cf.get<Fs>(h.h_slot0 + i), fe_mul<Fs>(coefH, xpr.get<Fs>(i))));
      }
    }
  }
#ifdef PM_ACC_PROFILE
  const uint64_t pc2 = wall_clock64();
#endif
  __syncthreads();
#ifdef PM_ACC_PROFILE
  const uint64_t pc3 = wall_clock64();
#endif
  if (live && role == 0) {
    // acc_lagrange_q's results
    const Fe<Fs> l_0 = wk.get<Fs>(0), l_last = wk.get<Fs>(1);
    const Fe<Fs> omb = fe_sub<Fs>(one, fe_add<Fs>(l_last, wk.get<Fs>(2)));
    const Fe<Fs> inv_xn1 = wk.get<Fs>(3);
    // expressions in order gates, permutation, lookups: h = h y + sel expr,
    // folded per selector by wave 1
    const Fe<Fs> hv = fe_add<Fs>(
        fe_add<Fs>(xr.get<Fs>(kAccXHvg), fe_mul<Fs>(l_0, xr.get<Fs>(kAccXFold))),
        fe_add<Fs>(fe_mul<Fs>(l_last, xr.get<Fs>(kAccXFold + 1)), fe_mul<Fs>(omb, xr.get<Fs>(kAccXFold + 2))));
    const Fe<Fs> h_eval = fe_mul<Fs>(hv, inv_xn1);
    if (h_out) stfe<Fs>(h_out, b, h_eval);
    const Fe<Fs> evs = fe_add<Fs>(xr.get<Fs>(kAccXEvs), xr.get<Fs>(kAccXEvs + kAccXW3));
    const Fe<Fs> ceh = fe_add<Fs>(xr.get<Fs>(kAccXCeh), xr.get<Fs>(kAccXCeh + kAccXW3));
    const Fe<Fs> ev = fe_add<Fs>(evs, fe_mul<Fs>(ceh, h_eval));
    cf.put<Fs>(h.T - 1, fe_neg<Fs>(ev));
  }
#ifdef PM_ACC_PROFILE
  const uint64_t pc4 = wall_clock64();
#endif
  __syncthreads();
  // the T coefficients of the nv proofs over all 256 threads (item = (t,
  // proof), consecutive threads on consecutive proofs): at np = 16 the
  // lane-per-proof form left 3/4 of every wave idle and took ~20 us
  for (uint32_t i = threadIdx.x; i < nv * h.T; i += blockDim.x) {
    const uint32_t t = i / nv, q = i - t * nv;
    const LdsRows cq{cf.base, q, cf.stride}, c3q{cf3.base, q, cf3.stride};
    const Fe<Fs> c = t < h.nslots ? fe_add<Fs>(cq.get<Fs>(t), c3q.get<Fs>(t)) : cq.get<Fs>(t);
    stfe<Fs>(coef + 8ull * h.T * (b0 + q), t, fe_from_mont<Fs>(c));
  }
#ifdef PM_ACC_PROFILE  // A/B builds only: per-wave phase times of block 0 (10 ns ticks)
  const uint64_t pc5 = wall_clock64();
  if (blockIdx.x == 0 && pl == 0)
    printf("acc_scalars role %u: stage %llu phase1 %llu sync1 %llu phase2 %llu conv %llu\n", role,
           (unsigned long long)(pc1 - pc0), (unsigned long long)(pc2 - pc1), (unsigned long long)(pc3 - pc2),
           (unsigned long long)(pc4 - pc3), (unsigned long long)(pc5 - pc4));
#endif
}

// The term tables of glv_mul_w3n live in LDS, [word][lane] (72 words per lane
// and term), picked by address instead of register selects (in registers the
// kernel spilled).
constexpr uint32_t kW3Words = 4 * 18;

// The rounded GLV split of k (|k_i| < 2^127) recoded into 43 signed base-8
// digits per half, as codes (magnitude | sign << 3, 8 per word, window 0
// lowest).  FOLD: the half's sign (s1, s2 = 8 when the half is negated) is
// folded into every nonzero digit; else it is returned for the use site
// (glv_mul_w3: fewer live registers in its loop, two waves per SIMD).
template <class Cv, bool FOLD>
__device__ __forceinline__ void w3_codes(const Fe<typename Cv::Scalar>& k, uint32_t c1[6], uint32_t c2[6],
                                         uint32_t& s1, uint32_t& s2) {
  constexpr int kWin = 43;  // 3-bit windows over bits 0..128
  uint32_t k1[6], k2[6];
  bool n1, n2;
  glv_split<Cv, true>(k, k1, k2, n1, n2);
  s1 = n1 ? 8u : 0u;
  s2 = n2 ? 8u : 0u;
  uint32_t cy1 = 0, cy2 = 0;
#pragma unroll
  for (int i = 0; i < kWin; i++) {
    const int b = 3 * i, wd = b >> 5, sh = b & 31;
    const uint64_t w1 = (uint64_t)k1[wd] | (wd + 1 < 6 ? (uint64_t)k1[wd + 1] << 32 : 0ull);
    const uint64_t w2 = (uint64_t)k2[wd] | (wd + 1 < 6 ? (uint64_t)k2[wd + 1] << 32 : 0ull);
    const uint32_t v1 = (uint32_t)(w1 >> sh) & 7u, v2 = (uint32_t)(w2 >> sh) & 7u;
    const uint32_t u1 = v1 + cy1, u2 = v2 + cy2;
    cy1 = u1 > 4u ? 1u : 0u;
    cy2 = u2 > 4u ? 1u : 0u;
    uint32_t e1, e2;
    if (FOLD) {  // u = 8: digit 0, carry 1; a nonzero digit's sign is flipped by the half's
      e1 = cy1 ? (u1 < 8u ? (8u - u1) | (8u ^ s1) : 0u) : (u1 ? u1 | s1 : 0u);
      e2 = cy2 ? (u2 < 8u ? (8u - u2) | (8u ^ s2) : 0u) : (u2 ? u2 | s2 : 0u);
    } else {     // u = 8: digit 0 (magnitude 0), carry 1
      e1 = cy1 ? ((8u - u1) | (u1 < 8u ? 8u : 0u)) : u1;
      e2 = cy2 ? ((8u - u2) | (u2 < 8u ? 8u : 0u)) : u2;
    }
    c1[i >> 3] |= e1 << (4 * (i & 7));
    c2[i >> 3] |= e2 << (4 * (i & 7));
  }
}

// The table [m]P, m = 1..4, affine canonical (one batched inversion) at LDS
// rows r0 + 18 (m - 1) + limb (x), + 9 (y), column threadIdx.x.
template <class Cv>
__device__ __forceinline__ void w3_table(const Aff<typename Cv::Base>& P, uint32_t (*tab)[256], uint32_t r0) {
  using F = typename Cv::Base;
  using K = F29Consts<F>;
  const uint32_t ln = threadIdx.x;
  auto put = [&](uint32_t row, const F29<F>& v) {
#pragma unroll
    for (int t = 0; t < 9; t++) tab[r0 + row + t][ln] = v.l[t];
  };
  const F29<F> one = f29_const<F>(K::ONE);
  const F29<F> x1 = f29_canon<F>(f29_from_r256<F>(P.x.l)), y1 = f29_canon<F>(f29_from_r256<F>(P.y.l));
  put(0, x1);
  put(9, y1);
  const Xyzz29<F> Q2 = xyzz29_dbl_impl<F, true>(x1, y1, one, one);
  bool qi = false;
  const Xyzz29<F> Q3 = xyzz29_madd<F>(Q2, x1, y1, qi);  // 2P + P: 2P != +-P (odd order)
  const Xyzz29<F> Q4 = xyzz29_dbl<F>(Q2);
  const F29<F> d2 = f29_mul_c<F>(Q2.ZZ, Q2.ZZZ), d3 = f29_mul_c<F>(Q3.ZZ, Q3.ZZZ), d4 = f29_mul_c<F>(Q4.ZZ, Q4.ZZZ);
  const F29<F> d23 = f29_mul_c<F>(d2, d3);
  const F29<F> inv = f29_inv<F>(f29_mul_c<F>(d23, d4));  // 1 / (d2 d3 d4)
  const F29<F> i4 = f29_mul_c<F>(inv, d23), i23 = f29_mul_c<F>(inv, d4);
  const F29<F> i2 = f29_mul_c<F>(i23, d3), i3 = f29_mul_c<F>(i23, d2);
  // 1 / ZZ = ZZZ / d, 1 / ZZZ = ZZ / d
  put(18, f29_canon<F>(f29_mul_c<F>(Q2.X, f29_mul_c<F>(i2, Q2.ZZZ))));
  put(27, f29_canon<F>(f29_mul_c<F>(Q2.Y, f29_mul_c<F>(i2, Q2.ZZ))));
  put(36, f29_canon<F>(f29_mul_c<F>(Q3.X, f29_mul_c<F>(i3, Q3.ZZZ))));
  put(45, f29_canon<F>(f29_mul_c<F>(Q3.Y, f29_mul_c<F>(i3, Q3.ZZ))));
  put(54, f29_canon<F>(f29_mul_c<F>(Q4.X, f29_mul_c<F>(i4, Q4.ZZZ))));
  put(63, f29_canon<F>(f29_mul_c<F>(Q4.Y, f29_mul_c<F>(i4, Q4.ZZ))));
}

// One term's half of the work in glv_mul_w3n: the codes with the halves'
// signs folded in, and the table at rows r0..
template <class Cv>
__device__ __forceinline__ void w3_prepare(const Fe<typename Cv::Scalar>& k, const Aff<typename Cv::Base>& P,
                                           uint32_t (*tab)[256], uint32_t r0, uint32_t c1[6], uint32_t c2[6]) {
  uint32_t s1, s2;
  w3_codes<Cv, true>(k, c1, c2, s1, s2);
  w3_table<Cv>(P, tab, r0);
}

// [k]P, one term (k_acc_termmul NT = 1): per window 3 doublings and the two
// halves' mixed additions, the half's sign applied at use.  (glv_mul_w3n<Cv,
// 1> over w3_prepare needs 322 registers against this loop's 247: one wave per
// SIMD instead of two.)
template <class Cv>
__device__ __forceinline__ Xyzz29<typename Cv::Base> glv_mul_w3(const Fe<typename Cv::Scalar>& k,
                                                               const Aff<typename Cv::Base>& P, uint32_t (*tab)[256]) {
  using F = typename Cv::Base;
  constexpr int kWin = 43;
  uint32_t c1[6] = {0, 0, 0, 0, 0, 0}, c2[6] = {0, 0, 0, 0, 0, 0}, s1, s2;
  w3_codes<Cv, false>(k, c1, c2, s1, s2);
  w3_table<Cv>(P, tab, 0);
  const uint32_t ln = threadIdx.x;
  const F29<F> beta = f29_const<F>(Glv<Cv>::BETA29);
  Xyzz29<F> acc = xyzz29_inf<F>();
  bool acc_inf = true;
  for (int i = kWin - 1; i >= 0; i--) {
    acc = xyzz29_dbl<F>(xyzz29_dbl<F>(xyzz29_dbl<F>(acc)));
    // this window's codes (register words picked by selects, not scratch)
    uint32_t w1 = 0, w2 = 0;
#pragma unroll
    for (int j = 0; j < 6; j++) {
      w1 = j == (i >> 3) ? c1[j] : w1;
      w2 = j == (i >> 3) ? c2[j] : w2;
    }
    const uint32_t sh = 4u * (uint32_t)(i & 7);
#pragma unroll
    for (int half = 0; half < 2; half++) {
      const uint32_t e = ((half ? w2 : w1) >> sh) & 15u, m = e & 7u;
      if (m == 0) continue;
      F29<F> qx, qy;
      const uint32_t r0 = 18u * (m - 1u);
#pragma unroll
      for (int t = 0; t < 9; t++) {
        qx.l[t] = tab[r0 + t][ln];
        qy.l[t] = tab[r0 + 9 + t][ln];
      }
      if (half) qx = f29_canon<F>(f29_mul_c<F>(beta, qx));
      if (((e ^ (half ? s2 : s1)) & 8u) != 0u) qy = f29_canon<F>(f29_neg_canon<F>(qy));
      acc = xyzz29_madd<F>(acc, qx, qy, acc_inf);
    }
  }
  return acc;
}

// sum_j [k_j] P_j over NT terms (NT = 1, 2) with signed base-8 windows
// (round 5): both rounded GLV halves of each k_j (|k_i| < 2^127) in 43 digits
// in [-4, 4], a table [m]P_j, m = 1..4 (affine, one batched inversion per
// term) serving both halves (phi: beta x per use).  Per window 3 doublings,
// shared by the NT terms (Straus), and 2 NT mixed additions: 129 + 86 steps per
// term against the 128 + 128 of a joint binary double-and-add (a wave adds
// whenever any of its lanes has a set bit, so a joint form's zero pairs save
// nothing; that form was retired in round 6), 65 + 86 at NT = 2.
// live: bit j set when term j is present and its point is not the identity.
template <class Cv, int NT>
__device__ __forceinline__ Xyzz29<typename Cv::Base> glv_mul_w3n(const Fe<typename Cv::Scalar>& k0,
                                                                const Aff<typename Cv::Base>& P0,
                                                                const Fe<typename Cv::Scalar>& k1,
                                                                const Aff<typename Cv::Base>& P1, uint32_t live,
                                                                uint32_t (*tab)[256]) {
  using F = typename Cv::Base;
  constexpr int kWin = 43;
  // four named code arrays (a [2][2][6] array went to scratch)
  uint32_t ca1[6] = {0, 0, 0, 0, 0, 0}, ca2[6] = {0, 0, 0, 0, 0, 0};
  uint32_t cb1[6] = {0, 0, 0, 0, 0, 0}, cb2[6] = {0, 0, 0, 0, 0, 0};
  if (live & 1u) w3_prepare<Cv>(k0, P0, tab, 0, ca1, ca2);
  if (NT > 1 && (live & 2u)) w3_prepare<Cv>(k1, P1, tab, kW3Words, cb1, cb2);
  const uint32_t ln = threadIdx.x;
  const F29<F> beta = f29_const<F>(Glv<Cv>::BETA29);
  Xyzz29<F> acc = xyzz29_inf<F>();
  bool acc_inf = true;
  for (int i = kWin - 1; i >= 0; i--) {
    acc = xyzz29_dbl<F>(xyzz29_dbl<F>(xyzz29_dbl<F>(acc)));
    const uint32_t sh = 4u * (uint32_t)(i & 7);
#pragma unroll
    for (int j = 0; j < NT; j++) {
#pragma unroll
      for (int half = 0; half < 2; half++) {
        // this window's code (register words picked by selects, not scratch)
        const uint32_t* cw = j == 0 ? (half ? ca2 : ca1) : (half ? cb2 : cb1);
        uint32_t wv = 0;
#pragma unroll
        for (int w = 0; w < 6; w++) wv = w == (i >> 3) ? cw[w] : wv;
        const uint32_t e = (wv >> sh) & 15u, m = e & 7u;
        if (m == 0) continue;
        F29<F> qx, qy;
        const uint32_t r0 = kW3Words * j + 18u * (m - 1u);
#pragma unroll
        for (int t = 0; t < 9; t++) {
          qx.l[t] = tab[r0 + t][ln];
          qy.l[t] = tab[r0 + 9 + t][ln];
        }
        if (half) qx = f29_canon<F>(f29_mul_c<F>(beta, qx));
        if (e & 8u) qy = f29_canon<F>(f29_neg_canon<F>(qy));
        acc = xyzz29_madd<F>(acc, qx, qy, acc_inf);
      }
    }
  }
  return acc;
}

// k_acc_termmul: a lane per term (NT = 1), or with NT = 2 a lane per pair of
// terms of one output (prog[p_pairs]: npair (t0, t1) per proof, t1 =
// kAccNoByte for a single); the lane stores the pair's sum at t0 and the
// identity at t1, so k_acc_sum folds the same rows.
template <class Cv, int NT = 1>
__global__ void __launch_bounds__(256) k_acc_termmul(AccumHdr h, const uint32_t* __restrict__ prog,
                                                     const uint32_t* __restrict__ coef,
                                                     const uint32_t* __restrict__ points,
                                                     const uint32_t* __restrict__ vk, uint32_t p_pairs,
                                                     uint32_t npair, Xyzz<typename Cv::Base>* __restrict__ part) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;  // part[] holds packed R261 (curve29.hpp) points
  __shared__ uint32_t w3tab[NT * kW3Words][256];
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t per = NT == 1 ? h.T : npair;
  if (gl >= h.B * per) return;
  const uint32_t b = gl / per, r = gl - b * per;
  const uint32_t t0 = NT == 1 ? r : prog[p_pairs + 2 * r];
  const uint32_t t1 = NT == 1 ? kAccNoByte : prog[p_pairs + 2 * r + 1];
  auto term_point = [&](uint32_t t) {
    const uint32_t src = prog[h.p_termsrc + t];
    const uint32_t idx = src & 0x0FFFFFFFu;
    return load_aff<F>((src >> 28) == 0 ? points + 16ull * ((size_t)h.npts * b + idx) : vk + 16ull * idx);
  };
  const Aff<F> P0 = term_point(t0);
  const Fe<Fs> k0 = ldfe<Fs>(coef, b * h.T + t0);
  uint32_t live = aff_is_inf<F>(P0) ? 0u : 1u;
  Aff<F> P1 = P0;
  Fe<Fs> k1 = k0;
  if (NT > 1 && t1 != kAccNoByte) {
    P1 = term_point(t1);
    k1 = ldfe<Fs>(coef, b * h.T + t1);
    if (!aff_is_inf<F>(P1)) live |= 2u;
  }
  Xyzz29<F> acc = xyzz29_inf<F>();
  if (NT == 1 && live) acc = glv_mul_w3<Cv>(k0, P0, w3tab);
  else if (live) acc = glv_mul_w3n<Cv, NT>(k0, P0, k1, P1, live, w3tab);
  store_xyzz29<F>(&part[b * h.T + t0], acc);
  if (NT > 1 && t1 != kAccNoByte) store_xyzz29<F>(&part[b * h.T + t1], xyzz29_inf<F>());
}


// ------------------------------------------------------- powers-of-two table
// At small batches one lane per term leaves most SIMDs idle and the term
// multiplication is a 128-step latency chain.  The split form stores every
// power of two of each term's point first; a term product is then a sum of
// table points only: [k]P = sum_i d_i [2^i] (+-P) + e_i [2^i] (+-phi P) over
// the non-adjacent forms d, e of the rounded GLV halves (|k_i| < 2^127, so
// 128 digits, about a third of them nonzero), spread over S lanes.  The
// table depends only on the points, so k_acc_powers runs on the main stream
// while the transcript replay and k_acc_scalars derive the coefficients.
// (Round 1 stored Q_j = [2^{16 j}] P only and each lane ran 16 dbl + add
// steps: the additions-only form has a 15-doubling longer table chain but
// ~40% fewer operations after it)
//
// The VK terms (fixed and sigma commitments, g1) have the same point in every
// proof: their tables are built once per verifying key and cached in the
// context (acc_vkpow), so only the proof commitments get a chain per proof.
//
// k_acc_powers: one quad per (proof, term) walks P, [2] P, ..., [2^127] P
// (127 Jacobian doublings, coop29.hpp) and stores every point in XYZZ form
// plus beta X: coordinates X, Y, ZZ, ZZZ, beta X (and a junk slot) of kPowWords
// uint4 each (limbs 0-3, 4-7, 8), holding the 9 radix-2^29 limbs as computed (no packing: every
// instruction on the doubling chain lanes costs, and the termadd lanes load
// them back as they are).  ZZ, ZZZ and beta X come from quad lanes that idle
// in the doubling's last two levels (jac29_dbl_q_ext), so the chain is as
// long as 127 plain doublings plus the stores.
constexpr uint32_t kPowPos = 128, kPowWords = 3, kPowCoord = 6, kPowPoint = kPowWords * kPowCoord;  // in uint4

template <class F>
__device__ __forceinline__ void pow_st(uint4* o, const F29<F>& v) {
  o[0] = make_uint4(v.l[0], v.l[1], v.l[2], v.l[3]);
  o[1] = make_uint4(v.l[4], v.l[5], v.l[6], v.l[7]);
  reinterpret_cast<uint32_t*>(o + 2)[0] = v.l[8];
}
template <class F>
__device__ __forceinline__ F29<F> pow_ld(const uint4* o) {
  const uint4 a = o[0], b = o[1];
  return F29<F>{{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, reinterpret_cast<const uint32_t*>(o + 2)[0]}};
}

// Stores of one step: the owners of jac29_dbl_q_ext's outputs write them,
// every lane executes the same four stores, and a lane that owns nothing at a
// site writes its register to the point's junk slot (coordinate 5).  (Stores
// under lane-dependent ifs were merged by the compiler into one store with a
// selected address and split into dword stores.)
//   X    every lane (all hold X3)           -> coordinate 0
//   Y    lanes 1, 2                         -> 1
//   zz   lane 3 (ZZ3)                       -> 2
//   ext  lane 3 (ZZZ3) -> 3, lane 0 (beta X3) -> 4
struct PowSites {
  uint32_t y, zz, ext;  // coordinate offsets (uint4) of this lane
  __device__ explicit PowSites(uint32_t q)
      : y((q == 1u || q == 2u ? 1u : 5u) * kPowWords),
        zz((q == 3u ? 2u : 5u) * kPowWords),
        ext((q == 3u ? 3u : q == 0u ? 4u : 5u) * kPowWords) {}
};
template <class F>
__device__ __forceinline__ void pow_store(uint4* o, const PowSites& ps, const Jac29<F>& p, const F29<F>& zz,
                                          const F29<F>& ext) {
  pow_st<F>(o, p.X);
  pow_st<F>(o + ps.y, p.Y);
  pow_st<F>(o + ps.zz, zz);
  pow_st<F>(o + ps.ext, ext);
}

// Start point of chain g < nprf + nvk as canonical R = 2^261 coordinates.
// Affine input (points / inst / vk, Rust R = 2^256 Montgomery): (x, y), inf
// for (0, 0).  From the proof bytes (h.twist): with A = x^3 + b, the point
// P_A = (A x, A^2) of E_A: y^2 = x^3 + A^3 b.  psi(X, Y) = (X / A, y0 Y / A^2)
// (y0 = sqrt(A), the decoded y) maps E_A onto the curve as a group
// isomorphism that commutes with phi (beta x, y), and doublings and additions
// never use b, so the ladder's table of E_A multiples is the curve's under
// psi; in XYZZ psi only scales ZZ by A and ZZZ by y0 A (y0^2 = A), which
// k_acc_termadd applies to each term's sum.  The chain thus needs only x: it
// runs beside the square-root decode instead of after it.  (An invalid x
// gives a meaningless chain; the decoder flags that proof.)
template <class Cv>
__device__ __forceinline__ void acc_chain_start(const AccumHdr& h, const uint32_t* __restrict__ prog,
                                                const uint32_t* __restrict__ points,
                                                const uint32_t* __restrict__ proofs,
                                                const uint32_t* __restrict__ inst, const uint32_t* __restrict__ vk,
                                                uint32_t g, F29<typename Cv::Base>& x, F29<typename Cv::Base>& y,
                                                bool& inf) {
  using F = typename Cv::Base;
  const uint32_t nprf = h.B * h.Tp;
  const uint32_t* pp;
  if (g < nprf) {
    const uint32_t b = g / h.Tp, tp = g - b * h.Tp, idx = prog[h.p_psrc + tp];
    const uint32_t off = h.twist ? prog[h.p_pbyte + tp] : kAccNoByte;
    if (off != kAccNoByte) {
      const uint4* src = reinterpret_cast<const uint4*>(proofs + ((size_t)b * h.pstride + off) / 4);
      const uint4 lo = src[0], hi = src[1];
      const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w & 0x7fffffffu};
      const F29<F> X = f29_mul_c<F>(f29_unpack<F>(w), f29_const<F>(F29Consts<F>::R522));  // < 2p
      const F29<F> A = f29_norm<F>(f29_add<F>(f29_mul_c<F>(f29_sqr_c<F>(X), X), f29_const<F>(Glv<Cv>::B29)));
      x = f29_canon<F>(f29_reduce3<F>(f29_mul_c<F>(A, X)));
      y = f29_canon<F>(f29_reduce3<F>(f29_sqr_c<F>(A)));
      inf = false;
      return;
    }
    pp = h.twist ? inst + 16ull * ((size_t)h.ninst * b + idx) : points + 16ull * ((size_t)h.npts * b + idx);
  } else {
    pp = vk + 16ull * (g - nprf);
  }
  const Aff<F> P = load_aff<F>(pp);
  inf = aff_is_inf<F>(P);
  x = f29_canon<F>(f29_from_r256<F>(P.x.l));
  y = f29_canon<F>(f29_from_r256<F>(P.y.l));
}

// Quad g < B Tp: proof b's proof-point term of rank tp (g = b Tp + tp) -> pw;
// quad B Tp + v (v < nvk): VK point v -> pwv, the per-VK tables shared by
// every proof of this and later batches (nvk = 0 when they are current).
template <class Cv>
__global__ void __launch_bounds__(256) k_acc_powers(AccumHdr h, const uint32_t* __restrict__ prog,
                                                    const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ proofs,
                                                    const uint32_t* __restrict__ inst,
                                                    const uint32_t* __restrict__ vk, uint32_t nvk,
                                                    uint4* __restrict__ pw, uint4* __restrict__ pwv) {
  using F = typename Cv::Base;
  using K = F29Consts<F>;
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = gl >> 2, q = gl & 3u;
  const uint32_t nprf = h.B * h.Tp;
  if (g >= nprf + nvk) return;  // whole quads
  uint4* out = g < nprf ? pw + (size_t)g * kPowPos * kPowPoint : pwv + (size_t)(g - nprf) * kPowPos * kPowPoint;
  F29<F> px, py;
  bool inf;
  acc_chain_start<Cv>(h, prog, points, proofs, inst, vk, g, px, py, inf);
  const PowSites ps(q);
  const F29<F> one = f29_const<F>(K::ONE);
  if (inf) {  // the identity (ZZ = 0) at every power
    const F29<F> zero = f29_zero<F>();
    for (uint32_t j = 0; j < kPowPos; j++) pow_store<F>(out + j * kPowPoint, ps, Jac29<F>{one, one, one}, zero, one);
    return;
  }
  const F29<F> beta = f29_const<F>(Glv<Cv>::BETA29);
  Jac29<F> cur{px, py, one};
  pow_store<F>(out, ps, cur, one, q == 0u ? f29_mul_c<F>(beta, px) : one);
  for (uint32_t j = 1; j < kPowPos; j++) {
    F29<F> zz, ext;
    cur = jac29_dbl_q_ext<F>(cur, beta, zz, ext);
    pow_store<F>(out + j * kPowPoint, ps, cur, zz, ext);
  }
}

// k_acc_powers_s: the same tables, one WAVE per (proof, term) chain with
// row-sliced field elements (slice29.hpp: an element is one VGPR across a
// 16-lane row, a product ~0.27 us instead of ~0.42 one-lane).  For few
// chains (config 3's 16 proofs, config 5's 32-proof rank slices: one wave per
// SIMD or less), where jac29_dbl_q_ext's quads leave most lanes idle.  The
// four rows take the quad's four lanes' roles, level by level:
//   L1  row 1 B = Y Y, row 2 Y Z, row 3 E = (3X) X            (row 0 idles)
//   L2  row 0 4C = (4B) B, row 1 D = (4X) B, row 2 F = E E, row 3 ZZ3 = Z3 Z3
//   L3  row 0 beta X3, rows 1, 2 E (D - X3), row 3 ZZZ3 = ZZ3 Z3
// with the results other rows need gathered by ds_bpermute.  The stored
// points equal k_acc_powers' as group elements; their X and Y are left
// unreduced (below 9.4p, limbs <= 2^29: see the loop).  Each row's lanes 0-8
// store one limb each: coordinate c of position j is 9 consecutive words.
// Blocks of four waves (four chains: one wave per SIMD of a CU), each with an
// LDS fence that keeps a second ladder block and every side-stream block
// (transcript, k_acc_scalars) off its CU.  Waves only talk inside themselves
// (DPP, ds_bpermute, ballot), so a wave past the last chain just exits.
template <class Cv>
__global__ void __launch_bounds__(256) k_acc_powers_s(AccumHdr h, const uint32_t* __restrict__ prog,
                                                    const uint32_t* __restrict__ points,
                                                    const uint32_t* __restrict__ proofs,
                                                    const uint32_t* __restrict__ inst,
                                                    const uint32_t* __restrict__ vk, uint32_t nvk,
                                                    uint4* __restrict__ pw, uint4* __restrict__ pwv) {
  using F = typename Cv::Base;
  const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6);
  const uint32_t nprf = h.B * h.Tp;
  if (g >= nprf + nvk) return;
  uint4* out = g < nprf ? pw + (size_t)g * kPowPos * kPowPoint : pwv + (size_t)(g - nprf) * kPowPos * kPowPoint;
  const uint32_t row = s_rowid(), l = s_lane();
  const bool limb = l < 9u;
  uint32_t* o32 = reinterpret_cast<uint32_t*>(out) + l;  // + position * kPowPoint * 4 + coordinate * 12
  constexpr uint32_t kPosW = kPowPoint * 4, kCoordW = kPowWords * 4;
  // store sites of the two stores per position (kPowCoord - 1 = the junk slot)
  const uint32_t site1 = (row == 0 ? 0u : row == 1 ? 1u : row == 3 ? 2u : 5u) * kCoordW;
  const uint32_t site2 = (row == 0 ? 4u : row == 3 ? 3u : 5u) * kCoordW;
  const SConst<F> k = SConst<F>::make();
  F29<F> px, py;
  bool inf;
  acc_chain_start<Cv>(h, prog, points, proofs, inst, vk, g, px, py, inf);
  if (inf) {  // the identity (ZZ = 0) at every power, as k_acc_powers stores it
    const uint32_t v1 = row == 3 ? 0u : k.one;
    for (uint32_t j = 0; j < kPowPos; j++)
      if (limb) {
        o32[j * kPosW + site1] = v1;
        o32[j * kPosW + site2] = k.one;
      }
    return;
  }
  const uint32_t m0 = row == 0 ? ~0u : 0u, m1 = row == 1 ? ~0u : 0u, m2 = row == 2 ? ~0u : 0u,
                 m3 = row == 3 ? ~0u : 0u;
  const S29<F> beta{s_limbs(Glv<Cv>::BETA29)};
  S29<F> X = s29_from<F>(px);
  S29<F> Y = s29_from<F>(py);
  S29<F> Z{k.one};
  {  // position 0: (x, y, 1, 1, beta x)
    const S29<F> bx = s29_norm_exact<F>(s29_mul<F>(beta, X, k));
    if (limb) {
      o32[site1] = bsel(m0, X.v, bsel(m1, Y.v, k.one));
      o32[site2] = bsel(m0, bx.v, k.one);
    }
  }
  for (uint32_t j = 1; j < kPowPos; j++) {
    // L1: (X, X) / (Y, Y) / (Y, Z) / (3X, X)
    const uint32_t a1 = bsel(m1 | m2, Y.v, bsel(m3, X.v * 3u, X.v));
    const uint32_t b1 = bsel(m2, Z.v, bsel(m1, Y.v, X.v));
    const uint32_t r1 = s29_mul<F>(S29<F>{a1}, S29<F>{b1}, k).v;
    const uint32_t B = s_row<1>(r1), YZ = s_row<2>(r1), E = s_row<3>(r1);
    const uint32_t Z3 = YZ + YZ;  // < 4p, limbs <= 2^30
    // L2: (4B, B) / (4X, B) / (E, E) / (Z3, Z3)
    const uint32_t a2 = bsel(m0, B << 2, bsel(m1, X.v << 2, bsel(m2, E, Z3)));
    const uint32_t b2 = bsel(m0 | m1, B, bsel(m2, E, Z3));
    const uint32_t r2 = s29_mul<F>(S29<F>{a2}, S29<F>{b2}, k).v;
    const uint32_t C4 = s_row<0>(r2), D = s_row<1>(r2), FF = s_row<2>(r2);
    // X3, Y3 stay unreduced (round 5): lazily normalised (limbs <= 2^29), with
    // X < 9.1p, Y < 9.4p at every position (bounds: products of inputs below
    // 10p stay below 2.94p (E), 1.69p (B), 1.48p (D), 1.09p (FF, C4), 1.31p
    // (E w); X3 = FF + 8p - 2D in (5.0p, 9.1p), w = D + 12p - X3 in (2.9p,
    // 13.5p), Y3 = E w + 8p - 2 C4 in (5.8p, 9.4p)); k_acc_termadd reduces
    // what it stores or negates.  Two f29_reduce3 / exact normalisations less
    // per doubling on the chain.
    const S29<F> X3 = s29_norm<F>(S29<F>{FF + k.k8x3 - (D + D)});
    const uint32_t w = D + k.k12 - X3.v;  // limbs < 2^31
    // L3: (beta, X3) / (E, w) / (E, w) / (ZZ3, Z3)
    const uint32_t a3 = bsel(m0, beta.v, bsel(m3, r2, E));
    const uint32_t b3 = bsel(m0, X3.v, bsel(m3, Z3, w));
    const uint32_t r3 = s29_mul<F>(S29<F>{a3}, S29<F>{b3}, k).v;
    const S29<F> Y3r = s29_norm<F>(S29<F>{r3 + k.k8x3 - (C4 + C4)});  // rows 1, 2
    const uint32_t Y3 = s_row<1>(Y3r.v);
    // stores: X3 (row 0), Y3 (row 1), ZZ3 (row 3) | beta X3 (row 0), ZZZ3 (row 3)
    const uint32_t v1 = bsel(m0, X3.v, bsel(m1, Y3, r2));
    if (limb) {
      o32[j * kPosW + site1] = v1;
      o32[j * kPosW + site2] = r3;
    }
    X = X3;
    Y = S29<F>{Y3};
    Z = S29<F>{Z3};
  }
}

// non-adjacent form of k < 2^127 (4 words): with h = 3 k, digit i is
// h_{i+1} - k_{i+1}; nz = its nonzero positions, ng = the negative ones
__device__ __forceinline__ void naf128(const uint32_t* k, uint32_t* nz, uint32_t* ng) {
  uint32_t hw[5];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    c += (uint64_t)k[i] * 3u;
    hw[i] = (uint32_t)c;
    c >>= 32;
  }
  hw[4] = (uint32_t)c;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t hp = (hw[i] >> 1) | (hw[i + 1] << 31);
    const uint32_t kp = (k[i] >> 1) | (i < 3 ? k[i + 1] << 31 : 0u);
    nz[i] = hp ^ kp;
    ng[i] = kp & ~hp;
  }
}

// k_acc_termadd: S lanes per (proof, term) (S a power of two <= 64); the
// nonzero digits of both halves, in order (k1's, then k2's), are dealt out
// round-robin, so lane j adds ranks j, j + S, ... (at most ceil(cnt / S)
// additions, cnt ~ 85) with full XYZZ additions; the next point's loads are
// issued before each addition.  Then log2(S) butterfly steps; lane 0 stores.
// QUAD (round 5, few terms): S quads per term instead of S lanes (S <= 16, a
// term within one wave), each addition quad-cooperative (coop29.hpp, ~half
// the latency of a one-lane addition): for B = 16 a term takes 6 + 4 quad
// additions instead of 3 + 5 lane additions at ~2x the latency each.
template <class Cv, bool QUAD = false>
__global__ void __launch_bounds__(256) k_acc_termadd(AccumHdr h, const uint32_t* __restrict__ prog,
                                                     const uint32_t* __restrict__ coef,
                                                     const uint4* __restrict__ pw, const uint4* __restrict__ pwv,
                                                     const uint4* __restrict__ corr, uint32_t lgS,
                                                     Xyzz<typename Cv::Base>* __restrict__ part) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  const uint32_t gl = (blockIdx.x * blockDim.x + threadIdx.x) >> (QUAD ? 2 : 0);  // lane or quad
  const uint32_t S = 1u << lgS, g = gl >> lgS, j = gl & (S - 1);
  if (g >= h.B * h.T) return;  // whole groups only
  uint32_t k1[6], k2[6];
  bool n1, n2;
  glv_split<Cv, true>(ldfe<Fs>(coef, g), k1, k2, n1, n2);
  uint32_t nz[8], ng[8];
  naf128(k1, nz, ng);
  naf128(k2, nz + 4, ng + 4);
  const uint32_t f1 = n1 ? ~0u : 0u, f2 = n2 ? ~0u : 0u;
  uint32_t skip = j;
#pragma unroll
  for (int w = 0; w < 8; w++) {
    ng[w] ^= w < 4 ? f1 : f2;  // sign of the half
    uint32_t m = nz[w], sel = 0;
    while (m) {
      const uint32_t lb = m & (0u - m);
      sel |= skip == 0 ? lb : 0u;
      skip = skip == 0 ? S - 1 : skip - 1;
      m ^= lb;
    }
    nz[w] = sel;
  }
  const uint32_t b = g / h.T, t = g - b * h.T;
  const uint32_t src = prog[h.p_termsrc + t];
  const uint4* base = (src >> 28) != 0 ? pwv + (size_t)(src & 0x0FFFFFFFu) * kPowPos * kPowPoint
                                       : pw + ((size_t)b * h.Tp + prog[h.p_rank + t]) * kPowPos * kPowPoint;
  // pops this lane's lowest remaining digit and issues its loads
  auto next = [&](Xyzz29<F>& Q, uint32_t& negm) -> bool {
    uint32_t w = 8, m = 0, s = 0;
#pragma unroll
    for (int i = 7; i >= 0; i--)
      if (nz[i]) {
        w = (uint32_t)i;
        m = nz[i];
        s = ng[i];
      }
    if (w == 8) return false;
    const uint32_t bit = __builtin_ctz(m);
#pragma unroll
    for (int i = 0; i < 8; i++)
      if ((uint32_t)i == w) nz[i] = m & (m - 1);
    negm = 0u - ((s >> bit) & 1u);
    const uint4* o = base + (((w & 3u) << 5) | bit) * kPowPoint;
    Q.X = pow_ld<F>(o + (w < 4 ? 0 : 4 * kPowWords));  // phi: (beta X, Y, ZZ, ZZZ)
    Q.Y = pow_ld<F>(o + kPowWords);
    Q.ZZ = pow_ld<F>(o + 2 * kPowWords);
    Q.ZZZ = pow_ld<F>(o + 3 * kPowWords);
    return true;
  };
  // table points: X, Y below 3p (k_acc_powers) or 9.4p (k_acc_powers_s,
  // unreduced), limbs <= 2^29; they only enter products, the negation
  // (12p - Y) and, reduced, the store
  Xyzz29<F> acc = xyzz29_inf<F>(), Q;
  uint32_t negm = 0;
  bool have = next(Q, negm);
  while (have) {
    const F29<F> yn = f29_reduce3<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), Q.Y, F29K12<F>::L)));  // < 3p
    Xyzz29<F> R = Q;
#pragma unroll
    for (int i = 0; i < 9; i++) R.Y.l[i] = bsel(negm, yn.l[i], Q.Y.l[i]);
    have = next(Q, negm);
    acc = QUAD ? xyzz29_add_q<F>(acc, R) : xyzz29_add<F>(acc, R);
  }
  for (uint32_t m = 1; m < S; m <<= 1) {
    const Xyzz29<F> o = xyzz29_shfl_xor<F>(acc, (int)(QUAD ? 4 * m : m));
    acc = QUAD ? xyzz29_add_q<F>(acc, o) : xyzz29_add<F>(acc, o);
  }
  if (j == 0 && (!QUAD || (threadIdx.x & 3u) == 0)) {  // a sum of one table point is that point, possibly unreduced
    if (h.twist && (src >> 28) == 0) {  // psi: E_A -> the curve (acc_chain_start)
      const uint4* c = corr + ((size_t)b * h.npts + (src & 0x0FFFFFFFu)) * kAccCorrWords;
      acc.ZZ = f29_mul_c<F>(acc.ZZ, pow_ld<F>(c));
      acc.ZZZ = f29_mul_c<F>(acc.ZZZ, pow_ld<F>(c + kPowWords));
    }
    acc.X = f29_reduce3<F>(f29_norm<F>(acc.X));
    acc.Y = f29_reduce3<F>(f29_norm<F>(acc.Y));
    store_xyzz29<F>(&part[g], acc);
  }
}

// k_acc_sum: 2^lgL lanes per (proof, output) (lgL <= 5): lane l sums terms
// lo + l, lo + l + 2^lgL, ... (pstep = 2 after k_acc_termmul's two-term
// lanes: only the pairs' first rows hold sums, the second the identity); a butterfly of cross-lane shuffles folds the
// partials and lane 0 converts to the unique affine point (binary-GCD
// inversion).  With >= 4 lanes the lanes work in quads (quad-cooperative
// additions).  Outputs in MultiopenVar order w, zw, f, e.
template <class Cv>
__global__ void __launch_bounds__(64) k_acc_sum(AccumHdr h, const Xyzz<typename Cv::Base>* __restrict__ part,
                                                uint32_t lgL, uint32_t* __restrict__ out, uint32_t pstep) {
  using F = typename Cv::Base;
  const uint32_t gl = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t NL = 1u << lgL, g = gl >> lgL, lane = gl & (NL - 1);
  if (g >= h.B * 4) return;  // whole groups only (a group never straddles a wave)
#ifdef PM_ACC_PROFILE
  const uint64_t pc0 = wall_clock64();
#endif
  const uint32_t b = g >> 2, o = g & 3;
  const uint32_t lo = o == 0 ? h.nslots : o == 1 ? h.nslots + h.nsets : o == 2 ? 0 : h.T - 1;
  const uint32_t hi = o == 0 ? h.nslots + h.nsets : o == 1 ? h.nslots + 2 * h.nsets : o == 2 ? h.nslots : h.T;
  Xyzz29<F> acc = xyzz29_inf<F>();
  if (NL >= 4) {
    // quads of lanes act as one lane (coop29.hpp: each addition at ~half the
    // latency); all 4 lanes of a quad see the same terms
    const uint32_t v = lane >> 2, NV = NL >> 2;
    for (uint32_t t = lo + v * pstep; t < hi; t += NV * pstep)
      acc = xyzz29_add_q<F>(acc, load_xyzz29<F>(&part[(size_t)b * h.T + t]));
    for (uint32_t m = 4; m < NL; m <<= 1) acc = xyzz29_add_q<F>(acc, xyzz29_shfl_xor<F>(acc, (int)m));
  } else {
    for (uint32_t t = lo + lane * pstep; t < hi; t += NL * pstep)
      acc = xyzz29_add<F>(acc, load_xyzz29<F>(&part[(size_t)b * h.T + t]));
    for (uint32_t m = 1; m < NL; m <<= 1) acc = xyzz29_add<F>(acc, xyzz29_shfl_xor<F>(acc, (int)m));
  }
  // affine conversion: by the group's first quad (quad-cooperative inversion,
  // each lane then stores one 16-B quarter), or by lane 0 alone
  const bool quad = NL >= 4;
  if (lane >= (quad ? 4u : 1u)) return;
#ifdef PM_ACC_PROFILE
  const uint64_t pc1 = wall_clock64();
  uint64_t pc2 = pc1;
#endif
  uint32_t wx[8] = {0, 0, 0, 0, 0, 0, 0, 0}, wy[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (!xyzz29_is_inf<F>(acc)) {  // uniform over the quad (equal acc)
    const F29<F> zz = f29_mul_c<F>(acc.ZZ, acc.ZZZ);
    const F29<F> inv = quad ? f29_inv_q<F>(zz) : f29_inv<F>(zz);  // 1 / (ZZ ZZZ)
#ifdef PM_ACC_PROFILE
    pc2 = wall_clock64();
#endif
    f29_to_r256<F>(f29_canon<F>(f29_mul_c<F>(acc.X, f29_mul_c<F>(inv, acc.ZZZ))), wx);
    f29_to_r256<F>(f29_canon<F>(f29_mul_c<F>(acc.Y, f29_mul_c<F>(inv, acc.ZZ))), wy);
  }
#ifdef PM_ACC_PROFILE  // A/B builds only: fold / inversion / affine times of group 0..3 (10 ns ticks)
  const uint64_t pc3 = wall_clock64();
  if (g < 4 && lane == 0)
    printf("acc_sum g %u NL %u: fold %llu inv %llu affine %llu\n", g, NL, (unsigned long long)(pc1 - pc0),
           (unsigned long long)(pc2 - pc1), (unsigned long long)(pc3 - pc2));
#endif
  uint4* q = reinterpret_cast<uint4*>(out + 16ull * g);
  if (!quad || lane == 0) q[0] = make_uint4(wx[0], wx[1], wx[2], wx[3]);
  if (!quad || lane == 1) q[1] = make_uint4(wx[4], wx[5], wx[6], wx[7]);
  if (!quad || lane == 2) q[2] = make_uint4(wy[0], wy[1], wy[2], wy[3]);
  if (!quad || lane == 3) q[3] = make_uint4(wy[4], wy[5], wy[6], wy[7]);
}

}  // namespace pm

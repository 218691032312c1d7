// proof_kernels.hpp -- batched decoding of halo2 proof bytes on the device.
//
// The reference verifier reads every commitment and evaluation of an inner
// proof from halo2's byte transcript (`Blake2bRead`): `t.read_point()` at
// /root/reference/src/verifier.rs:370, src/lookup.rs:64-65,96,
// src/permutation.rs:67, src/vanishing.rs:67,94, src/multiopen.rs:210, and
// `t.read_scalar()` at src/verifier.rs:443,456,469, src/vanishing.rs:122,
// src/permutation.rs:100-107,163, src/lookup.rs:124-128.  Any failure there
// aborts the verifier (`?`).  This kernel does those reads for B proofs at
// once [3P: halo2 Blake2bRead, pasta_curves / pairing_bn256 GroupEncoding and
// PrimeField; restated in oracle/proof_bytes.py]:
//   point : 32 bytes, canonical little-endian x with the parity of the
//           canonical y in bit 255; x >= p fails; x = 0 with the bit clear is
//           the identity, which fails too (the reader's common_point rejects
//           it); otherwise y = sqrt(x^3 + b) (a non-residue fails) negated
//           when its parity differs from the bit
//   scalar: 32 bytes, canonical little-endian, >= r fails
// and writes the accumulator's inputs (affine Montgomery points and
// Montgomery scalars, the pm_accum_batch layout) plus the canonical
// coordinates the transcript replay hashes (k_tr_canon's layout), so the
// replay starts straight from them.  Failed reads set PM_PROOF_BAD_POINT /
// PM_PROOF_BAD_SCALAR in the proof's status word; the slot then holds the
// identity / zero.
//
// Square roots, one lane per point, radix-2^29 Montgomery arithmetic
// (fp29.hpp):
//   * BN254 Fq (p = 3 mod 4): y = a^((p+1)/4);
//   * Pasta (p - 1 = 2^32 t): x = a^((t+1)/2), b = a^t = g^e in the 2^32-th
//     roots of unity (g = 5^t); e is found in four 8-bit windows from the top
//     (b^(2^24) = G3^(e mod 2^8) with G3 = g^(2^24), each window a lookup in
//     a sorted table of the 256 powers of G3 after removing the known low
//     digits with tables of g^(-2^j k)), e odd means a non-residue, else
//     y = x g^(-e/2) (Sarkar's table form of Tonelli-Shanks, ePrint 2020/1407).
// Every root is verified (y^2 == a) before it is accepted.  The exponent
// schedules (4-bit sliding window over odd powers kept in LDS) and the tables
// are built on the host once per context and curve.
#pragma once
#include <algorithm>
#include <cstring>
#include <type_traits>
#include <vector>

#include "curve.hpp"
#include "fp29.hpp"
#include "msm_kernels.hpp"
#include "slice29.hpp"
#include "runtime.hpp"
#include "accum_kernels.hpp"  // acc_chain_start's correction table layout

namespace pm {

template <class Cv>
constexpr int curve_slot() {  // pm_curve order
  return std::is_same<Cv, PallasCurve>::value ? 0 : std::is_same<Cv, VestaCurve>::value ? 1 : 2;
}

static constexpr uint32_t kProofBadPoint = 8;    // PM_PROOF_BAD_POINT
static constexpr uint32_t kProofBadScalar = 16;  // PM_PROOF_BAD_SCALAR
constexpr int kSqrtSched = 160;
constexpr int kSqrtWin = 8;  // odd powers a, a^3, .., a^15

struct SqrtTab {
  uint32_t r2[9];   // 2^522 mod p: canonical -> R = 2^261 Montgomery
  uint32_t b[9];    // curve b, R261
  uint32_t ts;      // 1: Pasta windows (2-adicity 32); 0: p = 3 mod 4
  uint32_t nsched;  // schedule of the exponent: (squarings << 8) | odd-power index (0xff: none)
  uint32_t sched[kSqrtSched];
  uint32_t key_lo[256], key_hi[256], kidx[256];  // G3^k sorted by (limb0 | limb1 << 29) of its canonical R261 form
  uint32_t tab[6][256][9];                       // g^(-k), g^(-2^7 k), g^(-2^8 k), g^(-2^15 k), g^(-2^16 k), g^(-2^23 k)
};
enum { kT0 = 0, kT7, kT8, kT15, kT16, kT23 };

// ---------------------------------------------------------------- host side
namespace sqrt_host {
template <class F>
Fe<F> pow_words(const Fe<F>& a, const uint32_t e[8]) {
  Fe<F> r = fe_one<F>();
  for (int i = 255; i >= 0; i--) {
    r = fe_sqr<F>(r);
    if ((e[i >> 5] >> (i & 31)) & 1u) r = fe_mul<F>(r, a);
  }
  return r;
}
template <class F>
Fe<F> small(uint32_t v) {
  Fe<F> r = fe_zero<F>();
  r.l[0] = v;
  return fe_to_mont<F>(r);
}
// R256 Montgomery (canonical) -> R261 Montgomery as 9 canonical 29-bit limbs
template <class F>
void to29(const Fe<F>& a, uint32_t out[9]) {
  const Fe<F> v = fe_mul<F>(a, small<F>(32));  // a 2^5
  for (int i = 0; i < 9; i++) {
    const int bit = 29 * i, k = bit >> 5, s = bit & 31;
    uint64_t w = v.l[k] >> s;
    if (k + 1 < 8) w |= (uint64_t)v.l[k + 1] << (32 - s);
    out[i] = (uint32_t)w & ((1u << 29) - 1u);
  }
}
inline void shr_words(uint32_t e[8], int n) {  // e >>= n (n < 32)
  for (int i = 0; i < 8; i++) e[i] = (e[i] >> n) | (i + 1 < 8 && n ? e[i + 1] << (32 - n) : 0u);
}
// 4-bit sliding window over the odd powers: first entry loads a power
inline int make_schedule(const uint32_t e[8], uint32_t* sched) {
  auto bit = [&](int i) { return (e[i >> 5] >> (i & 31)) & 1u; };
  int i = 255;
  while (i >= 0 && !bit(i)) i--;
  int n = 0, pend = 0;
  bool first = true;
  while (i >= 0) {
    if (!bit(i)) {
      pend++;
      i--;
      continue;
    }
    int j = i - 3 < 0 ? 0 : i - 3;
    while (!bit(j)) j++;
    uint32_t d = 0;
    for (int k = i; k >= j; k--) d = (d << 1) | bit(k);
    const uint32_t sq = first ? 0u : (uint32_t)(pend + i - j + 1);
    sched[n++] = (sq << 8) | ((d - 1) / 2);
    first = false;
    pend = 0;
    i = j - 1;
  }
  if (pend) sched[n++] = ((uint32_t)pend << 8) | 0xffu;
  return n;
}
}  // namespace sqrt_host

template <class Cv>
int sqrt_tab_build(SqrtTab& T) {
  using F = typename Cv::Base;
  using namespace sqrt_host;
  std::memset(&T, 0, sizeof(T));
  {
    // r2 = 2^522 mod p is the R261 form of 2^261
    const Fe<F> two = small<F>(2);
    Fe<F> t = fe_one<F>();
    for (int i = 0; i < 261; i++) t = fe_mul<F>(t, two);
    to29<F>(t, T.r2);
    to29<F>(small<F>((uint32_t)Cv::B), T.b);
  }
  uint32_t e[8];
  for (int i = 0; i < 8; i++) e[i] = F::MOD[i];
  if ((F::MOD[0] & 3u) == 3u) {  // (p + 1) / 4
    uint32_t c = 1;
    for (int i = 0; i < 8; i++) {
      const uint64_t s = (uint64_t)e[i] + c;
      e[i] = (uint32_t)s;
      c = (uint32_t)(s >> 32);
    }
    shr_words(e, 2);
    T.ts = 0;
  } else {
    // p - 1 = 2^32 t (Pasta: MOD[0] == 1); E = (t - 1) / 2
    if (F::MOD[0] != 1u) return set_error(PM_ERR_UNSUPPORTED, "sqrt: unsupported 2-adicity");
    uint32_t t[8];
    for (int i = 0; i < 7; i++) t[i] = e[i + 1];
    t[7] = 0;
    if (!(t[0] & 1u)) return set_error(PM_ERR_UNSUPPORTED, "sqrt: 2-adicity above 32");
    for (int i = 0; i < 8; i++) e[i] = t[i];
    e[0] &= ~1u;  // t - 1
    shr_words(e, 1);
    T.ts = 1;
    // g = 5^t, a primitive 2^32-th root iff 5 is a non-residue (checked)
    const Fe<F> g = pow_words<F>(small<F>(5), t);
    Fe<F> h = g;
    for (int i = 0; i < 31; i++) h = fe_sqr<F>(h);
    if (!fe_eq<F>(h, fe_neg<F>(fe_one<F>()))) return set_error(PM_ERR_UNSUPPORTED, "sqrt: 5 is a residue");
    Fe<F> G3 = g;
    for (int i = 0; i < 24; i++) G3 = fe_sqr<F>(G3);
    struct K {
      uint64_t key;
      uint32_t k;
    };
    std::vector<K> keys(256);
    Fe<F> v = fe_one<F>();
    for (uint32_t k = 0; k < 256; k++) {
      uint32_t l[9];
      to29<F>(v, l);
      keys[k] = K{(uint64_t)l[0] | ((uint64_t)l[1] << 29), k};
      v = fe_mul<F>(v, G3);
    }
    std::sort(keys.begin(), keys.end(), [](const K& a, const K& b) { return a.key < b.key; });
    for (int k = 0; k < 256; k++) {
      if (k && keys[k].key == keys[k - 1].key) return set_error(PM_ERR_UNSUPPORTED, "sqrt: table key collision");
      T.key_lo[k] = (uint32_t)keys[k].key;
      T.key_hi[k] = (uint32_t)(keys[k].key >> 32);
      T.kidx[k] = keys[k].k;
    }
    const Fe<F> ginv = fe_inv<F>(g);
    const int shifts[6] = {0, 7, 8, 15, 16, 23};
    for (int j = 0; j < 6; j++) {
      Fe<F> base = ginv;
      for (int s = 0; s < shifts[j]; s++) base = fe_sqr<F>(base);
      Fe<F> acc = fe_one<F>();
      for (int k = 0; k < 256; k++) {
        to29<F>(acc, T.tab[j][k]);
        acc = fe_mul<F>(acc, base);
      }
    }
  }
  T.nsched = (uint32_t)make_schedule(e, T.sched);
  if (T.nsched > (uint32_t)kSqrtSched) return set_error(PM_ERR_UNSUPPORTED, "sqrt: schedule too long");
  return PM_OK;
}

// -------------------------------------------------------------- device side
template <class F>
__device__ __forceinline__ F29<F> f29_ld(const uint32_t* p) {
  F29<F> r;
#pragma unroll
  for (int i = 0; i < 9; i++) r.l[i] = p[i];
  return r;
}
template <class F>
__device__ __forceinline__ bool f29_eq_canon(const F29<F>& a, const F29<F>& b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) d |= a.l[i] ^ b.l[i];
  return d == 0;
}

// a^E by the table's schedule; `odd` = this lane's LDS slots [kSqrtWin][9]
// (stride `ls` words between consecutive slots of one lane)
template <class F>
__device__ F29<F> sqrt_pow(const SqrtTab& T, const F29<F>& a, uint32_t* odd, uint32_t ls) {
  const F29<F> a2 = f29_sqr_c<F>(a);
  F29<F> p = a;
#pragma unroll
  for (int i = 0; i < kSqrtWin; i++) {
#pragma unroll
    for (int l = 0; l < 9; l++) odd[(i * 9 + l) * ls] = p.l[l];
    if (i + 1 < kSqrtWin) p = f29_mul_c<F>(p, a2);
  }
  auto ld_odd = [&](uint32_t idx) {
    F29<F> r;
#pragma unroll
    for (int l = 0; l < 9; l++) r.l[l] = odd[(idx * 9 + l) * ls];
    return r;
  };
  F29<F> acc = ld_odd(T.sched[0] & 0xffu);
  for (uint32_t k = 1; k < T.nsched; k++) {
    const uint32_t s = T.sched[k];
    for (uint32_t q = s >> 8; q; q--) acc = f29_sqr_c<F>(acc);
    if ((s & 0xffu) != 0xffu) acc = f29_mul_c<F>(acc, ld_odd(s & 0xffu));
  }
  return acc;
}

// sqrt_pow with row-sliced elements (slice29.hpp: one element per 16-lane
// row, a product ~0.27 us instead of ~0.42): the odd powers stay in eight
// VGPRs, the schedule is the same for every row (one exponent per curve).
template <class F>
__device__ S29<F> sqrt_pow_s(const SqrtTab& T, S29<F> a, const SConst<F>& k) {
  static_assert(kSqrtWin == 8, "eight odd powers");
  // eight named registers, not an array: the compiler promoted the array to
  // LDS and each pick then waited on an LDS read
  const S29<F> a2 = s29_mul<F>(a, a, k);
  const uint32_t o0 = a.v;
  const uint32_t o1 = s29_mul<F>(S29<F>{o0}, a2, k).v;
  const uint32_t o2 = s29_mul<F>(S29<F>{o1}, a2, k).v;
  const uint32_t o3 = s29_mul<F>(S29<F>{o2}, a2, k).v;
  const uint32_t o4 = s29_mul<F>(S29<F>{o3}, a2, k).v;
  const uint32_t o5 = s29_mul<F>(S29<F>{o4}, a2, k).v;
  const uint32_t o6 = s29_mul<F>(S29<F>{o5}, a2, k).v;
  const uint32_t o7 = s29_mul<F>(S29<F>{o6}, a2, k).v;
  // idx is wave-uniform; the empty asm keeps each select a register select
  // (the compiler otherwise turned the chain into a table of pointers in LDS
  // and an indirect scratch load per pick)
  auto pick = [=](uint32_t idx) {
    uint32_t v = o0;
#define PM_PICK(I, O)                 \
  v = idx == (I) ? (O) : v;           \
  asm volatile("" : "+v"(v));
    PM_PICK(1u, o1)
    PM_PICK(2u, o2)
    PM_PICK(3u, o3)
    PM_PICK(4u, o4)
    PM_PICK(5u, o5)
    PM_PICK(6u, o6)
    PM_PICK(7u, o7)
#undef PM_PICK
    return S29<F>{v};
  };
  // the schedule word is loaded one step ahead: its scalar load (and the wait
  // on it) no longer heads every step
  const uint32_t ns = T.nsched;
  S29<F> acc = pick(T.sched[0] & 0xffu);
  uint32_t s = ns > 1 ? T.sched[1] : 0u;
  for (uint32_t j = 1; j < ns; j++) {
    const uint32_t sn = T.sched[j + 1 < ns ? j + 1 : j];
    for (uint32_t q = s >> 8; q; q--) acc = s29_mul<F>(acc, acc, k);
    if ((s & 0xffu) != 0xffu) acc = s29_mul<F>(acc, pick(s & 0xffu), k);
    s = sn;
  }
  return acc;
}

// 8-bit discrete log of v (canonical R261, a power of G3) in the sorted LDS keys
__device__ __forceinline__ uint32_t sqrt_dlog(const uint32_t* klo, const uint32_t* khi, const uint32_t* kidx,
                                              const uint32_t l0, const uint32_t l1, bool& ok) {
  const uint64_t key = (uint64_t)l0 | ((uint64_t)l1 << 29);
  uint32_t lo = 0;
#pragma unroll
  for (uint32_t step = 128; step; step >>= 1) {
    const uint32_t m = lo + step - 1;
    const uint64_t km = (uint64_t)klo[m] | ((uint64_t)khi[m] << 32);
    if (km < key) lo += step;
  }
  lo = lo > 255 ? 255 : lo;
  ok = ok && (((uint64_t)klo[lo] | ((uint64_t)khi[lo] << 32)) == key);
  return kidx[lo];
}

// y with y^2 = a (a Norm < 3p, R261); false when a is a non-residue
// SLICED: the rows of the wave each decode one point (all 16 lanes of a row
// hold the same a), and the exponentiation runs row-sliced (p = 3 mod 4 only:
// the caller checks T.ts == 0)
template <class F, bool SLICED = false>
__device__ bool f29_sqrt(const SqrtTab& T, const F29<F>& a_in, F29<F>& y, uint32_t* odd, uint32_t ls,
                         const uint32_t* klo, const uint32_t* khi, const uint32_t* kidx) {
  const F29<F> a = f29_canon<F>(f29_reduce3<F>(a_in));
  F29<F> w;
  if constexpr (SLICED) {  // every row runs the chain (a zero a gives y = 0 below too)
    const SConst<F> k = SConst<F>::make();
    w = s29_to<F>(s29_norm_exact<F>(sqrt_pow_s<F>(T, s29_from<F>(a), k)));
  }
  if (f29_is_zero_exact<F>(a)) {
    y = a;
    return true;
  }
  if constexpr (!SLICED) w = sqrt_pow<F>(T, a, odd, ls);
  bool ok = true;
  if (!T.ts) {
    y = w;
  } else {
    const F29<F> x = f29_mul_c<F>(w, a);   // a^((t+1)/2)
    const F29<F> b0 = f29_mul_c<F>(x, w);  // a^t
    F29<F> b1 = b0, b2, b3;
    for (int i = 0; i < 8; i++) b1 = f29_sqr_c<F>(b1);
    b2 = b1;
    for (int i = 0; i < 8; i++) b2 = f29_sqr_c<F>(b2);
    b3 = b2;
    for (int i = 0; i < 8; i++) b3 = f29_sqr_c<F>(b3);
    auto tab = [&](int j, uint32_t k) { return f29_ld<F>(T.tab[j][k]); };
    auto dlog = [&](const F29<F>& v) {
      const F29<F> c = f29_canon<F>(v);
      return sqrt_dlog(klo, khi, kidx, c.l[0], c.l[1], ok);
    };
    const uint32_t d0 = dlog(b3);
    if (d0 & 1u) return false;  // e odd: a non-residue
    const uint32_t d1 = dlog(f29_mul_c<F>(b2, tab(kT16, d0)));
    const uint32_t d2 = dlog(f29_mul_c<F>(f29_mul_c<F>(b1, tab(kT8, d0)), tab(kT16, d1)));
    const uint32_t d3 =
        dlog(f29_mul_c<F>(f29_mul_c<F>(f29_mul_c<F>(b0, tab(kT0, d0)), tab(kT8, d1)), tab(kT16, d2)));
    y = f29_mul_c<F>(f29_mul_c<F>(x, tab(kT0, d0 >> 1)), tab(kT7, d1));
    y = f29_mul_c<F>(f29_mul_c<F>(y, tab(kT15, d2)), tab(kT23, d3));
  }
  y = f29_canon<F>(y);
  return ok && f29_eq_canon<F>(f29_canon<F>(f29_sqr_c<F>(y)), a);
}

// 8 canonical words < MOD?
template <class F>
__device__ __forceinline__ bool words_lt_mod(const uint32_t w[8]) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) (void)subb(w[i], F::MOD[i], br);
  return br != 0;
}

struct ProofDecodeHdr {
  uint32_t B, npts, nsc, ninst;
  uint32_t npp;        // points read from the proof bytes
  uint32_t sc_off;     // byte offset of the first scalar
  uint32_t stride;     // bytes per proof (multiple of 4)
  uint32_t nblk_pts;   // blocks of the point part (the scalar part follows)
};

// Point blocks (the last nblk_pts): one lane (SLICED: one 16-lane row) per
// proof point (pt_map: byte offset, destination point index per point).
// The blocks before: one lane per scalar, then per instance commitment.
// 256 (round 5, was 64): with the twisted ladder the decode runs beside it
// and takes whole CUs (kDecodeFence), so a block fills one CU's four SIMDs
constexpr int kDecodeThreads = 256;

// SLICED (p = 3 mod 4 curves, few points): one point per 16-lane row, the
// square root's exponentiation row-sliced (sqrt_pow_s); every lane of a row
// runs the rest of the point's code redundantly and lane 0 stores.
constexpr size_t kDecodeStaticLds = 4ull * (kSqrtWin * 9 * kDecodeThreads + 3 * 256);
template <class Cv, bool SLICED = false>
__global__ void __launch_bounds__(kDecodeThreads) k_proof_decode(
    ProofDecodeHdr h, const SqrtTab* __restrict__ tabp, const uint32_t* __restrict__ pt_map,
    const uint32_t* __restrict__ proofs, const uint32_t* __restrict__ inst, uint32_t* __restrict__ points,
    uint32_t* __restrict__ scalars, uint32_t* __restrict__ cpts, uint32_t* __restrict__ cscs,
    uint32_t* __restrict__ status, uint4* __restrict__ corr) {
  using F = typename Cv::Base;
  using Fs = typename Cv::Scalar;
  __shared__ uint32_t s_odd[kSqrtWin * 9 * kDecodeThreads];  // (kDecodeStaticLds)
  __shared__ uint32_t s_klo[256], s_khi[256], s_kidx[256];
  const SqrtTab& T = *tabp;
  const uint32_t lane = threadIdx.x;
  // blocks [0, nblk_sc): scalars and instance commitments (quick, first, so
  // that fenced point blocks never wait behind them); then the points
  const uint32_t nblk_sc = gridDim.x - h.nblk_pts;
  if (blockIdx.x >= nblk_sc) {
    const uint32_t pb = blockIdx.x - nblk_sc;
#ifdef PM_DECODE_PROFILE  // A/B builds only: phase times of the first point block's row 0 (10 ns ticks)
    const uint64_t pd0 = wall_clock64();
    uint64_t pd1 = 0, pd2 = 0;
    const bool prof = pb == 0 && lane == 0;
#endif
    if (!SLICED && T.ts) {
      for (uint32_t i = lane; i < 256; i += kDecodeThreads) {
        s_klo[i] = T.key_lo[i];
        s_khi[i] = T.key_hi[i];
        s_kidx[i] = T.kidx[i];
      }
      __syncthreads();
    }
    const size_t e = SLICED ? (size_t)pb * (kDecodeThreads / 16) + (lane >> 4) : (size_t)pb * kDecodeThreads + lane;
    if (e >= (size_t)h.B * h.npp) return;  // whole rows when SLICED
    const bool writer = !SLICED || (lane & 15u) == 0u;
    const uint32_t b = (uint32_t)(e / h.npp), j = (uint32_t)(e % h.npp);
    const uint32_t off = pt_map[2 * j], dst = pt_map[2 * j + 1];
    const uint32_t* src = proofs + ((size_t)b * h.stride + off) / 4;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = src[i];

    const uint32_t ysign = w[7] >> 31;
    w[7] &= 0x7fffffffu;
    uint32_t any = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) any |= w[i];
    bool ok = words_lt_mod<F>(w) && (any != 0 || ysign != 0);
    uint32_t xo[8] = {0, 0, 0, 0, 0, 0, 0, 0}, yo[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t xc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, yc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // the twisted ladder's factors (A, y A) for this point (accum_kernels.hpp
    // acc_chain_start): A = x^3 + b as the ladder computes it, y signed
    F29<F> cA = f29_const<F>(F29Consts<F>::ONE), cYA = cA;
    if (ok) {
#ifdef PM_DECODE_PROFILE
      pd1 = wall_clock64() + (w[0] & 0u);
#endif
      const F29<F> X = f29_mul_c<F>(f29_unpack<F>(w), f29_ld<F>(T.r2));  // R261
      const F29<F> rhs = f29_norm<F>(f29_add<F>(f29_mul_c<F>(f29_sqr_c<F>(X), X), f29_ld<F>(T.b)));
      F29<F> Y;
      ok = f29_sqrt<F, SLICED>(T, rhs, Y, s_odd + lane, kDecodeThreads, s_klo, s_khi, s_kidx);
#ifdef PM_DECODE_PROFILE
      pd2 = wall_clock64() + (Y.l[0] & 0u);
#endif
      if (ok) {
        F29<F> one = f29_zero<F>();
        one.l[0] = 1;
        F29<F> y = f29_canon<F>(f29_mul_c<F>(Y, one));  // plain canonical y
        if ((y.l[0] & 1u) != ysign) {
          using K = F29Consts<F>;
          y = f29_canon<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), y, K::K2)));
          Y = f29_canon<F>(f29_norm<F>(f29_sub<F>(f29_zero<F>(), Y, K::K2)));
        }
        f29_to_r256<F>(X, xo);
        f29_to_r256<F>(Y, yo);
        cA = rhs;
        cYA = f29_mul_c<F>(Y, rhs);
#pragma unroll
        for (int i = 0; i < 8; i++) xc[i] = w[i];
        f29_pack<F>(y, yc);
      }
    }
#ifdef PM_DECODE_PROFILE
    if (prof)
      printf("decode: start->loaded %llu loaded->sqrt_done %llu sqrt_done->end %llu (start %llu)\n",
             (unsigned long long)(pd1 - pd0), (unsigned long long)(pd2 - pd1),
             (unsigned long long)(wall_clock64() + (yc[0] & 0u) - pd2), (unsigned long long)pd0);
#endif
    if (!writer) return;
    if (!ok) atomicOr(&status[b], kProofBadPoint);
    const size_t pi = (size_t)b * h.npts + dst;
    uint4* po = reinterpret_cast<uint4*>(points + 16 * pi);
    uint4* co = reinterpret_cast<uint4*>(cpts + 16 * pi);
    po[0] = make_uint4(xo[0], xo[1], xo[2], xo[3]);
    po[1] = make_uint4(xo[4], xo[5], xo[6], xo[7]);
    po[2] = make_uint4(yo[0], yo[1], yo[2], yo[3]);
    po[3] = make_uint4(yo[4], yo[5], yo[6], yo[7]);
    co[0] = make_uint4(xc[0], xc[1], xc[2], xc[3]);
    co[1] = make_uint4(xc[4], xc[5], xc[6], xc[7]);
    co[2] = make_uint4(yc[0], yc[1], yc[2], yc[3]);
    co[3] = make_uint4(yc[4], yc[5], yc[6], yc[7]);
    if (corr) {
      pow_st<F>(corr + pi * kAccCorrWords, cA);
      pow_st<F>(corr + pi * kAccCorrWords + kPowWords, cYA);
    }
    return;
  }
  const size_t e = (size_t)blockIdx.x * kDecodeThreads + lane;
  const size_t nsc_all = (size_t)h.B * h.nsc;
  if (e < nsc_all) {  // a scalar: canonical check, Montgomery form
    const uint32_t b = (uint32_t)(e / h.nsc), k = (uint32_t)(e % h.nsc);
    const uint32_t* src = proofs + ((size_t)b * h.stride + h.sc_off + 32u * k) / 4;
    Fe<Fs> v;
#pragma unroll
    for (int i = 0; i < 8; i++) v.l[i] = src[i];
    const bool ok = words_lt_mod<Fs>(v.l);
    if (!ok) {
      atomicOr(&status[b], kProofBadScalar);
      v = fe_zero<Fs>();
    }
    store_fe4<Fs>(reinterpret_cast<uint4*>(cscs + 8 * e), v);
    store_fe4<Fs>(reinterpret_cast<uint4*>(scalars + 8 * e), fe_to_mont<Fs>(v));
    return;
  }
  const size_t ei = e - nsc_all;  // an instance commitment (caller's affine Montgomery points)
  if (ei >= (size_t)h.B * h.ninst) return;
  const uint32_t b = (uint32_t)(ei / h.ninst), k = (uint32_t)(ei % h.ninst);
  const uint4* src = reinterpret_cast<const uint4*>(inst + 16 * ei);
  const Fe<F> x = load_fe4<F>(src), y = load_fe4<F>(src + 2);
  const size_t pi = (size_t)b * h.npts + k;  // instance commitments lead the point layout
  uint4* po = reinterpret_cast<uint4*>(points + 16 * pi);
  store_fe4<F>(po, x);
  store_fe4<F>(po + 2, y);
  uint4* co = reinterpret_cast<uint4*>(cpts + 16 * pi);
  store_fe4<F>(co, fe_from_mont<F>(x));
  store_fe4<F>(co + 2, fe_from_mont<F>(y));
  if (corr) {  // an affine input: the ladder ran on the curve itself
    const F29<F> one = f29_const<F>(F29Consts<F>::ONE);
    pow_st<F>(corr + pi * kAccCorrWords, one);
    pow_st<F>(corr + pi * kAccCorrWords + kPowWords, one);
  }
}

}  // namespace pm

// ntt_kernels.hpp -- NTT over a scalar field: halo2's
// `best_fft(a, omega, log_n)` [3P], the transform behind EvaluationDomain's
// fft / ifft / coset conversions in create_proof.  Output is the natural-order
// DFT  A_k = sum_j a_j omega^{jk}; it is exact field arithmetic, so any
// correct factorisation is bit-identical to halo2's radix-2 DIT.
//
// Four-step factorisation n = n1 * n2 (both <= 2^12), two passes over HBM:
//   pass A (k_ntt_cols): for every column i2, the n1-point NTT over
//     x[i1 * n2 + i2] (root omega^{n2}), times omega^{i2 k1}, stored in place
//     at [k1 * n2 + i2];
//   pass B (k_ntt_rows): for every row k1, the n2-point NTT over the contiguous
//     row (root omega^{n1}), stored at out[k1 + n1 * k2]  (natural order),
//     optionally times a scale (ifft: the 1/n divisor).
// Each sub-transform runs in LDS (structure of arrays: 8 limb planes, so
// lane-consecutive elements hit consecutive banks) as a radix-2 DIT on
// bit-reversed positions.  A workgroup takes C adjacent columns (pass A) or
// rows (pass B) so its global loads / stores move C x 32 contiguous bytes.
// All roots come from one table tw[i] = omega^i, i < n/2, built once per
// (field, omega, log_n) and cached in the context (omega^{n/2} = -1 covers
// the upper half).
#pragma once
#include "msm_kernels.hpp"

namespace pm {

#ifndef PM_NTT_THREADS
#define PM_NTT_THREADS 256
#endif
constexpr int kNttThreads = PM_NTT_THREADS;
constexpr int kNttMaxLogL = 12;  // longest sub-transform (2^12 x 32 B = 128 KiB of LDS)

struct FeArg {
  uint32_t l[8];
};

template <class Fs>
__device__ __forceinline__ Fe<Fs> fe_of(const FeArg& a) {
  Fe<Fs> r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = a.l[i];
  return r;
}

// tw[i] = omega^i for i < half (one square-and-multiply per entry, built once)
template <class Fs>
__global__ void __launch_bounds__(256) k_ntt_twiddles(FeArg omega, uint32_t half, uint32_t* __restrict__ tw) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= half) return;
  Fe<Fs> r = fe_one<Fs>(), b = fe_of<Fs>(omega);
  for (uint32_t e = i; e; e >>= 1) {
    if (e & 1) r = fe_mul<Fs>(r, b);
    b = fe_sqr<Fs>(b);
  }
  store_fe4<Fs>(reinterpret_cast<uint4*>(tw + 8ull * i), r);
}

__device__ __forceinline__ uint32_t ntt_brev(uint32_t x, int bits) { return bits ? __brev(x) >> (32 - bits) : 0u; }

template <class Fs>
__device__ __forceinline__ Fe<Fs> lds_ld(const uint32_t* sm, uint32_t plane, uint32_t idx) {
  Fe<Fs> r;
#pragma unroll
  for (int k = 0; k < 8; k++) r.l[k] = sm[k * plane + idx];
  return r;
}
template <class Fs>
__device__ __forceinline__ void lds_st(uint32_t* sm, uint32_t plane, uint32_t idx, const Fe<Fs>& v) {
#pragma unroll
  for (int k = 0; k < 8; k++) sm[k * plane + idx] = v.l[k];
}

// omega^e for e < n from the half table (omega^{n/2} = -1)
template <class Fs>
__device__ __forceinline__ Fe<Fs> tw_full(const uint32_t* __restrict__ tw, uint32_t e, uint32_t half) {
  if (e < half) return load_fe4<Fs>(reinterpret_cast<const uint4*>(tw + 8ull * e));
  return fe_neg<Fs>(load_fe4<Fs>(reinterpret_cast<const uint4*>(tw + 8ull * (e - half))));
}

// In-LDS radix-2 DIT over C interleaved transforms of length L = 2^logL
// (layout [position][c], positions already bit-reversed).  Root of unity of
// the sub-transform: omega^{tstride}, looked up as tw[m * tstride].
template <class Fs>
__device__ __forceinline__ void lds_ntt(uint32_t* sm, int logL, int logC, uint32_t tstride,
                                        const uint32_t* __restrict__ tw) {
  const uint32_t plane = 1u << (logL + logC);
  const uint32_t nbf = plane >> 1;  // butterflies per stage
  const uint32_t cmask = (1u << logC) - 1;
  for (int t = 0; t < logL; t++) {
    const uint32_t h = 1u << t;
    for (uint32_t b = threadIdx.x; b < nbf; b += kNttThreads) {
      const uint32_t c = b & cmask, bb = b >> logC;
      const uint32_t lo = bb & (h - 1);
      const uint32_t j = ((bb >> t) << (t + 1)) | lo;
      const uint32_t ia = (j << logC) | c, ib = ((j + h) << logC) | c;
      const Fe<Fs> u = lds_ld<Fs>(sm, plane, ia);
      Fe<Fs> v = lds_ld<Fs>(sm, plane, ib);
      if (t > 0) {  // stage 0 twiddle is 1
        const Fe<Fs> w =
            load_fe4<Fs>(reinterpret_cast<const uint4*>(tw + 8ull * ((size_t)(lo << (logL - 1 - t)) * tstride)));
        v = fe_mul<Fs>(v, w);
      }
      lds_st<Fs>(sm, plane, ia, fe_add<Fs>(u, v));
      lds_st<Fs>(sm, plane, ib, fe_sub<Fs>(u, v));
    }
    __syncthreads();
  }
}

// The same transform with two stages per LDS round trip (radix-4 units on
// positions j, j + h, j + 2h, j + 3h, h = 2^t): stage t with the twiddle
// W_{2h}^lo on both pairs, then stage t + 1 with W_{4h}^lo and W_{4h}^{lo+h}.
// Same products as two radix-2 stages, half the LDS traffic and barriers.
// An odd logL starts with one radix-2 stage (twiddle 1).
#ifndef PM_NTT_RADIX4
#define PM_NTT_RADIX4 1
#endif
template <class Fs>
__device__ __forceinline__ void lds_ntt4(uint32_t* sm, int logL, int logC, uint32_t tstride,
                                         const uint32_t* __restrict__ tw) {
  const uint32_t plane = 1u << (logL + logC);
  const uint32_t cmask = (1u << logC) - 1;
  int t = 0;
  if (logL & 1) {  // stage 0: twiddle 1
    for (uint32_t b = threadIdx.x; b < (plane >> 1); b += kNttThreads) {
      const uint32_t c = b & cmask, j = (b >> logC) << 1;
      const uint32_t ia = (j << logC) | c, ib = ((j + 1) << logC) | c;
      const Fe<Fs> u = lds_ld<Fs>(sm, plane, ia), v = lds_ld<Fs>(sm, plane, ib);
      lds_st<Fs>(sm, plane, ia, fe_add<Fs>(u, v));
      lds_st<Fs>(sm, plane, ib, fe_sub<Fs>(u, v));
    }
    __syncthreads();
    t = 1;
  }
  for (; t + 1 < logL; t += 2) {
    const uint32_t h = 1u << t;
    for (uint32_t b = threadIdx.x; b < (plane >> 2); b += kNttThreads) {
      const uint32_t c = b & cmask, bb = b >> logC;
      const uint32_t lo = bb & (h - 1);
      const uint32_t j = ((bb >> t) << (t + 2)) | lo;
      const uint32_t i0 = (j << logC) | c, i1 = ((j + h) << logC) | c, i2 = ((j + 2 * h) << logC) | c,
                     i3 = ((j + 3 * h) << logC) | c;
      Fe<Fs> x0 = lds_ld<Fs>(sm, plane, i0), x1 = lds_ld<Fs>(sm, plane, i1);
      Fe<Fs> x2 = lds_ld<Fs>(sm, plane, i2), x3 = lds_ld<Fs>(sm, plane, i3);
      if (t > 0) {
        const Fe<Fs> w1 =
            load_fe4<Fs>(reinterpret_cast<const uint4*>(tw + 8ull * ((size_t)(lo << (logL - 1 - t)) * tstride)));
        x1 = fe_mul<Fs>(x1, w1);
        x3 = fe_mul<Fs>(x3, w1);
      }
      const Fe<Fs> y0 = fe_add<Fs>(x0, x1), y1 = fe_sub<Fs>(x0, x1);
      const Fe<Fs> y2 = fe_add<Fs>(x2, x3), y3 = fe_sub<Fs>(x2, x3);
      const Fe<Fs> w2 =
          load_fe4<Fs>(reinterpret_cast<const uint4*>(tw + 8ull * ((size_t)(lo << (logL - 2 - t)) * tstride)));
      const Fe<Fs> w3 = load_fe4<Fs>(
          reinterpret_cast<const uint4*>(tw + 8ull * ((size_t)((lo + h) << (logL - 2 - t)) * tstride)));
      const Fe<Fs> z2 = fe_mul<Fs>(y2, w2), z3 = fe_mul<Fs>(y3, w3);
      lds_st<Fs>(sm, plane, i0, fe_add<Fs>(y0, z2));
      lds_st<Fs>(sm, plane, i2, fe_sub<Fs>(y0, z2));
      lds_st<Fs>(sm, plane, i1, fe_add<Fs>(y1, z3));
      lds_st<Fs>(sm, plane, i3, fe_sub<Fs>(y1, z3));
    }
    __syncthreads();
  }
}

// XCD-aware block order: consecutive logical blocks (adjacent columns / rows,
// which share 128-B lines) land on the same XCD and its L2.
__device__ __forceinline__ uint32_t ntt_block(uint32_t nblocks) {
  const uint32_t b = blockIdx.x;
  if (nblocks % 8) return b;
  return (b % 8) * (nblocks / 8) + b / 8;
}

// pass A: C = 2^logC adjacent columns per block
template <class Fs>
__global__ void __launch_bounds__(kNttThreads) k_ntt_cols(const uint32_t* in, uint32_t* out,  // may alias
                                                          int logn, int log1, int logC,
                                                          const uint32_t* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int log2 = logn - log1;
  const uint32_t n2 = 1u << log2, L = 1u << log1, C = 1u << logC, half = 1u << (logn - 1);
  const uint32_t plane = L << logC;
  const uint32_t col0 = ntt_block(n2 >> logC) << logC;
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t i1 = e >> logC, c = e & (C - 1);
    const Fe<Fs> v = load_fe4<Fs>(reinterpret_cast<const uint4*>(in + 8ull * ((size_t)i1 * n2 + col0 + c)));
    lds_st<Fs>(sm, plane, (ntt_brev(i1, log1) << logC) | c, v);
  }
  __syncthreads();
  if (PM_NTT_RADIX4) lds_ntt4<Fs>(sm, log1, logC, n2, tw);  // root omega^{n2}
  else lds_ntt<Fs>(sm, log1, logC, n2, tw);
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t k1 = e >> logC, c = e & (C - 1), i2 = col0 + c;
    Fe<Fs> v = lds_ld<Fs>(sm, plane, e);
    if (log2 > 0 && i2 && k1) v = fe_mul<Fs>(v, tw_full<Fs>(tw, i2 * k1, half));  // i2 k1 < n
    store_fe4<Fs>(reinterpret_cast<uint4*>(out + 8ull * ((size_t)k1 * n2 + i2)), v);
  }
}

// Three-pass form (n = n1 * na * nb, every factor <= 2^10, for n >= 2^23):
// pass A is k_ntt_cols with n2 = na * nb; the middle pass (k_ntt_mid) runs
// the row NTTs of length n2 (root omega^{n1}) as a four-step of their own:
// for every row k1 and column ib of the row's na x nb matrix, the na-point
// NTT over ia (root omega^{n1 nb}), times omega^{n1 ib ka}, stored at
// [(ka n1 + k1) nb + ib] so that pass B (k_ntt_rows over the n1 na rows of
// length nb, root omega^{n1 na}) writes out[k1 + n1 ka + n1 na kb] =
// out[k1 + n1 k2] with k2 = ka + na kb: the natural order.
template <class Fs>
__global__ void __launch_bounds__(kNttThreads) k_ntt_mid(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                         int logn, int log1, int loga, int logC,
                                                         const uint32_t* __restrict__ tw) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int logb = logn - log1 - loga;
  const uint32_t n1 = 1u << log1, na = 1u << loga, nb = 1u << logb, C = 1u << logC, half = 1u << (logn - 1);
  const uint32_t plane = na << logC;
  const uint32_t groups = nb >> logC;  // column groups per row
  const uint32_t blk = ntt_block(n1 * groups);
  const uint32_t k1 = blk / groups, col0 = (blk - k1 * groups) << logC;
  const uint32_t* row = in + 8ull * ((size_t)k1 << (loga + logb));
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t ia = e >> logC, c = e & (C - 1);
    const Fe<Fs> v = load_fe4<Fs>(reinterpret_cast<const uint4*>(row + 8ull * ((size_t)ia * nb + col0 + c)));
    lds_st<Fs>(sm, plane, (ntt_brev(ia, loga) << logC) | c, v);
  }
  __syncthreads();
  if (PM_NTT_RADIX4) lds_ntt4<Fs>(sm, loga, logC, n1 * nb, tw);  // root omega^{n1 nb}
  else lds_ntt<Fs>(sm, loga, logC, n1 * nb, tw);
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t ka = e >> logC, c = e & (C - 1), ib = col0 + c;
    Fe<Fs> v = lds_ld<Fs>(sm, plane, e);
    if (ib && ka) v = fe_mul<Fs>(v, tw_full<Fs>(tw, n1 * ib * ka, half));  // n1 ib ka < n
    store_fe4<Fs>(reinterpret_cast<uint4*>(out + 8ull * (((size_t)ka * n1 + k1) * nb + ib)), v);
  }
}

// pass B: R = 2^logR adjacent rows per block; optional output scale
template <class Fs>
__global__ void __launch_bounds__(kNttThreads) k_ntt_rows(const uint32_t* in, uint32_t* out,  // may alias (log2 = 0)
                                                          int logn, int log2, int logR,
                                                          const uint32_t* __restrict__ tw, FeArg scale,
                                                          uint32_t use_scale) {
  extern __shared__ __attribute__((aligned(16))) uint32_t sm[];
  const int log1 = logn - log2;
  const uint32_t n1 = 1u << log1, L = 1u << log2, R = 1u << logR;
  const uint32_t plane = L << logR;
  const uint32_t row0 = ntt_block(n1 >> logR) << logR;
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t r = e >> log2, i2 = e & (L - 1);  // row-contiguous loads
    const Fe<Fs> v = load_fe4<Fs>(reinterpret_cast<const uint4*>(in + 8ull * ((size_t)(row0 + r) * L + i2)));
    lds_st<Fs>(sm, plane, (ntt_brev(i2, log2) << logR) | r, v);
  }
  __syncthreads();
  if (PM_NTT_RADIX4) lds_ntt4<Fs>(sm, log2, logR, n1, tw);  // root omega^{n1}
  else lds_ntt<Fs>(sm, log2, logR, n1, tw);
  const Fe<Fs> sc = fe_of<Fs>(scale);
  for (uint32_t e = threadIdx.x; e < plane; e += kNttThreads) {
    const uint32_t r = e & (R - 1), k2 = e >> logR;  // adjacent rows -> adjacent outputs
    Fe<Fs> v = lds_ld<Fs>(sm, plane, e);
    if (use_scale) v = fe_mul<Fs>(v, sc);
    store_fe4<Fs>(reinterpret_cast<uint4*>(out + 8ull * ((size_t)(row0 + r) + (size_t)n1 * k2)), v);
  }
}

}  // namespace pm

// selftest.hpp -- device self-test of the radix-2^29 lazy field (fp29.hpp)
// against the 32-bit FIPS arithmetic (fp256.hpp), exported as
// pm_selftest_field so the GPU test-suite can run it through the C-ABI.
// Each lane draws a, b (uniform < p, or an edge value) and checks conversion,
// product, square, loose-limb operands at the bound (A + 6p), the 16p -> 3p
// reduction, the zero-mod-p filter and negation.
#pragma once
#include "curve29.hpp"
#include "msm_kernels.hpp"

namespace pm {

template <class F>
__device__ __forceinline__ bool f29_eq_r256(const F29<F>& v, const Fe<F>& want) {
  uint32_t w[8];
  f29_to_r256<F>(v, w);
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= w[i] ^ want.l[i];
  return d == 0;
}

template <class F>
__device__ __forceinline__ Fe<F> st_edge(uint32_t k, const Fe<F>& r) {
  Fe<F> v = fe_zero<F>();
  switch (k) {
    case 0: return v;                                                                   // 0
    case 1: v.l[0] = 1; return v;                                                       // 1
    case 2: {                                                                           // p - 1
      uint32_t br = 0;
      const uint32_t one[8] = {1, 0, 0, 0, 0, 0, 0, 0};
      for (int i = 0; i < 8; i++) v.l[i] = subb(F::MOD[i], one[i], br);
      return v;
    }
    case 3: for (int i = 0; i < 8; i++) v.l[i] = F::ONE[i]; return v;                   // R256 one
    case 4: {                                                                           // p - 2
      uint32_t br = 0;
      const uint32_t two[8] = {2, 0, 0, 0, 0, 0, 0, 0};
      for (int i = 0; i < 8; i++) v.l[i] = subb(F::MOD[i], two[i], br);
      return v;
    }
    default: return r;
  }
}

template <class F>
__global__ void k_selftest_field(uint64_t seed, uint32_t n, uint32_t* __restrict__ bad) {
  using K = F29Consts<F>;
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const Fe<F> a = st_edge<F>(i % 32, synth_scalar<F>(seed, 2ull * i));
  const Fe<F> b = st_edge<F>((i / 32) % 32, synth_scalar<F>(seed, 2ull * i + 1));
  uint32_t nb = 0;
  const F29<F> A = f29_from_r256<F>(a.l), B = f29_from_r256<F>(b.l);
  const Fe<F> ab = fe_mul<F>(a, b), aa = fe_mul<F>(a, a);
  nb += !f29_eq_r256<F>(A, a);
  nb += !f29_eq_r256<F>(f29_mul<F>(A, B), ab);
  nb += !f29_eq_r256<F>(f29_sqr<F>(A), aa);
  nb += !f29_eq_r256<F>(f29_mul_c<F>(A, B), ab);
  nb += !f29_eq_r256<F>(f29_sqr_c<F>(A), aa);
  // loose operand at the limb bound: A + 6p (limbs up to 2^29 + K6_i), value < 8p
  const F29<F> L = f29_sub<F>(A, f29_zero<F>(), K::K6);
  nb += !f29_eq_r256<F>(f29_mul<F>(L, B), ab);
  nb += !f29_eq_r256<F>(f29_mul<F>(B, L), ab);
  nb += !f29_eq_r256<F>(f29_mul_c<F>(L, B), ab);
  nb += !f29_eq_r256<F>(f29_mul_c<F>(B, L), ab);
  const F29<F> Ln = f29_norm<F>(L);
  nb += !f29_eq_r256<F>(f29_sqr<F>(Ln), aa);
  nb += !f29_eq_r256<F>(f29_sqr_c<F>(Ln), aa);
  nb += !f29_eq_r256<F>(f29_mul<F>(Ln, Ln), aa);
  // 16p -> 3p reduction of (A + 6p) + (A + 6p) = 2A + 12p  (< 16p)
  const F29<F> T = f29_reduce3<F>(f29_norm<F>(f29_add<F>(L, L)));
  nb += !f29_eq_r256<F>(T, fe_add<F>(a, a));
  nb += !f29_eq_r256<F>(f29_canon<F>(T), fe_add<F>(a, a));
  // difference of products: a b - (2a) b = -a b, u = 2A reduced below 3p
  nb += !f29_eq_r256<F>(f29_mul2n_c<F>(A, B, T, B), fe_neg<F>(ab));
  nb += !f29_eq_r256<F>(f29_mul2n_c<F>(Ln, B, A, B), fe_sub<F>(fe_mul<F>(a, b), ab));
  // zero mod p: A - A + 6p = 6p
  nb += !f29_is_zero_mod<F>(f29_norm<F>(f29_sub<F>(A, A, K::K6)));
  nb += f29_is_zero_mod<F>(A) != fe_is_zero<F>(a);
  // negation of a canonical value
  nb += !f29_eq_r256<F>(f29_neg_canon<F>(f29_canon<F>(A)), fe_neg<F>(a));
  // pack / unpack round trip of a canonical value
  uint32_t w[8];
  f29_pack<F>(f29_canon<F>(A), w);
  nb += !f29_eq_r256<F>(f29_unpack<F>(w), a);
  // inversions: binary GCD (inv_bgcd.hpp) against Fermat, R256 and R261 forms
  // (f29_inv takes Norm < 4p: T = 2A reduced below 3p exercises its
  // canonicalisation)
  const Fe<F> ia = fe_inv<F>(a);
  const Fe<F> ib = fe_inv_fast<F>(a);
  uint32_t d = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) d |= ia.l[k] ^ ib.l[k];
  nb += d != 0;
  nb += !f29_eq_r256<F>(f29_inv<F>(A), ia);
  nb += !f29_eq_r256<F>(f29_inv<F>(T), fe_inv<F>(fe_add<F>(a, a)));
  nb += !f29_eq_r256<F>(f29_inv_fermat<F>(A), ia);
  // quad-cooperative inversion: the 4 lanes of a quad share one input (edge
  // case (i / 4) % 32), checked only for whole quads
  if ((i | 3u) < n) {
    const uint32_t i4 = i >> 2;
    const Fe<F> c = st_edge<F>(i4 % 32, synth_scalar<F>(seed ^ 0x9E37ull, i4));
    nb += !f29_eq_r256<F>(f29_inv_q<F>(f29_from_r256<F>(c.l)), fe_inv<F>(c));
  }
  if (nb) atomicAdd(bad, nb);
}

template <class Cv>
int selftest_field_impl(Ctx* ctx, uint64_t seed, uint32_t n, uint64_t* mismatches) {
  using F = typename Cv::Base;
  int rc;
  if ((rc = ctx->win.ensure(16))) return rc;
  HIP_TRY(hipMemsetAsync(ctx->win.p, 0, 4, ctx->stream));
  k_selftest_field<F><<<(n + 255) / 256, 256, 0, ctx->stream>>>(seed, n, (uint32_t*)ctx->win.p);
  HIP_TRY(hipGetLastError());
  uint32_t nb = 0;
  HIP_TRY(hipMemcpyAsync(&nb, ctx->win.p, 4, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(hipStreamSynchronize(ctx->stream));
  *mismatches = nb;
  return PM_OK;
}

}  // namespace pm

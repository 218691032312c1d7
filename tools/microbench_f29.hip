// microbench_f29.hip -- throughput / single-wave latency of the field product
// variants on gfx950: 32-bit FIPS (fp256.hpp) vs radix-2^29 lazy (fp29.hpp),
// plus the XYZZ mixed add in both representations.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_f29 tools/microbench_f29.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../halo2-aggregation_amd/csrc/curve29.hpp"
using namespace pm;
using F = PallasFp;

template <int V>
__global__ void __launch_bounds__(256) k_mul(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (V < 2) {
    Fe<F> a, b;
    for (int i = 0; i < 8; i++) { a.l[i] = t * 7 + i * 977; b.l[i] = t * 3 + i * 131; }
    a.l[7] &= 0x0fffffff; b.l[7] &= 0x0fffffff;
#if defined(__HIP_DEVICE_COMPILE__)
    for (int k = 0; k < iters; k++) a = V == 0 ? fe_mul_fips_g<F>(a, b) : fe_mul_fips_g<F>(a, a);
#endif
    for (int i = 0; i < 8; i++) out[8 * t + i] = a.l[i];
  } else {
    F29<F> a, b;
    for (int i = 0; i < 9; i++) { a.l[i] = (t * 7 + i * 977) & kM29; b.l[i] = (t * 3 + i * 131) & kM29; }
#if defined(__HIP_DEVICE_COMPILE__)
    for (int k = 0; k < iters; k++)
      a = V == 2 ? f29_mul<F>(a, b) : V == 3 ? f29_sqr<F>(a) : V == 4 ? f29_mul_c<F>(a, b) : f29_sqr_c<F>(a);
#endif
    for (int i = 0; i < 8; i++) out[8 * t + i] = a.l[i];
  }
}

template <int V>
__global__ void __launch_bounds__(256) k_madd(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (V == 0) {
    Aff<F> p; Xyzz<F> acc;
    for (int i = 0; i < 8; i++) { p.x.l[i] = t * 7 + i; p.y.l[i] = t * 3 + i; }
    p.x.l[7] &= 0x3fffffff; p.y.l[7] &= 0x3fffffff;
    acc.X = p.y; acc.Y = p.x; acc.ZZ = p.x; acc.ZZZ = p.y;
    for (int k = 0; k < iters; k++) acc = xyzz_add_aff<F>(acc, p);
    for (int i = 0; i < 8; i++) out[8 * t + i] = acc.X.l[i];
  } else {
    F29<F> x, y; Xyzz29<F> acc;
    for (int i = 0; i < 9; i++) { x.l[i] = (t * 7 + i) & kM29; y.l[i] = (t * 3 + i) & kM29; }
    x.l[8] &= 0x3fffff; y.l[8] &= 0x3fffff;
    acc.X = y; acc.Y = x; acc.ZZ = x; acc.ZZZ = y;
    bool inf = false;
    for (int k = 0; k < iters; k++)
      acc = V == 1   ? xyzz29_madd<F>(acc, x, y, inf)
            : V == 2 ? xyzz29_madd_signed<F>(acc, x, y, (uint32_t)k & 1u ? ~0u : 0u)
                     : xyzz29_madd_lazy<F>(acc, x, y, (uint32_t)k & 1u ? ~0u : 0u);  // k_accumulate's step (r5)
    for (int i = 0; i < 8; i++) out[8 * t + i] = acc.X.l[i];
  }
}

// field inversion throughput (f29_inv: binary GCD in round 2, the safegcd
// since round 5): the cost a batch-affine
// bucket accumulation would amortise over the independent additions of a batch
__global__ void __launch_bounds__(256) k_inv(uint32_t* out, int iters) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F29<F> a;
  for (int i = 0; i < 9; i++) a.l[i] = (t * 7 + i * 977 + 1) & kM29;
  a.l[8] &= 0x3fffff;
#if defined(__HIP_DEVICE_COMPILE__)
  for (int k = 0; k < iters; k++) {
    a = f29_inv<F>(a);
    a.l[0] += 1;  // keep it nonzero and varying
  }
#endif
  for (int i = 0; i < 8; i++) out[8 * t + i] = a.l[i];
}

// Batch-affine addition (the verdict's alternative to XYZZ buckets): each
// lane keeps K independent affine accumulators (x1, y1) and adds a base
// (x2, y2) to each per batch with ONE inversion: prefix products of
// d_k = x2 - x1_k (Montgomery's trick), f29_inv, then per k
// inv_k = inv c_{k-1}, inv *= d_k, lambda = (y2 - y1_k) inv_k,
// x3 = lambda^2 - x1 - x2, y3 = lambda (x1 - x3) - y1.  Throughput only
// (arbitrary field elements: no exceptional cases arise).  REG: the K
// accumulators and prefixes live in registers (small K); else in a
// lane-private global scratch, [k][word][lane] (coalesced), as a real
// bucket pass would need (LDS cannot hold K x 108 B for 1024 lanes per CU).
__device__ __forceinline__ F29<F> sub29(const F29<F>& a, const F29<F>& b) {
  return f29_reduce3<F>(f29_norm<F>(f29_sub<F>(a, b, F29Consts<F>::K6)));
}
template <int K, bool REG>
__global__ void __launch_bounds__(256) k_batch_affine(uint32_t* out, int iters, uint32_t* scratch, uint32_t nl) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  F29<F> x2, y2;
  for (int i = 0; i < 9; i++) { x2.l[i] = (t * 5 + i * 31) & kM29; y2.l[i] = (t * 11 + i * 7) & kM29; }
  x2.l[8] &= 0x3fffff; y2.l[8] &= 0x3fffff;
  F29<F> rx[REG ? K : 1], ry[REG ? K : 1], rc[REG ? K : 1];
  auto ld = [&](int k, int c) {
    F29<F> v;
    for (int i = 0; i < 9; i++) v.l[i] = scratch[((size_t)(k * 3 + c) * 9 + i) * nl + t];
    return v;
  };
  auto st = [&](int k, int c, const F29<F>& v) {
    for (int i = 0; i < 9; i++) scratch[((size_t)(k * 3 + c) * 9 + i) * nl + t] = v.l[i];
  };
#pragma unroll
  for (int k = 0; k < K; k++) {
    F29<F> x, y;
    for (int i = 0; i < 9; i++) { x.l[i] = (t * 7 + i + 13 * k) & kM29; y.l[i] = (t * 3 + i + 17 * k) & kM29; }
    x.l[8] &= 0x3fffff; y.l[8] &= 0x3fffff;
    if (REG) { rx[REG ? k : 0] = x; ry[REG ? k : 0] = y; } else { st(k, 0, x); st(k, 1, y); }
  }
#if defined(__HIP_DEVICE_COMPILE__)
  for (int it = 0; it < iters; it++) {
    F29<F> c = f29_const<F>(F29Consts<F>::ONE);
#pragma unroll(REG ? K : 1)
    for (int k = 0; k < K; k++) {
      const F29<F> x1 = REG ? rx[REG ? k : 0] : ld(k, 0);
      c = f29_mul_c<F>(c, sub29(x2, x1));
      if (REG) rc[REG ? k : 0] = c; else st(k, 2, c);
    }
    F29<F> inv = f29_inv<F>(c);
#pragma unroll(REG ? K : 1)
    for (int k = K - 1; k >= 0; k--) {
      const F29<F> x1 = REG ? rx[REG ? k : 0] : ld(k, 0), y1 = REG ? ry[REG ? k : 0] : ld(k, 1);
      const F29<F> cp = k ? (REG ? rc[REG ? k - 1 : 0] : ld(k - 1, 2)) : f29_const<F>(F29Consts<F>::ONE);
      const F29<F> ik = f29_mul_c<F>(inv, cp);
      inv = f29_mul_c<F>(inv, sub29(x2, x1));
      const F29<F> lam = f29_mul_c<F>(sub29(y2, y1), ik);
      const F29<F> x3 = sub29(sub29(f29_sqr_c<F>(lam), x1), x2);
      const F29<F> y3 = sub29(f29_mul_c<F>(lam, sub29(x1, x3)), y1);
      if (REG) { rx[REG ? k : 0] = x3; ry[REG ? k : 0] = y3; } else { st(k, 0, x3); st(k, 1, y3); }
    }
  }
#endif
  const F29<F> r = REG ? rx[0] : ld(0, 0);
  for (int i = 0; i < 8; i++) out[8 * t + i] = r.l[i];
}

template <class Kern>
void run(const char* name, Kern k, void* buf, int iters, double ops_per_iter) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  int blocks = 256 * 8, threads = 256;
  k<<<blocks, threads>>>((uint32_t*)buf, 4); hipDeviceSynchronize();
  hipEventRecord(e0);
  k<<<blocks, threads>>>((uint32_t*)buf, iters);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  double tput = (double)blocks * threads * iters * ops_per_iter / ms / 1e6;
  int li = 4000;
  k<<<1, 64>>>((uint32_t*)buf, 4); hipDeviceSynchronize();
  hipEventRecord(e0);
  k<<<1, 64>>>((uint32_t*)buf, li);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("{\"bench\":\"%s\",\"G_per_s\":%.2f,\"latency_ns\":%.1f}\n", name, tput, ms * 1e6 / li);
}

int main() {
  void* buf;
  hipMalloc(&buf, 256ull << 20);
  run("fe_mul_fips_g", k_mul<0>, buf, 1024, 1);
  run("fe_sqr_fips_g", k_mul<1>, buf, 1024, 1);
  run("f29_mul", k_mul<2>, buf, 1024, 1);
  run("f29_sqr", k_mul<3>, buf, 1024, 1);
  run("f29_mul_c", k_mul<4>, buf, 1024, 1);
  run("f29_sqr_c", k_mul<5>, buf, 1024, 1);
  run("xyzz_madd_32", k_madd<0>, buf, 128, 1);
  run("xyzz_madd_29", k_madd<1>, buf, 128, 1);
  run("xyzz_madd_signed_29", k_madd<2>, buf, 128, 1);
  run("xyzz_madd_lazy_29", k_madd<3>, buf, 128, 1);
  run("f29_inv_safegcd", k_inv, buf, 16, 1);
  // batch-affine: lanes = 1024 blocks x 256 (k_accumulate's grid at 2^20)
  {
    const uint32_t blocks = 1024, threads = 256, nl = blocks * threads;
    uint32_t* scratch;
    hipMalloc(&scratch, (size_t)nl * 256 * 27 * 4);
    auto ba = [&](const char* name, auto kern, int K, int iters) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0); hipEventCreate(&e1);
      float ms;
      kern<<<blocks, threads>>>((uint32_t*)buf, 1, scratch, nl); hipDeviceSynchronize();
      hipEventRecord(e0);
      kern<<<blocks, threads>>>((uint32_t*)buf, iters, scratch, nl);
      hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
      printf("{\"bench\":\"%s\",\"K\":%d,\"G_adds_per_s\":%.2f}\n", name, K,
             (double)nl * iters * K / ms / 1e6);
    };
    ba("batch_affine_reg", k_batch_affine<4, true>, 4, 16);
    ba("batch_affine_reg", k_batch_affine<8, true>, 8, 8);
    ba("batch_affine_mem", k_batch_affine<16, false>, 16, 4);
    ba("batch_affine_mem", k_batch_affine<32, false>, 32, 2);
    ba("batch_affine_mem", k_batch_affine<64, false>, 64, 1);
    ba("batch_affine_mem", k_batch_affine<128, false>, 128, 1);
    ba("batch_affine_mem", k_batch_affine<256, false>, 256, 1);
    hipFree(scratch);
  }
  return 0;
}

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
__global__ void k_mul(uint32_t* out, int iters) {
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
__global__ void k_madd(uint32_t* out, int iters) {
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
    for (int k = 0; k < iters; k++) acc = xyzz29_madd<F>(acc, x, y, inf);
    for (int i = 0; i < 8; i++) out[8 * t + i] = acc.X.l[i];
  }
}

// field inversion throughput (binary GCD, f29_inv): the cost a batch-affine
// bucket accumulation would amortise over the independent additions of a batch
__global__ void k_inv(uint32_t* out, int iters) {
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
  run("f29_inv_bgcd", k_inv, buf, 16, 1);
  return 0;
}

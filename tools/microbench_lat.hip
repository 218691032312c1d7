// microbench_lat.hip -- fe_mul_fips vs fe_mul_fips_g (grouped asm): throughput (full
// occupancy) and latency (one wave), plus a correctness cross-check.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_lat tools/microbench_lat.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../halo2-aggregation_amd/csrc/curve.hpp"
using namespace pm;

template <class P, int V>
__device__ __forceinline__ Fe<P> mulv(const Fe<P>& a, const Fe<P>& b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return V == 0 ? fe_mul_fips<P>(a, b) : fe_mul_fips_g<P>(a, b);
#else
  return a;
#endif
}

template <class P, int V>
__global__ void k_mul(uint32_t* out, int iters) {
  Fe<P> a, b;
  for (int i = 0; i < 8; i++) { a.l[i] = threadIdx.x * 7 + i * 977 + blockIdx.x; b.l[i] = blockIdx.x * 3 + i * 131; }
  a.l[7] &= 0x0fffffff; b.l[7] &= 0x0fffffff;
  for (int k = 0; k < iters; k++) a = mulv<P, V>(a, b);
  fe_store<P>(out + 8 * (blockIdx.x * blockDim.x + threadIdx.x), a);
}

// plain-C CIOS reference (no inline asm)
template <class P>
__device__ Fe<P> mul_ref(const Fe<P>& a, const Fe<P>& b) {
  uint32_t t[10];
  for (int i = 0; i < 10; i++) t[i] = 0;
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 8; j++) {
      uint64_t s = (uint64_t)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint32_t)s;
      c = s >> 32;
    }
    uint64_t s = (uint64_t)t[8] + c;
    t[8] = (uint32_t)s;
    t[9] = (uint32_t)(s >> 32);
    const uint32_t m = t[0] * P::INV;
    s = (uint64_t)m * P::MOD[0] + t[0];
    c = s >> 32;
    for (int j = 1; j < 8; j++) {
      s = (uint64_t)m * P::MOD[j] + t[j] + c;
      t[j - 1] = (uint32_t)s;
      c = s >> 32;
    }
    s = (uint64_t)t[8] + c;
    t[7] = (uint32_t)s;
    t[8] = t[9] + (uint32_t)(s >> 32);
  }
  return fe_reduce_once<P>(t, t[8]);
}

template <class P>
__global__ void k_check(uint32_t* bad, int n) {
  Fe<P> a, b;
  uint32_t s = threadIdx.x * 2654435761u + blockIdx.x * 40503u + 1;
  for (int t = 0; t < n; t++) {
    for (int i = 0; i < 8; i++) { s = s * 1664525u + 1013904223u; a.l[i] = s; s = s * 1664525u + 1013904223u; b.l[i] = s; }
    a.l[7] &= 0x1fffffff; b.l[7] &= 0x1fffffff;
    if (t == 0) { for (int i = 0; i < 8; i++) { a.l[i] = P::MOD[i]; b.l[i] = P::MOD[i]; } a.l[0] -= 1; b.l[0] -= 1; }
    const Fe<P> x = mulv<P, 0>(a, b), y = mulv<P, 2>(a, b), z = y, w = mul_ref<P>(a, b);
    if (!fe_eq<P>(x, w) || !fe_eq<P>(y, w) || !fe_eq<P>(z, w)) atomicAdd(bad, 1u);
  }
}

template <class P, int V>
void run(const char* name, void* buf, hipEvent_t e0, hipEvent_t e1) {
  float ms;
  int blocks = 256 * 8, threads = 256, iters = 1024;
  k_mul<P, V><<<blocks, threads>>>((uint32_t*)buf, 8); hipDeviceSynchronize();
  hipEventRecord(e0);
  k_mul<P, V><<<blocks, threads>>>((uint32_t*)buf, iters);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  double tput = (double)blocks * threads * iters / ms / 1e6;
  iters = 20000;
  k_mul<P, V><<<1, 64>>>((uint32_t*)buf, 8); hipDeviceSynchronize();
  hipEventRecord(e0);
  k_mul<P, V><<<1, 64>>>((uint32_t*)buf, iters);
  hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
  printf("{\"field\":\"%s\",\"variant\":\"%s\",\"Gmul_s\":%.2f,\"latency_ns\":%.1f}\n", name, V == 0 ? "fips" : "fips_grouped", tput,
         ms * 1e6 / iters);
}

int main() {
  void* buf;
  hipMalloc(&buf, 256ull << 20);
  uint32_t* bad;
  hipMalloc(&bad, 4);
  hipMemset(bad, 0, 4);
  k_check<PallasFp><<<256, 256>>>(bad, 64);
  k_check<Bn254Fq><<<256, 256>>>(bad, 64);
  k_check<Bn254Fr><<<256, 256>>>(bad, 64);
  uint32_t nb = 0;
  hipMemcpy(&nb, bad, 4, hipMemcpyDeviceToHost);
  printf("{\"check_mismatches\":%u}\n", nb);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  run<PallasFp, 0>("pallas", buf, e0, e1);
  run<PallasFp, 2>("pallas", buf, e0, e1);
  run<Bn254Fq, 0>("bn254", buf, e0, e1);
  run<Bn254Fq, 2>("bn254", buf, e0, e1);
  return nb != 0;
}

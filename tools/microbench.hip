// microbench.hip -- integer-VALU ceilings on gfx950 for the roofline report:
//   (1) raw v_mad_u64_u32 issue rate (independent chains, full occupancy)
//   (2) Montgomery fe_mul throughput (full occupancy) and (3) latency (1 wave)
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench tools/microbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>
#include "../halo2-aggregation_amd/csrc/curve.hpp"
using namespace pm;

__global__ void k_mad(uint64_t* out, int iters, uint32_t seed) {
  uint32_t a[8];
  uint64_t acc[8];
  for (int k = 0; k < 8; k++) { a[k] = seed * (threadIdx.x + k + 1); acc[k] = a[k]; }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = (uint64_t)a[k] * (uint32_t)(acc[k] >> 32) + acc[k];
  }
  uint64_t s = 0;
  for (int k = 0; k < 8; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_femul(uint32_t* out, int iters) {
  Fe<PallasFp> a, b;
  for (int i = 0; i < 8; i++) { a.l[i] = threadIdx.x * 7 + i; b.l[i] = blockIdx.x * 3 + i; }
  a.l[7] &= 0x3fffffff; b.l[7] &= 0x3fffffff;
  for (int k = 0; k < iters; k++) a = fe_mul<PallasFp>(a, b);
  fe_store<PallasFp>(out + 8 * (blockIdx.x * blockDim.x + threadIdx.x), a);
}

__global__ void k_madd(uint32_t* out, int iters) {
  Aff<PallasFp> p;
  Xyzz<PallasFp> acc;
  for (int i = 0; i < 8; i++) { p.x.l[i] = threadIdx.x * 7 + i; p.y.l[i] = blockIdx.x * 3 + i; }
  p.x.l[7] &= 0x3fffffff; p.y.l[7] &= 0x3fffffff;
  acc.X = p.y; acc.Y = p.x; acc.ZZ = p.x; acc.ZZZ = p.y;
  for (int k = 0; k < iters; k++) acc = xyzz_add_aff<PallasFp>(acc, p);
  fe_store<PallasFp>(out + 8 * (blockIdx.x * blockDim.x + threadIdx.x), acc.X);
}


int main() {
  void* buf;
  hipMalloc(&buf, 256ull << 20);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  float ms;
  int cus = 256;
  // (1) raw mad rate
  {
    int blocks = cus * 8, threads = 256, iters = 4096;
    k_mad<<<blocks, threads>>>((uint64_t*)buf, 16, 3); hipDeviceSynchronize();
    hipEventRecord(e0);
    k_mad<<<blocks, threads>>>((uint64_t*)buf, iters, 3);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * threads * iters * 8;
    printf("{\"bench\":\"v_mad_u64_u32\",\"Gops\":%.1f,\"ms\":%.3f}\n", ops / ms / 1e6, ms);
  }
  // (2) fe_mul throughput
  for (int wpb : {1, 2, 4, 8}) {
    int blocks = cus * wpb, threads = 256, iters = 2048;
    k_femul<<<blocks, threads>>>((uint32_t*)buf, 16); hipDeviceSynchronize();
    hipEventRecord(e0);
    k_femul<<<blocks, threads>>>((uint32_t*)buf, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * threads * iters;
    printf("{\"bench\":\"fe_mul\",\"blocks_per_cu\":%d,\"Gmul_s\":%.2f,\"ms\":%.3f}\n", wpb, ops / ms / 1e6, ms);
  }
  // (3) fe_mul latency: one wave
  {
    int iters = 20000;
    k_femul<<<1, 64>>>((uint32_t*)buf, 16); hipDeviceSynchronize();
    hipEventRecord(e0);
    k_femul<<<1, 64>>>((uint32_t*)buf, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("{\"bench\":\"fe_mul_latency_1wave\",\"ns_per_mul\":%.1f}\n", ms * 1e6 / iters);
  }
  // (4) mixed add throughput + latency
  {
    int blocks = cus * 4, threads = 256, iters = 256;
    k_madd<<<blocks, threads>>>((uint32_t*)buf, 4); hipDeviceSynchronize();
    hipEventRecord(e0);
    k_madd<<<blocks, threads>>>((uint32_t*)buf, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * threads * iters;
    printf("{\"bench\":\"xyzz_add_aff\",\"Gadd_s\":%.3f,\"ms\":%.3f}\n", ops / ms / 1e6, ms);
    iters = 2000;
    hipEventRecord(e0);
    k_madd<<<1, 64>>>((uint32_t*)buf, iters);
    hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1);
    printf("{\"bench\":\"xyzz_add_aff_latency_1wave\",\"ns_per_add\":%.1f}\n", ms * 1e6 / iters);
  }
  return 0;
}

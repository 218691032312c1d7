// microbench_fp64.hip -- issue rates of the multiply primitives a 255-bit
// Montgomery product could be built from on gfx950 (independent chains, full
// occupancy): v_mad_u64_u32 (32x32->64), v_fma_f64 (52x52 products via the
// hi/lo FMA split), v_mul_u32_u24 + v_mul_hi_u32_u24 (24x24->48).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/microbench_fp64 tools/microbench_fp64.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) (void)(x)

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

__global__ void k_fma64(double* out, int iters, double seed) {
  double a[8], acc[8];
  for (int k = 0; k < 8; k++) { a[k] = seed * (threadIdx.x + k + 1) * 1e-9; acc[k] = a[k]; }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) acc[k] = __fma_rn(a[k], acc[k], 0.5);
  }
  double s = 0;
  for (int k = 0; k < 8; k++) s += acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_mul24(uint32_t* out, int iters, uint32_t seed) {
  uint32_t a[8], lo[8], hi[8];
  for (int k = 0; k < 8; k++) { a[k] = (seed * (threadIdx.x + k + 1)) & 0xffffff; lo[k] = a[k]; hi[k] = k; }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t x = lo[k] & 0xffffff;
      const uint64_t p = (uint64_t)a[k] * x;  // 24 x 24 -> v_mul_u32_u24 + v_mul_hi_u32_u24
      lo[k] = (uint32_t)p + hi[k];
      hi[k] = (uint32_t)(p >> 32);
    }
  }
  uint32_t s = 0;
  for (int k = 0; k < 8; k++) s ^= lo[k] ^ hi[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  void* buf;
  CK(hipMalloc(&buf, 64ull << 20));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float ms;
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  const double ops = (double)blocks * threads * iters * 8;
  k_mad<<<blocks, threads>>>((uint64_t*)buf, 16, 3);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  k_mad<<<blocks, threads>>>((uint64_t*)buf, iters, 3);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("{\"bench\":\"v_mad_u64_u32\",\"Tops\":%.2f}\n", ops / ms / 1e9);
  k_fma64<<<blocks, threads>>>((double*)buf, 16, 3.0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  k_fma64<<<blocks, threads>>>((double*)buf, iters, 3.0);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("{\"bench\":\"v_fma_f64\",\"Tops\":%.2f}\n", ops / ms / 1e9);
  k_mul24<<<blocks, threads>>>((uint32_t*)buf, 16, 3);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  k_mul24<<<blocks, threads>>>((uint32_t*)buf, iters, 3);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  CK(hipEventElapsedTime(&ms, e0, e1));
  printf("{\"bench\":\"v_mul_u32_u24+v_mul_hi_u32_u24 pairs\",\"Tops\":%.2f}\n", ops / ms / 1e9);
  return 0;
}

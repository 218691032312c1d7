// microbench_isa.hip -- issue cost of the integer VALU instructions the
// radix-2^29 products are made of, and product throughput per variant, at a
// controlled number of waves per SIMD (256 x k blocks of 256 lanes).
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_isa tools/microbench_isa.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../halo2-aggregation_amd/csrc/curve29.hpp"
using namespace pm;
using F = PallasFp;

#define MAD(A, X, Y) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(A), "=&s"(c) : "v"(X), "v"(Y))

// NC independent v_mad_u64_u32 chains per lane
template <int NC>
__global__ void __launch_bounds__(256) k_mad(uint64_t* out, int iters) {
  uint64_t acc[NC], c;
  uint32_t x = threadIdx.x * 3 + 1, y = blockIdx.x + 7;
#pragma unroll
  for (int k = 0; k < NC; k++) acc[k] = x + k;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int k = 0; k < NC; k++) MAD(acc[k], x, y);
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < NC; k++) s ^= acc[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// 32-bit ops: v_and_b32 (OP 0), v_lshrrev_b64 (OP 1), v_add_u32 (OP 2), 8 independent chains
template <int OP>
__global__ void __launch_bounds__(256) k_alu(uint64_t* out, int iters) {
  uint32_t v[8];
  uint64_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) { v[k] = threadIdx.x + k; w[k] = ((uint64_t)v[k] << 40) | blockIdx.x; }
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int k = 0; k < 8; k++) {
        if (OP == 0) asm volatile("v_and_b32 %0, 0x1fffffff, %0" : "+v"(v[k]));
        if (OP == 1) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(w[k]));
        if (OP == 2) asm volatile("v_add_u32 %0, 0x1234, %0" : "+v"(v[k]));
      }
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) s ^= v[k] ^ w[k];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// NP independent products per iteration; V = 0: f29_mul_g, 1: f29_mul_a
template <int V, int NP>
__global__ void __launch_bounds__(256) k_prod(uint32_t* out, int iters) {
  F29<F> a[NP], b;
#pragma unroll
  for (int i = 0; i < 9; i++) b.l[i] = (blockIdx.x * 3 + i * 131) & kM29;
#pragma unroll
  for (int p = 0; p < NP; p++)
#pragma unroll
    for (int i = 0; i < 9; i++) a[p].l[i] = (threadIdx.x * 7 + i * 977 + p) & kM29;
  for (int k = 0; k < iters; k++) {
#pragma unroll
    for (int p = 0; p < NP; p++) a[p] = V == 0 ? f29_mul_g<F>(a[p], b) : f29_mul_a<F>(a[p], b);
  }
  uint32_t s = 0;
#pragma unroll
  for (int p = 0; p < NP; p++)
#pragma unroll
    for (int i = 0; i < 9; i++) s ^= a[p].l[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class T>
double timeit(void (*k)(T*, int), int blocks, void* vbuf, int iters) {
  T* buf = (T*)vbuf;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<<<blocks, 256>>>(buf, 2);
  hipDeviceSynchronize();
  float ms;
  hipEventRecord(e0);
  k<<<blocks, 256>>>(buf, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  void* buf;
  hipMalloc(&buf, 64ull << 20);
  for (int wps : {1, 2, 4, 8}) {
    const int blocks = 256 * wps;
    const double lanes = blocks * 256.0;
    auto rep = [&](const char* name, double ms, double ops) {
      printf("{\"bench\":\"%s\",\"waves_per_simd\":%d,\"ms\":%.4f,\"T_per_s\":%.3f}\n", name, wps, ms, lanes * ops / ms / 1e9);
    };
    const int it = 512;
    rep("mad_1chain", timeit((void (*)(uint64_t*, int))k_mad<1>, blocks, buf, it * 8), it * 8 * 16.0);
    rep("mad_2chain", timeit((void (*)(uint64_t*, int))k_mad<2>, blocks, buf, it * 4), it * 4 * 16.0 * 2);
    rep("mad_4chain", timeit((void (*)(uint64_t*, int))k_mad<4>, blocks, buf, it * 2), it * 2 * 16.0 * 4);
    rep("mad_8chain", timeit((void (*)(uint64_t*, int))k_mad<8>, blocks, buf, it), it * 16.0 * 8);
    rep("and_b32", timeit((void (*)(uint64_t*, int))k_alu<0>, blocks, buf, it), it * 16.0 * 8);
    rep("lshr_b64", timeit((void (*)(uint64_t*, int))k_alu<1>, blocks, buf, it), it * 16.0 * 8);
    rep("add_u32", timeit((void (*)(uint64_t*, int))k_alu<2>, blocks, buf, it), it * 16.0 * 8);
    const int pi = 64;
    rep("f29_mul_g_x1", timeit((void (*)(uint32_t*, int))k_prod<0, 1>, blocks, buf, pi), pi * 1.0 / 1000);
    rep("f29_mul_a_x1", timeit((void (*)(uint32_t*, int))k_prod<1, 1>, blocks, buf, pi), pi * 1.0 / 1000);
    rep("f29_mul_g_x2", timeit((void (*)(uint32_t*, int))k_prod<0, 2>, blocks, buf, pi), pi * 2.0 / 1000);
    rep("f29_mul_a_x2", timeit((void (*)(uint32_t*, int))k_prod<1, 2>, blocks, buf, pi), pi * 2.0 / 1000);
  }
  return 0;
}

// microbench_mad.hip -- issue vs dependency cost of v_mad_u64_u32 in ONE wave
// on gfx950 (is a lone wave's product chain latency- or issue-bound?).
//   chains = 1: every multiply-add depends on the previous one
//   chains = 2 / 4: 2 / 4 independent accumulators, interleaved
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/xpbin/microbench_mad tools/microbench_mad.hip
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define MAD(A, X, Y) asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(A), "=s"(c) : "v"(X), "v"(Y))

template <int CH>
__global__ void __launch_bounds__(64) k_chain(uint64_t* out, uint32_t x, uint32_t y, int iters) {
  uint64_t a0 = threadIdx.x, a1 = 1, a2 = 2, a3 = 3, c;
  const uint32_t xv = x + threadIdx.x, yv = y ^ threadIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {  // 64 multiply-adds per iteration in every variant
      if (CH == 1) {
        MAD(a0, xv, yv); MAD(a0, xv, yv); MAD(a0, xv, yv); MAD(a0, xv, yv);
      } else if (CH == 2) {
        MAD(a0, xv, yv); MAD(a1, xv, yv); MAD(a0, xv, yv); MAD(a1, xv, yv);
      } else {
        MAD(a0, xv, yv); MAD(a1, xv, yv); MAD(a2, xv, yv); MAD(a3, xv, yv);
      }
    }
  }
  out[threadIdx.x] = a0 + a1 + a2 + a3;
}

// 32-bit adds, dependent vs independent, for the same question on cheap ops
template <int CH>
__global__ void __launch_bounds__(64) k_add(uint32_t* out, uint32_t x, int iters) {
  uint32_t a0 = threadIdx.x, a1 = 1, a2 = 2, a3 = 3;
  const uint32_t xv = x + threadIdx.x;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (CH == 1) {
        asm volatile("v_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1\n\tv_add_u32 %0, %0, %1"
                     : "+v"(a0) : "v"(xv));
      } else {
        asm volatile("v_add_u32 %0, %0, %4\n\tv_add_u32 %1, %1, %4\n\tv_add_u32 %2, %2, %4\n\tv_add_u32 %3, %3, %4"
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3) : "v"(xv));
      }
    }
  }
  out[threadIdx.x] = a0 + a1 + a2 + a3;
}

template <class K>
void run(const char* name, K launch, void* buf) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  launch(buf, iters / 100);  // warm-up
  hipDeviceSynchronize();
  hipEventRecord(e0);
  launch(buf, iters);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double ns_per_op = ms * 1e6 / ((double)iters * 64);
  printf("{\"bench\":\"%s\",\"waves\":1,\"ns_per_op\":%.3f,\"cycles_at_2400MHz\":%.2f}\n", name, ns_per_op,
         ns_per_op * 2.4);
}

int main() {
  void* buf;
  hipMalloc(&buf, 1 << 20);
  run("mad64_1chain", [](void* b, int it) { k_chain<1><<<1, 64>>>((uint64_t*)b, 7, 9, it); }, buf);
  run("mad64_2chains", [](void* b, int it) { k_chain<2><<<1, 64>>>((uint64_t*)b, 7, 9, it); }, buf);
  run("mad64_4chains", [](void* b, int it) { k_chain<4><<<1, 64>>>((uint64_t*)b, 7, 9, it); }, buf);
  run("add32_1chain", [](void* b, int it) { k_add<1><<<1, 64>>>((uint32_t*)b, 7, it); }, buf);
  run("add32_4chains", [](void* b, int it) { k_add<4><<<1, 64>>>((uint32_t*)b, 7, it); }, buf);
  return 0;
}

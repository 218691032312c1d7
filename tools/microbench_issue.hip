// microbench_issue.hip -- single-wave issue cost per instruction class on
// MI355X, in the configuration of the accumulator's latency chains (one wave
// of 64 lanes per CU, 256 blocks): a long inline-asm stream of one
// instruction, either 8 independent chains (issue cost) or one dependent
// chain (issue + result latency).  Feeds tools/hw_floor.py (the hardware floor
// of the accumulator's critical path, profiles/r05/hw_floor.json).
// Output: one JSON line per instruction form, ns per instruction per wave.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_issue tools/microbench_issue.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define R8(x) x x x x x x x x
#define R64(x) R8(R8(x))

// 64 instructions per asm statement, kUnroll statements per loop iteration
constexpr int kUnroll = 8;

template <int V>
__global__ void __launch_bounds__(256) k_issue(uint32_t* out, uint64_t* clk, int iters) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = threadIdx.x * 0x9E3779B9u, y = x ^ 0x85EBCA6Bu, z = x + 7u;
  uint32_t w0 = x, w1 = y, w2 = z, w3 = x ^ z, w4 = x + 1, w5 = y + 1, w6 = z + 1, w7 = x + 2;
  uint64_t c;
  const uint64_t t0 = wall_clock64();
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++) {
      if (V == 0)  // v_mad_u64_u32, 8 independent accumulators
        asm volatile(R8("v_mad_u64_u32 %0, %8, %9, %10, %0\n\tv_mad_u64_u32 %1, %8, %9, %10, %1\n\t"
                        "v_mad_u64_u32 %2, %8, %9, %10, %2\n\tv_mad_u64_u32 %3, %8, %9, %10, %3\n\t"
                        "v_mad_u64_u32 %4, %8, %9, %10, %4\n\tv_mad_u64_u32 %5, %8, %9, %10, %5\n\t"
                        "v_mad_u64_u32 %6, %8, %9, %10, %6\n\tv_mad_u64_u32 %7, %8, %9, %10, %7\n\t")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "=&s"(c)
                     : "v"(x), "v"(y));
      if (V == 1)  // v_mad_u64_u32, one dependent chain
        asm volatile(R64("v_mad_u64_u32 %0, %1, %2, %3, %0\n\t") : "+v"(a0), "=&s"(c) : "v"(x), "v"(y));
      if (V == 2)  // v_and_b32, 8 independent
        asm volatile(R8("v_and_b32 %0, %8, %0\n\tv_and_b32 %1, %8, %1\n\tv_and_b32 %2, %8, %2\n\tv_and_b32 %3, %8, %3\n\t"
                        "v_and_b32 %4, %8, %4\n\tv_and_b32 %5, %8, %5\n\tv_and_b32 %6, %8, %6\n\tv_and_b32 %7, %8, %7\n\t")
                     : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(w3), "+v"(w4), "+v"(w5), "+v"(w6), "+v"(w7)
                     : "v"(y));
      if (V == 3)  // v_add_u32, one dependent chain
        asm volatile(R64("v_add_u32 %0, %1, %0\n\t") : "+v"(w0) : "v"(y));
      if (V == 4)  // v_lshrrev_b64, 8 independent
        asm volatile(R8("v_lshrrev_b64 %0, 1, %0\n\tv_lshrrev_b64 %1, 1, %1\n\tv_lshrrev_b64 %2, 1, %2\n\t"
                        "v_lshrrev_b64 %3, 1, %3\n\tv_lshrrev_b64 %4, 1, %4\n\tv_lshrrev_b64 %5, 1, %5\n\t"
                        "v_lshrrev_b64 %6, 1, %6\n\tv_lshrrev_b64 %7, 1, %7\n\t")
                     : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
      if (V == 5)  // v_mov_b32_dpp row_newbcast, 8 independent
        asm volatile(R8("v_mov_b32_dpp %0, %8 row_newbcast:1\n\tv_mov_b32_dpp %1, %8 row_newbcast:2\n\t"
                        "v_mov_b32_dpp %2, %8 row_newbcast:3\n\tv_mov_b32_dpp %3, %8 row_newbcast:4\n\t"
                        "v_mov_b32_dpp %4, %8 row_newbcast:5\n\tv_mov_b32_dpp %5, %8 row_newbcast:6\n\t"
                        "v_mov_b32_dpp %6, %8 row_newbcast:7\n\tv_mov_b32_dpp %7, %8 row_newbcast:8\n\t")
                     : "=&v"(w0), "=&v"(w1), "=&v"(w2), "=&v"(w3), "=&v"(w4), "=&v"(w5), "=&v"(w6), "=&v"(w7)
                     : "v"(y));
      if (V == 6)  // ds_bpermute_b32, one dependent chain (LDS crossbar latency)
        asm volatile(R64("ds_bpermute_b32 %0, %1, %0\n\ts_waitcnt lgkmcnt(0)\n\t") : "+v"(w0) : "v"(z & 252u));
    }
  }
  const uint64_t t1 = wall_clock64();
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7) ^ w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^
                                       w6 ^ w7;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// wpc: waves per CU (one block of wpc waves on each of 256 CUs; wave 0 timed)
template <int V>
void run(const char* name, uint32_t* buf, uint64_t* clk, int iters, int wpc = 1) {
  const int blocks = 256;
  k_issue<V><<<blocks, 64 * wpc>>>(buf, clk, 2);
  k_issue<V><<<blocks, 64 * wpc>>>(buf, clk, iters);
  (void)hipDeviceSynchronize();
  uint64_t h[256];
  (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  double s = 0;
  for (int b = 0; b < blocks; b++) s += (double)h[b];
  const double ns = s / blocks * 10.0 / ((double)iters * kUnroll * 64);  // wall_clock64 at 100 MHz
  if (wpc == 1)
    printf("{\"form\": \"%s\", \"ns_per_instruction\": %.4f}\n", name, ns);
  else
    printf("{\"form\": \"%s\", \"waves_per_cu\": %d, \"ns_per_instruction\": %.4f}\n", name, wpc, ns);
  fflush(stdout);
}

int main() {
  uint32_t* buf;
  uint64_t* clk;
  (void)hipMalloc(&buf, 256 * 256 * 4);
  (void)hipMalloc(&clk, 256 * 8);
  run<0>("v_mad_u64_u32 independent", buf, clk, 2000);
  run<1>("v_mad_u64_u32 dependent", buf, clk, 2000);
  run<2>("v_and_b32 independent", buf, clk, 2000);
  run<3>("v_add_u32 dependent", buf, clk, 2000);
  run<4>("v_lshrrev_b64 independent", buf, clk, 2000);
  run<5>("v_mov_b32_dpp row_newbcast independent", buf, clk, 2000);
  run<6>("ds_bpermute_b32 dependent (with s_waitcnt)", buf, clk, 500);
  // four waves per CU (one per SIMD): does the per-wave issue rate hold?
  run<0>("v_mad_u64_u32 independent", buf, clk, 2000, 4);
  run<2>("v_and_b32 independent", buf, clk, 2000, 4);
  run<5>("v_mov_b32_dpp row_newbcast independent", buf, clk, 2000, 4);
  return 0;
}

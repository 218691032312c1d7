// microbench_slice.hip -- single-wave latency of the row-sliced Montgomery
// product (slice29.hpp) against the one-lane product (fp29.hpp f29_mul_c),
// and their agreement: one wave per block, each of its four rows (sliced) or
// lanes (one-lane) iterating x <- x y; the final x of every chain is compared
// (canonical) between the two forms on the host.
// Output: one JSON line per field: us per product for each form, mismatches.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_slice tools/microbench_slice.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "../halo2-aggregation_amd/csrc/slice29.hpp"
using namespace pm;

template <class F>
__device__ void seed(uint32_t t, F29<F>& x, F29<F>& y) {
  for (int i = 0; i < 9; i++) {
    x.l[i] = (t * 7919u + i * 977u + 12345u) & kM29;
    y.l[i] = (t * 104729u + i * 131u + 777u) & kM29;
  }
  x.l[8] &= 0xfffff;
  y.l[8] &= 0xfffff;
}

// chain id = (blockIdx.x * waves per block + wave) * 4 + row; one or more
// waves per block (a block of W waves puts W chains' waves on one CU)
template <class F>
__global__ void __launch_bounds__(256) k_slice(uint32_t* out, uint64_t* clk, int iters) {
  const uint32_t row = (threadIdx.x >> 4) & 3u, id = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 4 + row;
  F29<F> x0, y0;
  seed<F>(id, x0, y0);
  const SConst<F> k = SConst<F>::make();
  S29<F> x = s29_from<F>(x0), y = s29_from<F>(y0);
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < iters; i++) x = s29_mul<F>(x, y, k);
  const F29<F> r = f29_canon<F>(f29_reduce3<F>(s29_to<F>(s29_norm_exact<F>(x))));
  const uint64_t t1 = wall_clock64() + (r.l[0] & 0u);
  if (s_lane() == 0)
    for (int i = 0; i < 9; i++) out[id * 9 + i] = r.l[i];
  if ((threadIdx.x & 63) == 0) clk[blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)] = t1 - t0;
}

template <class F>
__global__ void __launch_bounds__(64) k_lane(uint32_t* out, uint64_t* clk, int iters) {
  const uint32_t id = blockIdx.x * 64 + threadIdx.x;
  F29<F> x, y;
  seed<F>(id, x, y);
  const uint64_t t0 = wall_clock64();
  for (int i = 0; i < iters; i++) x = f29_mul_c<F>(x, y);
  const F29<F> r = f29_canon<F>(f29_reduce3<F>(x));
  const uint64_t t1 = wall_clock64() + (r.l[0] & 0u);
  for (int i = 0; i < 9; i++) out[id * 9 + i] = r.l[i];
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// inversion latency: one lane per input (bg_inverse on the VALU), one
// wave per input with wave-uniform operands (the compiler keeps the whole
// binary GCD on the scalar unit), or one lane per input with the
// variable-time safegcd (sg_inverse; lanes of a wave run the longest lane's
// loop counts)
template <class F, bool W, bool SG = false>
__global__ void __launch_bounds__(64) k_inv(const uint32_t* in, uint32_t* out, uint64_t* clk, int reps) {
  const uint32_t id = W ? blockIdx.x : blockIdx.x * 64 + threadIdx.x;
  uint32_t y[8], o[8];
  for (int i = 0; i < 8; i++) y[i] = W ? __builtin_amdgcn_readfirstlane(in[id * 8 + i]) : in[id * 8 + i];
  const uint64_t t0 = wall_clock64();
  for (int r = 0; r < reps; r++) {
    if (SG) sg_inverse<F>(y, o);
    else bg_inverse<F>(y, o);
    for (int i = 0; i < 8; i++) y[i] = o[i];
  }
  const uint64_t t1 = wall_clock64() + (o[0] & 0u);
  if (!W || threadIdx.x == 0)
    for (int i = 0; i < 8; i++) out[id * 8 + i] = o[i];
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

// quad-cooperative forms: the 4 lanes of a quad invert the same input
template <class F, bool SG>
__global__ void __launch_bounds__(64) k_invq(const uint32_t* in, uint32_t* out, uint64_t* clk, int reps) {
  const uint32_t id = blockIdx.x * 16 + (threadIdx.x >> 2);
  uint32_t y[8], o[8];
  for (int i = 0; i < 8; i++) y[i] = in[id * 8 + i];
  const uint64_t t0 = wall_clock64();
  for (int r = 0; r < reps; r++) {
    if (SG) sg_inverse_q<F>(y, o);
    else bg_inverse_q<F>(y, o);
    for (int i = 0; i < 8; i++) y[i] = o[i];
  }
  const uint64_t t1 = wall_clock64() + (o[0] & 0u);
  if ((threadIdx.x & 3) == 0)
    for (int i = 0; i < 8; i++) out[id * 8 + i] = o[i];
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <class F>
void run_invq(const char* name) {
  const int n = 256, reps = 20;
  std::vector<uint32_t> h(n * 8);
  uint64_t s = 0x243F6A8885A308D3ull;
  for (auto& w : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    w = (uint32_t)s;
  }
  for (int i = 0; i < n; i++) h[i * 8 + 7] &= 0x0fffffff;
  uint32_t *d_in, *d_a, *d_b;
  uint64_t *c_a, *c_b;
  (void)hipMalloc(&d_in, n * 32);
  (void)hipMalloc(&d_a, n * 32);
  (void)hipMalloc(&d_b, n * 32);
  (void)hipMalloc(&c_a, n * 8);
  (void)hipMalloc(&c_b, n * 8);
  (void)hipMemcpy(d_in, h.data(), n * 32, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) {
    k_invq<F, false><<<n / 16, 64>>>(d_in, d_a, c_a, reps);
    k_invq<F, true><<<n / 16, 64>>>(d_in, d_b, c_b, reps);
  }
  (void)hipDeviceSynchronize();
  std::vector<uint32_t> a(n * 8), b(n * 8);
  std::vector<uint64_t> ca(n / 16), cb(n / 16);
  (void)hipMemcpy(a.data(), d_a, n * 32, hipMemcpyDeviceToHost);
  (void)hipMemcpy(b.data(), d_b, n * 32, hipMemcpyDeviceToHost);
  (void)hipMemcpy(ca.data(), c_a, ca.size() * 8, hipMemcpyDeviceToHost);
  (void)hipMemcpy(cb.data(), c_b, cb.size() * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < n * 8; i++) bad += a[i] != b[i];
  double sa = 0, sb = 0;
  for (auto v : ca) sa += v;
  for (auto v : cb) sb += v;
  printf("{\"field\": \"%s\", \"inv_quad_bgcd_us\": %.3f, \"inv_quad_safegcd_us\": %.3f, \"mismatches\": %d}\n", name,
         sa / ca.size() * 0.01 / reps, sb / cb.size() * 0.01 / reps, bad);
}

template <class F>
void run_inv(const char* name) {
  const int n = 256, reps = 20;
  std::vector<uint32_t> h(n * 8);
  uint64_t s = 0x9E3779B97F4A7C15ull;
  for (auto& w : h) {
    s ^= s << 13; s ^= s >> 7; s ^= s << 17;
    w = (uint32_t)s;
  }
  for (int i = 0; i < n; i++) h[i * 8 + 7] &= 0x0fffffff;  // < 2^252 < p
  uint32_t *d_in, *d_a, *d_b, *d_c;
  uint64_t *c_a, *c_b, *c_c;
  hipMalloc(&d_in, n * 32);
  hipMalloc(&d_a, n * 32);
  hipMalloc(&d_b, n * 32);
  hipMalloc(&d_c, n * 32);
  hipMalloc(&c_a, n * 8);
  hipMalloc(&c_b, n * 8);
  hipMalloc(&c_c, n * 8);
  hipMemcpy(d_in, h.data(), n * 32, hipMemcpyHostToDevice);
  for (int rep = 0; rep < 2; rep++) {
    k_inv<F, false><<<n / 64, 64>>>(d_in, d_a, c_a, reps);
    k_inv<F, true><<<n, 64>>>(d_in, d_b, c_b, reps);
    k_inv<F, false, true><<<n / 64, 64>>>(d_in, d_c, c_c, reps);
  }
  hipDeviceSynchronize();
  std::vector<uint32_t> a(n * 8), b(n * 8), c(n * 8);
  std::vector<uint64_t> ca(n / 64), cb(n), cc(n / 64);
  hipMemcpy(a.data(), d_a, n * 32, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), d_b, n * 32, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), d_c, n * 32, hipMemcpyDeviceToHost);
  hipMemcpy(ca.data(), c_a, ca.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(cb.data(), c_b, cb.size() * 8, hipMemcpyDeviceToHost);
  hipMemcpy(cc.data(), c_c, cc.size() * 8, hipMemcpyDeviceToHost);
  int bad = 0, bad_sg = 0;
  for (int i = 0; i < n * 8; i++) {
    bad += a[i] != b[i];
    bad_sg += a[i] != c[i];
  }
  double sa = 0, sb = 0, sc = 0;
  for (auto v : ca) sa += v;
  for (auto v : cb) sb += v;
  for (auto v : cc) sc += v;
  printf("{\"field\": \"%s\", \"inv_lane_us\": %.3f, \"inv_wave_scalar_us\": %.3f, \"inv_safegcd_lane_us\": %.3f, "
         "\"mismatches\": %d, \"safegcd_mismatches\": %d}\n",
         name, sa / ca.size() * 0.01 / reps, sb / cb.size() * 0.01 / reps, sc / cc.size() * 0.01 / reps, bad, bad_sg);
}

template <class F>
void run(const char* name) {
  const int iters = 2000, blocks = 64;  // 256 sliced chains, 4096 one-lane chains
  uint32_t *d_s, *d_l;
  uint64_t *c_s, *c_l;
  hipMalloc(&d_s, blocks * 4 * 9 * 4);
  hipMalloc(&d_l, blocks * 64 * 9 * 4);
  hipMalloc(&c_s, blocks * 8);
  hipMalloc(&c_l, blocks * 8);
  for (int rep = 0; rep < 2; rep++) {
    k_slice<F><<<blocks, 64>>>(d_s, c_s, iters);
    k_lane<F><<<blocks, 64>>>(d_l, c_l, iters);
  }
  hipDeviceSynchronize();
  std::vector<uint32_t> hs(blocks * 4 * 9), hl(blocks * 64 * 9);
  std::vector<uint64_t> cs(blocks), cl(blocks);
  hipMemcpy(hs.data(), d_s, hs.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(hl.data(), d_l, hl.size() * 4, hipMemcpyDeviceToHost);
  hipMemcpy(cs.data(), c_s, blocks * 8, hipMemcpyDeviceToHost);
  hipMemcpy(cl.data(), c_l, blocks * 8, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int id = 0; id < blocks * 4; id++)
    for (int i = 0; i < 9; i++) bad += hs[id * 9 + i] != hl[id * 9 + i];
  double s = 0, l = 0;
  for (int b = 0; b < blocks; b++) {
    s += cs[b];
    l += cl[b];
  }
  // wall_clock64 runs at 100 MHz
  printf("{\"field\": \"%s\", \"sliced_us_per_mul\": %.4f, \"lane_us_per_mul\": %.4f, \"mismatches\": %d}\n", name,
         s / blocks * 0.01 / iters, l / blocks * 0.01 / iters, bad);
  // the same 256 sliced chains as 2 and 4 waves per block (per CU)
  for (int wpb = 2; wpb <= 4; wpb *= 2) {
    k_slice<F><<<blocks / wpb, 64 * wpb>>>(d_s, c_s, iters);
    k_slice<F><<<blocks / wpb, 64 * wpb>>>(d_s, c_s, iters);
    hipDeviceSynchronize();
    std::vector<uint32_t> h2(blocks * 4 * 9);
    hipMemcpy(h2.data(), d_s, h2.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(cs.data(), c_s, blocks * 8, hipMemcpyDeviceToHost);
    int bad2 = 0;
    for (size_t i = 0; i < h2.size(); i++) bad2 += h2[i] != hs[i];
    double s2 = 0;
    for (int b = 0; b < blocks; b++) s2 += cs[b];
    printf("{\"field\": \"%s\", \"waves_per_cu\": %d, \"sliced_us_per_mul\": %.4f, \"mismatches\": %d}\n", name,
           wpb, s2 / blocks * 0.01 / iters, bad2);
  }
  hipFree(d_s);
  hipFree(d_l);
  hipFree(c_s);
  hipFree(c_l);
}

int main() {
  run<Bn254Fq>("bn254_fq");
  run<PallasFp>("pallas_fp");
  run_inv<Bn254Fq>("bn254_fq");
  run_inv<PallasFp>("pallas_fp");
  run_invq<Bn254Fq>("bn254_fq");
  run_invq<PallasFp>("pallas_fp");
  return 0;
}

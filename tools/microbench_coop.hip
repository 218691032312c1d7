// microbench_coop.hip -- single-wave latency of the radix-2^29 group-law
// chains: one wave per CU (256 blocks of 64 lanes), each lane (or quad)
// iterating a dependent chain.  Compares the quad-cooperative forms of
// coop29.hpp with the one-lane forms of curve29.hpp.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_coop tools/microbench_coop.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include "../halo2-aggregation_amd/csrc/coop29.hpp"
using namespace pm;
using F = Bn254Fq;

namespace pm {
// Wave-uniform f29_inv (measured out, round 3: 66 us per inversion against
// 45 us for the quad VALU form; the scalar unit is no faster per dependent op): the input is read from lane `src` (readfirstlane of
// the packed words after a lane broadcast), so the whole binary GCD runs on
// the scalar unit; every lane receives the inverse.  The wave must be
// converged (all lanes call it with the same src).
template <class P>
__device__ F29<P> f29_inv_s(const F29<P>& a, int src) {
  uint32_t w[8], v[8];
  f29_pack<P>(f29_canon<P>(a), w);
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)w[i], src, 64));
  bg_inverse<P>(w, v);
  return f29_mul_c<P>(f29_unpack<P>(v), f29_const<P>(F29Consts<P>::R783));
}

}  // namespace pm

template <int V>
__global__ void __launch_bounds__(256) k_chain(uint32_t* out, int iters) {
  const uint32_t t = (V == 1 || V == 3 || V == 10) ? (threadIdx.x >> 2) : threadIdx.x;
  F29<F> x, y;
  for (int i = 0; i < 9; i++) { x.l[i] = (t * 7 + i * 977 + blockIdx.x) & kM29; y.l[i] = (t * 3 + i * 131) & kM29; }
  x.l[8] &= 0x3ffff; y.l[8] &= 0x3ffff;
  Jac29<F> j{x, y, f29_const<F>(F29Consts<F>::ONE)};
  Xyzz29<F> a{x, y, f29_const<F>(F29Consts<F>::ONE), f29_const<F>(F29Consts<F>::ONE)};
  Xyzz29<F> b{y, x, f29_const<F>(F29Consts<F>::ONE), f29_const<F>(F29Consts<F>::ONE)};
  for (int k = 0; k < iters; k++) {
    if (V == 0) j = jac29_dbl<F>(j);
    if (V == 1) j = jac29_dbl_q<F>(j);
    if (V == 2) a = xyzz29_add<F>(a, b);
    if (V == 3) a = xyzz29_add_q<F>(a, b);
    if (V == 4) x = f29_mul_c<F>(x, y);
    if (V == 5) x = f29_sqr_c<F>(x);
    if (V == 6) a = xyzz29_dbl<F>(a);
    if (V == 7) a = xyzz29_dbl_q<F>(a);
    if (V == 8) x = f29_inv<F>(f29_add<F>(x, y));
    if (V == 9) x = f29_inv_fermat<F>(f29_add<F>(x, y));
    if (V == 10) x = f29_inv_q<F>(f29_add<F>(x, y));
    if (V == 11) x = f29_inv_s<F>(f29_add<F>(x, y), k & 63);
  }
  uint32_t s = 0;
  for (int i = 0; i < 9; i++) s ^= j.X.l[i] ^ a.X.l[i] ^ x.l[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <int V>
void run(const char* name, uint32_t* buf, int blocks) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int it = V >= 8 ? 20 : 200;
  const int threads = V == 11 && blocks < 0 ? 256 : 64;  // blocks < 0: 4 waves per CU (SALU shared)
  if (blocks < 0) blocks = -blocks;
  k_chain<V><<<blocks, threads>>>(buf, 2);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  k_chain<V><<<blocks, threads>>>(buf, it);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  printf("{\"bench\":\"%s\",\"blocks\":%d,\"threads\":%d,\"us_per_op\":%.3f}\n", name, blocks, threads, ms * 1e3 / it);
}

int main() {
  uint32_t* buf;
  (void)hipMalloc(&buf, 1 << 24);
  for (int blocks : {256}) {
    run<8>("f29_inv_bgcd", buf, blocks);
    run<9>("f29_inv_fermat", buf, blocks);
    run<10>("f29_inv_bgcd_quad", buf, blocks);
    run<11>("f29_inv_bgcd_salu", buf, blocks);
    run<11>("f29_inv_bgcd_salu", buf, -blocks);
  }
  if (getenv("INV_ONLY")) return 0;
  for (int blocks : {256, 1024, 2048, 4096}) {
    run<4>("f29_mul_chain", buf, blocks);
    run<5>("f29_sqr_chain", buf, blocks);
    run<0>("jac29_dbl", buf, blocks);
    run<1>("jac29_dbl_q", buf, blocks);
    run<6>("xyzz29_dbl", buf, blocks);
    run<7>("xyzz29_dbl_q", buf, blocks);
    run<2>("xyzz29_add", buf, blocks);
    run<3>("xyzz29_add_q", buf, blocks);
  }
  return 0;
}

// microbench_chain.hip -- single-wave latency of every dependent step on the
// accumulator's critical path (round 4 latency roofline, bench.py
// `accumulator.roofline`): one wave per CU (256 blocks of 64 lanes), each lane
// (or quad) iterating a dependent chain of ONE step, no memory traffic.
//   f29_mul, f29_sqr          radix-2^29 Montgomery product / square (fp29.hpp)
//   fe_mul                    32-bit FIPS product (k_acc_scalars' field, fp256.hpp)
//   ladder_dbl                jac29_dbl_q_ext: one k_acc_powers step (coop29.hpp)
//   xyzz_add                  xyzz29_add: one k_acc_termadd step per lane
//   xyzz_add_q                xyzz29_add_q: one k_acc_sum butterfly step
//   inv_q                     f29_inv_q: k_acc_sum's affine conversion
//   sqrt_bn254, sqrt_pallas   f29_sqrt: one proof-point decompression (proof_kernels.hpp)
//   b2_compress_q             tr_compress_q: one Blake2b compression of k_transcript
// Output: one JSON line per step, us per step.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_chain tools/microbench_chain.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../halo2-aggregation_amd/csrc/coop29.hpp"
#include "../halo2-aggregation_amd/csrc/proof_kernels.hpp"
#include "../halo2-aggregation_amd/csrc/transcript_kernels.hpp"
using namespace pm;

template <class Cv, int V>
__global__ void __launch_bounds__(64) k_chain(uint32_t* out, int iters, const SqrtTab* tab) {
  using F = typename Cv::Base;
  __shared__ uint32_t s_odd[kSqrtWin * 9 * 64];
  __shared__ uint32_t s_klo[256], s_khi[256], s_kidx[256];
  __shared__ TrBuf buf;
  const uint32_t t = (V == 3 || V == 5 || V == 6 || V == 9) ? (threadIdx.x >> 2) : threadIdx.x;
  F29<F> x, y;
  for (int i = 0; i < 9; i++) {
    x.l[i] = (t * 7 + i * 977 + blockIdx.x) & kM29;
    y.l[i] = (t * 3 + i * 131) & kM29;
  }
  x.l[8] &= 0x3ffff;
  y.l[8] &= 0x3ffff;
  Jac29<F> j{x, y, f29_const<F>(F29Consts<F>::ONE)};
  Xyzz29<F> a{x, y, f29_const<F>(F29Consts<F>::ONE), f29_const<F>(F29Consts<F>::ONE)};
  Xyzz29<F> b{y, x, f29_const<F>(F29Consts<F>::ONE), f29_const<F>(F29Consts<F>::ONE)};
  Fe<F> fa, fb;
  for (int i = 0; i < 8; i++) {
    fa.l[i] = t * 7 + i * 977 + blockIdx.x;
    fb.l[i] = blockIdx.x * 3 + i * 131;
  }
  fa.l[7] &= 0x0fffffff;
  fb.l[7] &= 0x0fffffff;
  if (V == 7) {
    for (uint32_t i = threadIdx.x; i < 256; i += 64) {
      s_klo[i] = tab->key_lo[i];
      s_khi[i] = tab->key_hi[i];
      s_kidx[i] = tab->kidx[i];
    }
    __syncthreads();
  }
  TrLane ln{0x6a09e667f3bcc908ull ^ t, 0xbb67ae8584caa73bull, 0, 0, 0};
  if (V == 9)
    for (uint32_t w = threadIdx.x; w < 32 * kTrSlots; w += 64) buf[w / kTrSlots][w % kTrSlots] = w * 0x9E3779B97F4A7C15ull;
  uint32_t acc = 0;
  for (int k = 0; k < iters; k++) {
    if (V == 0) x = f29_mul_c<F>(x, y);
    if (V == 1) x = f29_sqr_c<F>(x);
    if (V == 2) fa = fe_mul<F>(fa, fb);
    if (V == 3) {
      F29<F> zz, ext;
      j = jac29_dbl_q_ext<F>(j, y, zz, ext);
      j.Y = f29_norm<F>(f29_add<F>(j.Y, f29_zero<F>()));
      acc ^= zz.l[0] ^ ext.l[0];
    }
    if (V == 4) a = xyzz29_add<F>(a, b);
    if (V == 5) a = xyzz29_add_q<F>(a, b);
    if (V == 6) x = f29_inv_q<F>(f29_add<F>(x, y));
    if (V == 7) {
      F29<F> r;
      const bool ok = f29_sqrt<F>(*tab, f29_norm<F>(f29_add<F>(x, y)), r, s_odd + threadIdx.x, 64, s_klo, s_khi,
                                  s_kidx);
      x = ok ? r : f29_sqr_c<F>(x);
    }
    if (V == 9)
      tr_compress_q(ln.h0, ln.h1, TrRingMsg{buf, threadIdx.x >> 2, (uint32_t)k & 15}, threadIdx.x & 3, 128 * (k + 1),
                    false);
  }
  uint32_t s = acc ^ (uint32_t)ln.h0 ^ fa.l[0];
  for (int i = 0; i < 9; i++) s ^= j.X.l[i] ^ a.X.l[i] ^ x.l[i];
  out[blockIdx.x * 64 + threadIdx.x] = s;
}

template <class Cv, int V>
void run(const char* name, uint32_t* buf, const SqrtTab* tab, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int blocks = 256;
  k_chain<Cv, V><<<blocks, 64>>>(buf, 2, tab);
  (void)hipDeviceSynchronize();
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    (void)hipEventRecord(e0);
    k_chain<Cv, V><<<blocks, 64>>>(buf, iters, tab);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    best = ms < best ? ms : best;
  }
  printf("{\"step\":\"%s\",\"blocks\":%d,\"threads\":64,\"iters\":%d,\"us_per_step\":%.4f}\n", name, blocks, iters,
         best * 1e3 / iters);
  fflush(stdout);
}

template <class Cv>
SqrtTab* upload_tab() {
  static SqrtTab h;
  if (sqrt_tab_build<Cv>(h)) {
    printf("{\"error\":\"sqrt_tab_build\"}\n");
    return nullptr;
  }
  SqrtTab* d = nullptr;
  (void)hipMalloc(&d, sizeof(SqrtTab));
  (void)hipMemcpy(d, &h, sizeof(SqrtTab), hipMemcpyHostToDevice);
  return d;
}

namespace pm {
int set_error(int code, const std::string&) { return code; }
}

int main() {
  uint32_t* buf;
  (void)hipMalloc(&buf, 1 << 24);
  SqrtTab* tb = upload_tab<Bn254Curve>();
  SqrtTab* tp = upload_tab<PallasCurve>();
  run<Bn254Curve, 0>("f29_mul", buf, tb, 400);
  run<Bn254Curve, 1>("f29_sqr", buf, tb, 400);
  run<Bn254Curve, 2>("fe_mul", buf, tb, 400);
  run<Bn254Curve, 3>("ladder_dbl", buf, tb, 200);
  run<Bn254Curve, 4>("xyzz_add", buf, tb, 200);
  run<Bn254Curve, 5>("xyzz_add_q", buf, tb, 200);
  run<Bn254Curve, 6>("inv_q", buf, tb, 20);
  run<Bn254Curve, 7>("sqrt_bn254", buf, tb, 6);
  run<PallasCurve, 7>("sqrt_pallas", buf, tp, 6);
  run<Bn254Curve, 9>("b2_compress_q", buf, tb, 200);
  return 0;
}

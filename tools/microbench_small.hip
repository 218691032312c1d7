// microbench_small.hip -- phase timeline of k_small_fused (msm_small.hpp,
// TRACE build): thread 0 of block 0 stamps the real-time clock (100 MHz) at
// every phase boundary: loads + R261 conversion, scalar from Montgomery, GLV
// split, recoding, three doublings, the term's addition, the tree, the
// finish (host store, fences, completion flag).  One JSON line per n.
// Build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/microbench_small tools/microbench_small.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../halo2-aggregation_amd/csrc/msm_small.hpp"
using namespace pm;

namespace pm {
int set_error(int code, const std::string&) { return code; }
}

int main() {
  using Cv = PallasCurve;
  using F = Cv::Base;
  const uint32_t N = 32;
  uint32_t *ds, *db, *done, *flag;
  uint64_t* tr;
  Xyzz<F>* out;
  (void)hipMalloc(&ds, N * 32);
  (void)hipMalloc(&db, N * 64);
  (void)hipMalloc(&done, 64);
  (void)hipMemset(done, 0, 64);
  (void)hipHostMalloc(&flag, 64, hipHostMallocMapped);
  (void)hipHostMalloc(&tr, 16 * 8, hipHostMallocMapped);
  (void)hipHostMalloc(&out, kSmallWin * sizeof(Xyzz<F>), hipHostMallocMapped);
  k_synth_scalars<Cv::Scalar><<<1, 256>>>(0x1234, 0, N, 1, ds);
  k_synth_bases<Cv><<<1, 256>>>(0x5678, 0, N, db);
  (void)hipDeviceSynchronize();
  // the same inputs in pinned mapped host memory (what pm_msm's staging hands the kernel)
  uint32_t *hs, *hb, *dhs, *dhb;
  (void)hipHostMalloc(&hs, N * 32, hipHostMallocMapped);
  (void)hipHostMalloc(&hb, N * 64, hipHostMallocMapped);
  (void)hipMemcpy(hs, ds, N * 32, hipMemcpyDeviceToHost);
  (void)hipMemcpy(hb, db, N * 64, hipMemcpyDeviceToHost);
  (void)hipHostGetDevicePointer((void**)&dhs, hs, 0);
  (void)hipHostGetDevicePointer((void**)&dhb, hb, 0);
  const char* names[] = {"loads_r261", "scalar_redc", "glv_split", "recode", "three_dbl", "add_phi_neg", "tree", "finish"};
  for (int host = 0; host < 2; host++)
  for (uint32_t n : {1u, 2u, 8u, 32u}) {
    SmallGeom g{n, 0u, 0u, 1u, 1u};
    double acc[8] = {0};
    const int reps = 20;
    for (int r = 0; r < reps + 2; r++) {
      k_small_fused<Cv, true><<<dim3(1, kSmallWin), 256>>>(g, host ? dhs : ds, host ? dhb : db, nullptr, nullptr, out,
                                                           done, flag, (uint32_t)r + 1, tr);
      (void)hipDeviceSynchronize();
      if (r >= 2)
        for (int k = 0; k < 8; k++) acc[k] += (double)(tr[k + 1] - tr[k]) * 0.01;  // 100 MHz ticks -> us
    }
    printf("{\"n\":%u,\"inputs\":\"%s\"", n, host ? "host_mapped" : "device");
    double tot = 0;
    for (int k = 0; k < 8; k++) {
      printf(",\"%s_us\":%.2f", names[k], acc[k] / reps);
      tot += acc[k] / reps;
    }
    printf(",\"total_us\":%.2f}\n", tot);
    fflush(stdout);
  }
  return 0;
}

// h2d_overlap.hip -- does a pageable hipMemcpyAsync on one stream overlap a
// kernel on another, and how long does the call block the host?  (Round 6,
// feasibility of a chunked scalar copy for the drop-in pm_msm.)
//   hipcc -O2 --offload-arch=gfx950 -o tools/h2d_overlap tools/h2d_overlap.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

// a VALU-bound busy kernel: every lane runs `iters` dependent multiply-adds
__global__ void k_busy(uint32_t* out, uint32_t iters) {
  uint32_t x = threadIdx.x + blockIdx.x * blockDim.x;
  for (uint32_t i = 0; i < iters; i++) x = x * 1664525u + 1013904223u;
  if (x == 0x12345678u) out[0] = x;  // keep the loop
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t bytes = 32u << 20;
  std::vector<uint8_t> host(bytes);
  std::memset(host.data(), 1, bytes);
  void* d = nullptr;
  uint32_t* o = nullptr;
  CK(hipMalloc(&d, bytes));
  CK(hipMalloc(&o, 4));
  hipStream_t a, c;
  CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&c, hipStreamNonBlocking));
  // calibrate the busy kernel to ~0.5 ms
  uint32_t iters = 20000;
  for (int k = 0; k < 3; k++) {
    k_busy<<<1024, 256, 0, a>>>(o, iters);
    CK(hipStreamSynchronize(a));
  }
  double t0 = now_ms();
  k_busy<<<1024, 256, 0, a>>>(o, iters);
  CK(hipStreamSynchronize(a));
  const double kms = now_ms() - t0;
  for (int rep = 0; rep < 3; rep++) {
    // copies alone: whole, two halves
    for (int parts : {1, 2, 4}) {
      const size_t pb = bytes / parts;
      double s = now_ms(), call = 0;
      for (int p = 0; p < parts; p++) {
        const double c0 = now_ms();
        CK(hipMemcpyAsync((char*)d + p * pb, host.data() + p * pb, pb, hipMemcpyHostToDevice, c));
        call += now_ms() - c0;
      }
      CK(hipStreamSynchronize(c));
      std::printf("{\"test\": \"copy\", \"parts\": %d, \"wall_ms\": %.4f, \"call_ms\": %.4f}\n", parts, now_ms() - s,
                  call);
    }
    // busy kernel on a, then the copy on c: overlap?
    double s = now_ms();
    k_busy<<<1024, 256, 0, a>>>(o, iters);
    const double c0 = now_ms();
    CK(hipMemcpyAsync(d, host.data(), bytes, hipMemcpyHostToDevice, c));
    const double call = now_ms() - c0;
    CK(hipStreamSynchronize(c));
    const double copy_done = now_ms() - s;
    CK(hipStreamSynchronize(a));
    std::printf("{\"test\": \"kernel||copy\", \"kernel_ms\": %.4f, \"copy_call_ms\": %.4f, \"copy_done_ms\": %.4f, "
                "\"wall_ms\": %.4f}\n",
                kms, call, copy_done, now_ms() - s);
  }
  CK(hipFree(d));
  CK(hipFree(o));
  return 0;
}

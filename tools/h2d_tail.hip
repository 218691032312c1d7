// h2d_tail.hip -- a pageable hipMemcpyAsync of (4 MiB + 32 B) at a 4 MiB
// offset: is the 32-byte tail in place for a kernel queued right behind the
// copy on the same stream, and after a synchronize?  (Round 6: the split
// scalar copy lost the last scalar of its second half exactly when that
// scalar's 32 bytes started at a multiple of 4 MiB.)
//   hipcc -O2 --offload-arch=gfx950 -o tools/h2d_tail tools/h2d_tail.hip
#include <hip/hip_runtime.h>

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

// copies 8 words at src into dst (queued behind the H2D copy)
__global__ void k_grab(const uint32_t* src, uint32_t* dst) {
  if (threadIdx.x < 8) dst[threadIdx.x] = src[threadIdx.x];
}

int main() {
  const size_t mib = size_t(1) << 20;
  for (size_t off : {size_t(0), 4 * mib, 6 * mib, 4 * mib + 4096}) {
    for (size_t len : {4 * mib + 32, 2 * mib + 32, 4 * mib + 4096 + 32, 4 * mib}) {
      for (int blocking = 0; blocking < 2; blocking++) {
        const size_t total = off + len;
        std::vector<uint32_t> host(total / 4);
        for (size_t i = 0; i < host.size(); i++) host[i] = (uint32_t)(i * 2654435761u + 1u);
        uint32_t *d = nullptr, *g = nullptr;
        CK(hipMalloc(&d, total));
        CK(hipMalloc(&g, 32));
        CK(hipMemset(d, 0, total));
        CK(hipMemset(g, 0, 32));
        hipStream_t s;
        CK(blocking ? hipStreamCreate(&s) : hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        CK(hipDeviceSynchronize());
        CK(hipMemcpyAsync((char*)d + off, (const char*)host.data() + off, len, hipMemcpyHostToDevice, s));
        k_grab<<<1, 64, 0, s>>>((const uint32_t*)((const char*)d + total - 32), g);
        CK(hipStreamSynchronize(s));
        uint32_t grabbed[8], after[8];
        CK(hipMemcpy(grabbed, g, 32, hipMemcpyDeviceToHost));
        CK(hipMemcpy(after, (const char*)d + total - 32, 32, hipMemcpyDeviceToHost));
        const bool ok_kernel = std::memcmp(grabbed, &host[(total - 32) / 4], 32) == 0;
        const bool ok_after = std::memcmp(after, &host[(total - 32) / 4], 32) == 0;
        std::printf("{\"off\": %zu, \"len\": %zu, \"blocking_stream\": %d, \"tail_seen_by_next_kernel\": %s, "
                    "\"tail_after_sync\": %s}\n",
                    off, len, blocking, ok_kernel ? "true" : "false", ok_after ? "true" : "false");
        CK(hipStreamDestroy(s));
        CK(hipFree(d));
        CK(hipFree(g));
      }
    }
  }
  return 0;
}

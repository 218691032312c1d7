// blake2b.hpp -- BLAKE2b (RFC 7693) compression shared by host and device.
//
// The reference derives every verifier challenge from halo2's Blake2b
// transcript (`Blake2bWrite<_, C, Challenge255<C>>`, used by TranscriptChip,
// /root/reference/src/transcript.rs:13-15,57-60,143) and hashes the pinned
// verifying key with a second personalisation (src/verifier.rs:341-358).
// Both are BLAKE2b-512 with a 16-byte personalisation and no key or salt
// (blake2b_simd `Params::new().hash_length(64).personal(..)`, [3P]).
//
// The device keeps one transcript per lane (transcript_kernels.hpp); the host
// class below serves the one-off VK hash (pm_vk_transcript_repr).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#include "fp256.hpp"

namespace pm {

struct Blake2bIV {
  static constexpr uint64_t v[8] = {0x6a09e667f3bcc908ull, 0xbb67ae8584caa73bull, 0x3c6ef372fe94f82bull,
                                    0xa54ff53a5f1d36f1ull, 0x510e527fade682d1ull, 0x9b05688c2b3e6c1full,
                                    0x1f83d9abfb41bd6bull, 0x5be0cd19137e2179ull};
};

PM_HD uint64_t b2_rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

// Device rotations by the constant amounts BLAKE2b uses: 32 is a half swap,
// 24 / 16 / 63 are two v_alignbit_b32 each (the compiler's default is a
// shift / shift / or sequence per half).
#if defined(__HIP_DEVICE_COMPILE__)
template <int N>
__device__ __forceinline__ uint64_t b2_rot(uint64_t x) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  if (N == 32) return ((uint64_t)lo << 32) | hi;
  if (N < 32) {
    const uint32_t nl = __builtin_amdgcn_alignbit(hi, lo, N), nh = __builtin_amdgcn_alignbit(lo, hi, N);
    return ((uint64_t)nh << 32) | nl;
  }
  const uint32_t nl = __builtin_amdgcn_alignbit(lo, hi, N - 32), nh = __builtin_amdgcn_alignbit(hi, lo, N - 32);
  return ((uint64_t)nh << 32) | nl;
}
#define PM_B2_ROT(x, n) b2_rot<n>(x)
#else
#define PM_B2_ROT(x, n) b2_rotr(x, n)
#endif

#define PM_B2_G(a, b, c, d, x, y)  \
  do {                             \
    a = a + b + (x);               \
    d = PM_B2_ROT(d ^ a, 32);      \
    c = c + d;                     \
    b = PM_B2_ROT(b ^ c, 24);      \
    a = a + b + (y);               \
    d = PM_B2_ROT(d ^ a, 16);      \
    c = c + d;                     \
    b = PM_B2_ROT(b ^ c, 63);      \
  } while (0)

// One round with message permutation sigma = S0..S15 (compile-time indices,
// so the message words stay in registers on the device).
#define PM_B2_ROUND(S0, S1, S2, S3, S4, S5, S6, S7, S8, S9, S10, S11, S12, S13, S14, S15) \
  PM_B2_G(v0, v4, v8, v12, m[S0], m[S1]);                                                \
  PM_B2_G(v1, v5, v9, v13, m[S2], m[S3]);                                                \
  PM_B2_G(v2, v6, v10, v14, m[S4], m[S5]);                                               \
  PM_B2_G(v3, v7, v11, v15, m[S6], m[S7]);                                               \
  PM_B2_G(v0, v5, v10, v15, m[S8], m[S9]);                                               \
  PM_B2_G(v1, v6, v11, v12, m[S10], m[S11]);                                             \
  PM_B2_G(v2, v7, v8, v13, m[S12], m[S13]);                                              \
  PM_B2_G(v3, v4, v9, v14, m[S14], m[S15]);

// F(h, m, t, f) of RFC 7693 §3.2; t < 2^64 (the high counter word stays 0).
PM_HD void blake2b_compress(uint64_t h[8], const uint64_t m[16], uint64_t t, bool last) {
  uint64_t v0 = h[0], v1 = h[1], v2 = h[2], v3 = h[3], v4 = h[4], v5 = h[5], v6 = h[6], v7 = h[7];
  uint64_t v8 = Blake2bIV::v[0], v9 = Blake2bIV::v[1], v10 = Blake2bIV::v[2], v11 = Blake2bIV::v[3];
  uint64_t v12 = Blake2bIV::v[4] ^ t, v13 = Blake2bIV::v[5], v14 = Blake2bIV::v[6], v15 = Blake2bIV::v[7];
  if (last) v14 = ~v14;
  PM_B2_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  PM_B2_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  PM_B2_ROUND(11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4)
  PM_B2_ROUND(7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8)
  PM_B2_ROUND(9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13)
  PM_B2_ROUND(2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9)
  PM_B2_ROUND(12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11)
  PM_B2_ROUND(13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10)
  PM_B2_ROUND(6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5)
  PM_B2_ROUND(10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0)
  PM_B2_ROUND(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15)
  PM_B2_ROUND(14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3)
  h[0] ^= v0 ^ v8;
  h[1] ^= v1 ^ v9;
  h[2] ^= v2 ^ v10;
  h[3] ^= v3 ^ v11;
  h[4] ^= v4 ^ v12;
  h[5] ^= v5 ^ v13;
  h[6] ^= v6 ^ v14;
  h[7] ^= v7 ^ v15;
}
#undef PM_B2_ROUND
#undef PM_B2_G

// Initial chaining value for a 64-byte digest, no key, no salt, 16-byte
// personalisation (RFC 7693 §2.5 parameter block: bytes 48..63).
PM_HD void blake2b_init_personal(uint64_t h[8], const uint8_t personal[16]) {
  for (int i = 0; i < 8; i++) h[i] = Blake2bIV::v[i];
  h[0] ^= 0x01010040ull;  // digest_length 64, key_length 0, fanout 1, depth 1
  uint64_t p0 = 0, p1 = 0;
  for (int i = 0; i < 8; i++) {
    p0 |= (uint64_t)personal[i] << (8 * i);
    p1 |= (uint64_t)personal[8 + i] << (8 * i);
  }
  h[6] ^= p0;
  h[7] ^= p1;
}

// Streaming host hasher with blake2b_simd's buffering: the last block (even
// a full one) stays buffered until finalisation.
struct Blake2bHost {
  uint64_t h[8];
  uint8_t buf[128];
  size_t pos = 0;
  uint64_t t = 0;

  explicit Blake2bHost(const char personal[16]) { blake2b_init_personal(h, (const uint8_t*)personal); }
  void update(const void* data, size_t n) {
    const uint8_t* p = (const uint8_t*)data;
    for (size_t i = 0; i < n; i++) {
      if (pos == 128) {
        uint64_t m[16];
        memcpy(m, buf, 128);
        t += 128;
        blake2b_compress(h, m, t, false);
        pos = 0;
      }
      buf[pos++] = p[i];
    }
  }
  void finalize(uint8_t out[64]) const {
    uint64_t hh[8], m[16];
    memcpy(hh, h, 64);
    uint8_t blk[128];
    memset(blk, 0, 128);
    memcpy(blk, buf, pos);
    memcpy(m, blk, 128);
    blake2b_compress(hh, m, t + pos, true);
    memcpy(out, hh, 64);  // little-endian hosts (x86-64)
  }
};

static constexpr char kTranscriptPersonal[17] = "Halo2-Transcript";  // halo2 transcript.rs [3P]
static constexpr char kVerifyKeyPersonal[17] = "Halo2-Verify-Key";   // src/verifier.rs:343

}  // namespace pm

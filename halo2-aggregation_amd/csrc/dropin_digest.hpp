// dropin_digest.hpp -- keyed content digest of a base set (the drop-in cache key).
//
// pm_msm keeps the base sets it sees resident on the device, keyed by a digest
// of their bytes (halo2 calls best_multiexp against the same params.g /
// g_lagrange over and over: examples/simple-example.rs:606,638-640,702).  A
// forged pair of base sets with equal digests would make the cache return the
// MSM of the wrong bases, so the digest is a universal hash under a secret
// key drawn per context from the OS RNG and never returned to the caller:
//
//   block  b (64 words = 512 B of base bytes, the last one zero-padded):
//          NH_j(b) = sum_i (b[2i] + K[2i+2j]) * (b[2i+1] + K[2i+1+2j]) mod 2^128
//          (NH of UMAC, RFC 4418 / Black et al. 1999, on 64-bit words;
//          j = 0, 1 use the key shifted by two words, Toeplitz style)
//   chunk  c (2^15 points): P_j(c) = Horner over its blocks of NH_j(b) in
//          GF(2^127 - 1) with the secret point kb_j
//   digest D_j = Horner over the chunks of P_j(c) with the secret point kc_j
//
// NH is 2^-64-almost-universal per block and the polynomial layers add
// (blocks per chunk + chunks) / 2^127, so for a key the caller does not know
// two different base sets of the same length collide in both 127-bit halves
// with probability about 2^-128 -- whatever the caller chose.  The chunks
// hash independently on the host pool (one 64x64 -> 128 multiply per 8 bytes,
// mulx with BMI2: ~0.8x the rate of the unkeyed XXH64-style digest it
// replaced, measured on one core).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <random>

namespace pm {

using u128 = unsigned __int128;

struct DigestKey {
  static constexpr int kNhWords = 64;
  uint64_t nh[kNhWords + 2];  // NH key (hash j reads nh[2j .. 2j + 63])
  u128 kb[2], kc[2];          // polynomial points, < 2^127 - 1
};

namespace digest_detail {
constexpr u128 kP127 = (((u128)1) << 127) - 1;

__attribute__((always_inline)) inline u128 fold127(u128 h) {  // h mod 2^127 - 1 for any 128-bit h
  u128 v = (h & kP127) + (h >> 127);
  return v >= kP127 ? v - kP127 : v;
}

// a * b mod 2^127 - 1, a, b < 2^127
__attribute__((always_inline)) inline u128 mulmod127(u128 a, u128 b) {
  const uint64_t a0 = (uint64_t)a, a1 = (uint64_t)(a >> 64), b0 = (uint64_t)b, b1 = (uint64_t)(b >> 64);
  const u128 lo = (u128)a0 * b0, m1 = (u128)a0 * b1, m2 = (u128)a1 * b0, hi = (u128)a1 * b1;
  // x = hi 2^128 + (m1 + m2) 2^64 + lo, and 2^128 = 2, 2^127 = 1 (mod p)
  const u128 mid = m1 + m2;                      // < 2^128 (a1, b1 < 2^63)
  u128 r = fold127(lo);
  r = fold127(r + fold127(hi << 1));             // hi < 2^126: 2 hi < 2^127
  // mid 2^64 = (mid_lo 2^64) + (mid_hi 2^128) with mid_lo, mid_hi < 2^64
  const u128 mlo = (u128)(uint64_t)mid << 64, mhi = (u128)(uint64_t)(mid >> 64) << 1;
  r = fold127(r + fold127(mlo));
  r = fold127(r + mhi);
  return r;
}
}  // namespace digest_detail

inline void digest_key_init(DigestKey& k) {
  std::random_device rd;  // getrandom / /dev/urandom
  auto w64 = [&] { return ((uint64_t)rd() << 32) ^ (uint64_t)rd(); };
  for (auto& w : k.nh) w = w64();
  auto fe = [&] {
    u128 v;
    do v = (((u128)w64() << 64) | w64()) & digest_detail::kP127;
    while (v == digest_detail::kP127 || v == 0);
    return v;
  };
  for (int j = 0; j < 2; j++) {
    k.kb[j] = fe();
    k.kc[j] = fe();
  }
}

// both chunk hashes of nwords 64-bit words (one body, two builds: with BMI2
// the 64 x 64 -> 128 products are mulx, ~1.7x the plain mul / adc form's rate
// on hipcc's host target; digest_chunk dispatches on the CPU)
template <bool BMI2>
__attribute__((always_inline)) inline void digest_chunk_t(const DigestKey& k, const uint64_t* p, size_t nwords, u128 out[2]) {
  using namespace digest_detail;
  constexpr int L = DigestKey::kNhWords;
  u128 acc0 = 1, acc1 = 1;
  for (size_t b = 0; b < nwords; b += L) {
    const size_t m = nwords - b < (size_t)L ? nwords - b : (size_t)L;
    u128 h0 = 0, h1 = 0;
    if (m == (size_t)L) {
      for (int i = 0; i < L; i += 2) {
        const uint64_t x = p[b + i], y = p[b + i + 1];
        h0 += (u128)(x + k.nh[i]) * (uint64_t)(y + k.nh[i + 1]);
        h1 += (u128)(x + k.nh[i + 2]) * (uint64_t)(y + k.nh[i + 3]);
      }
    } else {  // the chunk's last, partial block: zero padded
      for (int i = 0; i < L; i += 2) {
        const uint64_t x = (size_t)i < m ? p[b + i] : 0, y = (size_t)i + 1 < m ? p[b + i + 1] : 0;
        h0 += (u128)(x + k.nh[i]) * (uint64_t)(y + k.nh[i + 1]);
        h1 += (u128)(x + k.nh[i + 2]) * (uint64_t)(y + k.nh[i + 3]);
      }
    }
    acc0 = fold127(mulmod127(acc0, k.kb[0]) + fold127(h0));
    acc1 = fold127(mulmod127(acc1, k.kb[1]) + fold127(h1));
  }
  out[0] = acc0;
  out[1] = acc1;
}
__attribute__((target("bmi2"))) inline void digest_chunk_bmi2(const DigestKey& k, const uint64_t* p, size_t nwords,
                                                              u128 out[2]) {
  digest_chunk_t<true>(k, p, nwords, out);
}
inline void digest_chunk(const DigestKey& k, const uint64_t* p, size_t nwords, u128 out[2]) {
  static const bool bmi2 = __builtin_cpu_supports("bmi2");
  if (bmi2) digest_chunk_bmi2(k, p, nwords, out);
  else digest_chunk_t<false>(k, p, nwords, out);
}

// combine nchunks chunk hashes (2 per chunk) into the two 127-bit digests
inline void digest_combine(const DigestKey& k, const u128* part, size_t nchunks, uint64_t d[4]) {
  using namespace digest_detail;
  u128 a0 = 1, a1 = 1;
  for (size_t c = 0; c < nchunks; c++) {
    a0 = fold127(mulmod127(a0, k.kc[0]) + part[2 * c]);
    a1 = fold127(mulmod127(a1, k.kc[1]) + part[2 * c + 1]);
  }
  d[0] = (uint64_t)a0;
  d[1] = (uint64_t)(a0 >> 64);
  d[2] = (uint64_t)a1;
  d[3] = (uint64_t)(a1 >> 64);
}

}  // namespace pm

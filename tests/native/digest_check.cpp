// Host harness for csrc/dropin_digest.hpp (tests/test_dropin_digest.py).
// Commands on stdin, one per line:
//   mul <a hex> <b hex>           -> a * b mod 2^127 - 1
//   digest <seed> <nwords> <chunkwords> <word seed>
//                                 -> D_0, D_1 (hex) of nwords SplitMix64 words
//                                    under the key derived from <seed>
//   rand                          -> two freshly drawn keys' first NH words
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../halo2-aggregation_amd/csrc/dropin_digest.hpp"

using pm::u128;

static u128 parse128(const char* s) {
  u128 v = 0;
  for (; *s; s++) {
    const char c = *s;
    v = v * 16 + (u128)(c <= '9' ? c - '0' : (c | 32) - 'a' + 10);
  }
  return v;
}
static void print128(u128 v) { std::printf("%016llx%016llx", (unsigned long long)(uint64_t)(v >> 64), (unsigned long long)(uint64_t)v); }

static uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// deterministic key for the parity check (the library draws it from the OS RNG)
static void key_from_seed(pm::DigestKey& k, uint64_t seed) {
  for (auto& w : k.nh) w = splitmix(seed);
  for (int j = 0; j < 2; j++) {
    k.kb[j] = (((u128)splitmix(seed) << 64) | splitmix(seed)) & pm::digest_detail::kP127;
    k.kc[j] = (((u128)splitmix(seed) << 64) | splitmix(seed)) & pm::digest_detail::kP127;
  }
}

int main() {
  char cmd[32];
  while (std::scanf("%31s", cmd) == 1) {
    if (!std::strcmp(cmd, "mul")) {
      char a[64], b[64];
      if (std::scanf("%63s %63s", a, b) != 2) return 1;
      print128(pm::digest_detail::mulmod127(parse128(a), parse128(b)));
      std::printf("\n");
    } else if (!std::strcmp(cmd, "digest")) {
      unsigned long long seed, nwords, chunk, wseed;
      if (std::scanf("%llu %llu %llu %llu", &seed, &nwords, &chunk, &wseed) != 4) return 1;
      pm::DigestKey k;
      key_from_seed(k, seed);
      std::vector<uint64_t> w(nwords);
      uint64_t s = wseed;
      for (auto& x : w) x = splitmix(s);
      const size_t nch = (nwords + chunk - 1) / chunk;
      std::vector<u128> part(2 * nch);
      for (size_t c = 0; c < nch; c++) {
        const size_t lo = c * chunk, hi = std::min<size_t>(nwords, lo + chunk);
        pm::digest_chunk(k, w.data() + lo, hi - lo, &part[2 * c]);
      }
      uint64_t d[4];
      pm::digest_combine(k, part.data(), nch, d);
      std::printf("%016llx%016llx %016llx%016llx\n", (unsigned long long)d[1], (unsigned long long)d[0],
                  (unsigned long long)d[3], (unsigned long long)d[2]);
    } else if (!std::strcmp(cmd, "rand")) {
      pm::DigestKey a, b;
      pm::digest_key_init(a);
      pm::digest_key_init(b);
      std::printf("%016llx %016llx\n", (unsigned long long)a.nh[0], (unsigned long long)b.nh[0]);
    } else {
      return 2;
    }
  }
  return 0;
}

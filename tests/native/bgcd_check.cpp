// Host build of csrc/inv_bgcd.hpp for tests/test_inv_bgcd.py: reads lines
// "<field> <y as 64 hex digits, big endian>" and prints bg_inverse(y),
// sg_inverse(y) (safegcd) and
// fe_inv_bgcd(y) (y read as a Montgomery element) as 64 hex digits each,
// plus fe_inv(y) (Fermat) for the Montgomery form, and fe_redc(y) = y R^-1.
#include <cstdio>
#include <cstring>
#include <string>

#include "../../halo2-aggregation_amd/csrc/inv_bgcd.hpp"

using namespace pm;

static void parse(const char* hex, uint32_t w[8]) {
  for (int k = 0; k < 8; k++) {
    char buf[9];
    memcpy(buf, hex + 8 * (7 - k), 8);
    buf[8] = 0;
    w[k] = (uint32_t)strtoul(buf, nullptr, 16);
  }
}
static void emit(const uint32_t w[8]) {
  for (int k = 7; k >= 0; k--) printf("%08x", w[k]);
}

template <class P>
static void run(const uint32_t y[8]) {
  uint32_t r[8], r2[8];
  bg_inverse<P>(y, r);
  sg_inverse<P>(y, r2);
  emit(r);
  printf(" ");
  emit(r2);
  printf(" ");
  Fe<P> a;
  for (int i = 0; i < 8; i++) a.l[i] = y[i];
  emit(fe_inv_bgcd<P>(a).l);
  printf(" ");
  emit(fe_inv<P>(a).l);
  printf(" ");
  emit(fe_redc<P>(a).l);  // y R^-1 mod p (fe_from_mont)
  printf("\n");
}

int main() {
  char field[32], hex[80];
  while (scanf("%31s %79s", field, hex) == 2) {
    uint32_t y[8];
    parse(hex, y);
    std::string f(field);
    if (f == "PallasFp") run<PallasFp>(y);
    else if (f == "VestaFp") run<VestaFp>(y);
    else if (f == "Bn254Fq") run<Bn254Fq>(y);
    else if (f == "Bn254Fr") run<Bn254Fr>(y);
    else return 2;
  }
  return 0;
}

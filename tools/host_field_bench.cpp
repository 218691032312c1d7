// Host field / curve arithmetic latency (host_ec.hpp): dependent chains of
// Montgomery products, add, sub, Jacobian and XYZZ doublings / additions, on
// Pallas (portable and mulx/adx) and BN254 Fq.  CPU only; one JSON line per
// field and pass.  Build: g++ -O3 -std=c++17 -I halo2-aggregation_amd/csrc
// -o tools/host_field_bench tools/host_field_bench.cpp
#include <chrono>
#include <cstdio>
#include "host_ec.hpp"
using namespace pm;
template <class F, bool ADX>
__attribute__((target("bmi2,adx"))) void run(const char* name) {
  host::E<F> a{{0x1234567, 0x89abcdef, 0x1111, 0x2222}}, b{{0x7654321, 0xfedcba98, 0x3333, 0x1444}};
  const int N = 2000000;
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < N; i++) a = host::mulv<F, ADX>(a, b);
  auto t1 = std::chrono::steady_clock::now();
  host::E<F> c = a;
  for (int i = 0; i < N; i++) c = host::add<F>(c, b);
  auto ta = std::chrono::steady_clock::now();
  for (int i = 0; i < N; i++) c = host::sub<F>(c, a);
  auto tb = std::chrono::steady_clock::now();
  host::Jac<F> p{a, b, c};
  for (int i = 0; i < N / 10; i++) p = host::jdbl<F, ADX>(p);
  auto t2 = std::chrono::steady_clock::now();
  host::Jac<F> q{b, a, b};
  for (int i = 0; i < N / 20; i++) p = host::jadd<F, ADX>(p, q);
  auto t3 = std::chrono::steady_clock::now();
  host::Pt<F> x{a, b, a, b}, y{b, a, b, a};
  for (int i = 0; i < N / 20; i++) x = host::addp<F, ADX>(x, y);
  auto t4 = std::chrono::steady_clock::now();
  for (int i = 0; i < N / 20; i++) x = host::dbl<F, ADX>(x);
  auto t5 = std::chrono::steady_clock::now();
  auto ns = [](auto d, int n) { return std::chrono::duration<double, std::nano>(d).count() / n; };
  printf("{\"field\": \"%s\", \"adx\": %d, \"mul_ns\": %.2f, \"add_ns\": %.2f, \"sub_ns\": %.2f, \"jdbl_ns\": %.1f, "
         "\"jadd_ns\": %.1f, \"xyzz_add_ns\": %.1f, \"xyzz_dbl_ns\": %.1f, \"sink\": %lu}\n",
         name, ADX, ns(t1 - t0, N), ns(ta - t1, N), ns(tb - ta, N), ns(t2 - tb, N / 10), ns(t3 - t2, N / 20),
         ns(t4 - t3, N / 20), ns(t5 - t4, N / 20), (unsigned long)(a.v[0] ^ p.X.v[0] ^ x.X.v[0] ^ c.v[1]));
}
int main() {
  for (int r = 0; r < 2; r++) {
    run<PallasFp, false>("pallas");
    run<PallasFp, true>("pallas");
    run<Bn254Fq, true>("bn254");
  }
}

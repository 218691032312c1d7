// Host-side C++ of the product under AddressSanitizer + UBSan (SURVEY §5
// "race / memory error detection" for the CPU path): `make -C
// halo2-aggregation_amd asan` builds this with g++ -fsanitize=address,undefined
// -fno-sanitize-recover=all and runs it; tests/test_asan.py drives it.
//
// Covers the host code the library runs around the kernels:
//   * host_ec.hpp   the MSM's host Horner tail: 4 x u64 Montgomery products
//                   (portable and mulx/adx), XYZZ doubling / addition, the
//                   device-layout conversions, a Horner over sorted terms
//                   like msm_tail (engine.hpp);
//   * inv_bgcd.hpp  the binary-GCD inversion (host build of the PM_HD code);
//   * blake2b.hpp   the host Blake2b (pm_vk_transcript_repr), RFC 7693 KAT
//                   and personalised / multi-block streaming;
//   * accum_plan.hpp the accumulator's shape validation and query plan on
//                   valid shapes and on malformed ones (out-of-range query
//                   indices, unterminated or overflowing expression code, null
//                   arrays), which must be rejected without reading out of
//                   bounds.
// Exit status 0 = every check passed (a sanitizer report aborts first).
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <utility>
#include <vector>

#include "../../halo2-aggregation_amd/csrc/accum_plan.hpp"
#include "../../halo2-aggregation_amd/csrc/blake2b.hpp"
#include "../../halo2-aggregation_amd/csrc/host_ec.hpp"

using namespace pm;

static int g_fail = 0;
#define CHECK(c)                                                  \
  do {                                                            \
    if (!(c)) {                                                   \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                   \
    }                                                             \
  } while (0)

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint64_t rnd() {
  g_rng ^= g_rng << 13;
  g_rng ^= g_rng >> 7;
  g_rng ^= g_rng << 17;
  return g_rng;
}

template <class P>
static host::E<P> rnd_fe() {
  host::E<P> e;
  for (int i = 0; i < 4; i++) e.v[i] = rnd();
  e.v[3] %= host::F64<P>::mod(3);  // below p
  return e;
}

template <class P>
static host::E<P> from_fe(const Fe<P>& f) {
  host::E<P> e;
  for (int k = 0; k < 4; k++) e.v[k] = (uint64_t)f.l[2 * k] | ((uint64_t)f.l[2 * k + 1] << 32);
  return e;
}

// the curve generators (Montgomery): Pallas / Vesta (-1, 2), BN254 (1, 2)
template <class P>
static host::Pt<P> generator(bool minus_one) {
  const Fe<P> one = fe_one<P>();
  const Fe<P> x = minus_one ? fe_sub<P>(fe_zero<P>(), one) : one;
  return host::Pt<P>{from_fe<P>(x), from_fe<P>(fe_add<P>(one, one)), from_fe<P>(one), from_fe<P>(one)};
}

template <class P>
static Fe<P> to_fe(const host::E<P>& e) {
  Fe<P> f;
  for (int k = 0; k < 4; k++) {
    f.l[2 * k] = (uint32_t)e.v[k];
    f.l[2 * k + 1] = (uint32_t)(e.v[k] >> 32);
  }
  return f;
}

// host 64-bit Montgomery == the 32-bit library product; inversion round trip
template <class P>
static void field_checks(int n) {
  // the asm add / sub (host_ec.hpp) against the 32-bit library, at the edges
  // (0, 1, p - 1, p - 2) and on random canonical values
  host::E<P> pm1, pm2, zero, one;
  for (int k = 0; k < 4; k++) pm1.v[k] = host::F64<P>::mod(k), zero.v[k] = 0, one.v[k] = 0;
  pm1.v[0] -= 1;
  pm2 = pm1;
  pm2.v[0] -= 1;
  one.v[0] = 1;
  const host::E<P> edge[4] = {zero, one, pm1, pm2};
  for (int i = 0; i < 16 + n; i++) {
    const host::E<P> a = i < 16 ? edge[i & 3] : rnd_fe<P>(), b = i < 16 ? edge[i >> 2] : rnd_fe<P>();
    CHECK(std::memcmp(to_fe<P>(host::add<P>(a, b)).l, fe_add<P>(to_fe<P>(a), to_fe<P>(b)).l, 32) == 0);
    CHECK(std::memcmp(to_fe<P>(host::sub<P>(a, b)).l, fe_sub<P>(to_fe<P>(a), to_fe<P>(b)).l, 32) == 0);
  }
  for (int i = 0; i < n; i++) {
    const host::E<P> a = rnd_fe<P>(), b = rnd_fe<P>();
    const host::E<P> x = host::mul<P>(a, b);
    CHECK(std::memcmp(to_fe<P>(x).l, fe_mul<P>(to_fe<P>(a), to_fe<P>(b)).l, 32) == 0);
    if (host_has_bmi2()) {
      const host::E<P> y = host::mul_adx<P>(a, b);
      CHECK(std::memcmp(x.v, y.v, 32) == 0);
    }
    const Fe<P> fa = to_fe<P>(a);
    if (!fe_is_zero<P>(fa)) {
      const Fe<P> inv = fe_inv_bgcd<P>(fa);
      CHECK(std::memcmp(fe_mul<P>(fa, inv).l, fe_one<P>().l, 32) == 0);
    }
  }
}

// a Horner over terms sorted by descending position, as msm_tail runs it,
// equals adding the terms' 2^q multiples directly
template <class P>
static void horner_checks(bool minus_one) {
  using host::Pt;
  // terms: multiples of the generator G in the device layout
  const Pt<P> G = generator<P>(minus_one);
  const int nq = 40;
  std::vector<Xyzz<P>> dev(nq);
  std::vector<std::pair<int, int>> terms;
  Pt<P> cur = G;
  for (int i = 0; i < nq; i++) {
    dev[i] = host::to_dev<P>(cur);
    const Pt<P> back = host::from_dev<P>(dev[i]);
    CHECK(std::memcmp(&back, &cur, sizeof(cur)) == 0);
    terms.emplace_back((int)(rnd() % 70), i);
    cur = host::addp<P>(cur, G);
  }
  dev.push_back(host::to_dev<P>(host::inf<P>()));  // an identity term
  terms.emplace_back(3, nq);
  std::sort(terms.begin(), terms.end(), [](const std::pair<int, int>& a, const std::pair<int, int>& b) {
    return a.first > b.first || (a.first == b.first && a.second < b.second);
  });
  Pt<P> acc = host::inf<P>();
  size_t ti = 0;
  for (int q = terms.front().first; q >= 0; q--) {
    acc = host::dbl<P>(acc);
    for (; ti < terms.size() && terms[ti].first == q; ti++) acc = host::addp<P>(acc, host::from_dev<P>(dev[terms[ti].second]));
  }
  CHECK(ti == terms.size());
  // direct: sum_t 2^{q_t} term_t
  Pt<P> ref = host::inf<P>();
  for (const auto& t : terms) {
    Pt<P> v = host::from_dev<P>(dev[t.second]);
    for (int k = 0; k < t.first; k++) v = host::dbl<P>(v);
    ref = host::addp<P>(ref, v);
  }
  const Xyzz<P> a = host::to_dev<P>(acc), r = host::to_dev<P>(ref);
  // compare projectively: X1 ZZ2 == X2 ZZ1 and Y1 ZZZ2 == Y2 ZZZ1
  CHECK(std::memcmp(fe_mul<P>(a.X, r.ZZ).l, fe_mul<P>(r.X, a.ZZ).l, 32) == 0);
  CHECK(std::memcmp(fe_mul<P>(a.Y, r.ZZZ).l, fe_mul<P>(r.Y, a.ZZZ).l, 32) == 0);
  if (host_has_bmi2()) {
    const Pt<P> b = host::addp<P, true>(host::dbl<P, true>(G), G);
    const Pt<P> c = host::addp<P, false>(host::dbl<P, false>(G), G);
    CHECK(std::memcmp(&b, &c, sizeof(b)) == 0);
  }
}

static void blake2b_checks() {
  // RFC 7693 Appendix A: BLAKE2b-512("abc")
  static const uint8_t abc[64] = {
      0xBA, 0x80, 0xA5, 0x3F, 0x98, 0x1C, 0x4D, 0x0D, 0x6A, 0x27, 0x97, 0xB6, 0x9F, 0x12, 0xF6, 0xE9,
      0x4C, 0x21, 0x2F, 0x14, 0x68, 0x5A, 0xC4, 0xB7, 0x4B, 0x12, 0xBB, 0x6F, 0xDB, 0xFF, 0xA2, 0xD1,
      0x7D, 0x87, 0xC5, 0x39, 0x2A, 0xAB, 0x79, 0x2D, 0xC2, 0x52, 0xD5, 0xDE, 0x45, 0x33, 0xCC, 0x95,
      0x18, 0xD3, 0x8A, 0xA8, 0xDB, 0xF1, 0x92, 0x5A, 0xB9, 0x23, 0x86, 0xED, 0xD4, 0x00, 0x99, 0x23};
  const char zero[16] = {0};
  Blake2bHost h(zero);
  h.update("abc", 3);
  uint8_t d[64];
  h.finalize(d);
  CHECK(std::memcmp(d, abc, 64) == 0);
  // streaming: one update == byte-wise updates, across block boundaries
  std::vector<uint8_t> msg(1000);
  for (auto& b : msg) b = (uint8_t)rnd();
  for (size_t len : {0ul, 1ul, 127ul, 128ul, 129ul, 256ul, 1000ul}) {
    Blake2bHost a(kTranscriptPersonal), b(kTranscriptPersonal);
    a.update(msg.data(), len);
    for (size_t i = 0; i < len; i++) b.update(&msg[i], 1);
    uint8_t da[64], db[64];
    a.finalize(da);
    b.finalize(db);
    CHECK(std::memcmp(da, db, 64) == 0);
  }
}

// a small valid shape (2 advice, 1 fixed, 1 instance, 1 lookup, 3 perm columns)
struct ShapeBuf {
  pm_query iq[1] = {{0, 0}};
  pm_query aq[3] = {{0, 0}, {1, 0}, {0, 1}};
  pm_query fq[1] = {{0, 0}};
  pm_perm_column pc[3] = {{PM_COL_ADVICE, 0}, {PM_COL_ADVICE, 1}, {PM_COL_FIXED, 0}};
  // a0 * f0 - a1 + a0(rot 1) ; lookup input a0, table f0
  uint32_t gate[8] = {PM_EXPR_ADVICE | 0 << 8, PM_EXPR_FIXED | 0 << 8, PM_EXPR_PROD, PM_EXPR_ADVICE | 1 << 8,
                      PM_EXPR_NEG,           PM_EXPR_SUM,           PM_EXPR_ADVICE | 2 << 8, PM_EXPR_SUM};
  uint32_t gate_end[9];
  uint32_t lkin[2] = {PM_EXPR_ADVICE | 0 << 8, PM_EXPR_END};
  uint32_t lktab[2] = {PM_EXPR_FIXED | 0 << 8, PM_EXPR_END};
  uint64_t consts[4] = {1, 0, 0, 0};
  uint64_t fixed_c[8] = {0};
  uint64_t sigma_c[24] = {0};
  pm_proof_shape s{};
  ShapeBuf() {
    std::memcpy(gate_end, gate, sizeof(gate));
    gate_end[8] = PM_EXPR_END;
    s.log_n = 9;
    s.blinding_factors = 5;
    s.num_instance_columns = 1;
    s.num_advice_columns = 2;
    s.num_fixed_columns = 1;
    s.num_lookups = 1;
    s.perm_chunk_len = 2;
    s.quotient_degree = 3;
    s.n_instance_queries = 1;
    s.n_advice_queries = 3;
    s.n_fixed_queries = 1;
    s.n_perm_columns = 3;
    s.instance_queries = iq;
    s.advice_queries = aq;
    s.fixed_queries = fq;
    s.perm_columns = pc;
    s.gate_code = gate_end;
    s.gate_code_len = 9;
    s.lookup_input_code = lkin;
    s.lookup_input_code_len = 2;
    s.lookup_table_code = lktab;
    s.lookup_table_code_len = 2;
    s.constants = consts;
    s.n_constants = 1;
    s.fixed_commitments = fixed_c;
    s.sigma_commitments = sigma_c;
  }
};

static void plan_checks() {
  std::vector<AccQuery> q;
  AccLayout L;
  {
    ShapeBuf b;
    int ng = 0;
    const std::string e = acc_validate(&b.s, q, L, &ng);
    CHECK(e.empty());
    CHECK(ng == 1);
    CHECK(L.nsets >= 2);  // rotations 0 and 1 (and -1 from the permutation / lookup queries)
  }
  struct Bad {
    const char* what;
    void (*mutate)(ShapeBuf&);
  };
  const Bad bad[] = {
      {"advice query index past the columns", [](ShapeBuf& b) { b.aq[1].column = 7; }},
      {"gate code reads a missing advice query", [](ShapeBuf& b) { b.gate_end[3] = PM_EXPR_ADVICE | 9 << 8; }},
      {"gate code without END", [](ShapeBuf& b) { b.s.gate_code_len = 8; }},
      {"expression stack underflow", [](ShapeBuf& b) { b.gate_end[0] = PM_EXPR_SUM; }},
      {"constant index past the table", [](ShapeBuf& b) { b.lkin[0] = PM_EXPR_CONST | 5 << 8; }},
      {"lookup table code truncated", [](ShapeBuf& b) { b.s.lookup_table_code_len = 1; }},
      {"unknown opcode", [](ShapeBuf& b) { b.gate_end[2] = 99; }},
      {"null advice queries", [](ShapeBuf& b) { b.s.advice_queries = nullptr; }},
      {"null sigma commitments", [](ShapeBuf& b) { b.s.sigma_commitments = nullptr; }},
      {"perm column query past the queries", [](ShapeBuf& b) { b.pc[2].query_index = 4; }},
      {"log_n zero", [](ShapeBuf& b) { b.s.log_n = 0; }},
      {"quotient degree zero", [](ShapeBuf& b) { b.s.quotient_degree = 0; }},
  };
  for (const Bad& x : bad) {
    ShapeBuf b;
    x.mutate(b);
    q.clear();
    const std::string e = acc_validate(&b.s, q, L, nullptr);
    if (e.empty()) std::fprintf(stderr, "FAIL: accepted malformed shape: %s\n", x.what);
    g_fail += e.empty();
  }
  CHECK(!acc_validate(nullptr, q, L, nullptr).empty());
}

int main() {
  field_checks<PallasFp>(2000);
  field_checks<VestaFp>(2000);
  field_checks<Bn254Fq>(2000);
  horner_checks<PallasFp>(true);
  horner_checks<VestaFp>(true);
  horner_checks<Bn254Fq>(false);
  blake2b_checks();
  plan_checks();
  if (g_fail) {
    std::fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  std::printf("host_asan: all checks passed\n");
  return 0;
}

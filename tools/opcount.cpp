// Op counter + CPU run of the engine's own device algorithms (drand_amd/csrc/*.h compiled for the host
// with -DBLS_HOST). Counts Montgomery multiplications (fp_mul_u12 calls; 288 32x32->64 limb products
// each: 144 for a*b + 144 for m*p in CIOS) per pipeline stage for ONE chained beacon, and checks that
// the beacon verifies. The counts are the algorithmic work figures used for bench.py's roofline
// (DESIGN.md §Roofline). Build + run: make -C tools opcount && tools/opcount <pk48hex> <round> <prevhex> <sighex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../drand_amd/csrc/pairing.h"
#include "../drand_amd/csrc/hash.h"
#include "../drand_amd/csrc/tri.h"

namespace bls {
unsigned long long g_fp_mul_count = 0;
}
using namespace bls;

static std::vector<uint8_t> unhex(const char* s) {
  std::vector<uint8_t> v;
  size_t n = strlen(s);
  for (size_t i = 0; i + 1 < n; i += 2) {
    unsigned x;
    sscanf(s + i, "%2x", &x);
    v.push_back((uint8_t)x);
  }
  return v;
}

static void print_fp(const fp& a) {
  fp r = fp_from_mont(a);
  printf("\"");
  for (int i = 11; i >= 0; i--) printf("%08x", r.l[i]);
  printf("\"");
}

// hash <msghex>: KyberG2.Hash of an arbitrary message (xmd_b0_bytes path), affine raw coordinates
static int cmd_hash(const char* msghex) {
  auto msg = unhex(msghex);
  uint32_t b0[8];
  xmd_b0_bytes(b0, msg.data(), (uint32_t)msg.size(), DST);
  fp2 u0, u1;
  xmd_tail_to_field(b0, u0, u1);
  g2a h = g2_to_aff(hash_field_to_g2(u0, u1));
  printf("{\"x\": [");
  print_fp(h.x.c0);
  printf(", ");
  print_fp(h.x.c1);
  printf("], \"y\": [");
  print_fp(h.y.c0);
  printf(", ");
  print_fp(h.y.c1);
  printf("]}\n");
  return 0;
}

// fp_inv (binary GCD) against a^(p-2) on n seeded inputs in [0, 2p) plus edge values; prints the
// number of mismatches or out-of-range results as JSON
static int cmd_invfuzz(unsigned long n) {
  using namespace bls;
  unsigned long long s = 0x9e3779b97f4a7c15ull;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)(s >> 11);
  };
  // structured inputs (the shapes that stress the 64-bit approximations: long runs of equal top bits,
  // values just around p and its halvings): 2^k, 2^k - 1, p - 2^k, (p + 1) / 2^k, (p - 1) / 2^k,
  // p +- d and 2p - d for small d
  std::vector<fp> st;
  auto pow2 = [](int k) {
    fp r = {};
    if (k < 384) r.l[k / 32] = 1u << (k % 32);
    return r;
  };
  auto sub = [](const fp& a, const fp& b) {
    fp r;
    unsigned br = 0;
    for (int i = 0; i < 12; i++) r.l[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
    return r;
  };
  auto shr = [](fp a, int k) {
    for (; k > 0; k--) {
      for (int i = 0; i < 11; i++) a.l[i] = (a.l[i] >> 1) | (a.l[i + 1] << 31);
      a.l[11] >>= 1;
    }
    return a;
  };
  fp P, P1, Pm1, one = pow2(0);
  for (int i = 0; i < 12; i++) P.l[i] = P_RAW[i];
  Pm1 = sub(P, one);
  P1 = sub(P, sub(pow2(0), pow2(1)));  // p + 1 (p - (1 - 2) wraps to p + 1)
  for (int k = 0; k <= 381; k++) {
    st.push_back(pow2(k));
    st.push_back(sub(pow2(k), one));
    if (k < 381) st.push_back(sub(P, pow2(k)));
    st.push_back(shr(P1, k));
    st.push_back(shr(Pm1, k));
  }
  for (uint32_t d = 1; d < 64; d++) {
    fp dd = {};
    dd.l[0] = d;
    st.push_back(sub(P, dd));
    fp p2;
    for (int i = 0; i < 12; i++) p2.l[i] = P2_RAW[i];
    st.push_back(sub(p2, dd));
    st.push_back(sub(P, sub(fp{}, dd)));  // p + d
  }
  unsigned long bad = 0, unconverged = 0;
  const unsigned long total = n + st.size();
  for (unsigned long t = 0; t < total; t++) {
    fp x;
    for (int i = 0; i < 12; i++) x.l[i] = next();
    x.l[11] &= 0x1fffffffu;
    if (t < 6) {
      for (int i = 0; i < 12; i++) x.l[i] = (t == 2 || t == 3 || t == 5) ? P_RAW[i] : (t == 4 ? P2_RAW[i] : 0u);
      if (t == 1) x.l[0] = 1;
      if (t == 3) x.l[0] -= 1;  // p - 1
      if (t == 4) x.l[0] -= 1;  // 2p - 1
      if (t == 5) x.l[0] += 1;  // p + 1
    } else if (t >= n) {
      x = st[t - n];
    }
    uint32_t d[12];
    unsigned br = 0;
    for (int i = 0; i < 12; i++) d[i] = __builtin_subc(x.l[i], P2_RAW[i], br, &br);
    if (!br) for (int i = 0; i < 12; i++) x.l[i] = d[i];  // into [0, 2p)
    bool conv;
    const fp a = fp_from_u12(fp_inv_bingcd_raw(fp_to_u12(x), conv));  // the GCD alone, no fallback
    const fp b = fp_from_u12(fp_pow_p_minus_2(fp_to_u12(x)));
    br = 0;
    for (int i = 0; i < 12; i++) (void)__builtin_subc(a.l[i], P2_RAW[i], br, &br);
    bad += !fp_eq(a, b) || !br;
    unconverged += !conv;
  }
  printf("{\"inputs\": %lu, \"structured\": %zu, \"bad\": %lu, \"unconverged\": %lu}\n", total, st.size(), bad,
         unconverged);
  return bad != 0 || unconverged != 0;
}

// The square-root exponentiation (4-bit window, radix-2^28 running value) against the generic fixed-
// window one, and the Fp2 square (radix-2^28 sums) against Fp products, on random inputs including
// lazy sums (< 4p) as the callers pass them. Prints the mismatch count.
static int cmd_powfuzz(unsigned long n) {
  using namespace bls;
  unsigned long long s = 0x2545f4914f6cdd1dull;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)(s >> 11);
  };
  auto rnd2p = [&]() {  // a value < 2^381 < 2p (2p's top word is 0x340223d4)
    fp x;
    for (int i = 0; i < 12; i++) x.l[i] = next();
    x.l[11] &= 0x1fffffffu;
    return x;
  };
  unsigned long bad_pow = 0, bad_sqr = 0, bad_mul = 0, bad_fp4 = 0;
  for (unsigned long t = 0; t < n; t++) {
    fp x = rnd2p();
    if (t == 0) x = fp_zero();
    if (t == 1) x = fp_one();
    const fp w = fp_from_u12(fp_pow_p_minus_3_div_4(fp_to_u12(x)));
    const fp ref = fp_pow_words<12>(x, EXP_P_MINUS_3_DIV_4);
    bad_pow += !fp_eq(w, ref);
    // Fp2 square of a reduced value and of a lazy sum
    const fp2 a = {rnd2p(), rnd2p()}, b = {rnd2p(), rnd2p()};
    for (int lazy = 0; lazy < 2; lazy++) {
      const fp2 in = lazy ? fp2_add_lazy(a, b) : a;
      const fp2 red = lazy ? fp2_add(a, b) : a;
      const fp2 got = fp2_sqr(in);
      const fp2 want = {fp_mul(fp_add(red.c0, red.c1), fp_sub(red.c0, red.c1)), fp_dbl(fp_mul(red.c0, red.c1))};
      bad_sqr += !fp2_eq(got, want);
    }
    // Fp2 product (fp.h: three products per column) on operands of every lazy level up to < 8p,
    // against the two-term dot-product body and Fp products; the result must also be < 2p
    auto lvl = [&](int l) {
      fp v = rnd2p();
      if (l >= 1) v = fp_add_lazy(v, rnd2p());
      if (l >= 2) v = fp_add_lazy(v, fp_add_lazy(rnd2p(), rnd2p()));
      if (l == 3) {  // the largest 12-word value below 8p
        for (int i = 0; i < 12; i++) v.l[i] = P2_RAW[i];
        v = fp_add_lazy(fp_add_lazy(v, v), fp_add_lazy(v, v));
        v.l[0] -= 1;
      }
      return v;
    };
    for (int l = 0; l < 16; l++) {
      const fp2 x = {lvl(l & 3), lvl((l >> 2) & 3)}, y = {lvl((l + 1) & 3), lvl((l >> 1) & 3)};
      const u24 k = fp2_mul_body_kara(fp2_to_u24(x), fp_to_u12(y.c0), fp_to_u12(y.c1));
      uint32_t x0[14], x1[14], y0[14], y1[14], yn[14];
      fp_split28(fp_to_u12(x.c0), x0);
      fp_split28(fp_to_u12(x.c1), x1);
      fp_split28(fp_to_u12(y.c0), y0);
      fp_split28(fp_to_u12(y.c1), y1);
      fp_neg28(y1, yn);
      const fp2 d = {fp_from_u12(fp_mont_dot<true>(x0, y0, x1, yn)), fp_from_u12(fp_mont_dot<true>(x0, y1, x1, y0))};
      const fp2 got = fp2_from_u24(k);
      bool in_range = true;
      for (const fp* c : {&got.c0, &got.c1}) {
        unsigned br = 0;
        for (int i = 0; i < 12; i++) (void)__builtin_subc(c->l[i], P2_RAW[i], br, &br);
        in_range = in_range && br;
      }
      bad_mul += !fp2_eq(got, d) || !in_range;
    }
    // the cyclotomic squaring's Fp4 square (tri.h fp4_sqr_k7: seven product columns, signed Y.a)
    // against Fp2 squares and products, on reduced inputs including 0, p - 1 and 2p - 1 limbs
    {
      fp4 x = {{rnd2p(), rnd2p()}, {rnd2p(), rnd2p()}};
      if (t % 7 == 1) x.a.c0 = fp_zero();
      if (t % 7 == 2) for (int i = 0; i < 12; i++) x.b.c1.l[i] = P2_RAW[i] - (i == 0);
      if (t % 7 == 3) for (int i = 0; i < 12; i++) x.a.c1.l[i] = P2_RAW[i] - (i == 0), x.b.c0.l[i] = 0;
      if (t % 7 == 4) x.a = fp2_zero();
      const fp4 y = fp4_sqr_k7(x);
      const fp2 want_a = fp2_add(fp2_sqr(x.a), fp2_mul_xi(fp2_sqr(x.b)));
      const fp2 want_b = fp2_dbl(fp2_mul(x.a, x.b));
      bool in_range = true;
      for (const fp* c : {&y.a.c0, &y.a.c1, &y.b.c0, &y.b.c1}) {
        unsigned br = 0;
        for (int i = 0; i < 12; i++) (void)__builtin_subc(c->l[i], P2_RAW[i], br, &br);
        in_range = in_range && br;
      }
      bad_fp4 += !fp2_eq(y.a, want_a) || !fp2_eq(y.b, want_b) || !in_range;
      // the interleaved Fp2 additive operations (tower.h) against the per-component fp.h ones
      const fp2 u = {rnd2p(), rnd2p()}, v = x.b;
      for (int sub = 0; sub < 2; sub++) {
        const fp2 g = fp2_addsub(u, v, sub != 0), w = sub ? fp2_sub(u, v) : fp2_add(u, v);
        const fp2 wr = sub ? fp2{fp_sub(u.c0, v.c0), fp_sub(u.c1, v.c1)} : fp2{fp_add(u.c0, v.c0), fp_add(u.c1, v.c1)};
        bad_fp4 += !fp2_eq(g, wr) || !fp2_eq(w, wr) || memcmp(&g, &wr, sizeof g) != 0 || memcmp(&w, &wr, sizeof w) != 0;
      }
      const fp2 xi = fp2_mul_xi(u), xr = {fp_sub(u.c0, u.c1), fp_add(u.c0, u.c1)};
      bad_fp4 += memcmp(&xi, &xr, sizeof xi) != 0;
      const fp2 ng = fp2_neg(u), nr = {fp_neg(u.c0), fp_neg(u.c1)};
      bad_fp4 += memcmp(&ng, &nr, sizeof ng) != 0;
    }
  }
  printf("{\"inputs\": %lu, \"pow_mismatch\": %lu, \"fp2_sqr_mismatch\": %lu, \"fp2_mul_mismatch\": %lu,"
         " \"fp4_sqr_mismatch\": %lu}\n", n, bad_pow, bad_sqr, bad_mul, bad_fp4);
  return (bad_pow || bad_sqr || bad_mul || bad_fp4) ? 1 : 0;
}

// The cofactor chains' addition (curve.h g2_add_inl_exc: no exceptional branch, a flag instead) and
// the subgroup check's mixed addition (g2_madd_inl_exc) against jac_add on curve points from the SSWU map, each also in a second Jacobian representation
// (X z^2, Y z^3, Z z): for distinct points the sums agree projectively and the flag stays clear; for
// P + P, P + (-P) and a point at infinity on either side the flag is set. Prints the mismatch count.
static int cmd_addfuzz(unsigned long n) {
  using namespace bls;
  unsigned long long s = 0x5851f42d4c957f2dull;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)(s >> 11);
  };
  auto rnd = [&]() {
    fp x;
    for (int i = 0; i < 12; i++) x.l[i] = next();
    x.l[11] &= 0x0fffffffu;
    return fp_to_mont(x);
  };
  auto point = [&]() { return hash_field_to_q1(fp2{rnd(), rnd()}); };
  auto rescale = [&](const g2j& p) {
    const fp2 z = {rnd(), rnd()}, z2 = fp2_sqr(z);
    return g2j{fp2_mul(p.x, z2), fp2_mul(p.y, fp2_mul(z2, z)), fp2_mul(p.z, z)};
  };
  fp2 slots[3];
  const LdsFp2Slots park = {slots};
  unsigned long bad = 0;
  auto add = [&](const g2j& p, const g2j& q, bool& exc) {
    exc = false;
    return g2_add_inl_exc(p, [&]() { return q.x; }, [&]() { return q.y; }, [&]() { return q.z; }, park, exc);
  };
  auto madd = [&](const g2j& p, const g2a& q, bool& exc) {
    exc = false;
    return g2_madd_inl_exc(p, [&]() { return q.x; }, [&]() { return q.y; }, park, exc);
  };
  for (unsigned long t = 0; t < n; t++) {
    const g2j p = point(), q = point(), q2 = rescale(q), p2 = rescale(p);
    bool exc;
    // mixed addition (the subgroup check's): q affine
    const g2a qa = g2_to_aff(q), pa = g2_to_aff(p);
    const g2j m = madd(p2, qa, exc);
    bad += exc || !jac_eq(m, jac_add(p, q));
    (void)madd(p2, pa, exc);
    bad += !exc;
    (void)madd(p2, g2a{pa.x, fp2_neg(pa.y)}, exc);
    bad += !exc;
    (void)madd(jac_infinity<fp2>(), qa, exc);
    bad += !exc;
    const g2j r = add(p, q2, exc);
    bad += exc || !jac_eq(r, jac_add(p, q));
    (void)add(p, p2, exc);
    bad += !exc;
    (void)add(p, jac_neg(p2), exc);
    bad += !exc;
    (void)add(jac_infinity<fp2>(), q, exc);
    bad += !exc;
    (void)add(p, jac_infinity<fp2>(), exc);
    bad += !exc;
  }
  printf("{\"inputs\": %lu, \"add_mismatch\": %lu}\n", n, bad);
  return bad != 0;
}

// tower.h fp2_3u_pm_2x (the cyclotomic square's fused 3u +- 2x) against fp2_addsub + fp2_dbl +
// fp2_add on random operands in [0, 2p), the edges 0 and 2p - 1, and top words placed so that the
// quotient estimate sits on each boundary k D (k = 1..10) of its correction step; every result must
// equal the reference mod p and lie in [0, 2p).
static int cmd_linfuzz(unsigned long n) {
  using namespace bls;
  unsigned long long s = 0x9e3779b97f4a7c15ull;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)(s >> 11);
  };
  auto below2p = [&](uint32_t top) {  // top word < P2_RAW[11]: the value is < 2p
    fp x;
    for (int i = 0; i < 11; i++) x.l[i] = next();
    x.l[11] = top;
    return x;
  };
  auto rnd = [&]() { return below2p(next() % P2_RAW[11]); };
  fp zero = fp_zero(), max2p;
  {
    unsigned br = 0;
    for (int i = 0; i < 12; i++) max2p.l[i] = __builtin_subc(P2_RAW[i], i == 0 ? 1u : 0u, br, &br);
  }
  auto lt2p = [](const fp& a) {
    unsigned br = 0;
    for (int i = 0; i < 12; i++) (void)__builtin_subc(a.l[i], P2_RAW[i], br, &br);
    return br != 0;
  };
  unsigned long bad = 0, cases = 0, edges = 0;
  auto check = [&](const fp2& u, const fp2& x, bool sub) {
    const fp2 got = fp2_3u_pm_2x(u, x, sub);
    const fp2 want = fp2_add(fp2_dbl(fp2_addsub(u, x, sub)), u);
    bad += !(fp_eq(got.c0, want.c0) && fp_eq(got.c1, want.c1) && lt2p(got.c0) && lt2p(got.c1));
    cases++;
  };
  const uint32_t D = P_RAW[11] + 1u;
  for (unsigned long t = 0; t < n; t++) {
    for (int sub = 0; sub < 2; sub++) {
      check({rnd(), rnd()}, {rnd(), rnd()}, sub);
      check({zero, max2p}, {max2p, zero}, sub);
      check({max2p, max2p}, {max2p, max2p}, sub);
      check({zero, zero}, {zero, zero}, sub);
    }
    // T = t >> 352 ~ 3 u11 + 2 y11 (+ carries), y = x or 2p - x: aim it at k D - 1, k D, k D + 1
    for (uint32_t k = 1; k <= 10; k++) {
      for (int d = -1; d <= 1; d++) {
        const int64_t T = (int64_t)k * D + d;
        const uint32_t a = next() % P2_RAW[11];  // u's top word
        const int64_t b = (T - 3 * (int64_t)a) / 2;  // y's top word
        if (b < 0 || b >= (int64_t)P2_RAW[11]) continue;
        // sub = false: y = x
        check({below2p(a), rnd()}, {below2p((uint32_t)b), rnd()}, false);
        // sub = true: y = 2p - x, so x's top word ~ P2_11 - b
        const int64_t bx = (int64_t)P2_RAW[11] - 1 - b;
        if (bx >= 0) check({below2p(a), rnd()}, {below2p((uint32_t)bx), rnd()}, true);
        edges++;
      }
    }
  }
  printf("{\"cases\": %lu, \"boundary_cases\": %lu, \"lin_mismatch\": %lu}\n", cases, edges, bad);
  return bad ? 1 : 0;
}

// tower.h fp6_mul_lin / fp12_sqr_lin (one reduction per output component, q p by KpMad) against
// fp6_mul / fp12_sqr: random operands in [0, 2p), operands at 2p - 1, and the lazily added operands
// (< 4p) fp12_sqr feeds its second product; results equal mod p and in [0, 2p).
static int cmd_f6fuzz(unsigned long n) {
  using namespace bls;
  unsigned long long s = 0x2545f4914f6cdd1dull;
  auto next = [&]() {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    return (uint32_t)(s >> 11);
  };
  auto rnd = [&]() {
    fp x;
    for (int i = 0; i < 11; i++) x.l[i] = next();
    x.l[11] = next() % P2_RAW[11];
    return x;
  };
  fp max2p;
  {
    unsigned br = 0;
    for (int i = 0; i < 12; i++) max2p.l[i] = __builtin_subc(P2_RAW[i], i == 0 ? 1u : 0u, br, &br);
  }
  auto lt2p = [](const fp& a) {
    unsigned br = 0;
    for (int i = 0; i < 12; i++) (void)__builtin_subc(a.l[i], P2_RAW[i], br, &br);
    return br != 0;
  };
  auto r6 = [&](bool edge) {
    fp6 a;
    fp2* c[3] = {&a.c0, &a.c1, &a.c2};
    for (auto* x : c) *x = edge ? fp2{max2p, (next() & 1) ? max2p : rnd()} : fp2{rnd(), rnd()};
    return a;
  };
  auto eq6 = [&](const fp6& x, const fp6& y) {
    const fp2* a[3] = {&x.c0, &x.c1, &x.c2};
    const fp2* b[3] = {&y.c0, &y.c1, &y.c2};
    bool ok = true;
    for (int k = 0; k < 3; k++)
      ok &= fp_eq(a[k]->c0, b[k]->c0) && fp_eq(a[k]->c1, b[k]->c1) && lt2p(a[k]->c0) && lt2p(a[k]->c1);
    return ok;
  };
  unsigned long bad = 0, cases = 0;
  for (unsigned long t = 0; t < n; t++) {
    for (int e = 0; e < 3; e++) {
      const fp6 a = r6(e == 1), b = r6(e == 2);
      bad += !eq6(fp6_mul_lin(a, b), fp6_mul(a, b));
      const fp6 la = fp6_add_lazy(a, r6(e == 1)), lb = fp6_add_lazy(b, r6(e != 0));  // < 4p
      bad += !eq6(fp6_mul_lin(la, lb), fp6_mul(la, lb));
      const fp12 f = {a, b}, g = fp12_sqr_lin(f, KpMad()), h = fp12_sqr(f);
      bad += !(eq6(g.c0, h.c0) && eq6(g.c1, h.c1));
      cases += 3;
    }
  }
  printf("{\"cases\": %lu, \"f6_mismatch\": %lu}\n", cases, bad);
  return bad ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc == 3 && !strcmp(argv[1], "hash")) return cmd_hash(argv[2]);
  if (argc == 3 && !strcmp(argv[1], "powfuzz")) return cmd_powfuzz(strtoul(argv[2], nullptr, 10));
  if (argc == 3 && !strcmp(argv[1], "invfuzz")) return cmd_invfuzz(strtoul(argv[2], nullptr, 10));
  if (argc == 3 && !strcmp(argv[1], "addfuzz")) return cmd_addfuzz(strtoul(argv[2], nullptr, 10));
  if (argc == 3 && !strcmp(argv[1], "linfuzz")) return cmd_linfuzz(strtoul(argv[2], nullptr, 10));
  if (argc == 3 && !strcmp(argv[1], "f6fuzz")) return cmd_f6fuzz(strtoul(argv[2], nullptr, 10));
  if (argc != 5) {
    fprintf(stderr, "usage: %s pk48hex round prevhex|- sig96hex   (prev '-' = unchained V2)\n       %s hash msghex\n",
            argv[0], argv[0]);
    return 2;
  }
  auto pk = unhex(argv[1]);
  unsigned long long round = strtoull(argv[2], nullptr, 10);
  auto prev = unhex(argv[3]);
  auto sig = unhex(argv[4]);
  unsigned long long c0;

  // group setup (once per chain, not per beacon)
  g1a P;
  bool pinf;
  if (g1_decompress(pk.data(), P, pinf) != REJ_OK) return 3;

  c0 = g_fp_mul_count;
  uint32_t msg[8];
  if (!strcmp(argv[3], "-"))
    drand_message_v2(msg, round);
  else
    drand_message(msg, prev.data(), (int)prev.size(), round);
  g2j h = hash_to_g2(msg);
  g2a ha = g2_to_aff(h);
  unsigned long long n_hash = g_fp_mul_count - c0;

  c0 = g_fp_mul_count;
  g2a s;
  bool sinf;
  uint8_t cls = g2_decompress(sig.data(), s, sinf, true);
  unsigned long long n_decomp = g_fp_mul_count - c0;
  if (cls) {
    printf("{\"verified\": false, \"class\": %d}\n", cls);
    return 1;
  }

  c0 = g_fp_mul_count;
  g1a Ps[2] = {P, {fp_load_const(G1_GEN_X), fp_load_const(G1_GEN_NEG_Y)}};
  g2a Qs[2] = {ha, s};
  bool act[2] = {true, true};
  fp12 f = miller_loop_2(Ps, Qs, act);
  unsigned long long n_miller = g_fp_mul_count - c0;

  // the device's staged form (k_miller_lines + k_miller_f) must give the same f with the same work
  {
    static line lines[MILLER_STEPS][2];
    const unsigned long long s0 = g_fp_mul_count;
    for (int k = 0; k < 2; k++)
      miller_lines(Ps[k], [&]() { return Qs[k]; }, [&](int step, const line& l) { lines[step][k] = l; });
    fp12 fs = miller_f_from_lines([&](int step, int k) { return lines[step][k]; });
    if (!fp12_eq(fs, f) || g_fp_mul_count - s0 != n_miller) {
      printf("{\"verified\": false, \"staged_miller_mismatch\": true}\n");
      return 1;
    }
  }

  // the device's hard part (Granger-Scott squares on three lanes, k_fexp.hip) in register form
  c0 = g_fp_mul_count;
  const fp12 fe = final_exponentiation(f);
  bool ok = fp12_is_one(fe);
  unsigned long long n_fexp = g_fp_mul_count - c0;

  printf("{\"verified\": %s, \"fp_mul\": {\"hash\": %llu, \"decompress\": %llu, \"miller\": %llu, \"final_exp\": %llu},"
         " \"limb_products_per_fp_mul\": 288}\n",
         ok ? "true" : "false", n_hash, n_decomp, n_miller, n_fexp);
  return ok ? 0 : 1;
}

// Host build of the latency engine (drand_amd/csrc/w*.h, -DWV_HOST): the same source as the device
// kernels, with wv.h emulating the 64 lanes, so tests/test_wv_host.py can check every layer against
// Python integers and the golden vectors on the CPU.
//
// usage: wvtest field   < lines "a0 a1 b0 b1" (hex, raw values < p)  -> one line of results each
//        wvtest inv     < lines "a" (hex, raw < p)                    -> raw a^-1 in both halves (lane GCD)
//        wvtest teamadd < lines "sig96 case"                          -> ok / bad (team G2 addition)
//        wvtest verify  < lines "pk48 msg sig96" (hex)                -> reject class per line
//        wvtest hash    < lines "msg" (hex)                            -> affine H(msg) raw hex
//        wvtest pair    < lines "px py qx0 qx1 qy0 qy1" (affine raw)  -> Miller loop + final exp (raw)
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "../drand_amd/csrc/wrecover.h"
#include "../drand_amd/csrc/wvteam.h"

#include <thread>

namespace wv {
uint32_t g_host_lds[HOST_MAX_WAVES][LDS_WORDS];
thread_local int g_host_wave = 0;
thread_local unsigned long long g_wv_ops[OPC_N];
uint32_t g_host_blk[BLK_SLOTS * 64 + BLK_WORDS_EXTRA];
double g_host_blk_b[BLK_SLOTS];
std::atomic<uint32_t> g_host_ctr[BLK_CTRS];
}
namespace bls {
unsigned long long g_fp_mul_count = 0;
}

using namespace wv;

static std::vector<uint32_t> hex_to_limbs(const std::string& h) {  // 16 x 25-bit limbs of a hex integer
  std::vector<uint32_t> bits;
  for (int i = (int)h.size() - 1; i >= 0; i--) {
    const char c = h[i];
    const int v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
    for (int b = 0; b < 4; b++) bits.push_back((v >> b) & 1);
  }
  std::vector<uint32_t> l(16, 0);
  for (size_t i = 0; i < bits.size() && i < 400; i++) l[i / 25] |= bits[i] << (i % 25);
  return l;
}
static std::string limbs_to_hex(const V& x, int h) {  // strict limbs of half h -> hex
  std::vector<int> bits;
  for (int k = 0; k < 16; k++)
    for (int b = 0; b < 25; b++) bits.push_back((x.v[32 * h + k] >> b) & 1);
  std::string s;
  for (int i = 396; i >= 0; i -= 4) {
    int v = 0;
    for (int b = 3; b >= 0; b--) v = v * 2 + (i + b < 400 ? bits[i + b] : 0);
    s += "0123456789abcdef"[v];
  }
  size_t nz = s.find_first_not_of('0');
  return nz == std::string::npos ? "0" : s.substr(nz);
}
static F raw_fp2(const std::string& c0, const std::string& c1) {
  V x = vsplat(0);
  const auto a = hex_to_limbs(c0), b = hex_to_limbs(c1);
  for (int k = 0; k < 16; k++) x.v[k] = a[k], x.v[32 + k] = b[k];
  return mkF(x, 1.0);
}
static F to_mont(const F& raw) { return mulp(raw, cst(WC_R2_DUP)); }
static std::string out_fp2(const F& a) {
  const V r = raw_canon(a);
  return limbs_to_hex(r, 0) + " " + limbs_to_hex(r, 1);
}

static int cmd_field() {
  char a0[200], a1[200], b0[200], b1[200];
  while (scanf("%199s %199s %199s %199s", a0, a1, b0, b1) == 4) {
    wv_init();
    const F a = to_mont(raw_fp2(a0, a1)), b = to_mont(raw_fp2(b0, b1));
    printf("%s", out_fp2(mul2(a, b)).c_str());
    printf(" %s", out_fp2(sqr2(a)).c_str());
    printf(" %s", out_fp2(mulp(a, b)).c_str());
    printf(" %s", out_fp2(add(a, b)).c_str());
    printf(" %s", out_fp2(sub(a, b)).c_str());
    printf(" %s", out_fp2(mul_xi(a)).c_str());
    printf(" %s", out_fp2(conj(a)).c_str());
    printf(" %s", out_fp2(half(a)).c_str());
    printf(" %s", out_fp2(inv2(a)).c_str());
    printf(" %s", out_fp2(norm_dup(a)).c_str());
    printf(" %s", out_fp2(dot(a, b, b, a, a, a)).c_str());
    printf(" %d %d", (int)eq2(a, b), (int)is_zero2(a));
    printf("\n");
  }
  return 0;
}

// inv: "a" (hex, raw < p) -> raw a^-1 (0 -> 0) by the lane GCD, or "nc" if its divsteps did not
// reach b = 1 (the caller would take the exponentiation)
static int cmd_inv() {
  char a0[200];
  while (scanf("%199s", a0) == 1) {
    wv_init();
    const F a = to_mont(raw_fp2(a0, a0));
    F r;
    if (!inv_gcd_lanes(a, r)) {
      printf("nc\n");
      continue;
    }
    const V c = raw_canon(r);
    printf("%s %s\n", limbs_to_hex(c, 0).c_str(), limbs_to_hex(c, 1).c_str());
  }
  return 0;
}

static std::vector<uint8_t> unhex(const std::string& h) {
  std::vector<uint8_t> b;
  for (size_t i = 0; i + 1 < h.size(); i += 2) b.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
  return b;
}
static void msg_b0(const std::vector<uint8_t>& m, uint32_t (&b0)[8]) {
  if (m.size() == 32) {
    uint32_t w[8];
    for (int i = 0; i < 8; i++) w[i] = (uint32_t)m[4 * i] << 24 | (uint32_t)m[4 * i + 1] << 16 | (uint32_t)m[4 * i + 2] << 8 | m[4 * i + 3];
    xmd_b0_msg32(w, b0);
  } else {
    bls::xmd_b0_bytes(b0, m.data(), (uint32_t)m.size(), bls::DST);
  }
}

// verify: "pk48 msg sig96" -> reject class (pk that does not decode: -1)
static int cmd_verify() {
  char a[300], b[4000], c[300];
  while (scanf("%299s %3999s %299s", a, b, c) == 3) {
    wv_init();
    const auto pk = unhex(a), msg = unhex(strcmp(b, "-") ? b : ""), sig = unhex(c);
    bls::g1a P;
    bool pinf = false;
    if (bls::g1_decompress(pk.data(), P, pinf) != bls::REJ_OK) {
      printf("-1\n");
      continue;
    }
    uint32_t b0[8];
    msg_b0(msg, b0);
    F sx, sy;
    bool sinf;
    const int cls = sig.size() == 96 ? verify_item(sig.data(), b0, P.x.l, P.y.l, pinf, sx, sy, sinf) : bls::REJ_LENGTH;
    printf("%d\n", cls);
    fflush(stdout);
  }
  return 0;
}

// tverify: as verify, by the eight-wave team (wvteam.h), one host thread per wave
static int cmd_tverify() {
  char a[300], b[4000], c[300];
  while (scanf("%299s %3999s %299s", a, b, c) == 3) {
    const auto pk = unhex(a), msg = unhex(strcmp(b, "-") ? b : ""), sig = unhex(c);
    bls::g1a P;
    bool pinf = false;
    if (bls::g1_decompress(pk.data(), P, pinf) != bls::REJ_OK) {
      printf("-1\n");
      continue;
    }
    if (sig.size() != 96) {
      printf("%d\n", bls::REJ_LENGTH);
      continue;
    }
    uint32_t b0[8];
    msg_b0(msg, b0);
    for (auto& ctr : g_host_ctr) ctr.store(0);
    int cls[TEAM_WAVES];
    std::thread th[TEAM_WAVES];
    for (int w = 0; w < TEAM_WAVES; w++)
      th[w] = std::thread([&, w]() {
        g_host_wave = w;
        wv_init();
        F sx, sy;
        bool sinf = false;
        cls[w] = verify_team(sig.data(), b0, P.x.l, P.y.l, pinf, sx, sy, sinf);
      });
    for (auto& t : th) t.join();
    for (int w = 1; w < TEAM_WAVES; w++)
      if (cls[w] != cls[0]) fprintf(stderr, "waves disagree: %d vs %d\n", cls[w], cls[0]), abort();
    printf("%d\n", cls[0]);
    fflush(stdout);
  }
  return 0;
}

// tverify_pre: as tverify, through the fused round's two launches (wvteam.h team_hash_key, then
// verify_team_pre on the signature's affine point). The point is decoded by one wave and handed over
// the way k_lat_recover_sum hands over the interpolated sum: Jacobian (x z^2, y z^3, z) with z = x + 1,
// back to affine by g2_to_affine. Lines whose signature does not decode print its class (the
// speculative path never sees such a signature: its shares all verified).
static int cmd_tverify_pre() {
  char a[300], b[4000], c[300];
  static uint32_t hbuf[HOUT_WORDS], sbuf[SAFF_WORDS];
  while (scanf("%299s %3999s %299s", a, b, c) == 3) {
    const auto pk = unhex(a), msg = unhex(strcmp(b, "-") ? b : ""), sig = unhex(c);
    bls::g1a P;
    bool pinf = false;
    if (bls::g1_decompress(pk.data(), P, pinf) != bls::REJ_OK) {
      printf("-1\n");
      continue;
    }
    if (sig.size() != 96) {
      printf("%d\n", bls::REJ_LENGTH);
      continue;
    }
    uint32_t b0[8];
    msg_b0(msg, b0);
    g_host_wave = 0;
    wv_init();
    F x, y;
    bool sinf = false;
    const uint8_t dc = g2_decompress(sig.data(), x, y, sinf);
    if (dc != bls::REJ_OK) {
      printf("%d\n", dc);
      continue;
    }
    memset(sbuf, 0, sizeof sbuf);
    if (!sinf) {
      const F z = add(x, cst(WC_ONE2)), z2 = sqr2(z);
      F ax, ay;
      g2_to_affine({dot(x, z2), dot(y, dot(z2, z)), z}, ax, ay);
      gst_F(sbuf, ax);
      gst_F(sbuf + 64, ay);
    }
    gst_flag(sbuf + 128, sinf);
    memset(hbuf, 0, sizeof hbuf);
    for (int pass = 0; pass < 2; pass++) {
      for (auto& ctr : g_host_ctr) ctr.store(0);
      int cls[TEAM_WAVES];
      std::thread th[TEAM_WAVES];
      for (int w = 0; w < TEAM_WAVES; w++)
        th[w] = std::thread([&, w]() {
          g_host_wave = w;
          wv_init();
          if (pass == 0) team_hash_key(b0, P.x.l, P.y.l, pinf, hbuf);
          else cls[w] = verify_team_pre(hbuf, sbuf);
        });
      for (auto& t : th) t.join();
      if (pass == 0) continue;
      for (int w = 1; w < TEAM_WAVES; w++)
        if (cls[w] != cls[0]) fprintf(stderr, "waves disagree: %d vs %d\n", cls[w], cls[0]), abort();
      printf("%d\n", cls[0]);
    }
    fflush(stdout);
  }
  return 0;
}

// hash: "msg" -> "inf x0 x1 y0 y1" (affine raw hex)
static int cmd_hash() {
  char b[4000];
  while (scanf("%3999s", b) == 1) {
    wv_init();
    const auto msg = unhex(strcmp(b, "-") ? b : "");
    uint32_t b0[8];
    msg_b0(msg, b0);
    F hx, hy;
    const bool fin = hash_to_g2(b0, hx, hy);
    if (!fin) {
      printf("1 0 0 0 0\n");
      continue;
    }
    printf("0 %s %s\n", out_fp2(hx).c_str(), out_fp2(hy).c_str());
  }
  return 0;
}

// decompress: "sig96" -> "class x0 x1 y0 y1"
static int cmd_decompress() {
  char c[300];
  while (scanf("%299s", c) == 1) {
    wv_init();
    const auto sig = unhex(c);
    F x, y;
    bool inf;
    const int cls = g2_decompress(sig.data(), x, y, inf);
    if (cls || inf) {
      printf("%d %d 0 0 0 0\n", cls, (int)inf);
      continue;
    }
    printf("0 0 %s %s\n", out_fp2(x).c_str(), out_fp2(y).c_str());
  }
  return 0;
}

// opcount: "pk48 msg sig96" (an accepting item) -> JSON op counts per phase of verify_item
static void ops_line(const char* name, bool last) {
  static const char* nm[OPC_N] = {"dot1", "dot2", "dot3", "dot4", "dot5", "dot6", "mulp", "sqr2", "norm", "gcd"};
  printf("\"%s\": {", name);
  for (int k = 0; k < OPC_N; k++) printf("\"%s\": %llu%s", nm[k], g_wv_ops[k], k + 1 < OPC_N ? ", " : "");
  printf("}%s", last ? "}\n" : ", ");
  memset(g_wv_ops, 0, sizeof g_wv_ops);
}
static int cmd_opcount() {
  char a[300], b[4000], c[300];
  if (scanf("%299s %3999s %299s", a, b, c) != 3) return 2;
  wv_init();
  const auto pk = unhex(a), msg = unhex(strcmp(b, "-") ? b : ""), sig = unhex(c);
  bls::g1a P;
  bool pinf = false;
  if (bls::g1_decompress(pk.data(), P, pinf) != bls::REJ_OK) return 3;
  uint32_t b0[8];
  msg_b0(msg, b0);
  memset(g_wv_ops, 0, sizeof g_wv_ops);
  printf("{");
  F sx, sy, hx, hy;
  bool sinf;
  if (g2_decompress(sig.data(), sx, sy, sinf) != bls::REJ_OK) return 4;
  ops_line("decompress_subgroup", false);
  hash_to_g2(b0, hx, hy);
  ops_line("hash_to_g2", false);
  MPair pr[2];
  const bool active[2] = {true, true};
  pr[0] = mpair(g1_coord(P.x.l), g1_coord(P.y.l), hx, hy);
  pr[1] = mpair(cst(WC_NEG_G1_X), cst(WC_NEG_G1_Y), sx, sy);
  ops_line("pair_setup", false);
  const W12 f0 = miller_loop(pr, active);
  ops_line("miller", false);
  const bool ok = final_exp_is_one(f0);
  ops_line("final_exp", true);
  return ok ? 0 : 5;
}

// smul: "sig96 k" (k hex < r) -> compressed [k] S through the x-adic joint multiplication;
// "sum sig96 sig96" -> compressed S1 + S2
static int cmd_smul() {
  static uint32_t tab[15 * POINT_WORDS];
  char a[300], b[300];
  while (scanf("%299s %299s", a, b) == 2) {
    wv_init();
    const auto sig = unhex(a);
    F x, y;
    bool inf;
    if (g2_decompress(sig.data(), x, y, inf) || inf) {
      printf("-\n");
      continue;
    }
    uint32_t lam[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const std::string h(b);
    for (int i = 0; i < (int)h.size(); i++) {  // hex digit i from the right -> bits 4i..4i+3
      const char c = h[h.size() - 1 - i];
      const uint32_t v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
      lam[i / 8] |= v << (4 * (i % 8));
    }
    const G2J r = g2_mul_lambda(x, y, lam, tab);
    const V w = g2_compress_words(r);
    for (int j = 0; j < 24; j++) printf("%08x", lane_val(w, j));
    printf("\n");
    fflush(stdout);
  }
  return 0;
}

// smul4: "sig96 k" -> "ok" when the four-wave form (wrecover.h lambda_base, g2_mul_digit per digit,
// the four partial products summed) equals g2_mul_lambda's [k] S, else "bad"
static int cmd_smul4() {
  static uint32_t tab[15 * POINT_WORDS];
  char a[300], b[300];
  while (scanf("%299s %299s", a, b) == 2) {
    wv_init();
    const auto sig = unhex(a);
    F x, y;
    bool inf;
    if (g2_decompress(sig.data(), x, y, inf) || inf) {
      printf("-\n");
      continue;
    }
    uint32_t lam[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const std::string h(b);
    for (int i = 0; i < (int)h.size(); i++) {
      const char c = h[h.size() - 1 - i];
      const uint32_t v = c <= '9' ? c - '0' : (c | 32) - 'a' + 10;
      lam[i / 8] |= v << (4 * (i % 8));
    }
    const G2J ref = g2_mul_lambda(x, y, lam, tab);
    uint64_t d[4];
    decompose_xabs(lam, d);
    G2J sum = g2_infinity();
    for (int j = 0; j < 4; j++) {
      F px, py;
      lambda_base(x, y, j, px, py);
      sum = g2_add(sum, g2_mul_digit(px, py, d[j]));
    }
    printf(g2_eq(sum, ref) ? "ok\n" : "bad\n");
    fflush(stdout);
  }
  return 0;
}

// teamadd: "sig96 case" -> ok / bad: wvteam.h team_g2_add (three host threads as the hash team's
// waves 0, 4, 5) against wcurve.h g2_add for case sum (P' + 2P), dbl (P' + P), neg (P' + (-P)),
// ainf (O + 2P), binf (P' + O), with P' = P in scaled Jacobian coordinates (Z = x_P); and "chain"
// (team_mul_x_abs against g2_mul_x_abs on P')
static int cmd_teamadd() {
  char a[300], b[32];
  while (scanf("%299s %31s", a, b) == 2) {
    wv_init();
    const auto sig = unhex(a);
    F x, y;
    bool inf;
    if (g2_decompress(sig.data(), x, y, inf) || inf) {
      printf("-\n");
      continue;
    }
    const G2J p = {x, y, cst(WC_ONE2)};
    const F l2 = sqr2(x);
    const G2J ps = {dot(p.x, l2), dot(p.y, dot(l2, x)), dot(p.z, x)};
    const G2J p2 = g2_dbl(p);
    const std::string c(b);
    G2J A = ps, B = p2;
    if (c == "dbl") B = p;
    else if (c == "neg") B = g2_neg(p);
    else if (c == "ainf") A = g2_infinity();
    else if (c == "binf") B = g2_infinity();
    const bool chain = c == "chain";
    const G2J want = chain ? g2_mul_x_abs(ps) : g2_add(A, B);
    for (auto& ctr : g_host_ctr) ctr.store(0);
    xst_g2(HS_ACC, chain ? ps : A);
    xst_g2(HS_Q2, chain ? ps : B);
    std::thread th[3];
    const int waves[3] = {0, 4, 5};
    for (int k = 0; k < 3; k++)
      th[k] = std::thread([&, k]() {
        g_host_wave = waves[k];
        wv_init();
        Team t = make_team(HASH_TEAM, CTR_HASH);
        if (chain) team_mul_x_abs(t, HS_Q2, HS_ACC);
        else team_g2_add(t, HS_ACC, HS_Q2);
      });
    for (auto& t : th) t.join();
    printf("%s\n", g2_eq(xld_g2(HS_ACC), want) ? "ok" : "bad");
    fflush(stdout);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "field")) return cmd_field();
  if (argc >= 2 && !strcmp(argv[1], "inv")) return cmd_inv();
  if (argc >= 2 && !strcmp(argv[1], "teamadd")) return cmd_teamadd();
  if (argc >= 2 && !strcmp(argv[1], "verify")) return cmd_verify();
  if (argc >= 2 && !strcmp(argv[1], "tverify")) return cmd_tverify();
  if (argc >= 2 && !strcmp(argv[1], "tverify_pre")) return cmd_tverify_pre();
  if (argc >= 2 && !strcmp(argv[1], "hash")) return cmd_hash();
  if (argc >= 2 && !strcmp(argv[1], "decompress")) return cmd_decompress();
  if (argc >= 2 && !strcmp(argv[1], "opcount")) return cmd_opcount();
  if (argc >= 2 && !strcmp(argv[1], "smul")) return cmd_smul();
  if (argc >= 2 && !strcmp(argv[1], "smul4")) return cmd_smul4();
  fprintf(stderr, "usage: wvtest field|verify|hash|pair\n");
  return 2;
}

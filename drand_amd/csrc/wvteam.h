// One verification by a team of four waves (one per SIMD of a CU), the latency engine's device form
// (k_lat.hip). The work of wverify.h's verify_item, scheduled across the waves:
//
//   phase A  wave 0: hash-to-G2 of the message            waves 1-3: decompress + subgroup check of
//                                                          the signature (wave 1), then the Miller
//                                                          loop of the signature pair (e(-g1, S)),
//                                                          as a team of three
//   phase B  all four: the Miller loop of the key pair (e(pk, H(m)))
//   phase C  all four: the product of the two Miller values and the final exponentiation
//
// The two Miller loops run separately (f = f_0 f_1 with each f_k its own loop's product: squaring
// is multiplicative), so the signature's pair needs no hash and overlaps it. A Miller doubling step
// is two team rounds: (1) the six coefficients of f^2 two per wave beside the line pieces (A, X^2 ->
// l2, YZ -> l3, and B, C, E -> l0 with T's new Z on the fourth wave); (2) f^2 times the line two
// coefficients per wave while the fourth wave finishes T. Every Fp12 operation of the final
// exponentiation splits its six output coefficients two per wave over three waves.
#pragma once
#include "wteam.h"
#include "wverify.h"

namespace wv {

// ------------------------------------------------------------------ block LDS slots (wteam.h)
// team areas (one per Miller loop): f double buffer, f^2, T, line, step intermediates
constexpr int TA_FB = 0, TA_FSQ = 12, TA_TX = 18, TA_TY = 19, TA_TZ = 20, TA_L0 = 21, TA_L2 = 22, TA_L3 = 23,
              TA_A = 24, TA_B = 25, TA_E = 26, TA_G = 27, TA_ZN = 28, TA_SIZE = 32;
constexpr int TB0 = 0, TB1 = TA_SIZE;  // key pair, signature pair
// final exponentiation values (6 slots each)
constexpr int W_BASE = 2 * TA_SIZE;
constexpr int W_R = W_BASE, W_INV = W_BASE + 6, W_T = W_BASE + 12, W_U = W_BASE + 18, W_G = W_BASE + 24,
              W_P = W_BASE + 30, W_S = W_BASE + 36, W_A = W_BASE + 42, W_B = W_BASE + 48, W_C = W_BASE + 54;
constexpr int S_HX = W_BASE + 60, S_HY = S_HX + 1, S_SX = S_HX + 2, S_SY = S_HX + 3;
static_assert(S_SY < BLK_SLOTS, "block slots");
// scalar words
constexpr int XW_CLS = 0, XW_SINF = 1, XW_HFIN = 2, XW_F1 = 3;

WVI W12 xld_w12(int base, bool cj = false) {
  W12 r;
  for (int k = 0; k < 6; k++) {
    const F v = xld(base + k);
    r.c[k] = (cj && (k & 1)) ? neg<0>(v) : v;
  }
  return r;
}
WVI void xst_w12(int base, const W12& v) {
  for (int k = 0; k < 6; k++) xst(base + k, v.c[k]);
}

// output k of a six-output operation is computed by wave k / 2 of the team (a fourth wave idles)
template <class Fn>
WVI void team_op(Team& t, int dst, Fn fn) {
  for (int k = 2 * t.id; k < 6 && k < 2 * t.id + 2; k++) xst(dst + k, fn(k));
  team_sync(t);
}

// ------------------------------------------------------------------ Miller loop of one pair
// the four slots of a step run on waves s % n (a team of three doubles up slot 3 on wave 0)
WVI void team_miller_dbl(Team& t, const MPair& m, int tb, int& cur) {
  const int fin = tb + TA_FB + 6 * cur, fout = tb + TA_FB + 6 * (cur ^ 1);
  for (int s = t.id; s < 4; s += t.n) {
    if (s < 3) {
      const W12 f = xld_w12(fin);
      xst(tb + TA_FSQ + 2 * s, w12_sqr_c(f, 2 * s));
      xst(tb + TA_FSQ + 2 * s + 1, w12_sqr_c(f, 2 * s + 1));
      const F X = xld(tb + TA_TX), Y = xld(tb + TA_TY), Z = xld(tb + TA_TZ);
      if (s == 0) xst(tb + TA_A, half(dot(X, Y)));          // X Y / 2
      if (s == 1) xst(tb + TA_L2, mulp(sqr2(X), m.xp3));     // 3 X^2 xP
      if (s == 2) xst(tb + TA_L3, mulp(dot(Y, Z), m.m2yp));  // -2 Y Z yP
    } else {
      const F Y = xld(tb + TA_TY), Z = xld(tb + TA_TZ);
      const F B = sqr2(Y), C = sqr2(Z);
      const F E = dot(C, cst(WC_B2X3));  // 3 b' Z^2
      xst(tb + TA_L0, sub<0>(E, B));
      xst(tb + TA_B, B);
      xst(tb + TA_E, E);
      xst(tb + TA_G, half(add(B, mul_small<3>(E))));  // (B + 3E) / 2
      xst(tb + TA_ZN, dot(B, dbl(dot(Y, Z))));        // B H
    }
  }
  team_sync(t);
  for (int s = t.id; s < 4; s += t.n) {
    if (s < 3) {
      const W12 q = xld_w12(tb + TA_FSQ);
      const F l0 = xld(tb + TA_L0), l2 = xld(tb + TA_L2), l3 = xld(tb + TA_L3);
      xst(fout + 2 * s, w12_mul_line_c(q, l0, l2, l3, 2 * s));
      xst(fout + 2 * s + 1, w12_mul_line_c(q, l0, l2, l3, 2 * s + 1));
    } else {
      const F A = xld(tb + TA_A), B = xld(tb + TA_B), E = xld(tb + TA_E), G = xld(tb + TA_G);
      const F nE = neg<0>(E);
      xst(tb + TA_TX, dot(A, B, mul_small<3>(A), nE));  // A (B - 3E)
      xst(tb + TA_TY, dot(G, G, mul_small<3>(E), nE));  // G^2 - 3 E^2
      xst(tb + TA_TZ, xld(tb + TA_ZN));
    }
  }
  team_sync(t);
  cur ^= 1;
}

WVI void team_miller_add(Team& t, const MPair& m, int tb, int& cur) {
  if (t.id == 3 % t.n) {
    MPair mm = m;
    mm.t = {xld(tb + TA_TX), xld(tb + TA_TY), xld(tb + TA_TZ)};
    F l0, l2, l3;
    miller_add(mm, l0, l2, l3);
    xst(tb + TA_TX, mm.t.x);
    xst(tb + TA_TY, mm.t.y);
    xst(tb + TA_TZ, mm.t.z);
    xst(tb + TA_L0, l0);
    xst(tb + TA_L2, l2);
    xst(tb + TA_L3, l3);
  }
  team_sync(t);
  const int fin = tb + TA_FB + 6 * cur, fout = tb + TA_FB + 6 * (cur ^ 1);
  for (int s = t.id; s < 3; s += t.n) {
    const W12 f = xld_w12(fin);
    const F l0 = xld(tb + TA_L0), l2 = xld(tb + TA_L2), l3 = xld(tb + TA_L3);
    xst(fout + 2 * s, w12_mul_line_c(f, l0, l2, l3, 2 * s));
    xst(fout + 2 * s + 1, w12_mul_line_c(f, l0, l2, l3, 2 * s + 1));
  }
  team_sync(t);
  cur ^= 1;
}

// f_{|x|, Q}(P) of one pair (unconjugated, wpairing.h miller_loop); returns its slot base
WVI int team_miller(Team& t, const MPair& m, int tb) {
  if (t.id == 0) {
    xst_w12(tb + TA_FB, w12_one());
    xst(tb + TA_TX, m.t.x);
    xst(tb + TA_TY, m.t.y);
    xst(tb + TA_TZ, m.t.z);
  }
  team_sync(t);
  int cur = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    team_miller_dbl(t, m, tb, cur);
    if ((bls::BLS_X_ABS >> i) & 1ull) team_miller_add(t, m, tb, cur);
  }
  return tb + TA_FB + 6 * cur;
}

// ------------------------------------------------------------------ final exponentiation
// dst <- src^|x| (wpairing.h w12_pow_x_abs); scr is clobbered. 68 operations alternate between scr and
// dst, starting on scr, so the last lands on dst.
WVI void team_pow_x_abs(Team& t, int dst, int src, int scr) {
  constexpr uint64_t NSQ = 1ull | (2ull << 6) | (3ull << 12) | (9ull << 18) | (32ull << 24) | (16ull << 30);
  int in = src, out = scr;
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int n = (int)((NSQ >> (6 * s)) & 63u);
#pragma unroll 1
    for (int k = 0; k < n; k++) {
      team_op(t, out, [&](int c) { return w12_cyc_sqr_c(xld_w12(in), c); });
      in = out;
      out = out == scr ? dst : scr;
    }
    if (s < 5) {
      team_op(t, out, [&](int c) { return w12_mul_c(xld_w12(in), xld_w12(src), c); });
      in = out;
      out = out == scr ? dst : scr;
    }
  }
}

// wpairing.h final_exp_is_one of the Miller value in slots f0 (unconjugated)
WVI bool team_final_exp_is_one(Team& t, int f0) {
  if (t.id == 0) xst_w12(W_INV, w12_inv<true>(xld_w12(f0)));  // conj(f0^-1)
  team_sync(t);
  team_op(t, W_T, [&](int k) { return w12_mul_c(xld_w12(f0), xld_w12(W_INV), k); });
  team_op(t, W_U, [&](int k) { return w12_frob2_c(xld_w12(W_T), k); });
  team_op(t, W_G, [&](int k) { return w12_mul_c(xld_w12(W_U), xld_w12(W_T), k); });
  // a = g^(x-1), b = a^(x-1), c = b^(x+p); X^x = conj(X^|x|)
  if (t.id == 0) WV_MARK(8);
  team_pow_x_abs(t, W_P, W_G, W_S);
  if (t.id == 0) WV_MARK(9);
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_G, true), k); });
  team_pow_x_abs(t, W_P, W_A, W_S);
  team_op(t, W_B, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_A, true), k); });
  team_pow_x_abs(t, W_P, W_B, W_S);
  team_op(t, W_U, [&](int k) { return w12_frob_c(xld_w12(W_B), k); });
  team_op(t, W_C, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_U), k); });
  // e = (c^|x|)^|x| frob2(c) conj(c) g^2 g
  team_pow_x_abs(t, W_A, W_C, W_S);
  team_pow_x_abs(t, W_B, W_A, W_S);
  team_op(t, W_U, [&](int k) { return w12_frob2_c(xld_w12(W_C), k); });
  team_op(t, W_P, [&](int k) { return w12_mul_c(xld_w12(W_B), xld_w12(W_U), k); });
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P), xld_w12(W_C, true), k); });
  team_op(t, W_U, [&](int k) { return w12_cyc_sqr_c(xld_w12(W_G), k); });
  team_op(t, W_P, [&](int k) { return w12_mul_c(xld_w12(W_A), xld_w12(W_U), k); });
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P), xld_w12(W_G), k); });
  return w12_is_one(xld_w12(W_A));
}

// ------------------------------------------------------------------ the item
// wverify.h verify_item run by the four waves of a workgroup (each wave calls it); every wave returns
// the same class, and sx, sy, s_inf (the decoded signature) on REJ_OK / REJ_PAIRING
WVI uint8_t verify_team(const uint8_t* sig, const uint32_t (&b0)[8], const uint32_t* pkx, const uint32_t* pky,
                        bool pk_inf, F& sx, F& sy, bool& s_inf) {
  const int w = wave_id();
  Team all = make_team(0, 4, 0);
  if (w == 0) WV_MARK(0);
  if (w == 0) {
    F hx, hy;
    const bool fin = hash_to_g2(b0, hx, hy);
    WV_MARK(1);
    if (fin) {
      xst(S_HX, hx);
      xst(S_HY, hy);
    }
    xst_word(XW_HFIN, fin);
  } else {
    Team t1 = make_team(1, 3, 1);
    if (w == 1) {
      F x, y;
      bool inf;
      const uint8_t c = g2_decompress(sig, x, y, inf);
      WV_MARK(2);
      if (c == bls::REJ_OK && !inf) {
        xst(S_SX, x);
        xst(S_SY, y);
      }
      xst_word(XW_CLS, c);
      xst_word(XW_SINF, inf);
    }
    team_sync(t1);
    if (xld_word(XW_CLS) == bls::REJ_OK && !xld_word(XW_SINF)) {
      const MPair m1 = mpair(cst(WC_NEG_G1_X), cst(WC_NEG_G1_Y), xld(S_SX), xld(S_SY));
      const int f1 = team_miller(t1, m1, TB1);
      if (t1.id == 0) xst_word(XW_F1, (uint32_t)f1);
      if (t1.id == 0) WV_MARK(3);
    }
  }
  team_sync(all);
  if (w == 0) WV_MARK(4);
  const uint8_t cls = (uint8_t)xld_word(XW_CLS);
  if (cls != bls::REJ_OK) return cls;
  s_inf = xld_word(XW_SINF) != 0;
  if (!s_inf) {
    sx = xld(S_SX);
    sy = xld(S_SY);
  }
  const bool a0 = xld_word(XW_HFIN) && !pk_inf, a1 = !s_inf;
  if (!a0 && !a1) return bls::REJ_OK;  // empty product = 1 (kilic Check [ext])
  int f;
  if (a0) {
    const MPair m0 = mpair(g1_coord(pkx), g1_coord(pky), xld(S_HX), xld(S_HY));
    f = team_miller(all, m0, TB0);
    if (w == 0) WV_MARK(5);
    if (a1) {
      const int f1 = (int)xld_word(XW_F1);
      team_op(all, W_R, [&](int k) { return w12_mul_c(xld_w12(f), xld_w12(f1), k); });
      f = W_R;
    }
  } else {
    f = (int)xld_word(XW_F1);
  }
  if (w == 0) WV_MARK(6);
  const bool one = team_final_exp_is_one(all, f);
  if (w == 0) WV_MARK(7);
  return one ? bls::REJ_OK : bls::REJ_PAIRING;
}

}  // namespace wv

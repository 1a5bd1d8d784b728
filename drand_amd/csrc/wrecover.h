// tbls Recover's group-signature interpolation for the latency engine: sum_i [lambda_i] S_i over the
// t selected shares (share.RecoverCommit [ext]), one wave per share for the scalar multiplications,
// one workgroup for the sum, the affine conversion and the compression.
//
// [lambda] S uses the x-adic decomposition of the scalar: lambda < r < |x|^4, so lambda = sum_j d_j |x|^j
// with 64-bit digits d_j, and on G2 [|x|] S = [-x] S = -psi(S) (psi(S) = [x] S is the subgroup
// relation wcurve.h checks), hence [lambda] S = sum_j [d_j] P_j, P_j = (-psi)^j (S). The four 64-bit
// multiplications run jointly: 15 subset sums of P_0..P_3 in LDS, then 64 doublings and one table
// addition per nonzero digit column -- a quarter of the doublings of a plain 255-bit ladder.
#pragma once
#include "wverify.h"

namespace wv {

// Fp2 coordinate (slot 0 = x, 2 = y) of S entry k as the batch engine stores it: SoA words
// S[(f * 12 + w) * stride + k], f = 2 slot/2 + c, Montgomery R = 2^392, < 2p -> R = 2^400
WVI F fp2_from392(const uint32_t* S, size_t stride, size_t k, int slot) {
  const V l = lane_id(), kk = l & 15u, h = l >> 5;
  const V bit = kk * 25u, wi = bit >> 5, sh = bit & 31u;
  const uint32_t* base = S + k;
  const V f = (uint32_t)slot + h;
  auto word = [&](V w) { return gld(base, (f * 12u + sel(w < 12u, w, vsplat(11))) * (uint32_t)stride); };
  const V lo = word(wi), hi = word(sel(wi < 11u, wi + 1u, vsplat(11)));
  const V v = ((lo >> sh) | sel((sh == 0u) | (wi >= 11u), vsplat(0), hi << ((32u - sh) & 31u))) & M25;  // (sh == 0: discarded)
  return mulp(mkF(sel((l & 16u) == 0u, v, vsplat(0)), 2.0), cst(WC_C408_DUP));
}

// w <- w / |x|, returns w mod |x| (256-bit w as 8 little-endian words; restoring division, |x| >= 2^63)
WVI uint64_t div_xabs(uint32_t (&w)[8]) {
  const uint64_t X = bls::BLS_X_ABS;
  uint64_t r = 0;
  for (int i = 255; i >= 0; i--) {
    const uint64_t top = r >> 63;
    r = (r << 1) | ((w[i >> 5] >> (i & 31)) & 1u);
    const bool ge = top != 0 || r >= X;
    if (ge) r -= X;  // exact mod 2^64: the true value is below 2 |x|
    w[i >> 5] = (w[i >> 5] & ~(1u << (i & 31))) | ((uint32_t)ge << (i & 31));
  }
  return r;
}
// lambda (< r) -> digits d_0..d_3 < |x| with lambda = sum_j d_j |x|^j
WVI void decompose_xabs(const uint32_t (&lam)[8], uint64_t (&d)[4]) {
  uint32_t w[8];
  for (int i = 0; i < 8; i++) w[i] = lam[i];
  for (int j = 0; j < 3; j++) d[j] = div_xabs(w);
  d[3] = (uint64_t)w[0] | ((uint64_t)w[1] << 32);  // < |x| since lambda < |x|^4
}

// a stored point: every coordinate a reduced dot output (checked on the host)
constexpr double STORED_BOUND = 1.05;
WVI void st_point(uint32_t* base, const G2J& p, bool global) {
  const F* c[3] = {&p.x, &p.y, &p.z};
  for (int i = 0; i < 3; i++) {
    WV_REQUIRE(bnd(*c[i]), STORED_BOUND, "stored point coordinate");
    if (global)
      gst(base + 64 * i, lane_id(), c[i]->x);
    else
      lds_st(base + 64 * i, lane_id(), c[i]->x);
  }
}
WVI G2J ld_point(const uint32_t* base, bool global) {
  G2J p;
  F* c[3] = {&p.x, &p.y, &p.z};
  for (int i = 0; i < 3; i++) *c[i] = mkF(global ? gld(base + 64 * i, lane_id()) : lds_ld(base + 64 * i, lane_id()),
                                          STORED_BOUND);
  return p;
}
constexpr int POINT_WORDS = 192;

// -psi of an affine point (z = 1), every coordinate reduced
WVI G2J neg_psi_affine(const F& x, const F& y) {
  return {dot(conj<1>(x), cst(WC_PSI_KX)), dot(conj<1>(y), neg<0>(cst(WC_PSI_KY))), cst(WC_ONE2)};
}

// [lambda] (x, y) for an affine G2 point; tab = 15 * POINT_WORDS words of this wave's LDS
WVI G2J g2_mul_lambda(const F& x, const F& y, const uint32_t (&lam)[8], uint32_t* tab) {
  uint64_t d[4];
  decompose_xabs(lam, d);
  // P_0 = S, P_1 = -psi(S), P_2 = psi^2(S), P_3 = -psi(P_2); T[m] = sum of P_j over the bits j of m
  G2J P[4];
  P[0] = {x, y, cst(WC_ONE2)};
  P[1] = neg_psi_affine(x, y);
  P[2] = {mulp(x, cst(WC_PSI2_KX)), mulp(y, cst(WC_PSI2_KY)), cst(WC_ONE2)};
  P[3] = neg_psi_affine(P[2].x, P[2].y);
  for (int j = 0; j < 4; j++) {
    st_point(tab + ((1 << j) - 1) * POINT_WORDS, P[j], false);
    for (int m = 1; m < (1 << j); m++) {
      wsync();
      const G2J s = g2_add(ld_point(tab + (m - 1) * POINT_WORDS, false), P[j]);
      st_point(tab + ((1 << j) + m - 1) * POINT_WORDS, s, false);
    }
  }
  wsync();
  G2J acc = g2_infinity();
  bool started = false;
#pragma unroll 1
  for (int b = 63; b >= 0; b--) {
    if (started) acc = g2_dbl(acc);
    const uint32_t m = (uint32_t)((d[0] >> b) & 1u) | (uint32_t)(((d[1] >> b) & 1u) << 1) |
                       (uint32_t)(((d[2] >> b) & 1u) << 2) | (uint32_t)(((d[3] >> b) & 1u) << 3);
    if (m) {
      const G2J t = ld_point(tab + (m - 1) * POINT_WORDS, false);
      acc = started ? g2_add(acc, t) : t;
      started = true;
    }
  }
  return acc;
}

// The same product split over four waves (k_lat_recover_mul): wave j computes [d_j] P_j alone, P_j
// affine, by a left-to-right ladder of 63 doublings and one mixed addition per set bit below the top
// one. Its intermediate multiples [k] P_j, 2 <= k < 2^64 < r, never equal +-P_j for P_j of order r,
// so the addition needs no exceptional-case tests (g2_madd_noexc); a share outside G2 gives garbage
// here, but its partial then fails verification and the speculative result is discarded.
WVI G2J lambda_base(const F& x, const F& y, int j, F& px, F& py) {  // P_j, affine
  px = x;
  py = y;
  if (j >= 2) {
    px = mulp(x, cst(WC_PSI2_KX));
    py = mulp(y, cst(WC_PSI2_KY));
  }
  if (j & 1) {
    const G2J q = neg_psi_affine(px, py);
    px = q.x;
    py = q.y;
  }
  return {px, py, cst(WC_ONE2)};
}
WVI G2J g2_mul_digit(const F& qx, const F& qy, uint64_t k) {
  if (!k) return g2_infinity();
  const int top = 63 - __builtin_clzll(k);
  G2J acc = {qx, qy, cst(WC_ONE2)};
#pragma unroll 1
  for (int b = top - 1; b >= 0; b--) {
    acc = g2_dbl(acc);
    if ((k >> b) & 1u) acc = g2_madd_noexc(acc, qx, qy);
  }
  return acc;
}

// ZCash compressed encoding of a finite point given affine, as 24 big-endian words (lane j < 24
// returns word j)
WVI V g2_compress_affine_words(const F& x, const F& y) {
  const V l = lane_id();
  uint32_t w0[12], w1[12];
  const V xr = raw_canon(x);
  limbs_to_words(xr, 0, w0);
  limbs_to_words(xr, 1, w1);
  const V yr = raw_canon(y);
  const uint32_t gt = ge_halves(yr, cword(WC_PP1H_DUP));
  const uint64_t nz = ballot(((l & 16u) == 0u) & (yr != 0u));
  const bool largest = half_bits(nz, 1) != 0 ? ((gt >> 1) & 1u) != 0 : (gt & 1u) != 0;
  V out = vsplat(0);
  for (int j = 0; j < 12; j++) {
    out = sel(l == (uint32_t)j, vsplat(w1[11 - j]), out);       // x.c1, most significant word first
    out = sel(l == (uint32_t)(12 + j), vsplat(w0[11 - j]), out);  // x.c0
  }
  return out | sel(l == 0u, vsplat(0x80000000u | (largest ? 0x20000000u : 0u)), vsplat(0));
}
constexpr uint32_t COMPRESSED_INF_WORD0 = 0xc0000000u;

// ZCash compressed encoding of a point, as 24 big-endian words (lane j < 24 returns word j)
WVI V g2_compress_words(const G2J& p) {
  if (g2_is_inf(p)) return sel(lane_id() == 0u, vsplat(COMPRESSED_INF_WORD0), vsplat(0));
  F x, y;
  g2_to_affine(p, x, y);
  return g2_compress_affine_words(x, y);
}

}  // namespace wv

// Hash-to-G2 (RFC 9380 BLS12381G2_XMD:SHA-256_SSWU_RO_, KyberG2.Hash [ext]) and ZCash G2
// decompression (kilic G2.FromCompressed [ext]) for the latency engine, one item per wave.
// The SHA-256 work (chain.Message, expand_message_xmd) is wave-uniform: every lane runs the scalar
// code of hash.h on the same data. The field work uses the lane form; the two SSWU maps of a hash
// share their three Fp exponentiations (one per half: SSWU denominators' inversion, root of the norm,
// square root), the algorithms of hash.h / tower.h otherwise.
#pragma once
#include "wcurve.h"
#ifdef WV_HOST
#ifndef BLS_HOST
#define BLS_HOST
#endif
#endif
#include "hash.h"

namespace wv {

// 16 big-endian words of a 512-bit integer per half (w[h][0..15]) -> its value mod p in Montgomery
// form: hi 2^256 + lo with hi = words 0..7, lo = words 8..15. The words go through this wave's LDS
// scratch (slot 0 of the product area, restaged by the next product anyway).
WVI F fp2_from_be512(const uint32_t (&w0)[16], const uint32_t (&w1)[16]) {
  // the words pass through slot 0's negation area (L_BZ), which every Fp2 product restages
  uint32_t* lds = wave_lds() + L_BZ;
  const V l = lane_id();
  // little-endian 32-bit words of half h: hi at [h*16 + 0..7], lo at [h*16 + 8..15]; lane j of the
  // wave writes word j (j < 32)
  V wv = vsplat(0);
  for (int i = 0; i < 8; i++) {
    wv = sel(l == (uint32_t)i, vsplat(w0[7 - i]), wv);
    wv = sel(l == (uint32_t)(8 + i), vsplat(w0[15 - i]), wv);
    wv = sel(l == (uint32_t)(16 + i), vsplat(w1[7 - i]), wv);
    wv = sel(l == (uint32_t)(24 + i), vsplat(w1[15 - i]), wv);
  }
  wsync();
  lds_st(lds, l, wv);  // lanes 32..63 write zeros to words 32..63 (unused)
  wsync();
  // lane k of half h: bits 25k .. 25k+24 of the 256-bit hi (k < 11) and of lo
  const V k = l & 15u, h = l >> 5;
  const V bit = k * 25u, wi = bit >> 5, sh = bit & 31u;
  const M live = ((l & 16u) == 0u) & (k < 11u);
  auto limb = [&](uint32_t base) {
    const V lo = lds_ld(lds, h * 16u + base + sel(wi < 8u, wi, vsplat(0)));
    const V hi = lds_ld(lds, h * 16u + base + sel(wi < 7u, wi + 1u, vsplat(0)));
    const V v = ((lo >> sh) | sel((sh == 0u) | (wi >= 7u), vsplat(0), hi << ((32u - sh) & 31u))) & M25;  // (sh == 0: discarded)
    return sel(live, v, vsplat(0));
  };
  const V hv = limb(0), lv = limb(8);
  wsync();
  const F hi = mkF(hv, 0.0), lo = mkF(lv, 0.0);
  return add(mulp(hi, cst(WC_H256_R2_DUP)), mulp(lo, cst(WC_R2_DUP)));
}

// b_0 of expand_message_xmd for a 32-byte message (hash.h hash_to_field_fp2's first step)
WVI void xmd_b0_msg32(const uint32_t (&msg)[8], uint32_t (&b0)[8]) {
  uint32_t st[8];
  for (int i = 0; i < 8; i++) st[i] = bls::SHA256_ZPAD_MIDSTATE[i];
  uint32_t blk[16];
  for (int i = 0; i < 8; i++) {
    blk[i] = msg[i];
    blk[8 + i] = bls::XMD_B0_A_TAIL[i];
  }
  bls::sha256_compress_fast(st, blk);
  bls::sha256_compress_fast(st, bls::XMD_B0_B);
  for (int i = 0; i < 8; i++) b0[i] = st[i];
}

// b_1 .. b_8 from b_0, as the four 64-byte field-element strings e[0..3] (16 big-endian words each)
WVI void xmd_words(const uint32_t (&b0)[8], uint32_t (&e)[4][16]) {
  uint32_t prev[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = 1; k <= 8; k++) {
    uint32_t st[8];
    bls::sha256_init(st);
    uint32_t blk[16];
    for (int i = 0; i < 8; i++) {
      blk[i] = b0[i] ^ prev[i];
      blk[8 + i] = bls::XMD_BI_A_TAIL[i];
    }
    blk[8] |= (uint32_t)k << 24;
    bls::sha256_compress_fast(st, blk);
    bls::sha256_compress_fast(st, bls::XMD_BI_B);
    for (int i = 0; i < 8; i++) {
      e[(k - 1) / 2][((k - 1) & 1) * 8 + i] = st[i];
      prev[i] = st[i];
    }
  }
}

// ------------------------------------------------------------------ SSWU (two maps, pair exps)
struct Pair2 {
  F a, b;  // the same quantity for map 0 and map 1 (each an Fp2)
};
// [x.c0 of map 0 | x.c0 of map 1] and likewise c1: the Fp halves of two Fp2 values as pairs
WVI F pair_c0(const F& x0, const F& x1) { return select_halves(1u, dup0(x0), dup0(x1)); }
WVI F pair_c1(const F& x0, const F& x1) { return select_halves(1u, dup1(x0), dup1(x1)); }
// Fp2 value of map m from pairs (c0s, c1s): [c0s.h_m | c1s.h_m]
WVI F fp2_of_pairs(const F& c0s, const F& c1s, int m) {
  return m == 0 ? select_halves(1u, dup0(c0s), dup0(c1s)) : select_halves(1u, dup1(c0s), dup1(c1s));
}

// sgn0 (RFC 9380, Fp2) of a value: from its canonical raw halves
WVI bool sgn0_fp2(const F& a) {
  const V r = raw_canon(a);
  const bool s0 = lane0_of_half(r, 0) & 1u, s1 = lane0_of_half(r, 1) & 1u;
  const uint64_t nz = ballot(((lane_id() & 16u) == 0u) & (r != 0u));
  const bool z0 = half_bits(nz, 0) == 0;
  return s0 | (z0 & s1);
}

// a^((p-3)/4) on this wave alone (the team form hands the squarings' powers to a helper wave)
struct PowSelf {
  WVI F operator()(const F& a) const { return pow_pm3d4(a); }
};

// The affine side of the two SSWU maps: x1 = xN / xD and gx1 = (x1^2 + A) x1 + B from the projective
// xN, xD and the pair of norms N(xD) (inverted as one pair). sswu2 needs it only after the first
// exponentiation, so the team form runs it on another wave meanwhile (wvteam.h).
struct SswuAff {
  F ndi, x1[2], gx1[2];
};
WVI SswuAff sswu_affine(const F& nd, const F (&xN)[2], const F (&xD)[2]) {
  const F A = cst(WC_SSWU_A), B = cst(WC_SSWU_B), one = cst(WC_ONE2);
  SswuAff r;
  r.ndi = inv_pair_nz(nd);
  for (int m = 0; m < 2; m++) {
    const F ni = m == 0 ? dup0(r.ndi) : dup1(r.ndi);
    r.x1[m] = dot(xN[m], mulp(conj<0>(xD[m]), ni));                        // xN conj(xD) / N(xD)
    r.gx1[m] = dot(dot(sqr2(r.x1[m]), one, A, one), r.x1[m], B, one);     // (x^2 + A) x + B
  }
  return r;
}
// ... on this wave, when sswu2 asks for it
struct AffSelf {
  F nd, xN[2], xD[2];
  WVI void start(const F& n, const F (&a)[2], const F (&b)[2]) {
    nd = n;
    for (int m = 0; m < 2; m++) xN[m] = a[m], xD[m] = b[m];
  }
  WVI SswuAff get() const { return sswu_affine(nd, xN, xD); }
};

// both SSWU maps of a hash: (x_m, y_m) on E2' for u_m (hash.h map_to_curve_sswu with its tv1); pw
// computes a^((p-3)/4) per half. The first exponentiation (the root of N(gx1), whether gx1 is a
// square) runs on the projective x1 = xN / xD: N(gx1) = N(gxN) / N(xD)^3 = n' / N(xD)^4 with
// n' = N(gxN) N(xD), so its root is the root of n' times N(xD)^-2 and n' is a square exactly when
// N(gx1) is; the inversion and the affine x1, gx1 (aff) are needed only after it.
template <class Pow = PowSelf, class Aff = AffSelf>
WVI void sswu2(const F (&u)[2], F (&xo)[2], F (&yo)[2], Pow pw = Pow(), Aff aff = Aff()) {
  const F Z = cst(WC_SSWU_Z), A = cst(WC_SSWU_A), B = cst(WC_SSWU_B), one = cst(WC_ONE2);
  F zu2[2], den[2];
  for (int m = 0; m < 2; m++) {
    zu2[m] = dot(sqr2(u[m]), Z);
    den[m] = dot(zu2[m], zu2[m], zu2[m], one);  // Z^2 u^4 + Z u^2
  }
  const F ndr = select_halves(1u, norm_dup(den[0]), norm_dup(den[1]));
  const uint32_t dz = zero_halves(ndr);
  // x1 = xN / xD: xN = -B/A (den + 1), xD = den; den = 0: x1 = B / (Z A), xD = 1
  F xN[2], xD[2], gxN[2];
  for (int m = 0; m < 2; m++) {
    const bool z = (dz >> m) & 1u;
    xD[m] = z ? one : den[m];
    xN[m] = z ? cst(WC_SSWU_BZA) : dot(cst(WC_SSWU_NBA), den[m], cst(WC_SSWU_NBA), one);
    const F xD2 = sqr2(xD[m]);
    gxN[m] = dot(dot(sqr2(xN[m]), one, A, xD2), xN[m], B, dot(xD[m], xD2));  // (xN^2 + A xD^2) xN + B xD^3
  }
  const F nd = select_halves(dz, cst(WC_ONE_DUP), ndr);  // N(xD)
  aff.start(nd, xN, xD);
  const F np = mulp(select_halves(1u, norm_dup(gxN[0]), norm_dup(gxN[1])), nd);
  const F r1p = mulp(pw(np), np);
  const uint32_t sq1 = zero_halves(sub<0>(sqrp(r1p), np));
  const SswuAff af = aff.get();
  // r1: a root of N(gx1) when it is a square (r1^2 = -N(gx1) otherwise, as with the direct form)
  const F r1 = mulp(r1p, sqrp(af.ndi));
  // r2 = N(u)^3 sqrt(-N(Z)^3) r1 (the root for gx2 = (Z u^2)^3 gx1 when N(gx1) is not a square)
  const F nu = select_halves(1u, norm_dup(u[0]), norm_dup(u[1]));
  const F r2 = mulp(mulp(mulp(sqrp(nu), nu), cst(WC_SSWU_SQRT_MNZ3)), r1);
  const F s = select_halves(sq1, r1, r2);
  F gx[2];
  for (int m = 0; m < 2; m++) {
    const bool q = (sq1 >> m) & 1u;
    const F x2 = dot(zu2[m], af.x1[m]);
    xo[m] = q ? af.x1[m] : x2;
    gx[m] = q ? af.gx1[m] : dot(dot(sqr2(zu2[m]), zu2[m]), af.gx1[m]);
  }
  // sqrt of gx through the norm root s (tower.h fp2_sqrt_with_norm_root), both maps, both
  // candidates (a0 + s)/2 and (a0 - s)/2 -- per map the second replaces the first when it is 0
  const F a0 = pair_c0(gx[0], gx[1]), a1 = pair_c1(gx[0], gx[1]);
  F ap = half(add(a0, s));
  const F am = half(sub<0>(a0, s));
  ap = select_halves(zero_halves(ap), am, ap);
  const F w = pw(ap);
  const F t = mulp(w, ap);
  const uint32_t direct = zero_halves(sub<1>(sqrp(t), ap));
  const F inv2t = half(select_halves(direct, w, neg<0>(w)));
  const F other = mulp(a1, inv2t);
  const F c0s = select_halves(direct, t, other), c1s = select_halves(direct, other, t);
  for (int m = 0; m < 2; m++) {
    F y = fp2_of_pairs(c0s, c1s, m);
    if (sgn0_fp2(u[m]) != sgn0_fp2(y)) y = neg<0>(y);
    yo[m] = y;
  }
}

// RFC 9380 E.3 3-isogeny E2' -> E2 into Jacobian coordinates (hash.h iso_map_g2)
WVI G2J iso_map(const F& x, const F& y) {
  const F one = cst(WC_ONE2);
  auto horner = [&](int c_top, int n) {  // c[n-1] x^(n-1) + ... + c[0]
    F r = cst(c_top + n - 1);
    for (int i = n - 2; i >= 0; i--) r = dot(r, x, cst(c_top + i), one);
    return r;
  };
  const F xn = horner(WC_ISO_XNUM0, 4), yn = horner(WC_ISO_YNUM0, 4);
  const F xd = dot(add(x, cst(WC_ISO_XDEN1)), x, cst(WC_ISO_XDEN0), one);  // monic
  const F yd = dot(dot(add(x, cst(WC_ISO_YDEN2)), x, cst(WC_ISO_YDEN1), one), x, cst(WC_ISO_YDEN0), one);
  const F Z = dot(xd, yd);
  const F yd2 = sqr2(yd);
  const F X = dot(dot(xn, xd), yd2);
  const F xd3 = dot(sqr2(xd), xd);
  const F Y = dot(dot(y, yn), dot(xd3, yd2));
  return {X, Y, Z};  // Z == 0 (the isogeny's kernel) is the point at infinity
}

// the sum of the two mapped points (before the cofactor clearing) from the message's xmd b_0
template <class Pow = PowSelf, class Aff = AffSelf>
WVI G2J hash_to_curve_sum(const uint32_t (&b0)[8], Pow pw = Pow(), Aff aff = Aff()) {
  uint32_t e[4][16];
  xmd_words(b0, e);
  const F u[2] = {fp2_from_be512(e[0], e[1]), fp2_from_be512(e[2], e[3])};
  F x[2], y[2];
  WV_MARK(10);
  sswu2(u, x, y, pw, aff);
  WV_MARK(11);
  const G2J q = g2_add(iso_map(x[0], y[0]), iso_map(x[1], y[1]));
  WV_MARK(12);
  return q;
}

// H(msg) affine from the message's xmd b_0; returns false for the point at infinity (inactive pair)
WVI bool hash_to_g2(const uint32_t (&b0)[8], F& hx, F& hy) {
  const G2J h = g2_clear_cofactor(hash_to_curve_sum(b0));
  WV_MARK(13);
  if (g2_is_inf(h)) return false;
  g2_to_affine(h, hx, hy);
  return true;
}

// ------------------------------------------------------------------ G2 decompression
// 96-byte compressed point (wave-uniform bytes) -> affine (x, y), kilic FromCompressed check order;
// with subgroup = false the final subgroup check is left to the caller (wvteam.h runs it beside the
// signature's Miller loop)
template <class Pow = PowSelf>
WVI uint8_t g2_decompress(const uint8_t* in, F& ox, F& oy, bool& is_inf, bool subgroup = true, Pow pw = Pow()) {
  is_inf = false;
  const uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return bls::REJ_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = (b0 != 0xc0);
    for (int i = 1; i < 96; i++) acc |= in[i];
    if (acc) return bls::REJ_INF_NONZERO;
    is_inf = true;
    return bls::REJ_OK;
  }
  const bool sign = (b0 & 0x20) != 0;
  // x.c1 = bytes 0..47 (flags masked), x.c0 = bytes 48..95, big-endian: lane k of half h takes
  // bits 25k .. 25k+24 of its coordinate
  const V l = lane_id(), k = l & 15u, h = l >> 5;
  const M live = (l & 16u) == 0u;
  V limbs = vsplat(0);
  for (int c = 0; c < 2; c++) {  // c = half: 0 -> bytes 48..95 (c0), 1 -> bytes 0..47 (c1)
    const uint8_t* src = in + (c == 0 ? 48 : 0);
    uint32_t wd[13];  // little-endian 32-bit words of the 384-bit field, + 1 zero word
    for (int i = 0; i < 12; i++) {
      const uint8_t* q = src + 44 - 4 * i;
      wd[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
    }
    if (c == 1) wd[11] &= 0x1fffffffu;
    wd[12] = 0;
    V v = vsplat(0);
    for (int kk = 0; kk < 16; kk++) {
      const int bit = 25 * kk, wi = bit >> 5, sh = bit & 31;
      const uint32_t lo = wd[wi], hi = wi + 1 < 13 ? wd[wi + 1] : 0u;
      const uint32_t val = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & M25;
      v = sel(k == (uint32_t)kk, vsplat(val), v);
    }
    limbs = sel(live & (h == (uint32_t)c), v, limbs);
  }
  const V p = cword(WC_P_DUP);
  if (ge_halves(limbs, p) != 0) return bls::REJ_X_GE_P;
  const F x = mulp(mkF(limbs, 1.0), cst(WC_R2_DUP));
  const F rhs = dot(sqr2(x), x, cst(WC_B2), cst(WC_ONE2));  // x^3 + b'
  // sqrt through the norm: s = n^((p+1)/4) = w n, n a square iff s^2 == n
  const F n = norm_dup(rhs);
  const F s = mulp(pw(n), n);
  bool ok = zero_halves(sub<0>(sqrp(s), n)) == 3u;
  // candidates [(a0 + s)/2 | (a0 - s)/2], both exponentiated at once; the second when the first is 0
  const F a0 = dup0(rhs);
  const F cand = half(select_halves(1u, add(a0, s), sub<0>(a0, s)));
  const F wc = pw(cand);
  const int pick = (zero_halves(cand) & 1u) ? 1 : 0;
  const F ap = pick ? dup1(cand) : dup0(cand);
  const F w = pick ? dup1(wc) : dup0(wc);
  const F t = mulp(w, ap);
  const bool direct = (zero_halves(sub<1>(sqrp(t), ap)) & 1u) != 0;
  const F inv2t = half(direct ? w : neg<0>(w));
  const F other = mulp(dup1(rhs), inv2t);
  F y = direct ? select_halves(1u, t, other) : select_halves(1u, other, t);
  ok = ok & is_zero2(sub<0>(sqr2(y), rhs));
  if (!ok) return bls::REJ_NOT_ON_CURVE;
  // ZCash sign: y lexicographically largest (c1 decides unless it is 0)
  const V yr = raw_canon(y);
  const uint32_t gt = ge_halves(yr, cword(WC_PP1H_DUP));
  const uint64_t nz = ballot(((l & 16u) == 0u) & (yr != 0u));
  const bool largest = half_bits(nz, 1) != 0 ? ((gt >> 1) & 1u) != 0 : (gt & 1u) != 0;
  if (largest != sign) y = mul2(y, cst(WC_NEG1));  // -y, reduced (a later subtrahend)
  WV_MARK(14);
  if (subgroup && !g2_in_subgroup({x, y, cst(WC_ONE2)})) return bls::REJ_NOT_IN_SUBGROUP;
  ox = x;
  oy = y;
  return bls::REJ_OK;
}

}  // namespace wv

// Extension-field tower for BLS12-381 on gfx950, register resident:
//   Fp2  = Fp[i]  / (i^2 + 1)
//   Fp6  = Fp2[v] / (v^3 - xi),  xi = 1 + i
//   Fp12 = Fp6[w] / (w^2 - v)
// Replaces kilic/bls12-381 fp2.go / fp6.go / fp12.go ([ext]).
// Element sum_k c_k w^k (k = 0..5) maps to c0 = (c_0, c_2, c_4), c1 = (c_1, c_3, c_5).
#pragma once
#include "fp.h"

namespace bls {

struct fp2 {
  fp c0, c1;
};
struct fp6 {
  fp2 c0, c1, c2;
};
struct fp12 {
  fp6 c0, c1;
};

// ---------------------------------------------------------------- Fp2
DI fp2 fp2_load_const(const uint32_t (&c)[2][12]) { return {fp_load_const(c[0]), fp_load_const(c[1])}; }
DI fp2 fp2_zero() { return {fp_zero(), fp_zero()}; }
DI fp2 fp2_one() { return {fp_one(), fp_zero()}; }
DI bool fp2_is_zero(const fp2& a) { return fp_is_zero(a.c0) & fp_is_zero(a.c1); }
DI bool fp2_eq(const fp2& a, const fp2& b) { return fp_eq(a.c0, b.c0) & fp_eq(a.c1, b.c1); }
DI fp2 fp2_select(bool c, const fp2& a, const fp2& b) { return {fp_select(c, a.c0, b.c0), fp_select(c, a.c1, b.c1)}; }
// Fp2 additive operations as four interleaved carry chains (both components' sum and correction):
// three independent links separate any two dependent ones, so no carry link waits (fp.h fp_add)
DI fp2 fp2_add(const fp2& a, const fp2& b) {
  uint32_t s0[12], d0[12], s1[12], d1[12];
  unsigned c0 = 0, b0 = 0, c1 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    s0[i] = __builtin_addc(a.c0.l[i], b.c0.l[i], c0, &c0);
    s1[i] = __builtin_addc(a.c1.l[i], b.c1.l[i], c1, &c1);
    d0[i] = __builtin_subc(s0[i], P2_RAW[i], b0, &b0);
    d1[i] = __builtin_subc(s1[i], P2_RAW[i], b1, &b1);
  }
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = b0 ? s0[i] : d0[i];
    r.c1.l[i] = b1 ? s1[i] : d1[i];
  }
  return r;
}
// unreduced sum (< 4p for inputs < 2p; < 8p for two levels): only as a multiplier operand (fp.h
// operand contract)
DI fp2 fp2_add_lazy(const fp2& a, const fp2& b) {  // the two components' chains interleaved (fp.h)
  fp2 r;
  unsigned c0 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = __builtin_addc(a.c0.l[i], b.c0.l[i], c0, &c0);
    r.c1.l[i] = __builtin_addc(a.c1.l[i], b.c1.l[i], c1, &c1);
  }
  return r;
}
DI fp2 fp2_dbl(const fp2& a) { return fp2_add(a, a); }
DI fp2 fp2_sub(const fp2& a, const fp2& b) {
  uint32_t d0[12], e0[12], d1[12], e1[12];
  unsigned b0 = 0, c0 = 0, b1 = 0, c1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    d0[i] = __builtin_subc(a.c0.l[i], b.c0.l[i], b0, &b0);
    d1[i] = __builtin_subc(a.c1.l[i], b.c1.l[i], b1, &b1);
    e0[i] = __builtin_addc(d0[i], P2_RAW[i], c0, &c0);
    e1[i] = __builtin_addc(d1[i], P2_RAW[i], c1, &c1);
  }
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = b0 ? e0[i] : d0[i];
    r.c1.l[i] = b1 ? e1[i] : d1[i];
  }
  return r;
}
DI fp2 fp2_addsub(const fp2& a, const fp2& b, bool sub) {  // fp.h fp_addsub on both components, interleaved
  const uint32_t m = sub ? 0xffffffffu : 0u;
  uint32_t s0[12], d0[12], s1[12], d1[12];
  unsigned c0 = sub ? 1u : 0u, e0 = sub ? 0u : 1u, c1 = c0, e1 = e0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    s0[i] = __builtin_addc(a.c0.l[i], b.c0.l[i] ^ m, c0, &c0);
    s1[i] = __builtin_addc(a.c1.l[i], b.c1.l[i] ^ m, c1, &c1);
    d0[i] = __builtin_addc(s0[i], P2_RAW[i] ^ ~m, e0, &e0);
    d1[i] = __builtin_addc(s1[i], P2_RAW[i] ^ ~m, e1, &e1);
  }
  const bool t0 = sub ? (c0 == 0u) : (e0 != 0u), t1 = sub ? (c1 == 0u) : (e1 != 0u);
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = t0 ? d0[i] : s0[i];
    r.c1.l[i] = t1 ? d1[i] : s1[i];
  }
  return r;
}
// 3u + 2x (sub = false) or 3u - 2x (sub = true) per component, for u, x in [0, 2p), the result in
// [0, 2p): the Granger-Scott post-square combination (tri.h tri_cyclotomic_sqr) as one linear form and
// ONE reduction by an estimated multiple of p, instead of fp2_addsub + fp2_dbl + fp2_add (three):
//   y = sub ? 2p - x : x              in [0, 2p]
//   t = 2(u + y) + u                  in [0, 10p): 385 bits, hi = the carry out of word 11
//   q = floor(T / D), T = t >> 352 (33 bits), D = P11 + 1 (p's top word + 1): a float estimate that
//       is q or q - 1, then one exact 64-bit comparison
//   r = t - q p                       (q p from KP: a MAD chain, or tri.h's LDS table of k p)
// r >= 0: q p <= T p / D < T 2^352 <= t (p < D 2^352). r < 2p: q > T/D - 1 and p >= P11 2^352 give
// t - q p < 2^352 (T/D + 1) + p <= 11 * 2^352 + p (T/D < 10), and 11 * 2^352 < p / 10^7.
DI uint32_t fp_quot_top(const uint32_t (&t)[12], uint32_t hi) {
  constexpr uint32_t D = P_RAW[11] + 1u;
  // float(T) is within 2^10 of T and the product within 2^-22 relative: the estimate is within
  // 4e-6 of T / D, so subtracting 1e-4 makes it floor(T / D) or one less (clamped at 0)
  float e = ((float)t[11] + (float)hi * 4294967296.0f) * (1.0f / (float)D) - 1e-4f;
  e = e > 0.0f ? e : 0.0f;
  uint32_t q = (uint32_t)e;
  const uint64_t T = ((uint64_t)hi << 32) | t[11];
  return q + (T >= (uint64_t)(q + 1u) * D ? 1u : 0u);
}
// q p as 12 words (q <= 10: < 11p < 2^385, the 13th word is not needed: t - q p < 2^384) by a MAD
// chain; tri.h reads it from an LDS table instead
struct KpMad {
  DI u12 operator()(uint32_t q) const {
    u12 w;
    uint64_t k = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      k = (uint64_t)q * P_RAW[i] + (k >> 32);
      w[i] = (uint32_t)k;
    }
    return w;
  }
};
// N components at once (the cyclotomic square passes all four of its outputs): every carry chain is
// written interleaved across the N components, so no chain link waits for its predecessor (fp.h)
template <int N, typename KP = KpMad>
DI void fp_3u_pm_2x_n(const fp (&u)[N], const fp (&x)[N], const bool (&sub)[N], fp (&r)[N], KP kp = KP()) {
  uint32_t y[N][12];
  {
    uint32_t d[N][12];
    unsigned b[N];
#pragma unroll
    for (int c = 0; c < N; c++) b[c] = 0;
#pragma unroll
    for (int i = 0; i < 12; i++)
#pragma unroll
      for (int c = 0; c < N; c++) d[c][i] = __builtin_subc(P2_RAW[i], x[c].l[i], b[c], &b[c]);
#pragma unroll
    for (int i = 0; i < 12; i++)
#pragma unroll
      for (int c = 0; c < N; c++) y[c][i] = sub[c] ? d[c][i] : x[c].l[i];
  }
  uint32_t t[N][12];
  unsigned h[N];
  {
    uint32_t w[N][12];
    unsigned cs[N], cw[N];
#pragma unroll
    for (int c = 0; c < N; c++) cs[c] = cw[c] = h[c] = 0;
#pragma unroll
    for (int i = 0; i < 12; i++)
#pragma unroll
      for (int c = 0; c < N; c++) {  // s = u + y < 4p, 2s < 8p < 2^384: no carry out of either
        const uint32_t si = __builtin_addc(u[c].l[i], y[c][i], cs[c], &cs[c]);
        w[c][i] = __builtin_addc(si, si, cw[c], &cw[c]);
      }
#pragma unroll
    for (int i = 0; i < 12; i++)
#pragma unroll
      for (int c = 0; c < N; c++) t[c][i] = __builtin_addc(w[c][i], u[c].l[i], h[c], &h[c]);
  }
  u12 qp[N];
#pragma unroll
  for (int c = 0; c < N; c++) qp[c] = kp(fp_quot_top(t[c], h[c]));
  unsigned b[N];
#pragma unroll
  for (int c = 0; c < N; c++) b[c] = 0;
#pragma unroll
  for (int i = 0; i < 12; i++)
#pragma unroll
    for (int c = 0; c < N; c++) r[c].l[i] = __builtin_subc(t[c][i], qp[c][i], b[c], &b[c]);
}
template <typename KP = KpMad>
DI fp2 fp2_3u_pm_2x(const fp2& u, const fp2& x, bool sub, KP kp = KP()) {
  const fp uu[2] = {u.c0, u.c1}, xx[2] = {x.c0, x.c1};
  const bool ss[2] = {sub, sub};
  fp r[2];
  fp_3u_pm_2x_n<2>(uu, xx, ss, r, kp);
  return {r[0], r[1]};
}

DI fp2 fp2_neg(const fp2& a) {  // fp_neg per component, the two chains interleaved
  uint32_t d0[12], d1[12];
  unsigned b0 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    d0[i] = __builtin_subc(P2_RAW[i], a.c0.l[i], b0, &b0);
    d1[i] = __builtin_subc(P2_RAW[i], a.c1.l[i], b1, &b1);
  }
  const uint32_t m0 = fp_raw_is_zero(a.c0) ? 0u : 0xffffffffu, m1 = fp_raw_is_zero(a.c1) ? 0u : 0xffffffffu;
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = d0[i] & m0;
    r.c1.l[i] = d1[i] & m1;
  }
  return r;
}
DI fp2 fp2_conj(const fp2& a) { return {a.c0, fp_neg(a.c1)}; }

DI u24 fp2_to_u24(const fp2& a) { return u24_of(fp_to_u12(a.c0), fp_to_u12(a.c1)); }
DI fp2 fp2_from_u24(const u24& v) { return {fp_from_u12(u24_lo(v)), fp_from_u12(u24_hi(v))}; }

// one fused call each (fp.h fp2_mul_u24 / fp2_sqr_u24): 3 and 2 Fp-mul equivalents
DI fp2 fp2_mul(const fp2& a, const fp2& b) {
  fp2_arg_store(fp2_to_u24(b));
  return fp2_from_u24(fp2_mul_u24(fp2_to_u24(a)));
}
DI fp2 fp2_sqr(const fp2& a) { return fp2_from_u24(fp2_sqr_u24(fp2_to_u24(a))); }
// in-place expansions (no call): for call-free kernels whose register budget must stay small
template <bool KARA>
DI fp2 fp2_mul_inl_t(const fp2& a, const fp2& b) {
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  return fp2_from_u24(fp2_mul_body_t<KARA>(fp2_to_u24(a), fp_to_u12(b.c0), fp_to_u12(b.c1)));
}
DI fp2 fp2_mul_inl(const fp2& a, const fp2& b) { return fp2_mul_inl_t<BLS_FP2_KARA_INL>(a, b); }
// the Karatsuba body at the Miller doubling step's call sites whose live state leaves room for it:
// BLS_LINES_KARA bit 0 = Z3 = B H, bit 1 = A = X Y / 2 (pairing.h miller_dbl_step_ts)
#ifndef BLS_LINES_KARA
#define BLS_LINES_KARA 3
#endif
template <int SITE>
DI fp2 fp2_mul_inl_k(const fp2& a, const fp2& b) { return fp2_mul_inl_t<((BLS_LINES_KARA >> SITE) & 1) != 0>(a, b); }
DI fp2 fp2_sqr_inl(const fp2& a) {
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  return fp2_from_u24(fp2_sqr_body(fp2_to_u24(a)));
}

DI fp2 fp2_mul_fp(const fp2& a, const fp& b) { return {fp_mul(a.c0, b), fp_mul(a.c1, b)}; }
DI fp2 fp2_mul_fp_inl(const fp2& a, const fp& b) {
  const fp c0 = fp_mul_inl(a.c0, b);
  BLS_SCHED_FENCE();
  return {c0, fp_mul_inl(a.c1, b)};
}
DI fp2 fp2_mul3(const fp2& a) { return {fp_mul3(a.c0), fp_mul3(a.c1)}; }

// multiply by xi = 1 + i: (a0 - a1) + (a0 + a1) i
DI fp2 fp2_mul_xi(const fp2& a) {  // (a0 - a1, a0 + a1): four interleaved chains as fp2_sub / fp2_add
  uint32_t d[12], e[12], s[12], u[12];
  unsigned bd = 0, ce = 0, cs = 0, bu = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    d[i] = __builtin_subc(a.c0.l[i], a.c1.l[i], bd, &bd);
    s[i] = __builtin_addc(a.c0.l[i], a.c1.l[i], cs, &cs);
    e[i] = __builtin_addc(d[i], P2_RAW[i], ce, &ce);
    u[i] = __builtin_subc(s[i], P2_RAW[i], bu, &bu);
  }
  fp2 r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = bd ? e[i] : d[i];
    r.c1.l[i] = bu ? s[i] : u[i];
  }
  return r;
}

DI fp2 fp2_inv(const fp2& a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp ni = fp_inv(n);
  return {fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni))};
}

// ZCash/RFC helpers on Montgomery values
DI bool fp2_sgn0(const fp2& a) {  // RFC 9380 sgn0 for Fp2
  fp r0 = fp_from_mont(a.c0);
  fp r1 = fp_from_mont(a.c1);
  bool s0 = r0.l[0] & 1u;
  bool z0 = fp_is_zero(r0);
  bool s1 = r1.l[0] & 1u;
  return s0 | (z0 & s1);
}

DI bool fp2_lex_largest(const fp2& a) {  // ZCash sign bit rule for y
  fp r1 = fp_from_mont(a.c1);
  if (!fp_is_zero(r1)) return fp_raw_gt_half(r1);
  return fp_raw_gt_half(fp_from_mont(a.c0));
}

// Square root in Fp2 through the norm (p = 3 mod 4). a is a square in Fp2 iff its norm
// n = a0^2 + a1^2 is a square in Fp. Given s with s^2 = n:
//   a' = (a0 + s)/2 (or (a0 - s)/2 if that is 0); w = a'^((p-3)/4), t = w a':
//   t^2 == a'  -> root (t, a1/(2t)),  1/t = w
//   t^2 == -a' -> root (a1/(2t), t),  1/t = -w      (a1^2 = 2a'(s - a0) makes both work)
// so the second exponentiation yields the root AND the inverse it needs. Branch-free.
DI fp2 fp2_sqrt_with_norm_root(const fp2& a, const fp& s) {
  fp ap = fp_half(fp_add(a.c0, s));
  fp am = fp_half(fp_sub(a.c0, s));
  ap = fp_select(fp_is_zero(ap), am, ap);
  fp w = fp_pow_sqrt_inv(ap);
  fp t = fp_mul(w, ap);
  bool direct = fp_eq(fp_sqr(t), ap);
  fp inv2t = fp_half(fp_select(direct, w, fp_neg(w)));
  fp other = fp_mul(a.c1, inv2t);
  return {fp_select(direct, t, other), fp_select(direct, other, t)};
}

DI fp fp2_norm(const fp2& a) { return fp_add(fp_sqr(a.c0), fp_sqr(a.c1)); }

// root of the norm n: s = n^((p+1)/4) = w n; is_sq iff s^2 == n (else s^2 == -n)
DI fp fp_norm_root(const fp& n, bool& is_sq) {
  fp s = fp_mul(fp_pow_sqrt_inv(n), n);
  is_sq = fp_eq(fp_sqr(s), n);
  return s;
}

// Returns false if a is not a square (out is then garbage). Two Fp exponentiations.
DI bool fp2_sqrt(fp2& out, const fp2& a) {
  bool ok;
  fp s = fp_norm_root(fp2_norm(a), ok);
  fp2 r = fp2_sqrt_with_norm_root(a, s);
  ok = ok & fp2_eq(fp2_sqr(r), a);
  out = r;
  return ok;
}

DI fp2 fp2_half(const fp2& a) { return {fp_half(a.c0), fp_half(a.c1)}; }

// ---------------------------------------------------------------- Fp6
DI fp6 fp6_zero() { return {fp2_zero(), fp2_zero(), fp2_zero()}; }
DI fp6 fp6_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }
DI fp6 fp6_add(const fp6& a, const fp6& b) { return {fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)}; }
DI fp6 fp6_sub(const fp6& a, const fp6& b) { return {fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)}; }
DI fp6 fp6_neg(const fp6& a) { return {fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)}; }
DI bool fp6_eq(const fp6& a, const fp6& b) { return fp2_eq(a.c0, b.c0) & fp2_eq(a.c1, b.c1) & fp2_eq(a.c2, b.c2); }

// multiply by v: (a0 + a1 v + a2 v^2) v = xi a2 + a0 v + a1 v^2
DI fp6 fp6_mul_v(const fp6& a) { return {fp2_mul_xi(a.c2), a.c0, a.c1}; }

// ---- linear forms with one reduction (BLS_F6_LIN): an output that is a signed sum of Fp values
// in [0, 2p) is formed as T = P + (k p - N) from two lazily added sums P, N < 2^384 (N < k p) and
// reduced ONCE by q p, q = floor(T / 2^352 / (P11 + 1)) (fp_quot_top, T < 16p so q <= 15), instead
// of one conditional correction per addition, subtraction and multiplication by xi. KP supplies q p.
#ifndef BLS_F6_LIN
#define BLS_F6_LIN 1
#endif
struct Words12 {
  uint32_t w[12];
};
constexpr Words12 kp_words(uint32_t k) {
  Words12 r{};
  uint64_t c = 0;
  for (int i = 0; i < 12; i++) {
    c = (uint64_t)k * P_RAW[i] + (c >> 32);
    r.w[i] = (uint32_t)c;
  }
  return r;
}
#ifndef BLS_HOST
// k p for k < K in LDS, one copy per workgroup (16-byte aligned rows of 3 uint4): the q p of the
// one-reduction linear forms read per lane (3 ds_read_b128) instead of a 12-MAD chain.
// kp_lds_init<K>() runs once per workgroup, reached by every lane, before the first use.
template <int K>
DI uint32_t* kp_lds_tab() {
  static __shared__ __attribute__((aligned(16))) uint32_t tab[K * 12];
  return tab;
}
template <int K>
DI void kp_lds_init() {
  uint32_t* tab = kp_lds_tab<K>();
  for (unsigned j = threadIdx.x; j < (unsigned)K * 12u; j += blockDim.x) {
    const uint32_t k = j / 12u, word = j % 12u;
    uint64_t c = 0;
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      c = (uint64_t)k * P_RAW[i] + (c >> 32);
      if ((uint32_t)i == word) w = (uint32_t)c;
    }
    tab[j] = w;
  }
  __syncthreads();
}
template <int K>
struct KpLdsK {
  DI u12 operator()(uint32_t q) const {
    q = q < (uint32_t)(K - 1) ? q : (uint32_t)(K - 1);  // in range by the operand bounds; kept in the table
    const uint4* r = reinterpret_cast<const uint4*>(kp_lds_tab<K>()) + 3u * q;
    const uint4 a = r[0], b = r[1], c = r[2];
    u12 w;
    w[0] = a.x, w[1] = a.y, w[2] = a.z, w[3] = a.w, w[4] = b.x, w[5] = b.y;
    w[6] = b.z, w[7] = b.w, w[8] = c.x, w[9] = c.y, w[10] = c.z, w[11] = c.w;
    return w;
  }
};
#endif

// the last step of every linear form: r_j = T_j - q_j p for the 385-bit T_j (hi_j = bit 384)
template <typename KP>
DI fp2 fp2_lin_reduce(const uint32_t (&t0)[12], unsigned h0, const uint32_t (&t1)[12], unsigned h1, KP kp) {
  const u12 w0 = kp(fp_quot_top(t0, h0)), w1 = kp(fp_quot_top(t1, h1));
  fp2 r;
  unsigned b0 = 0, b1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    r.c0.l[i] = __builtin_subc(t0[i], w0[i], b0, &b0);
    r.c1.l[i] = __builtin_subc(t1[i], w1[i], b1, &b1);
  }
  return r;
}
// The Karatsuba Fp6 outputs from its six Fp2 products (t_j = a_j b_j, m_jk = (a_j + a_k)(b_j + b_k),
// every component in [0, 2p)):
//   c0 = xi (m12 - t1 - t2) + t0,  c1 = m01 - t0 - t1 + xi t2,  c2 = m02 - t0 - t2 + t1
// with xi (x + y i) = (x - y) + (x + y) i written out per component (u = t1 + t2):
//   c0 = (m12_0 + u_1 + t0_0 + 6p - (m12_1 + u_0),      m12_0 + m12_1 + t0_1 + 8p - (u_0 + u_1))
//   c1 = (m01_0 + t2_0 + 6p - (t0_0 + t1_0 + t2_1),      m01_1 + t2_0 + t2_1 + 4p - (t0_1 + t1_1))
//   c2 = (m02_0 + t1_0 + 4p - (t0_0 + t2_0),             m02_1 + t1_1 + 4p - (t0_1 + t2_1))
// Every partial sum stays below 8p < 2^384 and every T below 14p (q <= 13). The sums run as four to
// six carry chains interleaved word by word: a carry link then never waits for the previous one
// (two interleaved chains still cost an s_nop per link on gfx950).
template <typename KP>
DI fp2 kara6_c0(const fp2& m12, const fp2& t0, const fp2& t1, const fp2& t2, KP kp) {
  constexpr Words12 B0 = kp_words(6), B1 = kp_words(8);
  uint32_t pa0[12], pa1[12], na0[12], na1[12];
  {
    unsigned cu0 = 0, cu1 = 0, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint32_t u0 = __builtin_addc(t1.c0.l[i], t2.c0.l[i], cu0, &cu0);
      const uint32_t u1 = __builtin_addc(t1.c1.l[i], t2.c1.l[i], cu1, &cu1);
      pa0[i] = __builtin_addc(m12.c0.l[i], u1, c0, &c0);
      pa1[i] = __builtin_addc(m12.c0.l[i], m12.c1.l[i], c1, &c1);
      na0[i] = __builtin_addc(m12.c1.l[i], u0, c2, &c2);
      na1[i] = __builtin_addc(u0, u1, c3, &c3);
    }
  }
  uint32_t T0[12], T1[12];
  unsigned h0 = 0, h1 = 0;
  {
    unsigned c0 = 0, c1 = 0, b0 = 0, b1 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint32_t p0 = __builtin_addc(pa0[i], t0.c0.l[i], c0, &c0);
      const uint32_t p1 = __builtin_addc(pa1[i], t0.c1.l[i], c1, &c1);
      const uint32_t n0 = __builtin_subc(B0.w[i], na0[i], b0, &b0);
      const uint32_t n1 = __builtin_subc(B1.w[i], na1[i], b1, &b1);
      T0[i] = __builtin_addc(p0, n0, h0, &h0);
      T1[i] = __builtin_addc(p1, n1, h1, &h1);
    }
  }
  return fp2_lin_reduce(T0, h0, T1, h1, kp);
}
template <typename KP>
DI fp2 kara6_c1(const fp2& m01, const fp2& t0, const fp2& t1, const fp2& t2, KP kp) {
  constexpr Words12 B0 = kp_words(6), B1 = kp_words(4);
  uint32_t pa0[12], pa1[12], na0[12], na1[12];
  {
    unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      pa0[i] = __builtin_addc(m01.c0.l[i], t2.c0.l[i], c0, &c0);
      pa1[i] = __builtin_addc(m01.c1.l[i], t2.c0.l[i], c1, &c1);
      na0[i] = __builtin_addc(t0.c0.l[i], t1.c0.l[i], c2, &c2);
      na1[i] = __builtin_addc(t0.c1.l[i], t1.c1.l[i], c3, &c3);
    }
  }
  uint32_t T0[12], T1[12];
  unsigned h0 = 0, h1 = 0;
  {
    unsigned c1 = 0, c2 = 0, b0 = 0, b1 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint32_t p1 = __builtin_addc(pa1[i], t2.c1.l[i], c1, &c1);
      const uint32_t m0 = __builtin_addc(na0[i], t2.c1.l[i], c2, &c2);
      const uint32_t n0 = __builtin_subc(B0.w[i], m0, b0, &b0);
      const uint32_t n1 = __builtin_subc(B1.w[i], na1[i], b1, &b1);
      T0[i] = __builtin_addc(pa0[i], n0, h0, &h0);
      T1[i] = __builtin_addc(p1, n1, h1, &h1);
    }
  }
  return fp2_lin_reduce(T0, h0, T1, h1, kp);
}
template <typename KP>
DI fp2 kara6_c2(const fp2& m02, const fp2& t0, const fp2& t1, const fp2& t2, KP kp) {
  constexpr Words12 B = kp_words(4);
  uint32_t T0[12], T1[12];
  unsigned h0 = 0, h1 = 0;
  {
    unsigned c0 = 0, c1 = 0, c2 = 0, c3 = 0, b0 = 0, b1 = 0;
#pragma unroll
    for (int i = 0; i < 12; i++) {
      const uint32_t p0 = __builtin_addc(m02.c0.l[i], t1.c0.l[i], c0, &c0);
      const uint32_t p1 = __builtin_addc(m02.c1.l[i], t1.c1.l[i], c1, &c1);
      const uint32_t s0 = __builtin_addc(t0.c0.l[i], t2.c0.l[i], c2, &c2);
      const uint32_t s1 = __builtin_addc(t0.c1.l[i], t2.c1.l[i], c3, &c3);
      const uint32_t n0 = __builtin_subc(B.w[i], s0, b0, &b0);
      const uint32_t n1 = __builtin_subc(B.w[i], s1, b1, &b1);
      T0[i] = __builtin_addc(p0, n0, h0, &h0);
      T1[i] = __builtin_addc(p1, n1, h1, &h1);
    }
  }
  return fp2_lin_reduce(T0, h0, T1, h1, kp);
}

// fp6_mul with one reduction per output component; b's components through lb(c) (k_miller.hip reads
// them from LDS)
template <typename LB, typename KP>
DI fp6 fp6_mul_lin_lb(const fp6& a, LB lb, KP kp) {
  const fp2 t0 = fp2_mul(a.c0, lb(0));
  const fp2 t1 = fp2_mul(a.c1, lb(1));
  const fp2 t2 = fp2_mul(a.c2, lb(2));
  const fp2 c0 = kara6_c0(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(lb(1), lb(2))), t0, t1, t2, kp);
  const fp2 c1 = kara6_c1(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(lb(0), lb(1))), t0, t1, t2, kp);
  const fp2 c2 = kara6_c2(fp2_mul(fp2_add_lazy(a.c0, a.c2), fp2_add_lazy(lb(0), lb(2))), t0, t1, t2, kp);
  return {c0, c1, c2};
}
template <typename KP = KpMad>
DI fp6 fp6_mul_lin(const fp6& a, const fp6& b, KP kp = KP()) {
  return fp6_mul_lin_lb(a, [&](int c) { return c == 0 ? b.c0 : (c == 1 ? b.c1 : b.c2); }, kp);
}

DI fp6 fp6_mul(const fp6& a, const fp6& b) {  // Karatsuba, 6 Fp2 mul, a reduction per operation
  fp2 t0 = fp2_mul(a.c0, b.c0);
  fp2 t1 = fp2_mul(a.c1, b.c1);
  fp2 t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(b.c1, b.c2)), t1), t2)), t0);
  fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(b.c0, b.c1)), t0), t1), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c2), fp2_add_lazy(b.c0, b.c2)), t0), t2), t1);
  return {c0, c1, c2};
}

// fp6 sum for a multiplier input (fp6_mul / fp6_mul_by_* take operands < 2p per coefficient)
DI fp6 fp6_add_lazy(const fp6& a, const fp6& b) {
  return {fp2_add_lazy(a.c0, b.c0), fp2_add_lazy(a.c1, b.c1), fp2_add_lazy(a.c2, b.c2)};
}

DI fp6 fp6_sqr(const fp6& a) {  // CH-SQR2
  fp2 s0 = fp2_sqr(a.c0);
  fp2 ab = fp2_mul(a.c0, a.c1);
  fp2 s1 = fp2_dbl(ab);
  fp2 s2 = fp2_sqr(fp2_add_lazy(fp2_sub(a.c0, a.c1), a.c2));
  fp2 bc = fp2_mul(a.c1, a.c2);
  fp2 s3 = fp2_dbl(bc);
  fp2 s4 = fp2_sqr(a.c2);
  fp2 c0 = fp2_add(fp2_mul_xi(s3), s0);
  fp2 c1 = fp2_add(fp2_mul_xi(s4), s1);
  fp2 c2 = fp2_sub(fp2_sub(fp2_add(fp2_add(s1, s2), s3), s0), s4);
  return {c0, c1, c2};
}

// a * (b0 + b1 v): 5 Fp2 mul
DI fp6 fp6_mul_by_01(const fp6& a, const fp2& b0, const fp2& b1) {
  fp2 t0 = fp2_mul(a.c0, b0);
  fp2 t1 = fp2_mul(a.c1, b1);
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_mul(fp2_add_lazy(a.c1, a.c2), b1), t1)), t0);
  fp2 c1 = fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(b0, b1)), t0), t1);
  fp2 c2 = fp2_add(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c2), b0), t0), t1);
  return {c0, c1, c2};
}

// a * (b1 v): 3 Fp2 mul
DI fp6 fp6_mul_by_1(const fp6& a, const fp2& b1) {
  return {fp2_mul_xi(fp2_mul(a.c2, b1)), fp2_mul(a.c0, b1), fp2_mul(a.c1, b1)};
}

DI fp6 fp6_inv(const fp6& a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return {fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di)};
}

// ---------------------------------------------------------------- Fp12
DI fp12 fp12_one() { return {fp6_one(), fp6_zero()}; }
DI bool fp12_eq(const fp12& a, const fp12& b) { return fp6_eq(a.c0, b.c0) & fp6_eq(a.c1, b.c1); }
DI bool fp12_is_one(const fp12& a) { return fp12_eq(a, fp12_one()); }
DI fp12 fp12_conj(const fp12& a) { return {a.c0, fp6_neg(a.c1)}; }  // a^(p^6)

DI fp12 fp12_mul(const fp12& a, const fp12& b) {  // Karatsuba, 3 Fp6 mul
  fp6 t0 = fp6_mul(a.c0, b.c0);
  fp6 t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add_lazy(a.c0, a.c1), fp6_add_lazy(b.c0, b.c1)), t0), t1);
  fp6 c0 = fp6_add(t0, fp6_mul_v(t1));
  return {c0, c1};
}

// fp12_sqr with the one-reduction Fp6 products (k_miller.hip's f pass, q p from its LDS table)
template <typename KP>
DI fp12 fp12_sqr_lin(const fp12& a, KP kp) {
  fp6 ab = fp6_mul_lin(a.c0, a.c1, kp);
  fp6 t = fp6_mul_lin(fp6_add_lazy(a.c0, a.c1), fp6_add_lazy(a.c0, fp6_mul_v(a.c1)), kp);
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

DI fp12 fp12_sqr(const fp12& a) {  // complex squaring, 2 Fp6 mul
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add_lazy(a.c0, a.c1), fp6_add_lazy(a.c0, fp6_mul_v(a.c1)));
  fp6 c0 = fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab));
  fp6 c1 = fp6_add(ab, ab);
  return {c0, c1};
}

// f * l where l = (l00 + l01 v) + (l11 v) w  (sparse Miller-loop line, slots 0,1,4): 13 Fp2 mul
DI fp12 fp12_mul_by_014(const fp12& f, const fp2& l00, const fp2& l01, const fp2& l11) {
  fp6 a = fp6_mul_by_01(f.c0, l00, l01);
  fp6 b = fp6_mul_by_1(f.c1, l11);
  fp6 c = fp6_mul_by_01(fp6_add_lazy(f.c0, f.c1), l00, fp2_add_lazy(l01, l11));
  fp6 c1 = fp6_sub(fp6_sub(c, a), b);
  fp6 c0 = fp6_add(a, fp6_mul_v(b));
  return {c0, c1};
}

// Granger-Scott squaring for elements of the cyclotomic subgroup (after the easy part of the final
// exponentiation): Fp12 seen as Fp4^3 with Fp4 = Fp2[w^3]; 9 Fp2 squarings (18 Fp mul) instead of
// the 36 of fp12_sqr.
DI void fp4_sqr(fp2& c0, fp2& c1, const fp2& a, const fp2& b) {
  fp2 t0 = fp2_sqr(a);
  fp2 t1 = fp2_sqr(b);
  c0 = fp2_add(fp2_mul_xi(t1), t0);
  c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add_lazy(a, b)), t0), t1);
}

DI fp12 fp12_cyclotomic_sqr(const fp12& f) {
  fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2 t0, t1, t2, t3;
  fp4_sqr(t0, t1, z0, z1);
  z0 = fp2_add(fp2_dbl(fp2_sub(t0, z0)), t0);  // 3 t0 - 2 z0
  z1 = fp2_add(fp2_dbl(fp2_add(t1, z1)), t1);  // 3 t1 + 2 z1
  fp4_sqr(t0, t1, z2, z3);
  fp4_sqr(t2, t3, z4, z5);
  z4 = fp2_add(fp2_dbl(fp2_sub(t0, z4)), t0);
  z5 = fp2_add(fp2_dbl(fp2_add(t1, z5)), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(fp2_dbl(fp2_add(t0, z2)), t0);
  z3 = fp2_add(fp2_dbl(fp2_sub(t2, z3)), t2);
  return {{z0, z4, z3}, {z2, z1, z5}};
}

DI fp12 fp12_inv(const fp12& a) {  // (a0 + a1 w)^-1 = (a0 - a1 w) / (a0^2 - v a1^2)
  fp6 d = fp6_sub(fp6_sqr(a.c0), fp6_mul_v(fp6_sqr(a.c1)));
  fp6 di = fp6_inv(d);
  return {fp6_mul(a.c0, di), fp6_neg(fp6_mul(a.c1, di))};
}

// Frobenius: (sum c_k w^k)^p = sum conj(c_k) gamma1^k w^k; ^(p^2) = sum c_k gamma2^k w^k.
// w-power index of each tower slot: c0.c0->0, c1.c0->1, c0.c1->2, c1.c1->3, c0.c2->4, c1.c2->5
DI fp12 fp12_frob(const fp12& a) {
  fp12 r;
  r.c0.c0 = fp2_conj(a.c0.c0);
  r.c1.c0 = fp2_mul(fp2_conj(a.c1.c0), fp2_load_const(FROB1_GAMMA[1]));
  r.c0.c1 = fp2_mul(fp2_conj(a.c0.c1), fp2_load_const(FROB1_GAMMA[2]));
  r.c1.c1 = fp2_mul(fp2_conj(a.c1.c1), fp2_load_const(FROB1_GAMMA[3]));
  r.c0.c2 = fp2_mul(fp2_conj(a.c0.c2), fp2_load_const(FROB1_GAMMA[4]));
  r.c1.c2 = fp2_mul(fp2_conj(a.c1.c2), fp2_load_const(FROB1_GAMMA[5]));
  return r;
}

DI fp12 fp12_frob2(const fp12& a) {  // gamma2^k lies in Fp
  fp12 r;
  r.c0.c0 = a.c0.c0;
  r.c1.c0 = fp2_mul_fp(a.c1.c0, fp_load_const(FROB2_GAMMA[1][0]));
  r.c0.c1 = fp2_mul_fp(a.c0.c1, fp_load_const(FROB2_GAMMA[2][0]));
  r.c1.c1 = fp2_mul_fp(a.c1.c1, fp_load_const(FROB2_GAMMA[3][0]));
  r.c0.c2 = fp2_mul_fp(a.c0.c2, fp_load_const(FROB2_GAMMA[4][0]));
  r.c1.c2 = fp2_mul_fp(a.c1.c2, fp_load_const(FROB2_GAMMA[5][0]));
  return r;
}

}  // namespace bls

// Fp12 of the latency engine: f = sum_k c_k w^k (k = 0..5, c_k in Fp2, w^6 = xi = 1 + i), i.e. the
// same field as tower.h's Fp2 -> Fp6 -> Fp12 tower (w^2 = v, w^3 = s; tower slot c0.c0 = w^0,
// c1.c0 = w^1, c0.c1 = w^2, c1.c1 = w^3, c0.c2 = w^4, c1.c2 = w^5), written flat so that EVERY output
// coefficient of a product is one dot product of Fp2 terms with one reduction (wfield.h):
//   product    c_k = sum_i a_i b'_{k-i}, b'_j = b_j for j >= 0, xi b_{j+6} for j < 0: 6 dots of 6
//   square     21 distinct terms (cross terms against a doubled operand)
//   line       the sparse Miller line (w^0, w^2, w^3): 6 dots of 3
//   cyclotomic Granger-Scott with the 3t - 2z fix-ups folded in as constant terms: 15 terms
// so every stored coefficient is reduced (< 1.01 p) and no bound grows across loop iterations.
#pragma once
#include "wfield.h"

namespace wv {

struct W12 {
  F c[6];
};

WVI W12 w12_one() {
  W12 r;
  r.c[0] = cst(WC_ONE2);
  for (int k = 1; k < 6; k++) r.c[k] = zero();
  return r;
}

// Every product below is written per output coefficient (..._c(.., k)), so that the waves of a
// team (wteam.h) can each compute a share of the six; the whole-value forms loop over k.

// general product: c_k = sum_i a_i b'_{k-i}, b'_j = xi b_{j+6} for j < 0
WVI F w12_mul_c(const W12& a, const W12& b, int k) {
  auto B = [&](int j) -> F { return j >= 0 ? b.c[j] : mul_xi<1>(b.c[j + 6]); };  // b may be a conjugate
  return dot(a.c[0], B(k), a.c[1], B(k - 1), a.c[2], B(k - 2), a.c[3], B(k - 3), a.c[4], B(k - 4), a.c[5],
             B(k - 5));
}
WVI W12 w12_mul(const W12& a, const W12& b) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_mul_c(a, b, k);
  return r;
}

// square: c_k = sum over unordered {i, j}, i + j = k (mod 6, xi when it wraps): a_i a_j, doubled when
// i != j (the doubled operand 2 a_i sits in the window, a_j or xi a_j is broadcast)
WVI F w12_sqr_c(const W12& a, int k) {
  auto X = [&](int i) { return mul_xi<0>(a.c[i]); };
  auto D = [&](int i) { return dbl(a.c[i]); };
  switch (k) {
    case 0: return dot(a.c[0], a.c[0], D(1), X(5), D(2), X(4), a.c[3], X(3));  // (0,0) (1,5)x (2,4)x (3,3)x
    case 1: return dot(D(0), a.c[1], D(2), X(5), D(3), X(4));                  // (0,1) (2,5)x (3,4)x
    case 2: return dot(D(0), a.c[2], a.c[1], a.c[1], D(3), X(5), a.c[4], X(4));  // (0,2) (1,1) (3,5)x (4,4)x
    case 3: return dot(D(0), a.c[3], D(1), a.c[2], D(4), X(5));                  // (0,3) (1,2) (4,5)x
    case 4: return dot(D(0), a.c[4], D(1), a.c[3], a.c[2], a.c[2], a.c[5], X(5));  // (0,4) (1,3) (2,2) (5,5)x
    default: return dot(D(0), a.c[5], D(1), a.c[4], D(2), a.c[3]);               // (0,5) (1,4) (2,3)
  }
}
WVI W12 w12_sqr(const W12& a) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_sqr_c(a, k);
  return r;
}

// f * l for a Miller line l = l0 + l2 w^2 + l3 w^3 (tower: l00 + l01 v + l11 v w)
WVI F w12_mul_line_c(const W12& f, const F& l0, const F& l2, const F& l3, int k) {
  switch (k) {
    case 0: return dot(f.c[0], l0, f.c[4], mul_xi<0>(l2), f.c[3], mul_xi<0>(l3));
    case 1: return dot(f.c[1], l0, f.c[5], mul_xi<0>(l2), f.c[4], mul_xi<0>(l3));
    case 2: return dot(f.c[2], l0, f.c[0], l2, f.c[5], mul_xi<0>(l3));
    case 3: return dot(f.c[3], l0, f.c[1], l2, f.c[0], l3);
    case 4: return dot(f.c[4], l0, f.c[2], l2, f.c[1], l3);
    default: return dot(f.c[5], l0, f.c[3], l2, f.c[2], l3);
  }
}
WVI W12 w12_mul_line(const W12& f, const F& l0, const F& l2, const F& l3) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_mul_line_c(f, l0, l2, l3, k);
  return r;
}

// f^(p^6): negate the odd powers
WVI W12 w12_conj(const W12& a) {
  W12 r = a;
  r.c[1] = neg<0>(a.c[1]);
  r.c[3] = neg<0>(a.c[3]);
  r.c[5] = neg<0>(a.c[5]);
  return r;
}
// negated odd powers as a dot-ready operand is the same thing; conj output bounds are 4 p (neg)

// f^p: c_k -> conj(c_k) gamma1^k
WVI F w12_frob_c(const W12& a, int k) {
  return k == 0 ? conj<0>(a.c[0]) : mul2(conj<0>(a.c[k]), cst(WC_FROB1_0 + 2 * k));
}
WVI W12 w12_frob(const W12& a) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_frob_c(a, k);
  return r;
}
// f^(p^2): c_k -> c_k gamma2^k (gamma2^k in Fp)
WVI F w12_frob2_c(const W12& a, int k) { return k == 0 ? a.c[0] : mulp(a.c[k], cst(WC_FROB2_0 + 2 * k)); }
WVI W12 w12_frob2(const W12& a) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_frob2_c(a, k);
  return r;
}

// Granger-Scott cyclotomic square (tower.h fp12_cyclotomic_sqr) with z0..z5 = c0, c3, c1, c4, c2, c5
// (w-powers 0, 3, 1, 4, 2, 5): each output is one dot, the 3 t - 2 z / 3 t + 2 z fix-ups as terms
// against the Montgomery constants -2, 2 -- folded into the squared factor where it is the same
// coefficient (z0' = z0 (3 z0 - 2) + .., z1' = z1 (6 z0 + 2): 2 and 1 terms instead of 3 and 2)
WVI F w12_cyc_sqr_c(const W12& f, int k) {
  const F &z0 = f.c[0], &z1 = f.c[3], &z2 = f.c[1], &z3 = f.c[4], &z4 = f.c[2], &z5 = f.c[5];
  switch (k) {
    case 0: return dot(z0, sub<0>(mul_small<3>(z0), cst(WC_POS2)), z1, mul_small<3>(mul_xi<0>(z1)));  // z0' = z0 (3 z0 - 2) + 3 xi z1^2
    case 3: return dot(z1, add(mul_small<6>(z0), cst(WC_POS2)));                                    // z1' = z1 (6 z0 + 2)
    case 2: return dot(z2, mul_small<3>(z2), z3, mul_small<3>(mul_xi<0>(z3)), z4, cst(WC_NEG2));  // z4' = 3 (z2^2 + xi z3^2) - 2 z4
    case 5: return dot(z2, mul_small<6>(z3), z5, cst(WC_POS2));                                  // z5' = 6 z2 z3 + 2 z5
    case 1: return dot(z4, mul_small<6>(mul_xi<0>(z5)), z2, cst(WC_POS2));                       // z2' = 6 xi z4 z5 + 2 z2
    default: return dot(z4, mul_small<3>(z4), z5, mul_small<3>(mul_xi<0>(z5)), z3, cst(WC_NEG2));  // z3' = 3 (z4^2 + xi z5^2) - 2 z3
  }
}
WVI W12 w12_cyc_sqr(const W12& f) {
  W12 r;
#pragma unroll 1
  for (int k = 0; k < 6; k++) r.c[k] = w12_cyc_sqr_c(f, k);
  return r;
}

// ------------------------------------------------------------------ inverse (final exponentiation)
// f = A + B w with A = c0 + c2 v + c4 v^2, B = c1 + c3 v + c5 v^2 (Fp6 = Fp2[v]/(v^3 - xi)):
// f^-1 = (A - B w) / (A^2 - v B^2)
struct W6 {
  F c[3];
};
WVI W6 w6_mul(const W6& a, const W6& b) {
  const F x1 = mul_xi<0>(b.c[1]), x2 = mul_xi<0>(b.c[2]);
  return {{dot(a.c[0], b.c[0], a.c[1], x2, a.c[2], x1), dot(a.c[0], b.c[1], a.c[1], b.c[0], a.c[2], x2),
           dot(a.c[0], b.c[2], a.c[1], b.c[1], a.c[2], b.c[0])}};
}
WVI W6 w6_sqr(const W6& a) { return w6_mul(a, a); }
WVI W6 w6_inv(const W6& a) {
  // t0 = c0^2 - xi c1 c2, t1 = xi c2^2 - c0 c1, t2 = c1^2 - c0 c2
  const F nx1 = neg<1>(mul_xi<0>(a.c[1])), x2 = mul_xi<0>(a.c[2]);
  const F n0 = neg<0>(a.c[0]);
  const F t0 = dot(a.c[0], a.c[0], a.c[2], nx1);
  const F t1 = dot(a.c[2], x2, a.c[1], n0);
  const F t2 = dot(a.c[1], a.c[1], a.c[2], n0);
  // d = c0 t0 + xi (c2 t1 + c1 t2)
  const F d = dot(a.c[0], t0, x2, t1, mul_xi<0>(a.c[1]), t2);
  const F di = inv2(d);
  return {{mul2(t0, di), mul2(t1, di), mul2(t2, di)}};
}
// f^-1, or its conjugate conj(f^-1) = (A + B w) / (A^2 - v B^2) when CONJ (the easy part needs that)
template <bool CONJ = false>
WVI W12 w12_inv(const W12& f) {
  const W6 A = {{f.c[0], f.c[2], f.c[4]}}, B = {{f.c[1], f.c[3], f.c[5]}};
  const W6 A2 = w6_sqr(A), B2 = w6_sqr(B);
  // D = A^2 - v B^2, v (b0 + b1 v + b2 v^2) = xi b2 + b0 v + b1 v^2
  const F one = cst(WC_ONE2), m1 = cst(WC_NEG1);  // as dots: every coefficient of D reduced
  const W6 D = {{dot(A2.c[0], one, mul_xi<0>(B2.c[2]), m1), dot(A2.c[1], one, B2.c[0], m1),
                 dot(A2.c[2], one, B2.c[1], m1)}};
  const W6 Di = w6_inv(D);
  const W6 RA = w6_mul(A, Di), RB = w6_mul(B, Di);
  W12 r;
  r.c[0] = RA.c[0];
  r.c[2] = RA.c[1];
  r.c[4] = RA.c[2];
  r.c[1] = CONJ ? RB.c[0] : neg<0>(RB.c[0]);
  r.c[3] = CONJ ? RB.c[1] : neg<0>(RB.c[1]);
  r.c[5] = CONJ ? RB.c[2] : neg<0>(RB.c[2]);
  return r;
}

// f == 1 (every coefficient compared exactly)
WVI bool w12_is_one(const W12& f) {
  bool one = is_zero2(sub<0>(f.c[0], cst(WC_ONE2)));
#pragma unroll
  for (int k = 1; k < 6; k++) one = one & is_zero2(f.c[k]);
  return one;
}

}  // namespace wv

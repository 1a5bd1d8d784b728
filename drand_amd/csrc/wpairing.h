// Pairing product check e(P0, Q0) e(P1, Q1) == 1 of the latency engine (pairing.h's algorithms in
// lane form): optimal-ate Miller loop over x = -0xd201000000010000 with homogeneous projective T and
// affine Q, the sparse lines multiplied into f one at a time (w12_mul_line), one final
// exponentiation f^(3 (p^12 - 1) / r) -- easy part, then the hard part (x-1)^2 (x+p) (x^2+p^2-1) + 3
// as pairing.h fexp_step<0..4>. Pairs with a point at infinity are skipped (kilic Engine [ext]).
#pragma once
#include "whash.h"

namespace wv {

// one Miller pair: G1 point P as Fp scalars duplicated over both halves, Q on the twist (affine, or
// homogeneous projective (qx : qy : qz) for the team loop, wvteam.h)
struct MPair {
  F xp3;   // 3 xP        (doubling line l01 = 3 X^2 xP)
  F m2yp;  // -2 yP       (doubling line l11 = -H yP = -2 Y Z yP)
  F mxp;   // -xP         (addition line l01)
  F yp;    // yP          (addition line l11)
  F qx, qy, mqx, mqy;  // Q and -Q's coordinates
  G2J t;   // running T = [k] Q
  bool qaff = true;    // qz == 1
  F qz, mxpz, ypz;     // projective Q only: qz, -xP qz, yP qz
};

WVI MPair mpair(const F& xp, const F& yp, const F& qx, const F& qy) {
  MPair m;
  m.xp3 = mul_small<3>(xp);
  m.m2yp = neg<0>(dbl(yp));
  m.mxp = neg<0>(xp);
  m.yp = yp;
  m.qx = qx;
  m.qy = qy;
  m.mqx = neg<0>(qx);
  m.mqy = neg<0>(qy);
  m.t = {qx, qy, cst(WC_ONE2)};
  return m;
}

// Q = (qx : qy : qz) homogeneous: the addition lines come out scaled by qz^2, an Fp2 factor that the
// final exponentiation removes (every element of a proper subfield has order dividing p^6 - 1)
WVI MPair mpair_proj(const F& xp, const F& yp, const F& qx, const F& qy, const F& qz) {
  MPair m = mpair(xp, yp, qx, qy);
  m.t.z = qz;
  m.qaff = false;
  m.qz = qz;
  m.mxpz = mulp(qz, m.mxp);
  m.ypz = mulp(qz, yp);
  return m;
}

// doubling step (pairing.h miller_dbl_step): T <- 2T and the line l0 + l2 w^2 + l3 w^3
WVI void miller_dbl(MPair& m, F& l0, F& l2, F& l3) {
  const F &X = m.t.x, &Y = m.t.y, &Z = m.t.z;
  const F A = half(dot(X, Y));  // X Y / 2
  const F B = sqr2(Y), C = sqr2(Z), X2 = sqr2(X);
  const F E = dot(C, cst(WC_B2X3));  // 3 b' Z^2
  const F YZ = dot(Y, Z);
  l0 = sub<0>(E, B);
  l2 = mulp(X2, m.xp3);
  l3 = mulp(YZ, m.m2yp);  // -H yP, H = 2 Y Z
  const F G = half(add(B, mul_small<3>(E)));  // (B + 3E) / 2
  const F nE = neg<0>(E);
  m.t.x = dot(A, B, mul_small<3>(A), nE);          // A (B - 3E)
  m.t.y = dot(G, G, mul_small<3>(E), nE);          // G^2 - 3 E^2
  m.t.z = dot(B, dbl(YZ));                          // B H
}

// addition step with the affine Q (pairing.h miller_add_step)
WVI void miller_add(MPair& m, F& l0, F& l2, F& l3) {
  const F &X = m.t.x, &Y = m.t.y, &Z = m.t.z;
  const F one = cst(WC_ONE2);
  const F theta = dot(Y, one, Z, m.mqy);  // Y - y2 Z
  const F delta = dot(X, one, Z, m.mqx);  // X - x2 Z
  l0 = dot(theta, m.qx, delta, m.mqy);     // theta x2 - delta y2
  l2 = mulp(theta, m.mxp);                 // -theta xP
  l3 = mulp(delta, m.yp);                  // delta yP
  const F C = sqr2(theta), D = sqr2(delta);
  const F E = dot(D, delta), Fv = dot(Z, C), G = dot(X, D);
  const F H = sub<0>(add(E, Fv), dbl(G));  // E + F - 2G
  m.t.x = dot(delta, H);
  m.t.y = dot(theta, sub<1>(G, H), Y, neg<0>(E));  // theta (G - H) - Y E
  m.t.z = dot(Z, E);
}

// f = prod over the active pairs of f_{|x|, Q}(P), NOT yet conjugated for x < 0 (final_exp_is_one
// folds the conjugation in, so every coefficient it receives is reduced)
WVI W12 miller_loop(MPair (&pr)[2], const bool (&active)[2]) {
  W12 f = w12_one();
  bool first = true;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (!first) f = w12_sqr(f);
    first = false;
    for (int k = 0; k < 2; k++) {
      if (!active[k]) continue;
      F l0, l2, l3;
      miller_dbl(pr[k], l0, l2, l3);
      f = w12_mul_line(f, l0, l2, l3);
    }
    if ((bls::BLS_X_ABS >> i) & 1ull) {
      for (int k = 0; k < 2; k++) {
        if (!active[k]) continue;
        F l0, l2, l3;
        miller_add(pr[k], l0, l2, l3);
        f = w12_mul_line(f, l0, l2, l3);
      }
    }
  }
  return f;
}

// g^|x| in the cyclotomic subgroup: squaring runs of 1, 2, 3, 9, 32, 16 with a multiplication by g
// after each of the first five
WVI W12 w12_pow_x_abs(const W12& g) {
  constexpr uint64_t NSQ = 1ull | (2ull << 6) | (3ull << 12) | (9ull << 18) | (32ull << 24) | (16ull << 30);
  W12 r = g;
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int n = (int)((NSQ >> (6 * s)) & 63u);
#pragma unroll 1
    for (int k = 0; k < n; k++) r = w12_cyc_sqr(r);
    if (s < 5) r = w12_mul(r, g);
  }
  return r;
}

// f0: the Miller product before its final conjugation, f = conj(f0)
WVI bool final_exp_is_one(const W12& f0) {
  // easy part: g = f^((p^6 - 1)(p^2 + 1)); f^(p^6 - 1) = conj(f) f^-1 = f0 conj(f0^-1)
  const W12 t = w12_mul(f0, w12_inv<true>(f0));
  const W12 g = w12_mul(w12_frob2(t), t);
  // hard part (pairing.h fexp_step), X^x = conj(X^|x|)
  const W12 a = w12_mul(w12_conj(w12_pow_x_abs(g)), w12_conj(g));  // g^(x-1)
  const W12 b = w12_mul(w12_conj(w12_pow_x_abs(a)), w12_conj(a));  // a^(x-1)
  const W12 c = w12_mul(w12_conj(w12_pow_x_abs(b)), w12_frob(b));  // b^(x+p)
  // t = c^x = conj(c^|x|) and t^x = conj(t^|x|) = (c^|x|)^|x| (conjugation commutes with powers)
  W12 e = w12_pow_x_abs(w12_pow_x_abs(c));                         // t^x
  e = w12_mul(e, w12_frob2(c));
  e = w12_mul(e, w12_conj(c));
  e = w12_mul(e, w12_cyc_sqr(g));
  e = w12_mul(e, g);
  return w12_is_one(e);
}

}  // namespace wv

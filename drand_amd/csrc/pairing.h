// Optimal-ate pairing product check for BLS12-381 on gfx950.
// Replaces kilic/bls12-381 Engine.AddPair/AddPairInv/Check ([ext]) as called by kyber-bls12381
// Suite.ValidatePairing from sign/bls Verify:
//     e(pk, H(m)) * e(-g1, sigma) == 1
// One multi-Miller loop (shared Fp12 squaring for both pairs, G2 points in homogeneous
// projective coordinates, sparse 0/1/4 line multiplication) and ONE final exponentiation.
//
// Line functions (M-type twist, untwist (x,y) -> (x w^-2, y w^-3), lines scaled by Fp2 factors
// that the final exponentiation kills):
//   doubling T=(X:Y:Z): l = (3b'Z^2 - Y^2) + (3X^2 xP) v + (-2YZ yP) v w
//   adding affine Q=(x2,y2): theta = Y - y2 Z, delta = X - x2 Z,
//                            l = (theta x2 - delta y2) + (-theta xP) v + (delta yP) v w
// Final exponentiation: easy part f^((p^6-1)(p^2+1)), hard part via
//   3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3
// i.e. the engine computes e^3; since gcd(3, r) = 1 the "== 1" verdict is unchanged.
#pragma once
#include "curve.h"

namespace bls {

struct g2proj {
  fp2 x, y, z;
};

DI void miller_dbl_step(g2proj& t, fp2& l00, fp2& l01, fp2& l11, const fp& xp, const fp& yp) {
  const fp inv2 = fp_load_const(FP_INV2);
  fp2 A = fp2_mul_fp(fp2_mul(t.x, t.y), inv2);
  fp2 B = fp2_sqr(t.y);
  fp2 C = fp2_sqr(t.z);
  fp2 E = fp2_mul(C, fp2_load_const(B2_TWIST_X3));
  fp2 F = fp2_mul3(E);
  fp2 G = fp2_mul_fp(fp2_add(B, F), inv2);
  fp2 H = fp2_sub(fp2_sqr(fp2_add(t.y, t.z)), fp2_add(B, C));
  fp2 X2 = fp2_sqr(t.x);
  l00 = fp2_sub(E, B);
  l01 = fp2_mul_fp(fp2_mul3(X2), xp);
  l11 = fp2_neg(fp2_mul_fp(H, yp));
  t.x = fp2_mul(A, fp2_sub(B, F));
  t.y = fp2_sub(fp2_sqr(G), fp2_mul3(fp2_sqr(E)));
  t.z = fp2_mul(B, H);
}

DI void miller_add_step(g2proj& t, const g2a& q, fp2& l00, fp2& l01, fp2& l11, const fp& xp, const fp& yp) {
  fp2 theta = fp2_sub(t.y, fp2_mul(q.y, t.z));
  fp2 delta = fp2_sub(t.x, fp2_mul(q.x, t.z));
  l00 = fp2_sub(fp2_mul(theta, q.x), fp2_mul(delta, q.y));
  l01 = fp2_neg(fp2_mul_fp(theta, xp));
  l11 = fp2_mul_fp(delta, yp);
  fp2 C = fp2_sqr(theta);
  fp2 D = fp2_sqr(delta);
  fp2 E = fp2_mul(D, delta);
  fp2 F = fp2_mul(t.z, C);
  fp2 G = fp2_mul(t.x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  t.x = fp2_mul(delta, H);
  t.y = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(t.y, E));
  t.z = fp2_mul(t.z, E);
}

// f = prod_{k<npairs, active} f_{|x|, Q_k}(P_k), conjugated (x < 0). Inactive pairs (a point at
// infinity, skipped like kilic's Engine) contribute 1.
template <int NP>
DI fp12 miller_loop_multi(const g1a (&P)[NP], const g2a (&Q)[NP], const bool (&active)[NP]) {
  g2proj T[NP];
#pragma unroll
  for (int k = 0; k < NP; k++) T[k] = {Q[k].x, Q[k].y, fp2_one()};
  fp12 f = fp12_one();
  bool first = true;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (!first) f = fp12_sqr(f);
#pragma unroll
    for (int k = 0; k < NP; k++) {
      fp2 l00, l01, l11;
      miller_dbl_step(T[k], l00, l01, l11, P[k].x, P[k].y);
      if (active[k]) f = fp12_mul_by_014(f, l00, l01, l11);
    }
    first = false;
    if ((BLS_X_ABS >> i) & 1ull) {
#pragma unroll
      for (int k = 0; k < NP; k++) {
        fp2 l00, l01, l11;
        miller_add_step(T[k], Q[k], l00, l01, l11, P[k].x, P[k].y);
        if (active[k]) f = fp12_mul_by_014(f, l00, l01, l11);
      }
    }
  }
  return fp12_conj(f);
}

// g^|x| for g in the cyclotomic subgroup
DI fp12 fp12_pow_x_abs(const fp12& g) {
  fp12 r = g;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    r = fp12_sqr(r);
    if ((BLS_X_ABS >> i) & 1ull) r = fp12_mul(r, g);
  }
  return r;
}

// g^x, x = -|x| (inverse = conjugate in the cyclotomic subgroup)
DI fp12 fp12_pow_x(const fp12& g) { return fp12_conj(fp12_pow_x_abs(g)); }

// f^(3 (p^12 - 1) / r)
DI fp12 final_exponentiation(const fp12& f) {
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));  // f^(p^6 - 1)
  fp12 g = fp12_mul(fp12_frob2(t), t);           // ^(p^2 + 1)
  fp12 a = fp12_mul(fp12_pow_x(g), fp12_conj(g));        // g^(x-1)
  fp12 b = fp12_mul(fp12_pow_x(a), fp12_conj(a));        // g^((x-1)^2)
  fp12 c = fp12_mul(fp12_pow_x(b), fp12_frob(b));        // b^(x+p)
  fp12 d = fp12_mul(fp12_mul(fp12_pow_x(fp12_pow_x(c)), fp12_frob2(c)), fp12_conj(c));  // c^(x^2+p^2-1)
  return fp12_mul(d, fp12_mul(fp12_sqr(g), g));  // * g^3
}

}  // namespace bls

// G2 (y^2 = x^3 + 4(1 + i), M-type twist) in Jacobian coordinates for the latency engine: the same
// formulas as curve.h (dbl-2009-l, add-2007-bl with its exceptional cases, psi, the [|x|] chain, the
// psi-based subgroup check and cofactor clearing), each coordinate written as dot products so that
// every stored value is reduced (wfield.h).
#pragma once
#include "wtower.h"

namespace wv {

struct G2J {
  F x, y, z;
};

WVI G2J g2_infinity() { return {cst(WC_ONE2), cst(WC_ONE2), zero()}; }
WVI bool g2_is_inf(const G2J& p) { return is_zero2(p.z); }
WVI G2J g2_neg(const G2J& p) { return {p.x, neg<0>(p.y), p.z}; }

// dbl-2009-l: A = X^2, B = Y^2, C = B^2, D = 2((X + B)^2 - A - C) = 4 X B, E = 3 A,
// X3 = E^2 - 2 D, Y3 = E (D - X3) - 8 C, Z3 = 2 Y Z  (Z3 = 0 for infinity or y = 0)
WVI G2J g2_dbl(const G2J& p) {
  const F A = sqr2(p.x), B = sqr2(p.y);
  const F C = sqr2(B);
  const F D = dot(p.x, mul_small<4>(B));
  const F E = mul_small<3>(A);
  const F X3 = dot(E, E, D, cst(WC_NEG2));
  const F Y3 = dot(E, D, neg<0>(X3), E, C, cst(WC_NEG8));
  const F Z3 = dot(dbl(p.y), p.z);
  return {X3, Y3, Z3};
}

// add-2007-bl with the exceptional cases (P == Q -> dbl, P == -Q -> O, either O); the decisions are
// wave-uniform (one item per wave)
WVI G2J g2_add(const G2J& p, const G2J& q) {
  if (g2_is_inf(p)) return q;
  if (g2_is_inf(q)) return p;
  const F Z1Z1 = sqr2(p.z), Z2Z2 = sqr2(q.z);
  const F U1 = dot(p.x, Z2Z2);
  const F H = dot(q.x, Z1Z1, U1, cst(WC_NEG1));  // U2 - U1
  const F S1 = dot(dot(p.y, q.z), Z2Z2);
  const F r = dot(dot(q.y, p.z), dbl(Z1Z1), S1, cst(WC_NEG2));  // 2 (S2 - S1)
  if (is_zero2(H)) {
    if (is_zero2(r)) return g2_dbl(p);
    return g2_infinity();
  }
  const F I = dot(H, mul_small<4>(H));  // (2H)^2
  const F J = dot(H, I), V = dot(U1, I);
  const F X3 = dot(r, r, J, cst(WC_NEG1), V, cst(WC_NEG2));
  const F Y3 = dot(r, V, neg<0>(X3), r, S1, neg<0>(dbl(J)));
  const F Z3 = dot(dot(p.z, dbl(q.z)), H);  // ((Z1 + Z2)^2 - Z1Z1 - Z2Z2) H = 2 Z1 Z2 H
  return {X3, Y3, Z3};
}

// p + q for an affine q (z = 1) with no exceptional-case tests (madd-2007-bl): the caller guarantees
// p != +-q and neither is infinity -- as in a left-to-right ladder [k] q, 2 <= k < r, whose
// intermediate multiples never equal +-q (wrecover.h). Ten products against add-2007-bl's fifteen
// and its four zero tests.
WVI G2J g2_madd_noexc(const G2J& p, const F& qx, const F& qy) {
  const F Z1Z1 = sqr2(p.z);
  const F H = dot(qx, Z1Z1, p.x, cst(WC_NEG1));                          // U2 - X1
  const F r = dot(dot(qy, p.z), dbl(Z1Z1), p.y, cst(WC_NEG2));           // 2 (S2 - Y1)
  const F I = dot(H, mul_small<4>(H));                                    // (2H)^2
  const F J = dot(H, I), V = dot(p.x, I);
  const F X3 = dot(r, r, J, cst(WC_NEG1), V, cst(WC_NEG2));
  const F Y3 = dot(r, V, neg<0>(X3), r, p.y, neg<0>(dbl(J)));
  const F Z3 = dot(p.z, dbl(H));                                          // 2 Z1 H
  return {X3, Y3, Z3};
}

// projective equality (either may be infinity)
WVI bool g2_eq(const G2J& p, const G2J& q) {
  const bool pi = g2_is_inf(p), qi = g2_is_inf(q);
  if (pi | qi) return pi & qi;
  const F Z1Z1 = sqr2(p.z), Z2Z2 = sqr2(q.z);
  const bool ex = is_zero2(dot(p.x, Z2Z2, q.x, neg<0>(Z1Z1)));
  const bool ey = is_zero2(dot(dot(p.y, q.z), Z2Z2, dot(q.y, p.z), neg<0>(Z1Z1)));
  return ex & ey;
}

// [|x|] P, |x| = 0xd201000000010000 (bits 63, 62, 60, 57, 48, 16): 63 doublings, 5 additions
WVI G2J g2_mul_x_abs(const G2J& p) {
  G2J acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    acc = g2_dbl(acc);
    if ((bls::BLS_X_ABS >> i) & 1ull) acc = g2_add(acc, p);
  }
  return acc;
}

// psi(x, y, z) = (conj(x) kx, conj(y) ky, conj(z)); psi^2 = (x kx2, y ky2, z) with kx2, ky2 in Fp
WVI G2J g2_psi(const G2J& p) {
  return {mul2(conj<1>(p.x), cst(WC_PSI_KX)), mul2(conj<1>(p.y), cst(WC_PSI_KY)), conj<1>(p.z)};
}
WVI G2J g2_psi2(const G2J& p) { return {mulp(p.x, cst(WC_PSI2_KX)), mulp(p.y, cst(WC_PSI2_KY)), p.z}; }

// P in G2 <=> psi(P) == [x] P, x = -|x| (for P on the curve)
WVI bool g2_in_subgroup(const G2J& p) {
  if (g2_is_inf(p)) return true;
  return g2_eq(g2_psi(p), g2_neg(g2_mul_x_abs(p)));
}

// RFC 9380 G.3 h_eff P = [x^2 - x - 1] P + [x - 1] psi(P) + psi^2(2P), regrouped as in curve.h:
// A = [x] P + psi(P), B = [x] A, h_eff P = B - A - P + psi^2(2P)
WVI G2J g2_clear_cofactor(const G2J& p) {
  const G2J a = g2_add(g2_neg(g2_mul_x_abs(p)), g2_psi(p));
  G2J r = g2_add(g2_neg(g2_mul_x_abs(a)), g2_neg(a));
  r = g2_add(r, g2_neg(p));
  return g2_add(r, g2_psi2(g2_dbl(p)));
}

// affine (x, y) = (X / Z^2, Y / Z^3) of a finite point
WVI void g2_to_affine(const G2J& p, F& x, F& y) {
  const F zi = inv2(p.z);
  const F zi2 = sqr2(zi);
  x = dot(p.x, zi2);
  y = dot(p.y, dot(zi2, zi));
}

}  // namespace wv

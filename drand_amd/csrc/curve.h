// Short-Weierstrass curves of BLS12-381 on gfx950:
//   G1: y^2 = x^3 + 4 over Fp,  G2 (M-type sextic twist): y^2 = x^3 + 4(1+i) over Fp2.
// Jacobian coordinates (x = X/Z^2, y = Y/Z^3), Z == 0 <=> point at infinity.
// Replaces kilic/bls12-381 g1.go / g2.go arithmetic, FromCompressed/ToCompressed and
// InCorrectSubgroup ([ext]). Subgroup membership uses the
// endomorphism tests (G2: psi(P) == [x]P; G1: sigma(P) == [-x^2]P... see g1_in_subgroup), which
// agree with kilic's naive [r]P == O on every curve point (cross-checked against the oracle).
#pragma once
#include "tower.h"

namespace bls {

// ------------------------------------------------------------ overload set over Fp / Fp2
DI fp f_add(const fp& a, const fp& b) { return fp_add(a, b); }
DI fp f_sub(const fp& a, const fp& b) { return fp_sub(a, b); }
DI fp f_mul(const fp& a, const fp& b) { return fp_mul(a, b); }
DI fp f_sqr(const fp& a) { return fp_sqr(a); }
DI fp f_dbl(const fp& a) { return fp_dbl(a); }
DI fp f_neg(const fp& a) { return fp_neg(a); }
DI bool f_is_zero(const fp& a) { return fp_is_zero(a); }
DI bool f_eq(const fp& a, const fp& b) { return fp_eq(a, b); }
DI fp f_select(bool c, const fp& a, const fp& b) { return fp_select(c, a, b); }
DI fp2 f_add(const fp2& a, const fp2& b) { return fp2_add(a, b); }
DI fp2 f_sub(const fp2& a, const fp2& b) { return fp2_sub(a, b); }
DI fp2 f_mul(const fp2& a, const fp2& b) { return fp2_mul(a, b); }
DI fp2 f_sqr(const fp2& a) { return fp2_sqr(a); }
DI fp2 f_dbl(const fp2& a) { return fp2_dbl(a); }
DI fp2 f_neg(const fp2& a) { return fp2_neg(a); }
DI bool f_is_zero(const fp2& a) { return fp2_is_zero(a); }
DI bool f_eq(const fp2& a, const fp2& b) { return fp2_eq(a, b); }
DI fp2 f_select(bool c, const fp2& a, const fp2& b) { return fp2_select(c, a, b); }

template <typename F>
struct jac {
  F x, y, z;
};
template <typename F>
struct aff {
  F x, y;
};
using g1j = jac<fp>;
using g2j = jac<fp2>;
using g1a = aff<fp>;
using g2a = aff<fp2>;

DI fp f_zero_of(const fp&) { return fp_zero(); }
DI fp2 f_zero_of(const fp2&) { return fp2_zero(); }
DI fp f_one_of(const fp&) { return fp_one(); }
DI fp2 f_one_of(const fp2&) { return fp2_one(); }

template <typename F>
DI jac<F> jac_infinity() {
  F z = f_zero_of(F{});
  F o = f_one_of(F{});
  return {o, o, z};
}

template <typename F>
DI bool jac_is_inf(const jac<F>& p) { return f_is_zero(p.z); }

template <typename F>
DI jac<F> jac_from_aff(const aff<F>& a) { return {a.x, a.y, f_one_of(F{})}; }

template <typename F>
DI jac<F> jac_neg(const jac<F>& p) { return {p.x, f_neg(p.y), p.z}; }

template <typename F>
DI jac<F> jac_select(bool c, const jac<F>& a, const jac<F>& b) {
  return {f_select(c, a.x, b.x), f_select(c, a.y, b.y), f_select(c, a.z, b.z)};
}

// dbl-2009-l (a = 0): 2M + 5S
template <typename F>
DI jac<F> jac_dbl(const jac<F>& p) {
  F A = f_sqr(p.x);
  F B = f_sqr(p.y);
  F C = f_sqr(B);
  F D = f_dbl(f_sub(f_sub(f_sqr(f_add(p.x, B)), A), C));
  F E = f_add(f_dbl(A), A);
  F Fv = f_sqr(E);
  F X3 = f_sub(Fv, f_dbl(D));
  F C8 = f_dbl(f_dbl(f_dbl(C)));
  F Y3 = f_sub(f_mul(E, f_sub(D, X3)), C8);
  F Z3 = f_dbl(f_mul(p.y, p.z));
  return {X3, Y3, Z3};  // Z3 = 0 when p is infinity or y = 0
}

// add-2007-bl with the exceptional cases (P == Q -> dbl, P == -Q -> O, either O)
template <typename F>
DI jac<F> jac_add(const jac<F>& p, const jac<F>& q) {
  if (jac_is_inf(p)) return q;
  if (jac_is_inf(q)) return p;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  F U1 = f_mul(p.x, Z2Z2);
  F U2 = f_mul(q.x, Z1Z1);
  F S1 = f_mul(f_mul(p.y, q.z), Z2Z2);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, U1);
  F r = f_dbl(f_sub(S2, S1));
  if (f_is_zero(H)) {
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F I = f_sqr(f_dbl(H));
  F J = f_mul(H, I);
  F V = f_mul(U1, I);
  F X3 = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  F Y3 = f_sub(f_mul(r, f_sub(V, X3)), f_dbl(f_mul(S1, J)));
  F Z3 = f_mul(f_sub(f_sub(f_sqr(f_add(p.z, q.z)), Z1Z1), Z2Z2), H);
  return {X3, Y3, Z3};
}

// mixed addition with an affine (never infinity) q: madd-2007-bl + exceptional cases
template <typename F>
DI jac<F> jac_add_aff(const jac<F>& p, const aff<F>& q) {
  if (jac_is_inf(p)) return jac_from_aff(q);
  F Z1Z1 = f_sqr(p.z);
  F U2 = f_mul(q.x, Z1Z1);
  F S2 = f_mul(f_mul(q.y, p.z), Z1Z1);
  F H = f_sub(U2, p.x);
  F r = f_dbl(f_sub(S2, p.y));
  if (f_is_zero(H)) {
    if (f_is_zero(r)) return jac_dbl(p);
    return jac_infinity<F>();
  }
  F HH = f_sqr(H);
  F I = f_dbl(f_dbl(HH));
  F J = f_mul(H, I);
  F V = f_mul(p.x, I);
  F X3 = f_sub(f_sub(f_sqr(r), J), f_dbl(V));
  F Y3 = f_sub(f_mul(r, f_sub(V, X3)), f_dbl(f_mul(p.y, J)));
  F Z3 = f_sub(f_sub(f_sqr(f_add(p.z, H)), Z1Z1), HH);
  return {X3, Y3, Z3};
}

// projective equality (both may be infinity)
template <typename F>
DI bool jac_eq(const jac<F>& p, const jac<F>& q) {
  bool pi = jac_is_inf(p), qi = jac_is_inf(q);
  if (pi | qi) return pi & qi;
  F Z1Z1 = f_sqr(p.z);
  F Z2Z2 = f_sqr(q.z);
  bool ex = f_eq(f_mul(p.x, Z2Z2), f_mul(q.x, Z1Z1));
  bool ey = f_eq(f_mul(f_mul(p.y, q.z), Z2Z2), f_mul(f_mul(q.y, p.z), Z1Z1));
  return ex & ey;
}

// G2 doubling (dbl-2009-l, as jac_dbl) with the Fp2 products expanded in place: the [x] chains of
// the G2 cofactor clearing and subgroup check run their 63 doublings call-free, so the register
// allocator sees the whole step instead of the AMDGPU call ABI's caller/callee-saved split.
#define G2_DBL_FENCE() ((void)0)
// the doubling's two products: Karatsuba where the unit asks for it (BLS_G2_DBL_KARA, default
// BLS_FP2_KARA_INL); k_hash.hip keeps the dot form here, whose smaller working set lets its op
// program enter and leave the doubling loop without spills
#ifndef BLS_G2_DBL_KARA
#define BLS_G2_DBL_KARA BLS_FP2_KARA_INL
#endif
DI g2j g2_dbl_inl(const g2j& p) {
  const fp2 Z3 = fp2_dbl(fp2_mul_inl_t<BLS_G2_DBL_KARA != 0>(p.y, p.z));
  G2_DBL_FENCE();
  const fp2 A = fp2_sqr_inl(p.x);
  G2_DBL_FENCE();
  const fp2 B = fp2_sqr_inl(p.y);
  G2_DBL_FENCE();
  const fp2 C = fp2_sqr_inl(B);
  G2_DBL_FENCE();
  const fp2 D = fp2_dbl(fp2_sub(fp2_sub(fp2_sqr_inl(fp2_add(p.x, B)), A), C));
  G2_DBL_FENCE();
  const fp2 E = fp2_add(fp2_dbl(A), A);
  const fp2 X3 = fp2_sub(fp2_sqr_inl(E), fp2_dbl(D));
  G2_DBL_FENCE();
  const fp2 C8 = fp2_dbl(fp2_dbl(fp2_dbl(C)));
  const fp2 Y3 = fp2_sub(fp2_mul_inl_t<BLS_G2_DBL_KARA != 0>(E, fp2_sub(D, X3)), C8);
  return {X3, Y3, Z3};
}

template <typename F>
DI jac<F> jac_dbl_chain(const jac<F>& p) {
  if constexpr (sizeof(F) == sizeof(fp2)) {
    return g2_dbl_inl(p);
  } else {
    return jac_dbl(p);
  }
}

// [|x|] P, |x| = 0xd201000000010000 (bits 63,62,60,57,48,16): 63 dbl + 5 add
template <typename F>
DI jac<F> jac_mul_x_abs(const jac<F>& p) {
  jac<F> acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    acc = jac_dbl_chain(acc);
    if ((BLS_X_ABS >> i) & 1ull) acc = jac_add(acc, p);
  }
  return acc;
}

// [k] P for a 256-bit scalar given as 8 little-endian words (per-thread scalar: divergent adds)
template <typename F>
DI jac<F> jac_mul_scalar(const jac<F>& p, const uint32_t (&k)[8]) {
  jac<F> acc = jac_infinity<F>();
#pragma unroll 1
  for (int i = 255; i >= 0; i--) {
    acc = jac_dbl(acc);
    if ((k[i >> 5] >> (i & 31)) & 1u) acc = jac_add(acc, p);
  }
  return acc;
}

template <typename F, typename Finv>
DI aff<F> jac_to_aff(const jac<F>& p, Finv inv) {
  F zi = inv(p.z);
  F zi2 = f_sqr(zi);
  return {f_mul(p.x, zi2), f_mul(p.y, f_mul(zi2, zi))};
}

DI g2a g2_to_aff(const g2j& p) { return jac_to_aff(p, [](const fp2& z) { return fp2_inv(z); }); }
DI g1a g1_to_aff(const g1j& p) { return jac_to_aff(p, [](const fp& z) { return fp_inv(z); }); }

// ------------------------------------------------------------ G2 endomorphism psi
DI g2j g2_psi(const g2j& p) {
  return {fp2_mul(fp2_conj(p.x), fp2_load_const(PSI_KX)), fp2_mul(fp2_conj(p.y), fp2_load_const(PSI_KY)),
          fp2_conj(p.z)};
}
DI g2j g2_psi2(const g2j& p) {
  return {fp2_mul_fp(p.x, fp_load_const(PSI2_KX[0])), fp2_mul_fp(p.y, fp_load_const(PSI2_KY[0])), p.z};
}

// P in G2  <=>  psi(P) == [x] P  (x = -|x|), for P on E2'
DI bool g2_in_subgroup(const g2j& p) {
  if (jac_is_inf(p)) return true;
  g2j xp = jac_neg(jac_mul_x_abs(p));
  return jac_eq(g2_psi(p), xp);
}

// ------------------------------------------------------------ call-free [x] chains (2 waves/SIMD)
// A called Fp2 product makes everything live across it sit in the ~112 callee-saved VGPRs; the
// chain's point, its base point and a step's temporaries do not fit, so a called addition spills
// (7 KB/lane at 2 waves/SIMD for the subgroup check) and the chains ran at 1 wave/SIMD. Here the
// additions are expanded in place too, with the base point re-read from staging at its uses.
// madd-2007-bl (as jac_add_aff), q affine and never infinity
DI g2j g2_madd_inl(const g2j& p, const g2a& q) {
  const fp2 Z1Z1 = fp2_sqr_inl(p.z);
  const fp2 U2 = fp2_mul_inl(q.x, Z1Z1);
  const fp2 S2 = fp2_mul_inl(fp2_mul_inl(q.y, p.z), Z1Z1);
  const fp2 H = fp2_sub(U2, p.x);
  const fp2 r = fp2_dbl(fp2_sub(S2, p.y));
  const fp2 HH = fp2_sqr_inl(H);
  const fp2 I = fp2_dbl(fp2_dbl(HH));
  const fp2 J = fp2_mul_inl(H, I);
  const fp2 V = fp2_mul_inl(p.x, I);
  const fp2 X3 = fp2_sub(fp2_sub(fp2_sqr_inl(r), J), fp2_dbl(V));
  const fp2 Y3 = fp2_sub(fp2_mul_inl(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul_inl(p.y, J)));
  const fp2 Z3 = fp2_sub(fp2_sub(fp2_sqr_inl(fp2_add(p.z, H)), Z1Z1), HH);
  g2j out = {X3, Y3, Z3};
  const bool pinf = jac_is_inf(p), h0 = fp2_is_zero(H);
  if (pinf | h0) {
    const bool r0 = fp2_is_zero(r);
    out = pinf ? jac_from_aff(q) : (r0 ? jac_dbl(p) : jac_infinity<fp2>());
  }
  return out;
}

// add-2007-bl for the cofactor chains, ordered for the fewest live values: Z3 = 2 (Z1 Z2) H (one more
// product and one square fewer than (Z1 + Z2)^2 - Z1Z1 - Z2Z2, same value), q's coordinates fetched at
// their first use (qx(), qy(), qz() re-read them from staging), S1, U1, Z1 Z2 and Z3 parked in LDS
// between their computation and their uses (three `park` slots), and no exceptional branch: either
// point at infinity or H == 0 (P == +-Q) sets `exc` and leaves an unspecified result, which the
// caller replaces by the generic formulas' (k_hash.hip). With both points and the branch's operands
// live to the end, g2_add_inl spilled ~530 dwords to scratch per addition.
#ifndef BLS_HOST
// Per-lane Fp2 slots in LDS (slot k of lane l: six 16-byte words at base[(6k + q) * BLS_LANES + l]),
// for values that would otherwise stay live in registers across a long stretch of products. The
// compiler barriers keep the store where it is written and the load from being forwarded from it.
struct LdsFp2Slots {
  uint4* base;
  DI void put(int k, const fp2& v) const {
    uint4* q = base + 6 * k * BLS_LANES + threadIdx.x;
#pragma unroll
    for (int w = 0; w < 3; w++) {
      q[w * BLS_LANES] = make_uint4(v.c0.l[4 * w], v.c0.l[4 * w + 1], v.c0.l[4 * w + 2], v.c0.l[4 * w + 3]);
      q[(3 + w) * BLS_LANES] = make_uint4(v.c1.l[4 * w], v.c1.l[4 * w + 1], v.c1.l[4 * w + 2], v.c1.l[4 * w + 3]);
    }
    asm volatile("" ::: "memory");
  }
  DI fp2 get(int k) const {
    asm volatile("" ::: "memory");
    const uint4* q = base + 6 * k * BLS_LANES + threadIdx.x;
    fp2 v;
#pragma unroll
    for (int w = 0; w < 3; w++) {
      const uint4 a = q[w * BLS_LANES], b = q[(3 + w) * BLS_LANES];
      v.c0.l[4 * w] = a.x, v.c0.l[4 * w + 1] = a.y, v.c0.l[4 * w + 2] = a.z, v.c0.l[4 * w + 3] = a.w;
      v.c1.l[4 * w] = b.x, v.c1.l[4 * w + 1] = b.y, v.c1.l[4 * w + 2] = b.z, v.c1.l[4 * w + 3] = b.w;
    }
    return v;
  }
};
#else
// host build (tools/opcount.cpp): the slots are an array of the caller's
struct LdsFp2Slots {
  fp2* base;
  void put(int k, const fp2& v) const { base[k] = v; }
  fp2 get(int k) const { return base[k]; }
};
#endif

template <typename QX, typename QY, typename QZ>
DI g2j g2_add_inl_exc(const g2j& p, QX qx, QY qy, QZ qz, const LdsFp2Slots& park, bool& exc) {
  const fp2 Z2 = qz();
  const fp2 Z2Z2 = fp2_sqr_inl(Z2);
  park.put(0, fp2_mul_inl(fp2_mul_inl(p.y, Z2), Z2Z2));  // S1
  park.put(2, fp2_mul_inl(p.x, Z2Z2));                   // U1
  park.put(1, fp2_mul_inl(p.z, Z2));                     // Z1 Z2
  exc |= fp2_is_zero(p.z) | fp2_is_zero(Z2);
  BLS_SCHED_FENCE();
  const fp2 Z1Z1 = fp2_sqr_inl(p.z);
  const fp2 S2 = fp2_mul_inl(fp2_mul_inl(qy(), p.z), Z1Z1);
  BLS_SCHED_FENCE();
  const fp2 H = fp2_sub(fp2_mul_inl(qx(), Z1Z1), park.get(2));
  const fp2 r = fp2_dbl(fp2_sub(S2, park.get(0)));
  exc |= fp2_is_zero(H);
  park.put(1, fp2_dbl(fp2_mul_inl(park.get(1), H)));  // Z3
  const fp2 I = fp2_sqr_inl(fp2_dbl(H));
  const fp2 J = fp2_mul_inl(H, I);
  const fp2 V = fp2_mul_inl(park.get(2), I);
  const fp2 X3 = fp2_sub(fp2_sub(fp2_sqr_inl(r), J), fp2_dbl(V));
  const fp2 Y3 = fp2_sub(fp2_mul_inl(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul_inl(park.get(0), J)));
  return {X3, Y3, park.get(1)};
}

// madd-2007-bl for the subgroup check's chain in the same low-pressure form as g2_add_inl_exc: q
// affine, fetched per coordinate (qx(), qy()), Z3 = 2 Z1 H (a product in place of a square and two
// subtractions), Y1 and Z3 parked in LDS slots 0 and 1 and X1 in slot 2 between their computation and
// their last use; an exceptional case (p at infinity or H == 0: p == +-q) sets `exc` and leaves an
// unspecified result.
template <typename QX, typename QY>
DI g2j g2_madd_inl_exc(const g2j& p, QX qx, QY qy, const LdsFp2Slots& park, bool& exc) {
  park.put(0, p.y);
  park.put(2, p.x);
  const fp2 Z1Z1 = fp2_sqr_inl(p.z);
  const fp2 S2 = fp2_mul_inl(fp2_mul_inl(qy(), p.z), Z1Z1);
  BLS_SCHED_FENCE();
  const fp2 H = fp2_sub(fp2_mul_inl(qx(), Z1Z1), park.get(2));
  exc |= fp2_is_zero(p.z) | fp2_is_zero(H);
  park.put(1, fp2_dbl(fp2_mul_inl(p.z, H)));  // Z3
  const fp2 r = fp2_dbl(fp2_sub(S2, park.get(0)));
  BLS_SCHED_FENCE();
  const fp2 I = fp2_dbl(fp2_dbl(fp2_sqr_inl(H)));
  const fp2 J = fp2_mul_inl(H, I);
  const fp2 V = fp2_mul_inl(park.get(2), I);
  const fp2 X3 = fp2_sub(fp2_sub(fp2_sqr_inl(r), J), fp2_dbl(V));
  const fp2 Y3 = fp2_sub(fp2_mul_inl(r, fp2_sub(V, X3)), fp2_dbl(fp2_mul_inl(park.get(0), J)));
  return {X3, Y3, park.get(1)};
}

// [|x|] P call-free with mixed additions of the affine base() (re-read at each use); the exceptional
// cases take g2_madd_inl's rarely executed branch. The generic fix-up kernels' form (k_decomp.hip
// k_subgroup_g2_generic, g2_decompress with its subgroup check); the production chains are the
// flagged programs of k_hash.hip / k_decomp.hip.
template <typename Base>
DI g2j g2_mul_x_abs_aff_inl(const g2j& p, Base base) {
  g2j acc = p;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    acc = g2_dbl_inl(acc);
    if ((BLS_X_ABS >> i) & 1ull) acc = g2_madd_inl(acc, base());
  }
  return acc;
}

// g2_in_subgroup for an affine point re-read by `reload` (never infinity: the caller screens it)
template <typename Reload>
DI bool g2_in_subgroup_aff_reload(Reload reload) {
  const g2j xp = jac_neg(g2_mul_x_abs_aff_inl(jac_from_aff(reload()), reload));
  return jac_eq(g2_psi(jac_from_aff(reload())), xp);
}

// RFC 9380 G.3 clear_cofactor_bls12381_g2: h_eff P = [x^2 - x - 1]P + [x - 1]psi(P) + psi^2(2P)
// regrouped so that only two points are live across each [x] multiplication:
//   A = [x]P + psi(P),  B = [x]A = [x^2]P + [x]psi(P),  h_eff P = B - A - P + psi^2(2P)
// `reload` returns P again (the caller may re-read it from memory instead of keeping it live).
template <typename Reload>
DI g2j g2_clear_cofactor_reload(Reload reload) {
  g2j p = reload();
  g2j a = jac_add(jac_neg(jac_mul_x_abs(p)), g2_psi(p));
  g2j r = jac_add(jac_neg(jac_mul_x_abs(a)), jac_neg(a));
  p = reload();
  r = jac_add(r, jac_neg(p));
  return jac_add(r, g2_psi2(jac_dbl(p)));
}

DI g2j g2_clear_cofactor(const g2j& p) {
  return g2_clear_cofactor_reload([&]() { return p; });
}

// ------------------------------------------------------------ G1 subgroup check
// P in G1 <=> [r]P == O. Device form: r = x^4 - x^2 + 1, so [r]P = [x^2]([x^2]P - P) + P.
DI bool g1_in_subgroup(const g1j& p) {
  if (jac_is_inf(p)) return true;
  g1j x2p = jac_mul_x_abs(jac_mul_x_abs(p));        // [x^2]P (sign cancels)
  g1j t = jac_add(x2p, jac_neg(p));                 // [x^2 - 1]P
  g1j x2t = jac_mul_x_abs(jac_mul_x_abs(t));        // [x^4 - x^2]P
  return jac_eq(x2t, jac_neg(p));                   // [x^4 - x^2 + 1]P == O
}

// ------------------------------------------------------------ ZCash compressed encodings
// reject classes, shared with include/blsverify.h
enum : uint8_t {
  REJ_OK = 0,
  REJ_LENGTH = 1,
  REJ_FLAG = 2,
  REJ_INF_NONZERO = 3,
  REJ_X_GE_P = 4,
  REJ_NOT_ON_CURVE = 5,
  REJ_NOT_IN_SUBGROUP = 6,
  REJ_PAIRING = 7,
};

// 96-byte compressed G2 -> affine point (is_inf set for the canonical infinity encoding).
// Checks in kilic FromCompressed order: flag, infinity form, x < p, sqrt, sign, subgroup.
DI uint8_t g2_decompress(const uint8_t* in, g2a& out, bool& is_inf, bool check_subgroup) {
  is_inf = false;
  const uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return REJ_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = (b0 != 0xc0);
    for (int i = 1; i < 96; i++) acc |= in[i];
    if (acc) return REJ_INF_NONZERO;
    is_inf = true;
    out.x = fp2_zero();
    out.y = fp2_zero();
    return REJ_OK;
  }
  const bool sign = (b0 & 0x20) != 0;
  uint8_t hi[48];
  for (int i = 0; i < 48; i++) hi[i] = in[i];
  hi[0] &= 0x1f;
  fp x1 = fp_raw_from_be48(hi);
  fp x0 = fp_raw_from_be48(in + 48);
  if (!(fp_raw_lt_p(x1) & fp_raw_lt_p(x0))) return REJ_X_GE_P;
  fp2 x = {fp_to_mont(x0), fp_to_mont(x1)};
  fp2 rhs = fp2_add(fp2_mul(fp2_sqr(x), x), fp2_load_const(B2_TWIST));
  fp2 y;
  if (!fp2_sqrt(y, rhs)) return REJ_NOT_ON_CURVE;
  if (fp2_lex_largest(y) != sign) y = fp2_neg(y);
  out.x = x;
  out.y = y;
  // the device chain (k_subgroup_g2: mixed additions with the affine point)
  if (check_subgroup && !g2_in_subgroup_aff_reload([&]() { return out; })) return REJ_NOT_IN_SUBGROUP;
  return REJ_OK;
}

DI void g2_compress(uint8_t* out, const g2j& p) {
  if (jac_is_inf(p)) {
    out[0] = 0xc0;
    for (int i = 1; i < 96; i++) out[i] = 0;
    return;
  }
  g2a a = g2_to_aff(p);
  fp_raw_to_be48(out, fp_from_mont(a.x.c1));
  fp_raw_to_be48(out + 48, fp_from_mont(a.x.c0));
  out[0] |= 0x80 | (fp2_lex_largest(a.y) ? 0x20 : 0x00);
}

DI uint8_t g1_decompress(const uint8_t* in, g1a& out, bool& is_inf) {
  is_inf = false;
  const uint8_t b0 = in[0];
  if (!(b0 & 0x80)) return REJ_FLAG;
  if (b0 & 0x40) {
    uint32_t acc = (b0 != 0xc0);
    for (int i = 1; i < 48; i++) acc |= in[i];
    if (acc) return REJ_INF_NONZERO;
    is_inf = true;
    out.x = fp_zero();
    out.y = fp_zero();
    return REJ_OK;
  }
  const bool sign = (b0 & 0x20) != 0;
  uint8_t hi[48];
  for (int i = 0; i < 48; i++) hi[i] = in[i];
  hi[0] &= 0x1f;
  fp xr = fp_raw_from_be48(hi);
  if (!fp_raw_lt_p(xr)) return REJ_X_GE_P;
  fp x = fp_to_mont(xr);
  fp rhs = fp_add(fp_mul(fp_sqr(x), x), fp_mul4(fp_one()));
  fp y = fp_mul(fp_pow_sqrt_inv(rhs), rhs);
  if (!fp_eq(fp_sqr(y), rhs)) return REJ_NOT_ON_CURVE;
  if (fp_raw_gt_half(fp_from_mont(y)) != sign) y = fp_neg(y);
  out.x = x;
  out.y = y;
  if (!g1_in_subgroup(jac_from_aff(out))) return REJ_NOT_IN_SUBGROUP;
  return REJ_OK;
}

DI void g1_compress(uint8_t* out, const g1j& p) {
  if (jac_is_inf(p)) {
    out[0] = 0xc0;
    for (int i = 1; i < 48; i++) out[i] = 0;
    return;
  }
  g1a a = g1_to_aff(p);
  fp_raw_to_be48(out, fp_from_mont(a.x));
  out[0] |= 0x80 | (fp_raw_gt_half(fp_from_mont(a.y)) ? 0x20 : 0x00);
}

}  // namespace bls

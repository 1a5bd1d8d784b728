// Three lanes per Fp12 ("tri" layout) for the Fp12-heavy stages on gfx950.
//
// One lane per beacon holds an Fp12 in 144 VGPRs, and the Fp12 kernels then run at one wave per SIMD
// where a wave issues a v_mad_u64_u32 only every ~6.2 cycles (profiles/r01_madbench.txt; 2 waves:
// 5.0, 8 waves: 4.25). Here the Fp12 is split over 3 consecutive lanes of a wave:
//
//   Fp12 = Fp4[w] / (w^3 - s),  Fp4 = Fp2[s] / (s^2 - xi),  s = w^3
//   f = sum_k c_k w^k (k = 0..5)  ->  A_j = c_j + c_{j+3} s   (j = 0, 1, 2),  f = A0 + A1 w + A2 w^2
//
// In the tower of tower.h (c0.c0 = c_0, c1.c0 = c_1, c0.c1 = c_2, c1.c1 = c_3, c0.c2 = c_4, c1.c2 = c_5):
//   lane role 0: A0 = (c0.c0, c1.c1)   role 1: A1 = (c1.c0, c0.c2)   role 2: A2 = (c0.c1, c1.c2)
//
// Every lane runs the same instruction stream on its own third (no divergence); the few cross-third
// terms travel through ds_bpermute (4 bytes per lane per instruction, no LDS allocation). The work
// per Fp12 product is the tower's (18 Fp2 products, Karatsuba over the cubic extension); the
// Granger-Scott cyclotomic square is naturally three independent Fp4 squares.
// Lanes 0..62 form 21 groups; lane 63 computes on a dummy group and never stores.
#pragma once
#include "soa.h"

#ifndef BLS_HOST
namespace bls {

constexpr int TRI_GROUPS = 21;  // beacons per 64-lane wave

struct fp4 {
  fp2 a, b;  // a + b s
};

DI fp4 fp4_add(const fp4& x, const fp4& y) { return {fp2_add(x.a, y.a), fp2_add(x.b, y.b)}; }
DI fp4 fp4_sub(const fp4& x, const fp4& y) { return {fp2_sub(x.a, y.a), fp2_sub(x.b, y.b)}; }
DI fp4 fp4_dbl(const fp4& x) { return {fp2_dbl(x.a), fp2_dbl(x.b)}; }
DI fp4 fp4_add_lazy(const fp4& x, const fp4& y) { return {fp2_add_lazy(x.a, y.a), fp2_add_lazy(x.b, y.b)}; }
DI fp4 fp4_select(bool c, const fp4& x, const fp4& y) { return {fp2_select(c, x.a, y.a), fp2_select(c, x.b, y.b)}; }
// x * s = xi b + a s
DI fp4 fp4_mul_s(const fp4& x) { return {fp2_mul_xi(x.b), x.a}; }

// (xa + xb s)(ya + yb s) = xa ya + xi xb yb + ((xa + xb)(ya + yb) - xa ya - xb yb) s: 3 Fp2 products
DI fp4 fp4_mul(const fp4& x, const fp4& y) {
  const fp2 t0 = fp2_mul(x.a, y.a);
  const fp2 t1 = fp2_mul(x.b, y.b);
  const fp2 t2 = fp2_mul(fp2_add_lazy(x.a, x.b), fp2_add_lazy(y.a, y.b));
  return {fp2_add(t0, fp2_mul_xi(t1)), fp2_sub(fp2_sub(t2, t0), t1)};
}

// (a + b s)^2 = a^2 + xi b^2 + ((a + b)^2 - a^2 - b^2) s: 3 Fp2 squares, expanded in place (the
// cyclotomic squaring loop is call-free so its kernel keeps a small register budget)
DI fp4 fp4_sqr_inl(const fp4& x) {
  const fp2 t0 = fp2_sqr_inl(x.a);
  const fp2 t1 = fp2_sqr_inl(x.b);
  const fp2 t2 = fp2_sqr_inl(fp2_add_lazy(x.a, x.b));
  return {fp2_add(t0, fp2_mul_xi(t1)), fp2_sub(fp2_sub(t2, t0), t1)};
}

DI fp4 fp4_sqr(const fp4& x) {
  const fp2 t0 = fp2_sqr(x.a);
  const fp2 t1 = fp2_sqr(x.b);
  const fp2 t2 = fp2_sqr(fp2_add_lazy(x.a, x.b));
  return {fp2_add(t0, fp2_mul_xi(t1)), fp2_sub(fp2_sub(t2, t0), t1)};
}

// ------------------------------------------------------------------ lane bookkeeping
struct tri_lane {
  unsigned lane;   // 0..63
  unsigned role;   // j of A_j
  unsigned group;  // beacon slot within the wave (21 = the dummy lane 63)
  int next_b;      // ds_bpermute byte address of the role (j+1) mod 3 lane of the group
  int prev_b;      // ... of the role (j+2) mod 3 lane
};

DI tri_lane tri_lane_id() {
  tri_lane t;
  t.lane = threadIdx.x & 63u;
  t.group = t.lane / 3u;
  t.role = t.lane - 3u * t.group;
  const unsigned base = 3u * t.group;
  t.next_b = (int)(4u * ((base + (t.role + 1u) % 3u) & 63u));
  t.prev_b = (int)(4u * ((base + (t.role + 2u) % 3u) & 63u));
  return t;
}

// value of `v` held by the lane at byte address `src_b` (every lane of the wave must be active)
DI fp xchg_fp(const fp& v, int src_b) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = (uint32_t)__builtin_amdgcn_ds_bpermute(src_b, (int)v.l[i]);
  return r;
}
DI fp2 xchg_fp2(const fp2& v, int src_b) { return {xchg_fp(v.c0, src_b), xchg_fp(v.c1, src_b)}; }
DI fp4 xchg_fp4(const fp4& v, int src_b) { return {xchg_fp2(v.a, src_b), xchg_fp2(v.b, src_b)}; }

// SoA staging slots (soa.h st_fp12 order: c0.c0 = 0, c0.c1 = 2, c0.c2 = 4, c1.c0 = 6, c1.c1 = 8,
// c1.c2 = 10) of this lane's third
DI int tri_slot_a(unsigned role) { return role == 0 ? 0 : (role == 1 ? 6 : 2); }
DI int tri_slot_b(unsigned role) { return role == 0 ? 8 : (role == 1 ? 4 : 10); }

DI fp4 tri_load(const uint32_t* buf, size_t n, size_t i, unsigned role) {
  return {ld_fp2(buf, n, i, tri_slot_a(role)), ld_fp2(buf, n, i, tri_slot_b(role))};
}
DI void tri_store(uint32_t* buf, size_t n, size_t i, unsigned role, const fp4& x) {
  st_fp2(buf, n, i, tri_slot_a(role), x.a);
  st_fp2(buf, n, i, tri_slot_b(role), x.b);
}

// ------------------------------------------------------------------ Fp12 operations on thirds
// f^(p^6): negate the odd powers c1, c3, c5 -> role 0 negates b (c3), role 1 a (c1), role 2 b (c5)
DI fp4 tri_conj(const tri_lane& t, const fp4& x) {
  const bool neg_a = t.role == 1;
  return {fp2_select(neg_a, fp2_neg(x.a), x.a), fp2_select(neg_a, x.b, fp2_neg(x.b))};
}

// Granger-Scott cyclotomic square (tower.h fp12_cyclotomic_sqr) with z0..z5 = c0, c3, c1, c4, c2, c5:
// each lane squares its Fp4 (X = A_j^2); roles 1 and 2 swap their squares; then
//   role 0, 2: (a, b) <- (3 Y.a - 2 a, 3 Y.b + 2 b)     (role 0: Y = own square, role 2: role 1's)
//   role 1:    (a, b) <- (3 xi Y.b + 2 a, 3 Y.a - 2 b)  (Y = role 2's square)
DI fp4 tri_cyclotomic_sqr(const tri_lane& t, const fp4& x) {
  const fp4 sq = fp4_sqr_inl(x);
  const int src = t.role == 1 ? t.next_b : (t.role == 2 ? t.prev_b : (int)(4u * t.lane));
  const fp4 y = xchg_fp4(sq, src);
  const bool r1 = t.role == 1;
  const fp2 u = fp2_select(r1, fp2_mul_xi(y.b), y.a);
  const fp2 v = fp2_select(r1, y.a, y.b);
  const fp2 u3 = fp2_add(fp2_dbl(u), u), v3 = fp2_add(fp2_dbl(v), v);
  const fp2 a2 = fp2_dbl(x.a), b2 = fp2_dbl(x.b);
  return {fp2_select(r1, fp2_add(u3, a2), fp2_sub(u3, a2)), fp2_select(r1, fp2_sub(v3, b2), fp2_add(v3, b2))};
}

// general product (Karatsuba over the cubic): lane j forms P_j = A_j B_j and
// Q_j = (A_j + A_{j+1})(B_j + B_{j+1}); with w^3 = s
//   C0 = P0 + s (Q1 - P1 - P2),  C1 = Q0 - P0 - P1 + s P2,  C2 = Q2 - P2 - P0 + P1
DI fp4 tri_mul(const tri_lane& t, const fp4& a, const fp4& b) {
  const fp4 an = xchg_fp4(a, t.next_b);
  const fp4 bn = xchg_fp4(b, t.next_b);
  const fp4 P = fp4_mul(a, b);
  const fp4 Q = fp4_mul(fp4_add_lazy(a, an), fp4_add_lazy(b, bn));
  const fp4 Pn = xchg_fp4(P, t.next_b);                           // r0: P1  r1: P2  r2: P0
  const fp4 Pp = xchg_fp4(P, t.prev_b);                           // r0: P2  r1: P0  r2: P1
  const fp4 Qx = xchg_fp4(Q, t.role == 0 ? t.next_b : t.prev_b);  // r0: Q1  r1: Q0
  // r0: P + s (Qx - Pn - Pp);  r1: Qx - Pp - P + s Pn;  r2: Q - P - Pn + Pp
  const fp4 k0 = fp4_add(P, fp4_mul_s(fp4_sub(fp4_sub(Qx, Pn), Pp)));
  const fp4 k1 = fp4_add(fp4_sub(fp4_sub(Qx, Pp), P), fp4_mul_s(Pn));
  const fp4 k2 = fp4_add(fp4_sub(fp4_sub(Q, P), Pn), Pp);
  return fp4_select(t.role == 0, k0, fp4_select(t.role == 1, k1, k2));
}

// general square (Miller loop): S_j = A_j^2, M_j = A_j A_{j+1};
//   C0 = S0 + 2 s M1,  C1 = 2 M0 + s S2,  C2 = S1 + 2 M2
DI fp4 tri_sqr(const tri_lane& t, const fp4& a) {
  const fp4 an = xchg_fp4(a, t.next_b);
  const fp4 S = fp4_sqr(a);
  const fp4 M = fp4_mul(a, an);
  const fp4 Mx = xchg_fp4(M, t.role == 0 ? t.next_b : t.prev_b);  // r0: M1  r1: M0
  const fp4 Sx = xchg_fp4(S, t.role == 1 ? t.next_b : t.prev_b);  // r1: S2  r2: S1
  const fp4 k0 = fp4_add(S, fp4_mul_s(fp4_dbl(Mx)));
  const fp4 k1 = fp4_add(fp4_dbl(Mx), fp4_mul_s(Sx));
  const fp4 k2 = fp4_add(Sx, fp4_dbl(M));
  return fp4_select(t.role == 0, k0, fp4_select(t.role == 1, k1, k2));
}

// Frobenius f^p: c_k -> conj(c_k) gamma1^k; lane j holds c_j, c_{j+3}
DI fp4 tri_frob(const tri_lane& t, const fp4& x) {
  const int j = (int)t.role;
  fp2 ga = fp2_load_const(FROB1_GAMMA[0]), gb = fp2_load_const(FROB1_GAMMA[3]);
  ga = fp2_select(j == 1, fp2_load_const(FROB1_GAMMA[1]), fp2_select(j == 2, fp2_load_const(FROB1_GAMMA[2]), ga));
  gb = fp2_select(j == 1, fp2_load_const(FROB1_GAMMA[4]), fp2_select(j == 2, fp2_load_const(FROB1_GAMMA[5]), gb));
  return {fp2_mul(fp2_conj(x.a), ga), fp2_mul(fp2_conj(x.b), gb)};
}

// f^(p^2): c_k -> c_k gamma2^k (gamma2^k in Fp)
DI fp4 tri_frob2(const tri_lane& t, const fp4& x) {
  const int j = (int)t.role;
  fp ga = fp_load_const(FROB2_GAMMA[0][0]), gb = fp_load_const(FROB2_GAMMA[3][0]);
  ga = fp_select(j == 1, fp_load_const(FROB2_GAMMA[1][0]), fp_select(j == 2, fp_load_const(FROB2_GAMMA[2][0]), ga));
  gb = fp_select(j == 1, fp_load_const(FROB2_GAMMA[4][0]), fp_select(j == 2, fp_load_const(FROB2_GAMMA[5][0]), gb));
  return {fp2_mul_fp(x.a, ga), fp2_mul_fp(x.b, gb)};
}

// this lane's part of "f == 1": role 0 must hold (1, 0), roles 1, 2 zero; combined over the group
DI bool tri_is_one(const tri_lane& t, const fp4& x) {
  const fp2 want_a = fp2_select(t.role == 0, fp2_one(), fp2_zero());
  const int mine = (fp2_eq(x.a, want_a) & fp2_is_zero(x.b)) ? 1 : 0;
  const int n1 = __builtin_amdgcn_ds_bpermute(t.next_b, mine);
  const int n2 = __builtin_amdgcn_ds_bpermute(t.prev_b, mine);
  return (mine & n1 & n2) != 0;
}

}  // namespace bls
#endif  // BLS_HOST

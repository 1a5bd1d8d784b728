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

namespace bls {

struct fp4 {
  fp2 a, b;  // a + b s
};

// (a + b s)^2 = (a^2 + xi b^2) + 2ab s with SEVEN radix-2^28 product columns and four reductions
// (a, b < 2p), against ten products for four separate dot products (fp4_sqr_dot below):
//   Y.a.c0 = A + T - V      A = (a0 + a1)(a0 - a1)   T = (b0 + b1)(b0 - b1)   V = (2 b0) b1
//   Y.a.c1 = C + T + V      C = (2 a0) a1            (a^2 + xi b^2: xi (x0 + x1 i) = (x0 - x1) + (x0 + x1) i)
//   Y.b    = a (2b)         Karatsuba columns as fp2_mul_body_kara (three products, two reductions)
// T and V are formed once per column and added to both outputs. The differences a0 - a1, b0 - b1
// are SIGNED limbs (|.| < 2^28, products through v_mad_i64_i32), so every column of the Y.a pair
// stays within a signed 64-bit accumulator: |A_k|, |T_k| < 14 * 2^57, V_k, C_k < 14 * 2^57, the
// reduction < 14 * 2^56: |column| < 2^62.5. The totals can be negative (A + T - V >= -16 p^2,
// C + T + V >= -4 p^2), so a result may come out in (-p/128, 0): one conditional + p puts it in
// [0, 2p). Y.b: a0, a1 < 2p and 2b0, 2b1 < 4p keep fp2_mul_body_kara's bounds (its operands < 8p).
DI void fp4_sqr_ya_t(const uint32_t (&a0)[14], const uint32_t (&a1)[14], const uint32_t (&b0)[14],
                     const uint32_t (&b1)[14], uint32_t (&t0)[14], uint32_t (&t1)[14], bool& neg0, bool& neg1) {
  int32_t am[14], bm[14];
  uint32_t ap[14], bp[14], a02[14], b02[14];
#pragma unroll
  for (int k = 0; k < 14; k++) {
    ap[k] = a0[k] + a1[k];
    am[k] = (int32_t)a0[k] - (int32_t)a1[k];
    bp[k] = b0[k] + b1[k];
    bm[k] = (int32_t)b0[k] - (int32_t)b1[k];
    a02[k] = a0[k] << 1;
    b02[k] = b0[k] << 1;
  }
  uint32_t m0[14], m1[14];
  int64_t c0 = 0, c1 = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
    int64_t T = 0;
    uint64_t V = 0;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      c0 += (int64_t)(int32_t)ap[j] * (int64_t)am[k - j];
      c1 += (int64_t)((uint64_t)a02[j] * a1[k - j]);
      T += (int64_t)(int32_t)bp[j] * (int64_t)bm[k - j];
      V += (uint64_t)b02[j] * b1[k - j];
    }
    c0 += T - (int64_t)V;
    c1 += T + (int64_t)V;
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) {
        c0 += (int64_t)((uint64_t)m0[j] * P28[k - j]);
        c1 += (int64_t)((uint64_t)m1[j] * P28[k - j]);
      }
      m0[k] = ((uint32_t)c0 * P_INV28) & M28;
      m1[k] = ((uint32_t)c1 * P_INV28) & M28;
      c0 += (int64_t)((uint64_t)m0[k] * P28[0]);
      c1 += (int64_t)((uint64_t)m1[k] * P28[0]);
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) {
        c0 += (int64_t)((uint64_t)m0[j] * P28[k - j]);
        c1 += (int64_t)((uint64_t)m1[j] * P28[k - j]);
      }
      t0[k - 14] = (uint32_t)c0 & M28;
      t1[k - 14] = (uint32_t)c1 & M28;
    }
    c0 >>= 28;  // arithmetic: the column sums are signed
    c1 >>= 28;
  }
  t0[13] = (uint32_t)c0;
  t1[13] = (uint32_t)c1;
  neg0 = c0 < 0;
  neg1 = c1 < 0;
}

// 12-word value of limbs t (top limb signed) plus p when neg: [0, 2p) for a value in (-p, p)
DI u12 fp_join28_fix(const uint32_t (&t)[14], bool neg) {
  const u12 w = fp_join28(t);
  const uint32_t msk = neg ? 0xffffffffu : 0u;
  u12 r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = __builtin_addc(w[i], P_RAW[i] & msk, c, &c);
  return r;
}

DI fp4 fp4_sqr_k7(const fp4& x) {
  uint32_t a0[14], a1[14], b0[14], b1[14];
  fp_split28(fp_to_u12(x.a.c0), a0);
  fp_split28(fp_to_u12(x.a.c1), a1);
  fp_split28(fp_to_u12(x.b.c0), b0);
  fp_split28(fp_to_u12(x.b.c1), b1);
  fp4 y;
  {
    uint32_t t0[14], t1[14];
    bool n0, n1;
    fp4_sqr_ya_t(a0, a1, b0, b1, t0, t1, n0, n1);
    y.a.c0 = fp_from_u12(fp_join28_fix(t0, n0));
    y.a.c1 = fp_from_u12(fp_join28_fix(t1, n1));
  }
  BLS_SCHED_FENCE();
  {
    uint32_t ys[14], xz[14], xy[14], y0[14], y1[14], t0[14], t1[14];
#pragma unroll
    for (int k = 0; k < 14; k++) {  // Y.b = a (2b): y = 2b, limbs < 2^29
      y0[k] = b0[k] << 1;
      y1[k] = b1[k] << 1;
      ys[k] = y0[k] + y1[k];
      xz[k] = NEG28_32P[k] - a0[k] - a1[k];
      xy[k] = a1[k] + (NEG28_16P[k] - a0[k]);
    }
    fp2_mont_kara_t(a0, ys, y1, xz, y0, xy, t0, t1);
    y.b.c0 = fp_from_u12(fp_join28(t0));
    y.b.c1 = fp_from_u12(fp_join28(t1));
  }
  return y;
}

}  // namespace bls

#ifndef BLS_HOST
namespace bls {

constexpr int TRI_GROUPS = 21;  // beacons per 64-lane wave

// per-lane LDS columns of the staged product operands (see "low register pressure products" below)
constexpr int TRI_ARG_WORDS = 72;
static __shared__ __attribute__((aligned(16))) uint32_t g_tri_arg[TRI_ARG_WORDS * BLS_LANES];

// role-dependent additions as one fp_addsub (direction as data) instead of both results + a select

DI fp4 fp4_add(const fp4& x, const fp4& y) { return {fp2_add(x.a, y.a), fp2_add(x.b, y.b)}; }
DI fp4 fp4_sub(const fp4& x, const fp4& y) { return {fp2_sub(x.a, y.a), fp2_sub(x.b, y.b)}; }
DI fp4 fp4_dbl(const fp4& x) { return {fp2_dbl(x.a), fp2_dbl(x.b)}; }
DI fp4 fp4_add_lazy(const fp4& x, const fp4& y) { return {fp2_add_lazy(x.a, y.a), fp2_add_lazy(x.b, y.b)}; }
DI fp4 fp4_addsub(const fp4& x, const fp4& y, bool sub) { return {fp2_addsub(x.a, y.a, sub), fp2_addsub(x.b, y.b, sub)}; }
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

// (a + b s)^2 = (a^2 + xi b^2) + 2ab s as four Montgomery dot products, for a, b < 2p (one reduction
// per output component instead of two per Fp2 square, and no additions after the products):
//   Y.a.c0 = (a0 + a1)(a0 - a1) + (b0 + b1)(b0 - b1) + (2 b0)(-b1)      Y.a.c1 = (2 a0) a1 + (b0 + b1)(b0 - b1) + (2 b0) b1
//   Y.b.c0 = (2 a0) b0 + (2 a1)(-b1)                                  Y.b.c1 = (2 a0) b1 + (2 a1) b0
// with -y formed limb-wise as NEG28_4P - y (10 products, 4 reductions: 14 units against 12 for three
// squares, but without the 12 reductions' worth of glue around them)
DI fp4 fp4_sqr_dot(const fp4& x) {
  uint32_t a0[14], a1[14], b0[14], b1[14];
  fp_split28(fp_to_u12(x.a.c0), a0);
  fp_split28(fp_to_u12(x.a.c1), a1);
  fp_split28(fp_to_u12(x.b.c0), b0);
  fp_split28(fp_to_u12(x.b.c1), b1);
  uint32_t ap[14], am[14], bp[14], bm[14], b02[14], nb1[14];
#pragma unroll
  for (int k = 0; k < 14; k++) {
    ap[k] = a0[k] + a1[k];
    am[k] = a0[k] + (NEG28_4P[k] - a1[k]);
    bp[k] = b0[k] + b1[k];
    bm[k] = b0[k] + (NEG28_4P[k] - b1[k]);
    b02[k] = b0[k] << 1;
    nb1[k] = NEG28_4P[k] - b1[k];
  }
  fp4 y;
  y.a.c0 = fp_from_u12(fp_mont_dot3<3>(ap, am, bp, bm, b02, nb1));
  BLS_SCHED_FENCE();
  uint32_t a02[14];
#pragma unroll
  for (int k = 0; k < 14; k++) a02[k] = a0[k] << 1;
  y.a.c1 = fp_from_u12(fp_mont_dot3<3>(a02, a1, bp, bm, b02, b1));
  BLS_SCHED_FENCE();
  uint32_t a12[14];
#pragma unroll
  for (int k = 0; k < 14; k++) a12[k] = a1[k] << 1;
  y.b.c0 = fp_from_u12(fp_mont_dot3<2>(a02, b0, a12, nb1, a12, nb1));
  BLS_SCHED_FENCE();
  y.b.c1 = fp_from_u12(fp_mont_dot3<2>(a02, b1, a12, b0, a12, b0));
  return y;
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
  return {ld_fp2_v(buf, n, i, tri_slot_a(role)), ld_fp2_v(buf, n, i, tri_slot_b(role))};
}
DI void tri_store(uint32_t* buf, size_t n, size_t i, unsigned role, const fp4& x) {
  st_fp2_v(buf, n, i, tri_slot_a(role), x.a);
  st_fp2_v(buf, n, i, tri_slot_b(role), x.b);
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
#ifndef BLS_FP4_SQR_K7
#define BLS_FP4_SQR_K7 1
#endif
#ifndef BLS_CSQR_PARK
#define BLS_CSQR_PARK 1
#endif
#ifndef BLS_CSQR_LIN
#define BLS_CSQR_LIN 1
#endif
// x parked in this lane's first 48 words of g_tri_arg (the staging slots 0 and 1, free between the
// products) as 12 16-byte columns: the square's limb arrays then have the register file to themselves
// (with x held across the square, the K7 body spilled 24 dwords per square to scratch: 18 KB of HBM
// reads per beacon per fexp launch).
DI void tri_park4(const fp4& x) {
  uint4* q = reinterpret_cast<uint4*>(g_tri_arg) + threadIdx.x;
  const fp2* h[2] = {&x.a, &x.b};
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int k = 0; k < 3; k++) {
      q[(6 * s + k) * BLS_LANES] = make_uint4(h[s]->c0.l[4 * k], h[s]->c0.l[4 * k + 1], h[s]->c0.l[4 * k + 2], h[s]->c0.l[4 * k + 3]);
      q[(6 * s + 3 + k) * BLS_LANES] = make_uint4(h[s]->c1.l[4 * k], h[s]->c1.l[4 * k + 1], h[s]->c1.l[4 * k + 2], h[s]->c1.l[4 * k + 3]);
    }
}
DI fp4 tri_unpark4() {
  const uint4* q = reinterpret_cast<const uint4*>(g_tri_arg) + threadIdx.x;
  fp4 x;
  fp2* h[2] = {&x.a, &x.b};
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int k = 0; k < 3; k++) {
      const uint4 u = q[(6 * s + k) * BLS_LANES], v = q[(6 * s + 3 + k) * BLS_LANES];
      h[s]->c0.l[4 * k] = u.x, h[s]->c0.l[4 * k + 1] = u.y, h[s]->c0.l[4 * k + 2] = u.z, h[s]->c0.l[4 * k + 3] = u.w;
      h[s]->c1.l[4 * k] = v.x, h[s]->c1.l[4 * k + 1] = v.y, h[s]->c1.l[4 * k + 2] = v.z, h[s]->c1.l[4 * k + 3] = v.w;
    }
  return x;
}

// the reduction multiple of the fused 3u +- 2x (tower.h fp2_3u_pm_2x, q <= 10) from an LDS table of
// k p, k < 11 (528 bytes per workgroup, tower.h kp_lds_init / KpLdsK; k_fexp_tri writes it)
using KpLds = KpLdsK<11>;

DI fp4 tri_cyclotomic_sqr(const tri_lane& t, const fp4& x_in) {
#if BLS_CSQR_PARK
  tri_park4(x_in);
  asm volatile("" ::: "memory");  // the park is neither sunk below the square nor forwarded past it
#endif
  const fp4 sq = BLS_FP4_SQR_K7 ? fp4_sqr_k7(x_in) : fp4_sqr_dot(x_in);
  const int src = t.role == 1 ? t.next_b : (t.role == 2 ? t.prev_b : (int)(4u * t.lane));
  const fp4 y = xchg_fp4(sq, src);
#if BLS_CSQR_PARK
  asm volatile("" ::: "memory");
  const fp4 x = tri_unpark4();
#else
  const fp4& x = x_in;
#endif
  const bool r1 = t.role == 1;
  const fp2 u = fp2_select(r1, fp2_mul_xi(y.b), y.a);
  const fp2 v = fp2_select(r1, y.a, y.b);
#if BLS_CSQR_LIN
  // 3u +- 2a as one linear form and one reduction (tower.h fp2_3u_pm_2x), direction by role
  const fp uu[4] = {u.c0, u.c1, v.c0, v.c1}, xx[4] = {x.a.c0, x.a.c1, x.b.c0, x.b.c1};
  const bool ss[4] = {!r1, !r1, r1, r1};
  fp o[4];
  fp_3u_pm_2x_n<4>(uu, xx, ss, o, KpLds());
  return {{o[0], o[1]}, {o[2], o[3]}};
#else
  // 3u +- 2a = 2(u +- a) + u: one direction-by-role addition instead of both and a select
  const fp2 ta = fp2_addsub(u, x.a, !r1), tb = fp2_addsub(v, x.b, r1);
  return {fp2_add(fp2_dbl(ta), u), fp2_add(fp2_dbl(tb), v)};
#endif
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

// ------------------------------------------------------------------ low register pressure products
// A called fp2 product clobbers every caller-saved VGPR, so whatever the caller keeps live across the
// call must sit in the callee-saved half of the file (112 VGPRs at a 256-VGPR budget) or be spilled
// around each call. The Miller f pass therefore stages its second operands in LDS: each lane owns a
// 72-word column (3 Fp2 slots). A staged Fp4 y sits there as (y.a, y.b, y.a + y.b), and an Fp4
// product x y keeps only x and its partial products in VGPRs across the three calls. 72 words x 64
// lanes = 18 KB per one-wave workgroup: 8 workgroups (2 waves/SIMD) fit the CU's 160 KB.

DI void tri_arg_put(int slot, const fp2& v) {
  const unsigned l = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    g_tri_arg[(slot * 24 + k) * BLS_LANES + l] = v.c0.l[k];
    g_tri_arg[(slot * 24 + 12 + k) * BLS_LANES + l] = v.c1.l[k];
  }
}
DI fp2 tri_arg_get(int slot) {
  const unsigned l = threadIdx.x;
  fp2 v;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    v.c0.l[k] = g_tri_arg[(slot * 24 + k) * BLS_LANES + l];
    v.c1.l[k] = g_tri_arg[(slot * 24 + 12 + k) * BLS_LANES + l];
  }
  return v;
}

// LDS slot layout per lane: slot 0 = y.a, slot 1 = y.b, slot 2 = the product's result. The callee
// reads b = slot 0, slot 1, or their lazy sum (sel 2), and writes a * b to slot 2: neither b nor the
// result travels in registers (a returned 24-word vector is spilled whole around the call site).
NOINL void fp2_mul_slot_u24(u24 a, int sel) {
  const unsigned l = threadIdx.x;
  u12 b0, b1;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const uint32_t p0 = g_tri_arg[k * BLS_LANES + l], p1 = g_tri_arg[(12 + k) * BLS_LANES + l];
    const uint32_t q0 = g_tri_arg[(24 + k) * BLS_LANES + l], q1 = g_tri_arg[(36 + k) * BLS_LANES + l];
    b0[k] = sel == 0 ? p0 : q0;
    b1[k] = sel == 0 ? p1 : q1;
  }
  if (sel == 2) {  // y.a + y.b (< 4p each: the sum stays below 8p, fp.h operand contract)
    u12 a0, a1;
#pragma unroll
    for (int k = 0; k < 12; k++) {
      a0[k] = g_tri_arg[k * BLS_LANES + l];
      a1[k] = g_tri_arg[(12 + k) * BLS_LANES + l];
    }
    b0 = fp_add_raw_u12(b0, a0);
    b1 = fp_add_raw_u12(b1, a1);
  }
  const u24 r = fp2_mul_body(a, b0, b1);
#pragma unroll
  for (int k = 0; k < 24; k++) g_tri_arg[(48 + k) * BLS_LANES + l] = r[k];
}
// The argument vector is rebuilt from opaque words at every call: a CSE'd 24-word argument vector
// live across later calls would be spilled whole (as a 32-register tuple).
DI u24 fp2_to_u24_fresh(const fp2& a) {
  fp2 c = a;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    asm volatile("" : "+v"(c.c0.l[k]));
    asm volatile("" : "+v"(c.c1.l[k]));
  }
  return fp2_to_u24(c);
}
DI fp2 fp2_mul_slot(const fp2& a, int sel) {
  fp2_mul_slot_u24(fp2_to_u24_fresh(a), sel);
  return tri_arg_get(2);
}
// a^2 into slot 2 (slots 0, 1 untouched)
NOINL void fp2_sqr_slot_u24(u24 a) {
  const unsigned l = threadIdx.x;
  const u24 r = fp2_sqr_body(a);
#pragma unroll
  for (int k = 0; k < 24; k++) g_tri_arg[(48 + k) * BLS_LANES + l] = r[k];
}
DI fp2 fp2_sqr_slot(const fp2& a) {
  fp2_sqr_slot_u24(fp2_to_u24_fresh(a));
  return tri_arg_get(2);
}
DI fp4 fp4_sqr_slot(const fp4& x) {
  const fp2 t0 = fp2_sqr_slot(x.a);
  const fp2 t1 = fp2_sqr_slot(x.b);
  const fp2 t2 = fp2_sqr_slot(fp2_add_lazy(x.a, x.b));
  return {fp2_add(t0, fp2_mul_xi(t1)), fp2_sub(fp2_sub(t2, t0), t1)};
}
DI fp4 fp4_neg(const fp4& x) { return {fp2_neg(x.a), fp2_neg(x.b)}; }

// one product: b through slot 0
DI fp2 fp2_mul_staged1(const fp2& a, const fp2& b) {
  tri_arg_put(0, b);
  return fp2_mul_slot(a, 0);
}
DI void fp4_stage(const fp4& y) {
  tri_arg_put(0, y.a);
  tri_arg_put(1, y.b);
}
// x * (staged y), Karatsuba over s as fp4_mul
DI fp4 fp4_mul_staged(const fp4& x) {
  const fp2 t0 = fp2_mul_slot(x.a, 0);
  const fp2 t1 = fp2_mul_slot(x.b, 1);
  const fp2 t2 = fp2_mul_slot(fp2_add_lazy(x.a, x.b), 2);
  return {fp2_add(t0, fp2_mul_xi(t1)), fp2_sub(fp2_sub(t2, t0), t1)};
}

// tri_sqr with at most one Fp4 plus partial products live at any call: M is exchanged and parked in
// LDS while the squares run.
DI fp4 tri_sqr_lp(const tri_lane& t, const fp4& a) {
  const int self_b = (int)(4u * t.lane);
  fp4_stage(xchg_fp4(a, t.next_b));
  const fp4 M = fp4_mul_staged(a);                                                   // M_j = A_j A_{j+1}
  const fp4 Mx = xchg_fp4(M, t.role == 0 ? t.next_b : (t.role == 1 ? t.prev_b : self_b));  // r0: M1 r1: M0 r2: M2
  tri_arg_put(0, Mx.a);
  tri_arg_put(1, Mx.b);
  const fp4 S = fp4_sqr_slot(a);                                                      // S_j = A_j^2
  const fp4 Sx = xchg_fp4(S, t.role == 1 ? t.next_b : (t.role == 2 ? t.prev_b : self_b));  // r0: S0 r1: S2 r2: S1
  // r0: S0 + s 2 M1,  r1: 2 M0 + s S2,  r2: S1 + 2 M2
  const fp4 U = fp4_select(t.role == 1, fp4_mul_s(Sx), Sx);
  const fp4 D = fp4_dbl(fp4{tri_arg_get(0), tri_arg_get(1)});
  return fp4_add(U, fp4_select(t.role == 0, fp4_mul_s(D), D));
}

// This lane's third of L = l_0 l_1, the product of the two pairs' sparse lines of one Miller step
// (pairing.h line_mul_line; L.c1.c0 = 0), with two Fp2 products per lane:
//   r0: X = t00, Y = t44;  r1: X = t11, Y = K01;  r2: X = K04, Y = K14
// (t_kk = a_k b_k, K_jk = (a_j + a_k)(b_j + b_k); a = pair 0's line, b = pair 1's; components 0, 1, 2 =
// the line's a0, a1, a4). la(c) / lb(c) load component c of the two lines.
template <typename LoadA, typename LoadB>
DI fp4 tri_line_pair(const tri_lane& t, LoadA la, LoadB lb) {
  const unsigned r = t.role;
  const int xc = r == 1 ? 1 : 0;
  fp2 xa = la(xc), xb = lb(xc);
  if (r == 2) {
    xa = fp2_add_lazy(xa, la(2));
    xb = fp2_add_lazy(xb, lb(2));
  }
  const fp2 X = fp2_mul_staged1(xa, xb);
  const int yc = r == 0 ? 2 : (r == 1 ? 0 : 1);
  fp2 ya = la(yc), yb = lb(yc);
  if (r != 0) {
    const int yc2 = r == 1 ? 1 : 2;
    ya = fp2_add_lazy(ya, la(yc2));
    yb = fp2_add_lazy(yb, lb(yc2));
  }
  const fp2 Y = fp2_mul_staged1(ya, yb);
  const fp2 Xp = xchg_fp2(X, t.prev_b), Yp = xchg_fp2(Y, t.prev_b);
  const fp2 Xn = xchg_fp2(X, t.next_b), Yn = xchg_fp2(Y, t.next_b);
  // r0: (t00 + xi t44, K04 - t00 - t44)   r1: (0, t11)   r2: (K01 - t00 - t11, K14 - t11 - t44)
  const fp2 a0 = fp2_add(X, fp2_mul_xi(Y)), b0 = fp2_sub(fp2_sub(Xp, X), Y);
  const fp2 a2 = fp2_sub(fp2_sub(Yp, Xn), Xp), b2 = fp2_sub(fp2_sub(Y, Xp), Yn);
  return {fp2_select(r == 0, a0, fp2_select(r == 1, fp2_zero(), a2)), fp2_select(r == 0, b0, fp2_select(r == 1, X, b2))};
}

// tri_mul(a, b) with b staged in LDS; the partial result from P parks in `park` (a per-lane global
// SoA slot of 48 words: word w at park[w * park_n + park_i]) while Q is formed.
DI fp4 tri_mul_lp(const tri_lane& t, const fp4& a, const fp4& b, uint32_t* park, size_t park_n, size_t park_i) {
  const int self_b = (int)(4u * t.lane);
  fp4_stage(b);
  const fp4 P = fp4_mul_staged(a);  // P_j = A_j B_j
  {
    const fp4 br = {tri_arg_get(0), tri_arg_get(1)};
    fp4_stage(fp4_add_lazy(br, xchg_fp4(br, t.next_b)));  // B_j + B_{j+1}
  }
  // partial results without Q:  r0: P - s (Pn + Pp),  r1: s Pn - Pp - P,  r2: Pp - P - Pn, built one
  // exchanged term at a time (fewer Fp4 values live)
  fp4 R = fp4_select(t.role == 0, P, fp4_neg(P));
  {
    const fp4 Pn = xchg_fp4(P, t.next_b);
    const fp4 u = fp4_select(t.role == 2, Pn, fp4_mul_s(Pn));
    R = fp4_addsub(R, u, t.role != 1);
  }
  {
    const fp4 Pp = xchg_fp4(P, t.prev_b);
    const fp4 u = fp4_select(t.role == 0, fp4_mul_s(Pp), Pp);
    R = fp4_addsub(R, u, t.role != 2);
  }
  {
    size_t j = park_i;
    asm volatile("" : "+v"(j));  // park addresses are formed here, not hoisted out of the Miller loop
    st_fp2(park, park_n, j, 0, R.a);
    st_fp2(park, park_n, j, 2, R.b);
  }
  const fp4 Q = fp4_mul_staged(fp4_add_lazy(a, xchg_fp4(a, t.next_b)));  // Q_j
  const fp4 Qx = xchg_fp4(Q, t.role == 0 ? t.next_b : (t.role == 1 ? t.prev_b : self_b));  // r0: Q1 r1: Q0 r2: Q2
  size_t j = park_i;
  asm volatile("" : "+v"(j));  // the park reload stays here
  const fp4 Rp = {ld_fp2(park, park_n, j, 0), ld_fp2(park, park_n, j, 2)};
  // r0: R + s Q1,  r1: R + Q0,  r2: R + Q2
  return fp4_add(Rp, fp4_select(t.role == 0, fp4_mul_s(Qx), Qx));
}

// Frobenius f^p: c_k -> conj(c_k) gamma1^k; lane j holds c_j, c_{j+3}
DI fp4 tri_frob(const tri_lane& t, const fp4& x) {
  const int j = (int)t.role;
  fp2 ga = fp2_load_const(FROB1_GAMMA[0]), gb = fp2_load_const(FROB1_GAMMA[3]);
  ga = fp2_select(j == 1, fp2_load_const(FROB1_GAMMA[1]), fp2_select(j == 2, fp2_load_const(FROB1_GAMMA[2]), ga));
  gb = fp2_select(j == 1, fp2_load_const(FROB1_GAMMA[4]), fp2_select(j == 2, fp2_load_const(FROB1_GAMMA[5]), gb));
  return {fp2_mul_staged1(fp2_conj(x.a), ga), fp2_mul_staged1(fp2_conj(x.b), gb)};
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

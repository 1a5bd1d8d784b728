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

// 3b' C = 12 (1 + i) C by additions
DI fp2 fp2_mul_3b(const fp2& c) {
  fp2 x4 = fp2_dbl(fp2_dbl(fp2_mul_xi(c)));
  return fp2_add(fp2_dbl(x4), x4);
}

// INL: the Fp2 products expanded in place (call-free step, see g2_dbl_inl in curve.h)
template <bool INL = false>
DI void miller_dbl_step(g2proj& t, fp2& l00, fp2& l01, fp2& l11, const fp& xp, const fp& yp) {
  auto mul = [](const fp2& a, const fp2& b) { return INL ? fp2_mul_inl(a, b) : fp2_mul(a, b); };
  auto sqr = [](const fp2& a) { return INL ? fp2_sqr_inl(a) : fp2_sqr(a); };
  fp2 A = fp2_half(mul(t.x, t.y));
  fp2 B = sqr(t.y);
  fp2 C = sqr(t.z);
  fp2 E = fp2_mul_3b(C);
  fp2 F = fp2_mul3(E);
  fp2 G = fp2_half(fp2_add(B, F));
  fp2 H = fp2_sub(sqr(fp2_add_lazy(t.y, t.z)), fp2_add(B, C));
  fp2 X2 = sqr(t.x);
  l00 = fp2_sub(E, B);
  l01 = fp2_mul_fp(fp2_mul3(X2), xp);
  l11 = fp2_neg(fp2_mul_fp(H, yp));
  t.x = mul(A, fp2_sub(B, F));
  t.y = fp2_sub(sqr(G), fp2_mul3(sqr(E)));
  t.z = mul(B, H);
}


// Call-free Miller steps (k_miller_lines at 2 waves/SIMD): every product expanded
// in place, one after the other (fenced), ordered so that few values are live at once, and each
// line coefficient handed to put(c, v) (c = 0: l00, 1: l01, 2: l11) as soon as it is known; xp()/yp()
// and the addition's q() re-read their operands at the use. Same operations on the same values as
// miller_dbl_step / miller_add_step.

// The running point T of the call-free steps is reached through an accessor: TS::get(c) / set(c, v)
// for c = 0, 1, 2 (X, Y, Z). TReg keeps T in registers; k_miller_lines parks it in LDS (its
// register budget at 2 waves/SIMD is then left to the products). Each coordinate is written back as
// soon as its old value has had its last use.
struct g2proj_reg {
  g2proj& t;
  DI fp2 get(int c) const { return c == 0 ? t.x : c == 1 ? t.y : t.z; }
  DI void set(int c, const fp2& v) const {
    if (c == 0) t.x = v;
    else if (c == 1) t.y = v;
    else t.z = v;
  }
};

template <typename TS, typename Put, typename XP, typename YP>
DI void miller_dbl_step_ts(const TS& t, Put put, XP xp, YP yp) {
  const fp2 B = fp2_sqr_inl(t.get(1));
  BLS_SCHED_FENCE();
  const fp2 C = fp2_sqr_inl(t.get(2));
  BLS_SCHED_FENCE();
  const fp2 H = fp2_sub(fp2_sqr_inl(fp2_add_lazy(t.get(1), t.get(2))), fp2_add(B, C));
  BLS_SCHED_FENCE();
  put(2, fp2_neg(fp2_mul_fp_inl(H, yp())));
  BLS_SCHED_FENCE();
  t.set(2, fp2_mul_inl_k<0>(B, H));  // Z3 (Z has had its last use)
  BLS_SCHED_FENCE();
  const fp2 E = fp2_mul_3b(C);
  const fp2 F = fp2_mul3(E);
  const fp2 G = fp2_half(fp2_add(B, F));
  put(0, fp2_sub(E, B));
  const fp2 BF = fp2_sub(B, F);
  const fp2 A = fp2_half(fp2_mul_inl_k<1>(t.get(0), t.get(1)));
  BLS_SCHED_FENCE();
  put(1, fp2_mul_fp_inl(fp2_mul3(fp2_sqr_inl(t.get(0))), xp()));
  BLS_SCHED_FENCE();
  t.set(0, fp2_mul_inl(A, BF));  // X3
  BLS_SCHED_FENCE();
  const fp2 G2 = fp2_sqr_inl(G);
  BLS_SCHED_FENCE();
  t.set(1, fp2_sub(G2, fp2_mul3(fp2_sqr_inl(E))));  // Y3
}

template <typename TS, typename Put, typename Q, typename XP, typename YP>
DI void miller_add_step_ts(const TS& t, Q qload, Put put, XP xp, YP yp) {
  fp2 theta, delta;
  {
    const g2a q = qload();
    theta = fp2_sub(t.get(1), fp2_mul_inl(q.y, t.get(2)));
    BLS_SCHED_FENCE();
    delta = fp2_sub(t.get(0), fp2_mul_inl(q.x, t.get(2)));
    BLS_SCHED_FENCE();
    const fp2 u = fp2_mul_inl(theta, q.x);
    BLS_SCHED_FENCE();
    put(0, fp2_sub(u, fp2_mul_inl(delta, q.y)));
    BLS_SCHED_FENCE();
  }
  put(1, fp2_neg(fp2_mul_fp_inl(theta, xp())));
  BLS_SCHED_FENCE();
  put(2, fp2_mul_fp_inl(delta, yp()));
  BLS_SCHED_FENCE();
  const fp2 C = fp2_sqr_inl(theta);
  BLS_SCHED_FENCE();
  const fp2 D = fp2_sqr_inl(delta);
  BLS_SCHED_FENCE();
  const fp2 E = fp2_mul_inl(D, delta);
  BLS_SCHED_FENCE();
  const fp2 F = fp2_mul_inl(t.get(2), C);
  BLS_SCHED_FENCE();
  const fp2 G = fp2_mul_inl(t.get(0), D);
  BLS_SCHED_FENCE();
  const fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  t.set(0, fp2_mul_inl(delta, H));  // X3 (X has had its last use)
  BLS_SCHED_FENCE();
  t.set(1, fp2_sub(fp2_mul_inl(theta, fp2_sub(G, H)), fp2_mul_inl(t.get(1), E)));  // Y3
  BLS_SCHED_FENCE();
  t.set(2, fp2_mul_inl(t.get(2), E));  // Z3
}

template <typename Put, typename XP, typename YP>
DI void miller_dbl_step_inl(g2proj& t, Put put, XP xp, YP yp) {
  miller_dbl_step_ts(g2proj_reg{t}, put, xp, yp);
}
template <typename Put, typename Q, typename XP, typename YP>
DI void miller_add_step_inl(g2proj& t, Q qload, Put put, XP xp, YP yp) {
  miller_add_step_ts(g2proj_reg{t}, qload, put, xp, yp);
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

// Sparse line l = l00 + l01 v + l11 v w (tower slots c0.c0, c0.c1, c1.c1).
struct line {
  fp2 a0, a1, a4;
};

// Product of two sparse lines (6 Fp2 mul); c1.c0 of the result is zero:
//   c0 = (a0 b0 + xi a4 b4, a0 b1 + a1 b0, a1 b1),  c1 = (0, a0 b4 + a4 b0, a1 b4 + a4 b1)
DI fp12 line_mul_line(const line& a, const line& b) {
  fp2 t00 = fp2_mul(a.a0, b.a0), t11 = fp2_mul(a.a1, b.a1), t44 = fp2_mul(a.a4, b.a4);
  fp2 c01 = fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.a0, a.a1), fp2_add_lazy(b.a0, b.a1)), t00), t11);
  fp2 c11 = fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.a0, a.a4), fp2_add_lazy(b.a0, b.a4)), t00), t44);
  fp2 c12 = fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.a1, a.a4), fp2_add_lazy(b.a1, b.a4)), t11), t44);
  return {{fp2_add(t00, fp2_mul_xi(t44)), c01, t11}, {fp2_zero(), c11, c12}};
}

// a * (b1 v + b2 v^2) (5 Fp2 mul)
DI fp6 fp6_mul_by_12(const fp6& a, const fp2& b1, const fp2& b2) {
  fp2 t1 = fp2_mul(a.c1, b1), t2 = fp2_mul(a.c2, b2);
  fp2 m = fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(b1, b2)), t1), t2);  // a1 b2 + a2 b1
  return {fp2_mul_xi(m), fp2_add(fp2_mul(a.c0, b1), fp2_mul_xi(t2)), fp2_add(fp2_mul(a.c0, b2), t1)};
}

// f * L for L with L.c1.c0 == 0 (the product of two lines): 6 + 5 + 6 Fp2 mul
DI fp12 fp12_mul_by_line_pair(const fp12& f, const fp12& L) {
  fp6 t0 = fp6_mul(f.c0, L.c0);
  fp6 t1 = fp6_mul_by_12(f.c1, L.c1.c1, L.c1.c2);
  fp6 Ls = {L.c0.c0, fp2_add_lazy(L.c0.c1, L.c1.c1), fp2_add_lazy(L.c0.c2, L.c1.c2)};
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add_lazy(f.c0, f.c1), Ls), t0), t1);
  return {fp6_add(t0, fp6_mul_v(t1)), c1};
}

DI line line_one() { return {fp2_one(), fp2_zero(), fp2_zero()}; }

// f = prod_k f_{|x|, Q_k}(P_k), conjugated (x < 0), for exactly two pairs: the two lines of a
// step are multiplied together first and then into f. Inactive pairs (a point at infinity,
// skipped like kilic's Engine) contribute the line 1.
DI fp12 miller_loop_2(const g1a (&P)[2], const g2a (&Q)[2], const bool (&active)[2]) {
  g2proj T[2];
#pragma unroll
  for (int k = 0; k < 2; k++) T[k] = {Q[k].x, Q[k].y, fp2_one()};
  fp12 f = fp12_one();
  bool first = true;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (!first) f = fp12_sqr(f);
    line l[2];
#pragma unroll
    for (int k = 0; k < 2; k++) {
      miller_dbl_step(T[k], l[k].a0, l[k].a1, l[k].a4, P[k].x, P[k].y);
      if (!active[k]) l[k] = line_one();
    }
    // f = 1 at the first step: the line pair is f itself
    f = first ? line_mul_line(l[0], l[1]) : fp12_mul_by_line_pair(f, line_mul_line(l[0], l[1]));
    first = false;
    if ((BLS_X_ABS >> i) & 1ull) {
#pragma unroll
      for (int k = 0; k < 2; k++) {
        miller_add_step(T[k], Q[k], l[k].a0, l[k].a1, l[k].a4, P[k].x, P[k].y);
        if (!active[k]) l[k] = line_one();
      }
      f = fp12_mul_by_line_pair(f, line_mul_line(l[0], l[1]));
    }
  }
  return fp12_conj(f);
}

// ---------------------------------------------------------------- staged Miller loop (device path)
// The loop splits into two passes with a small live state each (k_miller.hip):
//   lines : per pair, T runs through the 63 doublings + 5 additions and every line
//           (3 Fp2) is written to HBM staging -- T (6 Fp) plus one step's temporaries live;
//   f     : f = f^2 * (l_0 l_1) over the 68 steps, the lines re-read from staging -- f plus one
//           line pair live.
// Same lines, same products, same order as miller_loop_2 (tools/opcount checks f is identical).
constexpr int MILLER_STEPS = 68;  // |x| = 0xd201000000010000: 63 doublings, 5 additions

template <typename LoadQ, typename Emit>
DI void miller_lines(const g1a& P, LoadQ load_q, Emit emit) {
  const g2a Q0 = load_q();
  g2proj T = {Q0.x, Q0.y, fp2_one()};
  int step = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    line l;
    miller_dbl_step<false>(T, l.a0, l.a1, l.a4, P.x, P.y);
    emit(step++, l);
    if ((BLS_X_ABS >> i) & 1ull) {
      miller_add_step(T, load_q(), l.a0, l.a1, l.a4, P.x, P.y);
      emit(step++, l);
    }
  }
}

// load(step, k) returns pair k's line of that step (line_one() for a skipped pair)
template <typename LoadLine>
DI fp12 miller_f_from_lines(LoadLine load) {
  fp12 f = fp12_one();
  int step = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    if (i != 62) f = fp12_sqr(f);
    const fp12 L = line_mul_line(load(step, 0), load(step, 1));
    f = step == 0 ? L : fp12_mul_by_line_pair(f, L);
    step++;
    if ((BLS_X_ABS >> i) & 1ull) {
      f = fp12_mul_by_line_pair(f, line_mul_line(load(step, 0), load(step, 1)));
      step++;
    }
  }
  return fp12_conj(f);
}

// single-pair form (test hook): same lines, f multiplied by each sparse line
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

// Final exponentiation f^(3 (p^12 - 1)/r), split into stages so that the device can run each as its
// own kernel with only one or two Fp12 values live (the operands are re-read from HBM staging at
// each use through the `load` callables instead of being held in registers):
//   easy : g = f^((p^6 - 1)(p^2 + 1))
//   hard : 3 (p^4 - p^2 + 1)/r = (x-1)^2 (x+p) (x^2+p^2-1) + 3 with x = -|x|, i.e.
//     a = g^(x-1)           step<0>(g)
//     b = a^(x-1)           step<1>(a)
//     c = b^(x+p)           step<2>(b)
//     t = c^x               step<3>(c)
//     e = t^x c^(p^2) c^-1 g^3   step<4>(t; c, g)
// g^|x| uses Granger-Scott cyclotomic squarings; |x| = 0xd201000000010000 has bits 63,62,60,57,48,16,
// i.e. runs of 1, 2, 3, 9, 32 squarings each followed by a multiplication, then 16 squarings.
DI fp12 fexp_easy(const fp12& f) {
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f));  // f^(p^6 - 1)
  return fp12_mul(fp12_frob2(t), t);             // ^(p^2 + 1)
}

template <typename Load>
DI fp12 fp12_pow_x_abs_reload(Load load) {
  constexpr uint64_t NSQ = 1ull | (2ull << 6) | (3ull << 12) | (9ull << 18) | (32ull << 24) | (16ull << 30);
  fp12 r = load();
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int n = (int)((NSQ >> (6 * s)) & 63u);
#pragma unroll 1
    for (int k = 0; k < n; k++) r = fp12_cyclotomic_sqr(r);
    if (s < 5) r = fp12_mul(r, load());
  }
  return r;
}

template <int MODE, typename LX, typename LC, typename LG>
DI fp12 fexp_step(LX lx, LC lc, LG lg) {
  fp12 r = fp12_conj(fp12_pow_x_abs_reload(lx));  // X^x (inverse = conjugate in the cyclotomic subgroup)
  if (MODE == 0 || MODE == 1) return fp12_mul(r, fp12_conj(lx()));
  if (MODE == 2) return fp12_mul(r, fp12_frob(lx()));
  if (MODE == 3) return r;
  r = fp12_mul(r, fp12_frob2(lc()));
  r = fp12_mul(r, fp12_conj(lc()));
  r = fp12_mul(r, fp12_cyclotomic_sqr(lg()));
  return fp12_mul(r, lg());
}

// whole final exponentiation in registers (host op counter, test hooks)
DI fp12 final_exponentiation(const fp12& f) {
  const fp12 g = fexp_easy(f);
  auto none = [&]() { return g; };
  const fp12 a = fexp_step<0>([&]() { return g; }, none, none);
  const fp12 b = fexp_step<1>([&]() { return a; }, none, none);
  const fp12 c = fexp_step<2>([&]() { return b; }, none, none);
  const fp12 t = fexp_step<3>([&]() { return c; }, none, none);
  return fexp_step<4>([&]() { return t; }, [&]() { return c; }, [&]() { return g; });
}

}  // namespace bls

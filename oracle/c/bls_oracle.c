/*
 * CPU ORACLE (test infrastructure only) -- plain-C restatement of drand's beacon verification
 * (chain.VerifyBeacon -> kyber bls.Verify -> kilic/bls12-381), used as
 *   (1) a second parity checker next to oracle/bls12381.py, pinned by the same reference KAT
 *       (key/curve_test.go:10-30) and golden vectors (tests/test_oracle_c.py), and
 *   (2) bench.py's cpu_baseline ("port"): the reference's Go verifier cannot be built in this image
 *       (no Go toolchain), so this restatement of the algorithm kilic runs is timed
 *       on the host cores instead.
 * ONLY tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * path (drand_amd/) never does.
 *
 * What it restates, following kilic/bls12-381 @6b2c19996391's *algorithms*:
 *   - Fp: 6 x 64-bit Montgomery (CIOS), the representation kilic uses on amd64.
 *   - Fp2/Fp6/Fp12 tower (v^3 = 1 + i, w^2 = v), Frobenius by precomputed gamma constants.
 *   - G2.FromCompressed (a8): ZCash flags, x < p, y = sqrt(x^3 + 4(1+i)) by the p = 3 mod 4
 *     "complex method", lexicographic sign, subgroup check by the naive [r]P == O.
 *   - G1.FromCompressed (a14) for the public key, same checks.
 *   - HashToCurve (a7): RFC 9380 expand_message_xmd(SHA-256), hash_to_field, straight-line
 *     simplified SWU with inversions, 3-isogeny to affine, cofactor clearing by the naive h_eff
 *     scalar multiplication.
 *   - Engine.AddPair/AddPairInv/Check (a9): multi-Miller loop over the non-infinity pairs with
 *     projective doubling/addition lines and sparse line multiplication, one final exponentiation
 *     (easy part, then the hard part (x-1)^2 (x+p) (x^2+p^2-1) + 3 with cyclotomic squaring),
 *     result == 1.
 *   - chain.Message (chain/beacon.go:103-108): sha256(prev || BE64(round)).
 * Reject classes follow include/blsverify.h (BLSV_REJ_*), the same vocabulary as the Python oracle.
 */
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <x86intrin.h>

#include "oracle_consts.h"

typedef unsigned __int128 u128;

/* ================================================================ Fp (Montgomery, R = 2^384) */
typedef struct {
  uint64_t l[6];
} fp;
typedef struct {
  fp c0, c1;
} fp2;
typedef struct {
  fp2 c0, c1, c2;
} fp6;
typedef struct {
  fp6 c0, c1;
} fp12;

static const uint64_t PINV = 0x89f3fffcfffcfffdull; /* -p^-1 mod 2^64 */
static fp FP_ONE, FP_R2, FP_2POW256, FP_HALF;

static inline int fp_geq_p(const uint64_t* t) {
  for (int i = 5; i >= 0; i--) {
    if (t[i] > C_P[i]) return 1;
    if (t[i] < C_P[i]) return 0;
  }
  return 1;
}

static inline void sub_p(uint64_t* t) {
  uint64_t br = 0;
  for (int i = 0; i < 6; i++) {
    u128 d = (u128)t[i] - C_P[i] - br;
    t[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1;
  }
}

static inline __attribute__((always_inline)) fp fp_add(fp a, fp b) { /* a + b < 2p < 2^382: no carry out of the top word */
  uint64_t s[6], d[6];
  unsigned char c = 0, br = 0;
  for (int i = 0; i < 6; i++) c = __builtin_ia32_addcarryx_u64(c, a.l[i], b.l[i], (unsigned long long*)&s[i]);
  for (int i = 0; i < 6; i++) br = __builtin_ia32_sbb_u64(br, s[i], C_P[i], (unsigned long long*)&d[i]);
  fp r;
  const uint64_t keep = (uint64_t)0 - (uint64_t)br; /* borrow: s < p, keep s */
  for (int i = 0; i < 6; i++) r.l[i] = (s[i] & keep) | (d[i] & ~keep);
  return r;
}

static inline __attribute__((always_inline)) fp fp_sub(fp a, fp b) {
  uint64_t d[6], e[6];
  unsigned char br = 0, c = 0;
  for (int i = 0; i < 6; i++) br = __builtin_ia32_sbb_u64(br, a.l[i], b.l[i], (unsigned long long*)&d[i]);
  const uint64_t mask = (uint64_t)0 - (uint64_t)br; /* borrow: add p back */
  for (int i = 0; i < 6; i++) c = __builtin_ia32_addcarryx_u64(c, d[i], C_P[i] & mask, (unsigned long long*)&e[i]);
  fp r;
  memcpy(r.l, e, 48);
  return r;
}

static inline int fp_is_zero(fp a) { return (a.l[0] | a.l[1] | a.l[2] | a.l[3] | a.l[4] | a.l[5]) == 0; }
static inline int fp_eq(fp a, fp b) { return memcmp(a.l, b.l, 48) == 0; }
static inline fp fp_zero(void) {
  fp r;
  memset(&r, 0, sizeof r);
  return r;
}
static inline fp fp_neg(fp a) { return fp_is_zero(a) ? a : fp_sub(fp_zero(), a); }
static inline fp fp_dbl(fp a) { return fp_add(a, a); }

/* CIOS Montgomery multiplication a*b*2^-384 mod p, with the "no carry word" simplification that
   p's top limb (< 2^63 - 1) allows: t never needs a 7th word. */
static inline __attribute__((always_inline)) fp fp_mul(fp a, fp b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 6; i++) {
    u128 A = (u128)a.l[0] * b.l[i] + t[0];
    const uint64_t m = (uint64_t)A * PINV;
    u128 C = (u128)m * C_P[0] + (uint64_t)A;
    for (int j = 1; j < 6; j++) {
      A = (u128)a.l[j] * b.l[i] + t[j] + (uint64_t)(A >> 64);
      C = (u128)m * C_P[j] + (uint64_t)A + (uint64_t)(C >> 64);
      t[j - 1] = (uint64_t)C;
    }
    t[5] = (uint64_t)(C >> 64) + (uint64_t)(A >> 64);
  }
  fp r;
  memcpy(r.l, t, 48);
  if (fp_geq_p(r.l)) sub_p(r.l);
  return r;
}
static inline fp fp_sqr(fp a) { return fp_mul(a, a); }

static fp fp_from_words(const uint64_t* w) { /* raw < p -> Montgomery */
  fp r;
  memcpy(r.l, w, 48);
  return fp_mul(r, FP_R2);
}

static fp fp_to_raw(fp a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}

static fp fp_pow(fp a, const uint64_t* e, int nwords) {
  fp r = FP_ONE;
  for (int w = nwords - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      r = fp_sqr(r);
      if ((e[w] >> b) & 1) r = fp_mul(r, a);
    }
  return r;
}
static fp fp_inv(fp a) { return fp_pow(a, C_P_MINUS_2, 6); }

/* raw value > (p-1)/2 (ZCash "lexicographically largest") */
static int fp_raw_gt_half(fp raw) {
  for (int i = 5; i >= 0; i--) {
    if (raw.l[i] > C_P_MINUS_1_DIV_2[i]) return 1;
    if (raw.l[i] < C_P_MINUS_1_DIV_2[i]) return 0;
  }
  return 0;
}

static fp fp_from_be48(const uint8_t* b) { /* raw big-endian bytes (caller checked < p) */
  uint64_t w[6];
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[(5 - i) * 8 + k];
    w[i] = v;
  }
  return fp_from_words(w);
}

static int be48_lt_p(const uint8_t* b) {
  uint64_t w[6];
  for (int i = 0; i < 6; i++) {
    uint64_t v = 0;
    for (int k = 0; k < 8; k++) v = (v << 8) | b[(5 - i) * 8 + k];
    w[i] = v;
  }
  return !fp_geq_p(w);
}

/* ================================================================ Fp2 = Fp[i]/(i^2 + 1) */
static inline fp2 f2(fp a, fp b) {
  fp2 r = {a, b};
  return r;
}
static inline fp2 fp2_add(fp2 a, fp2 b) { return f2(fp_add(a.c0, b.c0), fp_add(a.c1, b.c1)); }
static inline fp2 fp2_sub(fp2 a, fp2 b) { return f2(fp_sub(a.c0, b.c0), fp_sub(a.c1, b.c1)); }
static inline fp2 fp2_neg(fp2 a) { return f2(fp_neg(a.c0), fp_neg(a.c1)); }
static inline fp2 fp2_dbl(fp2 a) { return fp2_add(a, a); }
static inline fp2 fp2_conj(fp2 a) { return f2(a.c0, fp_neg(a.c1)); }
static inline int fp2_is_zero(fp2 a) { return fp_is_zero(a.c0) && fp_is_zero(a.c1); }
static inline int fp2_eq(fp2 a, fp2 b) { return fp_eq(a.c0, b.c0) && fp_eq(a.c1, b.c1); }
static inline fp2 fp2_zero(void) { return f2(fp_zero(), fp_zero()); }
static inline fp2 fp2_one(void) { return f2(FP_ONE, fp_zero()); }

static fp2 fp2_mul(fp2 a, fp2 b) {
  fp t0 = fp_mul(a.c0, b.c0), t1 = fp_mul(a.c1, b.c1);
  fp t2 = fp_mul(fp_add(a.c0, a.c1), fp_add(b.c0, b.c1));
  return f2(fp_sub(t0, t1), fp_sub(fp_sub(t2, t0), t1));
}
static fp2 fp2_sqr(fp2 a) {
  fp t = fp_mul(a.c0, a.c1);
  return f2(fp_mul(fp_add(a.c0, a.c1), fp_sub(a.c0, a.c1)), fp_dbl(t));
}
static inline fp2 fp2_mul_fp(fp2 a, fp b) { return f2(fp_mul(a.c0, b), fp_mul(a.c1, b)); }
static inline fp2 fp2_mul_xi(fp2 a) { return f2(fp_sub(a.c0, a.c1), fp_add(a.c0, a.c1)); } /* (1+i) a */
static fp2 fp2_inv(fp2 a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  fp ni = fp_inv(n);
  return f2(fp_mul(a.c0, ni), fp_neg(fp_mul(a.c1, ni)));
}
static fp2 fp2_pow(fp2 a, const uint64_t* e, int nwords) {
  fp2 r = fp2_one();
  for (int w = nwords - 1; w >= 0; w--)
    for (int b = 63; b >= 0; b--) {
      r = fp2_sqr(r);
      if ((e[w] >> b) & 1) r = fp2_mul(r, a);
    }
  return r;
}
static fp2 fp2_from_raw(const uint64_t (*c)[6]) { return f2(fp_from_words(c[0]), fp_from_words(c[1])); }

/* square root, p = 3 mod 4 complex method (kilic fp2.sqrt); returns 0 if a is not a square */
static int fp2_sqrt(fp2* out, fp2 a) {
  if (fp2_is_zero(a)) {
    *out = a;
    return 1;
  }
  fp2 a1 = fp2_pow(a, C_P_MINUS_3_DIV_4, 6);
  fp2 alpha = fp2_mul(fp2_sqr(a1), a);
  fp2 x0 = fp2_mul(a1, a);
  fp2 minus_one = f2(fp_neg(FP_ONE), fp_zero());
  fp2 cand;
  if (fp2_eq(alpha, minus_one)) {
    cand = f2(fp_neg(x0.c1), x0.c0); /* i * x0 */
  } else {
    fp2 b = fp2_pow(fp2_add(fp2_one(), alpha), C_P_MINUS_1_DIV_2, 6);
    cand = fp2_mul(b, x0);
  }
  if (!fp2_eq(fp2_sqr(cand), a)) return 0;
  *out = cand;
  return 1;
}

/* a is a square in Fp2 iff its norm is a square in Fp */
static int fp2_is_square(fp2 a) {
  fp n = fp_add(fp_sqr(a.c0), fp_sqr(a.c1));
  if (fp_is_zero(n)) return 1;
  return fp_eq(fp_pow(n, C_P_MINUS_1_DIV_2, 6), FP_ONE);
}

static int fp2_sgn0(fp2 a) { /* RFC 9380 sgn0 on raw values */
  fp r0 = fp_to_raw(a.c0), r1 = fp_to_raw(a.c1);
  int s0 = r0.l[0] & 1, z0 = fp_is_zero(r0), s1 = r1.l[0] & 1;
  return s0 | (z0 & s1);
}

/* ================================================================ Fp6, Fp12 */
static fp6 f6(fp2 a, fp2 b, fp2 c) {
  fp6 r = {a, b, c};
  return r;
}
static fp6 fp6_add(fp6 a, fp6 b) { return f6(fp2_add(a.c0, b.c0), fp2_add(a.c1, b.c1), fp2_add(a.c2, b.c2)); }
static fp6 fp6_sub(fp6 a, fp6 b) { return f6(fp2_sub(a.c0, b.c0), fp2_sub(a.c1, b.c1), fp2_sub(a.c2, b.c2)); }
static fp6 fp6_neg(fp6 a) { return f6(fp2_neg(a.c0), fp2_neg(a.c1), fp2_neg(a.c2)); }
static fp6 fp6_mul_v(fp6 a) { return f6(fp2_mul_xi(a.c2), a.c0, a.c1); }
static fp6 fp6_zero(void) { return f6(fp2_zero(), fp2_zero(), fp2_zero()); }

static fp6 fp6_mul(fp6 a, fp6 b) {
  fp2 t0 = fp2_mul(a.c0, b.c0), t1 = fp2_mul(a.c1, b.c1), t2 = fp2_mul(a.c2, b.c2);
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c1, a.c2), fp2_add(b.c1, b.c2)), t1), t2)), t0);
  fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c1), fp2_add(b.c0, b.c1)), t0), t1), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add(a.c0, a.c2), fp2_add(b.c0, b.c2)), t0), t2), t1);
  return f6(c0, c1, c2);
}

static fp6 fp6_inv(fp6 a) {
  fp2 t0 = fp2_sub(fp2_sqr(a.c0), fp2_mul_xi(fp2_mul(a.c1, a.c2)));
  fp2 t1 = fp2_sub(fp2_mul_xi(fp2_sqr(a.c2)), fp2_mul(a.c0, a.c1));
  fp2 t2 = fp2_sub(fp2_sqr(a.c1), fp2_mul(a.c0, a.c2));
  fp2 d = fp2_add(fp2_mul(a.c0, t0), fp2_mul_xi(fp2_add(fp2_mul(a.c2, t1), fp2_mul(a.c1, t2))));
  fp2 di = fp2_inv(d);
  return f6(fp2_mul(t0, di), fp2_mul(t1, di), fp2_mul(t2, di));
}

static fp12 f12(fp6 a, fp6 b) {
  fp12 r = {a, b};
  return r;
}
static fp12 fp12_one(void) { return f12(f6(fp2_one(), fp2_zero(), fp2_zero()), fp6_zero()); }
static fp12 fp12_conj(fp12 a) { return f12(a.c0, fp6_neg(a.c1)); }
static int fp12_is_one(fp12 a) {
  fp12 o = fp12_one();
  return fp2_eq(a.c0.c0, o.c0.c0) && fp2_is_zero(a.c0.c1) && fp2_is_zero(a.c0.c2) && fp2_is_zero(a.c1.c0) &&
         fp2_is_zero(a.c1.c1) && fp2_is_zero(a.c1.c2);
}

static fp12 fp12_mul(fp12 a, fp12 b) {
  fp6 t0 = fp6_mul(a.c0, b.c0), t1 = fp6_mul(a.c1, b.c1);
  fp6 c1 = fp6_sub(fp6_sub(fp6_mul(fp6_add(a.c0, a.c1), fp6_add(b.c0, b.c1)), t0), t1);
  return f12(fp6_add(t0, fp6_mul_v(t1)), c1);
}

static fp12 fp12_sqr(fp12 a) {
  fp6 ab = fp6_mul(a.c0, a.c1);
  fp6 t = fp6_mul(fp6_add(a.c0, a.c1), fp6_add(a.c0, fp6_mul_v(a.c1)));
  return f12(fp6_sub(fp6_sub(t, ab), fp6_mul_v(ab)), fp6_add(ab, ab));
}

static fp12 fp12_inv(fp12 a) {
  fp6 d = fp6_sub(fp6_mul(a.c0, a.c0), fp6_mul_v(fp6_mul(a.c1, a.c1)));
  fp6 di = fp6_inv(d);
  return f12(fp6_mul(a.c0, di), fp6_neg(fp6_mul(a.c1, di)));
}

/* sparse line l = l0 + l1 v + l4 v w (tower slots c0.c0, c0.c1, c1.c1) */
static fp12 fp12_mul_line(fp12 f, fp2 l0, fp2 l1, fp2 l4) {
  /* schoolbook on the sparse Fp6 halves: (a0 + a1 w)(b0 + b1 w) = a0 b0 + v a1 b1 + (a0 b1 + a1 b0) w */
  fp6 a0b0, a1b1, a0b1, a1b0;
  {
    fp6 a = f.c0; /* a * (l0 + l1 v) */
    fp2 t0 = fp2_mul(a.c0, l0), t1 = fp2_mul(a.c1, l1);
    a0b0 = f6(fp2_add(fp2_mul_xi(fp2_mul(a.c2, l1)), t0), fp2_add(fp2_mul(a.c0, l1), fp2_mul(a.c1, l0)),
              fp2_add(fp2_mul(a.c2, l0), t1));
  }
  {
    fp6 a = f.c1;
    fp2 t0 = fp2_mul(a.c0, l0), t1 = fp2_mul(a.c1, l1);
    a1b0 = f6(fp2_add(fp2_mul_xi(fp2_mul(a.c2, l1)), t0), fp2_add(fp2_mul(a.c0, l1), fp2_mul(a.c1, l0)),
              fp2_add(fp2_mul(a.c2, l0), t1));
  }
  /* x * (l4 v) = xi x2 l4 + x0 l4 v + x1 l4 v^2 */
  a0b1 = f6(fp2_mul_xi(fp2_mul(f.c0.c2, l4)), fp2_mul(f.c0.c0, l4), fp2_mul(f.c0.c1, l4));
  a1b1 = f6(fp2_mul_xi(fp2_mul(f.c1.c2, l4)), fp2_mul(f.c1.c0, l4), fp2_mul(f.c1.c1, l4));
  return f12(fp6_add(a0b0, fp6_mul_v(a1b1)), fp6_add(a0b1, a1b0));
}

static fp2 GAMMA1[6], GAMMA2[6], GAMMA3[6];

/* x^(p^n): coefficient of w^k (slot order c0.c0 w^0, c1.c0 w^1, c0.c1 w^2, c1.c1 w^3, c0.c2 w^4,
   c1.c2 w^5) is conjugated n times and multiplied by gamma_n[k] */
static fp12 fp12_frob(fp12 a, int n) {
  const fp2* g = n == 1 ? GAMMA1 : n == 2 ? GAMMA2 : GAMMA3;
  fp2* slot[6] = {&a.c0.c0, &a.c1.c0, &a.c0.c1, &a.c1.c1, &a.c0.c2, &a.c1.c2};
  for (int k = 0; k < 6; k++) {
    fp2 c = *slot[k];
    if (n & 1) c = fp2_conj(c);
    *slot[k] = fp2_mul(c, g[k]);
  }
  return a;
}

/* Granger-Scott squaring in the cyclotomic subgroup */
static void fp4_sqr(fp2* c0, fp2* c1, fp2 a, fp2 b) {
  fp2 t0 = fp2_sqr(a), t1 = fp2_sqr(b);
  *c0 = fp2_add(fp2_mul_xi(t1), t0);
  *c1 = fp2_sub(fp2_sub(fp2_sqr(fp2_add(a, b)), t0), t1);
}
static fp12 fp12_cyc_sqr(fp12 f) {
  fp2 z0 = f.c0.c0, z4 = f.c0.c1, z3 = f.c0.c2, z2 = f.c1.c0, z1 = f.c1.c1, z5 = f.c1.c2;
  fp2 t0, t1, t2, t3;
  fp4_sqr(&t0, &t1, z0, z1);
  z0 = fp2_add(fp2_dbl(fp2_sub(t0, z0)), t0);
  z1 = fp2_add(fp2_dbl(fp2_add(t1, z1)), t1);
  fp4_sqr(&t0, &t1, z2, z3);
  fp4_sqr(&t2, &t3, z4, z5);
  z4 = fp2_add(fp2_dbl(fp2_sub(t0, z4)), t0);
  z5 = fp2_add(fp2_dbl(fp2_add(t1, z5)), t1);
  t0 = fp2_mul_xi(t3);
  z2 = fp2_add(fp2_dbl(fp2_add(t0, z2)), t0);
  z3 = fp2_add(fp2_dbl(fp2_sub(t2, z3)), t2);
  return f12(f6(z0, z4, z3), f6(z2, z1, z5));
}

/* a^x for x = -|x| in the cyclotomic subgroup (inverse = conjugate) */
static fp12 fp12_exp_x(fp12 a) {
  fp12 r = a;
  for (int b = 62; b >= 0; b--) {
    r = fp12_cyc_sqr(r);
    if ((C_X_ABS >> b) & 1) r = fp12_mul(r, a);
  }
  return fp12_conj(r);
}

/* f^(3 (p^12 - 1)/r); == 1 iff f^((p^12-1)/r) == 1 (gcd(3, r) = 1) */
static fp12 final_exp(fp12 f) {
  fp12 t = fp12_mul(fp12_conj(f), fp12_inv(f)); /* ^(p^6 - 1) */
  fp12 g = fp12_mul(fp12_frob(t, 2), t);         /* ^(p^2 + 1) */
  fp12 a = fp12_mul(fp12_exp_x(g), fp12_conj(g)); /* g^(x-1) */
  fp12 b = fp12_mul(fp12_exp_x(a), fp12_conj(a)); /* ^(x-1) */
  fp12 c = fp12_mul(fp12_exp_x(b), fp12_frob(b, 1)); /* ^(x+p) */
  fp12 e = fp12_exp_x(fp12_exp_x(c));               /* c^(x^2) */
  e = fp12_mul(e, fp12_frob(c, 2));
  e = fp12_mul(e, fp12_conj(c));
  e = fp12_mul(e, fp12_mul(fp12_cyc_sqr(g), g)); /* * g^3 */
  return e;
}

/* ================================================================ curves (Jacobian) */
typedef struct {
  fp x, y, z;
} g1j;
typedef struct {
  fp2 x, y, z;
} g2j;
typedef struct {
  fp x, y;
  int inf;
} g1a;
typedef struct {
  fp2 x, y;
  int inf;
} g2a;

#define DEF_JAC(T, F, PFX)                                                                     \
  static T PFX##_dbl(T p) {                                                                    \
    F A = PFX##_f_sqr(p.x), B = PFX##_f_sqr(p.y), C = PFX##_f_sqr(B);                          \
    F D = PFX##_f_dbl(PFX##_f_sub(PFX##_f_sub(PFX##_f_sqr(PFX##_f_add(p.x, B)), A), C));        \
    F E = PFX##_f_add(PFX##_f_dbl(A), A), Fv = PFX##_f_sqr(E);                                  \
    T r;                                                                                       \
    r.x = PFX##_f_sub(Fv, PFX##_f_dbl(D));                                                     \
    F C8 = PFX##_f_dbl(PFX##_f_dbl(PFX##_f_dbl(C)));                                           \
    r.y = PFX##_f_sub(PFX##_f_mul(E, PFX##_f_sub(D, r.x)), C8);                                 \
    r.z = PFX##_f_dbl(PFX##_f_mul(p.y, p.z));                                                  \
    return r;                                                                                  \
  }                                                                                            \
  static T PFX##_add(T p, T q) {                                                               \
    if (PFX##_f_is_zero(p.z)) return q;                                                        \
    if (PFX##_f_is_zero(q.z)) return p;                                                        \
    F Z1Z1 = PFX##_f_sqr(p.z), Z2Z2 = PFX##_f_sqr(q.z);                                         \
    F U1 = PFX##_f_mul(p.x, Z2Z2), U2 = PFX##_f_mul(q.x, Z1Z1);                                 \
    F S1 = PFX##_f_mul(PFX##_f_mul(p.y, q.z), Z2Z2), S2 = PFX##_f_mul(PFX##_f_mul(q.y, p.z), Z1Z1); \
    F H = PFX##_f_sub(U2, U1), rr = PFX##_f_dbl(PFX##_f_sub(S2, S1));                            \
    if (PFX##_f_is_zero(H)) {                                                                  \
      if (PFX##_f_is_zero(rr)) return PFX##_dbl(p);                                            \
      T o = p;                                                                                 \
      o.z = PFX##_f_zero();                                                                    \
      return o;                                                                                \
    }                                                                                          \
    F I = PFX##_f_sqr(PFX##_f_dbl(H)), J = PFX##_f_mul(H, I), V = PFX##_f_mul(U1, I);          \
    T r;                                                                                       \
    r.x = PFX##_f_sub(PFX##_f_sub(PFX##_f_sqr(rr), J), PFX##_f_dbl(V));                         \
    r.y = PFX##_f_sub(PFX##_f_mul(rr, PFX##_f_sub(V, r.x)), PFX##_f_dbl(PFX##_f_mul(S1, J)));   \
    r.z = PFX##_f_mul(PFX##_f_sub(PFX##_f_sub(PFX##_f_sqr(PFX##_f_add(p.z, q.z)), Z1Z1), Z2Z2), H); \
    return r;                                                                                  \
  }                                                                                            \
  static T PFX##_mul_words(T p, const uint64_t* k, int nwords) {                               \
    T acc = p;                                                                                 \
    acc.z = PFX##_f_zero();                                                                    \
    for (int w = nwords - 1; w >= 0; w--)                                                      \
      for (int b = 63; b >= 0; b--) {                                                          \
        acc = PFX##_dbl(acc);                                                                  \
        if ((k[w] >> b) & 1) acc = PFX##_add(acc, p);                                          \
      }                                                                                        \
    return acc;                                                                                \
  }

#define g1_f_sqr fp_sqr
#define g1_f_mul fp_mul
#define g1_f_add fp_add
#define g1_f_sub fp_sub
#define g1_f_dbl fp_dbl
#define g1_f_is_zero fp_is_zero
#define g1_f_zero fp_zero
#define g2_f_sqr fp2_sqr
#define g2_f_mul fp2_mul
#define g2_f_add fp2_add
#define g2_f_sub fp2_sub
#define g2_f_dbl fp2_dbl
#define g2_f_is_zero fp2_is_zero
#define g2_f_zero fp2_zero
DEF_JAC(g1j, fp, g1)
DEF_JAC(g2j, fp2, g2)

static g2a g2_to_aff(g2j p) {
  g2a r;
  r.inf = fp2_is_zero(p.z);
  if (r.inf) return r;
  fp2 zi = fp2_inv(p.z), zi2 = fp2_sqr(zi);
  r.x = fp2_mul(p.x, zi2);
  r.y = fp2_mul(p.y, fp2_mul(zi2, zi));
  return r;
}

static g2j g2_from_aff(g2a a) {
  g2j r = {a.x, a.y, a.inf ? fp2_zero() : fp2_one()};
  return r;
}

/* ================================================================ encodings */
enum { REJ_OK = 0, REJ_LENGTH = 1, REJ_FLAG = 2, REJ_INF_NONZERO = 3, REJ_X_GE_P = 4, REJ_NOT_ON_CURVE = 5,
       REJ_NOT_IN_SUBGROUP = 6, REJ_PAIRING = 7 };

static fp2 B2; /* 4 (1 + i) */

static int g2_decompress(const uint8_t* in, size_t len, g2a* out) {
  if (len != 96) return REJ_LENGTH;
  uint8_t b[96];
  memcpy(b, in, 96);
  if (!(b[0] & 0x80)) return REJ_FLAG;
  if (b[0] & 0x40) {
    if (b[0] != 0xc0) return REJ_INF_NONZERO;
    for (int i = 1; i < 96; i++)
      if (b[i]) return REJ_INF_NONZERO;
    out->inf = 1;
    return REJ_OK;
  }
  const int sign = (b[0] & 0x20) != 0;
  b[0] &= 0x1f;
  if (!be48_lt_p(b) || !be48_lt_p(b + 48)) return REJ_X_GE_P;
  fp2 x = f2(fp_from_be48(b + 48), fp_from_be48(b));
  fp2 y;
  if (!fp2_sqrt(&y, fp2_add(fp2_mul(fp2_sqr(x), x), B2))) return REJ_NOT_ON_CURVE;
  fp r1 = fp_to_raw(y.c1);
  int largest = !fp_is_zero(r1) ? fp_raw_gt_half(r1) : fp_raw_gt_half(fp_to_raw(y.c0));
  if (largest != sign) y = fp2_neg(y);
  out->x = x;
  out->y = y;
  out->inf = 0;
  g2j rp = g2_mul_words(g2_from_aff(*out), C_R_ORDER, 4); /* kilic InCorrectSubgroup: [r]P == O */
  if (!fp2_is_zero(rp.z)) return REJ_NOT_IN_SUBGROUP;
  return REJ_OK;
}

static int g1_decompress(const uint8_t* in, g1a* out) {
  uint8_t b[48];
  memcpy(b, in, 48);
  if (!(b[0] & 0x80)) return REJ_FLAG;
  if (b[0] & 0x40) {
    if (b[0] != 0xc0) return REJ_INF_NONZERO;
    for (int i = 1; i < 48; i++)
      if (b[i]) return REJ_INF_NONZERO;
    out->inf = 1;
    return REJ_OK;
  }
  const int sign = (b[0] & 0x20) != 0;
  b[0] &= 0x1f;
  if (!be48_lt_p(b)) return REJ_X_GE_P;
  fp x = fp_from_be48(b);
  fp four = fp_add(fp_add(FP_ONE, FP_ONE), fp_add(FP_ONE, FP_ONE));
  fp rhs = fp_add(fp_mul(fp_sqr(x), x), four);
  fp y = fp_pow(rhs, C_P_PLUS_1_DIV_4, 6);
  if (!fp_eq(fp_sqr(y), rhs)) return REJ_NOT_ON_CURVE;
  if (fp_raw_gt_half(fp_to_raw(y)) != sign) y = fp_neg(y);
  out->x = x;
  out->y = y;
  out->inf = 0;
  g1j pj = {x, y, FP_ONE};
  g1j rp = g1_mul_words(pj, C_R_ORDER, 4);
  if (!fp_is_zero(rp.z)) return REJ_NOT_IN_SUBGROUP;
  return REJ_OK;
}

static void fp_to_be48(uint8_t* out, fp a) {
  fp r = fp_to_raw(a);
  for (int i = 0; i < 6; i++)
    for (int k = 0; k < 8; k++) out[(5 - i) * 8 + k] = (uint8_t)(r.l[i] >> (56 - 8 * k));
}

static void g2_compress(uint8_t* out, g2j p) {
  g2a a = g2_to_aff(p);
  if (a.inf) {
    memset(out, 0, 96);
    out[0] = 0xc0;
    return;
  }
  fp_to_be48(out, a.x.c1);
  fp_to_be48(out + 48, a.x.c0);
  out[0] |= 0x80;
  fp r1 = fp_to_raw(a.y.c1);
  int largest = !fp_is_zero(r1) ? fp_raw_gt_half(r1) : fp_raw_gt_half(fp_to_raw(a.y.c0));
  if (largest) out[0] |= 0x20;
}

/* ================================================================ SHA-256 */
static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

#define ROR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

static void sha256_block(uint32_t* st, const uint8_t* blk) {
  uint32_t w[64];
  for (int i = 0; i < 16; i++)
    w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
  for (int i = 16; i < 64; i++) {
    uint32_t s0 = ROR(w[i - 15], 7) ^ ROR(w[i - 15], 18) ^ (w[i - 15] >> 3);
    uint32_t s1 = ROR(w[i - 2], 17) ^ ROR(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4], f = st[5], g = st[6], h = st[7];
  for (int i = 0; i < 64; i++) {
    uint32_t t1 = h + (ROR(e, 6) ^ ROR(e, 11) ^ ROR(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    uint32_t t2 = (ROR(a, 2) ^ ROR(a, 13) ^ ROR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  st[0] += a, st[1] += b, st[2] += c, st[3] += d, st[4] += e, st[5] += f, st[6] += g, st[7] += h;
}

/* SHA-256 of the concatenation of up to 4 byte strings */
static void sha256_v(uint8_t out[32], const uint8_t* const* parts, const size_t* lens, int np) {
  uint32_t st[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a, 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  uint8_t blk[64];
  size_t fill = 0, total = 0;
  for (int p = 0; p < np; p++)
    for (size_t i = 0; i < lens[p]; i++) {
      blk[fill++] = parts[p][i];
      total++;
      if (fill == 64) sha256_block(st, blk), fill = 0;
    }
  blk[fill++] = 0x80;
  if (fill > 56) {
    memset(blk + fill, 0, 64 - fill);
    sha256_block(st, blk);
    fill = 0;
  }
  memset(blk + fill, 0, 56 - fill);
  uint64_t bits = (uint64_t)total * 8;
  for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)(bits >> (56 - 8 * i));
  sha256_block(st, blk);
  for (int i = 0; i < 8; i++)
    for (int k = 0; k < 4; k++) out[4 * i + k] = (uint8_t)(st[i] >> (24 - 8 * k));
}

/* ================================================================ hash to G2 (RFC 9380) */
static const uint8_t DST[] = "BLS_SIG_BLS12381G2_XMD:SHA-256_SSWU_RO_NUL_";
#define DST_LEN 43

static void expand_message_xmd(uint8_t out[256], const uint8_t* msg, size_t len) {
  static const uint8_t zpad[64] = {0};
  const uint8_t lib[3] = {1, 0, 0}; /* I2OSP(256, 2) || I2OSP(0, 1) */
  const uint8_t dlen = DST_LEN;
  uint8_t b0[32], x[32];
  const uint8_t* p0[5] = {zpad, msg, lib, DST, &dlen};
  const size_t l0[5] = {64, len, 3, DST_LEN, 1};
  sha256_v(b0, p0, l0, 5);
  for (int i = 1; i <= 8; i++) { /* b_i = H((b0 ^ b_{i-1}) || i || DST'), b_0 ^ "b_0" = b0 for i = 1 */
    for (int k = 0; k < 32; k++) x[k] = i == 1 ? b0[k] : (uint8_t)(b0[k] ^ out[32 * (i - 2) + k]);
    const uint8_t idx = (uint8_t)i;
    const uint8_t* p[4] = {x, &idx, DST, &dlen};
    const size_t l[4] = {32, 1, DST_LEN, 1};
    sha256_v(out + 32 * (i - 1), p, l, 4);
  }
}

static fp fp_from_be64(const uint8_t* b) { /* 512-bit big-endian -> Fp (Montgomery) */
  uint64_t hi[6] = {0}, lo[6] = {0};
  for (int i = 0; i < 4; i++) {
    uint64_t vh = 0, vl = 0;
    for (int k = 0; k < 8; k++) {
      vh = (vh << 8) | b[(3 - i) * 8 + k];
      vl = (vl << 8) | b[32 + (3 - i) * 8 + k];
    }
    hi[i] = vh;
    lo[i] = vl;
  }
  return fp_add(fp_mul(fp_from_words(hi), FP_2POW256), fp_from_words(lo));
}

static fp2 SSWU_A, SSWU_B, SSWU_Z, SSWU_MB_OVER_A, SSWU_B_OVER_ZA;
static fp2 ISO_XNUM[4], ISO_XDEN[3], ISO_YNUM[4], ISO_YDEN[4];

static g2a map_to_curve_sswu(fp2 u) {
  fp2 zu2 = fp2_mul(SSWU_Z, fp2_sqr(u));
  fp2 den = fp2_add(fp2_sqr(zu2), zu2);
  fp2 tv1 = fp2_is_zero(den) ? fp2_zero() : fp2_inv(den);
  fp2 x1 = fp2_is_zero(tv1) ? SSWU_B_OVER_ZA : fp2_mul(SSWU_MB_OVER_A, fp2_add(fp2_one(), tv1));
  fp2 gx1 = fp2_add(fp2_add(fp2_mul(fp2_sqr(x1), x1), fp2_mul(SSWU_A, x1)), SSWU_B);
  fp2 x2 = fp2_mul(zu2, x1);
  fp2 gx2 = fp2_add(fp2_add(fp2_mul(fp2_sqr(x2), x2), fp2_mul(SSWU_A, x2)), SSWU_B);
  g2a r;
  r.inf = 0;
  if (fp2_is_square(gx1)) {
    r.x = x1;
    fp2_sqrt(&r.y, gx1);
  } else {
    r.x = x2;
    fp2_sqrt(&r.y, gx2);
  }
  if (fp2_sgn0(u) != fp2_sgn0(r.y)) r.y = fp2_neg(r.y);
  return r;
}

static fp2 poly(const fp2* c, int n, fp2 x) {
  fp2 acc = fp2_zero();
  for (int i = n - 1; i >= 0; i--) acc = fp2_add(fp2_mul(acc, x), c[i]);
  return acc;
}

static g2a iso_map(g2a p) {
  fp2 xn = poly(ISO_XNUM, 4, p.x), xd = poly(ISO_XDEN, 3, p.x);
  fp2 yn = poly(ISO_YNUM, 4, p.x), yd = poly(ISO_YDEN, 4, p.x);
  g2a r;
  if (fp2_is_zero(xd) || fp2_is_zero(yd)) {
    r.inf = 1;
    return r;
  }
  r.inf = 0;
  r.x = fp2_mul(xn, fp2_inv(xd));
  r.y = fp2_mul(p.y, fp2_mul(yn, fp2_inv(yd)));
  return r;
}

static g2j hash_to_g2(const uint8_t* msg, size_t len) {
  uint8_t u[256];
  expand_message_xmd(u, msg, len);
  fp2 u0 = f2(fp_from_be64(u), fp_from_be64(u + 64));
  fp2 u1 = f2(fp_from_be64(u + 128), fp_from_be64(u + 192));
  g2j q = g2_add(g2_from_aff(iso_map(map_to_curve_sswu(u0))), g2_from_aff(iso_map(map_to_curve_sswu(u1))));
  return g2_mul_words(q, C_H_EFF, 10); /* kilic ClearCofactor: [h_eff] P */
}

/* ================================================================ pairing check */
typedef struct {
  fp2 x, y, z;
} g2proj;

static fp2 fp2_mul3(fp2 a) { return fp2_add(fp2_dbl(a), a); }
static fp2 fp2_half(fp2 a) { return fp2_mul_fp(a, FP_HALF); } /* FP_HALF = 1/2 */

/* doubling step on T (homogeneous projective, twist b' = 4(1+i)), line at P = (xp, yp) */
static void dbl_step(g2proj* t, fp2* l0, fp2* l1, fp2* l4, fp xp, fp yp) {
  fp2 A = fp2_half(fp2_mul(t->x, t->y));
  fp2 B = fp2_sqr(t->y), C = fp2_sqr(t->z);
  fp2 E = fp2_mul3(fp2_mul(C, B2)); /* 3 b' Z^2 */
  fp2 F = fp2_mul3(E);
  fp2 G = fp2_half(fp2_add(B, F));
  fp2 H = fp2_sub(fp2_sqr(fp2_add(t->y, t->z)), fp2_add(B, C));
  fp2 X2 = fp2_sqr(t->x);
  *l0 = fp2_sub(E, B);
  *l1 = fp2_mul_fp(fp2_mul3(X2), xp);
  *l4 = fp2_neg(fp2_mul_fp(H, yp));
  t->x = fp2_mul(A, fp2_sub(B, F));
  t->y = fp2_sub(fp2_sqr(G), fp2_mul3(fp2_sqr(E)));
  t->z = fp2_mul(B, H);
}

static void add_step(g2proj* t, g2a q, fp2* l0, fp2* l1, fp2* l4, fp xp, fp yp) {
  fp2 theta = fp2_sub(t->y, fp2_mul(q.y, t->z));
  fp2 lam = fp2_sub(t->x, fp2_mul(q.x, t->z));
  *l0 = fp2_sub(fp2_mul(theta, q.x), fp2_mul(lam, q.y));
  *l1 = fp2_neg(fp2_mul_fp(theta, xp));
  *l4 = fp2_mul_fp(lam, yp);
  fp2 C = fp2_sqr(theta), D = fp2_sqr(lam), E = fp2_mul(D, lam);
  fp2 F = fp2_mul(t->z, C), G = fp2_mul(t->x, D);
  fp2 H = fp2_sub(fp2_add(E, F), fp2_dbl(G));
  t->x = fp2_mul(lam, H);
  t->y = fp2_sub(fp2_mul(theta, fp2_sub(G, H)), fp2_mul(t->y, E));
  t->z = fp2_mul(t->z, E);
}

/* prod_k e(P_k, Q_k) == 1 over the pairs with neither point at infinity (kilic Engine.Check) */
static int pairing_check(const g1a* P, const g2a* Q, int n) {
  g2proj T[2];
  int act[2];
  int any = 0;
  for (int k = 0; k < n; k++) {
    act[k] = !P[k].inf && !Q[k].inf;
    any |= act[k];
    if (act[k]) T[k].x = Q[k].x, T[k].y = Q[k].y, T[k].z = fp2_one();
  }
  if (!any) return 1; /* empty product */
  fp12 f = fp12_one();
  for (int b = 62; b >= 0; b--) {
    if (b != 62) f = fp12_sqr(f);
    for (int k = 0; k < n; k++) {
      if (!act[k]) continue;
      fp2 l0, l1, l4;
      dbl_step(&T[k], &l0, &l1, &l4, P[k].x, P[k].y);
      f = fp12_mul_line(f, l0, l1, l4);
    }
    if ((C_X_ABS >> b) & 1) {
      for (int k = 0; k < n; k++) {
        if (!act[k]) continue;
        fp2 l0, l1, l4;
        add_step(&T[k], Q[k], &l0, &l1, &l4, P[k].x, P[k].y);
        f = fp12_mul_line(f, l0, l1, l4);
      }
    }
  }
  return fp12_is_one(final_exp(fp12_conj(f)));
}

/* ================================================================ API */
static g1a NEG_G1;
static int g_init = 0;

int bo_init(void) {
  if (g_init) return 0;
  /* R2 = 2^768 mod p by doubling 1 (raw arithmetic: fp_add is mod-p addition on any representative) */
  fp r = fp_zero();
  r.l[0] = 1;
  for (int i = 0; i < 768; i++) r = fp_add(r, r);
  FP_R2 = r;
  fp one = fp_zero();
  one.l[0] = 1;
  FP_ONE = fp_mul(one, FP_R2);
  uint64_t w256[6] = {0, 0, 0, 0, 1, 0};
  FP_2POW256 = fp_from_words(w256);
  FP_HALF = fp_inv(fp_add(FP_ONE, FP_ONE));
  B2 = f2(fp_add(fp_add(FP_ONE, FP_ONE), fp_add(FP_ONE, FP_ONE)), fp_add(fp_add(FP_ONE, FP_ONE), fp_add(FP_ONE, FP_ONE)));
  SSWU_A = fp2_from_raw(C_SSWU_A);
  SSWU_B = fp2_from_raw(C_SSWU_B);
  SSWU_Z = fp2_from_raw(C_SSWU_Z);
  SSWU_MB_OVER_A = fp2_mul(fp2_neg(SSWU_B), fp2_inv(SSWU_A));
  SSWU_B_OVER_ZA = fp2_mul(SSWU_B, fp2_inv(fp2_mul(SSWU_Z, SSWU_A)));
  for (int i = 0; i < 4; i++) ISO_XNUM[i] = fp2_from_raw(C_ISO_XNUM[i]);
  for (int i = 0; i < 3; i++) ISO_XDEN[i] = fp2_from_raw(C_ISO_XDEN[i]);
  for (int i = 0; i < 4; i++) ISO_YNUM[i] = fp2_from_raw(C_ISO_YNUM[i]);
  for (int i = 0; i < 4; i++) ISO_YDEN[i] = fp2_from_raw(C_ISO_YDEN[i]);
  for (int k = 0; k < 6; k++) {
    GAMMA1[k] = fp2_from_raw(C_GAMMA1[k]);
    GAMMA2[k] = fp2_from_raw(C_GAMMA2[k]);
    GAMMA3[k] = fp2_from_raw(C_GAMMA3[k]);
  }
  NEG_G1.x = fp_from_words(C_G1_X);
  NEG_G1.y = fp_neg(fp_from_words(C_G1_Y));
  NEG_G1.inf = 0;
  g_init = 1;
  return 0;
}

/* kyber bls.Verify(pk, msg, sig) -> reject class (0 = accept); -1 if pk does not decode */
static int verify_decoded(const g1a* pk, const uint8_t* msg, size_t len, const uint8_t* sig, size_t sig_len) {
  g2j h = hash_to_g2(msg, len);
  g2a s;
  int c = g2_decompress(sig, sig_len, &s);
  if (c != REJ_OK) return c;
  g1a Ps[2] = {*pk, NEG_G1};
  g2a Qs[2] = {g2_to_aff(h), s};
  return pairing_check(Ps, Qs, 2) ? REJ_OK : REJ_PAIRING;
}

int bo_verify(const uint8_t* pk48, const uint8_t* msg, size_t len, const uint8_t* sig, size_t sig_len) {
  bo_init();
  g1a pk;
  if (g1_decompress(pk48, &pk) != REJ_OK) return -1;
  return verify_decoded(&pk, msg, len, sig, sig_len);
}

/* chain.VerifyBeacon over a chained range (chain/beacon.go:87-92): beacon i has round
   first_round + i, PreviousSig = prev0 (i == 0) or sigs96[i-1]. cls[i] = reject class. Returns the
   number of accepted beacons, -1 if pk does not decode. */
long bo_verify_chained(const uint8_t* pk48, uint64_t first_round, const uint8_t* prev0, size_t prev0_len,
                       const uint8_t* sigs96, size_t n, uint8_t* cls) {
  bo_init();
  g1a pk;
  if (g1_decompress(pk48, &pk) != REJ_OK) return -1;
  long ok = 0;
  for (size_t i = 0; i < n; i++) {
    uint8_t rb[8], msg[32];
    const uint64_t rnd = first_round + i;
    for (int k = 0; k < 8; k++) rb[k] = (uint8_t)(rnd >> (56 - 8 * k));
    const uint8_t* parts[2] = {i == 0 ? prev0 : sigs96 + (i - 1) * 96, rb};
    size_t lens[2] = {i == 0 ? prev0_len : 96, 8};
    sha256_v(msg, parts, lens, 2);
    int c = verify_decoded(&pk, msg, 32, sigs96 + i * 96, 96);
    if (cls) cls[i] = (uint8_t)c;
    ok += c == REJ_OK;
  }
  return ok;
}

/* KyberG2.Hash(msg), compressed (test hook) */
int bo_hash_to_g2(const uint8_t* msg, size_t len, uint8_t out96[96]) {
  bo_init();
  g2_compress(out96, hash_to_g2(msg, len));
  return 0;
}

/* kyber bls.Sign: compress(sk * H(msg)); sk as 32 big-endian bytes (< r) (test hook) */
int bo_sign(const uint8_t* sk32, const uint8_t* msg, size_t len, uint8_t out96[96]) {
  bo_init();
  uint64_t k[4];
  for (int i = 0; i < 4; i++) {
    uint64_t v = 0;
    for (int j = 0; j < 8; j++) v = (v << 8) | sk32[(3 - i) * 8 + j];
    k[i] = v;
  }
  g2_compress(out96, g2_mul_words(hash_to_g2(msg, len), k, 4));
  return 0;
}

/* G2.FromCompressed reject class (test hook) */
int bo_g2_decode_class(const uint8_t* sig, size_t len) {
  bo_init();
  g2a s;
  return g2_decompress(sig, len, &s);
}

/* ================================================================ tbls (threshold) */
/* Scalars mod r as 4 little-endian 64-bit words (< r). Only the Lagrange coefficients use them, a few
   thousand products per Recover, so a shift-and-add product is plenty. */
typedef struct {
  uint64_t w[4];
} sc;
static int sc_geq_r(const uint64_t* a) {
  for (int i = 3; i >= 0; i--)
    if (a[i] != C_R_ORDER[i]) return a[i] > C_R_ORDER[i];
  return 1;
}
static sc sc_add(sc a, sc b) { /* a, b < r < 2^255: the sum fits 256 bits */
  sc s;
  unsigned __int128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (unsigned __int128)a.w[i] + b.w[i];
    s.w[i] = (uint64_t)c;
    c >>= 64;
  }
  if (sc_geq_r(s.w)) {
    __int128 d = 0;
    for (int i = 0; i < 4; i++) {
      d += (__int128)s.w[i] - C_R_ORDER[i];
      s.w[i] = (uint64_t)d;
      d >>= 64;
    }
  }
  return s;
}
static sc sc_neg(sc a) {
  sc z = {{0, 0, 0, 0}};
  if (!(a.w[0] | a.w[1] | a.w[2] | a.w[3])) return z;
  __int128 d = 0;
  for (int i = 0; i < 4; i++) {
    d += (__int128)C_R_ORDER[i] - a.w[i];
    z.w[i] = (uint64_t)d;
    d >>= 64;
  }
  return z;
}
static sc sc_mul(sc a, sc b) {
  sc acc = {{0, 0, 0, 0}};
  for (int i = 255; i >= 0; i--) {
    acc = sc_add(acc, acc);
    if ((b.w[i >> 6] >> (i & 63)) & 1) acc = sc_add(acc, a);
  }
  return acc;
}
static sc sc_small(uint64_t v) { /* v < r */
  sc s = {{v, 0, 0, 0}};
  return s;
}
static sc sc_inv(sc a) { /* a^(r-2) */
  uint64_t e[4];
  memcpy(e, C_R_ORDER, sizeof e);
  e[0] -= 2; /* r is odd and its low word is 1 -> no borrow */
  sc acc = sc_small(1);
  for (int i = 255; i >= 0; i--) {
    acc = sc_mul(acc, acc);
    if ((e[i >> 6] >> (i & 63)) & 1) acc = sc_mul(acc, a);
  }
  return acc;
}

/* [k] P for a small k (share indices): double-and-add from k's top bit */
static g1j g1_mul_small(g1j p, uint64_t k) {
  g1j acc = p;
  acc.z = fp_zero();
  int top = 63;
  while (top >= 0 && !((k >> top) & 1)) top--;
  for (int b = top; b >= 0; b--) {
    acc = g1_dbl(acc);
    if ((k >> b) & 1) acc = g1_add(acc, p);
  }
  return acc;
}
static g1a g1_to_aff(g1j p) {
  g1a r;
  r.inf = fp_is_zero(p.z);
  if (r.inf) return r;
  fp zi = fp_inv(p.z), zi2 = fp_sqr(zi);
  r.x = fp_mul(p.x, zi2);
  r.y = fp_mul(p.y, fp_mul(zi2, zi));
  return r;
}

/* the group's public polynomial (share.PubPoly): t decoded commitments */
typedef struct {
  int t;
  g1j c[];
} bo_group;

void* bo_group_new(const uint8_t* commits48, int t) {
  bo_init();
  if (t <= 0) return NULL;
  bo_group* g = (bo_group*)malloc(sizeof(bo_group) + (size_t)t * sizeof(g1j));
  if (!g) return NULL;
  g->t = t;
  for (int j = 0; j < t; j++) {
    g1a a;
    if (g1_decompress(commits48 + 48 * (size_t)j, &a) != REJ_OK) {
      free(g);
      return NULL;
    }
    g->c[j].x = a.x;
    g->c[j].y = a.y;
    g->c[j].z = a.inf ? fp_zero() : FP_ONE;
  }
  return g;
}
void bo_group_free(void* g) { free(g); }

/* share.PubPoly.Eval(i) = sum_j C_j (i+1)^j by Horner (oracle/bls12381.py pubpoly_eval) */
static g1a pubpoly_eval(const bo_group* g, unsigned i) {
  g1j v = g->c[g->t - 1];
  for (int j = g->t - 2; j >= 0; j--) v = g1_add(g1_mul_small(v, (uint64_t)i + 1), g->c[j]);
  return g1_to_aff(v);
}

/* tbls.VerifyPartial (kyber sign/tbls): index = the 2-byte big-endian prefix, then bls.Verify of
   the rest against PubPoly.Eval(index). Reject class (a share shorter than 2 bytes: REJ_LENGTH). */
int bo_tbls_verify_partial(const void* gp, const uint8_t* msg, size_t len, const uint8_t* part, size_t plen) {
  const bo_group* g = (const bo_group*)gp;
  if (plen < 2) return REJ_LENGTH;
  const unsigned idx = ((unsigned)part[0] << 8) | part[1];
  g1a pk = pubpoly_eval(g, idx);
  return verify_decoded(&pk, msg, len, part + 2, plen - 2);
}

/* tbls.Recover -> share.RecoverCommit, the same rules as oracle/bls12381.py tbls_recover: walk the
   shares in input order, skip invalid ones, take valid ones until t are held (a duplicate index
   counts toward t); keep the last point per index and drop indices >= n; fewer than t distinct ->
   -1. Otherwise out96 = compress(sum_i lambda_i S_i), lambda_i the Lagrange coefficient at 0 over
   x = index + 1. parts = `count` shares laid end to end, lens[k] bytes each. */
int bo_tbls_recover(const void* gp, const uint8_t* msg, size_t len, const uint8_t* parts, const size_t* lens,
                    size_t count, int t, int n, uint8_t out96[96]) {
  const bo_group* g = (const bo_group*)gp;
  if (t <= 0 || n <= 0 || n > 65536) return -1;
  int* idx = (int*)malloc(sizeof(int) * (size_t)t);
  g2a* pts = (g2a*)malloc(sizeof(g2a) * (size_t)t);
  int* slot = (int*)malloc(sizeof(int) * (size_t)n); /* index -> position in the distinct list */
  if (!idx || !pts || !slot) {
    free(idx), free(pts), free(slot);
    return -1;
  }
  for (int i = 0; i < n; i++) slot[i] = -1;
  int taken = 0, distinct = 0;
  size_t off = 0;
  for (size_t k = 0; k < count && taken < t; off += lens[k], k++) {
    const uint8_t* p = parts + off;
    if (lens[k] < 2 || bo_tbls_verify_partial(g, msg, len, p, lens[k]) != REJ_OK) continue;
    taken++;
    const int i = ((int)p[0] << 8) | p[1];
    if (i >= n) continue;
    g2a s;
    g2_decompress(p + 2, lens[k] - 2, &s);
    if (slot[i] < 0) {
      slot[i] = distinct;
      idx[distinct++] = i;
    }
    pts[slot[i]] = s;
  }
  int rc = -1;
  if (distinct >= t) {
    g2j acc = g2_from_aff(pts[0]);
    acc.z = fp2_zero();
    for (int a = 0; a < distinct; a++) {
      sc num = sc_small(1), den = sc_small(1);
      const sc xa = sc_small((uint64_t)idx[a] + 1);
      for (int b = 0; b < distinct; b++) {
        if (b == a) continue;
        const sc xb = sc_small((uint64_t)idx[b] + 1);
        num = sc_mul(num, xb);
        den = sc_mul(den, sc_add(xb, sc_neg(xa)));
      }
      const sc lam = sc_mul(num, sc_inv(den));
      acc = g2_add(acc, g2_mul_words(g2_from_aff(pts[a]), lam.w, 4));
    }
    g2_compress(out96, acc);
    rc = 0;
  }
  free(idx), free(pts), free(slot);
  return rc;
}

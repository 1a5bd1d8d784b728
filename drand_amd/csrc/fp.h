// Fp arithmetic for BLS12-381 on gfx950: 381-bit prime field, 12 x 32-bit little-endian limbs,
// Montgomery form (R = 2^392, see fp_mul_u12). Values live in the redundant range [0, 2p): a
// multiplier output needs no final subtraction (its bound is < 2p for ANY 12-word inputs, see the
// operand contract above fp_mul_u12), and add/sub/neg keep [0, 2p) with one 2p correction. Only
// comparisons (fp_is_zero, fp_eq) and leaving Montgomery form (fp_from_mont) canonicalise.
//
// This is the engine's replacement for kilic/bls12-381's fp.go + the amd64 assembly Montgomery
// multiply (the [ext] native code on the reference path). Everything above this
// file (fp2/fp6/fp12, curves, hash-to-curve, pairing) only uses the fp_* API below, so the limb
// representation can change without touching the tower.
//
// Multiplication: Montgomery product scanning in radix 2^28 (fp_mul_u12 below); each limb product
// is one v_mad_u64_u32 (full rate on gfx950: tools/intrate.hip -> profiles/intrate.json).
#pragma once
#include <stdint.h>
#include "bls_constants.h"

#ifdef BLS_HOST
// Host build of the device arithmetic (tools/opcount.cpp): the SAME source compiled by clang++ for
// the CPU, used to count Montgomery multiplications per stage and to run the engine's algorithms
// on the CPU against the oracle. Never linked into the product library.
#include <stddef.h>
#define DI inline
#define NOINL static inline
namespace bls {
extern unsigned long long g_fp_mul_count;
}
#define BLS_COUNT_MUL() (++::bls::g_fp_mul_count)
#else
#include <hip/hip_runtime.h>
#define DI __device__ __forceinline__
#define NOINL static __device__ __noinline__
#define BLS_COUNT_MUL() ((void)0)
#endif

namespace bls {

struct fp {
  uint32_t l[12];
};

DI fp fp_load_const(const uint32_t (&c)[12]) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c[i];
  return r;
}

DI fp fp_zero() {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = 0;
  return r;
}

DI fp fp_one() { return fp_load_const(FP_ONE); }

// a == 0 as a 12-word integer (not mod p)
DI bool fp_raw_is_zero(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i];
  return acc == 0;
}

// a == 0 mod p for a in [0, 2p): a is 0 or p
DI bool fp_is_zero(const fp& a) {
  uint32_t z = 0, q = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    z |= a.l[i];
    q |= a.l[i] ^ P_RAW[i];
  }
  return (z == 0) | (q == 0);
}

DI fp fp_select(bool c, const fp& a, const fp& b) {  // c ? a : b
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// r = s - 2p if s >= 2p else s, for s < 4p (< 2^383: no carry word)
DI fp fp_reduce_2p(const uint32_t (&s)[12]) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(s[i], P2_RAW[i], br, &br);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = br ? s[i] : d[i];
  return r;
}

// canonical representative: a - p if a >= p, for a in [0, 2p)
DI fp fp_canon(const fp& a) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(a.l[i], P_RAW[i], br, &br);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = br ? a.l[i] : d[i];
  return r;
}

// The additive operations below interleave their two carry chains limb by limb (the sum's and the
// correction's, or the two components' of an Fp2 value): a carry link that reads the previous link's
// carry needs one wait state on gfx950, which the other chain's link fills -- written chain after
// chain, the compiler pads every link with s_nop (82 -> 29 pads for two Fp2 additions, tools kt).
DI fp fp_add(const fp& a, const fp& b) {
  uint32_t s[12], d[12];
  unsigned c = 0, br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    s[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
    d[i] = __builtin_subc(s[i], P2_RAW[i], br, &br);
  }
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = br ? s[i] : d[i];
  return r;
}

DI fp fp_dbl(const fp& a) { return fp_add(a, a); }

// a + b WITHOUT reduction, for inputs < 2p: the result (< 4p) may only feed a multiplier (see the
// operand contract above fp_mul_u12) or one more fp_add_lazy (< 8p, the most any multiplier operand
// carries), never fp_add/fp_sub/fp_eq or serialization.
DI fp fp_add_lazy(const fp& a, const fp& b) {
  fp r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return r;
}

// a/2 mod p: (a + (a odd ? p : 0)) >> 1 (a < 2p: the sum is < 3p < 2^383, no 13th limb needed; the
// result is < 1.5p)
DI fp fp_half(const fp& a) {
  const uint32_t m = 0u - (a.l[0] & 1u);
  uint32_t s[12];
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = __builtin_addc(a.l[i], P_RAW[i] & m, c, &c);
  fp r;
#pragma unroll
  for (int i = 0; i < 11; i++) r.l[i] = (s[i] >> 1) | (s[i + 1] << 31);
  r.l[11] = s[11] >> 1;
  return r;
}

// a - b for a, b in [0, 2p): the difference is in (-2p, 2p); 2p is added back on a borrow
// (a - b and a - b + 2p as two interleaved chains, the borrow of the first picks)
DI fp fp_sub(const fp& a, const fp& b) {
  uint32_t d[12], e[12];
  unsigned br = 0, c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    d[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
    e[i] = __builtin_addc(d[i], P2_RAW[i], c, &c);
  }
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = br ? e[i] : d[i];
  return r;
}

// sub ? a - b : a + b for a, b in [0, 2p), result in [0, 2p): one operation whose direction is data
// (the 3-lane kernels pick it per lane role) instead of both results and a select.
//   chain 1: s = a + (b ^ m) + sub          (m = all ones when sub: a + ~b + 1 = a - b + 2^384)
//   chain 2: d = s + (2p ^ k) + !sub        (k = all ones when adding: d = s - 2p;  else d = s + 2p)
// adding: d is right iff s >= 2p (chain 2 carries out); subtracting: d is right iff a < b (chain 1
// does not carry out)
DI fp fp_addsub(const fp& a, const fp& b, bool sub) {
  const uint32_t m = sub ? 0xffffffffu : 0u;
  uint32_t s[12], d[12];
  unsigned c1 = sub ? 1u : 0u, c2 = sub ? 0u : 1u;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    s[i] = __builtin_addc(a.l[i], b.l[i] ^ m, c1, &c1);
    d[i] = __builtin_addc(s[i], P2_RAW[i] ^ ~m, c2, &c2);
  }
  const bool take_d = sub ? (c1 == 0u) : (c2 != 0u);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = take_d ? d[i] : s[i];
  return r;
}

// 2p - a, or 0 for a == 0 (keeps the result below 2p)
DI fp fp_neg(const fp& a) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(P2_RAW[i], a.l[i], br, &br);
  uint32_t m = fp_raw_is_zero(a) ? 0u : 0xffffffffu;
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = d[i] & m;
  return r;
}

// a == b mod p for a, b in [0, 2p)
DI bool fp_eq(const fp& a, const fp& b) { return fp_is_zero(fp_sub(a, b)); }

typedef uint32_t u12 __attribute__((ext_vector_type(12)));

// Operand contract of the multipliers (fp_mul_u12, fp_sqr_u12, fp2_mul_u24, fp2_sqr_u24): every
// input word-vector may be ANY 12-word value (< 2^384; in practice < 8p: at most two levels of lazily
// added values < 2p, see fp_add_lazy). Inside the Fp2 bodies negations (16p - y) and sums of such
// operands are formed limb-wise in radix 2^28 (limbs < 2^29.6, values < 2^386). The output is < 2p,
// with no final subtraction: a Montgomery dot product of two terms is < 2 * 2^771, so the result
// (T + m p) / R < 2^772 / 2^392 + p = 2^380 + p < 2p. Column sums stay < 2^63 (at most 28 limb
// products < 2^58, or 14 < 2^58.6, plus 14 of m_j p_{k-j} < 2^56 and the carried-in column).
// Montgomery product a*b*R^-1 mod p, R = 2^392.
// Deliberately NOT inlined: one copy of the body per code object keeps kernels small
// (instruction-cache resident) and compile times sane. Arguments/results are ext_vector u12 so
// they travel in v0..v23 / v0..v11 (a by-value struct would be passed through scratch).
//
// Storage stays 12 x 32-bit limbs; the product runs in radix 2^28 (14 limbs): every limb product is
// < 2^56, so a whole column (<= 28 products + the carried-in column < 2^62) accumulates in one
// 64-bit register with plain v_mad_u64_u32 -- no carry-propagation instructions at all (the
// 32-bit-limb form needs one v_addc per product): 588 VALU instructions per multiply instead of
// ~825, measured 67.7 G vs 59.8 G fp_mul/s on one MI355X (tools/fpbench.hip, profiles/).
// Product scanning with interleaved reduction (FIPS): column k adds a_j b_{k-j} + m_j p_{k-j};
// m_k = (low 28 bits of the column) * (-p^-1) mod 2^28. The result (< 2p, see above) is returned as
// it is; fp_canon adds the conditional subtraction where a canonical value is needed.
// Constants (bls_constants.h) are generated for R = 2^392 (gen_constants.py).
constexpr uint32_t M28 = (1u << 28) - 1u;

DI void fp_split28(const u12& a, uint32_t (&x)[14]) {
#pragma unroll
  for (int k = 0; k < 14; k++) {
    const int w = (28 * k) >> 5, s = (28 * k) & 31;
    const uint64_t cat = ((uint64_t)(w + 1 < 12 ? a[w + 1] : 0u) << 32) | a[w];
    x[k] = (uint32_t)(cat >> s) & M28;
  }
}

// 14 x 28-bit limbs (top limb < 2^18, value < 2p) -> 12 x 32-bit, still < 2p
DI u12 fp_join28(const uint32_t (&t)[14]) {
  u12 r;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    const int k = (32 * w) / 28, s = (32 * w) % 28;  // s <= 24: two limbs cover the word
    r[w] = (t[k] >> s) | (t[k + 1] << (28 - s));
  }
  return r;
}

NOINL u12 fp_mul_u12(u12 a, u12 b) {
  BLS_COUNT_MUL();
  uint32_t x[14], y[14], m[14], t[14];
  fp_split28(a, x);
  fp_split28(b, y);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
#pragma unroll
    for (int j = 0; j < k; j++) {
      acc += (uint64_t)x[j] * y[k - j];
      acc += (uint64_t)m[j] * P28[k - j];
    }
    acc += (uint64_t)x[k] * y[0];
    m[k] = ((uint32_t)acc * P_INV28) & M28;
    acc += (uint64_t)m[k] * P28[0];  // low 28 bits become 0
    acc >>= 28;
  }
#pragma unroll
  for (int k = 14; k < 27; k++) {
#pragma unroll
    for (int j = k - 13; j < 14; j++) {
      acc += (uint64_t)x[j] * y[k - j];
      acc += (uint64_t)m[j] * P28[k - j];
    }
    t[k - 14] = (uint32_t)acc & M28;
    acc >>= 28;
  }
  t[13] = (uint32_t)acc;  // < 2^18: the result is < 2p < 2^382
  return fp_join28(t);
}

// Montgomery square: the cross products x_j x_{k-j} (j < k-j) appear twice, so they are taken once
// against the doubled limbs 2x (29 bits, products < 2^57): 105 product MADs instead of 196.
// the square's column loop on split limbs x (< 2^28): t = x^2 R^-1 as 14 limbs (< 2^28, top < 2^18)
DI void fp_sqr28_t(const uint32_t (&x)[14], uint32_t (&t)[14]) {
  uint32_t x2[14], m[14];
#pragma unroll
  for (int k = 0; k < 14; k++) x2[k] = x[k] << 1;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
#pragma unroll
    for (int j = (k > 13 ? k - 13 : 0); 2 * j < k; j++) acc += (uint64_t)x[j] * x2[k - j];
    if ((k & 1) == 0) acc += (uint64_t)x[k / 2] * x[k / 2];
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) acc += (uint64_t)m[j] * P28[k - j];
      m[k] = ((uint32_t)acc * P_INV28) & M28;
      acc += (uint64_t)m[k] * P28[0];
      acc >>= 28;
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) acc += (uint64_t)m[j] * P28[k - j];
      t[k - 14] = (uint32_t)acc & M28;
      acc >>= 28;
    }
  }
  t[13] = (uint32_t)acc;
}

NOINL u12 fp_sqr_u12(u12 a) {
  BLS_COUNT_MUL();
  uint32_t x[14], t[14];
  fp_split28(a, x);
  fp_sqr28_t(x, t);
  return fp_join28(t);
}

// 4p - a for a in [0, 4p] (12-word borrow chain)
DI u12 fp_4p_minus_u12(const u12& a) {
  u12 r;
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = __builtin_subc(P4_RAW[i], a[i], br, &br);
  return r;
}

// 16p - y limb-wise for a split operand y < 8p (28-bit limbs): every limb of NEG28_16P is at least any
// such limb, so there are no borrows; the limbs stay below 2^29 (a multiplier operand, never stored)
DI void fp_neg28(const uint32_t (&y)[14], uint32_t (&r)[14]) {
#pragma unroll
  for (int k = 0; k < 14; k++) r[k] = NEG28_16P[k] - y[k];
}

// a + b as a 12-word integer (no reduction: a, b < 2p keep the sum < 2^384)
DI u12 fp_add_raw_u12(const u12& a, const u12& b) {
  u12 r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = __builtin_addc(a[i], b[i], c, &c);
  return r;
}

typedef uint32_t u24 __attribute__((ext_vector_type(24)));

// Montgomery "dot product" with one reduction (lazy reduction), operands in radix 2^28 with limbs
// below 2^29 (operand contract above fp_mul_u12):
//   DOT:  r = (x0 y0 + x1 y1) R^-1        !DOT: r = x0 y0 R^-1         (r < 2p)
template <bool DOT>
DI void fp_mont_dot_t(const uint32_t (&x0)[14], const uint32_t (&y0)[14], const uint32_t (&x1)[14],
                      const uint32_t (&y1)[14], uint32_t (&t)[14]) {
  uint32_t m[14];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      c += (uint64_t)x0[j] * y0[k - j];
      if (DOT) c += (uint64_t)x1[j] * y1[k - j];
    }
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) c += (uint64_t)m[j] * P28[k - j];
      m[k] = ((uint32_t)c * P_INV28) & M28;
      c += (uint64_t)m[k] * P28[0];
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) c += (uint64_t)m[j] * P28[k - j];
      t[k - 14] = (uint32_t)c & M28;
    }
    c >>= 28;
  }
  t[13] = (uint32_t)c;
}
// x0 y0 + x1 y1 + x2 y2 (NT = 3) or the first two (NT = 2), one reduction: limbs below 2^29 (operand
// splits and NEG28_4P negations of values < 2p), so a column holds at most 42 products < 2^58 plus 14
// m_j p_{k-j} < 2^56 and the carry: < 2^63.5. Values: three terms below 24 p^2 each keep the result
// below 2p (operand contract above fp_mul_u12).
template <int NT>
DI u12 fp_mont_dot3(const uint32_t (&x0)[14], const uint32_t (&y0)[14], const uint32_t (&x1)[14],
                    const uint32_t (&y1)[14], const uint32_t (&x2)[14], const uint32_t (&y2)[14]) {
  uint32_t m[14], t[14];
  uint64_t c = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      c += (uint64_t)x0[j] * y0[k - j];
      c += (uint64_t)x1[j] * y1[k - j];
      if (NT == 3) c += (uint64_t)x2[j] * y2[k - j];
    }
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) c += (uint64_t)m[j] * P28[k - j];
      m[k] = ((uint32_t)c * P_INV28) & M28;
      c += (uint64_t)m[k] * P28[0];
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) c += (uint64_t)m[j] * P28[k - j];
      t[k - 14] = (uint32_t)c & M28;
    }
    c >>= 28;
  }
  t[13] = (uint32_t)c;
  return fp_join28(t);
}

template <bool DOT>
DI u12 fp_mont_dot(const uint32_t (&x0)[14], const uint32_t (&y0)[14], const uint32_t (&x1)[14],
                   const uint32_t (&y1)[14]) {
  uint32_t t[14];
  fp_mont_dot_t<DOT>(x0, y0, x1, y1, t);
  return fp_join28(t);
}

DI u12 u24_lo(const u24& v) {
  u12 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = v[i];
  return r;
}
DI u12 u24_hi(const u24& v) {
  u12 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = v[12 + i];
  return r;
}
DI u24 u24_of(const u12& lo, const u12& hi) {
  u24 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = lo[i], r[12 + i] = hi[i];
  return r;
}

// The second Fp2 operand of fp2_mul_u24 travels through LDS: 24 + 24 argument words exceed the 32
// VGPR arguments of the AMDGPU calling convention (the excess would go through scratch). Each lane
// owns one 24-word column of the block (kernels run 64-lane workgroups, kcommon.h TPB), and only
// touches its own column, so no barrier is needed.
constexpr int BLS_LANES = 64;
#ifdef BLS_HOST
static uint32_t g_fp2_arg[24 * BLS_LANES];
DI unsigned bls_lane() { return 0; }
#define BLS_SCHED_FENCE() ((void)0)
#else
static __shared__ uint32_t g_fp2_arg[24 * BLS_LANES];
DI unsigned bls_lane() { return threadIdx.x; }
// keeps the scheduler from interleaving two independent halves (it would double the callee's VGPRs)
#define BLS_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
#endif

DI void fp2_arg_store(const u24& b) {
  const unsigned l = bls_lane();
#pragma unroll
  for (int i = 0; i < 24; i++) g_fp2_arg[i * BLS_LANES + l] = b[i];
}

// Fp2 product with three products per column (Karatsuba inside the column loop) and two reductions:
//   W  = a0 (b0 + b1)                   shared by both outputs
//   c0 = W + b1 (32p - a0 - a1)          = a0 b0 - a1 b1 + 32p b1
//   c1 = W + b0 (a1 + 16p - a0)          = a0 b1 + a1 b0 + 16p b0
// Column k forms W_k in its own 64-bit register, the second product of each output directly in that
// output's accumulator, and adds W_k to both (one v_lshl_add_u64 each): 3 x 196 product MADs + 2 x 196
// reduction MADs against 4 x 196 + 2 x 196 for the two-term dot products. The negations are formed
// limb-wise against NEG28_32P / NEG28_16P (no borrows: a0, a1 < 8p, the operand contract above
// fp_mul_u12), so every column sum is non-negative: W < 14 * 2^57, b1 (32p - a0 - a1) < 14 * 2^58,
// b0 (a1 + 16p - a0) < 14 * 2^57.6, the reduction < 14 * 2^56: < 2^62.6 with the carry. Values (a, b
// < 8p): c0 < 64p^2 + 256p^2, c1 < 128p^2 + 128p^2, so each result (T + m p) / R < 2p.
DI void fp2_mont_kara_t(const uint32_t (&x0)[14], const uint32_t (&ys)[14], const uint32_t (&y1)[14],
                        const uint32_t (&xz)[14], const uint32_t (&y0)[14], const uint32_t (&xy)[14],
                        uint32_t (&t0)[14], uint32_t (&t1)[14]) {
  uint32_t m0[14], m1[14];
  uint64_t c0 = 0, c1 = 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
    uint64_t w = 0;
#pragma unroll
    for (int j = lo; j <= hi; j++) {
      w += (uint64_t)x0[j] * ys[k - j];
      c0 += (uint64_t)y1[j] * xz[k - j];
      c1 += (uint64_t)y0[j] * xy[k - j];
    }
    c0 += w;
    c1 += w;
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) {
        c0 += (uint64_t)m0[j] * P28[k - j];
        c1 += (uint64_t)m1[j] * P28[k - j];
      }
      m0[k] = ((uint32_t)c0 * P_INV28) & M28;
      m1[k] = ((uint32_t)c1 * P_INV28) & M28;
      c0 += (uint64_t)m0[k] * P28[0];
      c1 += (uint64_t)m1[k] * P28[0];
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) {
        c0 += (uint64_t)m0[j] * P28[k - j];
        c1 += (uint64_t)m1[j] * P28[k - j];
      }
      t0[k - 14] = (uint32_t)c0 & M28;
      t1[k - 14] = (uint32_t)c1 & M28;
    }
    c0 >>= 28;
    c1 >>= 28;
  }
  t0[13] = (uint32_t)c0;
  t1[13] = (uint32_t)c1;
}

// BLS_FP2_KARA: the called body (fp2_mul_u24 and the tri.h slot forms); BLS_FP2_KARA_INL: the forms
// expanded in place (tower.h fp2_mul_inl), whose kernels run call-free at 2 waves/SIMD and feel its
// larger working set (two reductions in flight instead of one) as spills.
#ifndef BLS_FP2_KARA
#define BLS_FP2_KARA 1
#endif
#ifndef BLS_FP2_KARA_INL
#define BLS_FP2_KARA_INL 0
#endif

DI u24 fp2_mul_body_kara(const u24& a, const u12& b0, const u12& b1) {
  uint32_t x0[14], x1[14], y0[14], y1[14], ys[14], xz[14], xy[14], t0[14], t1[14];
  fp_split28(u24_lo(a), x0);
  fp_split28(u24_hi(a), x1);
  fp_split28(b0, y0);
  fp_split28(b1, y1);
#pragma unroll
  for (int k = 0; k < 14; k++) {
    ys[k] = y0[k] + y1[k];
    xz[k] = NEG28_32P[k] - x0[k] - x1[k];
    xy[k] = x1[k] + (NEG28_16P[k] - x0[k]);
  }
  fp2_mont_kara_t(x0, ys, y1, xz, y0, xy, t0, t1);
  return u24_of(fp_join28(t0), fp_join28(t1));
}

// Fp2 product (a0 + a1 i)(b0 + b1 i) in one body:
//   c0 = a0 b0 + a1 (16p - b1), c1 = a0 b1 + a1 b0
// i.e. two reductions instead of three multiplications' worth (counted as the 3 of Karatsuba).
template <bool KARA>
DI u24 fp2_mul_body_t(const u24& a, const u12& b0, const u12& b1) {
  if (KARA) return fp2_mul_body_kara(a, b0, b1);
  uint32_t x0[14], x1[14], y0[14], y1[14], yn[14];
  fp_split28(u24_lo(a), x0);
  fp_split28(u24_hi(a), x1);
  fp_split28(b0, y0);
  fp_split28(b1, y1);
  fp_neg28(y1, yn);
  const u12 c0 = fp_mont_dot<true>(x0, y0, x1, yn);
  BLS_SCHED_FENCE();
  const u12 c1 = fp_mont_dot<true>(x0, y1, x1, y0);
  return u24_of(c0, c1);
}
DI u24 fp2_mul_body(const u24& a, const u12& b0, const u12& b1) { return fp2_mul_body_t<BLS_FP2_KARA>(a, b0, b1); }

// Fp2 square: c0 = (a0 + a1)(a0 + 16p - a1), c1 = (2 a0) a1, the sums formed limb-wise in radix 2^28
// after splitting a0 and a1 once (no carry chains: a0 + a1 has limbs < 2^29, a0 + 16p - a1 < 2^29.6
// against NEG28_16P, whose limbs are at least any operand limb). A squaring operand is at most ONE
// lazy sum (< 4p; every fp2_sqr* call site squares a reduced value or one fp2_add_lazy): the values
// stay below 20p, the column sums below 2^62.6 and the result below 2p (operand contract above).
DI u24 fp2_sqr_body(const u24& a) {
  uint32_t s0[14], s1[14], x[14], y[14];
  fp_split28(u24_lo(a), s0);
  fp_split28(u24_hi(a), s1);
#pragma unroll
  for (int k = 0; k < 14; k++) {
    x[k] = s0[k] + s1[k];
    y[k] = s0[k] + (NEG28_16P[k] - s1[k]);
  }
  const u12 c0 = fp_mont_dot<false>(x, y, x, y);
  BLS_SCHED_FENCE();
#pragma unroll
  for (int k = 0; k < 14; k++) x[k] = s0[k] << 1;
  const u12 c1 = fp_mont_dot<false>(x, s1, x, s1);
  return u24_of(c0, c1);
}

// The called forms: b of fp2_mul_u24 comes from fp2_arg_store (LDS), one copy of each body per
// code object. The _inl forms (tower.h fp2_mul_inl / fp2_sqr_inl) expand the bodies in place for
// call-free hot loops (the 3-lane final exponentiation, tri.h).
NOINL u24 fp2_mul_u24(u24 a) {
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  const unsigned l = bls_lane();
  u12 b0, b1;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    b0[i] = g_fp2_arg[i * BLS_LANES + l];
    b1[i] = g_fp2_arg[(12 + i) * BLS_LANES + l];
  }
  return fp2_mul_body(a, b0, b1);
}

NOINL u24 fp2_sqr_u24(u24 a) {
  BLS_COUNT_MUL();
  BLS_COUNT_MUL();
  return fp2_sqr_body(a);
}

DI u12 fp_to_u12(const fp& a) {
  u12 v;
#pragma unroll
  for (int i = 0; i < 12; i++) v[i] = a.l[i];
  return v;
}

DI fp fp_from_u12(const u12& v) {
  fp a;
#pragma unroll
  for (int i = 0; i < 12; i++) a.l[i] = v[i];
  return a;
}

DI fp fp_mul(const fp& a, const fp& b) { return fp_from_u12(fp_mul_u12(fp_to_u12(a), fp_to_u12(b))); }
// fp_mul expanded in place (same column sums, same result) for call-free loops
DI fp fp_mul_inl(const fp& a, const fp& b) {
  BLS_COUNT_MUL();
  uint32_t x[14], y[14];
  fp_split28(fp_to_u12(a), x);
  fp_split28(fp_to_u12(b), y);
  return fp_from_u12(fp_mont_dot<false>(x, y, x, y));
}

DI fp fp_sqr(const fp& a) { return fp_from_u12(fp_sqr_u12(fp_to_u12(a))); }

// small-constant multiples via additions
DI fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
DI fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
DI fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }

DI fp fp_to_mont(const fp& raw) { return fp_mul(raw, fp_load_const(FP_R2)); }

// canonical raw value in [0, p)
DI fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_canon(fp_mul(a, one));
}

// a^e for a public exponent given as little-endian 32-bit words (uniform across the wave ->
// scalar branches, no divergence). Left-to-right 2-bit fixed window: a 4-entry table keeps the
// caller's VGPR budget small (every kernel that inverts inherits this function's register count).
template <int NW>
DI fp fp_pow_words(const fp& a, const uint32_t (&e)[NW]) {
  const fp a2 = fp_sqr(a);
  const fp a3 = fp_mul(a2, a);
  fp r = fp_one();
  bool started = false;
  for (int w = NW - 1; w >= 0; w--) {
    const uint32_t word = e[w];
    for (int dig = 15; dig >= 0; dig--) {
      const uint32_t d = (word >> (2 * dig)) & 3u;
      if (started) {
        r = fp_sqr(r);
        r = fp_sqr(r);
      }
      if (d) {
        const fp t = d == 1u ? a : (d == 2u ? a2 : a3);
        r = started ? fp_mul(r, t) : t;
        started = true;
      }
    }
  }
  return r;
}

NOINL u12 fp_pow_p_minus_2(u12 a) { return fp_to_u12(fp_pow_words<12>(fp_from_u12(a), EXP_P_MINUS_2)); }
NOINL u12 fp_pow_sqrt(u12 a) { return fp_to_u12(fp_pow_words<12>(fp_from_u12(a), EXP_P_PLUS_1_DIV_4)); }
NOINL u12 fp_pow_legendre(u12 a) { return fp_to_u12(fp_pow_words<12>(fp_from_u12(a), EXP_P_MINUS_1_DIV_2)); }
// Montgomery square / product with the running value kept split in radix 2^28 (14 limbs < 2^28, the
// output form of the column loops): an exponentiation's chain of squares skips fp_split28 /
// fp_join28 at every step
typedef uint32_t u14 __attribute__((ext_vector_type(14)));
NOINL u14 fp_sqr_r28(u14 xv) {
  BLS_COUNT_MUL();
  uint32_t x[14], t[14];
#pragma unroll
  for (int k = 0; k < 14; k++) x[k] = xv[k];
  fp_sqr28_t(x, t);
  u14 r;
#pragma unroll
  for (int k = 0; k < 14; k++) r[k] = t[k];
  return r;
}
NOINL u14 fp_mul_r28(u14 xv, u12 b) {
  BLS_COUNT_MUL();
  uint32_t x[14], y[14], t[14];
#pragma unroll
  for (int k = 0; k < 14; k++) x[k] = xv[k];
  fp_split28(b, y);
  fp_mont_dot_t<false>(x, y, x, y, t);
  u14 r;
#pragma unroll
  for (int k = 0; k < 14; k++) r[k] = t[k];
  return r;
}

// a^((p-3)/4) by a 4-bit sliding window (bls_constants.h EXP_SQRT_W4, from gen_constants.py): the odd
// powers a, a^3, ..., a^15 (8 values, 96 words: what the calling convention keeps across the calls),
// 375 squarings and 78 multiplications instead of the fixed 2-bit windows' ~380 and ~143. The digit
// of an entry is the same in every lane, so the table read is a wave-uniform select.
NOINL u12 fp_pow_p_minus_3_div_4(u12 a12) {
  const fp a = fp_from_u12(a12);
  fp tab[8];
  tab[0] = a;
  const fp a2 = fp_sqr(a);
#pragma unroll
  for (int k = 1; k < 8; k++) tab[k] = fp_mul(tab[k - 1], a2);
  u14 r;
  {
    uint32_t x[14];
    fp_split28(fp_to_u12(tab[(EXP_SQRT_W4[0] & 255) >> 1]), x);
#pragma unroll
    for (int k = 0; k < 14; k++) r[k] = x[k];
  }
#pragma unroll 1
  for (int e = 1; e < EXP_SQRT_W4_N; e++) {
    const int ent = EXP_SQRT_W4[e], nsq = ent >> 8, d = (ent & 255) >> 1;
#pragma unroll 1
    for (int k = 0; k < nsq; k++) {
      BLS_COUNT_MUL();
      uint32_t x[14], tt[14];
#pragma unroll
      for (int q = 0; q < 14; q++) x[q] = r[q];
      fp_sqr28_t(x, tt);
#pragma unroll
      for (int q = 0; q < 14; q++) r[q] = tt[q];
    }
    fp t = tab[0];
#pragma unroll
    for (int k = 1; k < 8; k++) t = fp_select(d == k, tab[k], t);
    r = fp_mul_r28(r, fp_to_u12(t));
  }
#pragma unroll 1
  for (int k = 0; k < EXP_SQRT_W4_TAIL; k++) r = fp_sqr_r28(r);
  uint32_t t[14];
#pragma unroll
  for (int k = 0; k < 14; k++) t[k] = r[k];
  return fp_join28(t);
}

// w = a^((p-3)/4): t = w*a satisfies t^2 = a (a a residue or 0) or t^2 = -a (non-residue), and
// 1/t = w or -w respectively: a square root AND its inverse from one exponentiation.
DI fp fp_pow_sqrt_inv(const fp& a) { return fp_from_u12(fp_pow_p_minus_3_div_4(fp_to_u12(a))); }

// ---------------------------------------------------------------- inversion by binary GCD
// Pornin's optimized binary GCD (eprint 2020/972, Algorithm 2): 25 outer iterations of 31 divsteps
// run on 64-bit approximations of (a, b) -- the low 31 bits and the top 33 bits of the longer one --
// and the resulting signed factors (|f|, |g| <= 2^31) are applied to the full-width values in radix
// 2^28. ~45 k VALU instructions against ~255 k for a^(p-2). The inputs are public (verification),
// so data-dependent lengths are fine; every lane runs the same instruction stream (selects only).
// Invariants a = u y k, b = v y k (mod p) with k = 2^(25 i) after i iterations; at the end b = 1, so
// y^-1 = v 2^625 and the Montgomery inverse is fp_mul(v, 2^625 R^3) (FP_INV_FIX). 0 -> 0.

// bit length of a 12-word integer (0 for 0)
DI int fp_bitlen12(const uint32_t (&c)[12]) {
  int n = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) n = c[i] ? 32 * i + 32 - __builtin_clz(c[i]) : n;
  return n;
}

// floor(x / 2^s) for x < 2^(s + 33): bits s .. s+32 lie in words s/32 and s/32 + 1
DI uint64_t fp_top33(const uint32_t (&x)[12], int s) {
  const int w = s >> 5, o = s & 31;
  uint32_t x0 = 0, x1 = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    x0 = i == w ? x[i] : x0;
    x1 = i == w + 1 ? x[i] : x1;
  }
  return ((((uint64_t)x1 << 32) | x0) >> o) & ((1ull << 33) - 1);
}

// x f + y g over radix-2^28 limbs (|f|, |g| <= 2^31): limbs L[0..13] in [0, 2^28), the signed rest
// returned (value = sum L_k 2^(28k) + rest 2^392)
DI int64_t fp_lincomb28(const uint32_t (&X)[14], const uint32_t (&Y)[14], int64_t f, int64_t g,
                        uint32_t (&L)[14]) {
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 14; k++) {
    acc += (int64_t)X[k] * f + (int64_t)Y[k] * g;
    L[k] = (uint32_t)acc & M28;
    acc >>= 28;
  }
  return acc;
}

// (x f + y g) / 2^31 for an exactly divisible combination of x, y < 2^381: |result| < 2^382, returned
// as its magnitude (12 words) with the sign in *neg
DI void fp_lincomb_shr31(const uint32_t (&X)[14], const uint32_t (&Y)[14], int64_t f, int64_t g, uint32_t (&r)[12],
                         bool& neg) {
  uint32_t L[16];
  uint32_t L14[14];
  const int64_t top = fp_lincomb28(X, Y, f, g, L14);
#pragma unroll
  for (int k = 0; k < 14; k++) L[k] = L14[k];
  L[14] = (uint32_t)top & M28;
  L[15] = (uint32_t)(top >> 28) & M28;
#pragma unroll
  for (int j = 0; j < 12; j++) {
    const int B = 31 + 32 * j, k = B / 28, o = B % 28;
    uint64_t v = ((uint64_t)L[k] >> o) | ((uint64_t)L[k + 1] << (28 - o));
    if (k + 2 < 16) v |= (uint64_t)L[k + 2] << (56 - o);
    r[j] = (uint32_t)v;
  }
  neg = top < 0;
  const uint32_t m = neg ? 0xffffffffu : 0u;
  unsigned c = neg ? 1u : 0u;
#pragma unroll
  for (int j = 0; j < 12; j++) r[j] = __builtin_addc(r[j] ^ m, 0u, c, &c);  // two's-complement negate
}

// (x f + y g) / 2^56 mod p for x, y in [0, 2p): two Montgomery limb steps, result in [0, 2p)
DI fp fp_lincomb_mont56(const uint32_t (&X)[14], const uint32_t (&Y)[14], int64_t f, int64_t g) {
  uint32_t m[2], L[14];
  int64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    if (k < 14) acc += (int64_t)X[k] * f + (int64_t)Y[k] * g;
#pragma unroll
    for (int j = 0; j < 2; j++)
      if (j < k && k - j < 14) acc += (int64_t)m[j] * P28[k - j];
    if (k < 2) {
      m[k] = ((uint32_t)acc * P_INV28) & M28;
      acc += (int64_t)m[k] * P28[0];  // low 28 bits become 0
      acc >>= 28;
    } else {
      L[k - 2] = (uint32_t)acc & M28;
      acc >>= 28;
    }
  }
  // value = sum L_k 2^(28k) + acc 2^392 lies in (-2p, 2p): low 384 bits, plus 2p when negative
  const u12 w = fp_join28(L);
  const uint32_t msk = acc < 0 ? 0xffffffffu : 0u;
  fp r;
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_addc(w[i], P2_RAW[i] & msk, c, &c);
  return r;
}

// The GCD proper. *converged = (b == 1 at the end, or y == 0): the exact algorithm needs at most
// 2*381 - 1 = 761 divsteps and 25 x 31 = 775 run here, but the 64-bit approximations carry no proof
// of that bound for every input, so the caller checks it (fp_inv_bingcd) and the host fuzz
// (tools/opcount invfuzz: random, structured 2^k / p - 2^k / (p +- 1) / 2^k / near-p inputs) counts
// any input that does not converge.
DI u12 fp_inv_bingcd_raw(u12 yin, bool& converged) {
  uint32_t a[12], b[12];
  const fp yc = fp_canon(fp_from_u12(yin));
#pragma unroll
  for (int i = 0; i < 12; i++) {
    a[i] = yc.l[i];
    b[i] = P_RAW[i];
  }
  fp u = fp_zero(), v = fp_zero();
  u.l[0] = 1;
#pragma unroll 1
  for (int it = 0; it < 25; it++) {
    uint32_t c[12];
#pragma unroll
    for (int i = 0; i < 12; i++) c[i] = a[i] | b[i];
    const int n0 = fp_bitlen12(c), n = n0 > 64 ? n0 : 64;
    uint64_t A = ((uint64_t)(a[0] & 0x7fffffffu)) | (fp_top33(a, n - 33) << 31);
    uint64_t B = ((uint64_t)(b[0] & 0x7fffffffu)) | (fp_top33(b, n - 33) << 31);
    int64_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
#pragma unroll
    for (int j = 0; j < 31; j++) {
      const bool odd = (A & 1u) != 0;
      const bool sw = odd & (A < B);
      const uint64_t A2 = sw ? B : A, B2 = sw ? A : B;
      const int64_t F0 = sw ? f1 : f0, G0 = sw ? g1 : g0, F1 = sw ? f0 : f1, G1 = sw ? g0 : g1;
      A = odd ? A2 - B2 : A2;
      f0 = odd ? F0 - F1 : F0;
      g0 = odd ? G0 - G1 : G0;
      B = B2;
      f1 = F1;
      g1 = G1;
      A >>= 1;
      f1 = (int64_t)((uint64_t)f1 << 1);  // 2 f1 (a signed left shift is undefined for f1 < 0 in C++17)
      g1 = (int64_t)((uint64_t)g1 << 1);
    }
    uint32_t X[14], Y[14];
    u12 av, bv;
#pragma unroll
    for (int i = 0; i < 12; i++) av[i] = a[i], bv[i] = b[i];
    fp_split28(av, X);
    fp_split28(bv, Y);
    bool na, nb;
    fp_lincomb_shr31(X, Y, f0, g0, a, na);
    fp_lincomb_shr31(X, Y, f1, g1, b, nb);
    f0 = na ? -f0 : f0;
    g0 = na ? -g0 : g0;
    f1 = nb ? -f1 : f1;
    g1 = nb ? -g1 : g1;
    fp_split28(fp_to_u12(u), X);
    fp_split28(fp_to_u12(v), Y);
    u = fp_lincomb_mont56(X, Y, f0, g0);
    v = fp_lincomb_mont56(X, Y, f1, g1);
  }
  uint32_t nb = b[0] ^ 1u;
#pragma unroll
  for (int i = 1; i < 12; i++) nb |= b[i];
  converged = (nb == 0) | fp_raw_is_zero(yc);
  return fp_to_u12(fp_mul(v, fp_load_const(FP_INV_FIX)));
}

NOINL u12 fp_inv_bingcd(u12 yin) {
  bool ok;
  u12 r = fp_inv_bingcd_raw(yin, ok);
  // never taken on any input the fuzz has seen; a lane that did not converge gets the exponentiation
  if (!ok) r = fp_pow_p_minus_2(yin);
  return r;
}

DI fp fp_inv(const fp& a) { return fp_from_u12(fp_inv_bingcd(fp_to_u12(a))); }  // 0 -> 0

// sqrt candidate a^((p+1)/4); caller checks the square
DI fp fp_sqrt_cand(const fp& a) { return fp_from_u12(fp_pow_sqrt(fp_to_u12(a))); }

// Legendre: true iff a is a non-zero square or zero
DI bool fp_is_square(const fp& a) {
  fp l = fp_from_u12(fp_pow_legendre(fp_to_u12(a)));
  return fp_is_zero(l) || fp_eq(l, fp_one());
}

// canonical big-endian 48-byte <-> raw limbs (no Montgomery conversion)
DI fp fp_raw_from_be48(const uint8_t* b) {
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    const uint8_t* q = b + 44 - 4 * i;
    r.l[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | (uint32_t)q[3];
  }
  return r;
}

DI void fp_raw_to_be48(uint8_t* b, const fp& a) {
#pragma unroll
  for (int i = 0; i < 12; i++) {
    uint8_t* q = b + 44 - 4 * i;
    q[0] = (uint8_t)(a.l[i] >> 24);
    q[1] = (uint8_t)(a.l[i] >> 16);
    q[2] = (uint8_t)(a.l[i] >> 8);
    q[3] = (uint8_t)a.l[i];
  }
}

// raw value < p ?
DI bool fp_raw_lt_p(const fp& a) {
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)__builtin_subc(a.l[i], P_RAW[i], br, &br);
  return br != 0;
}

// raw value > (p-1)/2 ?  (ZCash "lexicographically largest")
DI bool fp_raw_gt_half(const fp& a) {
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) (void)__builtin_subc(FP_P_MINUS_1_DIV_2_RAW[i], a.l[i], br, &br);
  return br != 0;  // (p-1)/2 - a < 0
}

DI bool fp_mont_is_odd(const fp& a) { return fp_from_mont(a).l[0] & 1u; }

}  // namespace bls

// Fp arithmetic for BLS12-381 on gfx950: 381-bit prime field, 12 x 32-bit little-endian limbs,
// Montgomery form (R = 2^384), values kept canonical in [0, p).
//
// This is the engine's replacement for kilic/bls12-381's fp.go + the amd64 assembly Montgomery
// multiply (the [ext] native code on the reference path). Everything above this
// file (fp2/fp6/fp12, curves, hash-to-curve, pairing) only uses the fp_* API below, so the limb
// representation can change without touching the tower.
//
// Multiplication: CIOS Montgomery with the "no final carry word" simplification, valid because the
// top limb of p (0x1a0111ea) is < 2^31 - 1 (so t never needs a 13th word). Each limb product is
// one v_mad_u64_u32 (measured half-rate on gfx950: tools/intrate.hip -> profiles/).
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

DI bool fp_is_zero(const fp& a) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i];
  return acc == 0;
}

DI bool fp_eq(const fp& a, const fp& b) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) acc |= a.l[i] ^ b.l[i];
  return acc == 0;
}

DI fp fp_select(bool c, const fp& a, const fp& b) {  // c ? a : b
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = c ? a.l[i] : b.l[i];
  return r;
}

// r = a - p if a >= p else a, for a < 2p (given as 12 limbs + carry word)
DI fp fp_reduce_once(const uint32_t (&s)[12], uint32_t carry) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(s[i], P_RAW[i], br, &br);
  // keep s if (carry == 0 and borrow) i.e. s < p
  bool keep = (carry == 0) & (br != 0);
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = keep ? s[i] : d[i];
  return r;
}

DI fp fp_add(const fp& a, const fp& b) {
  uint32_t s[12];
  unsigned c = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) s[i] = __builtin_addc(a.l[i], b.l[i], c, &c);
  return fp_reduce_once(s, c);
}

DI fp fp_dbl(const fp& a) { return fp_add(a, a); }

// a/2 mod p: (a + (a odd ? p : 0)) >> 1 (the sum is < 2p < 2^382, no 13th limb needed)
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

DI fp fp_sub(const fp& a, const fp& b) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  // if borrow, add p back
  uint32_t m = br ? 0xffffffffu : 0u;
  unsigned c = 0;
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = __builtin_addc(d[i], P_RAW[i] & m, c, &c);
  return r;
}

DI fp fp_neg(const fp& a) {
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(P_RAW[i], a.l[i], br, &br);
  uint32_t m = fp_is_zero(a) ? 0u : 0xffffffffu;
  fp r;
#pragma unroll
  for (int i = 0; i < 12; i++) r.l[i] = d[i] & m;
  return r;
}

typedef uint32_t u12 __attribute__((ext_vector_type(12)));

// Montgomery product a*b*R^-1 mod p.
// Deliberately NOT inlined: one copy of the body per code object keeps kernels small
// (instruction-cache resident) and compile times sane. Arguments/results are ext_vector u12 so
// they travel in v0..v23 / v0..v11 (a by-value struct would be passed through scratch), and the
// body stays within the caller-saved VGPRs so a call costs only the argument moves.
//
// Device: FIPS (finely integrated product scanning). Column k of a*b and of m*p accumulates into a
// 96-bit (acc64, top) register triple: each limb product is ONE v_mad_u64_u32 (64-bit addend = the
// accumulator itself, carry-out -> VCC) + ONE v_addc_co_u32 folding the carry into `top`, so there
// are no per-product moves (the compiler's CIOS needs ~2.2 moves + a 64-bit add per product:
// tools/fpbench.hip measured 43.4 G (CIOS) vs 59.3 G (this) fp_mul/s on one MI355X).
// Column sums stay < 2^69 (24 products < 2^64 each + the carried column), and the result of the
// last column is < 2p < 2^382, so 12 output limbs + one conditional subtraction suffice.
#ifndef BLS_HOST
#define BLS_MAC2(acc, top, x, y, mm, ps)                                                      \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"   \
      "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"         \
      : "+v"(acc), "+v"(top)                                                                 \
      : "v"(x), "v"(y), "v"(mm), "s"(ps)                                                     \
      : "vcc")
#define BLS_MAC(acc, top, x, y)                                                               \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"         \
      : "+v"(acc), "+v"(top)                                                                 \
      : "v"(x), "v"(y)                                                                       \
      : "vcc")
#define BLS_MACS(acc, top, x, ys)                                                             \
  asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"         \
      : "+v"(acc), "+v"(top)                                                                 \
      : "v"(x), "s"(ys)                                                                      \
      : "vcc")

NOINL u12 fp_mul_u12(u12 a, u12 b) {
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) BLS_MAC2(acc, top, a[j], b[i - j], m[j], P_RAW[i - j]);
    BLS_MAC(acc, top, a[i], b[0]);
    m[i] = (uint32_t)acc * P_INV32;
    BLS_MACS(acc, top, m[i], P_RAW[0]);  // low word becomes 0
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) BLS_MAC2(acc, top, a[j], b[i - j], m[j], P_RAW[i - j]);
    t[i - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(t[i], P_RAW[i], br, &br);
  u12 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? t[i] : d[i];
  return r;
}
#else
// Host (tools/opcount): portable CIOS, same results.
NOINL u12 fp_mul_u12(u12 a, u12 b) {
  BLS_COUNT_MUL();
  uint32_t t[12];
  for (int j = 0; j < 12; j++) t[j] = 0;
  for (int i = 0; i < 12; i++) {
    const uint32_t bi = b[i];
    uint64_t A = (uint64_t)a[0] * bi + t[0];
    const uint32_t m = (uint32_t)A * P_INV32;
    uint64_t C = (uint64_t)m * P_RAW[0] + (uint32_t)A;
    for (int j = 1; j < 12; j++) {
      A = (uint64_t)a[j] * bi + t[j] + (A >> 32);
      C = (uint64_t)m * P_RAW[j] + (uint32_t)A + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[11] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t d[12];
  unsigned br = 0;
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(t[i], P_RAW[i], br, &br);
  u12 r;
  for (int i = 0; i < 12; i++) r[i] = br ? t[i] : d[i];
  return r;
}
#endif

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

DI fp fp_sqr(const fp& a) { return fp_mul(a, a); }

// small-constant multiples via additions
DI fp fp_mul3(const fp& a) { return fp_add(fp_dbl(a), a); }
DI fp fp_mul4(const fp& a) { return fp_dbl(fp_dbl(a)); }
DI fp fp_mul8(const fp& a) { return fp_dbl(fp_mul4(a)); }

DI fp fp_to_mont(const fp& raw) { return fp_mul(raw, fp_load_const(FP_R2)); }

DI fp fp_from_mont(const fp& a) {
  fp one = fp_zero();
  one.l[0] = 1;
  return fp_mul(a, one);
}

// a^e for a public exponent given as little-endian 32-bit words (uniform across the wave ->
// scalar branches, no divergence). Left-to-right 2-bit fixed window: a 4-entry table keeps the
// caller's VGPR budget small (every kernel that inverts inherits this function's register count).
template <int NW>
DI fp fp_pow_words(const fp& a, const uint32_t (&e)[NW]) {
  const fp a2 = fp_mul(a, a);
  const fp a3 = fp_mul(a2, a);
  fp r = fp_one();
  bool started = false;
  for (int w = NW - 1; w >= 0; w--) {
    const uint32_t word = e[w];
    for (int dig = 15; dig >= 0; dig--) {
      const uint32_t d = (word >> (2 * dig)) & 3u;
      if (started) {
        r = fp_mul(r, r);
        r = fp_mul(r, r);
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
NOINL u12 fp_pow_p_minus_3_div_4(u12 a) { return fp_to_u12(fp_pow_words<12>(fp_from_u12(a), EXP_P_MINUS_3_DIV_4)); }

// w = a^((p-3)/4): t = w*a satisfies t^2 = a (a a residue or 0) or t^2 = -a (non-residue), and
// 1/t = w or -w respectively: a square root AND its inverse from one exponentiation.
DI fp fp_pow_sqrt_inv(const fp& a) { return fp_from_u12(fp_pow_p_minus_3_div_4(fp_to_u12(a))); }

DI fp fp_inv(const fp& a) { return fp_from_u12(fp_pow_p_minus_2(fp_to_u12(a))); }  // 0 -> 0

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

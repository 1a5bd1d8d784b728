// Field arithmetic of the wave-cooperative latency engine: one item per wave, an Fp value spread
// over 16 lanes as 25-bit limbs (wv.h lane layout), Montgomery form with R = 2^400.
//
// A register F holds either an Fp2 value (half 0 = c0, half 1 = c1) or a PAIR of independent Fp
// values (one per half: two exponentiations at once, or an Fp scalar duplicated into both halves to
// multiply an Fp2). Stored values are "semi-normalized": limbs in [0, 2^25 + 128] in the even row of
// each half, the odd row zero.
//
// The multiplier is a DOT PRODUCT sum_i a_i b_i of up to 6 Fp2 products with ONE Montgomery
// reduction (every formula of the tower and the curves is written as such sums, so every stored
// value comes out of a reduction, < 1.01 p):
//   product   per term, lane k of a half accumulates column k of the 31-column product: the shifted
//             operand a[k - j] comes from a zero-padded LDS window, limb j of the other operand is
//             an LDS broadcast; 32 v_mad_u64_u32 per Fp2 term into two accumulators (half 0:
//             a0 b0 | a1 b0, half 1: a1 (D - b1) | a0 b1), whose halves one v_permlane32_swap
//             combines into c0 = a0 b0 + a1 (D - b1), c1 = a0 b1 + a1 b0; the negation D - b1 is
//             formed limb-wise against a dominating multiple of p, with no borrows
//   m         carry rounds, then m = x mod R * (-p^-1) mod R: 16 row_shr DPP + 16 MADs, the
//             row-local carries dropping everything at or above R
//   U         U = x + m p: m broadcast limb by limb (row_newbcast) against a per-lane table of p's
//             limbs, three carry rounds; the low row is then 0 or R (one ballot), and the high row
//             moves down with one v_permlane16_swap.
// The host build (-DWV_HOST) carries a bound (units of p) with every F and checks every operation's
// contract: operand bounds of the products, subtrahends below the subtraction constant.
#pragma once
#include "wv.h"
#include "wv_constants.h"
#include "bls_constants.h"
#ifdef WV_HOST
#ifndef BLS_HOST
#define BLS_HOST
#endif
#endif
#include "fp.h"  // shared constants (exponents of the square root and the inverse)

#ifdef WV_HOST
#include <execinfo.h>
#include <stdio.h>
#include <stdlib.h>
#endif

namespace wv {

// Phase trace of the latency kernel (blsv_lat_trace): while profiling has turned the device-global
// flag on (blsv_lat_trace_enable), wave-lane 0 of item 0 (block 0) stamps the device wall clock at the
// marks of wvteam.h verify_team; a no-op in every other block, in production launches and on the host.
constexpr int LAT_TRACE_N = 16;
#ifdef WV_HOST
#define WV_MARK(k) ((void)0)
#else
extern __device__ uint64_t g_lat_trace[LAT_TRACE_N];
extern __device__ uint32_t g_lat_trace_on;
#define WV_MARK(k)                                                                                 \
  do {                                                                                             \
    if (blockIdx.x == 0 && (threadIdx.x & 63u) == 0u && g_lat_trace_on) g_lat_trace[(k)] = wall_clock64(); \
  } while (0)
#endif


constexpr uint32_t M25 = (1u << 25) - 1;
constexpr uint32_t LIMB_MAX = (1u << 25) + 128;  // semi-normalized limb bound
// LDS per product term: window (2 halves x 48 words: 16 zeros, 16 limbs, 16 zeros), the broadcast
// operand (64) and its negation (64); a dot product stages all its terms at once
constexpr int SLOT_WORDS = 224;
constexpr int MAX_TERMS = 6;
// hot per-lane constants (the PC_i table of the U product, DMUL, DSUB0..2, P) copied into LDS by
// wv_init, in table order WC_PC0.., so a product reads them at LDS latency instead of a global load's
constexpr int HOT_FIRST = WC_DSUB0;  // DSUB0, DSUB1, DSUB2, DMUL, PC0..PC15 are consecutive
constexpr int HOT_COUNT = WC_PC15 + 1 - WC_DSUB0;
// the table constants the team rounds read (the cyclotomic square's +-2, the curve formulas' -1, -2, -8,
// one, and p for the canonical forms): also per-wave LDS copies, read at LDS latency instead of a
// global load's in every round
constexpr int HOT2_IDS[] = {WC_ONE2, WC_NEG2, WC_NEG1, WC_POS2, WC_NEG8, WC_ONE_DUP, WC_P_DUP};
constexpr int HOT2_COUNT = sizeof(HOT2_IDS) / sizeof(HOT2_IDS[0]);
constexpr int hot2_index(int id) {
  for (int i = 0; i < HOT2_COUNT; i++)
    if (HOT2_IDS[i] == id) return i;
  return -1;
}
constexpr int LDS_WORDS = SLOT_WORDS * MAX_TERMS + 64 * HOT_COUNT + 64 * HOT2_COUNT;
constexpr int L_HOT = SLOT_WORDS * MAX_TERMS;
constexpr int L_HOT2 = L_HOT + 64 * HOT_COUNT;
constexpr int L_WIN = 0, L_BX = 96, L_BZ = 160;

#ifdef WV_HOST
struct F {
  V x;
  double b;  // bound on the value, units of p
};
[[noreturn]] inline void wv_fail(const char* what, double got, double lim) {
  fprintf(stderr, "wv contract violated: %s (%.17g > %.17g)\n", what, got, lim);
  void* bt[32];
  backtrace_symbols_fd(bt, backtrace(bt, 32), 2);  // host debug builds: -O0 -rdynamic
  abort();
}
#define WV_REQUIRE(v, lim, what)                    \
  do {                                              \
    if (!((v) <= (lim))) wv_fail(what, (v), (lim)); \
  } while (0)
inline F mkF(const V& x, double b) {
  for (int l = 0; l < 64; l++) {
    const bool odd_row = (l / 16) & 1;
    if (odd_row ? x.v[l] != 0 : x.v[l] > LIMB_MAX) {
      fprintf(stderr, "wv value form violated at lane %d: %u\n", l, x.v[l]);
      abort();
    }
  }
  return {x, b};
}
inline double bnd(const F& a) { return a.b; }
// the host runs each wave of a workgroup as a thread (wteam.h): per-wave LDS and op counters
constexpr int HOST_MAX_WAVES = 8;
extern uint32_t g_host_lds[HOST_MAX_WAVES][LDS_WORDS];
extern thread_local int g_host_wave;
inline uint32_t* wave_lds() { return g_host_lds[g_host_wave]; }
// host op counts (tools/wvtest opcount): dot1..dot6, mulp, sqr2, norm_dup, gcd inversions
enum { OPC_DOT1 = 0, OPC_MULP = 6, OPC_SQR2, OPC_NORM, OPC_GCD, OPC_N };
extern thread_local unsigned long long g_wv_ops[OPC_N];
#define WV_COUNT(k) (++g_wv_ops[k])
#else
struct F {
  V x;
};
#define WV_REQUIRE(v, lim, what) ((void)0)
#define WV_COUNT(k) ((void)0)
WVI F mkF(V x, double) { return {x}; }
WVI double bnd(const F&) { return 0.0; }
// each wave of a workgroup owns LDS_WORDS words
#ifndef WV_WAVES
#define WV_WAVES 1
#endif
static __shared__ uint32_t g_wv_lds[WV_WAVES * LDS_WORDS];
WVI uint32_t* wave_lds() { return g_wv_lds + (threadIdx.x >> 6) * LDS_WORDS; }
#endif

// ------------------------------------------------------------------ lane geometry and constants
WVI M in_half0() { return lane_id() < 32u; }
WVI V cword(int id) {
  const int h = hot2_index(id);  // a compile-time constant at every call with a literal id
  if (h >= 0) return lds_ld(wave_lds() + L_HOT2 + h * 64, lane_id());
  return gld(WV_CONST_TABLE + id * 64, lane_id());
}
// a hot constant (HOT_FIRST <= id < HOT_FIRST + HOT_COUNT) from the wave's LDS copy
WVI V hword(int id) { return lds_ld(wave_lds() + L_HOT + (id - HOT_FIRST) * 64, lane_id()); }
WVI F cst(int id) { return mkF(cword(id), 1.0); }  // every table constant used as a value is < p

// the calling wave zeroes the padding of its product windows (kernel prologue)
WVI void wv_init() {
  uint32_t* lds = wave_lds();
  const V l = lane_id();
  const V off = (l >> 5) * 48u + (l & 15u);  // words h*48 + 0..15 (odd-row lanes repeat them)
  for (int s = 0; s < MAX_TERMS; s++) lds_st(lds + s * SLOT_WORDS, off, vsplat(0));
  for (int c = 0; c < HOT_COUNT; c++) lds_st(lds + L_HOT + c * 64, l, cword(HOT_FIRST + c));
  for (int c = 0; c < HOT2_COUNT; c++) lds_st(lds + L_HOT2 + c * 64, l, gld(WV_CONST_TABLE + HOT2_IDS[c] * 64, l));
}

// LDS hand-off: a wave's ds instructions execute in order; this keeps the compiler from moving a
// load of other lanes' words above the stores that produce them (and stores above older loads)
WVI void wsync() {
#ifndef WV_HOST
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#endif
}

// ------------------------------------------------------------------ carries
// one carry round: limb k keeps its low 25 bits and takes limb k-1's carry. A stored value is far
// below 2^400, so no carry ever leaves its even row (its non-negative top limb is <= value / 2^375).
WVI V norm1(V x) { return (x & M25) + wave_shr1(x >> 25); }

// ------------------------------------------------------------------ Montgomery reduction
// T: 64-bit column sums (< 2^58) of the products of each half, columns 0..30 in lanes 0..30.
// Returns the value-form (T + m p) / R, m = -T p^-1 mod R.
WVI V mont_reduce(V64 T) {
  // first carry round in 64 bits (the carry may exceed 32 bits), then 32-bit rounds
  const V64 c = T >> 25;
  const V64 x64 = add64(widen(lo32(T) & M25), join64(wave_shr1(lo32(c)), wave_shr1(hi32(c))));  // < 2^34
  // < 2^25 + 2^9: enough for both products below (16 x (2^25 + 2^9) 2^25 < 2^55 in m's columns, and
  // x only seeds U's 64-bit accumulator)
  const V x = (lo32(x64) & M25) + wave_shr1(shr64_lo(x64, 25));
  // m = x * N' mod R
  V64 ma[4] = {vsplat64(0), vsplat64(0), vsplat64(0), vsplat64(0)};
  sfor<16>([&](auto J) { ma[J & 3] = mad(row_shr<J>(x), NP25[J], ma[J & 3]); });
  const V64 mm = add64(add64(ma[0], ma[1]), add64(ma[2], ma[3]));  // columns < 2^55
  V m = (lo32(mm) & M25) + row_shr<1>(shr64_lo(mm, 25));  // row-local: carries past R drop
  m = (m & M25) + row_shr<1>(m >> 25);                    // m limbs < 2^25 + 2^5
  const V md = pl16_swap(m, m).a;                          // m in both rows of its half
  V64 ua[4] = {widen(x), vsplat64(0), vsplat64(0), vsplat64(0)};
  sfor<16>([&](auto I) { ua[I & 3] = mad(row_bcast<I>(md), hword(WC_PC0 + I), ua[I & 3]); });
  const V64 u = add64(add64(ua[0], ua[1]), add64(ua[2], ua[3]));  // < 2^56
  V y = (lo32(u) & M25) + wave_shr1(shr64_lo(u, 25));  // < 2^25 + 2^31
  y = norm1(y);  // <= 2^25 + 63: semi-normalized even after the carry below
  // the even row now holds 0 or exactly R: carry one into the odd row's first limb when nonzero. Limbs
  // up to 2^25 + 63 below the top one sum to less than 2^400, so R has a nonzero top limb (lane 15 /
  // 47) and 0 does not: lanes 16 and 48 test their wave neighbour, no ballot
  const V l = lane_id();
  y = y + sel(((l & 0x1Fu) == 16u) & (wave_shr1(y) != 0u), vsplat(1), vsplat(0));
  return pl16_swap(y, vsplat(0)).b;  // odd rows -> even rows, odd rows zero
}

// ------------------------------------------------------------------ product terms
WVI V win_off() {
  const V l = lane_id();
  return L_WIN + (l >> 5) * 48u + 16u + (l & 31u);
}
// stage term s: window <- a, broadcast <- b (an Fp2 term also stores D - b, dot_body)
WVI void stage_term(int s, V a, V b) {
  uint32_t* lds = wave_lds() + s * SLOT_WORDS;
  const V l = lane_id();
  lds_st(lds, win_off(), a);
  lds_st(lds, L_BX + l, b);
}
// Fp2 term s into the accumulators (two chains per component): half 0 -> a0 b0 | a0 b1,
// half 1 -> a1 (D - b1) | a1 b0
WVI void acc_fp2(int s, V64 (&s1)[2], V64 (&s2)[2]) {
  const uint32_t* lds = wave_lds() + s * SLOT_WORDS;
  const M h0 = in_half0();
  const V win = win_off();
  const V src1 = sel(h0, vsplat(L_BX), vsplat(L_BZ + 32));
  const V src2 = sel(h0, vsplat(L_BX + 32), vsplat(L_BX));
  sfor<16>([&](auto J) {
    const V w = lds_ld(lds, win - (uint32_t)J);
    s1[J & 1] = mad(w, lds_ld(lds, src1 + (uint32_t)J), s1[J & 1]);
    s2[J & 1] = mad(w, lds_ld(lds, src2 + (uint32_t)J), s2[J & 1]);
  });
}
// pair term s into the accumulators: half h -> a_h b_h
WVI void acc_pair(int s, V64 (&acc)[4]) {
  const uint32_t* lds = wave_lds() + s * SLOT_WORDS;
  const V win = win_off();
  const V src = L_BX + (lane_id() >> 5) * 32u;
  sfor<16>([&](auto J) {
    acc[J & 3] = mad(lds_ld(lds, win - (uint32_t)J), lds_ld(lds, src + (uint32_t)J), acc[J & 3]);
  });
}
WVI V64 sum4(const V64 (&a)[4]) { return add64(add64(a[0], a[1]), add64(a[2], a[3])); }
// [x.h0 + x.h1 | y.h0 + y.h1] of two 64-bit accumulators
WVI V64 fold_halves(V64 x, V64 y) {
  const VP lo = pl32_swap(lo32(x), lo32(y)), hi = pl32_swap(hi32(x), hi32(y));
  return add64(join64(lo.a, hi.a), join64(lo.b, hi.b));
}

template <int N>
WVI V dot_body(const V (&a)[N], const V (&b)[N]) {
  static_assert(N >= 1 && N <= MAX_TERMS, "dot terms");
  WV_COUNT(OPC_DOT1 + N - 1);
  // D read once and first: the windows and broadcasts are stored while it is in flight, the negations
  // after it returns (one LDS round trip instead of one per term)
  const V dm = hword(WC_DMUL);
#pragma unroll
  for (int i = 0; i < N; i++) stage_term(i, a[i], b[i]);
#pragma unroll
  for (int i = 0; i < N; i++) lds_st(wave_lds() + i * SLOT_WORDS, L_BZ + lane_id(), dm - b[i]);
  wsync();
  V64 s1[2] = {vsplat64(0), vsplat64(0)}, s2[2] = {vsplat64(0), vsplat64(0)};
#pragma unroll
  for (int i = 0; i < N; i++) acc_fp2(i, s1, s2);
  wsync();
  return mont_reduce(fold_halves(add64(s1[0], s1[1]), add64(s2[0], s2[1])));
}

#ifdef WV_HOST
#define WV_NOINL inline
#else
#define WV_NOINL static __device__ __noinline__
#endif

// one body per term count per code object (instruction-cache resident); V arguments in VGPRs
WV_NOINL V dot1_v(V a0, V b0) {
  const V a[1] = {a0}, b[1] = {b0};
  return dot_body<1>(a, b);
}
WV_NOINL V dot2_v(V a0, V b0, V a1, V b1) {
  const V a[2] = {a0, a1}, b[2] = {b0, b1};
  return dot_body<2>(a, b);
}
WV_NOINL V dot3_v(V a0, V b0, V a1, V b1, V a2, V b2) {
  const V a[3] = {a0, a1, a2}, b[3] = {b0, b1, b2};
  return dot_body<3>(a, b);
}
WV_NOINL V dot4_v(V a0, V b0, V a1, V b1, V a2, V b2, V a3, V b3) {
  const V a[4] = {a0, a1, a2, a3}, b[4] = {b0, b1, b2, b3};
  return dot_body<4>(a, b);
}
WV_NOINL V dot5_v(V a0, V b0, V a1, V b1, V a2, V b2, V a3, V b3, V a4, V b4) {
  const V a[5] = {a0, a1, a2, a3, a4}, b[5] = {b0, b1, b2, b3, b4};
  return dot_body<5>(a, b);
}
WV_NOINL V dot6_v(V a0, V b0, V a1, V b1, V a2, V b2, V a3, V b3, V a4, V b4, V a5, V b5) {
  const V a[6] = {a0, a1, a2, a3, a4, a5}, b[6] = {b0, b1, b2, b3, b4, b5};
  return dot_body<6>(a, b);
}
// pair product [a0 b0 | a1 b1]
WVI V mulp_body(V a, V b) {
  stage_term(0, a, b);
  wsync();
  V64 s[4] = {vsplat64(0), vsplat64(0), vsplat64(0), vsplat64(0)};
  acc_pair(0, s);
  wsync();
  return mont_reduce(sum4(s));
}
WV_NOINL V mulp_v(V a, V b) {
  WV_COUNT(OPC_MULP);
  return mulp_body(a, b);
}
// Fp2 square [(a0 + a1)(a0 + D - a1) | (2 a0) a1] as one pair product
WV_NOINL V sqr2_v(V a) {
  WV_COUNT(OPC_SQR2);
  const M h0 = in_half0();
  const VP d = pl32_swap(a, a);  // .a = [a0 | a0], .b = [a1 | a1]
  const V u = d.a + sel(h0, d.b, d.a);
  const V v = norm1(sel(h0, d.a + hword(WC_DMUL) - d.b, d.b));
  stage_term(0, u, v);
  wsync();
  V64 s[4] = {vsplat64(0), vsplat64(0), vsplat64(0), vsplat64(0)};
  acc_pair(0, s);
  wsync();
  return mont_reduce(sum4(s));
}
// Fp2 norm a0^2 + a1^2 in both halves: one pair product, halves summed, one reduction
WV_NOINL V norm_dup_v(V a) {
  WV_COUNT(OPC_NORM);
  stage_term(0, a, a);
  wsync();
  V64 s4[4] = {vsplat64(0), vsplat64(0), vsplat64(0), vsplat64(0)};
  acc_pair(0, s4);
  wsync();
  const V64 s = sum4(s4);
  return mont_reduce(fold_halves(s, s));
}

constexpr double OPND_MAX = 128.0;    // product operand bound (DMUL covers b1 < 128 p)
constexpr double RED_SLACK = 1.0001;  // (T + m p) / R < T / R + 1.0001 p

WVI double term_bound(const F& a, const F& b) {
  WV_REQUIRE(bnd(a), OPND_MAX, "product operand a");
  WV_REQUIRE(bnd(b), DMUL_BMAX, "product operand b");
  return bnd(a) * (bnd(b) + DMUL_M);
}
// sum_i a_i b_i (Fp2), one reduction
WVI F dot(const F& a0, const F& b0) {
  return mkF(dot1_v(a0.x, b0.x), term_bound(a0, b0) * P_OVER_R + RED_SLACK);
}
WVI F dot(const F& a0, const F& b0, const F& a1, const F& b1) {
  return mkF(dot2_v(a0.x, b0.x, a1.x, b1.x), (term_bound(a0, b0) + term_bound(a1, b1)) * P_OVER_R + RED_SLACK);
}
WVI F dot(const F& a0, const F& b0, const F& a1, const F& b1, const F& a2, const F& b2) {
  return mkF(dot3_v(a0.x, b0.x, a1.x, b1.x, a2.x, b2.x),
             (term_bound(a0, b0) + term_bound(a1, b1) + term_bound(a2, b2)) * P_OVER_R + RED_SLACK);
}
WVI F dot(const F& a0, const F& b0, const F& a1, const F& b1, const F& a2, const F& b2, const F& a3, const F& b3) {
  return mkF(dot4_v(a0.x, b0.x, a1.x, b1.x, a2.x, b2.x, a3.x, b3.x),
             (term_bound(a0, b0) + term_bound(a1, b1) + term_bound(a2, b2) + term_bound(a3, b3)) * P_OVER_R +
                 RED_SLACK);
}
WVI F dot(const F& a0, const F& b0, const F& a1, const F& b1, const F& a2, const F& b2, const F& a3, const F& b3,
          const F& a4, const F& b4) {
  return mkF(dot5_v(a0.x, b0.x, a1.x, b1.x, a2.x, b2.x, a3.x, b3.x, a4.x, b4.x),
             (term_bound(a0, b0) + term_bound(a1, b1) + term_bound(a2, b2) + term_bound(a3, b3) +
              term_bound(a4, b4)) * P_OVER_R + RED_SLACK);
}
WVI F dot(const F& a0, const F& b0, const F& a1, const F& b1, const F& a2, const F& b2, const F& a3, const F& b3,
          const F& a4, const F& b4, const F& a5, const F& b5) {
  return mkF(dot6_v(a0.x, b0.x, a1.x, b1.x, a2.x, b2.x, a3.x, b3.x, a4.x, b4.x, a5.x, b5.x),
             (term_bound(a0, b0) + term_bound(a1, b1) + term_bound(a2, b2) + term_bound(a3, b3) +
              term_bound(a4, b4) + term_bound(a5, b5)) * P_OVER_R + RED_SLACK);
}
WVI F mul2(const F& a, const F& b) { return dot(a, b); }
WVI F mulp(const F& a, const F& b) {
  WV_REQUIRE(bnd(a), OPND_MAX, "mulp a");
  WV_REQUIRE(bnd(b), OPND_MAX, "mulp b");
  return mkF(mulp_v(a.x, b.x), bnd(a) * bnd(b) * P_OVER_R + RED_SLACK);
}
// (a pair square with each cross product once -- 9 products per lane against 16, lane-dependent LDS
// addresses -- measured 0.75 us against the general product's 0.69, profiles/r04zb_wvbench.json)
WVI F sqrp(const F& a) { return mulp(a, a); }
// the same square with its body inlined at the call site: for the long squaring chains (wvteam.h
// ring_pow_produce), where a call's entry wait for every outstanding LDS operation (the ring's stores
// and posts) and its argument moves sit on the critical path 378 times per exponentiation
WVI F sqrp_inl(const F& a) {
  WV_REQUIRE(bnd(a), OPND_MAX, "sqrp a");
  WV_COUNT(OPC_MULP);
  return mkF(mulp_body(a.x, a.x), bnd(a) * bnd(a) * P_OVER_R + RED_SLACK);
}
WVI F sqr2(const F& a) {
  WV_REQUIRE(bnd(a), DMUL_BMAX, "sqr2");
  return mkF(sqr2_v(a.x), 2 * bnd(a) * (bnd(a) + DMUL_M) * P_OVER_R + RED_SLACK);
}
WVI F norm_dup(const F& a) {
  WV_REQUIRE(bnd(a), OPND_MAX, "norm_dup");
  return mkF(norm_dup_v(a.x), 2 * bnd(a) * bnd(a) * P_OVER_R + RED_SLACK);
}

// ------------------------------------------------------------------ additive
WVI F add(const F& a, const F& b) { return mkF(norm1(a.x + b.x), bnd(a) + bnd(b)); }
WVI F dbl(const F& a) { return add(a, a); }
// a - b + DSUB_M[L] p, limb-wise with no borrows (b's limbs are below the constant's)
template <int L = 0>
WVI F sub(const F& a, const F& b) {
  WV_REQUIRE(bnd(b), DSUB_BMAX[L], "sub subtrahend");
  return mkF(norm1(a.x + hword(WC_DSUB0 + L) - b.x), bnd(a) + DSUB_M[L]);
}
template <int L = 0>
WVI F neg(const F& a) {
  WV_REQUIRE(bnd(a), DSUB_BMAX[L], "neg");
  return mkF(norm1(hword(WC_DSUB0 + L) - a.x), DSUB_M[L]);
}
template <uint32_t C>
WVI F mul_small(const F& a) {
  static_assert(C <= 64, "one carry round keeps limbs semi-normalized up to x64");
  return mkF(norm1(a.x * C), bnd(a) * C);
}
// a / 2 mod p: (a + (a odd ? p : 0)) >> 1, the parity being limb 0's (every other limb is weighted
// by an even power of two), per half
WVI F half(const F& a) {
  const V odd = row_bcast<0>(a.x) & 1u;
  const V t = a.x + sel(odd != 0u, cword(WC_P_DUP), vsplat(0));
  const V y = (t >> 1) + ((row_shl<1>(t) & 1u) << 24);
  return mkF(norm1(y), (bnd(a) + 1.0) / 2);
}
WVI F zero() { return mkF(vsplat(0), 0.0); }
WVI F select(bool c, const F& a, const F& b) {
#ifdef WV_HOST
  return mkF(c ? a.x : b.x, a.b > b.b ? a.b : b.b);
#else
  return {c ? a.x : b.x};
#endif
}
// per half: c_h = take_h ? a_h : b_h (bit h of `take`)
WVI F select_halves(uint32_t take, const F& a, const F& b) {
  const V t = sel(in_half0(), vsplat(take & 1u), vsplat((take >> 1) & 1u));
  return mkF(sel(t != 0u, a.x, b.x), bnd(a) > bnd(b) ? bnd(a) : bnd(b));
}

// ------------------------------------------------------------------ Fp2 structure
WVI F swap_halves(const F& a) {  // [a1 | a0]
  const VP d = pl32_swap(a.x, a.x);
  return mkF(sel(in_half0(), d.b, d.a), bnd(a));
}
WVI F dup0(const F& a) { return mkF(pl32_swap(a.x, a.x).a, bnd(a)); }  // [a0 | a0]
WVI F dup1(const F& a) { return mkF(pl32_swap(a.x, a.x).b, bnd(a)); }  // [a1 | a1]
// the same two halves as an Fp2 with c1 = 0: [a0 | 0]
WVI F lo_only(const F& a) { return mkF(sel(in_half0(), a.x, vsplat(0)), bnd(a)); }
template <int L = 0>
WVI F conj(const F& a) {  // [a0 | -a1]
  WV_REQUIRE(bnd(a), DSUB_BMAX[L], "conj");
  const V n = norm1(hword(WC_DSUB0 + L) - a.x);
  return mkF(sel(in_half0(), a.x, n), bnd(a) > DSUB_M[L] ? bnd(a) : DSUB_M[L]);
}
template <int L = 0>
WVI F mul_xi(const F& a) {  // (1 + i) a = (a0 - a1) + (a0 + a1) i
  WV_REQUIRE(bnd(a), DSUB_BMAX[L], "mul_xi");
  const F s = swap_halves(a);
  const V d = sel(in_half0(), hword(WC_DSUB0 + L) - s.x, s.x);
  return mkF(norm1(a.x + d), bnd(a) + (bnd(a) > DSUB_M[L] ? bnd(a) : DSUB_M[L]));
}

// ------------------------------------------------------------------ canonical forms, comparisons
// carry-in mask of an exact carry chain over 16 limbs: generate g (limb == 2^25, or a borrow source),
// propagate pm (limb == 2^25 - 1, or equal limbs); c_0 = 0, c_{k+1} = g_k | (pm_k & c_k). The
// masks are wave-uniform (ballots), so this is scalar work.
// As one binary addition (g and pm are disjoint): with x = g | pm, y = g the carries of x + y are
// generated where both bits are set (g) and propagated where exactly one is (pm), so the carry-in bits
// are (x + y) ^ x ^ y = ((g | pm) + g) ^ pm -- three scalar operations instead of a 16-step chain.
WVI uint32_t carry_in_mask(uint32_t g, uint32_t pm) { return (((g | pm) + g) ^ pm) & 0xFFFFu; }
WVI V mask_to_lanes(uint32_t m_half0, uint32_t m_half1) {
  const V l = lane_id();
  const V bits = sel(l < 32u, vsplat(m_half0), vsplat(m_half1));
  return sel((l & 16u) == 0u, (bits >> (l & 15u)) & 1u, vsplat(0));
}
WVI uint32_t half_bits(uint64_t b, int h) { return (uint32_t)(b >> (32 * h)) & 0xFFFFu; }
// fully normalized limbs (each < 2^25) of a value-form x
WVI V strict(V x) {
  x = norm1(norm1(x));  // limbs in [0, 2^25]
  const M ev = (lane_id() & 16u) == 0u;
  const uint64_t g = ballot(ev & (x == (1u << 25))), pm = ballot(ev & (x == M25));
  const uint32_t c0 = carry_in_mask(half_bits(g, 0), half_bits(pm, 0));
  const uint32_t c1 = carry_in_mask(half_bits(g, 1), half_bits(pm, 1));
  return (x + mask_to_lanes(c0, c1)) & M25;
}
WVI int msb16(uint32_t m) { return m ? 31 - __builtin_clz(m) : -1; }
// per half: bit h set when strict x_h >= strict c_h
WVI uint32_t ge_halves(V x, V c) {
  const M ev = (lane_id() & 16u) == 0u;
  const uint64_t gt = ballot(ev & (x > c)), lt = ballot(ev & (x < c));
  uint32_t r = 0;
  for (int h = 0; h < 2; h++) r |= (uint32_t)(msb16(half_bits(gt, h)) >= msb16(half_bits(lt, h))) << h;
  return r;  // equal: both msb -1 -> ge
}
// per half where bit h of `which` is set: x - c (strict, x >= c), exact borrows
WVI V sub_halves(V x, V c, uint32_t which) {
  const M ev = (lane_id() & 16u) == 0u;
  const uint64_t gb = ballot(ev & (x < c)), pb = ballot(ev & (x == c));
  const uint32_t b0 = carry_in_mask(half_bits(gb, 0), half_bits(pb, 0));
  const uint32_t b1 = carry_in_mask(half_bits(gb, 1), half_bits(pb, 1));
  const V d = (x - c - mask_to_lanes(b0, b1)) & M25;
  const V t = sel(in_half0(), vsplat(which & 1u), vsplat((which >> 1) & 1u));
  return sel(t != 0u, d, x);
}
// canonical residue (strict limbs, value in [0, p)) of a * y R^-1 for a table constant y: y = ONE_DUP
// (R mod p) gives a mod p itself, y = RAW_ONE_DUP the raw (non-Montgomery) value of a
WVI V canon_times(const F& a, int cid) {
  const V r = strict(mulp(a, cst(cid)).x);  // < 1.0002 p: at most one subtraction of p
  const V p = cword(WC_P_DUP);
  return sub_halves(r, p, ge_halves(r, p));
}
// per half: bit h set when a_h == 0 mod p
WVI uint32_t zero_halves(const F& a) {
  const V c = canon_times(a, WC_ONE_DUP);
  const uint64_t nz = ballot(((lane_id() & 16u) == 0u) & (c != 0u));
  return (half_bits(nz, 0) == 0 ? 1u : 0u) | (half_bits(nz, 1) == 0 ? 2u : 0u);
}
WVI bool is_zero2(const F& a) { return zero_halves(a) == 3u; }
template <int L = 1>
WVI bool eq2(const F& a, const F& b) { return is_zero2(sub<L>(a, b)); }
// raw canonical value (out of Montgomery form) of each half, strict limbs
WVI V raw_canon(const F& a) { return canon_times(a, WC_RAW_ONE_DUP); }
WVI uint32_t lane0_of_half(V x, int h) { return lane_val(x, 32 * h); }

// ------------------------------------------------------------------ exponentiation (pair)
// a^e per half, e = public exponent as NW little-endian 32-bit words (wave-uniform): 4-bit fixed
// window, table a^0..a^15 in registers, digits from the top. (A 5-bit sliding window over odd powers
// does 457 products for (p-3)/4 against 481 here but measured 7% slower: r04u, its runtime windows
// and table index)
template <int NW>
WVI F pow_pair(const F& a, const uint32_t (&e)[NW]) {
  F t[16];
  t[0] = cst(WC_ONE_DUP);
  t[1] = a;
  for (int i = 2; i < 16; i++) t[i] = mulp(t[i - 1], a);
  F r = t[0];
  bool started = false;
#pragma unroll 1
  for (int d = NW * 8 - 1; d >= 0; d--) {
    const uint32_t dig = (e[d >> 3] >> (4 * (d & 7))) & 15u;
    if (started) {
      r = sqrp(r);
      r = sqrp(r);
      r = sqrp(r);
      r = sqrp(r);
    }
    if (dig) {
      r = started ? mulp(r, t[dig]) : t[dig];
      started = true;
    }
  }
  return r;
}
WVI F inv_pair_pow(const F& a) { return pow_pair<12>(a, bls::EXP_P_MINUS_2); }  // 0 -> 0
WVI F pow_pm3d4(const F& a) { return pow_pair<12>(a, bls::EXP_P_MINUS_3_DIV_4); }  // sqrt and its inverse
// strict limbs of half h -> 12 little-endian 32-bit words (wave-uniform; wrecover.h's compression)
WVI void limbs_to_words(V strict_limbs, int h, uint32_t (&w)[12]) {
  uint32_t limb[16];
  for (int k = 0; k < 16; k++) limb[k] = lane_val(strict_limbs, 32 * h + k);
  for (int j = 0; j < 12; j++) {
    const int b = 32 * j, k = b / 25, s = b % 25;
    uint64_t v = (uint64_t)limb[k] >> s;
    if (k + 1 < 16) v |= (uint64_t)limb[k + 1] << (25 - s);
    if (k + 2 < 16) v |= (uint64_t)limb[k + 2] << (50 - s);
    w[j] = (uint32_t)v;
  }
}

// ------------------------------------------------------------------ inversion by a lane-parallel GCD
// The same binary GCD as fp.h fp_inv_bingcd_raw (Pornin: divsteps driven by 64-bit approximations of
// a and b, the accumulated 2x2 matrix then applied to the full-width values), restated for the lanes
// so that only the divsteps stay scalar: the four integers of the extended GCD -- a, b and their
// cofactors u, v with a = u y, b = v y (mod p) -- are the four DPP rows of ONE register, 16 signed
// limbs of 25 bits each. Each of the 31 iterations runs 25 divsteps on wave-uniform scalars, then
//   all four rows  t = own * c_own + partner * c_partner   (v_mad_i64_i32; partner = the other row
//                  of the pair via v_permlane16_swap; (a, b) and (u, v) take the same matrix)
//   rows u, v      t += m p with m = t_0 (-p^-1) mod 2^25, so every row is divisible by 2^25
//   all rows       one limb down (exact division by 2^25), three carry rounds
//   rows a, b      exact carries (ballots), and a negative result negated together with its cofactor
// 31 x 25 = 775 >= 761 divsteps; b ends at 1 and v = y^-1 (mod p), |v| < 32 p. The input y is the
// canonical 400-form value A 2^400, so A^-1 2^400 = v 2^800 = mulp(v, 2^1200).
constexpr int GCD_ITERS = 31, GCD_STEPS = 25;

WVI V64 sel64(M c, V64 a, V64 b) { return join64(sel(c, lo32(a), lo32(b)), sel(c, hi32(a), hi32(b))); }
template <int j>
WVI V64 row_shl64(V64 x) {
  return join64(row_shl<j>(lo32(x)), row_shl<j>(hi32(x)));
}
template <int j>
WVI V64 row_shr64(V64 x) {
  return join64(row_shr<j>(lo32(x)), row_shr<j>(hi32(x)));
}
// exact limbs of the rows in `rows` (bit r = DPP row r): lanes 0..14 from [-1, 2^25] to [0, 2^25),
// the top lane (15) signed and unbounded -- one carry pass, then one borrow pass
WVI V gcd_exact(V x, uint32_t rows) {
  const V l = lane_id(), k = l & 15u, row = l >> 4;
  const M low = (k != 15u) & (((vsplat(rows) >> row) & 1u) != 0u);
  auto pass = [&](M gen, M prop) {
    const uint64_t g = ballot(low & gen), pm = ballot(low & prop);
    V in = vsplat(0);
    for (int r = 0; r < 4; r++) {
      if (!((rows >> r) & 1u)) continue;
      const uint32_t c = carry_in_mask((uint32_t)(g >> (16 * r)) & 0xFFFFu, (uint32_t)(pm >> (16 * r)) & 0xFFFFu);
      in = sel(row == (uint32_t)r, (vsplat(c) >> k) & 1u, in);
    }
    return in;
  };
  const V cin = pass(x == (1u << 25), x == M25);
  x = x + cin;
  x = sel(low & (x >= (1u << 25)) & (x < 0x80000000u), x - (1u << 25), x);  // 2^25, 2^25 + 1 (not -1)
  const V bin = pass(x == 0xFFFFFFFFu, x == 0u);
  x = x - bin;
  return sel(low & (x >= 0x80000000u), x + (1u << 25), x);
}
// three carry rounds of signed 64-bit limbs (the top lane keeps its carries); limbs of |t| < 2^52 end
// in [-1, 2^25] as 32-bit two's complement
WVI V gcd_carry(V64 t) {
  const M topl = (lane_id() & 15u) == 15u;
  for (int r = 0; r < 3; r++) {
    const V64 c = sar64(t, 25);
    const V64 low = sel64(topl, t, join64(lo32(t) & M25, vsplat(0)));
    t = add64(low, row_shr64<1>(sel64(topl, vsplat64(0), c)));
  }
  return lo32(t);
}
// [a0^-1 | a0^-1] (0 -> 0); returns false (and leaves r alone) if the divsteps did not reach b = 1
WVI bool inv_gcd_lanes(const F& a, F& r) {
  WV_COUNT(OPC_GCD);
  const V l = lane_id(), k = l & 15u, row = l >> 4;
  const M ev = (row & 1u) == 0u;
  const V c = canon_times(a, WC_ONE_DUP);
  const V P = cword(WC_P_DUP), Pall = pl16_swap(P, P).a;  // p in every row
  V x = sel(row == 0u, c, sel(row == 1u, Pall, sel((row == 2u) & (k == 0u), vsplat(1), vsplat(0))));
  const uint32_t np0 = NP25[0];
#pragma unroll 1
  for (int it = 0; it < GCD_ITERS; it++) {
    // 64-bit approximations of a (row 0) and b (row 1), fp.h's: low 31 bits, and the 33 bits below
    // the top of the longer one
    const uint64_t nzb = ballot((l < 32u) & (x != 0u));
    const uint32_t nzr = ((uint32_t)nzb | (uint32_t)(nzb >> 16)) & 0xFFFFu;
    const int top = msb16(nzr);
    int n = 64;
    if (top >= 0) {
      const uint32_t tv = lane_val(x, top) | lane_val(x, 16 + top);
      const int nb = 25 * top + 32 - __builtin_clz(tv);
      n = nb > 64 ? nb : 64;
    }
    const int s = n - 33, i0 = s / 25, o = s % 25;
    auto approx = [&](int base) -> uint64_t {
      const uint64_t L0 = lane_val(x, base + i0), L1 = i0 + 1 < 16 ? lane_val(x, base + i0 + 1) : 0u,
                     L2 = i0 + 2 < 16 ? lane_val(x, base + i0 + 2) : 0u;
      const uint64_t hi = ((L0 >> o) | (L1 << (25 - o)) | (L2 << (50 - o))) & ((1ull << 33) - 1);
      const uint64_t lo = ((uint64_t)lane_val(x, base) | ((uint64_t)lane_val(x, base + 1) << 25)) & 0x7fffffffull;
      return lo | (hi << 31);
    };
    uint64_t A = approx(0), B = approx(16);
    int32_t f0 = 1, g0 = 0, f1 = 0, g1 = 1;
    for (int j = 0; j < GCD_STEPS; j++) {
      const bool odd = (A & 1u) != 0, sw = odd & (A < B);  // (32-bit halves compared on the scalar
                                                             // unit measured 7% slower than this)
      const uint64_t A2 = sw ? B : A, B2 = sw ? A : B;
      const int32_t F0 = sw ? f1 : f0, G0 = sw ? g1 : g0, F1 = sw ? f0 : f1, G1 = sw ? g0 : g1;
      A = odd ? A2 - B2 : A2;
      f0 = odd ? F0 - F1 : F0;
      g0 = odd ? G0 - G1 : G0;
      B = B2;
      f1 = F1 * 2;
      g1 = G1 * 2;
      A >>= 1;
    }
    // rows (a, u) take (f0, g0), rows (b, v) take (f1, g1), each against its pair partner
    const VP swp = pl16_swap(x, x);
    const V oth = sel(ev, swp.b, swp.a);
    const V cown = sel(ev, vsplat((uint32_t)f0), vsplat((uint32_t)g1));
    const V coth = sel(ev, vsplat((uint32_t)g0), vsplat((uint32_t)f1));
    V64 t = smad(x, cown, smad(oth, coth, vsplat64(0)));
    const uint32_t mu = (lane_val(lo32(t), 32) * np0) & M25, mv = (lane_val(lo32(t), 48) * np0) & M25;
    t = add64(t, mad(sel(row == 2u, vsplat(mu), sel(row == 3u, vsplat(mv), vsplat(0))), Pall, vsplat64(0)));
    // exact division by 2^25: limb 0 (a multiple of 2^25) carries into limb 1, then one limb down
    const V64 q = sar64(t, 25);
    t = add64(row_shl64<1>(t), sel64(k == 0u, q, vsplat64(0)));
    x = gcd_exact(gcd_carry(t), 0x3u);
    const bool na = (int32_t)lane_val(x, 15) < 0, nb = (int32_t)lane_val(x, 31) < 0;
    if (na | nb) {
      const V sa = vsplat(na ? 1u : 0u), sb = vsplat(nb ? 1u : 0u);
      const M neg_ab = ((row == 0u) & (sa != 0u)) | ((row == 1u) & (sb != 0u));
      const M neg_uv = ((row == 2u) & (sa != 0u)) | ((row == 3u) & (sb != 0u));
      // -X = ones' complement + 1 on an exact row; a redundant cofactor row just negates its limbs
      x = sel(neg_ab, sel(k != 15u, M25 - x, 0xFFFFFFFFu - x) + sel(k == 0u, vsplat(1), vsplat(0)), sel(neg_uv, 0u - x, x));
      x = gcd_exact(x, 0x3u);
    }
  }
  const uint64_t bnz = ballot((row == 1u) & (x != sel(k == 0u, vsplat(1), vsplat(0))));
  const uint64_t ynz = ballot((row == 0u) & (c != 0u));
  const bool y_zero = (ynz & 0xFFFFull) == 0;
  if (bnz != 0 && !y_zero) return false;
  // v (row 3) into both halves' even rows, + 32 p (non-negative), exact limbs
  const V h1 = pl32_swap(x, x).b;
  V v = sel(ev, pl16_swap(h1, h1).b, vsplat(0));
  v = sel(ev, v + (P << 5), vsplat(0));
  v = gcd_carry(join64(v, sel(sar32(v, 31) != 0u, vsplat(0xFFFFFFFFu), vsplat(0))));
  v = gcd_exact(v, 0x5u);
  if (y_zero) v = vsplat(0);
  r = mulp(mkF(v, 64.0), cst(WC_C1200_DUP));
  return true;
}

// [a0^-1 | a0^-1] (0 -> 0): the lane GCD, or the exponentiation if its divsteps did not reach b = 1
// (no input of the host fuzz, tests/test_wv_host.py, takes that branch)
WVI F inv_dup(const F& a) {
  F r;
  if (inv_gcd_lanes(a, r)) return r;
  return inv_pair_pow(dup0(a));
}

// per half: a_h^-1 for two NONZERO halves, one GCD (Montgomery's trick): 1 / (a0 a1) times the
// other half
WVI F inv_pair_nz(const F& a) {
  const F other = swap_halves(a);
  const F ni = inv_dup(mulp(a, other));
  return mulp(ni, other);
}

WVI F inv2(const F& a) {  // Fp2: conj(a) / N(a) (the norm is duplicated: one GCD)
  const F ni = inv_dup(norm_dup(a));
  return mulp(conj<0>(a), ni);
}

}  // namespace wv

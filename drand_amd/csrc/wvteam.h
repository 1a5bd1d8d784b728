// One verification by a team of eight waves (two per SIMD of a CU), the latency engine's device form
// (k_lat.hip). The work of wverify.h's verify_item, scheduled across the waves:
//
//   phase A  wave 0: hash-to-G2 of the message at raised issue priority: wave 5 multiplies for its
//            two SSWU square roots (ring_pow_*) and then maps the second point through the isogeny,
//            wave 3 computes the SSWU inversion and the affine x1, gx1 beside the first root
//            (aff_serve), waves 4 and 5 join it for the cofactor
//            clearing (team_clear_cofactor: each doubling in three rounds, each addition in five)
//            wave 1: decompression of the signature (wave 2 multiplying for its square roots), then
//            its subgroup check
//            waves 2, 3, 6, 7: as soon as wave 1 has the point, the Miller loop of the signature
//            pair (e(-g1, S)) -- the subgroup check runs beside it, its verdict joins at the end
//   phase B  all eight: the Miller loop of the key pair (e(pk, H(m)))
//   phase C  all eight: the product of the two Miller values and the final exponentiation
//
// The two Miller loops run separately (f = f_0 f_1 with each f_k its own loop's product: squaring
// is multiplicative), so the signature's pair needs no hash and overlaps it. A Miller doubling step
// is two team rounds of jobs (dbl_job1 / dbl_job2): (1) the six coefficients of f^2 and the line and
// T pieces (X^2 -> l2, Z^2 -> E, YZ -> l3, A, B), (2) the six coefficients of f^2 l and T's new X, Y,
// Z; an addition step is four rounds of one-product jobs. Every Fp12 operation of the final
// exponentiation gives its six output coefficients to six waves. Two waves per SIMD each run at ~0.8
// of a lone wave's pace (profiles/r04m_latency_sweep_4wave.log: 512 teams of four on 256 CUs take 1.21x
// the time of 256), so halving the rounds of a step pays.
#pragma once
#include "wteam.h"
#include "wverify.h"

namespace wv {

constexpr int TEAM_WAVES = 8;
constexpr uint32_t ALL_WAVES = 0xFFu;
constexpr uint32_t SIG_TEAM = (1u << 2) | (1u << 3) | (1u << 6) | (1u << 7);
constexpr uint32_t HASH_TEAM = (1u << 0) | (1u << 4) | (1u << 5);

// ------------------------------------------------------------------ block LDS slots (wteam.h)
// team areas (one per Miller loop): f double buffer, f^2, T, lines, step intermediates
constexpr int TA_FB = 0, TA_FSQ = 12, TA_TX = 18, TA_TY = 19, TA_TZ = 20, TA_L0 = 21, TA_L2 = 22, TA_L3 = 23,
              TA_A = 24, TA_B = 25, TA_E = 26, TA_YZ = 27, TA_TH = 28, TA_DL = 29, TA_AF = 30, TA_AG = 31,
              TA_SIZE = 32;
// the addition step's C, D, E reuse the doubling's A, B, E slots, its X qz, Y qz, Z qz those of f^2
// (free between the doubling's round 2 and the next doubling's round 1)
constexpr int TA_AC = TA_A, TA_AD = TA_B, TA_AE = TA_E, TA_QX = TA_FSQ, TA_QY = TA_FSQ + 1, TA_QZ = TA_FSQ + 2;
constexpr int TB0 = 0, TB1 = TA_SIZE;  // key pair, signature pair
// final exponentiation values (6 slots each)
constexpr int W_BASE = 2 * TA_SIZE;
constexpr int W_R = W_BASE, W_INV = W_BASE + 6, W_T = W_BASE + 12, W_U = W_BASE + 18, W_G = W_BASE + 24,
              W_P = W_BASE + 30, W_S = W_BASE + 36, W_A = W_BASE + 42, W_B = W_BASE + 48, W_C = W_BASE + 54;
constexpr int S_HX = W_BASE + 60, S_HY = S_HX + 1, S_SX = S_HX + 2, S_SY = S_HX + 3;
// H's homogeneous Z: the key area's last slot (written in phase A after the hash team's slots
// TB0 .. TB0 + 13, read into the key pair before its loop first writes TA_AG)
constexpr int S_HZ = TB0 + TA_AG;
static_assert(S_SY < BLK_SLOTS, "block slots");
// scalar words
constexpr int XW_CLS = 0, XW_SINF = 1, XW_HFIN = 2, XW_F1 = 3, XW_SUB = 4, XW_ONE = 8;  // XW_ONE .. +5
// counters: 0 all waves, 1 the signature team, 2 the decoded signature's hand-off, 3 the hash team
constexpr int CTR_ALL = 0, CTR_SIG = 1, CTR_DEC = 2, CTR_HASH = 3;
// the hash team's slots during phase A: the key pair's area (free until phase B)
constexpr int HS_P = TB0, HS_ACC = TB0 + 3, HS_A = TB0 + 6, HS_B = TB0 + 7, HS_C = TB0 + 8, HS_D = TB0 + 9,
              HS_EE = TB0 + 10, HS_Q2 = TB0 + 11;
// the chain additions: the base's Z^2, Z^3, -2 Z^3, then the step's intermediates
constexpr int HS_BZZ = TB0 + 14, HS_BZC = TB0 + 15, HS_BM2 = TB0 + 16, HS_ZZ = TB0 + 17, HS_U1 = TB0 + 18,
              HS_Y2Z1 = TB0 + 19, HS_H = TB0 + 20, HS_R = TB0 + 21, HS_S1 = TB0 + 22, HS_I = TB0 + 23,
              HS_Z2H = TB0 + 24, HS_RR = TB0 + 25, HS_J = TB0 + 26, HS_V = TB0 + 27;
constexpr int XW_AINF = 16, XW_HZ = 17, XW_BINF = 18;

WVI W12 xld_w12(int base, bool cj = false) {
  W12 r;
  for (int k = 0; k < 6; k++) {
    const F v = xld(base + k);
    r.c[k] = (cj && (k & 1)) ? neg<0>(v) : v;
  }
  return r;
}
WVI void xst_w12(int base, const W12& v) {
  for (int k = 0; k < 6; k++) xst(base + k, v.c[k]);
}

// output k of a six-output operation is computed by wave k of the team
template <class Fn>
WVI void team_op(Team& t, int dst, Fn fn) {
  for (int k = t.id; k < 6; k += t.n) xst(dst + k, fn(k));
  team_sync(t);
}
// the cyclotomic square's outputs by cost on the whole team: the three 2-term outputs (1, 3, 5) and
// one 3-term output on the two SIMDs that carry two active waves (waves 0 and 4, 1 and 5), the other
// two 3-term outputs alone on SIMDs 2 and 3
template <class Fn>
WVI void team_op_cyc(Team& t, int dst, Fn fn) {
  if (t.n != 8) return team_op(t, dst, fn);
  constexpr int8_t K[8] = {1, 5, 2, 4, 3, 0, -1, -1};
  if (K[t.id] >= 0) xst(dst + K[t.id], fn(K[t.id]));
  team_sync(t);
}

WVI void xst_g2(int base, const G2J& p) {
  xst(base, p.x);
  xst(base + 1, p.y);
  xst(base + 2, p.z);
}
WVI G2J xld_g2(int base) { return {xld(base), xld(base + 1), xld(base + 2)}; }

// ------------------------------------------------------------------ exponentiation by two waves
// a^e right to left: the producer squares (a, a^2, a^4, .. : the chain of 378 squarings) and hands
// every power whose exponent bit is set to the consumer through a ring of LDS slots; the consumer
// multiplies them up and hands the product back. The critical path is the squaring chain alone (the
// fixed-window exponentiation's 91 products and 14-entry table leave it), the consumer's ~190
// products run beside it on another SIMD. Two rings: the hash wave's (consumer wave 5) in the key
// pair's area, the signature decoder's (consumer wave 2) in the signature pair's area (both free
// until their Miller loops).
constexpr int RING = 8;
struct Ring {
  int slot0, ctr0;  // RING slots + the result slot; counters produced, consumed, results
};
constexpr Ring HASH_RING = {TB0, 4}, SIG_RING = {TB1, 8};
template <int NW>
WVI int exp_bits(const uint32_t (&e)[NW]) {
  int n = 0;
  for (int i = 0; i < NW; i++) n = e[i] ? 32 * i + 32 - __builtin_clz(e[i]) : n;
  return n;
}
template <int NW>
WVI uint32_t exp_ones(const uint32_t (&e)[NW]) {
  uint32_t c = 0;
  for (int i = 0; i < NW; i++) c += (uint32_t)__builtin_popcount(e[i]);
  return c;
}
struct RingCounts {
  uint32_t produced = 0, consumed = 0, results = 0;
};
template <int NW>
WVI F ring_pow_produce(const Ring& rg, const F& a, const uint32_t (&e)[NW], RingCounts& rc) {
  const int nb = exp_bits(e);
  F x = a;
#pragma unroll 1
  for (int i = 0; i < nb; i++) {
    if ((e[i >> 5] >> (i & 31)) & 1u) {
      if (rc.produced >= (uint32_t)RING) flag_wait(rg.ctr0 + 1, rc.produced - RING + 1);  // slot consumed
      xst(rg.slot0 + rc.produced % RING, x);
      flag_post_lds(rg.ctr0);
      rc.produced++;
    }
    if (i + 1 < nb) x = sqrp_inl(x);
  }
  rc.results++;
  flag_wait(rg.ctr0 + 2, rc.results);
  return xld(rg.slot0 + RING);
}
// one exponentiation's products; with stop_ctr >= 0, returns false without consuming when that counter
// is posted before the first power arrives (the producer finished without this exponentiation)
template <int NW>
WVI bool ring_pow_consume(const Ring& rg, const uint32_t (&e)[NW], RingCounts& rc, int stop_ctr = -1) {
  if (stop_ctr >= 0) {
    uint32_t* c = blk_base() + BLK_SLOTS * 64 + BLK_WORDS_EXTRA;
    for (;;) {
#ifdef WV_HOST
      const uint32_t prod = g_host_ctr[rg.ctr0].load(std::memory_order_acquire);
      const uint32_t stop = g_host_ctr[stop_ctr].load(std::memory_order_acquire);
#else
      const uint32_t stop = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(c + stop_ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
      const uint32_t prod = __builtin_amdgcn_readfirstlane(
          __hip_atomic_load(c + rg.ctr0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
#endif
      if (prod > rc.consumed) break;
      if (stop) return false;
#ifdef WV_HOST
      std::this_thread::yield();
#else
      __builtin_amdgcn_s_sleep(1);
#endif
    }
    (void)c;
  }
  const uint32_t ones = exp_ones(e);
  F acc;
#pragma unroll 1
  for (uint32_t k = 0; k < ones; k++) {
    flag_wait(rg.ctr0, rc.consumed + 1);
    const F v = xld(rg.slot0 + rc.consumed % RING);
    acc = k == 0 ? v : mulp(acc, v);
    rc.consumed++;
    flag_post(rg.ctr0 + 1);  // after the slot's read has returned (the producer reuses the slot)
  }
  xst(rg.slot0 + RING, acc);
  flag_post(rg.ctr0 + 2);
  return true;
}
// a^((p-3)/4) with a helper wave as the consumer
struct PowRing {
  const Ring* rg;
  RingCounts* rc;
  WVI F operator()(const F& a) const { return ring_pow_produce(*rg, a, bls::EXP_P_MINUS_3_DIV_4, *rc); }
};
constexpr int SSWU_POWS = 2;  // whash.h sswu2: the norms' root, then the candidates' root

// SSWU's affine side (whash.h sswu_affine: the pair inversion, x1 and gx1 of both maps) on a helper
// wave while the hash wave runs its first exponentiation: the request (N(xD), xN, xD) and the
// answer (1 / N(xD), x1, gx1) through slots of the key pair's area beside the ring
constexpr int AFF_Q = TB0 + 10, AFF_A = TB0 + 15, CTR_AFQ = 7, CTR_AFA = 11;
struct AffTeam {
  WVI void start(const F& nd, const F (&xN)[2], const F (&xD)[2]) const {
    xst(AFF_Q, nd);
    for (int m = 0; m < 2; m++) {
      xst(AFF_Q + 1 + m, xN[m]);
      xst(AFF_Q + 3 + m, xD[m]);
    }
    flag_post_lds(CTR_AFQ);
  }
  WVI SswuAff get() const {
    flag_wait(CTR_AFA, 1);
    SswuAff r;
    r.ndi = xld(AFF_A);
    for (int m = 0; m < 2; m++) {
      r.x1[m] = xld(AFF_A + 1 + m);
      r.gx1[m] = xld(AFF_A + 3 + m);
    }
    return r;
  }
};
// the second map's isogeny on wave 5 (after its ring products) beside the first map's on wave 0
constexpr int ISO_Q = TB0 + 20, ISO_A = TB0 + 22, CTR_ISOQ = 12, CTR_ISOA = 13;
// wave 0's hash up to the sum of the two mapped points (whash.h hash_to_curve_sum, the team form)
WVI G2J team_hash_to_curve_sum(const uint32_t (&b0)[8], RingCounts& rc) {
  uint32_t e[4][16];
  xmd_words(b0, e);
  const F u[2] = {fp2_from_be512(e[0], e[1]), fp2_from_be512(e[2], e[3])};
  F x[2], y[2];
  WV_MARK(10);
  sswu2(u, x, y, PowRing{&HASH_RING, &rc}, AffTeam{});
  WV_MARK(11);
  xst(ISO_Q, x[1]);
  xst(ISO_Q + 1, y[1]);
  flag_post_lds(CTR_ISOQ);
  const G2J q0 = iso_map(x[0], y[0]);
  flag_wait(CTR_ISOA, 1);
  const G2J q = g2_add(q0, xld_g2(ISO_A));
  WV_MARK(12);
  return q;
}
WVI void iso_serve() {
  flag_wait(CTR_ISOQ, 1);
  xst_g2(ISO_A, iso_map(xld(ISO_Q), xld(ISO_Q + 1)));
  flag_post(CTR_ISOA);
}

WVI void aff_serve() {
  flag_wait(CTR_AFQ, 1);
  const F xN[2] = {xld(AFF_Q + 1), xld(AFF_Q + 2)}, xD[2] = {xld(AFF_Q + 3), xld(AFF_Q + 4)};
  const SswuAff r = sswu_affine(xld(AFF_Q), xN, xD);
  xst(AFF_A, r.ndi);
  for (int m = 0; m < 2; m++) {
    xst(AFF_A + 1 + m, r.x1[m]);
    xst(AFF_A + 3 + m, r.gx1[m]);
  }
  flag_post(CTR_AFA);
}
constexpr int DEC_POWS = 2;   // whash.h g2_decompress (none when it rejects before its square root)

// ------------------------------------------------------------------ cofactor clearing by a team
// wcurve.h g2_dbl (dbl-2009-l) in three rounds of one product per wave, on the accumulator's slots:
// A = X^2, B = Y^2, Z3 = 2 Y Z | C = B^2, D = 4 X B, EE = (3A)^2 | X3 = E^2 - 2D, Y3 = E (3D - EE) - 8C
// (Y3 = E (D - X3) - 8C with X3 substituted, so X3 and Y3 are one round)
// rounds 1 and 2 (A, B, Z3 | C, D, EE), shared with team_g2_dbl2
WVI void team_g2_dbl_r12(Team& t, int acc) {
  for (int j = t.id; j < 3; j += t.n) {
    const F Y = xld(acc + 1);
    if (j == 0) xst(HS_A, sqr2(xld(acc)));
    else if (j == 1) xst(HS_B, sqr2(Y));
    else xst(acc + 2, dot(dbl(Y), xld(acc + 2)));
  }
  team_sync(t);
  for (int j = t.id; j < 3; j += t.n) {
    const F B = xld(HS_B);
    if (j == 0) xst(HS_C, sqr2(B));
    else if (j == 1) xst(HS_D, dot(xld(acc), mul_small<4>(B)));
    else xst(HS_EE, sqr2(mul_small<3>(xld(HS_A))));
  }
  team_sync(t);
}
WVI void team_g2_dbl(Team& t, int acc) {
  team_g2_dbl_r12(t, acc);
  for (int j = t.id; j < 2; j += t.n) {
    const F E = mul_small<3>(xld(HS_A)), D = xld(HS_D);
    if (j == 0) xst(acc, dot(E, E, D, cst(WC_NEG2)));
    else xst(acc + 1, dot(sub<0>(mul_small<3>(D), xld(HS_EE)), E, xld(HS_C), cst(WC_NEG8)));
  }
  team_sync(t);
}
// two doublings in five rounds instead of six. The first as above, except that X3 = EE - 2D is left as
// that linear form; the second from (X3, Y3, Z3) with A' = X3^2 as dbl-2009-l, written in products of
// the earlier rounds' outputs:
//   X5 = 9 A'^2 - 8 X3 B',  Y5 = 36 X3^3 B' - 27 (X3^3)^2 - 8 B'^2 = X3^3 (36 B' - 27 X3^3) - 8 B'^2,
//   Z5 = 2 Y3 Z3  (B' = Y3^2, X3^3 = A' X3)
// -- the same polynomials as two team_g2_dbl calls, so the same Jacobian coordinates:
//   A, B, Z3 | C, D, EE | Y3, A' | X3^3, B', Z5 | X5, Y5
// (Y's slot takes Y3 and Z's Z3 then Z5; A' goes to B's slot, X3^3 to C's, B' to A's, each after its
// last read)
WVI void team_g2_dbl2(Team& t, int acc) {
  team_g2_dbl_r12(t, acc);
  auto x3 = [&]() { return sub<0>(xld(HS_EE), dbl(xld(HS_D))); };  // X3 = EE - 2D (bound 5 p)
  for (int j = t.id; j < 2; j += t.n) {
    if (j == 0) {
      const F E = mul_small<3>(xld(HS_A)), D = xld(HS_D);
      xst(acc + 1, dot(sub<0>(mul_small<3>(D), xld(HS_EE)), E, xld(HS_C), cst(WC_NEG8)));
    } else {
      xst(HS_B, sqr2(x3()));
    }
  }
  team_sync(t);
  for (int j = t.id; j < 3; j += t.n) {
    const F Y3 = xld(acc + 1);
    if (j == 0) xst(HS_C, dot(xld(HS_B), x3()));
    else if (j == 1) xst(HS_A, sqr2(Y3));
    else xst(acc + 2, dot(dbl(Y3), xld(acc + 2)));
  }
  team_sync(t);
  for (int j = t.id; j < 2; j += t.n) {
    const F Bp = xld(HS_A), n8B = mul_small<8>(neg<0>(Bp));
    if (j == 0) {
      const F Ap = xld(HS_B);
      xst(acc, dot(Ap, mul_small<9>(Ap), x3(), n8B));
    } else {
      const F X33 = xld(HS_C);
      xst(acc + 1, dot(X33, sub<1>(mul_small<36>(Bp), mul_small<27>(X33)), Bp, n8B));
    }
  }
  team_sync(t);
}
// acc <- acc + base (wcurve.h g2_add: add-2007-bl with its exceptional cases) in five rounds, the base's
// Z^2, Z^3, -2 Z^3 and infinity flag prepared by team_mul_x_abs:
//   Z1Z1, U1 = X1 Z2^2, Y2 Z1, [acc = O?] | H = X2 Z1Z1 - U1, r = 2 (Y2 Z1 Z1Z1 - Y1 Z2^3), S1 = Y1 Z2^3 |
//   I = (2H)^2, 2 Z2 H, r^2, [H = 0?] | J = H I, V = U1 I, Z3 = Z1 (2 Z2 H) |
//   X3 = r^2 - J - 2V, Y3 = r (3V + J - r^2) - 2 S1 J   (= r (V - X3) - 2 S1 J)
WVI void team_g2_add_fixed(Team& t, int acc, int base) {
  if (xld_word(XW_BINF)) return;  // acc + O
  for (int j = t.id; j < 4; j += t.n) {
    const F Z1 = xld(acc + 2);
    if (j == 0) xst(HS_ZZ, sqr2(Z1));
    else if (j == 1) xst(HS_U1, dot(xld(acc), xld(HS_BZZ)));
    else if (j == 2) xst(HS_Y2Z1, dot(xld(base + 1), Z1));
    else xst_word(XW_AINF, is_zero2(Z1) ? 1u : 0u);
  }
  team_sync(t);
  if (xld_word(XW_AINF)) {  // O + base
    if (t.id == 0) xst_g2(acc, xld_g2(base));
    team_sync(t);
    return;
  }
  for (int j = t.id; j < 3; j += t.n) {
    const F Y1 = xld(acc + 1);
    if (j == 0) xst(HS_H, dot(xld(base), xld(HS_ZZ), xld(HS_U1), cst(WC_NEG1)));
    else if (j == 1) xst(HS_R, dot(xld(HS_Y2Z1), dbl(xld(HS_ZZ)), Y1, xld(HS_BM2)));
    else xst(HS_S1, dot(Y1, xld(HS_BZC)));
  }
  team_sync(t);
  for (int j = t.id; j < 4; j += t.n) {
    const F H = xld(HS_H);
    if (j == 0) xst(HS_I, dot(H, mul_small<4>(H)));
    else if (j == 1) xst(HS_Z2H, dot(xld(base + 2), dbl(H)));
    else if (j == 2) xst(HS_RR, sqr2(xld(HS_R)));
    else xst_word(XW_HZ, is_zero2(H) ? 1u : 0u);
  }
  team_sync(t);
  if (xld_word(XW_HZ)) {  // acc == +-base: doubling or the point at infinity
    if (t.id == 0) xst_g2(acc, is_zero2(xld(HS_R)) ? g2_dbl(xld_g2(acc)) : g2_infinity());
    team_sync(t);
    return;
  }
  for (int j = t.id; j < 3; j += t.n) {
    const F I = xld(HS_I);
    if (j == 0) xst(HS_J, dot(xld(HS_H), I));
    else if (j == 1) xst(HS_V, dot(xld(HS_U1), I));
    else xst(acc + 2, dot(xld(acc + 2), xld(HS_Z2H)));
  }
  team_sync(t);
  for (int j = t.id; j < 2; j += t.n) {
    const F r = xld(HS_R), J = xld(HS_J), V = xld(HS_V);
    if (j == 0) xst(acc, dot(r, r, add(J, dbl(V)), cst(WC_NEG1)));  // r^2 - (J + 2V)
    else xst(acc + 1, dot(sub<0>(add(mul_small<3>(V), J), xld(HS_RR)), r, xld(HS_S1), neg<0>(dbl(J))));
  }
  team_sync(t);
}
// acc <- [|x|] acc (wcurve.h g2_mul_x_abs, acc == base on entry): the doublings and the five additions
// by the team
WVI void team_mul_x_abs(Team& t, int base, int acc) {
  if (t.id == 0) {
    const F Z2 = xld(base + 2);
    const F zz = sqr2(Z2), zc = dot(Z2, zz);
    xst(HS_BZZ, zz);
    xst(HS_BZC, zc);
    xst(HS_BM2, dot(zc, cst(WC_NEG2)));
    xst_word(XW_BINF, is_zero2(Z2) ? 1u : 0u);
  }
  team_sync(t);
  // the runs of doublings between the additions (1, 2, 3, 9, 32, 16 for |x|) in pairs, an odd run's
  // last doubling alone
  int i = 62;
#pragma unroll 1
  while (i >= 0) {
    int run = 1;
    while (i - run >= 0 && !((bls::BLS_X_ABS >> (i - run + 1)) & 1ull)) run++;  // bits i .. i-run+1
#ifndef WV_DBL2
#define WV_DBL2 1
#endif
    if (WV_DBL2) {
#pragma unroll 1
      for (int k = 0; k + 1 < run; k += 2) team_g2_dbl2(t, acc);
      if (run & 1) team_g2_dbl(t, acc);
    } else {
#pragma unroll 1
      for (int k = 0; k < run; k++) team_g2_dbl(t, acc);
    }
    i -= run;
    if ((bls::BLS_X_ABS >> (i + 1)) & 1ull) team_g2_add_fixed(t, acc, base);
  }
}
// acc <- acc + base for any two points (wcurve.h g2_add) in five rounds, the base's Z powers included:
//   Z1^2, Z2^2, Y2 Z1, Y1 Z2, [acc = O?], [base = O?] | H = X2 Z1^2 - X1 Z2^2, r = 2 (Y2 Z1 Z1^2 - Y1 Z2 Z2^2),
//   U1 = X1 Z2^2, S1 = Y1 Z2 Z2^2 | I = (2H)^2, 2 Z1 H, r^2, [H = 0?] | J = H I, V = U1 I, Z3 = (2 Z1 H) Z2 |
//   X3, Y3 as team_g2_add_fixed
WVI void team_g2_add(Team& t, int acc, int base) {
  constexpr int S_Z2Z2 = HS_BZZ, S_Y1Z2 = HS_BZC;
  for (int j = t.id; j < 6; j += t.n) {
    const F Z1 = xld(acc + 2), Z2 = xld(base + 2);
    if (j == 0) xst(HS_ZZ, sqr2(Z1));
    else if (j == 1) xst(S_Z2Z2, sqr2(Z2));
    else if (j == 2) xst(HS_Y2Z1, dot(xld(base + 1), Z1));
    else if (j == 3) xst(S_Y1Z2, dot(xld(acc + 1), Z2));
    else if (j == 4) xst_word(XW_AINF, is_zero2(Z1) ? 1u : 0u);
    else xst_word(XW_BINF, is_zero2(Z2) ? 1u : 0u);
  }
  team_sync(t);
  if (xld_word(XW_BINF)) return;  // acc + O
  if (xld_word(XW_AINF)) {        // O + base
    if (t.id == 0) xst_g2(acc, xld_g2(base));
    team_sync(t);
    return;
  }
  for (int j = t.id; j < 4; j += t.n) {
    const F Z2Z2 = xld(S_Z2Z2);
    if (j == 0) xst(HS_H, dot(xld(base), xld(HS_ZZ), xld(acc), neg<0>(Z2Z2)));
    else if (j == 1) xst(HS_R, dot(xld(HS_Y2Z1), dbl(xld(HS_ZZ)), xld(S_Y1Z2), neg<0>(dbl(Z2Z2))));
    else if (j == 2) xst(HS_U1, dot(xld(acc), Z2Z2));
    else xst(HS_S1, dot(xld(S_Y1Z2), Z2Z2));
  }
  team_sync(t);
  for (int j = t.id; j < 4; j += t.n) {
    const F H = xld(HS_H);
    if (j == 0) xst(HS_I, dot(H, mul_small<4>(H)));
    else if (j == 1) xst(HS_Z2H, dot(xld(acc + 2), dbl(H)));
    else if (j == 2) xst(HS_RR, sqr2(xld(HS_R)));
    else xst_word(XW_HZ, is_zero2(H) ? 1u : 0u);
  }
  team_sync(t);
  if (xld_word(XW_HZ)) {
    if (t.id == 0) xst_g2(acc, is_zero2(xld(HS_R)) ? g2_dbl(xld_g2(acc)) : g2_infinity());
    team_sync(t);
    return;
  }
  for (int j = t.id; j < 3; j += t.n) {
    const F I = xld(HS_I);
    if (j == 0) xst(HS_J, dot(xld(HS_H), I));
    else if (j == 1) xst(HS_V, dot(xld(HS_U1), I));
    else xst(acc + 2, dot(xld(HS_Z2H), xld(base + 2)));
  }
  team_sync(t);
  for (int j = t.id; j < 2; j += t.n) {
    const F r = xld(HS_R), J = xld(HS_J), V = xld(HS_V);
    if (j == 0) xst(acc, dot(r, r, add(J, dbl(V)), cst(WC_NEG1)));  // r^2 - (J + 2V)
    else xst(acc + 1, dot(sub<0>(add(mul_small<3>(V), J), xld(HS_RR)), r, xld(HS_S1), neg<0>(dbl(J))));
  }
  team_sync(t);
}
// y <- -y of the point in slots p (one wave writes; the caller's next team round reads)
WVI void team_neg_y(Team& t, int p) {
  if (t.id == 0) xst(p + 1, neg<0>(xld(p + 1)));
  team_sync(t);
}

// wcurve.h g2_clear_cofactor by the hash team: p is the first wave's (the others pass anything);
// the result is the first wave's. A = -[|x|] P + psi(P), then -[|x|] A - A - P + psi^2(2P), every
// addition and doubling by the team
WVI G2J team_clear_cofactor(Team& t, const G2J& p) {
  if (t.id == 0) {
    xst_g2(HS_P, p);
    xst_g2(HS_ACC, p);
  }
  team_sync(t);
  team_mul_x_abs(t, HS_P, HS_ACC);
  // psi(P) into HS_Q2 (conj(x) kx, conj(y) ky, conj(z))
  for (int j = t.id; j < 3; j += t.n) {
    const F c = xld(HS_P + j);
    xst(HS_Q2 + j, j == 2 ? conj<1>(c) : mul2(conj<1>(c), cst(j == 0 ? WC_PSI_KX : WC_PSI_KY)));
  }
  team_sync(t);
  team_neg_y(t, HS_ACC);
  team_g2_add(t, HS_ACC, HS_Q2);  // A
  if (t.id == 0) xst_g2(HS_Q2, xld_g2(HS_ACC));
  team_sync(t);
  team_mul_x_abs(t, HS_Q2, HS_ACC);
  // -[|x|] A - A - P + psi^2(2P): HS_Q2 <- -A, then -P, then psi^2(2P) as the bases
  if (t.id == 0) xst(HS_ACC + 1, neg<0>(xld(HS_ACC + 1)));
  team_neg_y(t, HS_Q2);
  team_g2_add(t, HS_ACC, HS_Q2);
  if (t.id == 0) xst_g2(HS_Q2, g2_neg(xld_g2(HS_P)));
  team_sync(t);
  team_g2_add(t, HS_ACC, HS_Q2);
  if (t.id == 0) xst_g2(HS_Q2, xld_g2(HS_P));
  team_sync(t);
  team_g2_dbl(t, HS_Q2);
  for (int j = t.id; j < 2; j += t.n) xst(HS_Q2 + j, mulp(xld(HS_Q2 + j), cst(j == 0 ? WC_PSI2_KX : WC_PSI2_KY)));
  team_sync(t);
  team_g2_add(t, HS_ACC, HS_Q2);
  return t.id == 0 ? xld_g2(HS_ACC) : p;
}

// ------------------------------------------------------------------ Miller loop of one pair
// doubling round 1: 0..5 the coefficients of f^2, 6 X^2 -> l2 = 3 X^2 xP, 7 E = 3 b' Z^2,
// 8 YZ -> l3 = -2 Y Z yP, 9 A = X Y / 2, 10 B = Y^2 (pairing.h miller_dbl_step)
WVI void dbl_job1(int j, const MPair& m, int tb, int fin) {
  if (j < 6) {
    xst(tb + TA_FSQ + j, w12_sqr_c(xld_w12(fin), j));
    return;
  }
  const F X = xld(tb + TA_TX), Y = xld(tb + TA_TY), Z = xld(tb + TA_TZ);
  switch (j) {
    case 6: xst(tb + TA_L2, mulp(sqr2(X), m.xp3)); break;
    case 7: xst(tb + TA_E, dot(Z, mul_small<12>(mul_xi<0>(Z)))); break;  // 3 b' Z^2 with 3 b' = 12 xi: one product
    case 8: {
      const F YZ = dot(Y, Z);
      xst(tb + TA_YZ, YZ);
      xst(tb + TA_L3, mulp(YZ, m.m2yp));
      break;
    }
    case 9: xst(tb + TA_A, half(dot(X, Y))); break;
    default: xst(tb + TA_B, sqr2(Y)); break;
  }
}
// doubling round 2: 0..5 the coefficients of f^2 l (l0 = E - B), 6 X3 = A (B - 3E), 7 Y3 = G^2 - 3 E^2
// with G = (B + 3E) / 2, 8 Z3 = B H with H = 2 Y Z
WVI void dbl_job2(int j, int tb, int fout) {
  const F B = xld(tb + TA_B), E = xld(tb + TA_E);
  if (j < 6) {
    const W12 q = xld_w12(tb + TA_FSQ);
    xst(fout + j, w12_mul_line_c(q, sub<0>(E, B), xld(tb + TA_L2), xld(tb + TA_L3), j));
    return;
  }
  const F nE = neg<0>(E);
  if (j == 6) {
    xst(tb + TA_TX, dot(xld(tb + TA_A), sub<1>(B, mul_small<3>(E))));  // A (B - 3E): one product
  } else if (j == 7) {
    const F G = half(add(B, mul_small<3>(E)));
    xst(tb + TA_TY, dot(G, G, mul_small<3>(E), nE));
  } else {
    xst(tb + TA_TZ, dot(B, dbl(xld(tb + TA_YZ))));
  }
}
// round-1 jobs per wave (bit j = job j): jobs 6 and 8 are two products, the rest one
WVI uint32_t dbl_jobs1(const Team& t) {
  if (t.n == 8) {
    // the 4-term f^2 outputs (0, 2, 4) and the two-product lines alone, the 3-term outputs each
    // beside a one-product piece (waves w and w + 4 share a SIMD)
    constexpr uint16_t J8[8] = {1 << 0, 1 << 2, 1 << 4, 1 << 8, 1 << 6, (1 << 1) | (1 << 9), (1 << 3) | (1 << 10),
                                (1 << 5) | (1 << 7)};
    return J8[t.id];
  }
  if (t.n == 4) {
    constexpr uint16_t J4[4] = {(1 << 0) | (1 << 1) | (1 << 9), (1 << 2) | (1 << 3) | (1 << 10), (1 << 4) | (1 << 6),
                                (1 << 5) | (1 << 7) | (1 << 8)};
    return J4[t.id];
  }
  if (t.n == 5) {
    constexpr uint16_t J5[5] = {(1 << 6) | (1 << 9), (1 << 7) | (1 << 10), (1 << 8) | (1 << 0),
                                (1 << 1) | (1 << 2) | (1 << 3), (1 << 4) | (1 << 5)};
    return J5[t.id];
  }
  uint32_t m = 0;
  for (int j = t.id; j < 11; j += t.n) m |= 1u << j;
  return m;
}

WVI void team_miller_dbl(Team& t, const MPair& m, int tb, int& cur) {
  const int fin = tb + TA_FB + 6 * cur, fout = tb + TA_FB + 6 * (cur ^ 1);
  const uint32_t jobs = dbl_jobs1(t);
  for (int j = 0; j < 11; j++)
    if ((jobs >> j) & 1u) dbl_job1(j, m, tb, fin);
  team_sync(t);
  if (t.n == 8) {
    // waves 0..5 the six f^2 l coefficients (three-term products), wave 6 X3 and Z3, wave 7 Y3
    dbl_job2(t.id, tb, fout);
    if (t.id == 6) dbl_job2(8, tb, fout);
  } else if (t.n == 4) {
    // two three-term products per wave, the one-product X3 and Z3 with the fifth, the two-term Y3
    // with the sixth (at most two products' worth per wave instead of three for the strided split)
    constexpr uint8_t J[4][3] = {{0, 1, 9}, {2, 3, 9}, {4, 6, 8}, {5, 7, 9}};
    for (int q = 0; q < 3; q++)
      if (J[t.id][q] < 9) dbl_job2(J[t.id][q], tb, fout);
  } else {
    for (int j = t.id; j < 9; j += t.n) dbl_job2(j, tb, fout);
  }
  team_sync(t);
  cur ^= 1;
}

// addition step (pairing.h miller_add_step) in four rounds of one-product jobs. With a projective Q
// (qx : qy : qz) it is the affine step with T's X, Y, Z replaced by X qz, Y qz, Z qz (those three are
// extra round-1 jobs; theta, delta and the lines then carry a factor qz, qz^2):
//   theta = Y qz - qy Z, delta = X qz - qx Z | l0, l2, l3, C = theta^2, D = delta^2 |
//   f l, E = D delta, F = Zq C, G = Xq D | X3 = delta H, Y3 = theta (G - H) - Yq E, Z3 = Zq E,
// H = E + F - 2G (Xq, Yq, Zq = X qz, Y qz, Z qz, or X, Y, Z for an affine Q)
WVI void team_miller_add(Team& t, const MPair& m, int tb, int& cur) {
  const int nj1 = m.qaff ? 2 : 5;
  for (int j = t.id; j < nj1; j += t.n) {
    const F Z = xld(tb + TA_TZ);
    const F qz = m.qaff ? cst(WC_ONE2) : m.qz;
    if (j == 0) xst(tb + TA_TH, dot(xld(tb + TA_TY), qz, Z, m.mqy));       // Y qz - qy Z
    else if (j == 1) xst(tb + TA_DL, dot(xld(tb + TA_TX), qz, Z, m.mqx));  // X qz - qx Z
    else if (j == 2) xst(tb + TA_QX, dot(xld(tb + TA_TX), qz));
    else if (j == 3) xst(tb + TA_QY, dot(xld(tb + TA_TY), qz));
    else xst(tb + TA_QZ, dot(Z, qz));
  }
  team_sync(t);
  const int sx = m.qaff ? TA_TX : TA_QX, sy = m.qaff ? TA_TY : TA_QY, sz = m.qaff ? TA_TZ : TA_QZ;
  for (int j = t.id; j < 5; j += t.n) {
    const F theta = xld(tb + TA_TH), delta = xld(tb + TA_DL);
    switch (j) {
      case 0: xst(tb + TA_L0, dot(theta, m.qx, delta, m.mqy)); break;                        // theta qx - delta qy
      case 1: xst(tb + TA_L2, m.qaff ? mulp(theta, m.mxp) : dot(theta, m.mxpz)); break;  // -theta xP (qz)
      case 2: xst(tb + TA_L3, m.qaff ? mulp(delta, m.yp) : dot(delta, m.ypz)); break;    // delta yP (qz)
      case 3: xst(tb + TA_AC, sqr2(theta)); break;
      default: xst(tb + TA_AD, sqr2(delta)); break;
    }
  }
  team_sync(t);
  const int fin = tb + TA_FB + 6 * cur, fout = tb + TA_FB + 6 * (cur ^ 1);
  for (int j = t.id; j < 9; j += t.n) {
    if (j < 6) {
      xst(fout + j, w12_mul_line_c(xld_w12(fin), xld(tb + TA_L0), xld(tb + TA_L2), xld(tb + TA_L3), j));
    } else if (j == 6) {
      xst(tb + TA_AE, dot(xld(tb + TA_AD), xld(tb + TA_DL)));
    } else if (j == 7) {
      xst(tb + TA_AF, dot(xld(tb + sz), xld(tb + TA_AC)));
    } else {
      xst(tb + TA_AG, dot(xld(tb + sx), xld(tb + TA_AD)));
    }
  }
  team_sync(t);
  for (int j = t.id; j < 3; j += t.n) {
    const F E = xld(tb + TA_AE), G = xld(tb + TA_AG);
    const F H = sub<0>(add(E, xld(tb + TA_AF)), dbl(G));  // E + F - 2G
    if (j == 0) xst(tb + TA_TX, dot(xld(tb + TA_DL), H));
    else if (j == 1) xst(tb + TA_TY, dot(xld(tb + TA_TH), sub<1>(G, H), xld(tb + sy), neg<0>(E)));
    else xst(tb + TA_TZ, dot(xld(tb + sz), E));
  }
  team_sync(t);
  cur ^= 1;
}

// f_{|x|, Q}(P) of one pair (unconjugated, wpairing.h miller_loop); returns its slot base
WVI int team_miller(Team& t, const MPair& m, int tb) {
  if (t.id == 0) {
    xst_w12(tb + TA_FB, w12_one());
    xst(tb + TA_TX, m.t.x);
    xst(tb + TA_TY, m.t.y);
    xst(tb + TA_TZ, m.t.z);
  }
  team_sync(t);
  int cur = 0;
#pragma unroll 1
  for (int i = 62; i >= 0; i--) {
    team_miller_dbl(t, m, tb, cur);
    if ((bls::BLS_X_ABS >> i) & 1ull) team_miller_add(t, m, tb, cur);
  }
  return tb + TA_FB + 6 * cur;
}

// ------------------------------------------------------------------ final exponentiation
// dst <- src^|x| (wpairing.h w12_pow_x_abs); scr is clobbered. 68 operations alternate between scr and
// dst, starting on scr, so the last lands on dst.
WVI void team_pow_x_abs(Team& t, int dst, int src, int scr) {
  constexpr uint64_t NSQ = 1ull | (2ull << 6) | (3ull << 12) | (9ull << 18) | (32ull << 24) | (16ull << 30);
  int in = src, out = scr;
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int n = (int)((NSQ >> (6 * s)) & 63u);
#pragma unroll 1
    for (int k = 0; k < n; k++) {
      team_op_cyc(t, out, [&](int c) { return w12_cyc_sqr_c(xld_w12(in), c); });
      in = out;
      out = out == scr ? dst : scr;
    }
    if (s < 5) {
      team_op(t, out, [&](int c) { return w12_mul_c(xld_w12(in), xld_w12(src), c); });
      in = out;
      out = out == scr ? dst : scr;
    }
  }
}

// W_INV <- conj(f^-1) for the Fp12 value in slots f (wtower.h w12_inv<true>) in six rounds around one
// inversion: f = A + B w, A = (c0, c2, c4), B = (c1, c3, c5), D = A^2 - v B^2 (each coefficient one
// 4-term product straight from A and B) | t0 = D0^2 - xi D1 D2, t1 = xi D2^2 - D0 D1, t2 = D1^2 - D0 D2 |
// d = D0 t0 + xi (D2 t1 + D1 t2) | 1/d (one wave) | D^-1 = t / d | (A D^-1, B D^-1)
WVI void team_w12_inv_conj(Team& t, int f) {
  constexpr int SD = W_T, ST = W_T + 3, SDI = W_U, SI = W_U + 1;  // D, t, 1/d, D^-1 (free slots)
  for (int j = t.id; j < 3; j += t.n) {
    const F a0 = xld(f), a1 = xld(f + 2), a2 = xld(f + 4), b0 = xld(f + 1), b1 = xld(f + 3), b2 = xld(f + 5);
    F d;
    if (j == 0)  // a0^2 + 2 xi a1 a2 - xi (2 b0 b2 + b1^2)
      d = dot(a0, a0, a1, dbl(mul_xi<0>(a2)), b0, neg<1>(dbl(mul_xi<0>(b2))), b1, neg<1>(mul_xi<0>(b1)));
    else if (j == 1)  // 2 a0 a1 + xi a2^2 - (b0^2 + 2 xi b1 b2)
      d = dot(a0, dbl(a1), a2, mul_xi<0>(a2), b0, neg<0>(b0), b1, neg<1>(dbl(mul_xi<0>(b2))));
    else  // 2 a0 a2 + a1^2 - (2 b0 b1 + xi b2^2)
      d = dot(a0, dbl(a2), a1, a1, b0, neg<0>(dbl(b1)), b2, neg<1>(mul_xi<0>(b2)));
    xst(SD + j, d);
  }
  team_sync(t);
  for (int j = t.id; j < 3; j += t.n) {
    const F c0 = xld(SD), c1 = xld(SD + 1), c2 = xld(SD + 2);
    if (j == 0) xst(ST, dot(c0, c0, c2, neg<1>(mul_xi<0>(c1))));
    else if (j == 1) xst(ST + 1, dot(c2, mul_xi<0>(c2), c1, neg<0>(c0)));
    else xst(ST + 2, dot(c1, c1, c2, neg<0>(c0)));
  }
  team_sync(t);
  if (t.id == 0) {
    const F c0 = xld(SD), c1 = xld(SD + 1), c2 = xld(SD + 2);
    const F d = dot(c0, xld(ST), mul_xi<0>(c2), xld(ST + 1), mul_xi<0>(c1), xld(ST + 2));
    xst(SDI, inv2(d));
  }
  team_sync(t);
  for (int j = t.id; j < 3; j += t.n) xst(SI + j, mul2(xld(ST + j), xld(SDI)));
  team_sync(t);
  for (int j = t.id; j < 6; j += t.n) {
    // output slot k = 2 i + h: component i of (A or B) * D^-1 (h = 0: A, 1: B); conj keeps B's sign
    const int h = j & 1, i = j >> 1;
    const F x0 = xld(f + h), x1 = xld(f + 2 + h), x2 = xld(f + 4 + h);
    const F y0 = xld(SI), y1 = xld(SI + 1), y2 = xld(SI + 2);
    F r;
    if (i == 0) r = dot(x0, y0, x1, mul_xi<0>(y2), x2, mul_xi<0>(y1));
    else if (i == 1) r = dot(x0, y1, x1, y0, x2, mul_xi<0>(y2));
    else r = dot(x0, y2, x1, y1, x2, y0);
    xst(W_INV + j, r);
  }
  team_sync(t);
}

// wpairing.h final_exp_is_one of the Miller value in slots f0 (unconjugated)
WVI bool team_final_exp_is_one(Team& t, int f0) {
  team_w12_inv_conj(t, f0);  // conj(f0^-1)
  team_op(t, W_T, [&](int k) { return w12_mul_c(xld_w12(f0), xld_w12(W_INV), k); });
  team_op(t, W_U, [&](int k) { return w12_frob2_c(xld_w12(W_T), k); });
  team_op(t, W_G, [&](int k) { return w12_mul_c(xld_w12(W_U), xld_w12(W_T), k); });
  // a = g^(x-1), b = a^(x-1), c = b^(x+p); X^x = conj(X^|x|)
  if (t.id == 0) WV_MARK(8);
  team_pow_x_abs(t, W_P, W_G, W_S);
  if (t.id == 0) WV_MARK(9);
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_G, true), k); });
  team_pow_x_abs(t, W_P, W_A, W_S);
  team_op(t, W_B, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_A, true), k); });
  team_pow_x_abs(t, W_P, W_B, W_S);
  team_op(t, W_U, [&](int k) { return w12_frob_c(xld_w12(W_B), k); });
  team_op(t, W_C, [&](int k) { return w12_mul_c(xld_w12(W_P, true), xld_w12(W_U), k); });
  // e = (c^|x|)^|x| frob2(c) conj(c) g^2 g
  team_pow_x_abs(t, W_A, W_C, W_S);
  team_pow_x_abs(t, W_B, W_A, W_S);
  team_op(t, W_U, [&](int k) { return w12_frob2_c(xld_w12(W_C), k); });
  team_op(t, W_P, [&](int k) { return w12_mul_c(xld_w12(W_B), xld_w12(W_U), k); });
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P), xld_w12(W_C, true), k); });
  team_op_cyc(t, W_U, [&](int k) { return w12_cyc_sqr_c(xld_w12(W_G), k); });
  team_op(t, W_P, [&](int k) { return w12_mul_c(xld_w12(W_A), xld_w12(W_U), k); });
  team_op(t, W_A, [&](int k) { return w12_mul_c(xld_w12(W_P), xld_w12(W_G), k); });
  // e == 1: coefficient k checked by wave k, the six verdicts through scalar words
  for (int k = t.id; k < 6; k += t.n) {
    const F c = xld(W_A + k);
    xst_word(XW_ONE + k, is_zero2(k == 0 ? sub<0>(c, cst(WC_ONE2)) : c) ? 1u : 0u);
  }
  team_sync(t);
  bool one = true;
  for (int k = 0; k < 6; k++) one = one & (xld_word(XW_ONE + k) != 0u);
  return one;
}

// ------------------------------------------------------------------ the item
// wverify.h verify_item run by the eight waves of a workgroup (each wave calls it); every wave returns
// the same class, and sx, sy, s_inf (the decoded signature) on REJ_OK / REJ_PAIRING
WVI uint8_t verify_team(const uint8_t* sig, const uint32_t (&b0)[8], const uint32_t* pkx, const uint32_t* pky,
                        bool pk_inf, F& sx, F& sy, bool& s_inf) {
  const int w = wave_id();
  Team all = make_team(ALL_WAVES, CTR_ALL);
  if (w == 0) WV_MARK(0);
  if ((HASH_TEAM >> w) & 1u) {
    // xmd, both SSWU maps and the isogeny on wave 0, the cofactor clearing by the hash team
    Team th = make_team(HASH_TEAM, CTR_HASH);
    WV_PRIO(2);  // above the signature branch's waves on SIMD 1 (wave 5) and the decoder (wave 1)
    // wave 5 multiplies for the SSWU exponentiations of wave 0 (ring_pow_*), wave 4 (on wave 0's
    // SIMD) stays idle until the cofactor clearing
    RingCounts rc;
    G2J q = g2_infinity();
    if (w == 0) q = team_hash_to_curve_sum(b0, rc);
    if (w == 5) {
      for (int k = 0; k < SSWU_POWS; k++) ring_pow_consume(HASH_RING, bls::EXP_P_MINUS_3_DIV_4, rc);
      iso_serve();
    }
    const G2J h = team_clear_cofactor(th, q);
    if (w != 0) WV_PRIO(0);
    if (w == 0) {
      WV_MARK(13);
      const bool fin = !g2_is_inf(h);
      if (fin) {
        // Jacobian (X, Y, Z) -> homogeneous (X Z : Y : Z^3): no inversion (mpair_proj)
        xst(S_HX, dot(h.x, h.z));
        xst(S_HY, h.y);
        xst(S_HZ, dot(h.z, sqr2(h.z)));
      }
      WV_PRIO(0);
      WV_MARK(1);
      xst_word(XW_HFIN, fin);
    }
  } else if (w == 1) {
    F x, y;
    bool inf;
    RingCounts rc;
    const uint8_t c = g2_decompress(sig, x, y, inf, false, PowRing{&SIG_RING, &rc});
    if (c == bls::REJ_OK && !inf) {
      xst(S_SX, x);
      xst(S_SY, y);
    }
    xst_word(XW_CLS, c);
    xst_word(XW_SINF, inf);
    flag_post(CTR_DEC);
    WV_MARK(2);
    const bool sub_ok = c != bls::REJ_OK || inf || g2_in_subgroup({x, y, cst(WC_ONE2)});
    xst_word(XW_SUB, sub_ok);
    WV_MARK(15);
  } else if ((SIG_TEAM >> w) & 1u) {
    Team t1 = make_team(SIG_TEAM, CTR_SIG);
    if (w == 3) aff_serve();  // the hash's SSWU inversion and affine x1, gx1, idle time of this team
    if (w == 2) {  // the decoder's multiplier for its square roots
      RingCounts rc;
      for (int k = 0; k < DEC_POWS; k++)
        if (!ring_pow_consume(SIG_RING, bls::EXP_P_MINUS_3_DIV_4, rc, CTR_DEC)) break;
    }
    flag_wait(CTR_DEC, 1);
    if (xld_word(XW_CLS) == bls::REJ_OK && !xld_word(XW_SINF)) {
      const MPair m1 = mpair(cst(WC_NEG_G1_X), cst(WC_NEG_G1_Y), xld(S_SX), xld(S_SY));
      const int f1 = team_miller(t1, m1, TB1);
      if (t1.id == 0) xst_word(XW_F1, (uint32_t)f1);
      if (t1.id == 0) WV_MARK(3);
    }
  }
  team_sync(all);
  if (w == 0) WV_MARK(4);
  uint8_t cls = (uint8_t)xld_word(XW_CLS);
  if (cls == bls::REJ_OK && !xld_word(XW_SUB)) cls = bls::REJ_NOT_IN_SUBGROUP;
  if (cls != bls::REJ_OK) return cls;
  s_inf = xld_word(XW_SINF) != 0;
  if (!s_inf) {
    sx = xld(S_SX);
    sy = xld(S_SY);
  }
  const bool a0 = xld_word(XW_HFIN) && !pk_inf, a1 = !s_inf;
  if (!a0 && !a1) return bls::REJ_OK;  // empty product = 1 (kilic Check [ext])
  int f;
  if (a0) {
    const MPair m0 = mpair_proj(g1_coord(pkx), g1_coord(pky), xld(S_HX), xld(S_HY), xld(S_HZ));
    f = team_miller(all, m0, TB0);
    if (w == 0) WV_MARK(5);
    if (a1) {
      const int f1 = (int)xld_word(XW_F1);
      team_op(all, W_R, [&](int k) { return w12_mul_c(xld_w12(f), xld_w12(f1), k); });
      f = W_R;
    }
  } else {
    f = (int)xld_word(XW_F1);
  }
  if (w == 0) WV_MARK(6);
  const bool one = team_final_exp_is_one(all, f);
  if (w == 0) WV_MARK(7);
  return one ? bls::REJ_OK : bls::REJ_PAIRING;
}


// ------------------------------------------------------------------ VerifyRecovered in two launches
// The fused threshold round (blsverify.cpp spec_recover_launch) verifies the signature it recovers
// speculatively. Its message and the group key are known from the start, so phase A's hash branch
// and then phase B's key-pair Miller loop run as their own launch (team_hash_key) beside the partial
// verification and the recovery; the recovered signature reaches the check as the affine point the
// interpolation computed (k_lat_recover_sum), not as bytes, so there is no decompression and no
// subgroup check: the sum of shares whose partials all verified lies in G2, and on a miss the host
// verifies the recomputed signature the whole way. What is left after the recovery is the signature
// pair's Miller loop on all eight waves, the product and phase C (verify_team_pre): the class
// verify_team gives the compressed signature (compress -> decompress is the identity on G2).
// a hand-off buffer in global memory: Fp values at 64-word steps, then one flag row
constexpr int HOUT_WORDS = 7 * 64;  // the key pair's Miller value f0 (6 coefficients), its active flag at [384]
constexpr int SAFF_WORDS = 3 * 64;  // sigma = (x, y) affine, infinity flag at [128]
constexpr double HANDOFF_BOUND = 1.05;  // reduced dot outputs (checked on the host)
WVI void gst_F(uint32_t* base, const F& v) {
  WV_REQUIRE(bnd(v), HANDOFF_BOUND, "handed-off value");
  gst(base, lane_id(), v.x);
}
WVI F gld_F(const uint32_t* base) { return mkF(gld(base, lane_id()), HANDOFF_BOUND); }
WVI W12 gld_w12(const uint32_t* base) {
  W12 r;
  for (int k = 0; k < 6; k++) r.c[k] = gld_F(base + 64 * k);
  return r;
}
WVI void gst_flag(uint32_t* base, bool v) { gst(base, lane_id(), vsplat(v ? 1u : 0u)); }
WVI bool gld_flag(const uint32_t* base) {
#ifdef WV_HOST
  return base[0] != 0u;
#else
  return __builtin_amdgcn_readfirstlane(base[0]) != 0u;
#endif
}

// phase A's hash branch (verify_team's waves 0, 4, 5 and the SSWU helper wave 3), then phase B's key
// pair e(pk, H) on all eight waves: its Miller value and whether the pair is active into hout
WVI void team_hash_key(const uint32_t (&b0)[8], const uint32_t* pkx, const uint32_t* pky, bool pk_inf,
                       uint32_t* hout) {
  const int w = wave_id();
  Team all = make_team(ALL_WAVES, CTR_ALL);
  if ((HASH_TEAM >> w) & 1u) {
    Team th = make_team(HASH_TEAM, CTR_HASH);
    RingCounts rc;
    G2J q = g2_infinity();
    if (w == 0) q = team_hash_to_curve_sum(b0, rc);
    if (w == 5) {
      for (int k = 0; k < SSWU_POWS; k++) ring_pow_consume(HASH_RING, bls::EXP_P_MINUS_3_DIV_4, rc);
      iso_serve();
    }
    const G2J h = team_clear_cofactor(th, q);
    if (w == 0) {
      const bool fin = !g2_is_inf(h);
      if (fin) {  // Jacobian (X, Y, Z) -> homogeneous (X Z : Y : Z^3), as verify_team
        xst(S_HX, dot(h.x, h.z));
        xst(S_HY, h.y);
        xst(S_HZ, dot(h.z, sqr2(h.z)));
      }
      xst_word(XW_HFIN, fin);
    }
  } else if (w == 3) {
    aff_serve();
  }
  team_sync(all);
  const bool a0 = xld_word(XW_HFIN) && !pk_inf;
  if (a0) {
    const MPair m0 = mpair_proj(g1_coord(pkx), g1_coord(pky), xld(S_HX), xld(S_HY), xld(S_HZ));
    const int f = team_miller(all, m0, TB0);
    for (int k = all.id; k < 6; k += all.n) gst_F(hout + 64 * k, xld(f + k));
  }
  if (w == 0) gst_flag(hout + 384, a0);
}

// phases B and C of verify_team after team_hash_key (hin) for an affine signature sin (x, y,
// infinity flag): the signature pair's Miller loop on all eight waves, the product with the key
// pair's value and the final exponentiation
WVI uint8_t verify_team_pre(const uint32_t* hin, const uint32_t* sin) {
  Team all = make_team(ALL_WAVES, CTR_ALL);
  const bool a0 = gld_flag(hin + 384), a1 = !gld_flag(sin + 128);
  if (!a0 && !a1) return bls::REJ_OK;  // empty product = 1 (kilic Check [ext])
  int f;
  if (a1) {
    const MPair m1 = mpair(cst(WC_NEG_G1_X), cst(WC_NEG_G1_Y), gld_F(sin), gld_F(sin + 64));
    const int f1 = team_miller(all, m1, TB1);
    f = f1;
    if (a0) {
      team_op(all, W_R, [&](int k) { return w12_mul_c(gld_w12(hin), xld_w12(f1), k); });
      f = W_R;
    }
  } else {
    team_op(all, W_R, [&](int k) { return gld_F(hin + 64 * k); });
    f = W_R;
  }
  return team_final_exp_is_one(all, f) ? bls::REJ_OK : bls::REJ_PAIRING;
}

}  // namespace wv

// Stage 3: two-pair multi-Miller loop e(pk, H) * e(-g1, sigma), one lane per beacon, in two passes
// (pairing.h miller_lines / miller_f_from_lines): k_miller_lines writes the 68 x 2 sparse lines
// to HBM staging (SoA, 6 Fp slots per line), k_miller_f folds them into f. Each pass keeps only its
// own state live, which removes the scratch spills of the fused loop (13.6 KB/lane, ~160 KB of
// scratch traffic per beacon) for 2 x 39 KB of coalesced line traffic per beacon, and lets the
// lines pass run at 2 waves/SIMD (256 VGPRs).
// kilic Engine.AddPair / AddPairInv [ext] via kyber-bls12381 ValidatePairing.
#include "kcommon.h"

namespace blsk {

// line slot of (step, pair): 6 Fp slots (a0, a1, a4 as Fp2)
DI int line_slot(int step, int k) { return (step * 2 + k) * 6; }
// cache policy of the line staging's stores and loads (soa.h AUX; 0 = default)
// Cache policy of the line staging: written once by k_miller_lines, read once by k_miller_f, 13.8 KB
// per beacon -- nothing to keep in L2/MALL. Non-temporal (gfx950 aux 2) on both sides: Miller
// 196.2 -> 192.7 ms per 1M on one box, interleaved twice (profiles/r06s_ln_nt_ab.json); the loads
// carry the gain, the stores alone change nothing.
#ifndef BLS_LN_AUX
#define BLS_LN_AUX 2
#endif
#ifndef BLS_LN_AUX_ST
#define BLS_LN_AUX_ST BLS_LN_AUX
#endif
#ifndef BLS_LN_AUX_LD
#define BLS_LN_AUX_LD BLS_LN_AUX
#endif

// Item g = base + i of the chunk (H/S/F/cls stride cnt); its lines at LN index i (stride sub).
// The two pairs run in separate workgroups (k = blockIdx.x & 1: the pair of the whole wave), so a
// beacon's two line chains run side by side: half the latency of one lane walking both, twice the
// waves (a finer tail), and every store still one 256-byte access per wave.
static __shared__ uint32_t g_ml_T[72 * BLS_LANES];
// T = (X, Y, Z) in LDS, word w of coordinate c at [(24 c + w) * 64 + lane]: conflict-free dword access
struct g2proj_lds {
  uint32_t* base;
  DI fp2 get(int c) const {
    fp2 v;
#pragma unroll
    for (int w = 0; w < 12; w++) {
      v.c0.l[w] = base[(24 * c + w) * BLS_LANES];
      v.c1.l[w] = base[(24 * c + 12 + w) * BLS_LANES];
    }
    return v;
  }
  DI void set(int c, const fp2& v) const {
#pragma unroll
    for (int w = 0; w < 12; w++) {
      base[(24 * c + w) * BLS_LANES] = v.c0.l[w];
      base[(24 * c + 12 + w) * BLS_LANES] = v.c1.l[w];
    }
  }
};

BLS_KERNEL(BLS_WPE_LINES)
k_miller_lines(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
               const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
               size_t base, size_t m, size_t sub, uint32_t* LN) {
  const int k = (int)(blockIdx.x & 1u);
  const size_t i = (size_t)(blockIdx.x >> 1) * TPB + threadIdx.x;
  if (i >= m) return;
  const size_t g = base + i;
  if (cls[g] != REJ_OK) return;
  const uint32_t kk = pk_idx ? pk_idx[g] : 0u;
  const bool act[2] = {!(pk_inf[kk] | h_inf[g]), !s_inf[g]};
  {
    const uint32_t* Qb = k == 0 ? H : S;
    auto load_q = [&]() {
      size_t j = g;
      asm volatile("" : "+v"(j));  // re-read at each use (5 additions), never hoisted
      return g2a{ld_fp2(Qb, cnt, j, 0), ld_fp2(Qb, cnt, j, 2)};
    };
    auto emit = [&](int step, const line& l) {
      const int s = line_slot(step, k);
      const line o = act[k] ? l : line_one();
      st_fp2<BLS_LN_AUX_ST>(LN, sub, i, s + 0, o.a0);
      st_fp2<BLS_LN_AUX_ST>(LN, sub, i, s + 2, o.a1);
      st_fp2<BLS_LN_AUX_ST>(LN, sub, i, s + 4, o.a4);
    };
    // call-free steps (pairing.h miller_dbl_step_inl): P, Q and the lines never live across a call
    auto pcoord = [&](int c) {
      size_t o = (size_t)kk * G1_WORDS + 12 * c;
      asm volatile("" : "+v"(o));  // re-read at the use
      fp v;
#pragma unroll
      for (int w = 0; w < 12; w++) v.l[w] = pk_tab[o + w];
      return k == 0 ? v : fp_load_const(c == 0 ? G1_GEN_X : G1_GEN_NEG_Y);
    };
    if (!act[k]) {  // a skipped pair (a point at infinity) contributes the line 1 at every step
#pragma unroll 1
      for (int s = 0; s < MILLER_STEPS; s++) emit(s, line_one());
      return;
    }
    int step = 0;
    auto put = [&](int c, const fp2& v) { st_fp2<BLS_LN_AUX_ST>(LN, sub, i, line_slot(step, k) + 2 * c, v); };
    auto xp = [&]() { return pcoord(0); };
    auto yp = [&]() { return pcoord(1); };
    // T parks in LDS (72 words per lane, word-major: 18 KB per one-wave workgroup, 8 per CU at 2
    // waves/SIMD), read at each use and written back coordinate by coordinate
    const g2proj_lds T{g_ml_T + threadIdx.x};
    {
      const g2a Q0 = load_q();
      T.set(0, Q0.x);
      T.set(1, Q0.y);
      T.set(2, fp2_one());
    }
#pragma unroll 1
    for (int b = 62; b >= 0; b--) {
      miller_dbl_step_ts(T, put, xp, yp);
      step++;
      if ((BLS_X_ABS >> b) & 1ull) {
        miller_add_step_ts(T, load_q, put, xp, yp);
        step++;
      }
    }
  }
}

// The line-pair product L (5 Fp2: c0.c0, c0.c1, c0.c2, c1.c1, c1.c2) of the current step parks in LDS
// (one 120-word column per lane: 30 KB per one-wave workgroup, 4 per CU with g_fp2_arg) and is read
// back at each use, so f (144 words) and the partial products are all that stay in registers.
static __shared__ uint32_t g_mf_L[120 * BLS_LANES];
DI void mf_put(int c, const fp2& v) {
  const unsigned l = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    g_mf_L[(c * 24 + k) * BLS_LANES + l] = v.c0.l[k];
    g_mf_L[(c * 24 + 12 + k) * BLS_LANES + l] = v.c1.l[k];
  }
}
DI fp2 mf_get(int c) {
  unsigned l = threadIdx.x;
  asm volatile("" : "+v"(l));  // read at the use, never kept live
  fp2 v;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    v.c0.l[k] = g_mf_L[(c * 24 + k) * BLS_LANES + l];
    v.c1.l[k] = g_mf_L[(c * 24 + 12 + k) * BLS_LANES + l];
  }
  return v;
}
// q p of the one-reduction linear forms (tower.h fp2_lin_reduce, T < 16p) from an LDS table of k p,
// k < 16 (768 bytes per workgroup, tower.h kp_lds_init / KpLdsK)
using KpLds16 = KpLdsK<16>;

// fp6_mul(a, b) (tower.h, Karatsuba) with b's components read through lb
template <typename LB>
DI fp6 fp6_mul_lb(const fp6& a, LB lb) {
#if BLS_F6_LIN
  return fp6_mul_lin_lb(a, lb, KpLds16());
#else
  fp2 t0 = fp2_mul(a.c0, lb(0));
  fp2 t1 = fp2_mul(a.c1, lb(1));
  fp2 t2 = fp2_mul(a.c2, lb(2));
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(lb(1), lb(2))), t1), t2)), t0);
  fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(lb(0), lb(1))), t0), t1), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c2), fp2_add_lazy(lb(0), lb(2))), t0), t2), t1);
  return {c0, c1, c2};
#endif
}
// pairing.h fp12_mul_by_line_pair with L read from LDS (mf_get)
DI fp12 fp12_mul_by_line_pair_lds(const fp12& f) {
  const fp6 t0 = fp6_mul_lb(f.c0, [](int c) { return mf_get(c); });
  fp6 t1;
  {
    const fp2 b1 = mf_get(3), b2 = mf_get(4);
    t1 = fp6_mul_by_12(f.c1, b1, b2);
  }
  // Ls = (L.c0.c0, L.c0.c1 + L.c1.c1, L.c0.c2 + L.c1.c2)
  const fp6 c1 = fp6_sub(fp6_sub(fp6_mul_lb(fp6_add_lazy(f.c0, f.c1), [](int c) {
                                   return c == 0 ? mf_get(0) : fp2_add_lazy(mf_get(c), mf_get(c + 2));
                                 }),
                                 t0),
                         t1);
  return {fp6_add(t0, fp6_mul_v(t1)), c1};
}

BLS_KERNEL(BLS_WPE_MILLER_F) k_miller_f(const uint32_t* LN, const uint8_t* cls, size_t cnt, size_t base,
                                                  size_t m, size_t sub, uint32_t* F) {
#if BLS_F6_LIN
  kp_lds_init<16>();  // before the early exits: every lane of the workgroup writes its table words
#endif
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  const size_t g = base + i;
  if (cls[g] != REJ_OK) return;
  auto load = [&](int step, int k) {
    const int s = line_slot(step, k);
    return line{ld_fp2<BLS_LN_AUX_LD>(LN, sub, i, s + 0), ld_fp2<BLS_LN_AUX_LD>(LN, sub, i, s + 2),
                ld_fp2<BLS_LN_AUX_LD>(LN, sub, i, s + 4)};
  };
  // miller_f_from_lines (pairing.h) with the line-pair product parked in LDS
  fp12 f = fp12_one();
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int rep = 0; rep < 2; rep++) {
      if (rep == 1 && !((BLS_X_ABS >> b) & 1ull)) break;
#if BLS_F6_LIN
      if (rep == 0 && b != 62) f = fp12_sqr_lin(f, KpLds16());
#else
      if (rep == 0 && b != 62) f = fp12_sqr(f);
#endif
      {
        const fp12 L = line_mul_line(load(step, 0), load(step, 1));
        if (step == 0) {  // f = 1 * L: the first line pair is f itself
          f = L;
          step++;
          continue;
        }
        mf_put(0, L.c0.c0);
        mf_put(1, L.c0.c1);
        mf_put(2, L.c0.c2);
        mf_put(3, L.c1.c1);
        mf_put(4, L.c1.c2);
      }
      f = fp12_mul_by_line_pair_lds(f);
      step++;
    }
  }
  st_fp12(F, cnt, g, fp12_conj(f));
}

// ------------------------------------------------------------------ 3-lane f pass (tri.h)
// Same f as k_miller_f, each Fp12 spread over 3 lanes (Fp4 thirds), 21 beacons per wave: per step
// f = f^2 (tri_sqr_lp), L = l_0 l_1 (tri_line_pair: 2 Fp2 products per lane), f = f L (tri_mul_lp).
// Steps s = 0..67 follow miller_f_from_lines; bit s of MILLER_SQ says whether step s squares first.
constexpr uint64_t miller_sq_bits(int half) {
  uint64_t m = 0;
  int s = 0;
  for (int i = 62; i >= 0; i--) {
    if (i != 62 && s / 64 == half) m |= 1ull << (s % 64);
    s++;
    if ((BLS_X_ABS >> i) & 1ull) s++;  // addition step: no squaring
  }
  return m;
}
constexpr uint64_t MILLER_SQ_LO = miller_sq_bits(0), MILLER_SQ_HI = miller_sq_bits(1);

#ifndef BLS_MILLER_TRI_MAX
#define BLS_MILLER_TRI_MAX 65536
#endif
constexpr size_t kMillerTriMax = BLS_MILLER_TRI_MAX;

#ifndef BLS_WPE_MILLER_TRI
#define BLS_WPE_MILLER_TRI 2
#endif

BLS_KERNEL(BLS_WPE_MILLER_TRI) k_miller_f_tri(const uint32_t* LN, const uint8_t* cls, size_t cnt, size_t base,
                                              size_t m, size_t sub, uint32_t* F, uint32_t* park) {
  const tri_lane t = tri_lane_id();
  const size_t ir = (size_t)blockIdx.x * TRI_GROUPS + t.group;
  const bool in_range = t.group < TRI_GROUPS && ir < m;
  const size_t i = in_range ? ir : m - 1;  // dummy lanes compute on a real row, never store
  const bool live = in_range && cls[base + i] == REJ_OK;
  const size_t park_n = (size_t)gridDim.x * TPB, park_i = (size_t)blockIdx.x * TPB + t.lane;
  fp4 A;
#pragma unroll 1
  for (int s = 0; s < MILLER_STEPS; s++) {
    const bool sq = ((s < 64 ? MILLER_SQ_LO >> s : MILLER_SQ_HI >> (s - 64)) & 1ull) != 0;
    if (sq) A = tri_sqr_lp(t, A);
    const int s0 = line_slot(s, 0), s1 = line_slot(s, 1);
    // c is lane-role dependent: the line's 6 slots as one object, the slot in the VGPR offset
    auto la = [&](int c) {
      size_t j = i;
      asm volatile("" : "+v"(j));
      return ld_fp2_v<BLS_LN_AUX_LD>(LN + (size_t)s0 * 12 * sub, sub, j, 2 * c);
    };
    auto lb = [&](int c) {
      size_t j = i;
      asm volatile("" : "+v"(j));
      return ld_fp2_v<BLS_LN_AUX_LD>(LN + (size_t)s1 * 12 * sub, sub, j, 2 * c);
    };
    const fp4 L = tri_line_pair(t, la, lb);
    if (s == 0) {
      A = L;  // f = 1 * L
    } else {
      A = tri_mul_lp(t, A, L, park, park_n, park_i);
    }
  }
  A = tri_conj(t, A);
  if (live) tri_store(F, cnt, base + i, t.role, A);
}

// ------------------------------------------------------------------ launchers
// The line staging (MILLER_LINE_WORDS per beacon) holds `sub` beacons; the chunk runs in sub-chunks
// (one when sub >= cnt, which is what the host does: every sub-chunk adds a wave tail to both passes).
void launch_miller(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
                   const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
                   uint32_t* F, uint32_t* LN, size_t sub, uint32_t* park, hipStream_t st) {
  if (!cnt) return;
  for (size_t b = 0; b < cnt; b += sub) {
    const size_t m = cnt - b < sub ? cnt - b : sub;
    hipLaunchKernelGGL(k_miller_lines, dim3(2 * grid_for(m)), dim3(TPB), 0, st, pk_tab, pk_inf, pk_idx, H, h_inf,
                       S, s_inf, cls, cnt, b, m, sub, LN);
    // Below one full wave round of the single-lane pass (1 wave/SIMD x 1024 SIMDs x 64 lanes) the GPU is
    // not full and latency decides: the 3-lane pass runs 27.6 k instructions per lane-step against
    // 73.7 k. At full occupancy the single-lane pass has the higher throughput (profiles/r02_*).
    if (m <= kMillerTriMax) {
      hipLaunchKernelGGL(k_miller_f_tri, dim3((unsigned)((m + TRI_GROUPS - 1) / TRI_GROUPS)), dim3(TPB), 0, st, LN,
                         cls, cnt, b, m, sub, F, park);
    } else {
      hipLaunchKernelGGL(k_miller_f, dim3(grid_for(m)), dim3(TPB), 0, st, LN, cls, cnt, b, m, sub, F);
    }
  }
}

}  // namespace blsk

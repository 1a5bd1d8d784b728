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
      st_fp2(LN, sub, i, s + 0, o.a0);
      st_fp2(LN, sub, i, s + 2, o.a1);
      st_fp2(LN, sub, i, s + 4, o.a4);
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
    auto put = [&](int c, const fp2& v) { st_fp2(LN, sub, i, line_slot(step, k) + 2 * c, v); };
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
// fp6_mul(a, b) (tower.h, Karatsuba) with b's components read through lb
template <typename LB>
DI fp6 fp6_mul_lb(const fp6& a, LB lb) {
  fp2 t0 = fp2_mul(a.c0, lb(0));
  fp2 t1 = fp2_mul(a.c1, lb(1));
  fp2 t2 = fp2_mul(a.c2, lb(2));
  fp2 c0 = fp2_add(fp2_mul_xi(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c1, a.c2), fp2_add_lazy(lb(1), lb(2))), t1), t2)), t0);
  fp2 c1 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c1), fp2_add_lazy(lb(0), lb(1))), t0), t1), fp2_mul_xi(t2));
  fp2 c2 = fp2_add(fp2_sub(fp2_sub(fp2_mul(fp2_add_lazy(a.c0, a.c2), fp2_add_lazy(lb(0), lb(2))), t0), t2), t1);
  return {c0, c1, c2};
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
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  const size_t g = base + i;
  if (cls[g] != REJ_OK) return;
  auto load = [&](int step, int k) {
    const int s = line_slot(step, k);
    return line{ld_fp2(LN, sub, i, s + 0), ld_fp2(LN, sub, i, s + 2), ld_fp2(LN, sub, i, s + 4)};
  };
  // miller_f_from_lines (pairing.h) with the line-pair product parked in LDS
  fp12 f = fp12_one();
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int rep = 0; rep < 2; rep++) {
      if (rep == 1 && !((BLS_X_ABS >> b) & 1ull)) break;
      if (rep == 0 && b != 62) f = fp12_sqr(f);
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

// ------------------------------------------------------------------ team-of-two f pass
// The f pass of k_miller_f at 2 waves/SIMD: a workgroup of TWO waves runs 64 beacons, wave 0 holds
// the half c0 of every beacon's f = c0 + c1 w (72 VGPRs), wave 1 the half c1. Each Fp6 product of a
// step goes whole to one wave (same products as k_miller_f, no duplicate work), the partner's half
// is read from the workgroup's LDS at each use, and the few partial results the other wave needs go
// through the park (global scratch, the FW staging: 17 Fp2 per beacon, SoA of stride `sub`):
//   square  wave 0: ab = c0 c1              wave 1: t = (c0 + c1)(c0 + v c1)
//           then c0 = t - ab - v ab (wave 0), c1 = 2 ab (wave 1)
//   L       wave 0: l0.a_k l1.b_k (k = 0, 1, 4)   wave 1: the three Karatsuba cross products
//           -> L (5 Fp2) to the park
//   f L     wave 0: t0 = c0 L0 and d_k = X_k Y_k   wave 1: t1 = c1 L1 (L1 = (0, L11, L12)) and the
//           cross products e_ij = (X_i + X_j)(Y_i + Y_j), with X = c0 + c1, Y = L0 + L1
//           then c0 = t0 + v t1 (wave 0), c1 = m - t0 - t1 with m = X Y from d, e (wave 1)
// Per step 18 and 17 Fp2 products against the single lane's 35. Register budget per wave: its half
// (72) + one Fp6 result being accumulated (72) + one in-place Fp2 product (~100), products
// ordered so that each Karatsuba partial is consumed as soon as it is formed.
#ifndef BLS_MILLER_F2
#define BLS_MILLER_F2 0
#endif
static __shared__ uint32_t g_mf2_S[2 * 72 * BLS_LANES];
constexpr int MF2_L = 0, MF2_T0 = 5, MF2_T1 = 8, MF2_D = 11, MF2_E = 14, MF2_SLOTS = 17;  // park Fp2 slots
static_assert(2 * MF2_SLOTS * 12 <= 3 * F_WORDS, "the team f pass parks in FW");

// SoA staging through buffer loads/stores: the lane's byte offset in a VGPR, the word's byte offset
// (word * stride) in an SGPR recomputed at each use (an opaque stride keeps LLVM from hoisting the
// hundreds of distinct offsets into SGPRs and spilling them), no 64-bit VGPR address per word.
struct SoaRsrc {
  __amdgpu_buffer_rsrc_t r;
  uint32_t stride4;  // bytes between two words of one item (SoA stride * 4)
  uint32_t lane4;    // this item's byte offset
};
DI SoaRsrc soa_rsrc(const uint32_t* base, size_t stride, size_t words, size_t i) {
  const size_t bytes = words * stride * 4;
  return {__builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(base), 0,
                                            (int)(bytes < 0x7fffffffu ? bytes : 0x7fffffffu), 0x00020000),
          (uint32_t)(stride * 4), (uint32_t)(i * 4)};
}
DI uint32_t soa_off(const SoaRsrc& s, int word) {
  uint32_t s4 = s.stride4;
  asm volatile("" : "+s"(s4));
  return (uint32_t)word * s4;
}
DI fp2 soa_ld_fp2(const SoaRsrc& s, int slot) {  // Fp slots slot, slot + 1 (12 words each)
  uint32_t lo = s.lane4;
  asm volatile("" : "+v"(lo));  // at the use
  fp2 v;
#pragma unroll
  for (int q = 0; q < 12; q++) {
    v.c0.l[q] = __builtin_amdgcn_raw_buffer_load_b32(s.r, lo, soa_off(s, slot * 12 + q), 0);
    v.c1.l[q] = __builtin_amdgcn_raw_buffer_load_b32(s.r, lo, soa_off(s, slot * 12 + 12 + q), 0);
  }
  return v;
}
DI void soa_st_fp2(const SoaRsrc& s, int slot, const fp2& v) {
#pragma unroll
  for (int q = 0; q < 12; q++) {
    __builtin_amdgcn_raw_buffer_store_b32(v.c0.l[q], s.r, s.lane4, soa_off(s, slot * 12 + q), 0);
    __builtin_amdgcn_raw_buffer_store_b32(v.c1.l[q], s.r, s.lane4, soa_off(s, slot * 12 + 12 + q), 0);
  }
}

// x y for Fp6 x, y given as Fp2 getters X(k), Y(k) (Karatsuba; the cross products first, each
// diagonal product folded into the three outputs as soon as it is formed)
template <class GX, class GY>
DI fp6 mf2_mul6(GX X, GY Y) {
  fp6 c;
  c.c0 = fp2_mul_xi(fp2_mul_inl(fp2_add_lazy(X(1), X(2)), fp2_add_lazy(Y(1), Y(2))));
  BLS_SCHED_FENCE();
  c.c1 = fp2_mul_inl(fp2_add_lazy(X(0), X(1)), fp2_add_lazy(Y(0), Y(1)));
  BLS_SCHED_FENCE();
  c.c2 = fp2_mul_inl(fp2_add_lazy(X(0), X(2)), fp2_add_lazy(Y(0), Y(2)));
  BLS_SCHED_FENCE();
  {
    const fp2 t = fp2_mul_inl(X(0), Y(0));
    c.c0 = fp2_add(c.c0, t);
    c.c1 = fp2_sub(c.c1, t);
    c.c2 = fp2_sub(c.c2, t);
  }
  BLS_SCHED_FENCE();
  {
    const fp2 t = fp2_mul_inl(X(1), Y(1));
    c.c0 = fp2_sub(c.c0, fp2_mul_xi(t));
    c.c1 = fp2_sub(c.c1, t);
    c.c2 = fp2_add(c.c2, t);
  }
  BLS_SCHED_FENCE();
  {
    const fp2 t = fp2_mul_inl(X(2), Y(2));
    const fp2 xt = fp2_mul_xi(t);
    c.c0 = fp2_sub(c.c0, xt);
    c.c1 = fp2_add(c.c1, xt);
    c.c2 = fp2_sub(c.c2, t);
  }
  return c;
}

// x (b1 v + b2 v^2) (tower fp6_mul_by_12): 5 products, partials folded as formed
template <class GX>
DI fp6 mf2_mul6_by_12(GX X, const fp2& b1, const fp2& b2) {
  fp6 c;
  c.c0 = fp2_mul_xi(fp2_mul_inl(fp2_add_lazy(X(1), X(2)), fp2_add_lazy(b1, b2)));
  BLS_SCHED_FENCE();
  c.c1 = fp2_mul_inl(X(0), b1);
  BLS_SCHED_FENCE();
  c.c2 = fp2_mul_inl(X(0), b2);
  BLS_SCHED_FENCE();
  {
    const fp2 t = fp2_mul_inl(X(1), b1);
    c.c0 = fp2_sub(c.c0, fp2_mul_xi(t));
    c.c2 = fp2_add(c.c2, t);
  }
  BLS_SCHED_FENCE();
  {
    const fp2 t = fp2_mul_inl(X(2), b2);
    const fp2 xt = fp2_mul_xi(t);
    c.c0 = fp2_sub(c.c0, xt);
    c.c1 = fp2_add(c.c1, xt);
  }
  return c;
}

__global__ void __launch_bounds__(2 * TPB) __attribute__((amdgpu_waves_per_eu(2)))
k_miller_f2(const uint32_t* LN, const uint8_t* cls, size_t cnt, size_t base, size_t m, size_t sub, uint32_t* F,
            uint32_t* park) {
  const unsigned l = threadIdx.x & 63u;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t ir = (size_t)blockIdx.x * TPB + l;
  const size_t i = ir < m ? ir : m - 1;  // tail lanes compute on a real row, never store
  // Each wave's half of f lives in its LDS slot between the phases (72 words per lane, word-major);
  // products read both halves from LDS at each use, so no half is held in registers across them.
  uint32_t* const S_own = g_mf2_S + w * (72 * BLS_LANES);
  const uint32_t* const S_par = g_mf2_S + (1 - w) * (72 * BLS_LANES);
  auto s_get = [&](const uint32_t* S, int k) {
    unsigned ll = l;
    asm volatile("" : "+v"(ll));  // read at the use
    fp2 v;
#pragma unroll
    for (int q = 0; q < 12; q++) {
      v.c0.l[q] = S[(24 * k + q) * BLS_LANES + ll];
      v.c1.l[q] = S[(24 * k + 12 + q) * BLS_LANES + ll];
    }
    return v;
  };
  auto own = [&](int k) { return s_get(S_own, k); };
  auto par = [&](int k) { return s_get(S_par, k); };
  auto publish = [&](const fp6& v) {
    const fp2 c[3] = {v.c0, v.c1, v.c2};
#pragma unroll
    for (int k = 0; k < 3; k++)
#pragma unroll
      for (int q = 0; q < 12; q++) {
        S_own[(24 * k + q) * BLS_LANES + l] = c[k].c0.l[q];
        S_own[(24 * k + 12 + q) * BLS_LANES + l] = c[k].c1.l[q];
      }
  };
  const SoaRsrc pr = soa_rsrc(park, sub, 2 * MF2_SLOTS * 12, i);
  auto p_put = [&](int slot, const fp2& v) { soa_st_fp2(pr, 2 * slot, v); };
  auto p_get = [&](int slot) { return soa_ld_fp2(pr, 2 * slot); };
  // lines of one step: a resource over that step's 2 x 6 Fp slots
  auto ln_rsrc = [&](int step) { return soa_rsrc(LN + (size_t)line_slot(step, 0) * 12 * sub, sub, 2 * 6 * 12, i); };
  auto sync = [&]() { __syncthreads(); };
  auto gsync = [&]() {  // park (global) writes visible to the partner wave
    __threadfence_block();
    __syncthreads();
  };
  int step = 0;
#pragma unroll 1
  for (int b = 62; b >= 0; b--) {
#pragma unroll 1
    for (int rep = 0; rep < 2; rep++) {
      if (rep == 1 && !((BLS_X_ABS >> b) & 1ull)) break;
      if (rep == 0 && b != 62) {  // f = f^2 (complex squaring)
        sync();  // both halves published
        fp6 r;
        if (w == 0) {
          r = mf2_mul6(own, par);  // ab = c0 c1
        } else {
          // t = (c0 + c1)(c0 + v c1) with c0 the partner's half: v c1 = (xi c1_2, c1_0, c1_1)
          r = mf2_mul6([&](int k) { return fp2_add_lazy(par(k), own(k)); },
                       [&](int k) {
                         return k == 0 ? fp2_add_lazy(par(0), fp2_mul_xi(own(2))) : fp2_add_lazy(par(k), own(k - 1));
                       });
        }
        sync();
        publish(r);
        sync();
        fp6 hn;
        if (w == 0) {  // c0 = t - ab - v ab
          const fp6 vr = fp6_mul_v(r);
          hn.c0 = fp2_sub(fp2_sub(par(0), r.c0), vr.c0);
          hn.c1 = fp2_sub(fp2_sub(par(1), r.c1), vr.c1);
          hn.c2 = fp2_sub(fp2_sub(par(2), r.c2), vr.c2);
        } else {  // c1 = 2 ab
          hn.c0 = fp2_dbl(par(0));
          hn.c1 = fp2_dbl(par(1));
          hn.c2 = fp2_dbl(par(2));
        }
        sync();
        publish(hn);
      }
      // L = l0 l1 (pairing.h line_mul_line), three products per wave; the halves stay in LDS, the
      // exchange and L go through the park (T0 slots hold wave 0's diagonal products meanwhile)
      {
        const SoaRsrc lr = ln_rsrc(step);
        auto ln = [&](int, int k, int c) { return soa_ld_fp2(lr, 6 * k + 2 * c); };
        if (w == 0) {
          p_put(MF2_T0 + 0, fp2_mul_inl(ln(step, 0, 0), ln(step, 1, 0)));  // t00
          BLS_SCHED_FENCE();
          p_put(MF2_T0 + 1, fp2_mul_inl(ln(step, 0, 1), ln(step, 1, 1)));  // t11
          BLS_SCHED_FENCE();
          p_put(MF2_T0 + 2, fp2_mul_inl(ln(step, 0, 2), ln(step, 1, 2)));  // t44
        } else {
          p_put(MF2_T1 + 0, fp2_mul_inl(fp2_add_lazy(ln(step, 0, 0), ln(step, 0, 1)),
                                        fp2_add_lazy(ln(step, 1, 0), ln(step, 1, 1))));  // x01
          BLS_SCHED_FENCE();
          p_put(MF2_T1 + 1, fp2_mul_inl(fp2_add_lazy(ln(step, 0, 0), ln(step, 0, 2)),
                                        fp2_add_lazy(ln(step, 1, 0), ln(step, 1, 2))));  // x04
          BLS_SCHED_FENCE();
          p_put(MF2_T1 + 2, fp2_mul_inl(fp2_add_lazy(ln(step, 0, 1), ln(step, 0, 2)),
                                        fp2_add_lazy(ln(step, 1, 1), ln(step, 1, 2))));  // x14
        }
        gsync();
        if (w == 0) {  // L00 = t00 + xi t44, L02 = t11
          p_put(MF2_L + 0, fp2_add(p_get(MF2_T0 + 0), fp2_mul_xi(p_get(MF2_T0 + 2))));
          p_put(MF2_L + 2, p_get(MF2_T0 + 1));
        } else {  // L01 = x01 - t00 - t11, L11 = x04 - t00 - t44, L12 = x14 - t11 - t44
          p_put(MF2_L + 1, fp2_sub(fp2_sub(p_get(MF2_T1 + 0), p_get(MF2_T0 + 0)), p_get(MF2_T0 + 1)));
          p_put(MF2_L + 3, fp2_sub(fp2_sub(p_get(MF2_T1 + 1), p_get(MF2_T0 + 0)), p_get(MF2_T0 + 2)));
          p_put(MF2_L + 4, fp2_sub(fp2_sub(p_get(MF2_T1 + 2), p_get(MF2_T0 + 1)), p_get(MF2_T0 + 2)));
        }
        gsync();
      }
      if (step == 0) {  // f = 1 * L: the first line pair is f itself
        if (w == 0) {
          publish({p_get(MF2_L + 0), p_get(MF2_L + 1), p_get(MF2_L + 2)});
        } else {
          publish({fp2_zero(), p_get(MF2_L + 3), p_get(MF2_L + 4)});
        }
        step++;
        continue;
      }
      // f = f L (pairing.h fp12_mul_by_line_pair): X = c0 + c1, Y = L0 + L1 = (L00, L01 + L11, L02 + L12)
      sync();  // both halves published
      auto X = [&](int k) { return fp2_add_lazy(par(k), own(k)); };
      auto Y = [&](int k) { return k == 0 ? p_get(MF2_L + 0) : fp2_add_lazy(p_get(MF2_L + k), p_get(MF2_L + 2 + k)); };
      if (w == 0) {
        const fp6 t0 = mf2_mul6(own, [&](int k) { return p_get(MF2_L + k); });
        p_put(MF2_T0 + 0, t0.c0);
        p_put(MF2_T0 + 1, t0.c1);
        p_put(MF2_T0 + 2, t0.c2);
        BLS_SCHED_FENCE();
        p_put(MF2_D + 0, fp2_mul_inl(X(0), Y(0)));
        BLS_SCHED_FENCE();
        p_put(MF2_D + 1, fp2_mul_inl(X(1), Y(1)));
        BLS_SCHED_FENCE();
        p_put(MF2_D + 2, fp2_mul_inl(X(2), Y(2)));
      } else {
        const fp6 t1 = mf2_mul6_by_12(own, p_get(MF2_L + 3), p_get(MF2_L + 4));
        p_put(MF2_T1 + 0, t1.c0);
        p_put(MF2_T1 + 1, t1.c1);
        p_put(MF2_T1 + 2, t1.c2);
        BLS_SCHED_FENCE();
        p_put(MF2_E + 0, fp2_mul_inl(fp2_add_lazy(X(1), X(2)), fp2_add_lazy(Y(1), Y(2))));  // e12
        BLS_SCHED_FENCE();
        p_put(MF2_E + 1, fp2_mul_inl(fp2_add_lazy(X(0), X(1)), fp2_add_lazy(Y(0), Y(1))));  // e01
        BLS_SCHED_FENCE();
        p_put(MF2_E + 2, fp2_mul_inl(fp2_add_lazy(X(0), X(2)), fp2_add_lazy(Y(0), Y(2))));  // e02
      }
      gsync();
      fp6 hn;
      if (w == 0) {  // c0 = t0 + v t1
        hn.c0 = fp2_add(p_get(MF2_T0 + 0), fp2_mul_xi(p_get(MF2_T1 + 2)));
        hn.c1 = fp2_add(p_get(MF2_T0 + 1), p_get(MF2_T1 + 0));
        hn.c2 = fp2_add(p_get(MF2_T0 + 2), p_get(MF2_T1 + 1));
      } else {  // c1 = m - t0 - t1, m = X Y from d, e (Karatsuba)
        const fp2 d0 = p_get(MF2_D + 0), d1 = p_get(MF2_D + 1), d2 = p_get(MF2_D + 2);
        hn.c0 = fp2_sub(fp2_sub(fp2_add(d0, fp2_mul_xi(fp2_sub(fp2_sub(p_get(MF2_E + 0), d1), d2))), p_get(MF2_T0 + 0)),
                        p_get(MF2_T1 + 0));
        hn.c1 = fp2_sub(fp2_sub(fp2_add(fp2_sub(fp2_sub(p_get(MF2_E + 1), d0), d1), fp2_mul_xi(d2)), p_get(MF2_T0 + 1)),
                        p_get(MF2_T1 + 1));
        hn.c2 = fp2_sub(fp2_sub(fp2_add(fp2_sub(fp2_sub(p_get(MF2_E + 2), d0), d2), d1), p_get(MF2_T0 + 2)),
                        p_get(MF2_T1 + 2));
      }
      publish(hn);  // the partner read this wave's old half before the last sync
      step++;
    }
  }
  if (ir < m && cls[base + ir] == REJ_OK) {
    const size_t g = base + ir;
    if (w == 0) {  // f = conj(f): c1 negated
      st_fp2(F, cnt, g, 0, own(0));
      st_fp2(F, cnt, g, 2, own(1));
      st_fp2(F, cnt, g, 4, own(2));
    } else {
      st_fp2(F, cnt, g, 6, fp2_neg(own(0)));
      st_fp2(F, cnt, g, 8, fp2_neg(own(1)));
      st_fp2(F, cnt, g, 10, fp2_neg(own(2)));
    }
  }
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
      return ld_fp2_v(LN + (size_t)s0 * 12 * sub, sub, j, 2 * c);
    };
    auto lb = [&](int c) {
      size_t j = i;
      asm volatile("" : "+v"(j));
      return ld_fp2_v(LN + (size_t)s1 * 12 * sub, sub, j, 2 * c);
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
// The line staging (MILLER_LINE_WORDS per beacon) holds `sub` beacons; the chunk runs in sub-chunks.
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
    } else if (BLS_MILLER_F2) {
      hipLaunchKernelGGL(k_miller_f2, dim3(grid_for(m)), dim3(2 * TPB), 0, st, LN, cls, cnt, b, m, sub, F, park);
    } else {
      hipLaunchKernelGGL(k_miller_f, dim3(grid_for(m)), dim3(TPB), 0, st, LN, cls, cnt, b, m, sub, F);
    }
  }
}

}  // namespace blsk

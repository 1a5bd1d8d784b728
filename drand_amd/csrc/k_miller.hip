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
BLS_KERNEL(BLS_WPE_LINES)
k_miller_lines(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
               const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
               size_t base, size_t m, size_t sub, uint32_t* LN) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= m) return;
  const size_t g = base + i;
  if (cls[g] != REJ_OK) return;
  const uint32_t kk = pk_idx ? pk_idx[g] : 0u;
  const bool act[2] = {!(pk_inf[kk] | h_inf[g]), !s_inf[g]};
#pragma unroll 1
  for (int k = 0; k < 2; k++) {
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
    g1a P;
    if (k == 0) {
#pragma unroll
      for (int w = 0; w < 12; w++) {
        P.x.l[w] = pk_tab[(size_t)kk * G1_WORDS + w];
        P.y.l[w] = pk_tab[(size_t)kk * G1_WORDS + 12 + w];
      }
    } else {
      P.x = fp_load_const(G1_GEN_X);
      P.y = fp_load_const(G1_GEN_NEG_Y);
    }
    miller_lines(P, load_q, emit);
  }
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
  st_fp12(F, cnt, g, miller_f_from_lines(load));
}

// ------------------------------------------------------------------ launchers
// The line staging (MILLER_LINE_WORDS per beacon) holds `sub` beacons; the chunk runs in sub-chunks.
void launch_miller(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
                   const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
                   uint32_t* F, uint32_t* LN, size_t sub, hipStream_t st) {
  if (!cnt) return;
  for (size_t b = 0; b < cnt; b += sub) {
    const size_t m = cnt - b < sub ? cnt - b : sub;
    hipLaunchKernelGGL(k_miller_lines, dim3(grid_for(m)), dim3(TPB), 0, st, pk_tab, pk_inf, pk_idx, H, h_inf, S,
                       s_inf, cls, cnt, b, m, sub, LN);
    hipLaunchKernelGGL(k_miller_f, dim3(grid_for(m)), dim3(TPB), 0, st, LN, cls, cnt, b, m, sub, F);
  }
}

}  // namespace blsk

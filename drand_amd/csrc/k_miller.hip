// Stage 3: two-pair multi-Miller loop e(pk, H) * e(-g1, sigma), one lane per beacon.
// kilic Engine.AddPair / AddPairInv [ext] via kyber-bls12381 ValidatePairing.
#include "kcommon.h"

namespace blsk {

__global__ void __launch_bounds__(TPB) k_miller(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx,
                                                const uint32_t* H, const uint8_t* h_inf, const uint32_t* S,
                                                const uint8_t* s_inf, const uint8_t* cls, size_t cnt, uint32_t* F) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  if (cls[i] != REJ_OK) return;
  const uint32_t k = pk_idx ? pk_idx[i] : 0u;
  g1a P[2];
  g2a Q[2];
  bool act[2];
#pragma unroll
  for (int w = 0; w < 12; w++) {
    P[0].x.l[w] = pk_tab[(size_t)k * G1_WORDS + w];
    P[0].y.l[w] = pk_tab[(size_t)k * G1_WORDS + 12 + w];
  }
  P[1].x = fp_load_const(G1_GEN_X);
  P[1].y = fp_load_const(G1_GEN_NEG_Y);
  Q[0].x = ld_fp2(H, cnt, i, 0);
  Q[0].y = ld_fp2(H, cnt, i, 2);
  Q[1].x = ld_fp2(S, cnt, i, 0);
  Q[1].y = ld_fp2(S, cnt, i, 2);
  act[0] = !(pk_inf[k] | h_inf[i]);
  act[1] = !s_inf[i];
  fp12 f = miller_loop_2(P, Q, act);
  st_fp12(F, cnt, i, f);
}

// ------------------------------------------------------------------ launchers
void launch_miller(const uint32_t* pk_tab, const uint8_t* pk_inf, const uint32_t* pk_idx, const uint32_t* H,
                   const uint8_t* h_inf, const uint32_t* S, const uint8_t* s_inf, const uint8_t* cls, size_t cnt,
                   uint32_t* F, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_miller, dim3(grid_for(cnt)), dim3(TPB), 0, st, pk_tab, pk_inf, pk_idx, H, h_inf, S, s_inf,
                     cls, cnt, F);
}

}  // namespace blsk

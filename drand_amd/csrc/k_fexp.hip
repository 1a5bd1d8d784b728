// Stage 4: final exponentiation and the == 1 test, one lane per beacon. kilic Engine.Check [ext].
#include "kcommon.h"

namespace blsk {

__global__ void __launch_bounds__(TPB) k_final_exp(const uint32_t* F, size_t cnt, uint8_t* cls) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  if (cls[i] != REJ_OK) return;
  fp12 f = ld_fp12(F, cnt, i);
  fp12 e = final_exponentiation(f);
  if (!fp12_is_one(e)) cls[i] = REJ_PAIRING;
}

// ------------------------------------------------------------------ launchers
void launch_final_exp(const uint32_t* F, size_t cnt, uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_final_exp, dim3(grid_for(cnt)), dim3(TPB), 0, st, F, cnt, cls);
}

}  // namespace blsk

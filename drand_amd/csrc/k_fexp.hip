// Stage 4: final exponentiation and the == 1 test, one lane per beacon. kilic Engine.Check [ext].
// Six launches per chunk (pairing.h fexp_easy / fexp_step<0..4>), each holding at most two Fp12
// values in registers; intermediate Fp12 values live in HBM staging buffers (SoA, 576 B per beacon)
// and are re-read at each use, which keeps every kernel free of scratch spills.
#include "kcommon.h"

namespace blsk {

BLS_KERNEL(BLS_WPE_FEXP) k_fexp_easy(const uint32_t* F, size_t cnt, const uint8_t* cls, uint32_t* G) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  st_fp12(G, cnt, i, fexp_easy(ld_fp12(F, cnt, i)));
}

template <int MODE>
BLS_KERNEL(BLS_WPE_FEXP) k_fexp_step(const uint32_t* X, const uint32_t* C, const uint32_t* G, size_t cnt,
                                                   uint8_t* cls, uint32_t* OUT) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  // the re-reads must stay at their use sites: an opaque copy of the index keeps LICM from hoisting
  // them (a hoisted Fp12 would pin 144 VGPRs across the squaring loops)
  auto at = [&](const uint32_t* B) {
    size_t j = i;
    asm volatile("" : "+v"(j));
    return ld_fp12(B, cnt, j);
  };
  fp12 r = fexp_step<MODE>([&]() { return at(X); }, [&]() { return at(C); }, [&]() { return at(G); });
  if (MODE < 4) {
    st_fp12(OUT, cnt, i, r);
  } else if (!fp12_is_one(r)) {
    cls[i] = REJ_PAIRING;
  }
}

// ------------------------------------------------------------------ launchers
// F (Miller output) is consumed by the easy part and then reused as scratch; W holds 3 more Fp12
// staging slots of cnt entries each (G, B, C).
void launch_final_exp(uint32_t* F, uint32_t* W, size_t cnt, uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  uint32_t* G = W;
  uint32_t* B = W + cnt * F_WORDS;
  uint32_t* C = W + 2 * cnt * F_WORDS;
  const dim3 grid(grid_for(cnt)), blk(TPB);
  hipLaunchKernelGGL(k_fexp_easy, grid, blk, 0, st, F, cnt, cls, G);
  hipLaunchKernelGGL(k_fexp_step<0>, grid, blk, 0, st, G, nullptr, nullptr, cnt, cls, F);  // a -> F
  hipLaunchKernelGGL(k_fexp_step<1>, grid, blk, 0, st, F, nullptr, nullptr, cnt, cls, B);  // b -> B
  hipLaunchKernelGGL(k_fexp_step<2>, grid, blk, 0, st, B, nullptr, nullptr, cnt, cls, C);  // c -> C
  hipLaunchKernelGGL(k_fexp_step<3>, grid, blk, 0, st, C, nullptr, nullptr, cnt, cls, F);  // t -> F
  hipLaunchKernelGGL(k_fexp_step<4>, grid, blk, 0, st, F, C, G, cnt, cls, nullptr);
}

}  // namespace blsk

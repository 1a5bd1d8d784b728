// Stage 2: signature decompression (ZCash format) + psi-based G2 subgroup check, and the final
// verdict reduction (bitmap + first bad index). kilic G2.FromCompressed order [ext].
#include "kcommon.h"

namespace blsk {

// Two kernels: decoding (flag, infinity form, x < p, the Fp2 square root -- two Fp exponentiations with
// a small live state, run at high occupancy) and the psi subgroup check ([x] chain on a Jacobian point:
// many short calls). The reject order is kilic's: the subgroup check only runs on decoded points.
#ifndef BLS_WPE_SUBGROUP
#define BLS_WPE_SUBGROUP 2
#endif

BLS_KERNEL(BLS_WPE_DECOMP) k_decompress_g2(const uint8_t* sigs, size_t stride, size_t offset, size_t base,
                                           size_t cnt, uint32_t* S, uint8_t* s_inf, uint8_t* cls) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  uint8_t buf[96];
  const uint8_t* p = sigs + (base + i) * stride + offset;
  for (int k = 0; k < 96; k++) buf[k] = p[k];
  g2a a;
  bool inf;
  uint8_t c = g2_decompress(buf, a, inf, false);
  if (c != REJ_OK) {
    a.x = fp2_zero();
    a.y = fp2_zero();
    inf = true;
  }
  st_fp2(S, cnt, i, 0, a.x);
  st_fp2(S, cnt, i, 2, a.y);
  s_inf[i] = inf;
  cls[i] = c;
}

BLS_KERNEL(BLS_WPE_SUBGROUP) k_subgroup_g2(uint32_t* S, uint8_t* s_inf, uint8_t* cls, size_t cnt) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK || s_inf[i]) return;
  // the point is re-read at its uses (psi, the 5 additions) instead of living across the chain
  const bool in = g2_in_subgroup_aff_reload([&]() {
    size_t j = i;
    asm volatile("" : "+v"(j));
    return g2a{ld_fp2(S, cnt, j, 0), ld_fp2(S, cnt, j, 2)};
  });
  if (!in) {
    st_fp2(S, cnt, i, 0, fp2_zero());
    st_fp2(S, cnt, i, 2, fp2_zero());
    s_inf[i] = 1;
    cls[i] = REJ_NOT_IN_SUBGROUP;
  }
}

// first_bad receives label0 + (index of the first reject): label0 = first_round gives the ROUND
// (chained device batches), 0 the batch index (host entry points add their own round mapping).
__global__ void __launch_bounds__(256) k_finish(const uint8_t* cls, size_t base, size_t cnt, uint64_t* bitmap,
                                                unsigned long long* first_bad, uint64_t label0) {
  size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const bool in = i < cnt;
  const bool ok = in && cls[i] == REJ_OK;
  const bool bad = in && !ok;
  // base is a multiple of 64, so each wave owns one bitmap word
  const unsigned long long okm = __ballot(ok);
  const unsigned long long badm = __ballot(bad);
  const int lane = threadIdx.x & 63;
  const size_t wave0 = i - lane;
  if (lane == 0 && wave0 < cnt) {
    bitmap[(base + wave0) >> 6] = okm;
    if (badm) atomicMin(first_bad, (unsigned long long)(label0 + base + wave0 + __builtin_ctzll(badm)));
  }
}

// ------------------------------------------------------------------ launchers
void launch_decompress_g2(const uint8_t* sigs, size_t stride, size_t offset, size_t base, size_t cnt, uint32_t* S,
                          uint8_t* s_inf, uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_decompress_g2, dim3(grid_for(cnt)), dim3(TPB), 0, st, sigs, stride, offset, base, cnt, S,
                     s_inf, cls);
  hipLaunchKernelGGL(k_subgroup_g2, dim3(grid_for(cnt)), dim3(TPB), 0, st, S, s_inf, cls, cnt);
}

void launch_finish(const uint8_t* cls, size_t base, size_t cnt, uint64_t* bitmap, unsigned long long* first_bad,
                   uint64_t label0, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_finish, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, cls, base, cnt, bitmap,
                     first_bad, label0);
}

}  // namespace blsk

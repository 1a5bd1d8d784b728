// Raw building-block test hooks (parity tests against the CPU oracle; not used by the product path).
#include "kcommon.h"

namespace blsk {

// ------------------------------------------------------------------ test hooks
__global__ void k_test_fp_mul(const uint32_t* a, const uint32_t* b, size_t cnt, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  fp x, y;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    x.l[w] = a[i * 12 + w];
    y.l[w] = b[i * 12 + w];
  }
  fp r = fp_from_mont(fp_mul(fp_to_mont(x), fp_to_mont(y)));
#pragma unroll
  for (int w = 0; w < 12; w++) out[i * 12 + w] = r.l[w];
}

// raw affine P (24 words: x, y) and Q (48 words: x.c0, x.c1, y.c0, y.c1) -> e(P, Q)^3 raw (144 words,
// tower order c0.c0.c0, c0.c0.c1, c0.c1.c0, ..., c1.c2.c1)
__global__ void __launch_bounds__(TPB) k_test_pairing(const uint32_t* p_tab, const uint32_t* q_aff, size_t cnt,
                                                      uint32_t* out_f) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  fp v[6];
#pragma unroll
  for (int s = 0; s < 2; s++)
#pragma unroll
    for (int w = 0; w < 12; w++) v[s].l[w] = p_tab[i * 24 + s * 12 + w];
  g1a P1[1] = {{fp_to_mont(v[0]), fp_to_mont(v[1])}};
#pragma unroll
  for (int s = 0; s < 4; s++)
#pragma unroll
    for (int w = 0; w < 12; w++) v[s].l[w] = q_aff[i * 48 + s * 12 + w];
  g2a Q1[1] = {{{fp_to_mont(v[0]), fp_to_mont(v[1])}, {fp_to_mont(v[2]), fp_to_mont(v[3])}}};
  bool act[1] = {true};
  fp12 f = final_exponentiation(miller_loop_multi<1>(P1, Q1, act));
  const fp2* c[6] = {&f.c0.c0, &f.c0.c1, &f.c0.c2, &f.c1.c0, &f.c1.c1, &f.c1.c2};
#pragma unroll
  for (int s = 0; s < 6; s++) {
    fp r0 = fp_from_mont(c[s]->c0), r1 = fp_from_mont(c[s]->c1);
#pragma unroll
    for (int w = 0; w < 12; w++) {
      out_f[i * 144 + s * 24 + w] = r0.l[w];
      out_f[i * 144 + s * 24 + 12 + w] = r1.l[w];
    }
  }
}

// SoA Montgomery affine G2 staging -> raw AoS words (x.c0, x.c1, y.c0, y.c1)
__global__ void k_test_unpack_g2(const uint32_t* H, size_t cnt, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
#pragma unroll
  for (int s = 0; s < 4; s++) {
    fp v = fp_from_mont(ld_fp(H, cnt, i, s));
#pragma unroll
    for (int w = 0; w < 12; w++) out[i * 48 + s * 12 + w] = v.l[w];
  }
}

// raw AoS Fp12 (144 words, tower order) <-> Montgomery SoA staging (soa.h slot order is the same)
__global__ void k_test_pack_fp12(const uint32_t* f, size_t cnt, uint32_t* F) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  for (int s = 0; s < 12; s++) {
    fp v;
#pragma unroll
    for (int w = 0; w < 12; w++) v.l[w] = f[i * 144 + s * 12 + w];
    st_fp(F, cnt, i, s, fp_to_mont(v));
  }
}

__global__ void k_test_unpack_fp12(const uint32_t* F, size_t cnt, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  for (int s = 0; s < 12; s++) {
    fp v = fp_from_mont(ld_fp(F, cnt, i, s));
#pragma unroll
    for (int w = 0; w < 12; w++) out[i * 144 + s * 12 + w] = v.l[w];
  }
}

// one-lane register final exponentiation (pairing.h final_exponentiation) on SoA staging
__global__ void __launch_bounds__(TPB) k_test_final_exp_ref(const uint32_t* F, size_t cnt, uint32_t* out) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  st_fp12(out, cnt, i, final_exponentiation(ld_fp12(F, cnt, i)));
}

// ------------------------------------------------------------------ launchers
void launch_test_pack_fp12(const uint32_t* f, size_t cnt, uint32_t* F, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_pack_fp12, dim3(grid_for(cnt)), dim3(TPB), 0, st, f, cnt, F);
}

void launch_test_unpack_fp12(const uint32_t* F, size_t cnt, uint32_t* out, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_unpack_fp12, dim3(grid_for(cnt)), dim3(TPB), 0, st, F, cnt, out);
}

void launch_test_final_exp_ref(const uint32_t* F, size_t cnt, uint32_t* out, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_final_exp_ref, dim3(grid_for(cnt)), dim3(TPB), 0, st, F, cnt, out);
}

void launch_test_fp_mul(const uint32_t* a, const uint32_t* b, size_t cnt, uint32_t* out, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_fp_mul, dim3(grid_for(cnt)), dim3(TPB), 0, st, a, b, cnt, out);
}

void launch_test_pairing(const uint32_t* p_tab, const uint32_t* q_aff, size_t cnt, uint32_t* out_f, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_pairing, dim3(grid_for(cnt)), dim3(TPB), 0, st, p_tab, q_aff, cnt, out_f);
}

void launch_test_unpack_g2(const uint32_t* H, size_t cnt, uint32_t* out, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_test_unpack_g2, dim3(grid_for(cnt)), dim3(TPB), 0, st, H, cnt, out);
}

}  // namespace blsk

// Group setup, threshold (tbls) and signing kernels, (group part).
//   G1 decode          : chain.InfoFromProto / key.StringToPoint (chain/convert.go:15-18) [ext kilic]
//   PubPoly.Eval(i)    : kyber share.PubPoly (used by tbls.VerifyPartial, node.go:112) [ext]
//   Lagrange / Recover : kyber share.RecoverCommit (tbls.Recover, chain/beacon/chain.go:136) [ext]
//   Sign               : tbls.Sign / bls.Sign (chain/beacon/crypto.go:58) [ext]
//   gen_chained        : client/test/result/mock/result.go:98-132 (synthetic chained history)
#include "kcommon.h"

namespace blsk {


// ------------------------------------------------------------------ Fr (scalar field) helpers
struct fr {
  uint32_t l[8];
};

DI fr fr_mul(const fr& a, const fr& b) {  // CIOS, top limb of r < 2^31 - 1
  uint32_t t[8];
#pragma unroll
  for (int j = 0; j < 8; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.l[i];
    uint64_t A = (uint64_t)a.l[0] * bi + t[0];
    const uint32_t m = (uint32_t)A * FR_INV32;
    uint64_t C = (uint64_t)m * FR_RAW[0] + (uint32_t)A;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      A = (uint64_t)a.l[j] * bi + t[j] + (A >> 32);
      C = (uint64_t)m * FR_RAW[j] + (uint32_t)A + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[7] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  uint32_t d[8];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_subc(t[i], FR_RAW[i], br, &br);
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = br ? t[i] : d[i];
  return r;
}

DI fr fr_small(uint32_t v) {  // Montgomery form of a small integer
  fr raw = {{v, 0, 0, 0, 0, 0, 0, 0}};
  fr r2;
#pragma unroll
  for (int i = 0; i < 8; i++) r2.l[i] = FR_R2[i];
  return fr_mul(raw, r2);
}

DI fr fr_sub(const fr& a, const fr& b) {
  uint32_t d[8];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d[i] = __builtin_subc(a.l[i], b.l[i], br, &br);
  uint32_t m = br ? 0xffffffffu : 0u;
  unsigned c = 0;
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = __builtin_addc(d[i], FR_RAW[i] & m, c, &c);
  return r;
}

DI fr fr_inv(const fr& a) {  // a^(r-2)
  fr r;
#pragma unroll
  for (int i = 0; i < 8; i++) r.l[i] = FR_ONE[i];
  for (int w = 7; w >= 0; w--) {
    for (int b = 31; b >= 0; b--) {
      r = fr_mul(r, r);
      if ((EXP_R_MINUS_2[w] >> b) & 1u) r = fr_mul(r, a);
    }
  }
  return r;
}

// ------------------------------------------------------------------ G1 decode (group setup)
DI void st_g1(uint32_t* tab, size_t k, const g1a& a) {
#pragma unroll
  for (int w = 0; w < 12; w++) {
    tab[k * G1_WORDS + w] = a.x.l[w];
    tab[k * G1_WORDS + 12 + w] = a.y.l[w];
  }
}

DI g1a ld_g1(const uint32_t* tab, size_t k) {
  g1a a;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    a.x.l[w] = tab[k * G1_WORDS + w];
    a.y.l[w] = tab[k * G1_WORDS + 12 + w];
  }
  return a;
}

__global__ void __launch_bounds__(TPB) k_decompress_g1(const uint8_t* in, size_t cnt, uint32_t* tab, uint8_t* inf,
                                                       uint8_t* cls) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  uint8_t buf[48];
  for (int k = 0; k < 48; k++) buf[k] = in[i * 48 + k];
  g1a a;
  bool is_inf;
  uint8_t c = g1_decompress(buf, a, is_inf);
  if (c != REJ_OK) {
    a.x = fp_zero();
    a.y = fp_zero();
    is_inf = true;
  }
  st_g1(tab, i, a);
  inf[i] = is_inf;
  cls[i] = c;
}

// PubPoly.Eval(idx): sum_j C_j (idx+1)^j by Horner, x = idx + 1 < 2^17
__global__ void __launch_bounds__(TPB) k_pubpoly_eval(const uint32_t* commits, const uint8_t* commit_inf, uint32_t t,
                                                      const uint32_t* idx, size_t cnt, uint32_t* out_tab,
                                                      uint8_t* out_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  const uint32_t x = idx[i] + 1u;
  g1j v = jac_infinity<fp>();
  for (int j = (int)t - 1; j >= 0; j--) {
    // v = [x] v
    g1j acc = jac_infinity<fp>();
    for (int b = 31 - __builtin_clz(x); b >= 0; b--) {
      acc = jac_dbl(acc);
      if ((x >> b) & 1u) acc = jac_add(acc, v);
    }
    v = acc;
    if (!commit_inf[j]) v = jac_add_aff(v, ld_g1(commits, j));
  }
  const bool is_inf = jac_is_inf(v);
  g1a a = g1_to_aff(v);
  if (is_inf) {
    a.x = fp_zero();
    a.y = fp_zero();
  }
  st_g1(out_tab, i, a);
  out_inf[i] = is_inf;
}

// lambda_i = prod_{j != i} x_j / (x_j - x_i) mod r, x = idx + 1; written as plain scalars
// ------------------------------------------------------------------ launchers
void launch_decompress_g1(const uint8_t* in, size_t cnt, uint32_t* tab, uint8_t* inf, uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_decompress_g1, dim3(grid_for(cnt)), dim3(TPB), 0, st, in, cnt, tab, inf, cls);
}

void launch_pubpoly_eval(const uint32_t* commits, const uint8_t* commit_inf, uint32_t t, const uint32_t* idx,
                         size_t cnt, uint32_t* out_tab, uint8_t* out_inf, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_pubpoly_eval, dim3(grid_for(cnt)), dim3(TPB), 0, st, commits, commit_inf, t, idx, cnt,
                     out_tab, out_inf);
}



}  // namespace blsk

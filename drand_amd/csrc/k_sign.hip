// Signing kernels: tbls.Sign / bls.Sign (chain/beacon/crypto.go:58) [ext] and the synthetic chained
// history generator (client/test/result/mock/result.go:98-132 recipe, one lane per segment).
#include "kcommon.h"

namespace blsk {

// ------------------------------------------------------------------ signing
DI void sign_one(const uint32_t (&sk)[8], const g2j& h, uint8_t* out) {
  g2j s = jac_mul_scalar(h, sk);
  uint8_t buf[96];
  g2_compress(buf, s);
  for (int k = 0; k < 96; k++) out[k] = buf[k];
}

__global__ void __launch_bounds__(TPB) k_sign(const uint32_t* sk_words, int32_t index, const uint32_t* H,
                                              const uint8_t* h_inf, size_t cnt, uint8_t* out, size_t out_stride) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  uint32_t sk[8];
#pragma unroll
  for (int w = 0; w < 8; w++) sk[w] = sk_words[w];
  g2j h = h_inf[i] ? jac_infinity<fp2>() : jac_from_aff(g2a{ld_fp2(H, cnt, i, 0), ld_fp2(H, cnt, i, 2)});
  uint8_t* o = out + i * out_stride;
  if (index >= 0) {
    o[0] = (uint8_t)(index >> 8);
    o[1] = (uint8_t)index;
    o += 2;
  }
  sign_one(sk, h, o);
}

// one lane per chained segment: sig_r = sk * H(sha256(prev || r)), prev <- sig_r
__global__ void __launch_bounds__(TPB) k_gen_chained(const uint32_t* sk_words, ChainedSrc src, size_t n,
                                                     uint8_t* sigs_out) {
  const size_t seg = (size_t)blockIdx.x * TPB + threadIdx.x;
  const size_t n_seg = (n + src.seg_len - 1) / src.seg_len;
  if (seg >= n_seg) return;
  uint32_t sk[8];
#pragma unroll
  for (int w = 0; w < 8; w++) sk[w] = sk_words[w];
  const size_t g0 = seg * src.seg_len;
  const size_t g1 = g0 + src.seg_len < n ? g0 + src.seg_len : n;
  for (size_t g = g0; g < g1; g++) {
    const uint8_t* prev;
    int prev_len;
    if (g == g0) {
      prev = src.seeds + seg * 96;
      prev_len = seg == 0 ? (int)src.seed0_len : 96;
    } else {
      prev = sigs_out + (g - 1) * 96;
      prev_len = 96;
    }
    uint32_t msg[8];
    drand_message(msg, prev, prev_len, src.first_round + g);
    sign_one(sk, hash_to_g2(msg), sigs_out + g * 96);
  }
}

// ------------------------------------------------------------------ launchers
void launch_sign(const uint32_t* sk_words, int32_t index, const uint32_t* H, const uint8_t* h_inf, size_t cnt,
                 uint8_t* out, size_t out_stride, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_sign, dim3(grid_for(cnt)), dim3(TPB), 0, st, sk_words, index, H, h_inf, cnt, out, out_stride);
}

void launch_gen_chained(const uint32_t* sk_words, const ChainedSrc& src, size_t n, uint8_t* sigs_out, hipStream_t st) {
  if (!n) return;
  const size_t n_seg = (n + src.seg_len - 1) / src.seg_len;
  hipLaunchKernelGGL(k_gen_chained, dim3(grid_for(n_seg)), dim3(TPB), 0, st, sk_words, src, n, sigs_out);
}

}  // namespace blsk

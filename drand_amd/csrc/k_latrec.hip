// tbls Recover's interpolation sum_i [lambda_i] S_i in the latency engine's lane form (wrecover.h):
// one wave per selected share for the scalar multiplication, then one 8-wave workgroup for the
// sum, the affine conversion and the compression. Replaces a one-lane-per-share ladder whose
// 255 serial doublings dominated a threshold round.
#define WV_WAVES 8
#include "kcommon.h"
#include "wrecover.h"

namespace blsk {

constexpr int SUM_WAVES = WV_WAVES;

// scratch[i] <- [lambda_i] S[sel[i]] (Jacobian, POINT_WORDS words in lane order)
__global__ void __launch_bounds__(64) k_lat_recover_mul(const uint32_t* S, size_t n_s, const uint8_t* s_inf,
                                                        const uint32_t* sel, const uint32_t* lambdas, uint32_t t,
                                                        uint32_t* scratch) {
  __shared__ uint32_t tab[15 * wv::POINT_WORDS];
  const uint32_t i = blockIdx.x;
  if (i >= t) return;
  wv::wv_init();
  const size_t k = sel[i];
  wv::G2J r;
  if (s_inf[k]) {
    r = wv::g2_infinity();
  } else {
    uint32_t lam[8];
    for (int w = 0; w < 8; w++) lam[w] = lambdas[i * 8 + w];
    const wv::F x = wv::fp2_from392(S, n_s, k, 0), y = wv::fp2_from392(S, n_s, k, 2);
    r = wv::g2_mul_lambda(x, y, lam, tab);
  }
  wv::st_point(scratch + (size_t)i * wv::POINT_WORDS, r, true);
}

// out96 <- compress(sum of scratch[0 .. t)): strided partial sums per wave, then a tree in LDS
__global__ void __launch_bounds__(64 * SUM_WAVES) k_lat_recover_sum(const uint32_t* scratch, uint32_t t,
                                                                    uint8_t* out96) {
  __shared__ uint32_t xch[SUM_WAVES * wv::POINT_WORDS];
  wv::wv_init();
  const int w = threadIdx.x >> 6;
  wv::G2J acc = wv::g2_infinity();
  for (uint32_t i = w; i < t; i += SUM_WAVES) acc = wv::g2_add(acc, wv::ld_point(scratch + (size_t)i * wv::POINT_WORDS, true));
  for (int s = SUM_WAVES / 2; s >= 1; s >>= 1) {
    if (w >= s && w < 2 * s) wv::st_point(xch + (w - s) * wv::POINT_WORDS, acc, false);
    __syncthreads();
    if (w < s) acc = wv::g2_add(acc, wv::ld_point(xch + w * wv::POINT_WORDS, false));
    __syncthreads();
  }
  if (w == 0) {
    const uint32_t word = wv::g2_compress_words(acc);
    const uint32_t l = threadIdx.x;
    if (l < 24) reinterpret_cast<uint32_t*>(out96)[l] = __builtin_bswap32(word);
  }
}

void launch_lat_recover(const uint32_t* S, size_t n_s, const uint8_t* s_inf, const uint32_t* sel,
                        const uint32_t* lambdas, uint32_t t, uint32_t* scratch, uint8_t* out96, hipStream_t st) {
  if (!t) return;
  hipLaunchKernelGGL(k_lat_recover_mul, dim3(t), dim3(64), 0, st, S, n_s, s_inf, sel, lambdas, t, scratch);
  hipLaunchKernelGGL(k_lat_recover_sum, dim3(1), dim3(64 * SUM_WAVES), 0, st, scratch, t, out96);
}

}  // namespace blsk

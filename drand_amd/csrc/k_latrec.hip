// tbls Recover's interpolation sum_i [lambda_i] S_i in the latency engine's lane form (wrecover.h):
// four waves per selected share for the scalar multiplication, then one 8-wave workgroup for the
// sum, the affine conversion and the compression. Replaces a one-lane-per-share ladder whose
// 255 serial doublings dominated a threshold round.
#define WV_WAVES 8
#include "kcommon.h"
#include "wrecover.h"

namespace blsk {

constexpr int SUM_WAVES = WV_WAVES;

// scratch[i] <- [lambda_i] S[sel[i]] (Jacobian, POINT_WORDS words in lane order): four waves per share,
// wave j computing [d_j] P_j of lambda's x-adic digits (wrecover.h g2_mul_digit), wave 0 summing the
// four products. Each wave's 63 doublings and ~32 mixed additions replace one wave's 63 doublings and
// ~60 full additions of the joint table (g2_mul_lambda), and the four run on the CU's four SIMDs.
constexpr int MUL_WAVES = 4;
__global__ void __launch_bounds__(64 * MUL_WAVES) k_lat_recover_mul(const uint32_t* S, size_t n_s,
                                                                    const uint8_t* s_inf, const uint32_t* sel,
                                                                    const uint32_t* lambdas, uint32_t t,
                                                                    uint32_t* scratch) {
  __shared__ uint32_t part[(MUL_WAVES - 1) * wv::POINT_WORDS];
  const uint32_t i = blockIdx.x;
  if (i >= t) return;
  wv::wv_init();
  const int j = threadIdx.x >> 6;
  const size_t k = sel[i];
  const bool inf = s_inf[k] != 0;
  wv::G2J r = wv::g2_infinity();
  if (!inf) {
    uint32_t lam[8];
    for (int w = 0; w < 8; w++) lam[w] = lambdas[i * 8 + w];
    uint64_t d[4];
    wv::decompose_xabs(lam, d);
    const wv::F x = wv::fp2_from392(S, n_s, k, 0), y = wv::fp2_from392(S, n_s, k, 2);
    wv::F px, py;
    wv::lambda_base(x, y, j, px, py);
    r = wv::g2_mul_digit(px, py, d[j]);
  }
  if (j > 0) wv::st_point(part + (j - 1) * wv::POINT_WORDS, r, false);
  __syncthreads();
  if (j == 0) {
    for (int q = 0; q < MUL_WAVES - 1; q++) r = wv::g2_add(r, wv::ld_point(part + q * wv::POINT_WORDS, false));
    wv::st_point(scratch + (size_t)i * wv::POINT_WORDS, r, true);
  }
}

// out96 <- compress(sum of scratch[0 .. t)): strided partial sums per wave, then a tree in LDS
// saff (optional, wvteam.h SAFF_WORDS): the sum's affine x, y and its infinity flag, for the fused
// round's VerifyRecovered (wvteam.h verify_team_pre) without a decompression
__global__ void __launch_bounds__(64 * SUM_WAVES) k_lat_recover_sum(const uint32_t* scratch, uint32_t t,
                                                                    uint8_t* out96, uint32_t* saff) {
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
    const bool inf = wv::g2_is_inf(acc);
    uint32_t word = wv::COMPRESSED_INF_WORD0;
    const uint32_t l = threadIdx.x;
    if (!inf) {
      wv::F x, y;
      wv::g2_to_affine(acc, x, y);
      word = wv::g2_compress_affine_words(x, y);
      if (saff) {
        saff[l] = x.x;
        saff[64 + l] = y.x;
      }
    } else if (l != 0) {
      word = 0;
    }
    if (saff) saff[128 + l] = inf ? 1u : 0u;
    if (l < 24) reinterpret_cast<uint32_t*>(out96)[l] = __builtin_bswap32(word);
  }
}

void launch_lat_recover(const uint32_t* S, size_t n_s, const uint8_t* s_inf, const uint32_t* sel,
                        const uint32_t* lambdas, uint32_t t, uint32_t* scratch, uint8_t* out96, hipStream_t st,
                        uint32_t* saff) {
  if (!t) return;
  hipLaunchKernelGGL(k_lat_recover_mul, dim3(t), dim3(64 * MUL_WAVES), 0, st, S, n_s, s_inf, sel, lambdas, t,
                     scratch);
  hipLaunchKernelGGL(k_lat_recover_sum, dim3(1), dim3(64 * SUM_WAVES), 0, st, scratch, t, out96, saff);
}

}  // namespace blsk

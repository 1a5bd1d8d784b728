// Latency path: one workgroup of eight waves verifies one item end to end (wvteam.h: limbs across
// lanes, the item's independent work across the waves). Used for small batches (blsverify.cpp routes
// batches up to BLSV_LAT_MAX items here), where the batch pipeline's one-lane-per-item stages would
// leave the chip idle and pay a serial chain of ~16 M VALU instructions per lane. Same inputs and
// reject classes as the batch stages; the verdicts then go through launch_finish like theirs.
#define WV_WAVES 8
#include "kcommon.h"
#include "wvteam.h"

namespace wv {
__device__ uint64_t g_lat_trace[LAT_TRACE_N];
__device__ uint32_t g_lat_trace_on;  // 0 (production) unless blsv_lat_trace_enable turned it on
static_assert(TEAM_WAVES == WV_WAVES, "one wave of the workgroup per team member");
}

namespace blsk {

__constant__ uint8_t c_lat_dst[DST_LEN] = {66, 76, 83, 95, 83, 73, 71, 95, 66, 76, 83, 49, 50, 51, 56, 49, 71, 50, 95, 88,
                                           77, 68, 58, 83, 72, 65, 45, 50, 53, 54, 95, 83, 83, 87, 85, 95, 82, 79, 95,
                                           78, 85, 76, 95};

// sigma for recover_from (affine, batch form: 4 Fp slots, Montgomery R = 2^392, SoA of stride s_n)
DI void store_sigma(uint32_t* S, uint8_t* s_inf, size_t s_n, size_t i, const wv::F& sx, const wv::F& sy, bool inf) {
  uint32_t wx[2][12], wy[2][12];
  if (!inf) {
    wv::fp2_to392_words(sx, wx);
    wv::fp2_to392_words(sy, wy);
  }
  if (threadIdx.x == 0) {
    for (int c = 0; c < 2; c++)
      for (int k = 0; k < 12; k++) {
        S[(size_t)(c * 12 + k) * s_n + i] = inf ? 0u : wx[c][k];
        S[(size_t)((2 + c) * 12 + k) * s_n + i] = inf ? 0u : wy[c][k];
      }
    s_inf[i] = inf;
  }
}

// b0: expand_message_xmd's b_0 of item i's message (wave-uniform scalar work)
template <typename MsgB0>
DI void lat_verify(MsgB0 msg_b0, size_t i, const uint8_t* sig, const uint32_t* pk_tab, const uint8_t* pk_inf,
                   const uint32_t* pk_idx, uint8_t* cls, uint32_t* S, uint8_t* s_inf, size_t s_n) {
  wv::team_init();
  wv::wv_init();
  __syncthreads();
  uint32_t b0[8];
  msg_b0(b0);
  const uint32_t k = pk_idx ? pk_idx[i] : 0u;
  const uint32_t* pk = pk_tab + (size_t)k * G1_WORDS;
  wv::F sx, sy;
  bool sinf = false;
  const uint8_t c = wv::verify_team(sig, b0, pk, pk + 12, pk_inf[k] != 0, sx, sy, sinf);
  if (wv::wave_id() != 0) return;
  if (threadIdx.x == 0) cls[i] = c;
  if (S && (c == REJ_OK || c == REJ_PAIRING)) store_sigma(S, s_inf, s_n, i, sx, sy, sinf);
}

__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_chained(ChainedSrc src, size_t base, size_t cnt, const uint32_t* pk_tab,
                                                    const uint8_t* pk_inf, uint8_t* cls) {
  const size_t i = blockIdx.x;
  if (i >= cnt) return;
  const size_t g = base + i;
  lat_verify(
      [&](uint32_t(&b0)[8]) {
        const size_t seg = (g + src.seg_phase) / src.seg_len;
        const bool seg_start = g == 0 || (g + src.seg_phase - seg * src.seg_len) == 0;
        const uint8_t* prev = seg_start ? src.seeds + seg * 96 : src.sigs + (g - 1) * 96;
        const int prev_len = seg_start ? (seg == 0 ? (int)src.seed0_len : 96) : 96;
        uint32_t msg[8];
        drand_message<true>(msg, prev, prev_len, src.first_round + g);
        wv::xmd_b0_msg32(msg, b0);
      },
      i, src.sigs + g * 96, pk_tab, pk_inf, nullptr, cls, nullptr, nullptr, 0);
}

__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_unchained(const uint64_t* rounds, uint64_t first_round, const uint8_t* sigs,
                                                      size_t base, size_t cnt, const uint32_t* pk_tab,
                                                      const uint8_t* pk_inf, uint8_t* cls) {
  const size_t i = blockIdx.x;
  if (i >= cnt) return;
  lat_verify(
      [&](uint32_t(&b0)[8]) {
        uint32_t msg[8];
        drand_message_v2<true>(msg, rounds ? rounds[base + i] : first_round + base + i);
        wv::xmd_b0_msg32(msg, b0);
      },
      i, sigs + (base + i) * 96, pk_tab, pk_inf, nullptr, cls, nullptr, nullptr, 0);
}

__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len,
                                                     const uint8_t* sigs, size_t stride, size_t offset, size_t cnt,
                                                     const uint32_t* pk_tab, const uint8_t* pk_inf,
                                                     const uint32_t* pk_idx, uint8_t* cls, uint32_t* S,
                                                     uint8_t* s_inf) {
  const size_t i = blockIdx.x;
  if (i >= cnt) return;
  lat_verify([&](uint32_t(&b0)[8]) { xmd_b0_bytes<true>(b0, msgs + off[i], len[i], c_lat_dst); }, i,
             sigs + i * stride + offset, pk_tab, pk_inf, pk_idx, cls, S, s_inf, cnt);
}

// decode only (the speculative recovery's shares, blsverify.cpp spec_recover_launch): one workgroup of
// two waves per signature, wave 0 decoding (whash.h g2_decompress, no subgroup check: validity is the
// partials' verdict) while wave 1 multiplies for its two square roots, as the signature branch of
// wvteam.h verify_team does; sigma lands in S (stride cnt) as k_lat_messages stores it. Replaces the
// one-lane-per-item batch decompression there, whose serial chains took ~1.3 ms for a lone item.
__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_decode(const uint8_t* sigs, size_t stride, size_t offset,
                                                             size_t cnt, uint32_t* S, uint8_t* s_inf, uint8_t* cls) {
  const size_t i = blockIdx.x;
  if (i >= cnt) return;
  wv::team_init();
  wv::wv_init();
  __syncthreads();
  const int w = wv::wave_id();
  wv::RingCounts rc;
  if (w == 0) {
    wv::F x, y;
    bool inf = false;
    const uint8_t c = wv::g2_decompress(sigs + i * stride + offset, x, y, inf, false,
                                        wv::PowRing{&wv::SIG_RING, &rc});
    wv::flag_post(wv::CTR_DEC);  // stops the multiplier when the decode rejected before a root
    if (threadIdx.x == 0) cls[i] = c;
    store_sigma(S, s_inf, cnt, i, x, y, c != REJ_OK || inf);
  } else if (w == 1) {
    for (int k = 0; k < wv::DEC_POWS; k++)
      if (!wv::ring_pow_consume(wv::SIG_RING, bls::EXP_P_MINUS_3_DIV_4, rc, wv::CTR_DEC)) break;
  }
}

void launch_lat_decode(const uint8_t* sigs, size_t stride, size_t offset, size_t cnt, uint32_t* S, uint8_t* s_inf,
                       uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_lat_decode, dim3((unsigned)cnt), dim3(128), 0, st, sigs, stride, offset, cnt, S, s_inf, cls);
}

// the fused round's VerifyRecovered (blsverify.cpp spec_recover_launch): H(msg) and the key pair's
// Miller loop from the start of the round, then the rest of the check against the recovered
// signature's affine point (wvteam.h team_hash_key / verify_team_pre)
static_assert(kLatHoutWords == (size_t)wv::HOUT_WORDS && kLatSaffWords == (size_t)wv::SAFF_WORDS, "hand-off sizes");
__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_hash_key(const uint8_t* msgs, const uint64_t* off,
                                                               const uint32_t* len, const uint32_t* pk_tab,
                                                               const uint8_t* pk_inf, uint32_t* hout) {
  wv::team_init();
  wv::wv_init();
  __syncthreads();
  uint32_t b0[8];
  xmd_b0_bytes<true>(b0, msgs + off[0], len[0], c_lat_dst);
  wv::team_hash_key(b0, pk_tab, pk_tab + 12, pk_inf[0] != 0, hout);
}
__global__ void __launch_bounds__(64 * WV_WAVES) k_lat_verify_pre(const uint32_t* hout, const uint32_t* saff,
                                                                 uint8_t* cls) {
  wv::team_init();
  wv::wv_init();
  __syncthreads();
  const uint8_t c = wv::verify_team_pre(hout, saff);
  if (threadIdx.x == 0) cls[0] = c;
}
void launch_lat_hash_key(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, const uint32_t* pk_tab,
                         const uint8_t* pk_inf, uint32_t* hout, hipStream_t st) {
  hipLaunchKernelGGL(k_lat_hash_key, dim3(1), dim3(64 * WV_WAVES), 0, st, msgs, off, len, pk_tab, pk_inf, hout);
}
void launch_lat_verify_pre(const uint32_t* hout, const uint32_t* saff, uint8_t* cls, hipStream_t st) {
  hipLaunchKernelGGL(k_lat_verify_pre, dim3(1), dim3(64 * WV_WAVES), 0, st, hout, saff, cls);
}

// the phase marks of the last latency launch's item 0 (wteam.h WV_MARK), device wall-clock ticks
int lat_trace_read(uint64_t* out, int n, hipStream_t st) {
  if (n > wv::LAT_TRACE_N) n = wv::LAT_TRACE_N;
  if (hipMemcpyFromSymbolAsync(out, HIP_SYMBOL(wv::g_lat_trace), n * sizeof(uint64_t), 0, hipMemcpyDeviceToHost, st) !=
      hipSuccess)
    return -1;
  if (hipStreamSynchronize(st) != hipSuccess) return -1;
  return n;
}
int lat_trace_clear(hipStream_t st) {
  static const uint64_t z[wv::LAT_TRACE_N] = {};
  return hipMemcpyToSymbolAsync(HIP_SYMBOL(wv::g_lat_trace), z, sizeof z, 0, hipMemcpyHostToDevice, st) == hipSuccess
             ? 0
             : -1;
}

int lat_trace_enable(int on, hipStream_t st) {
  static const uint32_t v[2] = {0u, 1u};
  if (hipMemcpyToSymbolAsync(HIP_SYMBOL(wv::g_lat_trace_on), &v[on ? 1 : 0], sizeof(uint32_t), 0,
                             hipMemcpyHostToDevice, st) != hipSuccess)
    return -1;
  return hipStreamSynchronize(st) == hipSuccess ? 0 : -1;
}

void launch_lat_chained(const ChainedSrc& src, size_t base, size_t cnt, const uint32_t* pk_tab, const uint8_t* pk_inf,
                        uint8_t* cls, hipStream_t st) {
  if (cnt) hipLaunchKernelGGL(k_lat_chained, dim3((unsigned)cnt), dim3(64 * WV_WAVES), 0, st, src, base, cnt, pk_tab, pk_inf, cls);
}
void launch_lat_unchained(const uint64_t* rounds, uint64_t first_round, const uint8_t* sigs, size_t base, size_t cnt,
                          const uint32_t* pk_tab, const uint8_t* pk_inf, uint8_t* cls, hipStream_t st) {
  if (cnt)
    hipLaunchKernelGGL(k_lat_unchained, dim3((unsigned)cnt), dim3(64 * WV_WAVES), 0, st, rounds, first_round, sigs, base, cnt,
                       pk_tab, pk_inf, cls);
}
void launch_lat_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, const uint8_t* sigs,
                         size_t stride, size_t offset, size_t cnt, const uint32_t* pk_tab, const uint8_t* pk_inf,
                         const uint32_t* pk_idx, uint8_t* cls, uint32_t* S, uint8_t* s_inf, hipStream_t st) {
  if (cnt)
    hipLaunchKernelGGL(k_lat_messages, dim3((unsigned)cnt), dim3(64 * WV_WAVES), 0, st, msgs, off, len, sigs, stride, offset, cnt,
                       pk_tab, pk_inf, pk_idx, cls, S, s_inf);
}

}  // namespace blsk

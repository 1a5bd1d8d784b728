// Stage 1: drand message derivation + RFC 9380 hash-to-G2, one lane per beacon.
// chain.Message / MessageV2 (chain/beacon.go:103-114) -> KyberG2.Hash [ext].
#include "kcommon.h"

namespace blsk {

__constant__ uint8_t c_dst[DST_LEN] = {66, 76, 83, 95, 83, 73, 71, 95, 66, 76, 83, 49, 50, 51, 56, 49, 71, 50, 95, 88, 77, 68,
                                       58, 83, 72, 65, 45, 50, 53, 54, 95, 83, 83, 87, 85, 95, 82, 79, 95, 78, 85, 76, 95};

DI void store_h(uint32_t* H, uint8_t* h_inf, size_t cnt, size_t i, const g2j& h) {
  bool inf = jac_is_inf(h);
  g2a a = g2_to_aff(h);
  st_fp2(H, cnt, i, 0, a.x);
  st_fp2(H, cnt, i, 2, a.y);
  h_inf[i] = inf;
}

BLS_KERNEL(BLS_WPE_HASH) k_hash_chained(ChainedSrc src, size_t base, size_t cnt, uint32_t* H,
                                                      uint8_t* h_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  const size_t g = base + i;
  const size_t seg = (g + src.seg_phase) / src.seg_len;
  const bool seg_start = g == 0 || (g + src.seg_phase - seg * src.seg_len) == 0;
  const uint8_t* prev;
  int prev_len;
  if (seg_start) {
    prev = src.seeds + seg * 96;
    prev_len = seg == 0 ? (int)src.seed0_len : 96;
  } else {
    prev = src.sigs + (g - 1) * 96;
    prev_len = 96;
  }
  uint32_t msg[8];
  drand_message(msg, prev, prev_len, src.first_round + g);
  store_h(H, h_inf, cnt, i, hash_to_g2(msg));
}

BLS_KERNEL(BLS_WPE_HASH) k_hash_unchained(const uint64_t* rounds, uint64_t first_round, size_t base,
                                                        size_t cnt, uint32_t* H, uint8_t* h_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  const uint64_t round = rounds ? rounds[base + i] : first_round + base + i;
  uint32_t msg[8];
  drand_message_v2(msg, round);
  store_h(H, h_inf, cnt, i, hash_to_g2(msg));
}

BLS_KERNEL(BLS_WPE_HASH) k_hash_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len,
                                                       size_t cnt, uint32_t* H, uint8_t* h_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  uint32_t b0[8];
  xmd_b0_bytes(b0, msgs + off[i], len[i], c_dst);
  fp2 u0, u1;
  xmd_tail_to_field(b0, u0, u1);
  store_h(H, h_inf, cnt, i, hash_field_to_g2(u0, u1));
}

// ------------------------------------------------------------------ launchers
void launch_hash_chained(const ChainedSrc& src, size_t base, size_t cnt, uint32_t* H, uint8_t* h_inf,
                         hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_hash_chained, dim3(grid_for(cnt)), dim3(TPB), 0, st, src, base, cnt, H, h_inf);
}

void launch_hash_unchained(const uint64_t* rounds, uint64_t first_round, size_t base, size_t cnt, uint32_t* H,
                           uint8_t* h_inf, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_hash_unchained, dim3(grid_for(cnt)), dim3(TPB), 0, st, rounds, first_round, base, cnt, H,
                     h_inf);
}

void launch_hash_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t cnt, uint32_t* H,
                          uint8_t* h_inf, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_hash_messages, dim3(grid_for(cnt)), dim3(TPB), 0, st, msgs, off, len, cnt, H, h_inf);
}

}  // namespace blsk

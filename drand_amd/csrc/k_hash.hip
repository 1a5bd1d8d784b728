// Stage 1: drand message derivation + RFC 9380 hash-to-G2, one lane per beacon, in three kernels.
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

// ------------------------------------------------------------------ three phases
// Hash-to-G2 runs as three kernels with different register needs, the hand-off in SoA staging Q
// (HQ_WORDS = 144 words per item, stride cnt: two Jacobian G2 points, slots 0..5 and 6..11):
//   A  message, expand_message_xmd, both SSWU maps, 3-isogeny -> q0, q1 (slots 0..11): inversions and
//      four Fp exponentiations, long calls with a small live state, run at high occupancy (two forms,
//      see below).
//   B  q0 + q1, h_eff cofactor clearing (two [x] chains) -> slots 6..11 (P = q0 + q1 parked in 0..5).
//      Many short calls on two Jacobian points: the register-bound phase.
//   C  affine conversion (one inversion) and the infinity flag -> H.
DI g2j load_jac(const uint32_t* Q, size_t cnt, size_t i, int slot) {
  return {ld_fp2(Q, cnt, i, slot), ld_fp2(Q, cnt, i, slot + 2), ld_fp2(Q, cnt, i, slot + 4)};
}
DI void store_jac(uint32_t* Q, size_t cnt, size_t i, int slot, const g2j& p) {
  st_fp2(Q, cnt, i, slot, p.x);
  st_fp2(Q, cnt, i, slot + 2, p.y);
  st_fp2(Q, cnt, i, slot + 4, p.z);
}

#ifndef BLS_WPE_HASH_A
#define BLS_WPE_HASH_A 4
#endif
#ifndef BLS_WPE_HASH_B
#define BLS_WPE_HASH_B 2
#endif
#ifndef BLS_WPE_HASH_C
#define BLS_WPE_HASH_C 4
#endif

// Phase A, two forms. SPLIT (small batches, latency): one lane per (item, point), k = blockIdx.x & 1
// picks u_k, so the two SSWU maps of a hash -- each with its own (binary-GCD) inversion and two
// exponentiations -- run side by side; both lanes derive the message and field elements. !SPLIT
// (throughput): one lane per item, both maps sharing one inversion (fewer instructions per item).
template <bool SPLIT>
DI void hash_a_store(const fp2& u0, const fp2& u1, int k, uint32_t* Q, size_t cnt, size_t i) {
  if (SPLIT) {
    store_jac(Q, cnt, i, 6 * k, hash_field_to_q1(k == 0 ? u0 : u1));
  } else {
    g2j q0, q1;
    hash_field_to_q(u0, u1, q0, q1);
    store_jac(Q, cnt, i, 0, q0);
    store_jac(Q, cnt, i, 6, q1);
  }
}

template <bool SPLIT>
DI void hash_a_index(int& k, size_t& i) {
  k = SPLIT ? (int)(blockIdx.x & 1u) : 0;
  i = (size_t)(SPLIT ? blockIdx.x >> 1 : blockIdx.x) * TPB + threadIdx.x;
}

template <bool SPLIT>
BLS_KERNEL(BLS_WPE_HASH_A) k_hash_chained(ChainedSrc src, size_t base, size_t cnt, uint32_t* Q) {
  int k;
  size_t i;
  hash_a_index<SPLIT>(k, i);
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
  fp2 u0, u1;
  hash_to_field_fp2(msg, u0, u1);
  hash_a_store<SPLIT>(u0, u1, k, Q, cnt, i);
}

template <bool SPLIT>
BLS_KERNEL(BLS_WPE_HASH_A) k_hash_unchained(const uint64_t* rounds, uint64_t first_round, size_t base,
                                            size_t cnt, uint32_t* Q) {
  int k;
  size_t i;
  hash_a_index<SPLIT>(k, i);
  if (i >= cnt) return;
  const uint64_t round = rounds ? rounds[base + i] : first_round + base + i;
  uint32_t msg[8];
  drand_message_v2(msg, round);
  fp2 u0, u1;
  hash_to_field_fp2(msg, u0, u1);
  hash_a_store<SPLIT>(u0, u1, k, Q, cnt, i);
}

template <bool SPLIT>
BLS_KERNEL(BLS_WPE_HASH_A) k_hash_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len,
                                           size_t cnt, uint32_t* Q) {
  int k;
  size_t i;
  hash_a_index<SPLIT>(k, i);
  if (i >= cnt) return;
  uint32_t b0[8];
  xmd_b0_bytes(b0, msgs + off[i], len[i], c_dst);
  fp2 u0, u1;
  xmd_tail_to_field(b0, u0, u1);
  hash_a_store<SPLIT>(u0, u1, k, Q, cnt, i);
}

BLS_KERNEL(BLS_WPE_HASH_B) k_hash_cofactor(uint32_t* Q, size_t cnt) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  store_jac(Q, cnt, i, 0, jac_add(load_jac(Q, cnt, i, 0), load_jac(Q, cnt, i, 6)));
  auto at = [&](int slot) {
    size_t j = i;
    asm volatile("" : "+v"(j));  // re-read at each use, never kept live across the [x] chains
    return load_jac(Q, cnt, j, slot);
  };
  // P in slots 0..5; the second chain's base A parks in slots 6..11 (q1 is dead by then)
  const g2j r = g2_clear_cofactor_inl([&]() { return at(0); }, [&](const g2j& a) { store_jac(Q, cnt, i, 6, a); },
                                      [&]() { return at(6); });
  store_jac(Q, cnt, i, 6, r);
}

BLS_KERNEL(BLS_WPE_HASH_C) k_hash_affine(const uint32_t* Q, size_t cnt, uint32_t* H, uint8_t* h_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  store_h(H, h_inf, cnt, i, load_jac(Q, cnt, i, 6));
}

// ------------------------------------------------------------------ launchers
static void launch_hash_bc(uint32_t* Q, size_t cnt, uint32_t* H, uint8_t* h_inf, hipStream_t st) {
  hipLaunchKernelGGL(k_hash_cofactor, dim3(grid_for(cnt)), dim3(TPB), 0, st, Q, cnt);
  hipLaunchKernelGGL(k_hash_affine, dim3(grid_for(cnt)), dim3(TPB), 0, st, Q, cnt, H, h_inf);
}

// Below one wave round of phase A (4 waves/SIMD x 1024 SIMDs x 64 lanes) the GPU is not full and
// latency decides: the split form halves the per-lane chain of phase A.
#ifndef BLS_HASH_SPLIT_MAX
#define BLS_HASH_SPLIT_MAX 65536
#endif
static inline dim3 hash_a_grid(size_t cnt, bool split) { return dim3((split ? 2u : 1u) * grid_for(cnt)); }

void launch_hash_chained(const ChainedSrc& src, size_t base, size_t cnt, uint32_t* H, uint8_t* h_inf,
                         uint32_t* Q, hipStream_t st) {
  if (!cnt) return;
  const bool split = cnt <= BLS_HASH_SPLIT_MAX;
  if (split)
    hipLaunchKernelGGL(k_hash_chained<true>, hash_a_grid(cnt, true), dim3(TPB), 0, st, src, base, cnt, Q);
  else
    hipLaunchKernelGGL(k_hash_chained<false>, hash_a_grid(cnt, false), dim3(TPB), 0, st, src, base, cnt, Q);
  launch_hash_bc(Q, cnt, H, h_inf, st);
}

void launch_hash_unchained(const uint64_t* rounds, uint64_t first_round, size_t base, size_t cnt, uint32_t* H,
                           uint8_t* h_inf, uint32_t* Q, hipStream_t st) {
  if (!cnt) return;
  const bool split = cnt <= BLS_HASH_SPLIT_MAX;
  if (split)
    hipLaunchKernelGGL(k_hash_unchained<true>, hash_a_grid(cnt, true), dim3(TPB), 0, st, rounds, first_round, base,
                       cnt, Q);
  else
    hipLaunchKernelGGL(k_hash_unchained<false>, hash_a_grid(cnt, false), dim3(TPB), 0, st, rounds, first_round, base,
                       cnt, Q);
  launch_hash_bc(Q, cnt, H, h_inf, st);
}

void launch_hash_messages(const uint8_t* msgs, const uint64_t* off, const uint32_t* len, size_t cnt, uint32_t* H,
                          uint8_t* h_inf, uint32_t* Q, hipStream_t st) {
  if (!cnt) return;
  const bool split = cnt <= BLS_HASH_SPLIT_MAX;
  if (split)
    hipLaunchKernelGGL(k_hash_messages<true>, hash_a_grid(cnt, true), dim3(TPB), 0, st, msgs, off, len, cnt, Q);
  else
    hipLaunchKernelGGL(k_hash_messages<false>, hash_a_grid(cnt, false), dim3(TPB), 0, st, msgs, off, len, cnt, Q);
  launch_hash_bc(Q, cnt, H, h_inf, st);
}

}  // namespace blsk

// Stage 1: drand message derivation + RFC 9380 hash-to-G2, one lane per beacon, in three kernels.
// chain.Message / MessageV2 (chain/beacon.go:103-114) -> KyberG2.Hash [ext].
// The in-place Fp2 products of this unit's G2 chains use the Karatsuba body (tower.h
// fp2_mul_inl): their live state leaves room for its extra operand arrays here, unlike the Miller
// lines kernel (same-box A/B, profiles/r05_ab.json r05l: hash + decompression 100.7 -> 98.6 ms).
#define BLS_FP2_KARA_INL 1
#ifndef BLS_G2_DBL_KARA
#define BLS_G2_DBL_KARA 0
#endif
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
#define BLS_WPE_HASH_A 3
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
  drand_message<BLS_SHA_FAST_BATCH>(msg, prev, prev_len, src.first_round + g);
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
  drand_message_v2<BLS_SHA_FAST_BATCH>(msg, round);
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
  xmd_b0_bytes<BLS_SHA_FAST_BATCH>(b0, msgs + off[i], len[i], c_dst);
  fp2 u0, u1;
  xmd_tail_to_field(b0, u0, u1);
  hash_a_store<SPLIT>(u0, u1, k, Q, cnt, i);
}

// Phase B. h_eff P = [x]A - A - P + psi^2(2P), A = [x]P + psi(P) (curve.h g2_clear_cofactor_reload),
// every addition call-free (g2_add_inl_exc) with its second operand fetched from staging one coordinate
// at a time; only the accumulator lives in registers. Staging: P in slots 0..5 throughout (the
// exceptional path re-reads it), A and then the partial sum [x]A - A in slots 6..11. A lane whose
// additions met an exceptional case (a point at infinity, equal or opposite points: never for a hash
// output in practice) is marked in redo[] and recomputed by k_hash_cofactor_generic with the generic
// formulas, which handle every case (in a kernel of its own: their called-product frame would size
// this kernel's scratch at ~10 KB per lane).
//
// The sequence runs as a short program of uniform operations (c_cof_prog) over one copy of the
// doubling and one of the addition: written out, the compiler laid down every addition of both [x]
// chains separately (200K instructions, ~1.3 MB of code streamed through the instruction cache).
enum : uint8_t { COF_LOAD, COF_STORE, COF_DBL, COF_ADD, COF_NEG, COF_PSI2, COF_CHECK, COF_END };
constexpr uint8_t COF_NEGY = 1, COF_PSI = 2;  // COF_ADD flags: q.y negated, q -> psi(q)
struct CofOp {
  uint8_t op, arg, flags, pad;  // arg: staging slot (LOAD / STORE / ADD) or doubling count (DBL)
};
#define COF_CHAIN(s)                                                                                  \
  {COF_DBL, 1, 0, 0}, {COF_ADD, s, 0, 0}, {COF_DBL, 2, 0, 0}, {COF_ADD, s, 0, 0}, {COF_DBL, 3, 0, 0}, \
      {COF_ADD, s, 0, 0}, {COF_DBL, 9, 0, 0}, {COF_ADD, s, 0, 0}, {COF_DBL, 32, 0, 0}, {COF_ADD, s, 0, 0}, \
      {COF_DBL, 16, 0, 0}  // acc <- [|x|] acc for acc == the point in slot s (bits 62, 60, 57, 48, 16)
__constant__ CofOp c_cof_prog[] = {
    {COF_LOAD, 0, 0, 0}, {COF_ADD, 6, 0, 0}, {COF_CHECK, 0, 0, 0}, {COF_STORE, 0, 0, 0},  // P = q0 + q1
    COF_CHAIN(0), {COF_NEG, 0, 0, 0}, {COF_ADD, 0, COF_PSI, 0}, {COF_STORE, 6, 0, 0},        // A
    COF_CHAIN(6), {COF_NEG, 0, 0, 0}, {COF_ADD, 6, COF_NEGY, 0}, {COF_STORE, 6, 0, 0},       // R = [x]A - A
    {COF_LOAD, 0, 0, 0}, {COF_DBL, 1, 0, 0}, {COF_PSI2, 0, 0, 0}, {COF_ADD, 0, COF_NEGY, 0},  // psi^2(2P) - P
    {COF_ADD, 6, 0, 0}, {COF_STORE, 6, 0, 0}, {COF_END, 0, 0, 0}};                          // + R
#undef COF_CHAIN

BLS_KERNEL(BLS_WPE_HASH_B) k_hash_cofactor(uint32_t* Q, size_t cnt, uint8_t* redo) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  auto ld = [&](int slot) {  // re-read at each use, never kept live
    size_t j = i;
    asm volatile("" : "+v"(j));
    return ld_fp2(Q, cnt, j, slot);
  };
  __shared__ uint4 park_lds[18 * TPB];  // three Fp2 slots per lane (LdsFp2Slots): 18 KB per workgroup, 8 per CU
  const LdsFp2Slots park = {park_lds};
  g2j acc = {};
  bool exc = false;
#pragma unroll 1
  for (int pc = 0;; pc++) {
    const CofOp o = c_cof_prog[pc];
    if (o.op == COF_END) break;
    const int s = o.arg;
    if (o.op == COF_LOAD) {
      acc = {ld(s), ld(s + 2), ld(s + 4)};
    } else if (o.op == COF_STORE) {
      store_jac(Q, cnt, i, s, acc);
    } else if (o.op == COF_DBL) {
#pragma unroll 1
      for (int k = 0; k < s; k++) acc = g2_dbl_inl(acc);
    } else if (o.op == COF_ADD) {
      const bool psi = o.flags & COF_PSI, negy = o.flags & COF_NEGY;
      acc = g2_add_inl_exc(
          acc,
          [&]() {
            const fp2 x = ld(s);
            return psi ? fp2_mul_inl(fp2_conj(x), fp2_load_const(PSI_KX)) : x;
          },
          [&]() {
            fp2 y = ld(s + 2);
            if (psi) y = fp2_mul_inl(fp2_conj(y), fp2_load_const(PSI_KY));
            return negy ? fp2_neg(y) : y;
          },
          [&]() {
            const fp2 z = ld(s + 4);
            return psi ? fp2_conj(z) : z;
          },
          park, exc);
    } else if (o.op == COF_NEG) {
      acc.y = fp2_neg(acc.y);
    } else if (o.op == COF_PSI2) {
      const fp kx = fp_load_const(PSI2_KX[0]), ky = fp_load_const(PSI2_KY[0]);
      acc.x = {fp_mul_inl(acc.x.c0, kx), fp_mul_inl(acc.x.c1, kx)};
      acc.y = {fp_mul_inl(acc.y.c0, ky), fp_mul_inl(acc.y.c1, ky)};
    } else if (o.op == COF_CHECK) {  // q0 + q1 exceptional: both stay in staging for the generic kernel
      if (exc) {
        redo[i] = 2;
        return;
      }
    }
  }
  redo[i] = exc;
}

// Phase B's exceptional lanes, or every lane when `all`: h_eff P by the generic formulas. redo[i] = 2:
// q0 + q1 met an exceptional case and both are still in slots 0..11; otherwise P is in slots 0..5.
BLS_KERNEL(BLS_WPE_HASH_B) k_hash_cofactor_generic(uint32_t* Q, size_t cnt, const uint8_t* redo, int all) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  const uint8_t rd = redo[i];
  if (!(all || rd)) return;
  if (rd == 2) store_jac(Q, cnt, i, 0, jac_add(load_jac(Q, cnt, i, 0), load_jac(Q, cnt, i, 6)));
  store_jac(Q, cnt, i, 6, g2_clear_cofactor_reload([&]() { return load_jac(Q, cnt, i, 0); }));
}

BLS_KERNEL(BLS_WPE_HASH_C) k_hash_affine(const uint32_t* Q, size_t cnt, uint32_t* H, uint8_t* h_inf) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  store_h(H, h_inf, cnt, i, load_jac(Q, cnt, i, 6));
}

// ------------------------------------------------------------------ launchers
// nonzero: every lane takes the generic cofactor clearing and subgroup check (blsv_test_generic_chains)
int g_generic_chains_all = 0;
static void launch_hash_bc(uint32_t* Q, size_t cnt, uint32_t* H, uint8_t* h_inf, hipStream_t st) {
  hipLaunchKernelGGL(k_hash_cofactor, dim3(grid_for(cnt)), dim3(TPB), 0, st, Q, cnt, h_inf);
  hipLaunchKernelGGL(k_hash_cofactor_generic, dim3(grid_for(cnt)), dim3(TPB), 0, st, Q, cnt, h_inf,
                     g_generic_chains_all);
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

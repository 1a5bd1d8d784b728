// Stage 2: signature decompression (ZCash format) + psi-based G2 subgroup check, and the final
// verdict reduction (bitmap + first bad index). kilic G2.FromCompressed order [ext].
// The in-place Fp2 products of this unit's G2 chains use the Karatsuba body (tower.h
// fp2_mul_inl): their live state leaves room for its extra operand arrays here, unlike the Miller
// lines kernel (same-box A/B, profiles/r05_ab.json r05l: hash + decompression 100.7 -> 98.6 ms).
#define BLS_FP2_KARA_INL 1
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

// psi(P) == [x]P as one copy of the in-place doubling and one of the mixed addition in a loop over
// the runs of |x|'s bits (1, 2, 3, 9, 32 doublings, each followed by + P, then 16), P re-read from
// staging per coordinate, the addition's long-lived values parked in LDS (k_hash.hip's cofactor
// program, same reasons). The comparison is inline: [|x|]P = (X : Y : Z) equals -psi(P) iff
// X = psi(P).x Z^2 and -Y = psi(P).y Z^3. A lane whose chain met an exceptional case (the running
// point at infinity or equal to +-P: only for points of small order) is marked SUBGROUP_PENDING and
// decided by k_subgroup_g2_generic with the formulas that handle every case.
constexpr uint8_t SUBGROUP_PENDING = 0xfe;  // internal cls value between the two kernels
__constant__ uint8_t c_x_runs[6] = {1, 2, 3, 9, 32, 16};

BLS_KERNEL(BLS_WPE_SUBGROUP) k_subgroup_g2(uint32_t* S, uint8_t* s_inf, uint8_t* cls, size_t cnt) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK || s_inf[i]) return;
  auto ld = [&](int slot) {  // re-read at each use, never kept live
    size_t j = i;
    asm volatile("" : "+v"(j));
    return ld_fp2(S, cnt, j, slot);
  };
  __shared__ uint4 park_lds[18 * TPB];  // three Fp2 slots per lane (LdsFp2Slots)
  const LdsFp2Slots park = {park_lds};
  g2j acc = {ld(0), ld(2), fp2_one()};
  bool exc = false;
#pragma unroll 1
  for (int r = 0; r < 6; r++) {
    const int n = c_x_runs[r];
#pragma unroll 1
    for (int k = 0; k < n; k++) acc = g2_dbl_inl(acc);
    if (r < 5) acc = g2_madd_inl_exc(acc, [&]() { return ld(0); }, [&]() { return ld(2); }, park, exc);
  }
  if (exc) {
    cls[i] = SUBGROUP_PENDING;
    return;
  }
  const fp2 z2 = fp2_sqr_inl(acc.z);
  const bool ex = fp2_eq(acc.x, fp2_mul_inl(fp2_mul_inl(fp2_conj(ld(0)), fp2_load_const(PSI_KX)), z2));
  const fp2 z3 = fp2_mul_inl(z2, acc.z);
  const bool ey = fp2_eq(fp2_neg(acc.y), fp2_mul_inl(fp2_mul_inl(fp2_conj(ld(2)), fp2_load_const(PSI_KY)), z3));
  if (!(ex & ey) || fp2_is_zero(acc.z)) {
    st_fp2(S, cnt, i, 0, fp2_zero());
    st_fp2(S, cnt, i, 2, fp2_zero());
    s_inf[i] = 1;
    cls[i] = REJ_NOT_IN_SUBGROUP;
  }
}

// the SUBGROUP_PENDING lanes, or every decoded lane when `all` (blsv_test_generic_chains)
BLS_KERNEL(BLS_WPE_SUBGROUP) k_subgroup_g2_generic(uint32_t* S, uint8_t* s_inf, uint8_t* cls, size_t cnt,
                                                   int all) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt) return;
  const uint8_t c = cls[i];
  if (!(c == SUBGROUP_PENDING || (all && c == REJ_OK && !s_inf[i]))) return;
  const bool in = g2_in_subgroup_aff_reload([&]() { return g2a{ld_fp2(S, cnt, i, 0), ld_fp2(S, cnt, i, 2)}; });
  if (in) {
    cls[i] = REJ_OK;
  } else {
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
  hipLaunchKernelGGL(k_subgroup_g2_generic, dim3(grid_for(cnt)), dim3(TPB), 0, st, S, s_inf, cls, cnt,
                     g_generic_chains_all);
}

// decoding only (no subgroup check): the speculative recovery's shares, whose validity the round's
// own partial verification decides (blsverify.cpp spec_recover_launch)
void launch_decompress_g2_only(const uint8_t* sigs, size_t stride, size_t offset, size_t cnt, uint32_t* S,
                               uint8_t* s_inf, uint8_t* cls, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_decompress_g2, dim3(grid_for(cnt)), dim3(TPB), 0, st, sigs, stride, offset, size_t(0), cnt, S,
                     s_inf, cls);
}

void launch_finish(const uint8_t* cls, size_t base, size_t cnt, uint64_t* bitmap, unsigned long long* first_bad,
                   uint64_t label0, hipStream_t st) {
  if (!cnt) return;
  hipLaunchKernelGGL(k_finish, dim3((unsigned)((cnt + 255) / 256)), dim3(256), 0, st, cls, base, cnt, bitmap,
                     first_bad, label0);
}

}  // namespace blsk

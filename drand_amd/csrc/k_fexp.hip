// Stage 4: final exponentiation and the == 1 test, one lane per beacon. kilic Engine.Check [ext].
// Six launches per chunk (pairing.h fexp_easy / fexp_step<0..4>), each holding at most two Fp12
// values in registers; intermediate Fp12 values live in HBM staging buffers (SoA, 576 B per beacon)
// and are re-read at each use, which keeps every kernel free of scratch spills.
#include "kcommon.h"

namespace blsk {

BLS_KERNEL(BLS_WPE_FEXP) k_fexp_easy(const uint32_t* F, size_t cnt, const uint8_t* cls, uint32_t* G) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  st_fp12(G, cnt, i, fexp_easy(ld_fp12(F, cnt, i)));
}

// ------------------------------------------------------------------ 3-lane hard part (tri.h)
// Same fexp_step<MODE> sequence, each Fp12 spread over 3 lanes (Fp4 thirds): the 63 cyclotomic
// squares per exponentiation are call-free (3 in-place Fp2 squares per lane), the 5 multiplications
// use the called Fp2 product. 21 beacons per wave.
#ifndef BLS_WPE_FEXP_TRI
#define BLS_WPE_FEXP_TRI 2
#endif

// Park slot of the staged products (tri.h tri_mul_lp): 48 words per lane of the grid.
struct TriPark {
  uint32_t* p;
  size_t n, i;
};

template <typename LoadX>
DI fp4 tri_pow_x_abs(const tri_lane& t, LoadX lx, const TriPark& pk) {
  constexpr uint64_t NSQ = 1ull | (2ull << 6) | (3ull << 12) | (9ull << 18) | (32ull << 24) | (16ull << 30);
  fp4 r = lx();
#pragma unroll 1
  for (int s = 0; s < 6; s++) {
    const int n = (int)((NSQ >> (6 * s)) & 63u);
#pragma unroll 1
    for (int k = 0; k < n; k++) r = tri_cyclotomic_sqr(t, r);
    if (s < 5) r = tri_mul_lp(t, r, lx(), pk.p, pk.n, pk.i);
  }
  return r;
}

// fexp_step<MODE> on thirds: X^|x| by 63 Granger-Scott squares and 5 products (tri_pow_x_abs), then
// the step's own products. Measured and not kept (same-box A/B, 1M beacons, profiles/r03j_*): a
// Karabina compressed squaring chain on 2 lanes + batch decompression (162.8 ms against 160.9) and
// the A0 / (A1, A2) halves of the squaring as two one-lane kernels (169.6 ms); git history holds them.
template <int MODE>
BLS_KERNEL(BLS_WPE_FEXP_TRI) k_fexp_tri(const uint32_t* X, const uint32_t* C, const uint32_t* G, size_t cnt,
                                        uint8_t* cls, uint32_t* OUT, uint32_t* park) {
  const tri_lane t = tri_lane_id();
#if BLS_CSQR_LIN
  kp_lds_init<11>();
#endif
  const size_t ir = (size_t)blockIdx.x * TRI_GROUPS + t.group;
  const bool in_range = t.group < TRI_GROUPS && ir < cnt;
  const size_t i0 = in_range ? ir : cnt - 1;  // dummy lanes compute on a real row, never store
  const bool live = in_range && cls[i0] == REJ_OK;
  const TriPark pk = {park, (size_t)gridDim.x * TPB, (size_t)blockIdx.x * TPB + t.lane};
  // every lane stays active to the end (ds_bpermute reads its partners' registers)
  auto at = [&](const uint32_t* B) {
    size_t j = i0;
    asm volatile("" : "+v"(j));  // re-read at each use, never hoisted (a hoisted Fp12 pins its registers)
    return tri_load(B, cnt, j, t.role);
  };
  fp4 r = tri_conj(t, tri_pow_x_abs(t, [&]() { return at(X); }, pk));
  if (MODE == 0 || MODE == 1) r = tri_mul_lp(t, r, tri_conj(t, at(X)), pk.p, pk.n, pk.i);
  if (MODE == 2) r = tri_mul_lp(t, r, tri_frob(t, at(X)), pk.p, pk.n, pk.i);
  if (MODE == 4) {
    r = tri_mul_lp(t, r, tri_frob2(t, at(C)), pk.p, pk.n, pk.i);
    r = tri_mul_lp(t, r, tri_conj(t, at(C)), pk.p, pk.n, pk.i);
    r = tri_mul_lp(t, r, tri_cyclotomic_sqr(t, at(G)), pk.p, pk.n, pk.i);
    r = tri_mul_lp(t, r, at(G), pk.p, pk.n, pk.i);
  }
  if (MODE < 4 || OUT) {  // MODE 4 with OUT: the final value too (blsv_test_final_exp)
    if (live) tri_store(OUT, cnt, i0, t.role, r);
  }
  if (MODE == 4) {
    const bool one = tri_is_one(t, r);
    if (live && t.role == 0 && !one) cls[i0] = REJ_PAIRING;
  }
}

// ------------------------------------------------------------------ launchers
// F (Miller output) is consumed by the easy part and then reused as scratch; W holds 3 more Fp12
// staging slots of cnt entries each (G, B, C). park: FEXP_PARK_WORDS(cnt) words for the 3-lane
// products' parked partial results.
void launch_final_exp(uint32_t* F, uint32_t* W, size_t cnt, uint8_t* cls, hipStream_t st, uint32_t* park,
                      uint32_t* out) {
  if (!cnt) return;
  uint32_t* G = W;
  uint32_t* B = W + cnt * F_WORDS;
  uint32_t* C = W + 2 * cnt * F_WORDS;
  const dim3 grid(grid_for(cnt)), blk(TPB);
  hipLaunchKernelGGL(k_fexp_easy, grid, blk, 0, st, F, cnt, cls, G);
  const dim3 tgrid((unsigned)((cnt + TRI_GROUPS - 1) / TRI_GROUPS));
  hipLaunchKernelGGL(k_fexp_tri<0>, tgrid, blk, 0, st, G, nullptr, nullptr, cnt, cls, F, park);    // a -> F
  hipLaunchKernelGGL(k_fexp_tri<1>, tgrid, blk, 0, st, F, nullptr, nullptr, cnt, cls, B, park);    // b -> B
  hipLaunchKernelGGL(k_fexp_tri<2>, tgrid, blk, 0, st, B, nullptr, nullptr, cnt, cls, C, park);    // c -> C
  hipLaunchKernelGGL(k_fexp_tri<3>, tgrid, blk, 0, st, C, nullptr, nullptr, cnt, cls, F, park);    // t -> F
  hipLaunchKernelGGL(k_fexp_tri<4>, tgrid, blk, 0, st, F, C, G, cnt, cls, out, park);
}

}  // namespace blsk

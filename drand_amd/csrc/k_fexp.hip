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

// ------------------------------------------------------------------ compressed squaring chains
// X^|x| = X^(2^16) X^(2^48) X^(2^57) X^(2^60) X^(2^62) X^(2^63). k_csq_chain squares X 63 times in
// Karabina's compressed form (tri.h: only A1, A2 of the thirds, the Granger-Scott square's roles 1
// and 2) on TWO lanes per beacon, 32 beacons per wave against the full square's 21, and stores the six
// kept powers' A1, A2 into Fp12 staging slots; k_csq_decompress (one lane per beacon) recovers each
// A0 with one Fp2 inversion for all six (Montgomery's trick); k_fexp_tri multiplies the six. A beacon
// whose six denominators include a zero (X^(2^k) with a1 a2 = xi b1 b2, e.g. X = 1) is flagged, and
// the waves holding one run the full Granger-Scott chain instead. Off: -DBLS_FEXP_CSQ=0.
#ifndef BLS_FEXP_CSQ
#define BLS_FEXP_CSQ 1
#endif
constexpr int CSQ_GROUPS = 32;  // beacons per 64-lane wave
__constant__ uint8_t c_csq_runs[FEXP_KEPT] = {16, 32, 9, 3, 2, 1};  // squarings before each kept power

DI uint32_t* kept_slot(uint32_t* K, size_t cnt, int j) { return K + (size_t)j * cnt * F_WORDS; }

BLS_KERNEL(BLS_WPE_FEXP_TRI) k_csq_chain(const uint32_t* X, size_t cnt, const uint8_t* cls, uint32_t* K) {
  const unsigned lane = threadIdx.x & 63u;
  tri_lane t;  // the partner lane is both "next" (for role 1) and "prev" (for role 2)
  t.lane = lane;
  t.group = lane >> 1;
  t.role = 1u + (lane & 1u);
  t.next_b = t.prev_b = (int)(4u * (lane ^ 1u));
  const size_t ir = (size_t)blockIdx.x * CSQ_GROUPS + t.group;
  const bool in_range = ir < cnt;
  const size_t i0 = in_range ? ir : cnt - 1;  // lanes past the end compute on a real row, never store
  const bool live = in_range && cls[i0] == REJ_OK;
  fp4 r = tri_load(X, cnt, i0, t.role);
#pragma unroll 1
  for (int j = 0; j < (int)FEXP_KEPT; j++) {
    const int n = c_csq_runs[j];
#pragma unroll 1
    for (int k = 0; k < n; k++) r = tri_cyclotomic_sqr(t, r);
    if (live) tri_store(kept_slot(K, cnt, j), cnt, i0, t.role, r);
  }
}

BLS_KERNEL(BLS_WPE_FEXP) k_csq_decompress(uint32_t* K, size_t cnt, const uint8_t* cls, uint8_t* fb) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  auto third = [&](int j, unsigned role) {
    size_t q = i;
    asm volatile("" : "+v"(q));  // re-read at each use
    return tri_load(kept_slot(K, cnt, j), cnt, q, role);
  };
  // pass 1: the denominators and their prefix products, parked in the A0 slots (a: prefix, b: den)
  fp2 pre = fp2_one();
#pragma unroll 1
  for (int j = 0; j < (int)FEXP_KEPT; j++) {
    const fp2 d = csq_den(third(j, 1), third(j, 2));
    pre = j ? fp2_mul(pre, d) : d;
    st_fp2(kept_slot(K, cnt, j), cnt, i, tri_slot_a(0), pre);
    st_fp2(kept_slot(K, cnt, j), cnt, i, tri_slot_b(0), d);
  }
  const bool zero = fp2_is_zero(pre);
  fb[i] = zero;
  if (zero) return;
  // pass 2: one inversion for the six, then A0 = (na, nb) / den of each kept power
  fp2 inv = fp2_inv(pre);
#pragma unroll 1
  for (int j = (int)FEXP_KEPT - 1; j >= 0; j--) {
    uint32_t* kj = kept_slot(K, cnt, j);
    const fp2 dj = j ? fp2_mul(inv, ld_fp2(kept_slot(K, cnt, j - 1), cnt, i, tri_slot_a(0))) : inv;
    if (j) inv = fp2_mul(inv, ld_fp2(kj, cnt, i, tri_slot_b(0)));
    fp2 na, nb;
    csq_num(third(j, 1), third(j, 2), na, nb);
    st_fp2(kj, cnt, i, tri_slot_a(0), fp2_mul(na, dj));
    st_fp2(kj, cnt, i, tri_slot_b(0), fp2_mul(nb, dj));
  }
}

// fexp_step<MODE> on thirds: X^|x|, then the step's own products. FULL = false: X^|x| as the product
// of the six kept powers, for every beacon not flagged by k_csq_decompress. FULL = true: 63
// Granger-Scott squares and 5 products (tri_pow_x_abs) -- with fb, only in the waves that hold a
// flagged beacon (the others leave at once) and stored for the flagged beacons only; without fb
// (compressed chains off) for every beacon. The FULL launch runs first, while cls still marks every
// live beacon. Measured and not kept (same-box A/B, 1M beacons, profiles/r03j_*): a Karabina chain
// with separate Fp2 squares on 2 lanes + batch decompression (162.8 ms against 160.9) and the A0 /
// (A1, A2) halves of the squaring as two one-lane kernels (169.6 ms); git history holds them.
template <int MODE, bool FULL>
BLS_KERNEL(BLS_WPE_FEXP_TRI) k_fexp_tri(const uint32_t* X, const uint32_t* C, const uint32_t* G, size_t cnt,
                                        uint8_t* cls, uint32_t* OUT, uint32_t* park, const uint32_t* K,
                                        const uint8_t* fb) {
  const tri_lane t = tri_lane_id();
  const size_t ir = (size_t)blockIdx.x * TRI_GROUPS + t.group;
  const bool in_range = t.group < TRI_GROUPS && ir < cnt;
  const size_t i0 = in_range ? ir : cnt - 1;  // dummy lanes compute on a real row, never store
  const bool flagged = fb && fb[i0] != 0;
  const bool live = in_range && cls[i0] == REJ_OK && (fb ? flagged == FULL : true);
  if (FULL && fb && !__ballot(live)) return;  // wave-uniform: no flagged beacon here
  const TriPark pk = {park, (size_t)gridDim.x * TPB, (size_t)blockIdx.x * TPB + t.lane};
  // every lane stays active to the end (ds_bpermute reads its partners' registers)
  auto at = [&](const uint32_t* B) {
    size_t j = i0;
    asm volatile("" : "+v"(j));  // re-read at each use, never hoisted (a hoisted Fp12 pins its registers)
    return tri_load(B, cnt, j, t.role);
  };
  fp4 r;
  if constexpr (FULL) {
    r = tri_pow_x_abs(t, [&]() { return at(X); }, pk);
  } else {
    uint32_t* k = const_cast<uint32_t*>(K);
    r = at(kept_slot(k, cnt, (int)FEXP_KEPT - 1));
#pragma unroll 1
    for (int j = (int)FEXP_KEPT - 2; j >= 0; j--) r = tri_mul_lp(t, r, at(kept_slot(k, cnt, j)), pk.p, pk.n, pk.i);
  }
  r = tri_conj(t, r);
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
// staging slots of cnt entries each (G, B, C). park: FEXP_STAGE_WORDS(cnt) words: the 3-lane
// products' parked partial results, the six kept powers of a chain, the fallback flags.
void launch_final_exp(uint32_t* F, uint32_t* W, size_t cnt, uint8_t* cls, hipStream_t st, uint32_t* park,
                      uint32_t* out) {
  if (!cnt) return;
  uint32_t* G = W;
  uint32_t* B = W + cnt * F_WORDS;
  uint32_t* C = W + 2 * cnt * F_WORDS;
  uint32_t* K = BLS_FEXP_CSQ ? park + FEXP_PARK_WORDS(cnt) : nullptr;  // kept powers (see k_csq_chain)
  uint8_t* fb = reinterpret_cast<uint8_t*>(park + FEXP_PARK_WORDS(cnt) + FEXP_KEPT * F_WORDS * cnt);
  const dim3 grid(grid_for(cnt)), blk(TPB);
  hipLaunchKernelGGL(k_fexp_easy, grid, blk, 0, st, F, cnt, cls, G);
  const dim3 tgrid((unsigned)((cnt + TRI_GROUPS - 1) / TRI_GROUPS));
  const dim3 cgrid((unsigned)((cnt + CSQ_GROUPS - 1) / CSQ_GROUPS));
  // one exponentiation step: the compressed chain and its decompression, the flagged beacons' full
  // chain, then everyone else's product of kept powers
  auto step = [&](auto full, auto prod, const uint32_t* X, const uint32_t* Cs, const uint32_t* Gs, uint32_t* out_) {
    if (!K) {
      hipLaunchKernelGGL(full, tgrid, blk, 0, st, X, Cs, Gs, cnt, cls, out_, park, nullptr, nullptr);
      return;
    }
    hipLaunchKernelGGL(k_csq_chain, cgrid, blk, 0, st, X, cnt, cls, K);
    hipLaunchKernelGGL(k_csq_decompress, grid, blk, 0, st, K, cnt, cls, fb);
    hipLaunchKernelGGL(full, tgrid, blk, 0, st, X, Cs, Gs, cnt, cls, out_, park, K, fb);
    hipLaunchKernelGGL(prod, tgrid, blk, 0, st, X, Cs, Gs, cnt, cls, out_, park, K, fb);
  };
  step(k_fexp_tri<0, true>, k_fexp_tri<0, false>, G, nullptr, nullptr, F);  // a -> F
  step(k_fexp_tri<1, true>, k_fexp_tri<1, false>, F, nullptr, nullptr, B);  // b -> B
  step(k_fexp_tri<2, true>, k_fexp_tri<2, false>, B, nullptr, nullptr, C);  // c -> C
  step(k_fexp_tri<3, true>, k_fexp_tri<3, false>, C, nullptr, nullptr, F);  // t -> F
  step(k_fexp_tri<4, true>, k_fexp_tri<4, false>, F, C, G, out);
}

}  // namespace blsk

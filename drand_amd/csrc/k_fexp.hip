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

template <int MODE>
BLS_KERNEL(BLS_WPE_FEXP) k_fexp_step(const uint32_t* X, const uint32_t* C, const uint32_t* G, size_t cnt,
                                                   uint8_t* cls, uint32_t* OUT) {
  size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  // the re-reads must stay at their use sites: an opaque copy of the index keeps LICM from hoisting
  // them (a hoisted Fp12 would pin 144 VGPRs across the squaring loops)
  auto at = [&](const uint32_t* B) {
    size_t j = i;
    asm volatile("" : "+v"(j));
    return ld_fp12(B, cnt, j);
  };
  fp12 r = fexp_step<MODE>([&]() { return at(X); }, [&]() { return at(C); }, [&]() { return at(G); });
  if (MODE < 4 || OUT) st_fp12(OUT, cnt, i, r);  // MODE 4 with OUT: the final value (blsv_test_final_exp)
  if (MODE == 4 && !fp12_is_one(r)) cls[i] = REJ_PAIRING;
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

// ------------------------------------------------------------------ squaring chains, then products
// X^|x| = prod_e X^(2^b_e), b = 16, 48, 57, 60, 62, 63 (pairing.h fp12_pow_x_abs_karabina): all 63
// squares first, each kept X^(2^b_e) stored into the Fp12 slot K_e (SoA, tower order), then the 5
// products on three lanes (k_fexp_tri<MODE, true>). BLS_FEXP_CHAIN selects the squaring chain:
//   0  none: k_fexp_tri square-and-multiplies on three lanes (Granger-Scott squares, tri.h)
//   1  Karabina: k_fexp_ksq, two lanes per beacon (tri.h duo), 63 compressed squares (c1, c4, c2, c5);
//      k_fexp_kdec, one lane per beacon, recovers c0, c3 of the six K_e (Montgomery's trick: one
//      binary-GCD Fp inversion for the six denominators)
//   2  split Granger-Scott: the square of (A1, A2) never reads A0 and A0's never reads (A1, A2), so
//      the two chains run as two one-lane kernels (k_fexp_sq0: 48 words of state, k_fexp_sq12: 96),
//      call-free, with no exchange, no idle lane and no role selects
// Same-box A/B on MI355X, 1M beacons (profiles/r03j_*): final exponentiation 160.9 ms (0), 162.8 ms
// (1), 169.6 ms (2). The squares are issue-bound at every layout (about 25% of their instructions
// are the [0, 2p) additions around the Fp2 squares), Karabina's six decompressions with their
// inversion cost what its 2-lane squares save, and the split chains re-run the glue the 3-lane form
// shares, so 0 stays the default.
#ifndef BLS_FEXP_CHAIN
#define BLS_FEXP_CHAIN 0
#endif
#define BLS_FEXP_KARABINA (BLS_FEXP_CHAIN == 1)
#ifndef BLS_WPE_FEXP_KSQ
#define BLS_WPE_FEXP_KSQ 2
#endif
#ifndef BLS_WPE_FEXP_KDEC
#define BLS_WPE_FEXP_KDEC 2
#endif
#ifndef BLS_WPE_FEXP_SQ0
#define BLS_WPE_FEXP_SQ0 3
#endif
#ifndef BLS_WPE_FEXP_SQ12
#define BLS_WPE_FEXP_SQ12 2
#endif

#if BLS_FEXP_CHAIN == 2
// A0 = (c0.c0, c1.c1) chain (pairing.h cyclotomic_sqr_a0)
BLS_KERNEL(BLS_WPE_FEXP_SQ0) k_fexp_sq0(const uint32_t* X, size_t cnt, const uint8_t* cls, uint32_t* K) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  fp2 c0 = ld_fp2(X, cnt, i, 0), c3 = ld_fp2(X, cnt, i, 8);
  int e = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; k++) {
    cyclotomic_sqr_a0<true>(c0, c3);
    if ((KARABINA_KEEP >> k) & 1ull) {
      uint32_t* Ke = K + (size_t)e * cnt * F_WORDS;
      st_fp2(Ke, cnt, i, 0, c0);
      st_fp2(Ke, cnt, i, 8, c3);
      e++;
    }
  }
}

// (A1, A2) = (c1.c0, c0.c2; c0.c1, c1.c2) chain (pairing.h karabina_sqr)
BLS_KERNEL(BLS_WPE_FEXP_SQ12) k_fexp_sq12(const uint32_t* X, size_t cnt, const uint8_t* cls, uint32_t* K) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  fp12c c = {ld_fp2(X, cnt, i, 6), ld_fp2(X, cnt, i, 4), ld_fp2(X, cnt, i, 2), ld_fp2(X, cnt, i, 10)};
  int e = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; k++) {
    c = karabina_sqr<true>(c);
    if ((KARABINA_KEEP >> k) & 1ull) {
      uint32_t* Ke = K + (size_t)e * cnt * F_WORDS;
      st_fp2(Ke, cnt, i, 6, c.c1);
      st_fp2(Ke, cnt, i, 4, c.c4);
      st_fp2(Ke, cnt, i, 2, c.c2);
      st_fp2(Ke, cnt, i, 10, c.c5);
      e++;
    }
  }
}
#endif

#if BLS_FEXP_CHAIN == 1
BLS_KERNEL(BLS_WPE_FEXP_KSQ) k_fexp_ksq(const uint32_t* X, size_t cnt, const uint8_t* cls, uint32_t* K) {
  const unsigned lane = threadIdx.x & 63u;
  const size_t ir = (size_t)blockIdx.x * DUO_GROUPS + (lane >> 1);
  const bool r1 = (lane & 1u) == 0u;
  const unsigned role = r1 ? 1u : 2u;
  const size_t i = ir < cnt ? ir : cnt - 1;  // tail lanes compute on a real row, never store
  const bool live = ir < cnt && cls[i] == REJ_OK;
  // every lane stays active to the end (the partner's square crosses over DPP)
  fp4 x = tri_load(X, cnt, i, role);
  int e = 0;
#pragma unroll 1
  for (int k = 1; k <= 63; k++) {
    x = duo_karabina_sqr(r1, x);
    if ((KARABINA_KEEP >> k) & 1ull) {
      if (live) tri_store(K + (size_t)e * cnt * F_WORDS, cnt, i, role, x);
      e++;
    }
  }
}

// T: 12 Fp slots of scratch per beacon (the six numerators), free during this launch
BLS_KERNEL(BLS_WPE_FEXP_KDEC) k_fexp_kdec(uint32_t* K, size_t cnt, const uint8_t* cls, uint32_t* T) {
  const size_t i = (size_t)blockIdx.x * TPB + threadIdx.x;
  if (i >= cnt || cls[i] != REJ_OK) return;
  auto slot = [&](int e) { return K + (size_t)e * cnt * F_WORDS; };
  auto at = [&](const uint32_t* B, int s) {
    size_t j = i;
    asm volatile("" : "+v"(j));  // loads stay at their use sites
    return ld_fp2(B, cnt, j, s);
  };
  auto ldc = [&](int e) {
    const uint32_t* B = slot(e);
    return fp12c{at(B, 6), at(B, 4), at(B, 2), at(B, 10)};
  };
  // pass 1: numerators to T, prefix products of the denominators to the c0 slots, denominators to c3
  fp2 pre;
#pragma unroll 1
  for (int e = 0; e < KARABINA_N; e++) {
    fp2 num, den;
    karabina_num_den(ldc(e), num, den);
    pre = e ? fp2_mul(pre, den) : den;
    st_fp2(T, cnt, i, 2 * e, num);
    st_fp2(slot(e), cnt, i, 0, pre);
    st_fp2(slot(e), cnt, i, 8, den);
  }
  // pass 2: one inversion, then backwards 1/den_e = inv(prefix_e) * prefix_(e-1)
  fp2 inv = fp2_inv(pre);
#pragma unroll 1
  for (int e = KARABINA_N - 1; e >= 0; e--) {
    fp2 dinv = inv;
    if (e) {
      dinv = fp2_mul(inv, at(slot(e - 1), 0));
      inv = fp2_mul(inv, at(slot(e), 8));
    }
    const fp2 c3 = fp2_mul(at(T, 2 * e), dinv);
    const fp2 c0 = karabina_c0(ldc(e), c3);
    st_fp2(slot(e), cnt, i, 0, c0);
    st_fp2(slot(e), cnt, i, 8, c3);
  }
}

#endif  // BLS_FEXP_CHAIN == 1

// fexp_step<MODE> on thirds. KARA: X^|x| = the product of the six decompressed K_e (k_fexp_ksq +
// k_fexp_kdec, or k_fexp_sq0 + k_fexp_sq12, ran before); else 63 Granger-Scott squares and 5
// products here (tri_pow_x_abs).
template <int MODE, bool KARA>
BLS_KERNEL(BLS_WPE_FEXP_TRI) k_fexp_tri(const uint32_t* X, const uint32_t* C, const uint32_t* G, size_t cnt,
                                        uint8_t* cls, uint32_t* OUT, uint32_t* park, const uint32_t* K) {
  const tri_lane t = tri_lane_id();
  const size_t ir = (size_t)blockIdx.x * TRI_GROUPS + t.group;
  const bool in_range = t.group < TRI_GROUPS && ir < cnt;
  const size_t i0 = in_range ? ir : cnt - 1;  // dummy lanes compute on a real row, never store
  const bool live = in_range && cls[i0] == REJ_OK;
  const TriPark pk = {park, (size_t)gridDim.x * TPB, (size_t)blockIdx.x * TPB + t.lane};
  // every lane stays active to the end (ds_bpermute reads its partners' registers)
  auto at = [&](const uint32_t* B) {
    size_t j = i0;
    asm volatile("" : "+v"(j));  // re-read at each use, never hoisted (as in k_fexp_step)
    return tri_load(B, cnt, j, t.role);
  };
  fp4 r;
  if (KARA) {
    r = at(K);
#pragma unroll 1
    for (int e = 1; e < KARABINA_N; e++) r = tri_mul_lp(t, r, at(K + (size_t)e * cnt * F_WORDS), pk.p, pk.n, pk.i);
    r = tri_conj(t, r);
  } else {
    r = tri_conj(t, tri_pow_x_abs(t, [&]() { return at(X); }, pk));
  }
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
// staging slots of cnt entries each (G, B, C). park: KARABINA_N * cnt * F_WORDS words for the
// compressed chain's K_e, then TRI_PARK_WORDS(cnt) for the 3-lane products (FEXP_PARK_WORDS).
void launch_final_exp(uint32_t* F, uint32_t* W, size_t cnt, uint8_t* cls, hipStream_t st, uint32_t* park,
                      uint32_t* out) {
  if (!cnt) return;
  uint32_t* G = W;
  uint32_t* B = W + cnt * F_WORDS;
  uint32_t* C = W + 2 * cnt * F_WORDS;
  const dim3 grid(grid_for(cnt)), blk(TPB);
  hipLaunchKernelGGL(k_fexp_easy, grid, blk, 0, st, F, cnt, cls, G);
#ifdef BLS_FEXP_SINGLE_LANE
  hipLaunchKernelGGL(k_fexp_step<0>, grid, blk, 0, st, G, nullptr, nullptr, cnt, cls, F);  // a -> F
  hipLaunchKernelGGL(k_fexp_step<1>, grid, blk, 0, st, F, nullptr, nullptr, cnt, cls, B);  // b -> B
  hipLaunchKernelGGL(k_fexp_step<2>, grid, blk, 0, st, B, nullptr, nullptr, cnt, cls, C);  // c -> C
  hipLaunchKernelGGL(k_fexp_step<3>, grid, blk, 0, st, C, nullptr, nullptr, cnt, cls, F);  // t -> F
  hipLaunchKernelGGL(k_fexp_step<4>, grid, blk, 0, st, F, C, G, cnt, cls, out);  // out: test hook
  (void)park;
#else
  const dim3 tgrid((unsigned)((cnt + TRI_GROUPS - 1) / TRI_GROUPS));
  constexpr bool KA = BLS_FEXP_CHAIN != 0;
  uint32_t* K = park;
  uint32_t* pk = KA ? park + (size_t)KARABINA_N * cnt * F_WORDS : park;
  // X -> K_0..5 (squaring chains; Karabina's decompression uses T as scratch); the products run in
  // k_fexp_tri
  auto chain = [&](const uint32_t* X, uint32_t* T) {
    (void)X;
    (void)T;
#if BLS_FEXP_CHAIN == 1
    hipLaunchKernelGGL(k_fexp_ksq, dim3((unsigned)((cnt + DUO_GROUPS - 1) / DUO_GROUPS)), blk, 0, st, X, cnt, cls, K);
    hipLaunchKernelGGL(k_fexp_kdec, grid, blk, 0, st, K, cnt, cls, T);
#elif BLS_FEXP_CHAIN == 2
    hipLaunchKernelGGL(k_fexp_sq0, grid, blk, 0, st, X, cnt, cls, K);
    hipLaunchKernelGGL(k_fexp_sq12, grid, blk, 0, st, X, cnt, cls, K);
#endif
  };
  chain(G, F);
  hipLaunchKernelGGL((k_fexp_tri<0, KA>), tgrid, blk, 0, st, G, nullptr, nullptr, cnt, cls, F, pk, K);  // a -> F
  chain(F, B);
  hipLaunchKernelGGL((k_fexp_tri<1, KA>), tgrid, blk, 0, st, F, nullptr, nullptr, cnt, cls, B, pk, K);  // b -> B
  chain(B, C);
  hipLaunchKernelGGL((k_fexp_tri<2, KA>), tgrid, blk, 0, st, B, nullptr, nullptr, cnt, cls, C, pk, K);  // c -> C
  chain(C, F);
  hipLaunchKernelGGL((k_fexp_tri<3, KA>), tgrid, blk, 0, st, C, nullptr, nullptr, cnt, cls, F, pk, K);  // t -> F
  chain(F, B);  // B (b) is dead after step 2
  hipLaunchKernelGGL((k_fexp_tri<4, KA>), tgrid, blk, 0, st, F, C, G, cnt, cls, out, pk, K);
#endif
}

}  // namespace blsk

// Instruction-level parallelism inside the Fp2 product on gfx950 (not part of the product library).
// fp.h's product scanning accumulates each column in ONE 64-bit register, so every v_mad_u64_u32
// waits for the previous one; a wave alone on its SIMD (the register-bound 1-wave kernels: Miller
// f pass, [x] chains, subgroup check) then issues a MAD only every few cycles. fp_mont_dot_ilp
// sums the next column's products in separate accumulators while the current column reduces.
// Result (profiles/r03i_ilpbench.json): 0.98x at 1 wave/SIMD, 1.03x at 2-4 in isolation, and slower
// in the kernels (profiles/r03k_g2_chain_ab.json: fexpilp, hashilp), so the product keeps one chain.
// Measures called Fp2 products (the form the kernels use, b through LDS) per second for both bodies
// at 1, 2 and 4 waves per SIMD, and checks that they agree word for word.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/ilpbench tools/ilpbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../drand_amd/csrc/fp.h"

using namespace bls;

#define BLS_OPAQUE64(v) asm volatile("" : "+v"(v))

// fp_mont_dot with three independent accumulation chains per column instead of one: the x0 y0 and
// x1 y1 products of column k + 1 are summed in their own 64-bit accumulators while column k's
// reduction chain (carry + its products + m_j p_{k-j}) runs, so a wave alone on its SIMD finds an
// independent v_mad_u64_u32 to issue while a dependent one is in flight (the accumulate-to-accumulate
// latency is about three issue slots at one wave per SIMD, tools/latbench.hip). Same result, same
// MAD count, same bounds (each accumulator holds a subset of fp_mont_dot's column sum).
template <bool DOT>
__device__ __forceinline__ u12 fp_mont_dot_ilp(const uint32_t (&x0)[14], const uint32_t (&y0)[14], const uint32_t (&x1)[14],
                       const uint32_t (&y1)[14]) {
  uint32_t m[14], t[14];
  auto prod0 = [&](int k) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
    uint64_t s = 0;
#pragma unroll
    for (int j = lo; j <= hi; j++) s += (uint64_t)x0[j] * y0[k - j];
    BLS_OPAQUE64(s);  // a chain of its own: never re-associated into the reduction chain
    return s;
  };
  auto prod1 = [&](int k) {
    const int lo = k > 13 ? k - 13 : 0, hi = k < 13 ? k : 13;
    uint64_t s = 0;
#pragma unroll
    for (int j = lo; j <= hi; j++) s += (uint64_t)x1[j] * y1[k - j];
    BLS_OPAQUE64(s);
    return s;
  };
  uint64_t c = 0, pa = prod0(0), pb = DOT ? prod1(0) : 0;
#pragma unroll
  for (int k = 0; k < 27; k++) {
    uint64_t r = c + pa;
    if (DOT) r += pb;
    if (k < 26) {  // next column's products: independent of this column's reduction
      pa = prod0(k + 1);
      if (DOT) pb = prod1(k + 1);
    }
    if (k < 14) {
#pragma unroll
      for (int j = 0; j < k; j++) r += (uint64_t)m[j] * P28[k - j];
      m[k] = ((uint32_t)r * P_INV28) & M28;
      r += (uint64_t)m[k] * P28[0];
    } else {
#pragma unroll
      for (int j = k - 13; j < 14; j++) r += (uint64_t)m[j] * P28[k - j];
      t[k - 14] = (uint32_t)r & M28;
    }
    c = r >> 28;
  }
  t[13] = (uint32_t)c;
  return fp_join28(t);
}


template <bool ILP>
__device__ __noinline__ u24 mul_v(u24 a) {
  const unsigned l = threadIdx.x;
  u12 b0, b1;
#pragma unroll
  for (int i = 0; i < 12; i++) {
    b0[i] = g_fp2_arg[i * BLS_LANES + l];
    b1[i] = g_fp2_arg[(12 + i) * BLS_LANES + l];
  }
  uint32_t x0[14], x1[14], y0[14], y1[14], yn[14];
  fp_split28(u24_lo(a), x0);
  fp_split28(u24_hi(a), x1);
  fp_split28(b0, y0);
  fp_split28(b1, y1);
  fp_neg28(y1, yn);
  const u12 c0 = ILP ? fp_mont_dot_ilp<true>(x0, y0, x1, yn) : fp_mont_dot<true>(x0, y0, x1, yn);
  BLS_SCHED_FENCE();
  const u12 c1 = ILP ? fp_mont_dot_ilp<true>(x0, y1, x1, y0) : fp_mont_dot<true>(x0, y1, x1, y0);
  return u24_of(c0, c1);
}

template <bool ILP>
__device__ __noinline__ u24 sqr_v(u24 a) {
  const u12 a0 = u24_lo(a), a1 = u24_hi(a);
  uint32_t x[14], y[14];
  fp_split28(fp_add_raw_u12(a0, a1), x);
  fp_split28(fp_add_raw_u12(a0, fp_4p_minus_u12(a1)), y);
  const u12 c0 = ILP ? fp_mont_dot_ilp<false>(x, y, x, y) : fp_mont_dot<false>(x, y, x, y);
  BLS_SCHED_FENCE();
  fp_split28(fp_add_raw_u12(a0, a0), x);
  fp_split28(a1, y);
  const u12 c1 = ILP ? fp_mont_dot_ilp<false>(x, y, x, y) : fp_mont_dot<false>(x, y, x, y);
  return u24_of(c0, c1);
}

// per iteration: a <- a * b (called, b staged in LDS), b <- b^2 (called)
template <bool ILP, int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_bench(const uint32_t* in, uint32_t* out,
                                                                                           int iters) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  u24 a, b;
#pragma unroll
  for (int k = 0; k < 24; k++) {
    a[k] = in[k * 64 + threadIdx.x];
    b[k] = in[(24 + k) * 64 + threadIdx.x];
  }
  for (int it = 0; it < iters; it++) {
    fp2_arg_store(b);
    a = mul_v<ILP>(a);
    b = sqr_v<ILP>(b);
  }
#pragma unroll
  for (int k = 0; k < 24; k++) {
    out[(size_t)k * gridDim.x * 64 + i] = a[k];
    out[(size_t)(24 + k) * gridDim.x * 64 + i] = b[k];
  }
}

#define CHECK(x)                                                  \
  do {                                                            \
    hipError_t e = (x);                                           \
    if (e != hipSuccess) {                                        \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                   \
    }                                                             \
  } while (0)

template <bool ILP, int WPE>
static float run(const uint32_t* din, uint32_t* dout, int iters) {
  const int blocks = 256 * 4 * WPE;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_bench<ILP, WPE>), dim3(blocks), dim3(64), 0, 0, din, dout, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
  }
  return ms;
}

int main() {
  // operands < 2p: random words with a small top word
  static uint32_t h[48 * 64];
  srand(11);
  for (int k = 0; k < 48; k++)
    for (int l = 0; l < 64; l++) h[k * 64 + l] = (k % 12 == 11) ? ((uint32_t)rand() & 0x0fffffffu) : ((uint32_t)rand() << 16) ^ (uint32_t)rand();
  uint32_t *din, *d0, *d1;
  const size_t maxw = (size_t)256 * 4 * 4 * 64 * 48;
  CHECK(hipMalloc(&din, sizeof(h)));
  CHECK(hipMalloc(&d0, maxw * 4));
  CHECK(hipMalloc(&d1, maxw * 4));
  CHECK(hipMemcpy(din, h, sizeof(h), hipMemcpyHostToDevice));
  const int iters = 200;
  static uint32_t o0[256 * 4 * 4 * 64 * 48], o1[256 * 4 * 4 * 64 * 48];
  for (int w : {1, 2, 4}) {
    float m0 = 0, m1 = 0;
    if (w == 1) { m0 = run<false, 1>(din, d0, iters); m1 = run<true, 1>(din, d1, iters); }
    if (w == 2) { m0 = run<false, 2>(din, d0, iters); m1 = run<true, 2>(din, d1, iters); }
    if (w == 4) { m0 = run<false, 4>(din, d0, iters); m1 = run<true, 4>(din, d1, iters); }
    const size_t words = (size_t)256 * 4 * w * 64 * 48;
    CHECK(hipMemcpy(o0, d0, words * 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(o1, d1, words * 4, hipMemcpyDeviceToHost));
    const bool same = !memcmp(o0, o1, words * 4);
    const double pairs = (double)256 * 4 * w * 64 * iters;
    printf("{\"waves_per_simd\": %d, \"serial_ms\": %.3f, \"ilp_ms\": %.3f, \"speedup\": %.3f, "
           "\"serial_fp2_mulsqr_pairs_per_s\": %.4e, \"ilp_pairs_per_s\": %.4e, \"identical\": %s}\n",
           w, m0, m1, m0 / m1, pairs / (m0 * 1e-3), pairs / (m1 * 1e-3), same ? "true" : "false");
  }
  return 0;
}

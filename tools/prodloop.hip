// Feasibility microbenchmark for a memory-parked Miller f pass: Fp2 products in a runtime loop, both
// operands (each optionally a lazy sum of two parked values) loaded from a per-lane SoA park in
// global memory through buffer resources, the product expanded in place (fp.h fp2_mul_body), the
// result stored back to the park -- one lane per item at a register budget that allows 2 waves/SIMD.
// Against it, the same number of products through the called body with operands in registers at
// one wave/SIMD (the k_miller_f structure). Prints products/s of each form.
//   hipcc -O3 --offload-arch=gfx950 -o tools/prodloop tools/prodloop.hip && tools/prodloop
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "../drand_amd/csrc/soa.h"

using namespace bls;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

constexpr int SLOTS = 16;  // Fp2 slots per item in the park
constexpr int NP = 12;     // products per table pass

struct Prod {
  int8_t a, a2, b, b2, o;  // operand slots (a2/b2 < 0: no sum), output slot
};
__constant__ Prod c_tab[NP];

#ifndef PL_WPE
#define PL_WPE 2
#endif

// parked form: loop over the table, operands from the park
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PL_WPE)))
k_park(uint32_t* park, size_t n, int iters) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
#pragma unroll 1
    for (int p = 0; p < NP; p++) {
      const Prod t = c_tab[p];
      size_t j = i;
      asm volatile("" : "+v"(j));
      fp2 a = ld_fp2(park, n, j, 2 * t.a), b = ld_fp2(park, n, j, 2 * t.b);
      if (t.a2 >= 0) a = fp2_add_lazy(a, ld_fp2(park, n, j, 2 * t.a2));
      if (t.b2 >= 0) b = fp2_add_lazy(b, ld_fp2(park, n, j, 2 * t.b2));
      const fp2 r = fp2_from_u24(fp2_mul_body(fp2_to_u24(a), fp_to_u12(b.c0), fp_to_u12(b.c1)));
      st_fp2(park, n, j, 2 * t.o, r);
    }
  }
}

// register form: an Fp6-shaped working set (6 Fp2) in registers, products through the called body
__global__ void __launch_bounds__(64) k_reg(uint32_t* park, size_t n, int iters) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  fp2 v[SLOTS];
#pragma unroll
  for (int s = 0; s < SLOTS; s++) v[s] = ld_fp2(park, n, i, 2 * s);
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int p = 0; p < NP; p++) {
      const int a = (p * 5 + 1) % SLOTS, b = (p * 3 + 2) % SLOTS, o = (p * 7 + 3) % SLOTS;
      v[o] = fp2_mul(p & 1 ? fp2_add_lazy(v[a], v[(a + 1) % SLOTS]) : v[a], v[b]);
    }
  }
#pragma unroll
  for (int s = 0; s < SLOTS; s++) st_fp2(park, n, i, 2 * s, v[s]);
}

int main() {
  const size_t n = size_t(1) << 20;
  const int iters = 8;
  std::vector<uint32_t> h(n * SLOTS * 24);
  uint64_t s = 88172645463325252ull;
  for (auto& x : h) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    x = (uint32_t)s & 0x0fffffffu;  // values well below 2p
  }
  uint32_t* d;
  CK(hipMalloc(&d, h.size() * 4));
  CK(hipMemcpy(d, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  Prod tab[NP];
  for (int p = 0; p < NP; p++) {
    tab[p].a = (int8_t)((p * 5 + 1) % SLOTS);
    tab[p].a2 = (int8_t)(p & 1 ? (tab[p].a + 1) % SLOTS : -1);
    tab[p].b = (int8_t)((p * 3 + 2) % SLOTS);
    tab[p].b2 = (int8_t)(p % 3 == 0 ? (tab[p].b + 1) % SLOTS : -1);
    tab[p].o = (int8_t)((p * 7 + 3) % SLOTS);
  }
  CK(hipMemcpyToSymbol(HIP_SYMBOL(c_tab), tab, sizeof tab));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const dim3 grid((unsigned)(n / 64));
  for (int form = 0; form < 2; form++) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; rep++) {
      CK(hipEventRecord(e0));
      if (form == 0)
        hipLaunchKernelGGL(k_park, grid, dim3(64), 0, 0, d, n, iters);
      else
        hipLaunchKernelGGL(k_reg, grid, dim3(64), 0, 0, d, n, iters);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) best = ms < best ? ms : best;
    }
    const double prods = (double)n * iters * NP;
    printf("{\"form\": \"%s\", \"ms\": %.3f, \"G_fp2_products_per_s\": %.3f}\n", form == 0 ? "park_loop" : "reg_called",
           best, prods / best / 1e6);
  }
  return 0;
}

// Fp-multiply microbenchmark for gfx950 (not part of the product library).
// Measures fp_mul_u12 (drand_amd/csrc/fp.h, the product's Montgomery multiply) throughput as a
// function of resident waves per SIMD (grid sized to 256 CUs x 4 SIMDs x W one-wave blocks) and of
// the number of independent multiply chains per lane (ILP), plus the interleaved two-product
// fp_mul2_u12. Prints one JSON line per configuration.
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -o tools/fpbench tools/fpbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../drand_amd/csrc/fp.h"

using namespace bls;

template <int CH>
__global__ void __launch_bounds__(64) k_chain(const uint32_t* A, uint32_t* O, int iters) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  u12 x[CH], y;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const uint32_t v = A[(i & 1023) * 12 + k];
#pragma unroll
    for (int c = 0; c < CH; c++) x[c][k] = v ^ c;
    y[k] = A[((i + 7) & 1023) * 12 + k];
  }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) x[c] = fp_mul_u12(x[c], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int k = 0; k < 12; k++) s ^= x[c][k];
  O[i] = s;
}

#ifdef HAVE_MUL2
__global__ void __launch_bounds__(64) k_pair(const uint32_t* A, uint32_t* O, int iters) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  u12 x0, x1, y;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    const uint32_t v = A[(i & 1023) * 12 + k];
    x0[k] = v;
    x1[k] = v ^ 1;
    y[k] = A[((i + 7) & 1023) * 12 + k];
  }
  for (int it = 0; it < iters; it++) fp_mul2_u12(x0, x1, y, y);
  uint32_t s = 0;
#pragma unroll
  for (int k = 0; k < 12; k++) s ^= x0[k] ^ x1[k];
  O[i] = s;
}
#endif

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__);              \
      return 1;                                                                \
    }                                                                          \
  } while (0)

template <typename K>
static int run(const char* name, K kern, int chains, int waves_per_simd, const uint32_t* dA, uint32_t* dO) {
  const int blocks = 256 * 4 * waves_per_simd, iters = 512;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, dA, dO, iters);
    hipEventRecord(e1);
    CHECK(hipEventSynchronize(e1));
    hipEventElapsedTime(&ms, e0, e1);
  }
  const double muls = (double)blocks * 64 * iters * chains;
  printf("{\"kernel\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"ms\": %.3f, \"fp_mul_per_s\": %.4e}\n", name,
         chains, waves_per_simd, ms, muls / (ms * 1e-3));
  return 0;
}

int main() {
  uint32_t h[1024 * 12];
  srand(5);
  for (int i = 0; i < 1024 * 12; i++) h[i] = ((uint32_t)rand() << 16) ^ (uint32_t)rand();
  for (int i = 0; i < 1024; i++) h[i * 12 + 11] &= 0x0fffffff;
  uint32_t *dA, *dO;
  CHECK(hipMalloc(&dA, sizeof(h)));
  CHECK(hipMalloc(&dO, 256 * 4 * 8 * 64 * 4));
  CHECK(hipMemcpy(dA, h, sizeof(h), hipMemcpyHostToDevice));
  for (int w : {1, 2, 4, 8}) {
    run("chain", k_chain<1>, 1, w, dA, dO);
    run("chain", k_chain<2>, 2, w, dA, dO);
    run("chain", k_chain<3>, 3, w, dA, dO);
#ifdef HAVE_MUL2
    run("mul2", k_pair, 2, w, dA, dO);
#endif
  }
  return 0;
}

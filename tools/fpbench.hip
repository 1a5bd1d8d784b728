// Fp-multiply microbenchmark for gfx950 (not part of the product library).
// Measures fp_mul_u12 (drand_amd/csrc/fp.h, the product's Montgomery multiply) throughput as a
// function of resident waves per SIMD (grid sized to 256 CUs x 4 SIMDs x W one-wave blocks) and of
// the number of independent multiply chains per lane (ILP), plus the interleaved two-product
// fp_mul2_u12. Prints one JSON line per configuration.
// Also a separated-operand-scanning multiplier in 13 x 30-bit limbs (fp_mul_sos30: the product's 169
// column MADs, carried into 30-bit limbs, then a column-wise Montgomery reduction with another 169,
// R = 2^390; 338 MADs against the radix-2^28 interleaved form's 392), checked against fp_mul_u12 on
// the device (mont30(a, b) = 4 mont28(a, b) mod p) before it is timed.
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

// ------------------------------------------------------------------ 13 x 30-bit SOS multiplier
constexpr uint32_t M30 = (1u << 30) - 1u;
__constant__ uint32_t P30[13] = {0x3fffaaabu, 0x27fbffffu, 0x153ffffbu, 0x2affffacu, 0x30f6241eu, 0x034a83dau, 0x112bf673u,
                                 0x12e13ce1u, 0x2cd76477u, 0x1ed90d2eu, 0x29a4b1bau, 0x3a8e5ff9u, 0x001a0111u};
constexpr uint32_t P_INV30 = 0x3ffcfffdu;  // -p^-1 mod 2^30

DI void split30(const u12& a, uint32_t (&x)[13]) {
#pragma unroll
  for (int k = 0; k < 13; k++) {
    const int w = (30 * k) >> 5, sh = (30 * k) & 31;
    const uint64_t cat = ((uint64_t)(w + 1 < 12 ? a[w + 1] : 0u) << 32) | a[w];
    x[k] = (uint32_t)(cat >> sh) & M30;
  }
}
DI u12 join30(const uint32_t (&r)[13]) {
  u12 o;
#pragma unroll
  for (int w = 0; w < 12; w++) {
    const int k = (32 * w) / 30, sh = (32 * w) % 30;
    uint64_t v = (uint64_t)r[k] >> sh;
    if (k + 1 < 13) v |= (uint64_t)r[k + 1] << (30 - sh);
    if (k + 2 < 13) v |= (uint64_t)r[k + 2] << (60 - sh);
    o[w] = (uint32_t)v;
  }
  return o;
}
// a b 2^-390 mod p, < 2p for any 12-word inputs: T = a b (25 columns of <= 13 products < 2^60, carried
// into 26 limbs of 30 bits), then m_k = t_k (-p^-1) mod 2^30 column by column (<= 13 products < 2^60
// plus t_k and the carry: < 2^64)
NOINL u12 fp_mul_sos30(u12 a, u12 b) {
  uint32_t x[13], y[13], t[26], m[13], r[13];
  split30(a, x);
  split30(b, y);
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 25; k++) {
    const int lo = k > 12 ? k - 12 : 0, hi = k < 12 ? k : 12;
#pragma unroll
    for (int j = lo; j <= hi; j++) acc += (uint64_t)x[j] * y[k - j];
    t[k] = (uint32_t)acc & M30;
    acc >>= 30;
  }
  t[25] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int k = 0; k < 26; k++) {
    acc += t[k];
    const int lo = k > 12 ? k - 12 : 0, hi = k < 13 ? k - 1 : 12;
#pragma unroll
    for (int j = lo; j <= hi; j++) acc += (uint64_t)m[j] * P30[k - j];
    if (k < 13) {
      m[k] = ((uint32_t)acc * P_INV30) & M30;
      acc += (uint64_t)m[k] * P30[0];  // low 30 bits become 0
    } else {
      r[k - 13] = (uint32_t)acc & M30;
    }
    acc >>= 30;
  }
  return join30(r);
}

template <int CH>
__global__ void __launch_bounds__(64) k_chain30(const uint32_t* A, uint32_t* O, int iters) {
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
    for (int c = 0; c < CH; c++) x[c] = fp_mul_sos30(x[c], y);
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; c++)
#pragma unroll
    for (int k = 0; k < 12; k++) s ^= x[c][k];
  O[i] = s;
}

// mismatches of canon(mont30(a, b)) against canon(4 mont28(a, b)) over n random pairs (inputs < 2p)
__global__ void k_check30(const uint32_t* A, int n, unsigned* bad) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  u12 a, b;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    a[k] = A[(i % 1024) * 12 + k];
    b[k] = A[((i * 7 + 3) % 1024) * 12 + k];
  }
  const fp r30 = fp_canon(fp_from_u12(fp_mul_sos30(a, b)));
  const fp r28 = fp_canon(fp_dbl(fp_dbl(fp_from_u12(fp_mul_u12(a, b)))));
  bool eq = true;
#pragma unroll
  for (int k = 0; k < 12; k++) eq = eq && r30.l[k] == r28.l[k];
  if (!eq) atomicAdd(bad, 1u);
}

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
  {
    unsigned* dBad;
    CHECK(hipMalloc(&dBad, 4));
    CHECK(hipMemset(dBad, 0, 4));
    hipLaunchKernelGGL(k_check30, dim3(64), dim3(64), 0, 0, dA, 4096, dBad);
    unsigned bad = 0;
    CHECK(hipMemcpy(&bad, dBad, 4, hipMemcpyDeviceToHost));
    printf("{\"check\": \"sos30 = 4 x radix-28 Montgomery mod p\", \"pairs\": 4096, \"mismatches\": %u}\n", bad);
    if (bad) return 1;
  }
  for (int w : {1, 2, 4, 8}) {
    run("sos30", k_chain30<1>, 1, w, dA, dO);
    run("sos30", k_chain30<2>, 2, w, dA, dO);
    run("chain", k_chain<1>, 1, w, dA, dO);
    run("chain", k_chain<2>, 2, w, dA, dO);
    run("chain", k_chain<3>, 3, w, dA, dO);
#ifdef HAVE_MUL2
    run("mul2", k_pair, 2, w, dA, dO);
#endif
  }
  return 0;
}

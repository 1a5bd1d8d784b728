// fp_mul variant microbenchmark + cross-check (gfx950). Not part of the product library.
// Variants: CIOS (current fp.h), FIPS with inline-asm v_mad_u64_u32 + carry accumulate.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/fpbench tools/fpbench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include "../drand_amd/csrc/fp.h"

using namespace bls;

// ---------------------------------------------------------------- FIPS
#define MAC(acc, top, x, y)                                                                     \
  do {                                                                                          \
    uint64_t cc_;                                                                               \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, 0, %2, %1"               \
        : "+v"(acc), "=s"(cc_), "+v"(top)                                                       \
        : "v"(x), "v"(y));                                                                      \
  } while (0)
#define MACS(acc, top, x, ys)                                                                   \
  do {                                                                                          \
    uint64_t cc_;                                                                               \
    asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, 0, %2, %1"               \
        : "+v"(acc), "=s"(cc_), "+v"(top)                                                       \
        : "v"(x), "s"(ys));                                                                     \
  } while (0)

// two products per asm statement (a_j*b_{i-j} and m_j*p_{i-j}): half the asm boundaries
#define MAC2(acc, top, x, y, mm, ps)                                                            \
  do {                                                                                          \
    asm("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc\n\t"      \
        "v_mad_u64_u32 %0, vcc, %4, %5, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"            \
        : "+v"(acc), "+v"(top)                                                                  \
        : "v"(x), "v"(y), "v"(mm), "s"(ps)                                                      \
        : "vcc");                                                                               \
  } while (0)

template <bool PAIR>
__device__ __forceinline__ u12 fips_body(u12 a, u12 b) {
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      if (PAIR) {
        MAC2(acc, top, a[j], b[i - j], m[j], P_RAW[i - j]);
      } else {
        MAC(acc, top, a[j], b[i - j]);
        MACS(acc, top, m[j], P_RAW[i - j]);
      }
    }
    MAC(acc, top, a[i], b[0]);
    m[i] = (uint32_t)acc * P_INV32;
    MACS(acc, top, m[i], P_RAW[0]);
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) {
      if (PAIR) {
        MAC2(acc, top, a[j], b[i - j], m[j], P_RAW[i - j]);
      } else {
        MAC(acc, top, a[j], b[i - j]);
        MACS(acc, top, m[j], P_RAW[i - j]);
      }
    }
    t[i - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(t[i], P_RAW[i], br, &br);
  u12 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? t[i] : d[i];
  return r;
}
static __device__ __noinline__ u12 fp_mul_fips2(u12 a, u12 b) { return fips_body<true>(a, b); }

static __device__ __noinline__ u12 fp_mul_fips(u12 a, u12 b) {
  uint32_t m[12], t[12];
  uint64_t acc = 0;
  uint32_t top = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) {
#pragma unroll
    for (int j = 0; j < i; j++) {
      MAC(acc, top, a[j], b[i - j]);
      MACS(acc, top, m[j], P_RAW[i - j]);
    }
    MAC(acc, top, a[i], b[0]);
    m[i] = (uint32_t)acc * P_INV32;
    MACS(acc, top, m[i], P_RAW[0]);
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
#pragma unroll
  for (int i = 12; i < 24; i++) {
#pragma unroll
    for (int j = i - 11; j < 12; j++) {
      MAC(acc, top, a[j], b[i - j]);
      MACS(acc, top, m[j], P_RAW[i - j]);
    }
    t[i - 12] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)top << 32);
    top = 0;
  }
  uint32_t d[12];
  unsigned br = 0;
#pragma unroll
  for (int i = 0; i < 12; i++) d[i] = __builtin_subc(t[i], P_RAW[i], br, &br);
  u12 r;
#pragma unroll
  for (int i = 0; i < 12; i++) r[i] = br ? t[i] : d[i];
  return r;
}

template <int V>
__device__ __forceinline__ u12 vmul(u12 a, u12 b) {
  if (V == 0) return fp_mul_u12(a, b);
  if (V == 1) return fp_mul_fips(a, b);
  return fp_mul_fips2(a, b);
}

template <int V>
__global__ void __launch_bounds__(256) k_check(const uint32_t* A, const uint32_t* B, uint32_t* O, int n) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  u12 a, b;
  for (int k = 0; k < 12; k++) {
    a[k] = A[i * 12 + k];
    b[k] = B[i * 12 + k];
  }
  u12 r = vmul<V>(a, b);
  for (int k = 0; k < 12; k++) O[i * 12 + k] = r[k];
}

// throughput: 4 independent chains per lane
template <int V>
__global__ void __launch_bounds__(256) k_tput(const uint32_t* A, uint32_t* O, int iters) {
  int i = blockIdx.x * 256 + threadIdx.x;
  u12 x0, x1, x2, x3, y;
  for (int k = 0; k < 12; k++) {
    uint32_t v = A[(i & 1023) * 12 + k];
    x0[k] = v;
    x1[k] = v ^ 1;
    x2[k] = v ^ 2;
    x3[k] = v ^ 3;
    y[k] = A[((i + 7) & 1023) * 12 + k];
  }
  for (int it = 0; it < iters; it++) {
    x0 = vmul<V>(x0, y);
    x1 = vmul<V>(x1, y);
    x2 = vmul<V>(x2, y);
    x3 = vmul<V>(x3, y);
  }
  uint32_t s = 0;
  for (int k = 0; k < 12; k++) s ^= x0[k] ^ x1[k] ^ x2[k] ^ x3[k];
  O[i] = s;
}

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

int main() {
  const int n = 1 << 16;
  uint32_t *hA = (uint32_t*)malloc(n * 48), *hB = (uint32_t*)malloc(n * 48), *h0 = (uint32_t*)malloc(n * 48),
           *h1 = (uint32_t*)malloc(n * 48);
  srand(5);
  for (int i = 0; i < n; i++) {
    for (int k = 0; k < 12; k++) {
      hA[i * 12 + k] = (rand() << 16) ^ rand();
      hB[i * 12 + k] = (rand() << 16) ^ rand();
    }
    hA[i * 12 + 11] &= 0x0fffffff;  // < p
    hB[i * 12 + 11] &= 0x0fffffff;
    if (i < 4) {  // edge cases: p-1 and 0
      for (int k = 0; k < 12; k++) { hA[i * 12 + k] = P_RAW[k]; hB[i * 12 + k] = i & 1 ? 0 : P_RAW[k]; }
      hA[i * 12] -= 1; if (i & 2) hB[i * 12] -= 1;
    }
  }
  uint32_t *dA, *dB, *d0, *d1;
  CHECK(hipMalloc(&dA, n * 48)); CHECK(hipMalloc(&dB, n * 48)); CHECK(hipMalloc(&d0, n * 48)); CHECK(hipMalloc(&d1, n * 48));
  CHECK(hipMemcpy(dA, hA, n * 48, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(dB, hB, n * 48, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check<0>, dim3(n / 256), dim3(256), 0, 0, dA, dB, d0, n);
  CHECK(hipDeviceSynchronize());
  CHECK(hipMemcpy(h0, d0, n * 48, hipMemcpyDeviceToHost));
  for (int v = 1; v < 3; v++) {
    if (v == 1) hipLaunchKernelGGL(k_check<1>, dim3(n / 256), dim3(256), 0, 0, dA, dB, d1, n);
    else hipLaunchKernelGGL(k_check<2>, dim3(n / 256), dim3(256), 0, 0, dA, dB, d1, n);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(h1, d1, n * 48, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < n * 12; i++) bad += h0[i] != h1[i];
    printf("{\"variant\": %d, \"check_mismatch_words\": %d}\n", v, bad);
  }
  const int blocks = 256 * 8, iters = 256;
  uint32_t* dO;
  CHECK(hipMalloc(&dO, blocks * 256 * 4));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const char* names[3] = {"cios", "fips_asm", "fips_asm_pair"};
  for (int v = 0; v < 3; v++) {
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      if (v == 0) hipLaunchKernelGGL(k_tput<0>, dim3(blocks), dim3(256), 0, 0, dA, dO, iters);
      else if (v == 1) hipLaunchKernelGGL(k_tput<1>, dim3(blocks), dim3(256), 0, 0, dA, dO, iters);
      else hipLaunchKernelGGL(k_tput<2>, dim3(blocks), dim3(256), 0, 0, dA, dO, iters);
      hipEventRecord(e1);
      CHECK(hipEventSynchronize(e1));
      float ms; hipEventElapsedTime(&ms, e0, e1);
      double muls = (double)blocks * 256 * iters * 4;
      if (rep == 2) printf("{\"variant\": \"%s\", \"ms\": %.3f, \"fp_mul_per_s\": %.4e}\n", names[v], ms, muls / (ms * 1e-3));
    }
  }
  return 0;
}

// Calibration of rocprofv3 FETCH_SIZE for the engine's own SoA access patterns (the MI355X guide's x2
// correction is measured for 16-byte-per-lane streaming reads; "other access widths are uncalibrated").
// Each kernel reads a known 576 bytes per item (one Fp12 in SoA staging, soa.h layout) and writes
// one word per item:
//   soa   one lane per item (the one-lane kernels: 64 items per wave, 256 contiguous bytes per word)
//   tri   three lanes per item, each its 48-word third (tri.h tri_load: 21 items per wave)
// Run: rocprofv3 --pmc FETCH_SIZE -- tools/pmccal   (prints the known bytes per kernel)
//   hipcc -O3 --offload-arch=gfx950 -o tools/pmccal tools/pmccal.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../drand_amd/csrc/tri.h"

using namespace bls;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e = (x);                                                              \
    if (e != hipSuccess) {                                                           \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void __launch_bounds__(64) k_cal_soa(const uint32_t* F, size_t n, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const fp12 f = ld_fp12(F, n, i);
  uint32_t x = 0;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&f);
#pragma unroll
  for (int k = 0; k < 144; k++) x ^= w[k];
  out[i] = x;
}

__global__ void __launch_bounds__(64) k_cal_tri(const uint32_t* F, size_t n, uint32_t* out) {
  const tri_lane t = tri_lane_id();
  const size_t i = (size_t)blockIdx.x * TRI_GROUPS + t.group;
  if (t.group >= TRI_GROUPS || i >= n) return;
  const fp4 a = tri_load(F, n, i, t.role);
  uint32_t x = 0;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&a);
#pragma unroll
  for (int k = 0; k < 48; k++) x ^= w[k];
  out[3 * i + t.role] = x;
}

int main() {
  const size_t n = size_t(1) << 20;  // 576 MiB of Fp12: past the 256 MiB Infinity Cache
  uint32_t *F, *out;
  CK(hipMalloc(&F, n * 576));
  CK(hipMalloc(&out, n * 12));
  CK(hipMemset(F, 1, n * 576));
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(k_cal_soa, dim3((unsigned)(n / 64)), dim3(64), 0, 0, F, n, out);
    hipLaunchKernelGGL(k_cal_tri, dim3((unsigned)((n + TRI_GROUPS - 1) / TRI_GROUPS)), dim3(64), 0, 0, F, n, out);
  }
  CK(hipDeviceSynchronize());
  printf("{\"items\": %zu, \"known_read_bytes_per_item\": 576, \"known_write_bytes_per_item\": {\"soa\": 4, \"tri\": 12}}\n", n);
  return 0;
}

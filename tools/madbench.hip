// v_mad_u64_u32 issue-rate microbenchmark for gfx950 (not part of the product library): one wave per
// SIMD vs eight, carry-out SGPR pair fixed vs rotating vs VCC, 8 independent accumulators per lane.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/madbench tools/madbench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define MAD8(c0, c1, c2, c3, c4, c5, c6, c7)                                                            \
  asm volatile("v_mad_u64_u32 %0, " c0 ", %8, %9, %0\n\t"                                               \
               "v_mad_u64_u32 %1, " c1 ", %8, %9, %1\n\t"                                               \
               "v_mad_u64_u32 %2, " c2 ", %8, %9, %2\n\t"                                               \
               "v_mad_u64_u32 %3, " c3 ", %8, %9, %3\n\t"                                               \
               "v_mad_u64_u32 %4, " c4 ", %8, %9, %4\n\t"                                               \
               "v_mad_u64_u32 %5, " c5 ", %8, %9, %5\n\t"                                               \
               "v_mad_u64_u32 %6, " c6 ", %8, %9, %6\n\t"                                               \
               "v_mad_u64_u32 %7, " c7 ", %8, %9, %7"                                                   \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
               : "v"(x), "v"(y)                                                                         \
               : "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "vcc")
#define DEP8(c0, c1, c2, c3, c4, c5, c6, c7)                                                             \
  asm volatile("v_mad_u64_u32 %0, " c0 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c1 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c2 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c3 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c4 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c5 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c6 ", %1, %2, %0\n\t"                                               \
               "v_mad_u64_u32 %0, " c7 ", %1, %2, %0"                                                   \
               : "+v"(a0)                                                                               \
               : "v"(x), "v"(y)                                                                         \
               : "s0", "s1", "s2", "s3", "s4", "s5", "s6", "s7", "vcc")

template <int MODE>
__global__ void __launch_bounds__(64) k_mad(const uint32_t* in, uint64_t* out, int iters) {
  uint32_t x = in[threadIdx.x], y = in[threadIdx.x + 64];
  uint64_t a0 = x, a1 = y, a2 = x ^ 1, a3 = y ^ 1, a4 = x ^ 2, a5 = y ^ 2, a6 = x ^ 3, a7 = y ^ 3;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      if (MODE == 0) MAD8("s[0:1]", "s[0:1]", "s[0:1]", "s[0:1]", "s[0:1]", "s[0:1]", "s[0:1]", "s[0:1]");
      if (MODE == 1) MAD8("s[0:1]", "s[2:3]", "s[4:5]", "s[6:7]", "s[0:1]", "s[2:3]", "s[4:5]", "s[6:7]");
      if (MODE == 2) MAD8("vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc", "vcc");
      if (MODE == 3) DEP8("s[0:1]", "s[2:3]", "s[4:5]", "s[6:7]", "s[0:1]", "s[2:3]", "s[4:5]", "s[6:7]");
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

int main() {
  uint32_t* din;
  uint64_t* dout;
  hipMalloc(&din, 128 * 4);
  hipMemset(din, 7, 128 * 4);
  hipMalloc(&dout, 256 * 4 * 8 * 64 * 8);
  const char* names[4] = {"fixed_sgpr", "rotating_sgpr", "vcc", "dependent_chain"};
  for (int w : {1, 2, 8}) {
    for (int m = 0; m < 4; m++) {
      const int blocks = 256 * 4 * w, iters = 2000;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        if (m == 0) hipLaunchKernelGGL(k_mad<0>, dim3(blocks), dim3(64), 0, 0, din, dout, iters);
        if (m == 1) hipLaunchKernelGGL(k_mad<1>, dim3(blocks), dim3(64), 0, 0, din, dout, iters);
        if (m == 2) hipLaunchKernelGGL(k_mad<2>, dim3(blocks), dim3(64), 0, 0, din, dout, iters);
        if (m == 3) hipLaunchKernelGGL(k_mad<3>, dim3(blocks), dim3(64), 0, 0, din, dout, iters);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      const double wave_instr = (double)blocks * iters * 64;  // 64 mads per iteration per wave
      const double cyc_per_instr = (ms * 1e-3 * 2.4e9) / (wave_instr / (1024.0 * w)) / w;
      printf("{\"mode\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.2f}\n", names[m], w,
             ms, (ms * 1e-3 * 2.4e9) / (wave_instr / 1024.0));
      (void)cyc_per_instr;
    }
  }
  return 0;
}

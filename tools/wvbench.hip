// Latency / throughput microbenchmark of the latency engine's field products (drand_amd/csrc/
// wfield.h) on MI355X: dependent chains of one product kind per wave, timed in-kernel with
// s_memtime (one wave alone on the chip: the per-product latency a lone verification pays) and
// with HIP events over growing grids (throughput when many items share the chip). The final value of
// block 0 is printed so tools/wvbench_check.py can verify the chain against Python integers.
// usage: wvbench [iters]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "../drand_amd/csrc/wverify.h"

using namespace wv;

__global__ void __launch_bounds__(64) kchain(const uint32_t* in, uint32_t* out, int iters, int mode,
                                             unsigned long long* cyc) {
  wv_init();
  F a = mkF(in[threadIdx.x], 1.0), b = mkF(in[64 + threadIdx.x], 1.0);
  const unsigned long long t0 = __builtin_readcyclecounter();
#pragma unroll 1
  for (int i = 0; i < iters; i++) {
    if (mode == 0) a = mul2(a, b);
    else if (mode == 1) a = sqr2(a);
    else if (mode == 2) a = mulp(a, b);
    else if (mode == 3) a = dot(a, b, b, a, a, b, b, a, a, b, b, a);
    else a = half(a);
  }
  const unsigned long long t1 = __builtin_readcyclecounter();
  if (blockIdx.x == 0) out[threadIdx.x] = a.x;
  if (blockIdx.x == 0 && threadIdx.x == 0) cyc[mode] = t1 - t0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 2000;
  // inputs: Montgomery-form values given as 25-bit limbs of two fixed integers (< p)
  uint32_t h_in[128] = {0};
  unsigned s = 12345;
  for (int half = 0; half < 2; half++)
    for (int k = 0; k < 15; k++) {
      s = s * 1103515245u + 12345u;
      h_in[32 * half + k] = (s >> 7) & ((1u << 25) - 1);
      s = s * 1103515245u + 12345u;
      h_in[64 + 32 * half + k] = (s >> 7) & ((1u << 25) - 1);
    }
  printf("{\"inputs\": [");
  for (int i = 0; i < 128; i++) printf("%u%s", h_in[i], i < 127 ? "," : "],\n");
  uint32_t *d_in, *d_out;
  unsigned long long* d_cyc;
  hipMalloc(&d_in, sizeof h_in);
  hipMalloc(&d_out, 64 * 4);
  hipMalloc(&d_cyc, 8 * 8);
  hipMemcpy(d_in, h_in, sizeof h_in, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"mul2", "sqr2", "mulp", "dot6", "half"};
  printf("\"iters\": %d, \"modes\": {", iters);
  for (int mode = 0; mode < 5; mode++) {
    printf("%s\"%s\": {", mode ? ", " : "", names[mode]);
    const int grids[] = {1, 256, 1024, 4096};
    for (int g = 0; g < 4; g++) {
      hipLaunchKernelGGL(kchain, dim3(grids[g]), dim3(64), 0, 0, d_in, d_out, 10, mode, d_cyc);  // warm
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kchain, dim3(grids[g]), dim3(64), 0, 0, d_in, d_out, iters, mode, d_cyc);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long cyc = 0;
      hipMemcpy(&cyc, d_cyc + mode, 8, hipMemcpyDeviceToHost);
      printf("%s\"grid%d\": {\"ms\": %.3f, \"us_per_op\": %.4f, \"ops_per_s\": %.4g, \"cycles_per_op_wave0\": %.1f}",
             g ? ", " : "", grids[g], ms, ms * 1e3 / iters, (double)grids[g] * iters / (ms * 1e-3),
             (double)cyc / iters);
      if (g == 0) {
        uint32_t h_out[64];
        hipMemcpy(h_out, d_out, sizeof h_out, hipMemcpyDeviceToHost);
        printf(", \"out\": [");
        for (int i = 0; i < 64; i++) printf("%u%s", h_out[i], i < 63 ? "," : "]");
      }
    }
    printf("}");
  }
  printf("}}\n");
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}

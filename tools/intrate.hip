// gfx950 integer-VALU throughput microbenchmark (feeds the roofline peak in DESIGN.md / bench.py).
//
// For each instruction of interest, every lane runs ITERS x 8 *independent* instances (8 separate
// accumulator chains, so dependent-issue latency is hidden), across a grid large enough to fill
// all 256 CUs many times over. Reported: instructions per second chip-wide and per CU per clock
// (clock from the device attribute, i.e. the nominal peak; DVFS can hold it lower under load).
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/intrate tools/intrate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); return 1; } } while (0)

constexpr int ITERS = 4096;

// v_mad_u64_u32 with 64-bit addend (carry-out to an SGPR pair), 8 independent chains
__global__ void __launch_bounds__(256) k_mad64(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint64_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = (uint64_t)(a + j) << 7;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(acc[j]) : "v"(a), "v"(b) : "vcc");
    }
  }
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mullo(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(acc[j]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mulhi(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(acc[j]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_mul24(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(acc[j]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_add_co_u32 + v_addc_co_u32 pairs: 4 independent (add, addc) pairs per iteration, each pair is
// a 64-bit add through VCC (the carry-chain idiom of multi-limb arithmetic)
__global__ void __launch_bounds__(256) k_addc(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t lo[4], hi[4];
#pragma unroll
  for (int j = 0; j < 4; j++) { lo[j] = a + j; hi[j] = b + j; }
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
      unsigned c;
      lo[j] = __builtin_addc(lo[j], b, 0u, &c);
      hi[j] = __builtin_addc(hi[j], a, c, &c);
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 4; j++) s ^= lo[j] ^ hi[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_add32(uint64_t* out, uint32_t seed) {
  uint32_t a = threadIdx.x ^ seed, b = blockIdx.x * 2654435761u + seed;
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[j]) : "v"(b));
  }
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s ^= acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_fma64(uint64_t* out, uint32_t seed) {
  double a = 1.0 + threadIdx.x * 1e-9, b = 1.0 - seed * 1e-12;
  double acc[8];
#pragma unroll
  for (int j = 0; j < 8; j++) acc[j] = a + j;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[j]) : "v"(b), "v"(a));
  }
  double s = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) s += acc[j];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

typedef void (*kfn)(uint64_t*, uint32_t);

static int run(const char* name, kfn k, double insts_per_lane_iter, uint64_t* d_out, int blocks,
               double clk_hz, int cus) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d_out, 1u);  // warmup
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int rep = 0; rep < 5; rep++) {
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, d_out, 2u + rep);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double lanes = (double)blocks * 256.0;
  double insts = lanes * ITERS * insts_per_lane_iter;
  double per_s = insts / (best * 1e-3);
  double per_cu_clk = per_s / cus / clk_hz;
  printf("{\"inst\": \"%s\", \"ms\": %.3f, \"lane_ops_per_s\": %.4e, \"lane_ops_per_cu_per_clk\": %.2f}\n",
         name, best, per_s, per_cu_clk);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  int cus = prop.multiProcessorCount;
  double clk = prop.clockRate * 1e3;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_hz\": %.0f}\n", prop.gcnArchName, cus, clk);
  int blocks = cus * 8 * 4;
  uint64_t* d_out;
  CHECK(hipMalloc(&d_out, (size_t)blocks * 256 * sizeof(uint64_t)));
  run("v_mad_u64_u32", k_mad64, 8, d_out, blocks, clk, cus);
  run("v_mul_lo_u32", k_mullo, 8, d_out, blocks, clk, cus);
  run("v_mul_hi_u32", k_mulhi, 8, d_out, blocks, clk, cus);
  run("v_mad_u32_u24", k_mul24, 8, d_out, blocks, clk, cus);
  run("v_add_co+v_addc_co(pairs)", k_addc, 4, d_out, blocks, clk, cus);
  run("v_add_u32", k_add32, 8, d_out, blocks, clk, cus);
  run("v_fma_f64", k_fma64, 8, d_out, blocks, clk, cus);
  CHECK(hipFree(d_out));
  return 0;
}

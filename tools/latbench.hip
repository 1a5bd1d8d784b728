// Dependent-issue latencies of the instructions the latency engine chains (one wave alone on a
// SIMD), measured with s_memtime around 64-deep chains in inline asm (nothing reordered):
//   mad_dep     v_mad_u64_u32 whose accumulator is the previous result
//   mad_ind8    8 interleaved independent accumulators (issue-bound)
//   add_dep     v_add_u32 chain
//   dpp_dep     v_mov_b32_dpp row_shr:1 of the previous result (with the required s_nop 1)
//   pl32_dep    v_permlane32_swap chain
//   lds_rt      ds_write_b32 -> ds_read_b32 of another lane's word -> s_waitcnt, dependent
// prints cycles per instruction (or per round trip) as JSON
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

__global__ void klat(unsigned long long* out, uint32_t seed) {
  uint32_t a = seed + threadIdx.x, b = seed * 3 + 1;
  uint64_t acc = a;
  unsigned long long t0, t1;
  // mad dependent
  t0 = __builtin_readcyclecounter();
  REP64(asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b) : "s40", "s41");)
  t1 = __builtin_readcyclecounter();
  out[0] = t1 - t0;
  // 8 independent accumulators
  uint64_t c0 = 1, c1 = 2, c2 = 3, c3 = 4, c4 = 5, c5 = 6, c6 = 7, c7 = 8;
  t0 = __builtin_readcyclecounter();
  REP8(asm volatile(
      "v_mad_u64_u32 %0, s[40:41], %8, %9, %0\n v_mad_u64_u32 %1, s[40:41], %8, %9, %1\n"
      "v_mad_u64_u32 %2, s[40:41], %8, %9, %2\n v_mad_u64_u32 %3, s[40:41], %8, %9, %3\n"
      "v_mad_u64_u32 %4, s[40:41], %8, %9, %4\n v_mad_u64_u32 %5, s[40:41], %8, %9, %5\n"
      "v_mad_u64_u32 %6, s[40:41], %8, %9, %6\n v_mad_u64_u32 %7, s[40:41], %8, %9, %7\n"
      : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(c4), "+v"(c5), "+v"(c6), "+v"(c7)
      : "v"(a), "v"(b)
      : "s40", "s41");)
  t1 = __builtin_readcyclecounter();
  out[1] = t1 - t0;
  uint32_t x = a;
  t0 = __builtin_readcyclecounter();
  REP64(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));)
  t1 = __builtin_readcyclecounter();
  out[2] = t1 - t0;
  t0 = __builtin_readcyclecounter();
  REP64(asm volatile("s_nop 1\n v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(x));)
  t1 = __builtin_readcyclecounter();
  out[3] = t1 - t0;
  uint32_t y = b;
  t0 = __builtin_readcyclecounter();
  REP64(asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));)
  t1 = __builtin_readcyclecounter();
  out[4] = t1 - t0;
  __shared__ uint32_t s[64];
  uint32_t addr = threadIdx.x * 4, raddr = ((threadIdx.x + 1) & 63) * 4;
  t0 = __builtin_readcyclecounter();
  for (int i = 0; i < 32; i++) {
    asm volatile("ds_write_b32 %0, %1\n ds_read_b32 %1, %2\n s_waitcnt lgkmcnt(0)" : : "v"(addr), "v"(x), "v"(raddr));
    asm volatile("" : "+v"(x));
  }
  t1 = __builtin_readcyclecounter();
  out[5] = t1 - t0;
  out[6] = acc + c0 + c1 + c2 + c3 + c4 + c5 + c6 + c7 + x + y + s[threadIdx.x];
}

int main() {
  unsigned long long* d;
  hipMalloc(&d, 8 * 8);
  unsigned long long h[8];
  hipLaunchKernelGGL(klat, dim3(1), dim3(64), 0, 0, d, 7u);
  hipLaunchKernelGGL(klat, dim3(1), dim3(64), 0, 0, d, 7u);
  hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
  printf("{\"cycles_per_instr\": {\"mad_dep\": %.2f, \"mad_ind8\": %.2f, \"add_dep\": %.2f, \"dpp_dep_with_nop\": %.2f, "
         "\"pl32_dep\": %.2f}, \"lds_roundtrip_cycles\": %.1f}\n",
         h[0] / 64.0, h[1] / 64.0, h[2] / 64.0, h[3] / 64.0, h[4] / 64.0, h[5] / 32.0);
  return 0;
}

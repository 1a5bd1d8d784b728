// VALU issue-rate microbenchmark for gfx950 (not part of the product library): SIMD cycles per wave
// instruction for the instruction classes of the Fp arithmetic (v_mad_u64_u32, 32-bit carry-chain
// adds, v_cndmask, plain 32-bit ALU, a MAD/ALU mix, v_mul_lo_u32, v_alignbit, 64-bit shifts, DPP moves) at 1, 2, 3, 4 and 8 waves per SIMD.
// 8 independent accumulators per lane; cycles assume 2.4 GHz.
// Caveat: the v_cndmask_b32_e32 (vcc) row (~23.5 cycles) is an artifact of this synthetic pattern; replacing
// every such select in fp.h with v_bfi_b32 changed no stage time of the real kernels (r02 A/B run).
// build: hipcc -O3 --offload-arch=gfx950 -o tools/issuebench tools/issuebench.hip
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define R8(op)                                                                                          \
  asm volatile(op(0) op(1) op(2) op(3) op(4) op(5) op(6) op(7)                                          \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)         \
               : "v"(x), "v"(y)                                                                         \
               : "vcc", "s0", "s1")
// 64-bit accumulators for the MAD forms (a_i are uint64_t there)
#define OP_MAD(i) "v_mad_u64_u32 %" #i ", s[0:1], %8, %9, %" #i "\n\t"
#define OP_ADDC(i) "v_addc_co_u32 %" #i ", vcc, %" #i ", %8, vcc\n\t"
#define OP_ADD(i) "v_add_co_u32 %" #i ", vcc, %" #i ", %8\n\t"
#define OP_CND(i) "v_cndmask_b32 %" #i ", %" #i ", %8, vcc\n\t"
#define OP_AND(i) "v_and_b32 %" #i ", %" #i ", %8\n\t"
#define OP_CND64(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, s[0:1]\n\t"
#define OP_CNDI(i) "v_cndmask_b32_e64 %" #i ", %" #i ", %8, exec\n\t"
#define OP_BFI(i) "v_bfi_b32 %" #i ", %9, %" #i ", %8\n\t"
#define OP_MIX(i) "v_mad_u64_u32 %" #i ", s[0:1], %8, %9, %" #i "\n\t v_and_b32 %8, %8, %9\n\t"
#define OP_MULLO(i) "v_mul_lo_u32 %" #i ", %" #i ", %8\n\t"
#define OP_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 28\n\t"
#define OP_SUBB(i) "v_subb_co_u32 %" #i ", vcc, %" #i ", %8, vcc\n\t"
#define OP_DPP(i) "v_mov_b32_dpp %" #i ", %" #i " row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
// 64-bit forms (a_i are uint64_t)
#define OP_SHR64(i) "v_lshrrev_b64 %" #i ", 28, %" #i "\n\t"
#define OP_LSHLADD(i) "v_lshl_add_u64 %" #i ", %" #i ", 0, %" #i "\n\t"

template <int MODE>
__global__ void __launch_bounds__(64) k_issue(const uint32_t* in, uint64_t* out, int iters) {
  uint32_t x = in[threadIdx.x], y = in[threadIdx.x + 64];
  asm volatile("s_mov_b64 s[0:1], 0x5\n\ts_mov_b64 vcc, 0x5" ::: "s0", "s1", "vcc");
  if (MODE == 0 || MODE == 5 || MODE == 13 || MODE == 14) {
    uint64_t a0 = x, a1 = y, a2 = x ^ 1, a3 = y ^ 1, a4 = x ^ 2, a5 = y ^ 2, a6 = x ^ 3, a7 = y ^ 3;
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int r = 0; r < 8; r++) {
        if (MODE == 0) R8(OP_MAD);
        if (MODE == 5) R8(OP_MIX);
        if (MODE == 13) R8(OP_SHR64);
        if (MODE == 14) R8(OP_LSHLADD);
      }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  } else {
    uint32_t a0 = x, a1 = y, a2 = x ^ 1, a3 = y ^ 1, a4 = x ^ 2, a5 = y ^ 2, a6 = x ^ 3, a7 = y ^ 3;
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int r = 0; r < 8; r++) {
        if (MODE == 1) R8(OP_ADDC);
        if (MODE == 2) R8(OP_ADD);
        if (MODE == 3) R8(OP_CND);
        if (MODE == 4) R8(OP_AND);
        if (MODE == 6) R8(OP_CND64);
        if (MODE == 7) R8(OP_CNDI);
        if (MODE == 8) R8(OP_BFI);
        if (MODE == 9) R8(OP_MULLO);
        if (MODE == 10) R8(OP_ALIGN);
        if (MODE == 11) R8(OP_SUBB);
        if (MODE == 12) R8(OP_DPP);
      }
    }
    out[blockIdx.x * 64 + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  }
}

int main() {
  uint32_t* din;
  uint64_t* dout;
  hipMalloc(&din, 128 * 4);
  hipMemset(din, 7, 128 * 4);
  hipMalloc(&dout, (size_t)256 * 4 * 8 * 64 * 8);
  const char* names[15] = {"mad_u64_u32", "addc_co_u32", "add_co_u32", "cndmask_b32 (vcc)", "and_b32", "mad+and (2 instr)", "cndmask_b32_e64 (sgpr pair)", "cndmask_b32_e64 (exec)", "bfi_b32",
                          "mul_lo_u32", "alignbit_b32", "subb_co_u32", "mov_b32_dpp row_ror", "lshrrev_b64", "lshl_add_u64"};
  for (int w : {1, 2, 8}) {
    for (int m = 0; m < 15; m++) {
      const int blocks = 256 * 4 * w, iters = 1000;
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      float ms = 0;
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        switch (m) {
          case 0: hipLaunchKernelGGL(k_issue<0>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 1: hipLaunchKernelGGL(k_issue<1>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 2: hipLaunchKernelGGL(k_issue<2>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 3: hipLaunchKernelGGL(k_issue<3>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 4: hipLaunchKernelGGL(k_issue<4>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 5: hipLaunchKernelGGL(k_issue<5>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 6: hipLaunchKernelGGL(k_issue<6>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 7: hipLaunchKernelGGL(k_issue<7>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 8: hipLaunchKernelGGL(k_issue<8>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 9: hipLaunchKernelGGL(k_issue<9>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 10: hipLaunchKernelGGL(k_issue<10>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 11: hipLaunchKernelGGL(k_issue<11>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 12: hipLaunchKernelGGL(k_issue<12>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 13: hipLaunchKernelGGL(k_issue<13>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
          case 14: hipLaunchKernelGGL(k_issue<14>, dim3(blocks), dim3(64), 0, 0, din, dout, iters); break;
        }
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms, e0, e1);
      }
      const double per_wave = (double)iters * 64 * (m == 5 ? 2 : 1);  // instructions per wave
      const double wave_instr = (double)blocks * per_wave;
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"simd_cycles_per_wave_instr\": %.2f}\n", names[m], w,
             ms, (ms * 1e-3 * 2.4e9) / (wave_instr / 1024.0));
    }
  }
  return 0;
}

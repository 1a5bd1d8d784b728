// Carry-chain cost on gfx950: the compiler emits each 12-limb add/sub chain of fp_add/fp_sub on VCC,
// one chain after the other, with `s_nop 1` between every two links (VALU carry write -> carry read
// hazard). Measures, per wave at 1 and 2 waves/SIMD, the time of
//   C : fp2_add + fp2_sub as compiled from fp.h (chains on VCC, hazard nops)
//   A : the same two operations with the four chains of each (add, 2p-correction per component)
//       interleaved in asm with their own SGPR-pair carries, so no link waits on its predecessor
//   S : the same, every chain on VCC one after the other (the form of the register-bound kernels)
// and checks that both give identical words.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/carrybench tools/carrybench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../drand_amd/csrc/tower.h"

using namespace bls;

#define CB_ITERS 256

template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_c(const uint32_t* in, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  fp2 a, b;
  for (int k = 0; k < 12; k++) {
    a.c0.l[k] = in[(0 * 12 + k) * 64 + threadIdx.x];
    a.c1.l[k] = in[(1 * 12 + k) * 64 + threadIdx.x];
    b.c0.l[k] = in[(2 * 12 + k) * 64 + threadIdx.x];
    b.c1.l[k] = in[(3 * 12 + k) * 64 + threadIdx.x];
  }
#pragma unroll 1
  for (int it = 0; it < CB_ITERS; it++) {
    a = fp2_add(a, b);
    b = fp2_sub(b, a);
  }
  for (int k = 0; k < 12; k++) {
    out[(0 * 12 + k) * gridDim.x * 64 + i] = a.c0.l[k];
    out[(1 * 12 + k) * gridDim.x * 64 + i] = a.c1.l[k];
    out[(2 * 12 + k) * gridDim.x * 64 + i] = b.c0.l[k];
    out[(3 * 12 + k) * gridDim.x * 64 + i] = b.c1.l[k];
  }
}

// carry links with explicit SGPR-pair carries (asm volatile keeps the written order: the chains
// interleave and no link directly follows its predecessor)
__device__ __forceinline__ void add_l(bool first, uint32_t& d, uint64_t& c, uint32_t a, uint32_t b) {
  if (first)
    asm volatile("v_add_co_u32 %0, %1, %2, %3" : "=v"(d), "=s"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_addc_co_u32 %0, %1, %2, %3, %1" : "=v"(d), "+s"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void sub_l(bool first, uint32_t& d, uint64_t& c, uint32_t a, uint32_t b) {
  if (first)
    asm volatile("v_sub_co_u32 %0, %1, %2, %3" : "=v"(d), "=s"(c) : "v"(a), "v"(b));
  else
    asm volatile("v_subb_co_u32 %0, %1, %2, %3, %1" : "=v"(d), "+s"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ uint32_t sel_l(uint64_t c, uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(c));
  return r;
}

// r = a + b, then r - 2p unless that borrows (fp_add), both components interleaved (4 chains)
__device__ __forceinline__ fp2 fp2_add_asm(const fp2& a, const fp2& b) {
  fp2 s, d, r;
  uint64_t ca, cb, ba, bb;
#pragma unroll
  for (int k = 0; k <= 12; k++) {
    if (k < 12) {
      add_l(k == 0, s.c0.l[k], ca, a.c0.l[k], b.c0.l[k]);
      add_l(k == 0, s.c1.l[k], cb, a.c1.l[k], b.c1.l[k]);
    }
    if (k > 0) {
      sub_l(k == 1, d.c0.l[k - 1], ba, s.c0.l[k - 1], P2_RAW[k - 1]);
      sub_l(k == 1, d.c1.l[k - 1], bb, s.c1.l[k - 1], P2_RAW[k - 1]);
    }
  }
#pragma unroll
  for (int k = 0; k < 12; k++) {
    r.c0.l[k] = sel_l(ba, s.c0.l[k], d.c0.l[k]);
    r.c1.l[k] = sel_l(bb, s.c1.l[k], d.c1.l[k]);
  }
  return r;
}

// r = a - b, then + 2p on a borrow (fp_sub), both components interleaved
__device__ __forceinline__ fp2 fp2_sub_asm(const fp2& a, const fp2& b) {
  fp2 d, r;
  uint64_t ba, bb, ca, cb;
#pragma unroll
  for (int k = 0; k < 12; k++) {
    sub_l(k == 0, d.c0.l[k], ba, a.c0.l[k], b.c0.l[k]);
    sub_l(k == 0, d.c1.l[k], bb, a.c1.l[k], b.c1.l[k]);
  }
#pragma unroll
  for (int k = 0; k < 12; k++) {
    add_l(k == 0, r.c0.l[k], ca, d.c0.l[k], sel_l(ba, P2_RAW[k], 0u));
    add_l(k == 0, r.c1.l[k], cb, d.c1.l[k], sel_l(bb, P2_RAW[k], 0u));
  }
  return r;
}

// the serialized form the compiler emits under register pressure: every chain on VCC, one after the
// other (the hazard recognizer then pads each link with s_nop 1)
__device__ __forceinline__ void add_v(bool first, uint32_t& d, uint32_t a, uint32_t b) {
  if (first)
    asm volatile("v_add_co_u32 %0, vcc, %1, %2" : "=v"(d) : "v"(a), "v"(b) : "vcc");
  else
    asm volatile("v_addc_co_u32 %0, vcc, %1, %2, vcc" : "=v"(d) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ void sub_v(bool first, uint32_t& d, uint32_t a, uint32_t b) {
  if (first)
    asm volatile("v_sub_co_u32 %0, vcc, %1, %2" : "=v"(d) : "v"(a), "v"(b) : "vcc");
  else
    asm volatile("v_subb_co_u32 %0, vcc, %1, %2, vcc" : "=v"(d) : "v"(a), "v"(b) : "vcc");
}
__device__ __forceinline__ uint32_t sel_v(uint32_t if_set, uint32_t if_clear) {
  uint32_t r;
  asm volatile("v_cndmask_b32 %0, %1, %2, vcc" : "=v"(r) : "v"(if_clear), "v"(if_set));
  return r;
}
__device__ __forceinline__ fp serial_add(const fp& a, const fp& b) {
  fp s, d, r;
#pragma unroll
  for (int k = 0; k < 12; k++) add_v(k == 0, s.l[k], a.l[k], b.l[k]);
#pragma unroll
  for (int k = 0; k < 12; k++) sub_v(k == 0, d.l[k], s.l[k], P2_RAW[k]);
#pragma unroll
  for (int k = 0; k < 12; k++) r.l[k] = sel_v(s.l[k], d.l[k]);
  return r;
}
__device__ __forceinline__ fp serial_sub(const fp& a, const fp& b) {
  fp d, m, r;
#pragma unroll
  for (int k = 0; k < 12; k++) sub_v(k == 0, d.l[k], a.l[k], b.l[k]);
#pragma unroll
  for (int k = 0; k < 12; k++) m.l[k] = sel_v(P2_RAW[k], 0u);
#pragma unroll
  for (int k = 0; k < 12; k++) add_v(k == 0, r.l[k], d.l[k], m.l[k]);
  return r;
}

template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_s(const uint32_t* in, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  fp2 a, b;
  for (int k = 0; k < 12; k++) {
    a.c0.l[k] = in[(0 * 12 + k) * 64 + threadIdx.x];
    a.c1.l[k] = in[(1 * 12 + k) * 64 + threadIdx.x];
    b.c0.l[k] = in[(2 * 12 + k) * 64 + threadIdx.x];
    b.c1.l[k] = in[(3 * 12 + k) * 64 + threadIdx.x];
  }
#pragma unroll 1
  for (int it = 0; it < CB_ITERS; it++) {
    a = {serial_add(a.c0, b.c0), serial_add(a.c1, b.c1)};
    b = {serial_sub(b.c0, a.c0), serial_sub(b.c1, a.c1)};
  }
  for (int k = 0; k < 12; k++) {
    out[(0 * 12 + k) * gridDim.x * 64 + i] = a.c0.l[k];
    out[(1 * 12 + k) * gridDim.x * 64 + i] = a.c1.l[k];
    out[(2 * 12 + k) * gridDim.x * 64 + i] = b.c0.l[k];
    out[(3 * 12 + k) * gridDim.x * 64 + i] = b.c1.l[k];
  }
}

template <int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_a(const uint32_t* in, uint32_t* out) {
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  fp2 a, b;
  for (int k = 0; k < 12; k++) {
    a.c0.l[k] = in[(0 * 12 + k) * 64 + threadIdx.x];
    a.c1.l[k] = in[(1 * 12 + k) * 64 + threadIdx.x];
    b.c0.l[k] = in[(2 * 12 + k) * 64 + threadIdx.x];
    b.c1.l[k] = in[(3 * 12 + k) * 64 + threadIdx.x];
  }
#pragma unroll 1
  for (int it = 0; it < CB_ITERS; it++) {
    a = fp2_add_asm(a, b);
    b = fp2_sub_asm(b, a);
  }
  for (int k = 0; k < 12; k++) {
    out[(0 * 12 + k) * gridDim.x * 64 + i] = a.c0.l[k];
    out[(1 * 12 + k) * gridDim.x * 64 + i] = a.c1.l[k];
    out[(2 * 12 + k) * gridDim.x * 64 + i] = b.c0.l[k];
    out[(3 * 12 + k) * gridDim.x * 64 + i] = b.c1.l[k];
  }
}

int main() {
  const int words = 48 * 64;
  uint32_t h[48 * 64];
  srand(7);
  // values < 2p: random 380-bit words (top word small)
  for (int k = 0; k < 48; k++)
    for (int l = 0; l < 64; l++) h[k * 64 + l] = (k % 12 == 11) ? (uint32_t)(rand() & 0x0fffffff) : (uint32_t)rand() * 2654435761u;
  uint32_t *din, *dout_c, *dout_a, *dout_s;
  const int maxblocks = 256 * 4 * 2;
  hipMalloc(&din, words * 4);
  hipMalloc(&dout_c, (size_t)maxblocks * words * 4);
  hipMalloc(&dout_a, (size_t)maxblocks * words * 4);
  hipMalloc(&dout_s, (size_t)maxblocks * words * 4);
  hipMemcpy(din, h, words * 4, hipMemcpyHostToDevice);
  for (int w : {1, 2}) {
    const int blocks = 256 * 4 * w;
    float ms[3] = {0, 0, 0};
    for (int v = 0; v < 3; v++) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      for (int rep = 0; rep < 3; rep++) {
        hipEventRecord(e0);
        if (v == 0)
          hipLaunchKernelGGL(w == 1 ? k_c<1> : k_c<2>, dim3(blocks), dim3(64), 0, 0, din, dout_c);
        else if (v == 1)
          hipLaunchKernelGGL(w == 1 ? k_a<1> : k_a<2>, dim3(blocks), dim3(64), 0, 0, din, dout_a);
        else
          hipLaunchKernelGGL(w == 1 ? k_s<1> : k_s<2>, dim3(blocks), dim3(64), 0, 0, din, dout_s);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        hipEventElapsedTime(&ms[v], e0, e1);
      }
    }
    static uint32_t oc[256 * 4 * 2 * 48 * 64], oa[256 * 4 * 2 * 48 * 64], os[256 * 4 * 2 * 48 * 64];
    hipMemcpy(os, dout_s, (size_t)blocks * words * 4, hipMemcpyDeviceToHost);
    hipMemcpy(oc, dout_c, (size_t)blocks * words * 4, hipMemcpyDeviceToHost);
    hipMemcpy(oa, dout_a, (size_t)blocks * words * 4, hipMemcpyDeviceToHost);
    const bool same = !memcmp(oc, oa, (size_t)blocks * words * 4) && !memcmp(oc, os, (size_t)blocks * words * 4);
    // ns per (fp2_add + fp2_sub) pair per wave
    printf("{\"waves_per_simd\": %d, \"compiled_ms\": %.4f, \"asm_interleaved_ms\": %.4f, \"serial_vcc_ms\": %.4f, \"serial_over_interleaved\": %.3f, \"identical\": %s}\n",
           w, ms[0], ms[1], ms[2], ms[2] / ms[1], same ? "true" : "false");
  }
  return 0;
}

// Per-operation latency of the latency engine's primitives (wfield.h / wteam.h) on an MI355X: one
// workgroup of eight waves (the k_lat shape); an op runs `iters` times back to back on wave 0 alone
// ("lone") or on waves 0..5 at once ("six": two waves share SIMDs 0 and 1, as in a team round), and
// the device wall clock brackets the loop. Team modes time a whole team round (op + team_sync).
//   hipcc --offload-arch=gfx950 -O3 -o wvbench wvbench.hip && ./wvbench
#define WV_WAVES 8
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../drand_amd/csrc/kcommon.h"
#include "../drand_amd/csrc/wvteam.h"

namespace wv {
__device__ uint64_t g_lat_trace[LAT_TRACE_N];
__device__ uint32_t g_lat_trace_on;  // wfield.h WV_MARK: off here (no trace in the microbenchmark)
}
using namespace wv;

enum { OP_MULP, OP_SQRP, OP_DOT1, OP_DOT3, OP_DOT6, OP_SQR2, OP_INV2, OP_INV1, OP_ISZERO, OP_SYNC, OP_TEAM_CYC, OP_TEAM_MUL,
       OP_N };
static const char* NAMES[OP_N] = {"mulp", "sqrp", "dot1", "dot3", "dot6", "sqr2", "inv_pair_nz", "inv_dup", "is_zero2",
                                  "team_sync8", "team_cyc_sqr8", "team_mul8"};

__global__ void __launch_bounds__(512) k_wvbench(int op, int six, int iters, uint64_t* out) {
  team_init();
  wv_init();
  __syncthreads();
  const int w = wave_id();
  F a = cst(WC_SSWU_Z), b = cst(WC_B2);
  const bool team = op >= OP_SYNC;
  const bool active = team || (six ? w < 6 : w == 0);
  uint64_t t0 = 0, t1 = 0;
  uint32_t keep = 0;
  if (team) {
    Team t = make_team(ALL_WAVES, CTR_ALL);
    if (w == 0) {
      W12 f;
      for (int k = 0; k < 6; k++) f.c[k] = k & 1 ? a : b;
      xst_w12(W_G, f);
      xst_w12(W_S, f);
    }
    team_sync(t);
    t0 = wall_clock64();
    int in = W_G, o = W_S;
    for (int i = 0; i < iters; i++) {
      if (op == OP_SYNC) team_sync(t);
      else if (op == OP_TEAM_CYC) team_op(t, o, [&](int c) { return w12_cyc_sqr_c(xld_w12(in), c); });
      else team_op(t, o, [&](int c) { return w12_mul_c(xld_w12(in), xld_w12(W_G), c); });
      const int x = in;
      in = o;
      o = x == W_G ? W_P : x;
    }
    t1 = wall_clock64();
    keep = xld(in).x;
  } else if (active) {
    t0 = wall_clock64();
#pragma unroll 1
    for (int i = 0; i < iters; i++) {
      switch (op) {
        case OP_MULP: a = mulp(a, b); break;
        case OP_SQRP: a = sqrp(a); break;
        case OP_DOT1: a = dot(a, b); break;
        case OP_DOT3: a = dot(a, b, b, a, a, a); break;
        case OP_DOT6: a = dot(a, b, b, a, a, a, b, b, a, b, b, a); break;
        case OP_SQR2: a = sqr2(a); break;
        case OP_INV2: a = inv_pair_nz(a); break;
        case OP_INV1: a = inv_dup(a); break;
        default: a = is_zero2(a) ? b : add(a, zero()); break;
      }
    }
    t1 = wall_clock64();
    keep = a.x;
  }
  if (active && (threadIdx.x & 63u) == 0u) {
    out[2 * w] = t1 - t0;
    out[2 * w + 1] = keep;
  }
}

int main() {
  uint64_t* d;
  if (hipMalloc(&d, 16 * sizeof(uint64_t)) != hipSuccess) return 1;
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || khz <= 0) return 1;
  const double tick_us = 1000.0 / khz;
  printf("{\"wall_clock_khz\": %d", khz);
  for (int op = 0; op < OP_N; op++) {
    for (int six = 0; six < (op < OP_SYNC ? 2 : 1); six++) {
      const int iters = (op == OP_INV2 || op == OP_INV1) ? 20 : 400;
      uint64_t h[16] = {};
      for (int rep = 0; rep < 2; rep++) {  // the first launch warms the code object
        hipMemset(d, 0, sizeof h);
        hipLaunchKernelGGL(k_wvbench, dim3(1), dim3(512), 0, 0, op, six, iters, d);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
      }
      hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
      uint64_t mx = 0;
      for (int w = 0; w < 8; w++) mx = h[2 * w] > mx ? h[2 * w] : mx;
      printf(", \"%s%s\": %.3f", NAMES[op], op < OP_SYNC ? (six ? "_six" : "_lone") : "", mx * tick_us / iters);
    }
  }
  printf(", \"unit\": \"us per op\"}\n");
  return 0;
}

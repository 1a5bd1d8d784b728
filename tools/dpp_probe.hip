// Probe of the cross-lane primitives the wave-cooperative latency engine (drand_amd/csrc/wv.h)
// relies on, on the real gfx950: prints PASS/FAIL per primitive against the lane mapping wv.h's
// host emulation assumes (the host build of the engine is only as good as that emulation).
//   row_newbcast:i   lane l <- lane 16*(l/16) + i
//   row_shr:j        lane l <- lane l-j within its row of 16, 0 when l%16 < j (bound_ctrl)
//   row_shl:j        lane l <- lane l+j within its row, 0 past the row end
//   wave_shr:1       lane l <- lane l-1 across the whole wave, lane 0 <- 0
//   row_mask         rows outside the mask keep `old`
//   permlane16_swap  first: odd rows <- second arg's even rows; second: even rows <- first arg's odd rows
//   permlane32_swap  first: rows 2,3 <- second arg's rows 0,1; second: rows 0,1 <- first arg's rows 2,3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

__global__ void probe(uint32_t* out) {
  const uint32_t l = threadIdx.x;
  const uint32_t x = 100 + l, y = 1000 + l;
  out[0 * 64 + l] = __builtin_amdgcn_update_dpp(0u, x, 0x150 + 5, 0xf, 0xf, false);  // row_newbcast:5
  out[1 * 64 + l] = __builtin_amdgcn_update_dpp(0u, x, 0x110 + 3, 0xf, 0xf, true);   // row_shr:3
  out[2 * 64 + l] = __builtin_amdgcn_update_dpp(0u, x, 0x100 + 5, 0xf, 0xf, true);   // row_shl:5
  out[3 * 64 + l] = __builtin_amdgcn_update_dpp(0u, x, 0x138, 0xf, 0xf, true);       // wave_shr:1
  uint32_t m = __builtin_amdgcn_update_dpp(7u, x, 0x110 + 2, 0x5, 0xf, true);        // row_shr:2 rows 0,2
  out[4 * 64 + l] = __builtin_amdgcn_update_dpp(m, x, 0x100 + 3, 0xa, 0xf, true);    // row_shl:3 rows 1,3
  auto p = __builtin_amdgcn_permlane16_swap(x, y, false, false);
  out[5 * 64 + l] = p[0];
  out[6 * 64 + l] = p[1];
  auto q = __builtin_amdgcn_permlane32_swap(x, y, false, false);
  out[7 * 64 + l] = q[0];
  out[8 * 64 + l] = q[1];
  out[9 * 64 + l] = (uint32_t)(__builtin_amdgcn_ballot_w64(l % 3 == 0) >> (l & 32));
}

static uint32_t expect(int t, uint32_t l) {
  const uint32_t x0 = 100, y0 = 1000, row = l / 16, r = l % 16;
  switch (t) {
    case 0: return x0 + 16 * row + 5;
    case 1: return r >= 3 ? x0 + l - 3 : 0;
    case 2: return r + 5 < 16 ? x0 + l + 5 : 0;
    case 3: return l >= 1 ? x0 + l - 1 : 0;
    case 4: return (row & 1) == 0 ? (r >= 2 ? x0 + l - 2 : 0) : (r + 3 < 16 ? x0 + l + 3 : 0);
    case 5: return (row & 1) ? y0 + l - 16 : x0 + l;
    case 6: return (row & 1) ? y0 + l : x0 + l + 16;
    case 7: return row >= 2 ? y0 + l - 32 : x0 + l;
    case 8: return row >= 2 ? y0 + l : x0 + l + 32;
    default: {
      uint64_t b = 0;
      for (int k = 0; k < 64; k++) b |= (uint64_t)(k % 3 == 0) << k;
      return (uint32_t)(b >> (l & 32));
    }
  }
}

int main() {
  const char* names[] = {"row_newbcast:5", "row_shr:3", "row_shl:5", "wave_shr:1", "row_mask shr/shl",
                         "permlane16_swap.first", "permlane16_swap.second", "permlane32_swap.first",
                         "permlane32_swap.second", "ballot_w64"};
  uint32_t* d = nullptr;
  if (hipMalloc(&d, 10 * 64 * 4) != hipSuccess) return 2;
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
  uint32_t h[10 * 64];
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  int bad = 0;
  for (int t = 0; t < 10; t++) {
    int ok = 1;
    for (uint32_t l = 0; l < 64; l++) ok &= h[t * 64 + l] == expect(t, l);
    printf("%-24s %s\n", names[t], ok ? "PASS" : "FAIL");
    if (!ok) {
      bad++;
      for (uint32_t l = 0; l < 64; l++) printf("%u%c", h[t * 64 + l], l == 63 ? '\n' : ' ');
    }
  }
  hipFree(d);
  printf("dpp_probe %s\n", bad ? "FAILED" : "ok");
  return bad ? 1 : 0;
}

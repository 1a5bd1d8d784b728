// Structure-of-arrays staging layout in HBM for inter-kernel hand-off.
// An object of S Fp "slots" for item i lives at buf[(slot*12 + limb) * n + i]: lane-consecutive
// items are word-consecutive, so every load/store of a wave is one coalesced 256-byte access.
#pragma once
#include "tower.h"

namespace bls {

DI void st_fp(uint32_t* buf, size_t n, size_t i, int slot, const fp& a) {
#pragma unroll
  for (int k = 0; k < 12; k++) buf[(size_t)(slot * 12 + k) * n + i] = a.l[k];
}

DI fp ld_fp(const uint32_t* buf, size_t n, size_t i, int slot) {
  fp a;
#pragma unroll
  for (int k = 0; k < 12; k++) a.l[k] = buf[(size_t)(slot * 12 + k) * n + i];
  return a;
}

DI void st_fp2(uint32_t* buf, size_t n, size_t i, int slot, const fp2& a) {
  st_fp(buf, n, i, slot, a.c0);
  st_fp(buf, n, i, slot + 1, a.c1);
}

DI fp2 ld_fp2(const uint32_t* buf, size_t n, size_t i, int slot) {
  return {ld_fp(buf, n, i, slot), ld_fp(buf, n, i, slot + 1)};
}

DI void st_fp12(uint32_t* buf, size_t n, size_t i, const fp12& a) {
  st_fp2(buf, n, i, 0, a.c0.c0);
  st_fp2(buf, n, i, 2, a.c0.c1);
  st_fp2(buf, n, i, 4, a.c0.c2);
  st_fp2(buf, n, i, 6, a.c1.c0);
  st_fp2(buf, n, i, 8, a.c1.c1);
  st_fp2(buf, n, i, 10, a.c1.c2);
}

DI fp12 ld_fp12(const uint32_t* buf, size_t n, size_t i) {
  fp12 a;
  a.c0.c0 = ld_fp2(buf, n, i, 0);
  a.c0.c1 = ld_fp2(buf, n, i, 2);
  a.c0.c2 = ld_fp2(buf, n, i, 4);
  a.c1.c0 = ld_fp2(buf, n, i, 6);
  a.c1.c1 = ld_fp2(buf, n, i, 8);
  a.c1.c2 = ld_fp2(buf, n, i, 10);
  return a;
}

}  // namespace bls

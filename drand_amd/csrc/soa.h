// Structure-of-arrays staging layout in HBM for inter-kernel hand-off.
// An object of S Fp "slots" for item i lives at buf[(slot*12 + limb) * n + i]: lane-consecutive
// items are word-consecutive, so every load/store of a wave is one coalesced 256-byte access.
#pragma once
#include "tower.h"

namespace bls {


#ifdef BLS_HOST
template <int AUX = 0>
DI void st_fp(uint32_t* buf, size_t n, size_t i, int slot, const fp& a) {
#pragma unroll
  for (int k = 0; k < 12; k++) buf[(size_t)(slot * 12 + k) * n + i] = a.l[k];
}

template <int AUX = 0>
DI fp ld_fp(const uint32_t* buf, size_t n, size_t i, int slot) {
  fp a;
#pragma unroll
  for (int k = 0; k < 12; k++) a.l[k] = buf[(size_t)(slot * 12 + k) * n + i];
  return a;
}
#else
// Device form through buffer resources: the slot's 12 words are one resource (base = the slot's
// first column, at most 12 n words), the item's byte offset i * 4 is the one VGPR offset and each
// word's k * n * 4 an SGPR offset recomputed at its use (an opaque stride keeps LLVM from hoisting a
// kernel's hundreds of distinct offsets into SGPRs it then spills) -- no 64-bit VGPR address per
// word. Against plain global pointers (r04 A/B, profiles/r04i_soabuf_team_f_ab.json): scratch of the
// 3-lane final exponentiation 480 -> 128 B/lane, cofactor clearing 1,884 -> 988, the 3-lane f pass
// 1,328 -> 144; 2.100 -> 2.129 M beacons/s on one box. Loads past the resource return 0, never fault.
DI __amdgpu_buffer_rsrc_t soa_slot_rsrc(const uint32_t* buf, size_t n, int slot) {
  const size_t bytes = (size_t)12 * n * 4;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf) + (size_t)slot * 12 * n, 0,
                                           (int)(bytes < 0x7fffffffu ? bytes : 0x7fffffffu), 0x00020000);
}
DI uint32_t soa_word_off(size_t n, int k) {
  uint32_t n4 = (uint32_t)(n * 4);
  asm volatile("" : "+s"(n4));
  return (uint32_t)k * n4;
}
// AUX: the cache-policy bits of the access (0: default; gfx950 NT = 2 streams past the caches)
template <int AUX = 0>
DI void st_fp(uint32_t* buf, size_t n, size_t i, int slot, const fp& a) {
  const __amdgpu_buffer_rsrc_t r = soa_slot_rsrc(buf, n, slot);
#pragma unroll
  for (int k = 0; k < 12; k++) __builtin_amdgcn_raw_buffer_store_b32(a.l[k], r, (uint32_t)(i * 4), soa_word_off(n, k), AUX);
}

template <int AUX = 0>
DI fp ld_fp(const uint32_t* buf, size_t n, size_t i, int slot) {
  const __amdgpu_buffer_rsrc_t r = soa_slot_rsrc(buf, n, slot);
  fp a;
#pragma unroll
  for (int k = 0; k < 12; k++) a.l[k] = __builtin_amdgcn_raw_buffer_load_b32(r, (uint32_t)(i * 4), soa_word_off(n, k), AUX);
  return a;
}
#endif

// A lane-varying slot (the 3-lane layouts pick slots by lane role): the buffer form keeps ONE
// resource over the whole object -- at most 12 Fp slots from `buf` (an Fp12, a line pair's six
// slots) -- since a resource must be wave-uniform, and moves the slot into the VGPR offset; the
// host form is the same as st_fp / ld_fp.
#ifdef BLS_HOST
DI void st_fp_v(uint32_t* buf, size_t n, size_t i, int slot, const fp& a) { st_fp(buf, n, i, slot, a); }
template <int AUX = 0>
DI fp ld_fp_v(const uint32_t* buf, size_t n, size_t i, int slot) { return ld_fp(buf, n, i, slot); }
#else
DI __amdgpu_buffer_rsrc_t soa_obj_rsrc(const uint32_t* buf, size_t n, int slots) {
  const size_t bytes = (size_t)slots * 12 * n * 4;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(buf), 0,
                                           (int)(bytes < 0x7fffffffu ? bytes : 0x7fffffffu), 0x00020000);
}
DI void st_fp_v(uint32_t* buf, size_t n, size_t i, int slot, const fp& a) {
  const __amdgpu_buffer_rsrc_t r = soa_obj_rsrc(buf, n, 12);
  const uint32_t vo = (uint32_t)(((size_t)slot * 12 * n + i) * 4);
#pragma unroll
  for (int k = 0; k < 12; k++) __builtin_amdgcn_raw_buffer_store_b32(a.l[k], r, vo, soa_word_off(n, k), 0);
}
template <int AUX = 0>
DI fp ld_fp_v(const uint32_t* buf, size_t n, size_t i, int slot) {
  const __amdgpu_buffer_rsrc_t r = soa_obj_rsrc(buf, n, 12);
  const uint32_t vo = (uint32_t)(((size_t)slot * 12 * n + i) * 4);
  fp a;
#pragma unroll
  for (int k = 0; k < 12; k++) a.l[k] = __builtin_amdgcn_raw_buffer_load_b32(r, vo, soa_word_off(n, k), AUX);
  return a;
}
#endif
DI void st_fp2_v(uint32_t* buf, size_t n, size_t i, int slot, const fp2& a) {
  st_fp_v(buf, n, i, slot, a.c0);
  st_fp_v(buf, n, i, slot + 1, a.c1);
}
template <int AUX = 0>
DI fp2 ld_fp2_v(const uint32_t* buf, size_t n, size_t i, int slot) {
  return {ld_fp_v<AUX>(buf, n, i, slot), ld_fp_v<AUX>(buf, n, i, slot + 1)};
}

template <int AUX = 0>
DI void st_fp2(uint32_t* buf, size_t n, size_t i, int slot, const fp2& a) {
  st_fp<AUX>(buf, n, i, slot, a.c0);
  st_fp<AUX>(buf, n, i, slot + 1, a.c1);
}

template <int AUX = 0>
DI fp2 ld_fp2(const uint32_t* buf, size_t n, size_t i, int slot) {
  return {ld_fp<AUX>(buf, n, i, slot), ld_fp<AUX>(buf, n, i, slot + 1)};
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

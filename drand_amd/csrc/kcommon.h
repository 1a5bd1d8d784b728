// Shared prelude of the stage-kernel translation units (see kernels.h for the pipeline).
#pragma once
#include "kernels.h"
#include "hash.h"
#include "pairing.h"
#include "soa.h"
#include "tri.h"

namespace blsk {
using namespace bls;

constexpr int TPB = 64;  // one wave per workgroup: register-heavy lanes, many workgroups per CU

static inline unsigned grid_for(size_t n) { return (unsigned)((n + TPB - 1) / TPB); }

// Waves per SIMD each stage kernel is compiled for (amdgpu_waves_per_eu caps its VGPR budget at
// 512 / n). 1 = the full 512 VGPR+AGPR budget; 2 = 256 VGPRs, twice the resident waves, some
// spilling. Chosen per kernel from same-box A/B runs on the MI355X (scripts/gpu_check.sh,
// DESIGN.md §4.3); the hash-to-G2 phases have their own knobs in k_hash.hip (BLS_WPE_HASH_A/B/C),
// the subgroup check in k_decomp.hip, the 3-lane kernels in k_miller.hip / k_fexp.hip.
#ifndef BLS_WPE_DECOMP
#define BLS_WPE_DECOMP 4
#endif
#ifndef BLS_WPE_LINES
#define BLS_WPE_LINES 2
#endif
#ifndef BLS_WPE_MILLER_F
#define BLS_WPE_MILLER_F 1
#endif
#ifndef BLS_WPE_FEXP
#define BLS_WPE_FEXP 1
#endif
// amdgpu_waves_per_eu(n) asks for AT LEAST n waves/SIMD and the compiler may settle for fewer (it
// gives the 4-wave exponentiation kernels 145 VGPRs = 3 waves); min = max = n measured no better.
#define BLS_KERNEL(wpe) __global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(wpe)))

}  // namespace blsk

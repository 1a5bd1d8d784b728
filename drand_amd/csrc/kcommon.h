// Shared prelude of the stage-kernel translation units (see kernels.h for the pipeline).
#pragma once
#include "kernels.h"
#include "hash.h"
#include "pairing.h"
#include "soa.h"

namespace blsk {
using namespace bls;

constexpr int TPB = 64;  // one wave per workgroup: register-heavy lanes, many workgroups per CU

static inline unsigned grid_for(size_t n) { return (unsigned)((n + TPB - 1) / TPB); }

}  // namespace blsk

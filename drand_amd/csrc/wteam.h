// Teams of waves for the latency engine: the waves of one workgroup cooperate on ONE item. A wave
// still computes whole field values (wfield.h, limbs across its lanes); a team splits the independent
// outputs of an operation (the six coefficients of an Fp12 product, the pieces of a Miller step)
// across its waves, which exchange the results through the workgroup's LDS.
//
//   exchange  a value lives in an LDS slot of 64 words (lane l's word at l); xst / xld
//   team sync a monotonic LDS counter per team: every wave adds one and waits for gen * n -- waves of
//             different teams run different code; a team of the whole workgroup (phases B and C,
//             where every wave runs the same sequence of syncs) uses the hardware barrier instead
//
// Host build: each wave of the workgroup is a std::thread running the same function (wvtest), the
// slots carry their values' bounds, and the counters are std::atomic.
#pragma once
#include "wfield.h"

#ifdef WV_HOST
#include <atomic>
#include <thread>
#endif

namespace wv {

// the polling waves' back-off between counter reads (s_sleep units of 64 clocks; 0: none)
#ifndef WV_POLL_SLEEP
#define WV_POLL_SLEEP 0
#endif
#ifndef WV_BLK_SLOTS
#define WV_BLK_SLOTS 128
#endif
constexpr int BLK_SLOTS = WV_BLK_SLOTS;
constexpr int BLK_CTRS = 16;  // team counters
constexpr int BLK_WORDS_EXTRA = 64;  // scalar words (verdicts, flags)

#ifdef WV_HOST
extern uint32_t g_host_blk[BLK_SLOTS * 64 + BLK_WORDS_EXTRA];
extern double g_host_blk_b[BLK_SLOTS];
extern std::atomic<uint32_t> g_host_ctr[BLK_CTRS];
inline uint32_t* blk_base() { return g_host_blk; }
inline int wave_id() { return g_host_wave; }
#else
static __shared__ uint32_t g_wv_blk[BLK_SLOTS * 64 + BLK_WORDS_EXTRA + BLK_CTRS];
WVI uint32_t* blk_base() { return g_wv_blk; }
WVI int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
#endif

WVI void xst(int slot, const F& v) {
  lds_st(blk_base() + slot * 64, lane_id(), v.x);
#ifdef WV_HOST
  g_host_blk_b[slot] = v.b;
#endif
}
WVI F xld(int slot) {
#ifdef WV_HOST
  return mkF(lds_ld(blk_base() + slot * 64, lane_id()), g_host_blk_b[slot]);
#else
  return {lds_ld(blk_base() + slot * 64, lane_id())};
#endif
}
// a wave-uniform scalar word (written by one lane, read by all)
WVI void xst_word(int i, uint32_t v) {
  uint32_t* p = blk_base() + BLK_SLOTS * 64 + i;
#ifdef WV_HOST
  *p = v;
#else
  if (threadIdx.x % 64 == 0) *p = v;
#endif
}
WVI uint32_t xld_word(int i) {
  const uint32_t* p = blk_base() + BLK_SLOTS * 64 + i;
#ifdef WV_HOST
  return *p;
#else
  return __builtin_amdgcn_readfirstlane(*(volatile const uint32_t*)p);
#endif
}

struct Team {
  int n, id;     // members; this wave's index among them (waves in increasing order)
  int ctr;       // its counter
  uint32_t gen;  // syncs passed
  bool whole;    // every wave of the workgroup: team_sync is the hardware barrier
};
// the waves of `mask` (bit w = wave w); only members may call team_sync
WVI Team make_team(uint32_t mask, int ctr) {
  const uint32_t below = mask & ((1u << wave_id()) - 1u);
#ifdef WV_HOST
  const bool whole = false;
#else
  const bool whole = __builtin_popcount(mask) * 64 == (int)blockDim.x;
#endif
  return {__builtin_popcount(mask), __builtin_popcount(below), ctr, 0u, whole};
}

WVI void team_sync(Team& t) {
  t.gen++;
  const uint32_t target = t.gen * (uint32_t)t.n;
#ifdef WV_HOST
  g_host_ctr[t.ctr].fetch_add(1, std::memory_order_acq_rel);
  while (g_host_ctr[t.ctr].load(std::memory_order_acquire) < target) std::this_thread::yield();
#else
  if (t.whole) {  // every wave takes the same sequence of whole-team syncs (uniform control flow)
    __syncthreads();
    return;
  }
  uint32_t* c = blk_base() + BLK_SLOTS * 64 + BLK_WORDS_EXTRA + t.ctr;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (threadIdx.x % 64 == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) <
         target)
    if (WV_POLL_SLEEP) __builtin_amdgcn_s_sleep(WV_POLL_SLEEP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
}

// one-shot hand-off between waves outside a common team: the producer posts after its LDS stores,
// consumers wait for `count` posts
WVI void flag_post(int ctr) {
#ifdef WV_HOST
  g_host_ctr[ctr].fetch_add(1, std::memory_order_acq_rel);
#else
  uint32_t* c = blk_base() + BLK_SLOTS * 64 + BLK_WORDS_EXTRA + ctr;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (threadIdx.x % 64 == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
// flag_post for data this wave wrote to LDS only: a wave's ds operations execute in order in the LDS,
// so a consumer that reads the counter's new value reads the data too; no wait for the stores
WVI void flag_post_lds(int ctr) {
#ifdef WV_HOST
  g_host_ctr[ctr].fetch_add(1, std::memory_order_acq_rel);
#else
  uint32_t* c = blk_base() + BLK_SLOTS * 64 + BLK_WORDS_EXTRA + ctr;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // keeps the compiler from sinking the stores
  if (threadIdx.x % 64 == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#endif
}
WVI void flag_wait(int ctr, uint32_t count) {
#ifdef WV_HOST
  while (g_host_ctr[ctr].load(std::memory_order_acquire) < count) std::this_thread::yield();
#else
  uint32_t* c = blk_base() + BLK_SLOTS * 64 + BLK_WORDS_EXTRA + ctr;
  while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) < count)
    if (WV_POLL_SLEEP) __builtin_amdgcn_s_sleep(WV_POLL_SLEEP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#endif
}

// issue priority of the calling wave among the waves of its SIMD (0 .. 3; the critical path's wave
// runs above the wave that shares its SIMD)
#ifdef WV_HOST
#define WV_PRIO(p) ((void)0)
#else
#define WV_PRIO(p) __builtin_amdgcn_s_setprio(p)
#endif

// the workgroup prologue: counters to zero (then a workgroup barrier before any team sync)
WVI void team_init() {
#ifdef WV_HOST
  // the host driver zeroes the counters before it starts the wave threads
#else
  if (threadIdx.x < BLK_CTRS) blk_base()[BLK_SLOTS * 64 + BLK_WORDS_EXTRA + threadIdx.x] = 0u;
#endif
}

}  // namespace wv

// Internal to libblsverify.so (never installed, no C ABI): the context object and the helpers the
// C-ABI entry points (blsverify.cpp) and the thread-safe service (service.cpp) share.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/blsverify.h"
#include "kernels.h"

namespace blsv_detail {

// Beacons per pipeline pass. The staging of one pass is kStagingBytesPerItem per item (~42.4 KB, 39 KB
// of it the Miller line staging): ~43 GB of the 288 GB at the full 2^20 chunk. A context's chunk is
// capped by blsv_set_chunk / BLSV_CHUNK and halves itself when an allocation fails (ensure_workspace).
constexpr size_t kMaxChunk = size_t(1) << 20;
constexpr size_t kMinChunk = size_t(1) << 14;  // the OOM fallback stops here
// Miller line staging holds a whole chunk. Same-box A/B (profiles/r04k_line_sub_ab.json): 128 Ki
// sub-chunks 216.9 ms, 256 Ki 215.8, the whole chunk 210.7 per 1M (one lines + one f launch instead of
// eight of each, so one wave tail instead of eight).
constexpr size_t kLineSub = kMaxChunk;
constexpr size_t kPkTable = 4096;  // member indices with a precomputed PK_i (drand groups are far smaller)
constexpr size_t kStagingBytesPerItem =
    4 * (blsk::H_WORDS + blsk::HQ_WORDS + blsk::S_WORDS + 4 * blsk::F_WORDS + blsk::MILLER_LINE_WORDS) + 3;
// Every SoA staging object is reached through 32-bit buffer resources (soa.h): num_records is
// min(bytes, 2^31 - 1) and offsets are uint32. The largest object resource (soa_obj_rsrc over 12 Fp
// slots, 576 bytes per item) and the largest VGPR offset ((11 * 12 * n + i) * 4) must fit at the
// largest chunk, or a load past the clamp would silently read 0 (a false reject, never a fault).
static_assert(576ull * kMaxChunk < 0x7fffffffull, "SoA object resource exceeds its 31-bit num_records");
static_assert((133ull * kMaxChunk) * 4 < 0xffffffffull, "SoA VGPR byte offset exceeds 32 bits");
static_assert(48ull * 4 * kMaxChunk < 0x7fffffffull, "3-lane park slot resource exceeds 31 bits");  // park_n < 3.05 n

struct DBuf {
  void* p = nullptr;
  size_t sz = 0;
  ~DBuf() {
    if (p) (void)hipFree(p);
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    sz = 0;
  }
  hipError_t ensure(size_t need) {
    if (need <= sz) return hipSuccess;
    if (p) {
      (void)hipFree(p);
      p = nullptr;
      sz = 0;
    }
    size_t want = std::max(need, size_t(256));
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) sz = want;
    return e;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

// Page-locked host staging (hipHostMalloc): copies from it are truly asynchronous.
struct PinBuf {
  void* p = nullptr;
  size_t sz = 0;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
  hipError_t ensure(size_t need) {
    if (need <= sz) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    sz = 0;
    const size_t want = std::max(need + need / 2, size_t(4096));
    hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
    if (e == hipSuccess) sz = want;
    return e;
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

}  // namespace blsv_detail
using namespace blsv_detail;

// Stage timing (blsv_profile_*): HIP events recorded around every stage launch on the launch stream.
enum Stage { ST_HASH = 0, ST_DECOMP = 1, ST_MILLER = 2, ST_FEXP = 3, ST_FINISH = 4, ST_LAT = 5, ST_N = 6 };
struct ProfRec {
  int stage;
  size_t items;
  hipEvent_t a, b;
};

// Cutover between the latency path (one workgroup per item, k_lat.hip) and the batch pipeline: a batch
// of at most this many items runs on the latency path. BLSV_LAT_MAX overrides it (0 = batch pipeline
// only). Any value is clamped to kMaxChunk: the latency kernels write one class byte per item into the
// chunk-sized class buffer, so a larger batch always takes the chunked pipeline.
constexpr size_t kLatMaxDefault = 1536;  // profiles/r04zk_latency_sweep.json: the paths cross near 1,750
// Default chunk: BLSV_CHUNK (items, rounded up to a multiple of 64, clamped to [kMinChunk, kMaxChunk]),
// else kMaxChunk.
inline size_t chunk_env() {
  static const size_t v = [] {
    const char* e = getenv("BLSV_CHUNK");
    if (!e) return kMaxChunk;
    char* end = nullptr;
    errno = 0;
    const unsigned long long x = strtoull(e, &end, 10);
    if (end == e || *end != '\0' || errno == ERANGE || e[0] == '-' || x == 0) {
      fprintf(stderr, "blsverify: ignoring BLSV_CHUNK=\"%s\" (not a positive integer); chunk stays %zu\n", e, kMaxChunk);
      return kMaxChunk;
    }
    const size_t c = (size_t)std::min<unsigned long long>(std::max<unsigned long long>(x, kMinChunk), kMaxChunk);
    return (c + 63) & ~size_t(63);
  }();
  return v;
}

inline size_t lat_max_env() {
  static const size_t v = [] {
    const char* e = getenv("BLSV_LAT_MAX");
    if (!e) return kLatMaxDefault;
    char* end = nullptr;
    errno = 0;
    const unsigned long long x = strtoull(e, &end, 10);
    if (end == e || *end != '\0' || errno == ERANGE || e[0] == '-') {
      fprintf(stderr, "blsverify: ignoring BLSV_LAT_MAX=\"%s\" (not a non-negative integer); cutover stays %zu\n", e,
              kLatMaxDefault);
      return kLatMaxDefault;
    }
    return (size_t)std::min<unsigned long long>(x, kMaxChunk);
  }();
  return v;
}

struct blsv_ctx {
  int device = 0;
  bool prof = false;
  size_t chunk = chunk_env();                      // items per pipeline pass (blsv_set_chunk)
  size_t lat_max = std::min(lat_max_env(), chunk);  // latency-path cutover, never above the chunk
  uint64_t oom_halvings = 0;                        // times ensure_workspace halved the chunk
  std::vector<ProfRec> recs;
  std::vector<hipEvent_t> event_pool;
  hipStream_t stream = nullptr;
  // decompression runs beside hash-to-G2 (they are independent): a side stream forked from and
  // joined back into the launch stream with these two events
  hipStream_t side = nullptr;
  hipEvent_t fork_ev = nullptr, join_ev = nullptr;
  // the speculative VerifyRecovered's hash-to-G2 of its message from the start of a threshold round
  // (blsverify.cpp spec_recover_launch, launch_lat_hash_key): a second side stream, joined into `side`
  // through hash_ev[slot]. Three streams in all: the boxes run 4 hardware queues per process.
  hipStream_t side2 = nullptr;
  hipEvent_t hash_ev[2] = {nullptr, nullptr};
  std::string err;
  // group
  bool has_group = false;
  size_t t = 0, n = 0;
  DBuf commits, commit_inf;
  std::vector<uint8_t> group_bytes;  // the commitments of the current group (set_group is a no-op on a repeat)
  // PubPoly.Eval(i) for every share index i < min(n, kPkTable), computed once per group on its first
// partials call; indices beyond the table are evaluated per batch
  DBuf pk_all, pk_all_inf;
  size_t pk_all_n = 0;
  bool pk_all_built = false;
  // explicit-pk override (verify_messages with pk48)
  DBuf pk_tab, pk_inf;
  uint8_t pk_cache[48];
  bool pk_cache_valid = false;
  // staging workspace (cap items, at most chunk)
  size_t cap = 0;
  DBuf H, S, F, FW, LN, h_inf, s_inf, cls;
  DBuf HQ;  // hash-to-G2 phase staging (kernels.h HQ_WORDS per item)
  // inputs / outputs
  DBuf in_sigs, in_msgs, in_off, in_len, in_rounds, seeds, bitmap, first_bad, sk, idx, lambdas, scratch, out,
      pp_tab, pp_inf, sel, g1_cls, misc;
  // one packed upload / download per service batch (svc_verify_mixed)
  PinBuf pin;
  // pinned staging of the small copies on the main stream (blsverify.cpp h2d / download_sync): uploads
  // append at io_up_off and wrap after a synchronisation of the stream
  PinBuf io_up, io_down;
  size_t io_up_off = 0;
  // speculative recovery beside a round's partial verification (blsverify.cpp spec_recover_*): two
  // slots (V1, V2), each with its decoded shares, Lagrange coefficients, products and output
  struct SpecSlot {
    DBuf sig, S, s_inf, cls, sel, lam, scratch, out, vmsg, voff, vlen, vcls;
    DBuf hout, saff;  // H(msg) and the recovered signature's affine point (kernels.h kLat*Words)
    PinBuf host;  // staged sigma bytes + indices in, the 96-byte result out (async copies only)
  } spec[2];
  uint64_t spec_hits = 0, spec_misses = 0;  // speculative recoveries kept / recomputed
  DBuf arena;
};

#define HIPCHK(ctx, expr)                                                             \
  do {                                                                                \
    hipError_t e_ = (expr);                                                           \
    if (e_ != hipSuccess) return fail((ctx), BLSV_EHIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

inline int fail(blsv_ctx* ctx, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (ctx) ctx->err = buf;
  return code;
}


// Pipeline staging for min(cnt, chunk) items (rounded to 64). On an out-of-memory failure every
// staging buffer is released, the context's chunk halves (not below kMinChunk) and the allocation is
// retried, so several contexts or ranks sharing one GPU degrade to smaller passes instead of failing.
int ensure_workspace(blsv_ctx* c, size_t cnt);
// Releases the pipeline staging (the next call reallocates what it needs).
void release_workspace(blsv_ctx* c);

// One mixed batch of the thread-safe service (service.cpp): item i verifies sigs96[i] over message i
// (msgs[off[i] .. off[i] + lens[i])) against entry idx[i] of the device G1 table (d_tab, d_tab_inf).
// The latency path up to lat_max items, else the batch pipeline in chunk-sized passes. cls_out gets
// BLSV_REJ_* per item. One host-to-device copy of everything, one device-to-host copy of the classes.
int svc_verify_mixed(blsv_ctx* c, size_t n, const uint8_t* msgs, const uint64_t* off, const uint32_t* lens,
                     const uint8_t* sigs96, const uint32_t* idx, const uint32_t* d_tab, const uint8_t* d_tab_inf,
                     uint8_t* cls_out);

// Host side of the C ABI (include/blsverify.h): context, HBM workspace, chunked stage pipeline.
// Every verdict is computed by the device kernels (kernels.h); this file only moves bytes, sequences
// launches and does the reference's control-flow bookkeeping (share selection order, index parsing).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include <cstdlib>
#include <thread>
#include <vector>

#include "../../include/blsverify.h"
#include "../../include/blsverify_testing.h"
#include "kernels.h"
#include "engine_ctx.h"

void release_workspace(blsv_ctx* c) {
  for (DBuf* d : {&c->H, &c->HQ, &c->S, &c->F, &c->FW, &c->LN, &c->h_inf, &c->s_inf, &c->cls}) d->release();
  c->cap = 0;
}

int ensure_workspace(blsv_ctx* c, size_t cnt) {
  for (;;) {
    size_t want = std::min(std::max(cnt, size_t(64)), c->chunk);
    want = (want + 63) & ~size_t(63);
    if (want <= c->cap) return BLSV_OK;
    hipError_t e = hipSuccess;
    auto need = [&](DBuf& d, size_t bytes) {
      if (e == hipSuccess) e = d.ensure(bytes);
    };
    need(c->H, want * blsk::H_WORDS * 4);
    need(c->HQ, want * blsk::HQ_WORDS * 4);
    need(c->S, want * blsk::S_WORDS * 4);
    need(c->F, want * blsk::F_WORDS * 4);
    need(c->FW, 3 * want * blsk::F_WORDS * 4);
    // LN doubles as the final exponentiation's park
    need(c->LN, std::max(std::min(want, kLineSub) * blsk::MILLER_LINE_WORDS, blsk::FEXP_PARK_WORDS(want)) * 4);
    need(c->h_inf, want);
    need(c->s_inf, want);
    need(c->cls, want);
    static_assert(3 * blsk::F_WORDS >= 48 * 64 / 21 + 1, "FW holds the Miller park of a sub-chunk");
    if (e == hipSuccess) {
      c->cap = want;
      return BLSV_OK;
    }
    release_workspace(c);
    (void)hipGetLastError();  // clear the sticky allocation error
    if (e != hipErrorOutOfMemory || want <= kMinChunk)
      return fail(c, BLSV_EHIP, "staging for %zu items: %s", want, hipGetErrorString(e));
    // out of HBM (other contexts or ranks on this GPU): halve the pass size and retry
    c->chunk = std::max(kMinChunk, ((want / 2) + 63) & ~size_t(63));
    c->lat_max = std::min(c->lat_max, c->chunk);
    c->oom_halvings++;
  }
}

// Small copies on the main stream go through pinned staging: hipMemcpyAsync from pageable memory is
// staged by the runtime and costs ~10 us per copy, which is most of a lone verify's host time.
// Uploads are copied into io_up (the caller's buffer is free on return) and DMA'd from there; the
// staging is appended to and reused from offset 0 only after a synchronisation of the stream, so no
// copy still in flight is overwritten. Downloads land in io_down and reach the caller's buffers after
// the synchronisation download_sync itself does. Larger copies take the pageable path as before.
constexpr size_t kIoCap = size_t(1) << 20;

static hipError_t h2d(blsv_ctx* c, void* dst, const void* src, size_t len) {
  if (!len) return hipSuccess;
  if (len > kIoCap / 4) return hipMemcpyAsync(dst, src, len, hipMemcpyHostToDevice, c->stream);
  if (!c->io_up.p) {
    hipError_t e = c->io_up.ensure(kIoCap);
    if (e != hipSuccess) return e;
  }
  if (c->io_up_off + len > kIoCap) {
    hipError_t e = hipStreamSynchronize(c->stream);
    if (e != hipSuccess) return e;
    c->io_up_off = 0;
  }
  uint8_t* h = c->io_up.as<uint8_t>() + c->io_up_off;
  memcpy(h, src, len);
  c->io_up_off += (len + 63) & ~size_t(63);
  return hipMemcpyAsync(dst, h, len, hipMemcpyHostToDevice, c->stream);
}

struct Down {
  void* user;
  const void* dev;
  size_t len;
};
// every download enqueued, one synchronisation of the main stream, then the bytes to the callers
static hipError_t download_sync(blsv_ctx* c, std::initializer_list<Down> ds) {
  size_t total = 0;
  for (const Down& d : ds) total += (d.len + 63) & ~size_t(63);
  const bool staged = total <= kIoCap && (c->io_down.p || c->io_down.ensure(kIoCap) == hipSuccess);
  hipError_t e = hipSuccess;
  size_t off = 0;
  for (const Down& d : ds) {
    if (!d.len) continue;
    void* to = staged ? (void*)(c->io_down.as<uint8_t>() + off) : d.user;
    if (e == hipSuccess) e = hipMemcpyAsync(to, d.dev, d.len, hipMemcpyDeviceToHost, c->stream);
    off += (d.len + 63) & ~size_t(63);
  }
  const hipError_t es = hipStreamSynchronize(c->stream);
  if (e == hipSuccess) e = es;
  if (e == hipSuccess) c->io_up_off = 0;  // every staged upload has completed too
  if (e != hipSuccess || !staged) return e;
  off = 0;
  for (const Down& d : ds) {
    if (d.len) memcpy(d.user, c->io_down.as<uint8_t>() + off, d.len);
    off += (d.len + 63) & ~size_t(63);
  }
  return hipSuccess;
}

static hipEvent_t take_event(blsv_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// Brackets one stage launch with events when profiling is on (no cost otherwise).
struct StageTimer {
  blsv_ctx* c;
  int stage;
  size_t items;
  hipStream_t st;
  hipEvent_t a = nullptr;
  StageTimer(blsv_ctx* c_, int stage_, size_t items_, hipStream_t st_) : c(c_), stage(stage_), items(items_), st(st_) {
    if (c->prof && (a = take_event(c))) (void)hipEventRecord(a, st);
  }
  ~StageTimer() {
    if (!a) return;
    hipEvent_t b = take_event(c);
    if (!b) return;
    (void)hipEventRecord(b, st);
    c->recs.push_back({stage, items, a, b});
  }
};

// reduce a 32-byte big-endian scalar mod r -> 8 little-endian words
static void scalar_mod_r(const uint8_t* be32, uint32_t out[8]) {
  static const uint32_t R[8] = {0x00000001u, 0xffffffffu, 0xfffe5bfeu, 0x53bda402u,
                                0x09a1d805u, 0x3339d808u, 0x299d7d48u, 0x73eda753u};
  for (int i = 0; i < 8; i++) {
    const uint8_t* q = be32 + 28 - 4 * i;
    out[i] = ((uint32_t)q[0] << 24) | ((uint32_t)q[1] << 16) | ((uint32_t)q[2] << 8) | q[3];
  }
  for (int rep = 0; rep < 4; rep++) {  // value < 2^256 < 3r: at most 2 subtractions
    bool ge = true;
    for (int i = 7; i >= 0; i--) {
      if (out[i] != R[i]) {
        ge = out[i] > R[i];
        break;
      }
    }
    if (!ge) break;
    uint64_t br = 0;
    for (int i = 0; i < 8; i++) {
      uint64_t d = (uint64_t)out[i] - R[i] - br;
      out[i] = (uint32_t)d;
      br = (d >> 63) & 1;
    }
  }
}

// ---------------------------------------------------------------- Lagrange coefficients on the host
// kyber share.RecoverCommit's basis at 0 ([ext] drand/kyber@d59c3367dcde share/poly.go, restated) over
// Fr for the shares x_i = index_i + 1: lambda_i = prod_{j != i} x_j / (x_j - x_i). Every factor is a
// small integer (|x_j - x_i| < 2^16), so a coefficient is ~2t small products and the t inverses share
// one Fermat inversion (Montgomery's trick): ~30 us for t = 33 against 0.56 ms for the serial
// one-lane-per-coefficient device kernel this replaced, and the recovery no longer waits on it.
namespace hfr {
typedef unsigned __int128 u128;
static const uint64_t RM[4] = {0xffffffff00000001ull, 0x53bda402fffe5bfeull, 0x3339d80809a1d805ull,
                               0x73eda753299d7d48ull};
struct E {
  uint64_t l[4];
};
static bool geq_r(const uint64_t (&a)[5]) {
  if (a[4]) return true;
  for (int i = 3; i >= 0; i--)
    if (a[i] != RM[i]) return a[i] > RM[i];
  return true;
}
static void sub_r(uint64_t (&a)[5]) {
  uint64_t br = 0;
  for (int i = 0; i < 4; i++) {
    const u128 d = (u128)a[i] - RM[i] - br;
    a[i] = (uint64_t)d;
    br = (uint64_t)(d >> 64) & 1u;
  }
  a[4] -= br;
}
static uint64_t n0() {  // -r^-1 mod 2^64 (Newton)
  uint64_t inv = 1;
  for (int k = 0; k < 7; k++) inv *= 2 - RM[0] * inv;
  return (uint64_t)0 - inv;
}
// a b 2^-256 mod r (CIOS), inputs and output < r
static E mul(const E& a, const E& b) {
  static const uint64_t N0 = n0();
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; i++) {
    uint64_t c = 0;
    for (int j = 0; j < 4; j++) {
      const u128 v = (u128)a.l[j] * b.l[i] + t[j] + c;
      t[j] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    u128 v = (u128)t[4] + c;
    t[4] = (uint64_t)v;
    t[5] = (uint64_t)(v >> 64);
    const uint64_t m = t[0] * N0;
    v = (u128)m * RM[0] + t[0];
    c = (uint64_t)(v >> 64);
    for (int j = 1; j < 4; j++) {
      v = (u128)m * RM[j] + t[j] + c;
      t[j - 1] = (uint64_t)v;
      c = (uint64_t)(v >> 64);
    }
    v = (u128)t[4] + c;
    t[3] = (uint64_t)v;
    t[4] = t[5] + (uint64_t)(v >> 64);
  }
  uint64_t r[5] = {t[0], t[1], t[2], t[3], t[4]};
  if (geq_r(r)) sub_r(r);
  return {{r[0], r[1], r[2], r[3]}};
}
static E add(const E& a, const E& b) {
  uint64_t r[5];
  uint64_t c = 0;
  for (int i = 0; i < 4; i++) {
    const u128 v = (u128)a.l[i] + b.l[i] + c;
    r[i] = (uint64_t)v;
    c = (uint64_t)(v >> 64);
  }
  r[4] = c;
  if (geq_r(r)) sub_r(r);
  return {{r[0], r[1], r[2], r[3]}};
}
static const E& r2() {  // 2^512 mod r: 1 doubled 512 times
  static const E v = [] {
    E x = {{1, 0, 0, 0}};
    for (int k = 0; k < 512; k++) x = add(x, x);
    return x;
  }();
  return v;
}
// the Montgomery form of the integer v (|v| < 2^63), negative values as r - |v|
static E from_int(int64_t v) {
  E x = {{(uint64_t)(v < 0 ? -v : v), 0, 0, 0}};
  if (v < 0) {
    uint64_t a[5] = {RM[0], RM[1], RM[2], RM[3], 0};
    uint64_t br = 0;
    for (int i = 0; i < 4; i++) {
      const u128 d = (u128)a[i] - x.l[i] - br;
      a[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) & 1u;
    }
    x = {{a[0], a[1], a[2], a[3]}};
  }
  return mul(x, r2());
}
static E inv(const E& a) {  // a^(r - 2), Montgomery form in and out
  uint64_t e[4] = {RM[0] - 2, RM[1], RM[2], RM[3]};
  E acc = from_int(1);
  for (int i = 255; i >= 0; i--) {
    acc = mul(acc, acc);
    if ((e[i >> 6] >> (i & 63)) & 1u) acc = mul(acc, a);
  }
  return acc;
}
}  // namespace hfr

// lambda_i (plain, canonical, 8 little-endian words each) for the share indices idx[0 .. t)
static void host_lagrange(const uint32_t* idx, size_t t, uint32_t* out) {
  std::vector<hfr::E> num(t), den(t), pre(t + 1);
  for (size_t i = 0; i < t; i++) {
    const int64_t xi = (int64_t)idx[i] + 1;
    hfr::E n = hfr::from_int(1), d = n;
    for (size_t j = 0; j < t; j++) {
      if (j == i) continue;
      const int64_t xj = (int64_t)idx[j] + 1;
      n = hfr::mul(n, hfr::from_int(xj));
      d = hfr::mul(d, hfr::from_int(xj - xi));
    }
    num[i] = n;
    den[i] = d;
  }
  // Montgomery's trick: one inversion for the t denominators (none is 0: the indices are distinct)
  pre[0] = hfr::from_int(1);
  for (size_t i = 0; i < t; i++) pre[i + 1] = hfr::mul(pre[i], den[i]);
  hfr::E run = hfr::inv(pre[t]);
  const hfr::E one_plain = {{1, 0, 0, 0}};
  for (size_t i = t; i-- > 0;) {
    const hfr::E di = hfr::mul(run, pre[i]);  // 1 / den_i
    run = hfr::mul(run, den[i]);
    const hfr::E lam = hfr::mul(hfr::mul(num[i], di), one_plain);  // out of Montgomery form
    for (int w = 0; w < 4; w++) {
      out[i * 8 + 2 * w] = (uint32_t)lam.l[w];
      out[i * 8 + 2 * w + 1] = (uint32_t)(lam.l[w] >> 32);
    }
  }
}

int blsv_test_lagrange(const uint32_t* idx, size_t t, uint32_t* out) {
  if (!idx || !out) return BLSV_EINVAL;
  for (size_t i = 0; i < t; i++)
    for (size_t j = 0; j < i; j++)
      if (idx[i] == idx[j]) return BLSV_EINVAL;
  host_lagrange(idx, t, out);
  return BLSV_OK;
}

// Run stages 2..5 (decompress, miller, final exp, finish) on chunk [base, base + cnt) after
// the hash stage filled H. pk_mode: 0 = group key / override entry 0, 1 = per-item table.
struct PkSel {
  const uint32_t* tab;
  const uint8_t* inf;
  const uint32_t* idx;  // nullptr -> entry 0
};

// Stage 1 (hash-to-G2, `hash` launches it on st) and stage 2 (decompression) side by side: the
// decompression goes to the side stream after everything already queued on st (the previous chunk
// reads S and cls), and st waits for it before the Miller stage. The two stages fill each other's
// wave-round tails, and a small batch pays max(hash, decompress) instead of the sum.
// BLSV_SERIAL_STAGES=1 in the environment runs the two on the launch stream one after the other
// (profiling: per-kernel durations without the overlap).
static bool serial_stages() {
  static const bool on = [] {
    const char* e = getenv("BLSV_SERIAL_STAGES");
    return e && e[0] == '1';
  }();
  return on;
}

template <typename HashFn>
static int run_head(blsv_ctx* c, const uint8_t* d_sigs, size_t stride, size_t offset, size_t base, size_t cnt,
                    hipStream_t st, HashFn hash) {
  if (serial_stages()) {
    {
      StageTimer tm(c, ST_DECOMP, cnt, st);
      blsk::launch_decompress_g2(d_sigs, stride, offset, base, cnt, c->S.as<uint32_t>(), c->s_inf.as<uint8_t>(),
                                 c->cls.as<uint8_t>(), st);
    }
    StageTimer tm(c, ST_HASH, cnt, st);
    hash();
    return BLSV_OK;
  }
  HIPCHK(c, hipEventRecord(c->fork_ev, st));
  HIPCHK(c, hipStreamWaitEvent(c->side, c->fork_ev, 0));
  {
    StageTimer tm(c, ST_DECOMP, cnt, c->side);
    blsk::launch_decompress_g2(d_sigs, stride, offset, base, cnt, c->S.as<uint32_t>(), c->s_inf.as<uint8_t>(),
                               c->cls.as<uint8_t>(), c->side);
  }
  HIPCHK(c, hipEventRecord(c->join_ev, c->side));
  {
    StageTimer tm(c, ST_HASH, cnt, st);
    hash();
  }
  HIPCHK(c, hipStreamWaitEvent(st, c->join_ev, 0));
  return BLSV_OK;
}

// Stages 3..5 (Miller, final exponentiation, finish) after run_head
static int run_tail(blsv_ctx* c, const uint8_t* d_sigs, size_t stride, size_t offset, size_t base, size_t cnt,
                    const PkSel& pk, uint64_t* d_bitmap, unsigned long long* d_first_bad, uint8_t* d_cls_out,
                    hipStream_t st, uint64_t label0 = 0) {
  (void)d_sigs;
  (void)stride;
  (void)offset;
  {
    StageTimer tm(c, ST_MILLER, cnt, st);
    blsk::launch_miller(pk.tab, pk.inf, pk.idx, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->S.as<uint32_t>(),
                        c->s_inf.as<uint8_t>(), c->cls.as<uint8_t>(), cnt, c->F.as<uint32_t>(), c->LN.as<uint32_t>(),
                        std::min(cnt, kLineSub), c->FW.as<uint32_t>(), st);
  }
  {
    StageTimer tm(c, ST_FEXP, cnt, st);
    // the final exponentiation parks its kept squares and 3-lane products in LN (free after the Miller stage)
    blsk::launch_final_exp(c->F.as<uint32_t>(), c->FW.as<uint32_t>(), cnt, c->cls.as<uint8_t>(), st,
                           c->LN.as<uint32_t>());
  }
  {
    StageTimer tm(c, ST_FINISH, cnt, st);
    blsk::launch_finish(c->cls.as<uint8_t>(), base, cnt, d_bitmap, d_first_bad, label0, st);
  }
  if (d_cls_out) HIPCHK(c, hipMemcpyAsync(d_cls_out + base, c->cls.p, cnt, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipGetLastError());
  return BLSV_OK;
}

static void bitmap_words_to_bytes(const std::vector<uint64_t>& w, size_t n, uint8_t* out) {
  for (size_t i = 0; i < (n + 7) / 8; i++) {
    uint8_t b = (uint8_t)(w[i / 8] >> (8 * (i % 8)));
    if (i == (n + 7) / 8 - 1 && (n % 8)) b &= (uint8_t)((1u << (n % 8)) - 1);
    out[i] = b;
  }
}

// latency path of a whole batch (n <= lat_max): `lat(cls)` launches the k_lat kernel writing the
// classes, then the verdicts go through launch_finish as the pipeline's do
template <typename LatFn>
static int run_lat(blsv_ctx* c, size_t n, LatFn lat, uint64_t* d_bitmap, unsigned long long* d_first_bad,
                   uint8_t* d_cls_out, hipStream_t st, uint64_t label0 = 0) {
  {
    StageTimer tm(c, ST_LAT, n, st);
    lat(c->cls.as<uint8_t>());
  }
  blsk::launch_finish(c->cls.as<uint8_t>(), 0, n, d_bitmap, d_first_bad, label0, st);
  if (d_cls_out) HIPCHK(c, hipMemcpyAsync(d_cls_out, c->cls.p, n, hipMemcpyDeviceToDevice, st));
  HIPCHK(c, hipGetLastError());
  return BLSV_OK;
}

// lat_max is clamped to the context's chunk on every path that sets it (the latency kernels write one
// class byte per item into the chunk-sized class buffer); the min keeps the bound local anyway
static bool use_lat(const blsv_ctx* c, size_t n) { return n > 0 && n <= std::min(c->lat_max, c->cap); }

struct NoLat {
  void operator()(uint8_t*) const {}
};

// common host-side driver: hash stage chosen by `hash`, signatures already on device; `lat` (when
// given) runs the whole batch on the latency path instead when it is small enough
template <typename HashFn, typename LatFn = NoLat>
static int verify_driver(blsv_ctx* c, size_t n, const uint8_t* d_sigs, size_t stride, size_t offset, const PkSel& pk,
                         HashFn hash, uint8_t* ok_bitmap, uint64_t* first_bad_idx, uint8_t* reject_class,
                         LatFn lat = LatFn(), bool has_lat = false) {
  const size_t words = (n + 63) / 64;
  int rc = ensure_workspace(c, n);
  if (rc) return rc;
  if (has_lat && use_lat(c, n)) {
    // the kernel's class bytes come back in one copy and the bitmap and first bad index are read
    // off them here (launch_finish's rule): no finish kernel, memset or further copies on a call
    // whose every operation is latency
    {
      StageTimer tm(c, ST_LAT, n, c->stream);
      lat(c->cls.as<uint8_t>());
    }
    HIPCHK(c, hipGetLastError());
    std::vector<uint8_t> own;
    uint8_t* cls = reject_class;
    if (!cls) {
      own.resize(n);
      cls = own.data();
    }
    HIPCHK(c, download_sync(c, {{cls, c->cls.p, n}}));
    uint64_t fb = UINT64_MAX;
    for (size_t i = 0; i < n; i++) {
      if (cls[i] != BLSV_REJ_OK && fb == UINT64_MAX) fb = i;
      if (ok_bitmap) {
        if (i % 8 == 0) ok_bitmap[i / 8] = 0;
        ok_bitmap[i / 8] |= (uint8_t)((cls[i] == BLSV_REJ_OK) << (i % 8));
      }
    }
    if (first_bad_idx) *first_bad_idx = fb;
    return BLSV_OK;
  }
  HIPCHK(c, c->bitmap.ensure(words * 8 + 8));
  HIPCHK(c, c->first_bad.ensure(8));
  HIPCHK(c, hipMemsetAsync(c->first_bad.p, 0xff, 8, c->stream));
  if (reject_class) HIPCHK(c, c->misc.ensure(n + 64));
  for (size_t base = 0; base < n; base += c->cap) {
    const size_t cnt = std::min(c->cap, n - base);
    rc = run_head(c, d_sigs, stride, offset, base, cnt, c->stream, [&]() { hash(base, cnt); });
    if (rc) return rc;
    rc = run_tail(c, d_sigs, stride, offset, base, cnt, pk, c->bitmap.as<uint64_t>(),
                  c->first_bad.as<unsigned long long>(), reject_class ? c->misc.as<uint8_t>() : nullptr, c->stream);
    if (rc) return rc;
  }
  std::vector<uint64_t> w(words + 1, 0);
  uint64_t fb = UINT64_MAX;
  HIPCHK(c, download_sync(c, {{w.data(), c->bitmap.p, words * 8},
                              {&fb, c->first_bad.p, 8},
                              {reject_class, c->misc.p, reject_class ? n : 0}}));
  if (ok_bitmap) bitmap_words_to_bytes(w, n, ok_bitmap);
  if (first_bad_idx) *first_bad_idx = fb;
  return BLSV_OK;
}

static PkSel group_pk(blsv_ctx* c) { return {c->commits.as<uint32_t>(), c->commit_inf.as<uint8_t>(), nullptr}; }

// decode one 48-byte G1 point into (tab, inf) entry 0 on device; returns class via *cls
static int decode_g1(blsv_ctx* c, const uint8_t* pk48, size_t cnt, DBuf& tab, DBuf& inf, std::vector<uint8_t>& cls) {
  HIPCHK(c, tab.ensure(cnt * blsk::G1_WORDS * 4));
  HIPCHK(c, inf.ensure(cnt));
  HIPCHK(c, c->g1_cls.ensure(cnt));
  HIPCHK(c, c->misc.ensure(cnt * 48));
  HIPCHK(c, hipMemcpyAsync(c->misc.p, pk48, cnt * 48, hipMemcpyHostToDevice, c->stream));
  blsk::launch_decompress_g1(c->misc.as<uint8_t>(), cnt, tab.as<uint32_t>(), inf.as<uint8_t>(),
                             c->g1_cls.as<uint8_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  cls.assign(cnt, 0);
  HIPCHK(c, hipMemcpyAsync(cls.data(), c->g1_cls.p, cnt, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

// hash of arbitrary messages (packed) on device into H[0..n)
static int upload_messages(blsv_ctx* c, const uint8_t* msgs, const uint32_t* msg_lens, size_t n) {
  std::vector<uint64_t> off(n + 1, 0);
  for (size_t i = 0; i < n; i++) off[i + 1] = off[i] + msg_lens[i];
  if (off[n] && !msgs) return fail(c, BLSV_EINVAL, "messages: %llu message bytes but no buffer",
                                   (unsigned long long)off[n]);
  HIPCHK(c, c->in_msgs.ensure(off[n] + 1));
  HIPCHK(c, c->in_off.ensure((n + 1) * 8));
  HIPCHK(c, c->in_len.ensure(n * 4 + 4));
  const size_t staged_max = kIoCap / 4;
  HIPCHK(c, h2d(c, c->in_msgs.p, msgs, off[n]));
  HIPCHK(c, h2d(c, c->in_off.p, off.data(), (n + 1) * 8));
  HIPCHK(c, h2d(c, c->in_len.p, msg_lens, n * 4));
  // a pageable copy of the offsets reads them when it runs: keep the vector alive until then
  if ((n + 1) * 8 > staged_max) HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int svc_verify_mixed(blsv_ctx* c, size_t n, const uint8_t* msgs, const uint64_t* off, const uint32_t* lens,
                     const uint8_t* sigs96, const uint32_t* idx, const uint32_t* d_tab, const uint8_t* d_tab_inf,
                     uint8_t* cls_out) {
  if (!n) return BLSV_OK;
  if (n > kMaxChunk) return fail(c, BLSV_EINVAL, "service batch larger than %zu", kMaxChunk);
  (void)hipSetDevice(c->device);
  int rc = ensure_workspace(c, std::min(n, c->chunk));
  if (rc) return rc;
  // packed upload: off[n + 1] | lens[n] | idx[n] | sigs[n][96] | message bytes (8-byte aligned parts)
  const size_t mbytes = off[n];
  const size_t o_len = (n + 1) * 8, o_idx = o_len + ((n * 4 + 7) & ~size_t(7)),
               o_sig = o_idx + ((n * 4 + 7) & ~size_t(7)), o_msg = o_sig + n * 96, total = o_msg + mbytes + 8;
  HIPCHK(c, c->pin.ensure(std::max(total, n + 8)));
  uint8_t* h = c->pin.as<uint8_t>();
  memcpy(h, off, (n + 1) * 8);
  memcpy(h + o_len, lens, n * 4);
  memcpy(h + o_idx, idx, n * 4);
  memcpy(h + o_sig, sigs96, n * 96);
  if (mbytes) memcpy(h + o_msg, msgs, mbytes);
  HIPCHK(c, c->arena.ensure(total));
  HIPCHK(c, c->misc.ensure(n + 64));
  HIPCHK(c, hipMemcpyAsync(c->arena.p, h, total, hipMemcpyHostToDevice, c->stream));
  uint8_t* d = c->arena.as<uint8_t>();
  const uint64_t* d_off = reinterpret_cast<const uint64_t*>(d);
  const uint32_t* d_len = reinterpret_cast<const uint32_t*>(d + o_len);
  const uint32_t* d_idx = reinterpret_cast<const uint32_t*>(d + o_idx);
  const uint8_t* d_sig = d + o_sig;
  const uint8_t* d_msg = d + o_msg;
  if (use_lat(c, n)) {
    blsk::launch_lat_messages(d_msg, d_off, d_len, d_sig, 96, 0, n, d_tab, d_tab_inf, d_idx, c->misc.as<uint8_t>(),
                              nullptr, nullptr, c->stream);
  } else {
    const size_t words = (n + 63) / 64;
    HIPCHK(c, c->bitmap.ensure(words * 8 + 8));
    HIPCHK(c, c->first_bad.ensure(8));
    HIPCHK(c, hipMemsetAsync(c->first_bad.p, 0xff, 8, c->stream));
    for (size_t base = 0; base < n; base += c->cap) {
      const size_t cnt = std::min(c->cap, n - base);
      // the Miller stage indexes pk_idx by the chunk-local item: hand it this pass's slice of the
      // per-item key entries (a batch spans several passes once an OOM halving shrank the chunk)
      const PkSel pk{d_tab, d_tab_inf, d_idx + base};
      rc = run_head(c, d_sig, 96, 0, base, cnt, c->stream, [&]() {
        blsk::launch_hash_messages(d_msg, d_off + base, d_len + base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(),
                                   c->HQ.as<uint32_t>(), c->stream);
      });
      if (rc) return rc;
      rc = run_tail(c, d_sig, 96, 0, base, cnt, pk, c->bitmap.as<uint64_t>(), c->first_bad.as<unsigned long long>(),
                    c->misc.as<uint8_t>(), c->stream);
      if (rc) return rc;
    }
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(h, c->misc.p, n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(cls_out, h, n);
  return BLSV_OK;
}

extern "C" {

const char* blsv_version(void) { return "drand_amd blsverify 0.1 (gfx950)"; }

int blsv_device_count(void) {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

int blsv_create(int device, blsv_ctx** out) {
  if (!out) return BLSV_EINVAL;
  *out = nullptr;
  blsv_ctx* c = new blsv_ctx();
  c->device = device;
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side2, hipStreamNonBlocking);
  for (hipEvent_t& ev : c->hash_ev)
    if (e == hipSuccess) e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork_ev, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->join_ev, hipEventDisableTiming);
  if (e != hipSuccess) {
    fprintf(stderr, "blsv_create: %s\n", hipGetErrorString(e));
    blsv_destroy(c);  // releases whatever was created
    return BLSV_EHIP;
  }
  *out = c;
  return BLSV_OK;
}

void blsv_destroy(blsv_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (hipStream_t s : {c->stream, c->side, c->side2}) {
    if (!s) continue;
    (void)hipStreamSynchronize(s);
    (void)hipStreamDestroy(s);
  }
  for (hipEvent_t ev : c->hash_ev)
    if (ev) (void)hipEventDestroy(ev);
  if (c->fork_ev) (void)hipEventDestroy(c->fork_ev);
  if (c->join_ev) (void)hipEventDestroy(c->join_ev);
  (void)hipDeviceSynchronize();
  for (auto& r : c->recs) {
    (void)hipEventDestroy(r.a);
    (void)hipEventDestroy(r.b);
  }
  for (auto e : c->event_pool) (void)hipEventDestroy(e);
  delete c;
}

const char* blsv_last_error(const blsv_ctx* c) { return c ? c->err.c_str() : "null context"; }

int blsv_synchronize(blsv_ctx* c) {
  if (!c) return BLSV_EINVAL;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int blsv_set_group(blsv_ctx* c, const uint8_t* commits48, size_t t, size_t n) {
  if (!c || !commits48 || t == 0 || t > 65536) return fail(c, BLSV_EINVAL, "set_group: bad arguments");
  (void)hipSetDevice(c->device);
  // the same group again (every caller sets its key per call): nothing to decode or evaluate
  if (c->has_group && c->t == t && c->n == n && c->group_bytes.size() == t * 48 &&
      memcmp(c->group_bytes.data(), commits48, t * 48) == 0)
    return BLSV_OK;
  c->has_group = false;
  c->group_bytes.clear();
  std::vector<uint8_t> cls;
  int rc = decode_g1(c, commits48, t, c->commits, c->commit_inf, cls);
  if (rc) return rc;
  for (size_t i = 0; i < t; i++)
    if (cls[i]) return fail(c, BLSV_EINVAL, "set_group: commitment %zu rejected (class %d)", i, (int)cls[i]);
  c->pk_all_n = 0;  // the PK_i table of the new group is built by the first partials call
  c->pk_all_built = false;
  c->t = t;
  c->n = n;
  c->group_bytes.assign(commits48, commits48 + t * 48);
  c->has_group = true;
  return BLSV_OK;
}

int blsv_verify_chained(blsv_ctx* c, uint64_t first_round, const uint8_t* prev0, size_t prev0_len,
                        const uint8_t* sigs96, size_t n, uint8_t* ok_bitmap, uint64_t* first_bad,
                        uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if (!c->has_group) return fail(c, BLSV_ENOGROUP, "verify_chained: no group key set");
  if (n && (!sigs96 || !prev0 || (prev0_len != 32 && prev0_len != 96)))
    return fail(c, BLSV_EINVAL, "verify_chained: prev0 must be 32 or 96 bytes");
  if (n > SIZE_MAX / 96 - 1) return fail(c, BLSV_EINVAL, "verify_chained: %zu rounds overflow the byte count", n);
  (void)hipSetDevice(c->device);
  HIPCHK(c, c->in_sigs.ensure(n * 96 + 96));
  HIPCHK(c, c->seeds.ensure(96));
  if (n) {
    HIPCHK(c, h2d(c, c->in_sigs.p, sigs96, n * 96));
    HIPCHK(c, h2d(c, c->seeds.p, prev0, prev0_len));
  }
  blsk::ChainedSrc src{c->in_sigs.as<uint8_t>(), c->seeds.as<uint8_t>(), first_round, std::max<uint64_t>(n, 1),
                       (uint32_t)prev0_len};
  uint64_t fb = UINT64_MAX;
  const PkSel pk = group_pk(c);
  int rc = verify_driver(
      c, n, c->in_sigs.as<uint8_t>(), 96, 0, pk,
      [&](size_t base, size_t cnt) {
        blsk::launch_hash_chained(src, base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->HQ.as<uint32_t>(), c->stream);
      },
      ok_bitmap, &fb, reject_class,
      [&](uint8_t* cls) { blsk::launch_lat_chained(src, 0, n, pk.tab, pk.inf, cls, c->stream); }, true);
  if (rc) return rc;
  if (first_bad) *first_bad = fb == UINT64_MAX ? UINT64_MAX : first_round + fb;
  return BLSV_OK;
}

// OR the first cnt bits of src (LSB first) into dst starting at bit pos
static void or_bits_at(uint8_t* dst, const uint8_t* src, size_t cnt, size_t pos) {
  const size_t nb = (cnt + 7) / 8, q = pos / 8, s = pos % 8;
  for (size_t j = 0; j < nb; j++) {
    uint8_t b = src[j];
    if (j == nb - 1 && (cnt % 8)) b &= (uint8_t)((1u << (cnt % 8)) - 1);
    dst[q + j] |= (uint8_t)(b << s);
    if (s && (b >> (8 - s))) dst[q + j + 1] |= (uint8_t)(b >> (8 - s));
  }
}

int blsv_verify_chained_multi(blsv_ctx* const* ctxs, size_t n_ctx, const size_t* shard_counts, uint64_t first_round,
                              const uint8_t* prev0, size_t prev0_len, const uint8_t* sigs96, size_t n,
                              uint8_t* ok_bitmap, uint64_t* first_bad, uint8_t* reject_class) {
  if (!ctxs || n_ctx == 0) return BLSV_EINVAL;
  for (size_t k = 0; k < n_ctx; k++) {
    if (!ctxs[k]) return BLSV_EINVAL;
    for (size_t j = 0; j < k; j++)
      if (ctxs[j] == ctxs[k]) return fail(ctxs[k], BLSV_EINVAL, "verify_chained_multi: context %zu repeated", k);
  }
  blsv_ctx* c0 = ctxs[0];
  for (size_t k = 0; k < n_ctx; k++) {
    if (!ctxs[k]->has_group) return fail(ctxs[k], BLSV_ENOGROUP, "verify_chained_multi: context %zu has no group", k);
    if (ctxs[k]->group_bytes != c0->group_bytes)
      return fail(ctxs[k], BLSV_EINVAL, "verify_chained_multi: context %zu holds another group", k);
  }
  if (n && (!sigs96 || !prev0 || (prev0_len != 32 && prev0_len != 96)))
    return fail(c0, BLSV_EINVAL, "verify_chained_multi: prev0 must be 32 or 96 bytes");
  std::vector<size_t> cnt(n_ctx), start(n_ctx);
  size_t sum = 0;
  for (size_t k = 0; k < n_ctx; k++) {
    cnt[k] = shard_counts ? shard_counts[k] : n / n_ctx + (k < n % n_ctx ? 1 : 0);
    start[k] = sum;
    sum += cnt[k];
  }
  if (sum != n) return fail(c0, BLSV_EINVAL, "verify_chained_multi: shard counts sum to %zu, not %zu", sum, n);
  std::vector<std::vector<uint8_t>> bms(n_ctx);
  std::vector<uint64_t> fbs(n_ctx, UINT64_MAX);
  std::vector<int> rcs(n_ctx, BLSV_OK);
  auto shard = [&](size_t k) {
    if (!cnt[k]) return;
    bms[k].assign((cnt[k] + 7) / 8, 0);
    const bool head = start[k] == 0;
    const uint8_t* halo = head ? prev0 : sigs96 + (start[k] - 1) * 96;  // the true PreviousSig of its first round
    rcs[k] = blsv_verify_chained(ctxs[k], first_round + start[k], halo, head ? prev0_len : 96, sigs96 + start[k] * 96,
                                 cnt[k], bms[k].data(), &fbs[k], reject_class ? reject_class + start[k] : nullptr);
  };
  std::vector<std::thread> th;
  for (size_t k = 1; k < n_ctx; k++)
    if (cnt[k]) th.emplace_back(shard, k);
  shard(0);
  for (auto& t : th) t.join();
  for (size_t k = 0; k < n_ctx; k++)
    if (rcs[k]) return rcs[k];
  uint64_t fb = UINT64_MAX;
  for (size_t k = 0; k < n_ctx; k++) fb = std::min(fb, fbs[k]);
  if (first_bad) *first_bad = fb;
  if (ok_bitmap && n) {
    memset(ok_bitmap, 0, (n + 7) / 8);
    for (size_t k = 0; k < n_ctx; k++)
      if (cnt[k]) or_bits_at(ok_bitmap, bms[k].data(), cnt[k], start[k]);
  }
  return BLSV_OK;
}

int blsv_verify_prevs(blsv_ctx* c, uint64_t first_round, const uint8_t* prevs96, size_t prev0_len,
                      const uint8_t* sigs96, size_t n, uint8_t* ok_bitmap, uint64_t* first_bad,
                      uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if (!c->has_group) return fail(c, BLSV_ENOGROUP, "verify_prevs: no group key set");
  if (n && (!sigs96 || !prevs96 || (prev0_len != 32 && prev0_len != 96)))
    return fail(c, BLSV_EINVAL, "verify_prevs: row 0's prev must be 32 or 96 bytes");
  (void)hipSetDevice(c->device);
  HIPCHK(c, c->in_sigs.ensure(n * 96 + 96));
  HIPCHK(c, c->seeds.ensure(n * 96 + 96));
  if (n) {
    HIPCHK(c, h2d(c, c->in_sigs.p, sigs96, n * 96));
    HIPCHK(c, h2d(c, c->seeds.p, prevs96, n * 96));
  }
  // segments of length 1: every round hashes its own prev row (seeds[i]); row 0 uses prev0_len bytes
  blsk::ChainedSrc src{c->in_sigs.as<uint8_t>(), c->seeds.as<uint8_t>(), first_round, 1, (uint32_t)prev0_len};
  uint64_t fb = UINT64_MAX;
  const PkSel pk = group_pk(c);
  int rc = verify_driver(
      c, n, c->in_sigs.as<uint8_t>(), 96, 0, pk,
      [&](size_t base, size_t cnt) {
        blsk::launch_hash_chained(src, base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->HQ.as<uint32_t>(), c->stream);
      },
      ok_bitmap, &fb, reject_class,
      [&](uint8_t* cls) { blsk::launch_lat_chained(src, 0, n, pk.tab, pk.inf, cls, c->stream); }, true);
  if (rc) return rc;
  if (first_bad) *first_bad = fb == UINT64_MAX ? UINT64_MAX : first_round + fb;
  return BLSV_OK;
}

int blsv_verify_unchained(blsv_ctx* c, const uint64_t* rounds, uint64_t first_round, const uint8_t* sigs96, size_t n,
                          uint8_t* ok_bitmap, uint64_t* first_bad, uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if (!c->has_group) return fail(c, BLSV_ENOGROUP, "verify_unchained: no group key set");
  if (n && !sigs96) return fail(c, BLSV_EINVAL, "verify_unchained: null signatures");
  (void)hipSetDevice(c->device);
  HIPCHK(c, c->in_sigs.ensure(n * 96 + 96));
  if (n) HIPCHK(c, h2d(c, c->in_sigs.p, sigs96, n * 96));
  const uint64_t* d_rounds = nullptr;
  if (rounds && n) {
    HIPCHK(c, c->in_rounds.ensure(n * 8));
    HIPCHK(c, h2d(c, c->in_rounds.p, rounds, n * 8));
    d_rounds = c->in_rounds.as<uint64_t>();
  }
  uint64_t fb = UINT64_MAX;
  const PkSel pk = group_pk(c);
  int rc = verify_driver(
      c, n, c->in_sigs.as<uint8_t>(), 96, 0, pk,
      [&](size_t base, size_t cnt) {
        blsk::launch_hash_unchained(d_rounds, first_round, base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(),
                                    c->HQ.as<uint32_t>(), c->stream);
      },
      ok_bitmap, &fb, reject_class,
      [&](uint8_t* cls) {
        blsk::launch_lat_unchained(d_rounds, first_round, c->in_sigs.as<uint8_t>(), 0, n, pk.tab, pk.inf, cls,
                                   c->stream);
      },
      true);
  if (rc) return rc;
  if (first_bad) *first_bad = fb == UINT64_MAX ? UINT64_MAX : (rounds ? rounds[fb] : first_round + fb);
  return BLSV_OK;
}

int blsv_verify_messages(blsv_ctx* c, const uint8_t* pk48, const uint8_t* msgs, const uint32_t* msg_lens, size_t n,
                         const uint8_t* sigs96, uint8_t* ok_bitmap, uint64_t* first_bad, uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if (n && (!msg_lens || !sigs96)) return fail(c, BLSV_EINVAL, "verify_messages: null arguments");
  (void)hipSetDevice(c->device);
  PkSel pk;
  if (pk48) {
    if (!c->pk_cache_valid || memcmp(c->pk_cache, pk48, 48) != 0) {
      std::vector<uint8_t> cls;
      int rc = decode_g1(c, pk48, 1, c->pk_tab, c->pk_inf, cls);
      if (rc) return rc;
      if (cls[0]) return fail(c, BLSV_EINVAL, "verify_messages: public key rejected (class %d)", (int)cls[0]);
      memcpy(c->pk_cache, pk48, 48);
      c->pk_cache_valid = true;
    }
    pk = {c->pk_tab.as<uint32_t>(), c->pk_inf.as<uint8_t>(), nullptr};
  } else {
    if (!c->has_group) return fail(c, BLSV_ENOGROUP, "verify_messages: no group key set");
    pk = group_pk(c);
  }
  if (n > kMaxChunk) return fail(c, BLSV_EINVAL, "verify_messages: batch larger than %zu", kMaxChunk);
  int rc = upload_messages(c, msgs, msg_lens, n);
  if (rc) return rc;
  HIPCHK(c, c->in_sigs.ensure(n * 96 + 96));
  if (n) HIPCHK(c, h2d(c, c->in_sigs.p, sigs96, n * 96));
  return verify_driver(
      c, n, c->in_sigs.as<uint8_t>(), 96, 0, pk,
      [&](size_t base, size_t cnt) {
        blsk::launch_hash_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>() + base,
                                   c->in_len.as<uint32_t>() + base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(),
                                   c->HQ.as<uint32_t>(), c->stream);
      },
      ok_bitmap, first_bad, reject_class,
      [&](uint8_t* cls) {
        blsk::launch_lat_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>(), c->in_len.as<uint32_t>(),
                                  c->in_sigs.as<uint8_t>(), 96, 0, n, pk.tab, pk.inf, pk.idx, cls, nullptr, nullptr,
                                  c->stream);
      },
      true);
}

// shared by verify_partials / recover: returns per-partial class in cls (host), S staged on device
// msg_lens == nullptr: every partial signs the same msg[0 .. msg_len); else partial i signs its own
// message, msgs packed back to back with msg_lens[i] bytes each.

// PK_i = PubPoly.Eval(i) for every member index below min(n, kPkTable) (key/keys.go:239-241; share
// x = i + 1), built once per group: the partial verifications index this table instead of running
// Horner per partial and call. Lazily, on the group's first partials call, so a set_group that is
// only used for VerifyRecovered never pays the O(t n) G1 work.
static int ensure_pk_table(blsv_ctx* c) {
  if (c->pk_all_built) return BLSV_OK;
  const size_t m = std::min(c->n, kPkTable);
  if (m) {
    std::vector<uint32_t> ident(m);
    for (size_t i = 0; i < m; i++) ident[i] = (uint32_t)i;
    HIPCHK(c, c->idx.ensure(m * 4));
    HIPCHK(c, c->pk_all.ensure(m * blsk::G1_WORDS * 4));
    HIPCHK(c, c->pk_all_inf.ensure(m));
    HIPCHK(c, hipMemcpyAsync(c->idx.p, ident.data(), m * 4, hipMemcpyHostToDevice, c->stream));
    blsk::launch_pubpoly_eval(c->commits.as<uint32_t>(), c->commit_inf.as<uint8_t>(), (uint32_t)c->t,
                              c->idx.as<uint32_t>(), m, c->pk_all.as<uint32_t>(), c->pk_all_inf.as<uint8_t>(),
                              c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // ident must outlive the copy
  }
  c->pk_all_n = m;
  c->pk_all_built = true;
  return BLSV_OK;
}

static int partials_stage(blsv_ctx* c, const uint8_t* msg, size_t msg_len, const uint8_t* partials,
                          size_t partial_len, size_t k, std::vector<uint8_t>& cls, std::vector<uint32_t>& index,
                          const uint32_t* msg_lens = nullptr) {
  cls.assign(k, BLSV_REJ_OK);
  index.assign(k, 0);
  if (!c->has_group) return fail(c, BLSV_ENOGROUP, "partials: no group set");
  if (k > c->chunk) return fail(c, BLSV_EINVAL, "partials: more than the context chunk (%zu) in one call", c->chunk);
  for (size_t i = 0; i < k; i++) {
    if (partial_len < 2) {
      cls[i] = BLSV_REJ_SHARE_INDEX;
      continue;
    }
    const uint8_t* p = partials + i * partial_len;
    index[i] = ((uint32_t)p[0] << 8) | p[1];
    if (partial_len != 98) cls[i] = BLSV_REJ_LENGTH;
  }
  if (partial_len != 98) return BLSV_OK;  // every share has the wrong signature length
  int rc = ensure_pk_table(c);
  if (rc) return rc;
  rc = ensure_workspace(c, k);
  if (rc) return rc;
  if (k > c->cap) return fail(c, BLSV_EINVAL, "partials: more than the context chunk (%zu) in one call", c->cap);
  // H(msg) once per item slot (all identical); the per-item PubPoly.Eval(index) table
  std::vector<uint32_t> lens(k, (uint32_t)msg_len);
  std::vector<uint8_t> packed;
  if (msg_lens) {
    rc = upload_messages(c, msg, msg_lens, k);
  } else {
    packed.reserve(k * msg_len);
    for (size_t i = 0; i < k; i++) packed.insert(packed.end(), msg, msg + msg_len);
    rc = upload_messages(c, packed.data(), lens.data(), k);
  }
  if (rc) return rc;
  HIPCHK(c, c->idx.ensure(k * 4));
  HIPCHK(c, h2d(c, c->idx.p, index.data(), k * 4));
  // PubPoly.Eval(index): the per-group table when every index is a member index (< n), else
  // evaluated for this batch (an index >= n still has a well-defined Eval in kyber)
  bool in_table = true;
  for (size_t i = 0; i < k; i++) in_table = in_table && index[i] < c->pk_all_n;
  std::vector<uint32_t> ident;
  PkSel pk{c->pk_all.as<uint32_t>(), c->pk_all_inf.as<uint8_t>(), c->idx.as<uint32_t>()};
  if (!in_table) {
    HIPCHK(c, c->pp_tab.ensure(k * blsk::G1_WORDS * 4));
    HIPCHK(c, c->pp_inf.ensure(k));
    HIPCHK(c, c->sel.ensure(k * 4));
    ident.resize(k);
    for (size_t i = 0; i < k; i++) ident[i] = (uint32_t)i;
    HIPCHK(c, h2d(c, c->sel.p, ident.data(), k * 4));
    blsk::launch_pubpoly_eval(c->commits.as<uint32_t>(), c->commit_inf.as<uint8_t>(), (uint32_t)c->t,
                              c->idx.as<uint32_t>(), k, c->pp_tab.as<uint32_t>(), c->pp_inf.as<uint8_t>(), c->stream);
    pk = {c->pp_tab.as<uint32_t>(), c->pp_inf.as<uint8_t>(), c->sel.as<uint32_t>()};
  }
  HIPCHK(c, c->in_sigs.ensure(k * partial_len + 96));
  HIPCHK(c, h2d(c, c->in_sigs.p, partials, k * partial_len));
  if (use_lat(c, k)) {
    // one workgroup per partial; the decoded sigmas land in S (stride k) for recover_from. Only the
    // class bytes are read back (below), so no bitmap pass
    StageTimer tm(c, ST_LAT, k, c->stream);
    blsk::launch_lat_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>(), c->in_len.as<uint32_t>(),
                              c->in_sigs.as<uint8_t>(), partial_len, 2, k, pk.tab, pk.inf, pk.idx, c->cls.as<uint8_t>(),
                              c->S.as<uint32_t>(), c->s_inf.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
  } else {
    HIPCHK(c, c->bitmap.ensure(((k + 63) / 64) * 8 + 8));
    HIPCHK(c, c->first_bad.ensure(8));
    HIPCHK(c, hipMemsetAsync(c->first_bad.p, 0xff, 8, c->stream));
    blsk::launch_hash_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>(), c->in_len.as<uint32_t>(), k,
                               c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->HQ.as<uint32_t>(), c->stream);
    rc = run_head(c, c->in_sigs.as<uint8_t>(), partial_len, 2, 0, k, c->stream, []() {});  // hashed above
    if (rc) return rc;
    rc = run_tail(c, c->in_sigs.as<uint8_t>(), partial_len, 2, 0, k, pk, c->bitmap.as<uint64_t>(),
                  c->first_bad.as<unsigned long long>(), nullptr, c->stream);
    if (rc) return rc;
  }
  HIPCHK(c, download_sync(c, {{cls.data(), c->cls.p, k}}));
  return BLSV_OK;
}

int blsv_verify_partials(blsv_ctx* c, const uint8_t* msg, size_t msg_len, const uint8_t* partials, size_t partial_len,
                         size_t k, uint8_t* ok, uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if ((k && (!partials || !ok)) || (msg_len && !msg)) return fail(c, BLSV_EINVAL, "verify_partials: null arguments");
  (void)hipSetDevice(c->device);
  std::vector<uint8_t> cls;
  std::vector<uint32_t> index;
  int rc = partials_stage(c, msg, msg_len, partials, partial_len, k, cls, index);
  if (rc) return rc;
  for (size_t i = 0; i < k; i++) {
    ok[i] = cls[i] == BLSV_REJ_OK;
    if (reject_class) reject_class[i] = cls[i];
  }
  return BLSV_OK;
}

int blsv_verify_partials_multi(blsv_ctx* c, const uint8_t* msgs, const uint32_t* msg_lens, const uint8_t* partials,
                               size_t partial_len, size_t k, uint8_t* ok, uint8_t* reject_class) {
  if (!c) return BLSV_EINVAL;
  if (k && (!partials || !ok || !msgs || !msg_lens)) return fail(c, BLSV_EINVAL, "verify_partials_multi: null arguments");
  (void)hipSetDevice(c->device);
  std::vector<uint8_t> cls;
  std::vector<uint32_t> index;
  int rc = partials_stage(c, msgs, 0, partials, partial_len, k, cls, index, msg_lens);
  if (rc) return rc;
  for (size_t i = 0; i < k; i++) {
    ok[i] = cls[i] == BLSV_REJ_OK;
    if (reject_class) reject_class[i] = cls[i];
  }
  return BLSV_OK;
}

static int recover_from(blsv_ctx* c, const std::vector<uint8_t>& cls, const std::vector<uint32_t>& index, size_t lo,
                        size_t hi, size_t t, size_t n, uint8_t* out_sig96);

int blsv_recover(blsv_ctx* c, const uint8_t* msg, size_t msg_len, const uint8_t* partials, size_t partial_len,
                 size_t k, size_t t, size_t n, uint8_t* out_sig96) {
  if (!c) return BLSV_EINVAL;
  if (!out_sig96 || t == 0 || (k && !partials) || (msg_len && !msg)) return fail(c, BLSV_EINVAL, "recover: bad arguments");
  (void)hipSetDevice(c->device);
  std::vector<uint8_t> cls;
  std::vector<uint32_t> index;
  int rc = partials_stage(c, msg, msg_len, partials, partial_len, k, cls, index);
  if (rc) return rc;
  return recover_from(c, cls, index, 0, k, t, n, out_sig96);
}

// kyber tbls.Recover + share.RecoverCommit ([ext] drand/kyber@d59c3367dcde sign/tbls/tbls.go,
// share/poly.go, restated from the published source; parity unpinned by any reference test):
// walk the shares of items [lo, hi) in input order, skip invalid ones, keep appending valid ones until
// t are held -- a duplicate index counts toward t; then xyCommit keys them by index (duplicates
// collapse) and drops indices >= n; fewer than t distinct -> "not enough good public shares".
// Lagrange at 0 over those t shares (x = index + 1) of the batch partials_stage just decompressed
// into c->S, then the G2 MSM and compression.
// the shares recover_from interpolates: valid ones of [lo, hi) in input order until t are held, then
// deduplicated by index and restricted to indices < n; false when fewer than t distinct remain
static bool select_shares(const std::vector<uint8_t>& cls, const std::vector<uint32_t>& index, size_t lo, size_t hi,
                          size_t t, size_t n, std::vector<uint32_t>& sel, std::vector<uint32_t>& idx) {
  sel.clear();
  idx.clear();
  size_t taken = 0;
  for (size_t i = lo; i < hi && taken < t; i++) {
    if (cls[i] != BLSV_REJ_OK) continue;
    taken++;
    if (index[i] >= n || std::find(idx.begin(), idx.end(), index[i]) != idx.end()) continue;
    sel.push_back((uint32_t)i);
    idx.push_back(index[i]);
  }
  return sel.size() >= t;
}

static int recover_from(blsv_ctx* c, const std::vector<uint8_t>& cls, const std::vector<uint32_t>& index, size_t lo,
                        size_t hi, size_t t, size_t n, uint8_t* out_sig96) {
  std::vector<uint32_t> sel, idx;
  if (!select_shares(cls, index, lo, hi, t, n, sel, idx))
    return fail(c, BLSV_ENOTENOUGH, "share: not enough good public shares to reconstruct secret commitment");
  HIPCHK(c, c->sel.ensure(t * 4));
  HIPCHK(c, c->idx.ensure(t * 4));
  HIPCHK(c, c->lambdas.ensure(t * 32));
  HIPCHK(c, c->scratch.ensure(t * 192 * 4));
  HIPCHK(c, c->out.ensure(96));
  HIPCHK(c, h2d(c, c->sel.p, sel.data(), t * 4));
  std::vector<uint32_t> lam(t * 8);
  host_lagrange(idx.data(), t, lam.data());
  HIPCHK(c, h2d(c, c->lambdas.p, lam.data(), t * 32));
  blsk::launch_lat_recover(c->S.as<uint32_t>(), cls.size(), c->s_inf.as<uint8_t>(), c->sel.as<uint32_t>(),
                           c->lambdas.as<uint32_t>(), (uint32_t)t, c->scratch.as<uint32_t>(), c->out.as<uint8_t>(),
                           c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, download_sync(c, {{out_sig96, c->out.p, 96}}));
  return BLSV_OK;
}

// Speculative recovery. A round's partials are all verified before recover_from picks its shares,
// and the recovered signature is verified after: three latency launches in a row. The shares the
// selection would pick if every partial verified are known before any verification, so they are
// decoded (no subgroup check: validity is the partials' verdict), interpolated and compressed on the
// side stream WHILE the partials verify on the main stream. The result is kept when the verdicts
// leave the selection unchanged -- the same shares, hence the same bytes as recover_from -- and
// recomputed by recover_from otherwise (a selected share failed). Only for rounds on the latency
// path, whose partial verification leaves the side stream idle.
struct SpecRecover {
  bool launched = false;
  bool verified = false;      // VerifyRecovered of the speculative signature queued behind it too
  std::vector<uint32_t> sel;  // round positions of the shares used
};

static int spec_recover_launch(blsv_ctx* c, int slot, const uint8_t* partials, size_t partial_len,
                               const std::vector<uint32_t>& index, size_t lo, size_t hi, size_t t, size_t n,
                               SpecRecover& sr, const uint8_t* vmsg = nullptr, size_t vmsg_len = 0) {
  sr.launched = false;
  sr.verified = false;
  std::vector<uint8_t> all_ok(index.size(), BLSV_REJ_OK);
  std::vector<uint32_t> idx;
  if (!select_shares(all_ok, index, lo, hi, t, n, sr.sel, idx)) return BLSV_OK;  // recover_from will say so
  auto& sp = c->spec[slot];
  const size_t tt = sr.sel.size();
  // host staging: sigmas | indices | selection | 96-byte result | verify class | message, offsets,
  // length | Lagrange coefficients
  const size_t v_off = tt * 96 + tt * 8 + 96, m_off = v_off + 64;
  const bool verify = vmsg != nullptr && vmsg_len <= kIoCap / 4;
  const size_t lam_off = (m_off + (verify ? vmsg_len + 64 : 0) + 7) & ~size_t(7);
  const size_t host_need = lam_off + tt * 32 + 64;
  if (sp.host.sz < host_need) {  // no copy may be pending on it
    HIPCHK(c, hipStreamSynchronize(c->side));
    HIPCHK(c, hipStreamSynchronize(c->side2));
  }
  HIPCHK(c, sp.host.ensure(host_need));
  uint8_t* h_sig = sp.host.as<uint8_t>();
  uint32_t* h_idx = reinterpret_cast<uint32_t*>(h_sig + tt * 96);
  uint32_t* h_sel = h_idx + tt;
  uint32_t* h_lam = reinterpret_cast<uint32_t*>(h_sig + lam_off);
  for (size_t j = 0; j < tt; j++) {
    std::memcpy(h_sig + j * 96, partials + (size_t)sr.sel[j] * partial_len + 2, 96);
    h_idx[j] = idx[j];
    h_sel[j] = (uint32_t)j;
  }
  HIPCHK(c, sp.sig.ensure(tt * 96));
  HIPCHK(c, sp.S.ensure(tt * blsk::S_WORDS * 4));
  HIPCHK(c, sp.s_inf.ensure(tt));
  HIPCHK(c, sp.cls.ensure(tt));
  HIPCHK(c, sp.sel.ensure(tt * 4));
  HIPCHK(c, sp.lam.ensure(tt * 32));
  HIPCHK(c, sp.scratch.ensure(tt * 192 * 4));
  HIPCHK(c, sp.out.ensure(96));
  if (verify) {
    // VerifyRecovered's message and key do not depend on the recovery: its hash-to-G2 and the key
    // pair's Miller loop start now, on the second side stream, beside the partial verification and
    // the recovery (wvteam.h team_hash_key)
    uint8_t* h_msg = h_sig + m_off;
    std::memcpy(h_msg, vmsg, vmsg_len);
    uint64_t* h_off = reinterpret_cast<uint64_t*>(h_msg + ((vmsg_len + 7) & ~size_t(7)));
    h_off[0] = 0;
    h_off[1] = vmsg_len;
    uint32_t* h_len = reinterpret_cast<uint32_t*>(h_off + 2);
    h_len[0] = (uint32_t)vmsg_len;
    HIPCHK(c, sp.vmsg.ensure(vmsg_len + 1));
    HIPCHK(c, sp.voff.ensure(16));
    HIPCHK(c, sp.vlen.ensure(4));
    HIPCHK(c, sp.vcls.ensure(64));
    HIPCHK(c, sp.hout.ensure(blsk::kLatHoutWords * 4));
    HIPCHK(c, sp.saff.ensure(blsk::kLatSaffWords * 4));
    if (vmsg_len) HIPCHK(c, hipMemcpyAsync(sp.vmsg.p, h_msg, vmsg_len, hipMemcpyHostToDevice, c->side2));
    HIPCHK(c, hipMemcpyAsync(sp.voff.p, h_off, 16, hipMemcpyHostToDevice, c->side2));
    HIPCHK(c, hipMemcpyAsync(sp.vlen.p, h_len, 4, hipMemcpyHostToDevice, c->side2));
    const PkSel pk = group_pk(c);
    blsk::launch_lat_hash_key(sp.vmsg.as<uint8_t>(), sp.voff.as<uint64_t>(), sp.vlen.as<uint32_t>(), pk.tab, pk.inf,
                              sp.hout.as<uint32_t>(), c->side2);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(c->hash_ev[slot], c->side2));
  }
  // the shares' decoding first, then the Lagrange coefficients on the host (host_lagrange, ~30 us)
  // while it runs; the interpolation follows on the same stream
  hipStream_t st = c->side;
  HIPCHK(c, hipMemcpyAsync(sp.sig.p, h_sig, tt * 96, hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(sp.sel.p, h_sel, tt * 4, hipMemcpyHostToDevice, st));
  blsk::launch_lat_decode(sp.sig.as<uint8_t>(), 96, 0, tt, sp.S.as<uint32_t>(), sp.s_inf.as<uint8_t>(),
                          sp.cls.as<uint8_t>(), st);
  host_lagrange(h_idx, tt, h_lam);
  HIPCHK(c, hipMemcpyAsync(sp.lam.p, h_lam, tt * 32, hipMemcpyHostToDevice, st));
  blsk::launch_lat_recover(sp.S.as<uint32_t>(), tt, sp.s_inf.as<uint8_t>(), sp.sel.as<uint32_t>(),
                           sp.lam.as<uint32_t>(), (uint32_t)tt, sp.scratch.as<uint32_t>(), sp.out.as<uint8_t>(), st,
                           verify ? sp.saff.as<uint32_t>() : nullptr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(h_sig + tt * 96 + tt * 8, sp.out.p, 96, hipMemcpyDeviceToHost, st));
  if (verify) {
    // VerifyRecovered(group key, msg, speculative signature) right behind the recovery: the signature
    // pair of the sum's affine point, the product with the key pair's Miller value computed above and
    // the final exponentiation (wvteam.h verify_team_pre: the class verify_messages would give the
    // compressed bytes; kept on a hit)
    HIPCHK(c, hipStreamWaitEvent(st, c->hash_ev[slot], 0));
    blsk::launch_lat_verify_pre(sp.hout.as<uint32_t>(), sp.saff.as<uint32_t>(), sp.vcls.as<uint8_t>(), st);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipMemcpyAsync(h_sig + v_off, sp.vcls.p, 1, hipMemcpyDeviceToHost, st));
    sr.verified = true;
  }
  sr.launched = true;
  return BLSV_OK;
}

// after the partials' verdicts (cls): the speculative result if its selection stands, else
// recover_from; the side stream is drained either way
static int spec_recover_finish(blsv_ctx* c, int slot, const SpecRecover& sr, const std::vector<uint8_t>& cls,
                               const std::vector<uint32_t>& index, size_t lo, size_t hi, size_t t, size_t n,
                               uint8_t* out_sig96, int* vcls = nullptr) {
  if (vcls) *vcls = -1;  // no speculative VerifyRecovered verdict
  if (sr.launched) {
    HIPCHK(c, hipStreamSynchronize(c->side));
    std::vector<uint32_t> sel, idx;
    if (select_shares(cls, index, lo, hi, t, n, sel, idx) && sel == sr.sel) {
      const size_t tt = sr.sel.size();
      const uint8_t* h = c->spec[slot].host.as<uint8_t>();
      std::memcpy(out_sig96, h + tt * 96 + tt * 8, 96);
      if (vcls && sr.verified) *vcls = h[tt * 96 + tt * 8 + 96];
      c->spec_hits++;
      return BLSV_OK;
    }
    c->spec_misses++;
  }
  return recover_from(c, cls, index, lo, hi, t, n, out_sig96);
}

// Drains both side streams when a call that launched speculative work returns, on every path: an
// early error return must not leave async copies into the slots' pinned staging in flight (the next
// call's spec_recover_launch writes that staging without a synchronisation when it is large enough).
// On the normal path spec_recover_finish has drained `side` already and this costs two idle syncs.
struct SideDrain {
  blsv_ctx* c;
  bool armed = false;
  ~SideDrain() {
    if (!armed) return;
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamSynchronize(c->side2);
  }
};

// partial_len == 98 and the round small enough for the latency path (partials_stage's choice)
static bool spec_applies(const blsv_ctx* c, size_t k, size_t partial_len) {
  return partial_len == 98 && c->has_group && k > 0 && k <= std::min(c->lat_max, c->chunk);
}

static void share_indices(const uint8_t* partials, size_t partial_len, size_t k, std::vector<uint32_t>& index) {
  index.assign(k, 0);
  for (size_t i = 0; i < k; i++) index[i] = ((uint32_t)partials[i * partial_len] << 8) | partials[i * partial_len + 1];
}

int blsv_aggregate(blsv_ctx* c, const uint8_t* msg, size_t msg_len, const uint8_t* partials, size_t partial_len,
                   size_t k, size_t t, size_t n, uint8_t* ok, uint8_t* reject_class, uint8_t* out_sig96,
                   uint8_t* group_ok) {
  if (!c) return BLSV_EINVAL;
  if (!out_sig96 || !ok || !group_ok || t == 0 || (k && !partials) || (msg_len && !msg))
    return fail(c, BLSV_EINVAL, "aggregate: bad arguments");
  (void)hipSetDevice(c->device);
  std::vector<uint8_t> cls;
  std::vector<uint32_t> index;
  SpecRecover sr;
  SideDrain drain{c};
  if (spec_applies(c, k, partial_len)) {
    share_indices(partials, partial_len, k, index);
    drain.armed = true;
    int rc0 = spec_recover_launch(c, 0, partials, partial_len, index, 0, k, t, n, sr, msg, msg_len);
    if (rc0) return rc0;
  }
  int rc = partials_stage(c, msg, msg_len, partials, partial_len, k, cls, index);
  if (rc) return rc;
  for (size_t i = 0; i < k; i++) {
    ok[i] = cls[i] == BLSV_REJ_OK;
    if (reject_class) reject_class[i] = cls[i];
  }
  *group_ok = 0;
  int vcls = -1;
  rc = spec_recover_finish(c, 0, sr, cls, index, 0, k, t, n, out_sig96, &vcls);
  if (rc) return rc;
  if (vcls >= 0) {  // the speculative VerifyRecovered of this very signature
    *group_ok = vcls == BLSV_REJ_OK;
    return BLSV_OK;
  }
  // VerifyRecovered(group key, msg, sig) (chain/beacon/chain.go:141)
  const uint32_t len = (uint32_t)msg_len;
  uint8_t bm = 0, cls1 = 0;
  uint64_t fb = 0;
  rc = blsv_verify_messages(c, nullptr, msg, &len, 1, out_sig96, &bm, &fb, &cls1);
  if (rc) return rc;
  *group_ok = bm & 1;
  return BLSV_OK;
}

int blsv_aggregate_round(blsv_ctx* c, const uint8_t* msg1, size_t msg1_len, const uint8_t* partials1, size_t k1,
                         const uint8_t* msg2, size_t msg2_len, const uint8_t* partials2, size_t k2,
                         size_t partial_len, size_t t, size_t n, uint8_t* ok1, uint8_t* ok2, uint8_t* sig1_96,
                         uint8_t* sig2_96, int32_t* status, uint8_t* v2_valid) {
  if (!c) return BLSV_EINVAL;
  if (!sig1_96 || !sig2_96 || !status || !v2_valid || t == 0 || (k1 && (!partials1 || !ok1)) ||
      (k2 && (!partials2 || !ok2 || !msg2)) || (msg1_len && !msg1))
    return fail(c, BLSV_EINVAL, "aggregate_round: bad arguments");
  (void)hipSetDevice(c->device);
  *status = BLSV_AGG_V1_RECOVER_FAIL;
  *v2_valid = 0;
  const size_t k = k1 + k2;
  // pass 1: every V1 and V2 partial in ONE verification pass (per-item message)
  std::vector<uint8_t> msgs, parts;
  std::vector<uint32_t> lens(k);
  msgs.reserve(k1 * msg1_len + k2 * msg2_len);
  parts.reserve(k * partial_len);
  for (size_t i = 0; i < k1; i++) {
    msgs.insert(msgs.end(), msg1, msg1 + msg1_len);
    lens[i] = (uint32_t)msg1_len;
  }
  for (size_t i = 0; i < k2; i++) {
    msgs.insert(msgs.end(), msg2, msg2 + msg2_len);
    lens[k1 + i] = (uint32_t)msg2_len;
  }
  if (k1) parts.insert(parts.end(), partials1, partials1 + k1 * partial_len);
  if (k2) parts.insert(parts.end(), partials2, partials2 + k2 * partial_len);
  std::vector<uint8_t> cls;
  std::vector<uint32_t> index;
  const bool try_v2 = k2 >= t;
  SpecRecover sr1, sr2;  // both recoveries speculated on the side stream (see spec_recover_launch)
  SideDrain drain{c};
  if (spec_applies(c, k, partial_len)) {
    share_indices(parts.data(), partial_len, k, index);
    drain.armed = true;
    int rc0 = spec_recover_launch(c, 0, parts.data(), partial_len, index, 0, k1, t, n, sr1, msg1 ? msg1 : parts.data(),
                                  msg1_len);
    if (!rc0 && try_v2)
      rc0 = spec_recover_launch(c, 1, parts.data(), partial_len, index, k1, k, t, n, sr2, msg2, msg2_len);
    if (rc0) return rc0;
  }
  int rc = partials_stage(c, msgs.data(), 0, parts.data(), partial_len, k, cls, index, lens.data());
  if (rc) return rc;
  for (size_t i = 0; i < k1; i++) ok1[i] = cls[i] == BLSV_REJ_OK;
  for (size_t i = 0; i < k2; i++) ok2[i] = cls[k1 + i] == BLSV_REJ_OK;
  // Recover V1 (chain.go:136) and, with LenV2 >= thr, V2 (chain.go:153-155) from the staged shares
  int vc1 = -1, vc2 = -1;
  rc = spec_recover_finish(c, 0, sr1, cls, index, 0, k1, t, n, sig1_96, &vc1);
  if (rc == BLSV_ENOTENOUGH) return BLSV_OK;  // "invalid_recovery": no beacon this time (drain syncs sr2)
  if (rc) return rc;
  bool v2_recovered = false;
  if (try_v2) {
    rc = spec_recover_finish(c, 1, sr2, cls, index, k1, k, t, n, sig2_96, &vc2);
    if (rc && rc != BLSV_ENOTENOUGH) return rc;
    v2_recovered = rc == BLSV_OK;
  }
  // pass 2: VerifyRecovered(pub.Commit(), msg, sig) for both group signatures in one pass
  const uint32_t vlens[2] = {(uint32_t)msg1_len, (uint32_t)msg2_len};
  std::vector<uint8_t> vmsg(msg1, msg1 + msg1_len), vsig(sig1_96, sig1_96 + 96);
  if (v2_recovered) {
    vmsg.insert(vmsg.end(), msg2, msg2 + msg2_len);
    vsig.insert(vsig.end(), sig2_96, sig2_96 + 96);
  }
  uint8_t bm = 0, vcls[2] = {0, 0};
  uint64_t fb = 0;
  if (vc1 >= 0 && (!v2_recovered || vc2 >= 0)) {  // both verdicts already computed speculatively
    bm = (uint8_t)((vc1 == BLSV_REJ_OK) | ((v2_recovered && vc2 == BLSV_REJ_OK) << 1));
  } else {
    rc = blsv_verify_messages(c, nullptr, vmsg.data(), vlens, v2_recovered ? 2 : 1, vsig.data(), &bm, &fb, vcls);
    if (rc) return rc;
  }
  if (!(bm & 1)) {
    *status = BLSV_AGG_V1_INVALID;  // chain.go:141-144 "invalid_sig": no beacon
    return BLSV_OK;
  }
  if (try_v2 && !v2_recovered) {
    *status = BLSV_AGG_V2_RECOVER_FAIL;  // chain.go:155-160: never accept a beacon with an invalid v2
    return BLSV_OK;
  }
  *v2_valid = v2_recovered ? (uint8_t)((bm >> 1) & 1) : 0;  // chain.go:162-164: a failure only logs
  *status = v2_recovered ? BLSV_AGG_OK_V2 : BLSV_AGG_OK;
  return BLSV_OK;
}

int blsv_sign(blsv_ctx* c, const uint8_t* sk32, int32_t index, const uint8_t* msgs, const uint32_t* msg_lens, size_t n,
              uint8_t* out) {
  if (!c) return BLSV_EINVAL;
  if (!sk32 || (n && (!msg_lens || !out)) || index > 65535) return fail(c, BLSV_EINVAL, "sign: bad arguments");
  if (n > kMaxChunk) return fail(c, BLSV_EINVAL, "sign: batch larger than %zu", kMaxChunk);
  (void)hipSetDevice(c->device);
  if (!n) return BLSV_OK;
  uint32_t sk[8];
  scalar_mod_r(sk32, sk);
  int rc = ensure_workspace(c, n);
  if (rc) return rc;
  rc = upload_messages(c, msgs, msg_lens, n);
  if (rc) return rc;
  const size_t stride = index >= 0 ? 98 : 96;
  HIPCHK(c, c->sk.ensure(32));
  HIPCHK(c, c->out.ensure(n * stride));
  HIPCHK(c, hipMemcpyAsync(c->sk.p, sk, 32, hipMemcpyHostToDevice, c->stream));
  for (size_t base = 0; base < n; base += c->cap) {  // H staging holds one chunk
    const size_t cnt = std::min(c->cap, n - base);
    blsk::launch_hash_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>() + base,
                               c->in_len.as<uint32_t>() + base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(),
                               c->HQ.as<uint32_t>(), c->stream);
    blsk::launch_sign(c->sk.as<uint32_t>(), index, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), cnt,
                      c->out.as<uint8_t>() + base * stride, stride, c->stream);
  }
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, c->out.p, n * stride, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int blsv_verify_chained_dev(blsv_ctx* c, uint64_t first_round, uint64_t seg_len, uint64_t seg_phase,
                            const uint8_t* d_seeds96, size_t seed0_len, const uint8_t* d_sigs96, size_t n,
                            uint64_t* d_bitmap, uint64_t* d_first_bad, uint8_t* d_reject_class, void* stream) {
  if (!c) return BLSV_EINVAL;
  if (!c->has_group) return fail(c, BLSV_ENOGROUP, "verify_chained_dev: no group key set");
  if (n && (!d_seeds96 || !d_sigs96 || !d_bitmap || !d_first_bad || (seed0_len != 32 && seed0_len != 96)))
    return fail(c, BLSV_EINVAL, "verify_chained_dev: bad arguments");
  if (seg_phase && (!seg_len || seg_phase >= seg_len))
    return fail(c, BLSV_EINVAL, "verify_chained_dev: seg_phase must be < seg_len");
  (void)hipSetDevice(c->device);
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  HIPCHK(c, hipMemsetAsync(d_first_bad, 0xff, 8, st));
  int rc = ensure_workspace(c, n);
  if (rc) return rc;
  blsk::ChainedSrc src{d_sigs96, d_seeds96, first_round, seg_len ? seg_len : std::max<uint64_t>(n, 1),
                       (uint32_t)seed0_len, seg_phase};
  if (use_lat(c, n)) {
    const PkSel pk = group_pk(c);
    return run_lat(
        c, n, [&](uint8_t* cls) { blsk::launch_lat_chained(src, 0, n, pk.tab, pk.inf, cls, st); }, d_bitmap,
        (unsigned long long*)d_first_bad, d_reject_class, st, first_round);
  }
  for (size_t base = 0; base < n; base += c->cap) {
    const size_t cnt = std::min(c->cap, n - base);
    rc = run_head(c, d_sigs96, 96, 0, base, cnt, st, [&]() {
      blsk::launch_hash_chained(src, base, cnt, c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->HQ.as<uint32_t>(), st);
    });
    if (rc) return rc;
    rc = run_tail(c, d_sigs96, 96, 0, base, cnt, group_pk(c), d_bitmap, (unsigned long long*)d_first_bad,
                  d_reject_class, st, first_round);  // d_first_bad holds a ROUND (include/blsverify.h)
    if (rc) return rc;
  }
  return BLSV_OK;
}

int blsv_generate_chained_dev(blsv_ctx* c, const uint8_t* sk32, uint64_t first_round, uint64_t seg_len,
                              const uint8_t* d_seeds96, size_t seed0_len, uint8_t* d_sigs96, size_t n, void* stream) {
  if (!c) return BLSV_EINVAL;
  if (!sk32 || (n && (!d_seeds96 || !d_sigs96)) || (seed0_len != 32 && seed0_len != 96))
    return fail(c, BLSV_EINVAL, "generate_chained_dev: bad arguments");
  (void)hipSetDevice(c->device);
  hipStream_t st = stream ? (hipStream_t)stream : c->stream;
  uint32_t sk[8];
  scalar_mod_r(sk32, sk);
  HIPCHK(c, c->sk.ensure(32));
  HIPCHK(c, hipMemcpyAsync(c->sk.p, sk, 32, hipMemcpyHostToDevice, st));
  blsk::ChainedSrc src{d_sigs96, d_seeds96, first_round, seg_len ? seg_len : std::max<uint64_t>(n, 1),
                       (uint32_t)seed0_len};
  blsk::launch_gen_chained(c->sk.as<uint32_t>(), src, n, d_sigs96, st);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(st));  // sk staging buffer is reused by later calls
  return BLSV_OK;
}

// ------------------------------------------------------------------ stage profiling
int blsv_profile_enable(blsv_ctx* c, int on) {
  if (!c) return BLSV_EINVAL;
  c->prof = on != 0;
  return BLSV_OK;
}

int blsv_profile_read(blsv_ctx* c, double* ms, uint64_t* launches, uint64_t* items, int nstages) {
  if (!c || nstages < 0) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  for (int s = 0; s < nstages; s++) {
    if (ms) ms[s] = 0;
    if (launches) launches[s] = 0;
    if (items) items[s] = 0;
  }
  for (auto& r : c->recs) {
    HIPCHK(c, hipEventSynchronize(r.b));
    float t = 0;
    HIPCHK(c, hipEventElapsedTime(&t, r.a, r.b));
    if (r.stage < nstages) {
      if (ms) ms[r.stage] += t;
      if (launches) launches[r.stage] += 1;
      if (items) items[r.stage] += r.items;
    }
    c->event_pool.push_back(r.a);
    c->event_pool.push_back(r.b);
  }
  c->recs.clear();
  return ST_N;
}

int blsv_test_spec_stats(blsv_ctx* c, uint64_t* hits, uint64_t* misses) {
  if (!c || !hits || !misses) return BLSV_EINVAL;
  *hits = c->spec_hits;
  *misses = c->spec_misses;
  return BLSV_OK;
}

int blsv_test_generic_chains(blsv_ctx* c, int on) {
  if (!c) return BLSV_EINVAL;
  blsk::g_generic_chains_all = on != 0;
  return BLSV_OK;
}

int blsv_lat_trace_enable(blsv_ctx* c, int on) {
  if (!c) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  if (blsk::lat_trace_enable(on, c->stream) != 0) return fail(c, BLSV_EHIP, "lat_trace_enable: symbol copy failed");
  return BLSV_OK;
}

int blsv_lat_trace(blsv_ctx* c, uint64_t* ticks, int n, double* ticks_per_us, int clear) {
  if (!c || n < 0 || (n && !ticks)) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  // the marks are device-global: wait for every latency launch on the device (any stream, any context)
  HIPCHK(c, hipDeviceSynchronize());
  int got = 0;
  if (n) {
    got = blsk::lat_trace_read(ticks, n, c->stream);
    if (got < 0) return fail(c, BLSV_EHIP, "lat_trace: symbol copy failed");
  }
  if (ticks_per_us) {
    int khz = 0;
    HIPCHK(c, hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
    *ticks_per_us = khz / 1000.0;
  }
  if (clear && blsk::lat_trace_clear(c->stream) != 0) return fail(c, BLSV_EHIP, "lat_trace: clear failed");
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return got;
}

// latency-path cutover (include/blsverify.h latency contract)
size_t blsv_set_lat_max(blsv_ctx* c, size_t lat_max) {
  if (!c) return 0;
  const size_t prev = c->lat_max;
  c->lat_max = std::min(lat_max, c->chunk);  // see lat_max_env: larger batches take the pipeline
  return prev;
}

// per-context pass size (include/blsverify.h memory contract)
size_t blsv_set_chunk(blsv_ctx* c, size_t items) {
  if (!c) return 0;
  const size_t prev = c->chunk;
  size_t v = items ? std::min(std::max(items, kMinChunk), kMaxChunk) : chunk_env();
  v = (v + 63) & ~size_t(63);
  (void)hipSetDevice(c->device);
  if (v < c->cap) {  // give the HBM back now: the next call allocates at the new size
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->side);
    release_workspace(c);
  }
  c->chunk = v;
  c->lat_max = std::min(c->lat_max, v);
  return prev;
}

size_t blsv_workspace_bytes(const blsv_ctx* c) {
  if (!c) return 0;
  size_t b = 0;
  for (const DBuf* d : {&c->H, &c->HQ, &c->S, &c->F, &c->FW, &c->LN, &c->h_inf, &c->s_inf, &c->cls}) b += d->sz;
  return b;
}

// ------------------------------------------------------------------ testing hooks

int blsv_test_fp_mul(blsv_ctx* c, const uint32_t* a, const uint32_t* b, size_t n, uint32_t* out) {
  if (!c || (n && (!a || !b || !out))) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  DBuf da, db, dout;
  HIPCHK(c, da.ensure(n * 48));
  HIPCHK(c, db.ensure(n * 48));
  HIPCHK(c, dout.ensure(n * 48));
  HIPCHK(c, hipMemcpyAsync(da.p, a, n * 48, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(db.p, b, n * 48, hipMemcpyHostToDevice, c->stream));
  blsk::launch_test_fp_mul(da.as<uint32_t>(), db.as<uint32_t>(), n, dout.as<uint32_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, dout.p, n * 48, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int blsv_test_pairing(blsv_ctx* c, const uint32_t* p, const uint32_t* q, size_t n, uint32_t* out_f) {
  if (!c || (n && (!p || !q || !out_f))) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  DBuf dp, dq, dout;
  HIPCHK(c, dp.ensure(n * 96));
  HIPCHK(c, dq.ensure(n * 192));
  HIPCHK(c, dout.ensure(n * 576));
  HIPCHK(c, hipMemcpyAsync(dp.p, p, n * 96, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemcpyAsync(dq.p, q, n * 192, hipMemcpyHostToDevice, c->stream));
  blsk::launch_test_pairing(dp.as<uint32_t>(), dq.as<uint32_t>(), n, dout.as<uint32_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out_f, dout.p, n * 576, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int blsv_test_final_exp(blsv_ctx* c, const uint32_t* f, size_t n, uint32_t* out_pipeline, uint32_t* out_ref) {
  if (!c || (n && (!f || !out_pipeline || !out_ref))) return BLSV_EINVAL;
  if (n > kMaxChunk) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  int rc = ensure_workspace(c, n);
  if (rc) return rc;
  if (n > c->cap) return fail(c, BLSV_EINVAL, "test_final_exp: more than the context chunk");
  if (!n) return BLSV_OK;
  DBuf din, dout, dref;
  HIPCHK(c, din.ensure(n * 576));
  HIPCHK(c, dout.ensure(n * 576));
  HIPCHK(c, dref.ensure(n * 576));
  HIPCHK(c, hipMemcpyAsync(din.p, f, n * 576, hipMemcpyHostToDevice, c->stream));
  HIPCHK(c, hipMemsetAsync(c->cls.p, 0, n, c->stream));
  blsk::launch_test_pack_fp12(din.as<uint32_t>(), n, c->F.as<uint32_t>(), c->stream);
  blsk::launch_test_final_exp_ref(c->F.as<uint32_t>(), n, dref.as<uint32_t>(), c->stream);
  // the production stage (clobbers F), its final value captured into dout
  blsk::launch_final_exp(c->F.as<uint32_t>(), c->FW.as<uint32_t>(), n, c->cls.as<uint8_t>(), c->stream,
                         c->LN.as<uint32_t>(), dout.as<uint32_t>());
  blsk::launch_test_unpack_fp12(dout.as<uint32_t>(), n, din.as<uint32_t>(), c->stream);
  HIPCHK(c, hipMemcpyAsync(out_pipeline, din.p, n * 576, hipMemcpyDeviceToHost, c->stream));
  blsk::launch_test_unpack_fp12(dref.as<uint32_t>(), n, dout.as<uint32_t>(), c->stream);
  HIPCHK(c, hipMemcpyAsync(out_ref, dout.p, n * 576, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

int blsv_test_hash_to_g2(blsv_ctx* c, const uint8_t* msgs, const uint32_t* msg_lens, size_t n, uint32_t* out,
                         uint8_t* inf) {
  if (!c || (n && (!msg_lens || !out || !inf))) return BLSV_EINVAL;
  if (n > kMaxChunk) return BLSV_EINVAL;
  (void)hipSetDevice(c->device);
  int rc = ensure_workspace(c, n);
  if (rc) return rc;
  if (n > c->cap) return fail(c, BLSV_EINVAL, "test_hash_to_g2: more than the context chunk");
  rc = upload_messages(c, msgs, msg_lens, n);
  if (rc) return rc;
  DBuf dout;
  HIPCHK(c, dout.ensure(n * 192));
  blsk::launch_hash_messages(c->in_msgs.as<uint8_t>(), c->in_off.as<uint64_t>(), c->in_len.as<uint32_t>(), n,
                             c->H.as<uint32_t>(), c->h_inf.as<uint8_t>(), c->HQ.as<uint32_t>(), c->stream);
  blsk::launch_test_unpack_g2(c->H.as<uint32_t>(), n, dout.as<uint32_t>(), c->stream);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipMemcpyAsync(out, dout.p, n * 192, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipMemcpyAsync(inf, c->h_inf.p, n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return BLSV_OK;
}

}  // extern "C"

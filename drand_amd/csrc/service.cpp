// Thread-safe service of the C ABI (include/blsverify.h blsv_service_*): concurrent single-item
// callers -- one goroutine per partial packet (core/drand_public.go:39 -> chain/beacon/node.go:112,125),
// per gossip message (lp2p/client/validator.go:64), per client.Get (client/verify.go:185-207) -- block
// in their own call while the dispatcher thread (coalesce.h) verifies every item that arrived close
// together in ONE launch (svc_verify_mixed) and scatters the classes back.
//
// Public keys of a batch come from one device table, the "key arena": every group seen keeps its
// PubPoly.Eval(i) table for i < min(n, kPkTable) (key/keys.go:239-241, built once on device), every
// explicit VerifyRecovered key its decoded point; each item carries its entry index. Share indices
// beyond a group's table are evaluated per batch into the arena's tail. When the arena is full it is
// rebuilt for the batch at hand.
#include <memory>
#include <mutex>

#include "coalesce.h"
#include "engine_ctx.h"

namespace {

constexpr size_t kArenaEntries = 16384;    // G1 entries (96 bytes each): 1.5 MB of HBM
constexpr size_t kServiceChunk = 65536;    // the service context's pass size (~2.7 GB of staging)
constexpr size_t kServiceMaxBatch = 65536;  // items per launch (the latency path up to lat_max of them)

uint32_t env_us(const char* name, uint32_t dflt) {
  const char* e = getenv(name);
  if (!e) return dflt;
  char* end = nullptr;
  const unsigned long v = strtoul(e, &end, 10);
  if (end == e || *end != '\0' || v > 1000000ul) {
    fprintf(stderr, "blsverify: ignoring %s=\"%s\"; keeping %u us\n", name, e, dflt);
    return dflt;
  }
  return (uint32_t)v;
}

struct SvcItem {
  // inputs (the caller's buffers, valid while it blocks in submit)
  bool partial = false;
  const uint8_t* msg = nullptr;
  size_t msg_len = 0;
  const uint8_t* sig96 = nullptr;
  uint32_t index = 0;                    // share index (partials)
  const uint8_t* commits = nullptr;      // partials: t x 48 bytes
  size_t t = 0, n = 0;
  const uint8_t* pk48 = nullptr;         // VerifyRecovered
  // outputs
  uint8_t cls = BLSV_REJ_OK;
  int rc = BLSV_OK;
  // dispatcher scratch
  size_t entry = 0;
};

struct GroupEnt {
  std::vector<uint8_t> bytes;
  size_t t = 0, n = 0, off = 0, m = 0;
  DBuf commits, commit_inf;  // decoded commitments (Horner for indices beyond the table)
};

struct KeyEnt {
  uint8_t pk[48];
  size_t off = 0;
};

}  // namespace

struct blsv_service {
  blsv_ctx* c = nullptr;
  DBuf tab, tab_inf;           // the key arena (kArenaEntries G1 entries)
  size_t used = 0;             // entries taken by cached groups and keys
  std::vector<std::unique_ptr<GroupEnt>> groups;
  std::vector<KeyEnt> keys;
  DBuf in48, cls48, idx;       // decode / Horner staging
  size_t arena_cap = kArenaEntries;  // entries usable (lowered only by blsv_test_service_limits)
  uint64_t launches = 0;       // svc_verify_mixed calls (sub-batches included)
  std::unique_ptr<Coalescer<SvcItem>> co;

  void reset_arena() {
    groups.clear();
    keys.clear();
    used = 0;
  }

  // decode cnt compressed G1 points into arena entries [off, off + cnt); classes to the host
  int decode_into(const uint8_t* pts48, size_t cnt, uint32_t* d_tab, uint8_t* d_inf, std::vector<uint8_t>& cls) {
    HIPCHK(c, in48.ensure(cnt * 48));
    HIPCHK(c, cls48.ensure(cnt));
    HIPCHK(c, hipMemcpyAsync(in48.p, pts48, cnt * 48, hipMemcpyHostToDevice, c->stream));
    blsk::launch_decompress_g1(in48.as<uint8_t>(), cnt, d_tab, d_inf, cls48.as<uint8_t>(), c->stream);
    HIPCHK(c, hipGetLastError());
    cls.assign(cnt, 0);
    HIPCHK(c, hipMemcpyAsync(cls.data(), cls48.p, cnt, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    return BLSV_OK;
  }

  // PubPoly.Eval(idx[i]) of group g into arena entries [off, off + cnt)
  int eval_into(GroupEnt& g, const std::vector<uint32_t>& ix, size_t off) {
    if (ix.empty()) return BLSV_OK;
    HIPCHK(c, idx.ensure(ix.size() * 4));
    HIPCHK(c, hipMemcpyAsync(idx.p, ix.data(), ix.size() * 4, hipMemcpyHostToDevice, c->stream));
    blsk::launch_pubpoly_eval(g.commits.as<uint32_t>(), g.commit_inf.as<uint8_t>(), (uint32_t)g.t, idx.as<uint32_t>(),
                              ix.size(), tab.as<uint32_t>() + off * blsk::G1_WORDS, tab_inf.as<uint8_t>() + off,
                              c->stream);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipStreamSynchronize(c->stream));  // ix must outlive the copy
    return BLSV_OK;
  }

  GroupEnt* find_group(const SvcItem& it) {
    for (auto& g : groups)
      if (g->t == it.t && g->n == it.n && memcmp(g->bytes.data(), it.commits, it.t * 48) == 0) return g.get();
    return nullptr;
  }
  KeyEnt* find_key(const uint8_t* pk48) {
    for (auto& k : keys)
      if (memcmp(k.pk, pk48, 48) == 0) return &k;
    return nullptr;
  }

  // installs a group: commitments decoded, PK_i table built; nullptr + *rc on a bad commitment.
  // `reserve` entries above `used` are already promised to this sub-batch's out-of-table indices.
  GroupEnt* add_group(const SvcItem& it, size_t reserve, int* rc) {
    const size_t m = std::min(it.n, kPkTable);
    *rc = BLSV_OK;
    if (used + m + reserve > arena_cap) return nullptr;  // the sub-batch ends here
    auto g = std::make_unique<GroupEnt>();
    g->bytes.assign(it.commits, it.commits + it.t * 48);
    g->t = it.t;
    g->n = it.n;
    g->m = m;
    g->off = used;
    if (g->commits.ensure(it.t * blsk::G1_WORDS * 4) != hipSuccess || g->commit_inf.ensure(it.t) != hipSuccess) {
      *rc = fail(c, BLSV_EHIP, "service: commitment staging");
      return nullptr;
    }
    std::vector<uint8_t> cls;
    if ((*rc = decode_into(it.commits, it.t, g->commits.as<uint32_t>(), g->commit_inf.as<uint8_t>(), cls))) return nullptr;
    for (uint8_t k : cls)
      if (k) {
        *rc = BLSV_EINVAL;  // set_group's rule: every commitment must decode
        return nullptr;
      }
    std::vector<uint32_t> ident(m);
    for (size_t i = 0; i < m; i++) ident[i] = (uint32_t)i;
    if ((*rc = eval_into(*g, ident, g->off))) return nullptr;
    used += m;
    groups.push_back(std::move(g));
    return groups.back().get();
  }

  KeyEnt* add_key(const uint8_t* pk48, size_t reserve, int* rc) {
    *rc = BLSV_OK;
    if (used + 1 + reserve > arena_cap) return nullptr;  // the sub-batch ends here
    std::vector<uint8_t> cls;
    if ((*rc = decode_into(pk48, 1, tab.as<uint32_t>() + used * blsk::G1_WORDS, tab_inf.as<uint8_t>() + used, cls)))
      return nullptr;
    if (cls[0]) {
      *rc = BLSV_EINVAL;  // verify_messages' rule for an explicit key that does not decode
      return nullptr;
    }
    KeyEnt k;
    memcpy(k.pk, pk48, 48);
    k.off = used++;
    keys.push_back(k);
    return &keys.back();
  }

  // Resolves the arena entries of b[pos, end) for the largest end whose keys fit the arena and returns
  // end (items whose own key fails get rc != 0 and stay in the range). Out-of-table share indices are
  // evaluated per sub-batch into the arena's tail, above every cached group and key.
  size_t resolve(std::vector<SvcItem*>& b, size_t pos) {
    std::vector<std::pair<GroupEnt*, SvcItem*>> beyond;
    size_t i = pos;
    for (; i < b.size(); i++) {
      SvcItem* it = b[i];
      it->entry = 0;
      if (it->rc) continue;
      int rc = BLSV_OK;
      if (it->partial) {
        GroupEnt* g = find_group(*it);
        if (!g) g = add_group(*it, beyond.size(), &rc);
        if (!g) {
          if (rc) {
            it->rc = rc;
            continue;
          }
          break;
        }
        if (it->index < g->m) {
          it->entry = g->off + it->index;
        } else {  // an index >= n still has a well-defined Eval in kyber
          if (used + beyond.size() + 1 > arena_cap) break;
          beyond.push_back({g, it});
        }
      } else {
        KeyEnt* k = find_key(it->pk48);
        if (!k) k = add_key(it->pk48, beyond.size(), &rc);
        if (!k) {
          if (rc) {
            it->rc = rc;
            continue;
          }
          break;
        }
        it->entry = k->off;
      }
    }
    // per-sub-batch Horner for the out-of-table indices, one launch per group
    std::stable_sort(beyond.begin(), beyond.end(),
                     [](const std::pair<GroupEnt*, SvcItem*>& a, const std::pair<GroupEnt*, SvcItem*>& b) {
                       return a.first < b.first;
                     });
    size_t tail = used;
    for (size_t q = 0; q < beyond.size();) {
      size_t j = q;
      std::vector<uint32_t> ix;
      for (; j < beyond.size() && beyond[j].first == beyond[q].first; j++) {
        ix.push_back(beyond[j].second->index);
        beyond[j].second->entry = tail + (j - q);
      }
      const int rc = eval_into(*beyond[q].first, ix, tail);
      if (rc)
        for (size_t r = q; r < j; r++) beyond[r].second->rc = rc;
      tail += j - q;
      q = j;
    }
    return i;
  }

  // one launch over the live items of b[lo, hi)
  void launch(std::vector<SvcItem*>& b, size_t lo, size_t hi) {
    std::vector<SvcItem*> live;
    for (size_t i = lo; i < hi; i++)
      if (!b[i]->rc) live.push_back(b[i]);
    const size_t n = live.size();
    if (!n) return;
    std::vector<uint64_t> off(n + 1, 0);
    std::vector<uint32_t> lens(n), ix(n);
    std::vector<uint8_t> msgs, sigs(n * 96), cls(n);
    for (size_t i = 0; i < n; i++) {
      off[i + 1] = off[i] + live[i]->msg_len;
      lens[i] = (uint32_t)live[i]->msg_len;
      ix[i] = (uint32_t)live[i]->entry;
      memcpy(&sigs[i * 96], live[i]->sig96, 96);
    }
    msgs.reserve(off[n]);
    for (SvcItem* it : live) msgs.insert(msgs.end(), it->msg, it->msg + it->msg_len);
    const int rc = svc_verify_mixed(c, n, msgs.data(), off.data(), lens.data(), sigs.data(), ix.data(),
                                    tab.as<uint32_t>(), tab_inf.as<uint8_t>(), cls.data());
    for (size_t i = 0; i < n; i++) {
      live[i]->rc = rc;
      live[i]->cls = rc ? (uint8_t)BLSV_REJ_OK : cls[i];
    }
    launches++;
  }

  // A batch whose keys overflow the arena (many groups or keys, or out-of-table share indices: one tail
  // entry each) runs as consecutive sub-batches, the arena rebuilt between them, so no caller fails
  // because of what the others sent.
  void run(std::vector<SvcItem*>& b) {
    (void)hipSetDevice(c->device);
    size_t pos = 0;
    bool fresh = false;  // the arena holds nothing of an earlier sub-batch
    while (pos < b.size()) {
      const size_t end = resolve(b, pos);
      if (end == pos) {  // b[pos]'s keys do not fit beside the cached ones
        if (!fresh) {
          reset_arena();
          fresh = true;
          continue;
        }
        b[pos]->rc = fail(c, BLSV_EINVAL, "service: one item's keys exceed the key arena");
        pos++;
        continue;
      }
      launch(b, pos, end);
      pos = end;
      fresh = false;
      if (pos < b.size()) {
        reset_arena();
        fresh = true;
      }
    }
  }
};

extern "C" {

int blsv_service_create(int device, uint32_t gap_us, uint32_t max_wait_us, blsv_service** out) {
  if (!out) return BLSV_EINVAL;
  *out = nullptr;
  blsv_ctx* c = nullptr;
  int rc = blsv_create(device, &c);
  if (rc) return rc;
  blsv_set_chunk(c, kServiceChunk);
  auto* s = new blsv_service();
  s->c = c;
  if (s->tab.ensure(kArenaEntries * blsk::G1_WORDS * 4) != hipSuccess || s->tab_inf.ensure(kArenaEntries) != hipSuccess) {
    blsv_destroy(c);
    delete s;
    return BLSV_EHIP;
  }
  const uint32_t gap = gap_us ? gap_us : env_us("BLSV_SVC_GAP_US", 100);
  const uint32_t wait = max_wait_us ? max_wait_us : env_us("BLSV_SVC_MAX_WAIT_US", 2000);
  s->co = std::make_unique<Coalescer<SvcItem>>([s](std::vector<SvcItem*>& b) { s->run(b); }, gap, wait, kServiceMaxBatch,
      // run() threw (std::bad_alloc of a large batch's host staging): the call fails, the process lives
      [](SvcItem* it) {
        if (!it->rc) it->rc = BLSV_EHIP;
      });
  *out = s;
  return BLSV_OK;
}

void blsv_service_destroy(blsv_service* s) {
  if (!s) return;
  s->co.reset();  // drains and joins the dispatcher
  s->groups.clear();
  s->tab.release();
  s->tab_inf.release();
  blsv_destroy(s->c);
  delete s;
}

int blsv_service_verify_partial(blsv_service* s, const uint8_t* commits48, size_t t, size_t n, const uint8_t* msg,
                                size_t msg_len, const uint8_t* partial, size_t partial_len, uint8_t* ok,
                                uint8_t* reject_class) {
  if (!s || !commits48 || t == 0 || t > 65536 || !ok || (msg_len && !msg) || (partial_len && !partial))
    return BLSV_EINVAL;
  // tbls IndexOf / SigShare (key/curve.go scheme, kyber tbls): host-side rejects, no launch
  uint8_t cls = BLSV_REJ_OK;
  if (partial_len < 2)
    cls = BLSV_REJ_SHARE_INDEX;
  else if (partial_len != BLSV_PARTIAL_LEN)
    cls = BLSV_REJ_LENGTH;
  if (cls) {
    *ok = 0;
    if (reject_class) *reject_class = cls;
    return BLSV_OK;
  }
  SvcItem it;
  it.partial = true;
  it.msg = msg;
  it.msg_len = msg_len;
  it.sig96 = partial + 2;
  it.index = ((uint32_t)partial[0] << 8) | partial[1];
  it.commits = commits48;
  it.t = t;
  it.n = n;
  s->co->submit(&it);
  if (it.rc) return it.rc;
  *ok = it.cls == BLSV_REJ_OK;
  if (reject_class) *reject_class = it.cls;
  return BLSV_OK;
}

int blsv_service_verify_recovered(blsv_service* s, const uint8_t* pk48, const uint8_t* msg, size_t msg_len,
                                  const uint8_t* sig96, uint8_t* ok, uint8_t* reject_class) {
  if (!s || !pk48 || !sig96 || !ok || (msg_len && !msg)) return BLSV_EINVAL;
  SvcItem it;
  it.msg = msg;
  it.msg_len = msg_len;
  it.sig96 = sig96;
  it.pk48 = pk48;
  s->co->submit(&it);
  if (it.rc) return it.rc;
  *ok = it.cls == BLSV_REJ_OK;
  if (reject_class) *reject_class = it.cls;
  return BLSV_OK;
}

int blsv_test_service_limits(blsv_service* s, size_t chunk, size_t lat_max, size_t arena_entries,
                             uint64_t* sub_launches) {
  if (!s) return BLSV_EINVAL;
  if (sub_launches) *sub_launches = s->launches;
  if (!chunk && !lat_max && !arena_entries) return BLSV_OK;
  // every field is only read by the dispatcher thread inside run(): take it out of service first
  return s->co->with_idle([&] {
    blsv_ctx* c = s->c;
    (void)hipSetDevice(c->device);
    if (chunk) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamSynchronize(c->side);
      release_workspace(c);
      c->chunk = (std::max<size_t>(chunk, 64) + 63) & ~size_t(63);  // below kMinChunk on purpose
    }
    c->lat_max = std::min(lat_max == SIZE_MAX ? c->lat_max : lat_max, c->chunk);
    if (arena_entries) {
      s->arena_cap = std::min(arena_entries, kArenaEntries);
      s->reset_arena();
    }
    return BLSV_OK;
  });
}

int blsv_service_stats(blsv_service* s, uint64_t* launches, uint64_t* items, uint64_t* max_batch) {
  if (!s) return BLSV_EINVAL;
  const auto st = s->co->stats();
  if (launches) *launches = st.launches;
  if (items) *items = st.items;
  if (max_batch) *max_batch = st.max_batch;
  return BLSV_OK;
}

}  // extern "C"

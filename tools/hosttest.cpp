// Host tests of the library's pure host logic, built with sanitizers (tools/Makefile hosttest-asan,
// hosttest-tsan; tests/test_sanitize.py runs them):
//   coalesce  the blsv_service request coalescer (drand_amd/csrc/coalesce.h) with a stand-in run():
//             64 threads x rounds of bursts, every request answered exactly once with its own
//             result, bursts coalesced, stats consistent, destruction drains; and a lone request
//             leaves after the gap; a run() that throws fails only its own batch's calls.
//   boltload  the drand.db loader (drand_amd/csrc/boltload.cpp, include/boltload.h) over the files
//             named on the command line (written by tests/support/boltwriter.py), plus truncated and
//             bit-flipped copies of each: every call must fail cleanly or succeed, never fault.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <new>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../drand_amd/csrc/coalesce.h"
#include "../include/boltload.h"

using blsv_detail::Coalescer;

namespace {

struct Req {
  int in = 0;
  int out = -1;
  int runs = 0;
};

int fails = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: CHECK(%s) failed\n", __FILE__, __LINE__, #c); \
      fails++;                                                     \
    }                                                              \
  } while (0)

int test_coalesce() {
  std::atomic<uint64_t> batches{0}, seen{0};
  std::atomic<size_t> largest{0};
  {
    Coalescer<Req> co(
        [&](std::vector<Req*>& b) {
          batches++;
          seen += b.size();
          size_t cur = largest.load();
          while (b.size() > cur && !largest.compare_exchange_weak(cur, b.size())) {
          }
          std::this_thread::sleep_for(std::chrono::microseconds(300));  // the "launch"
          for (Req* r : b) {
            r->out = r->in * 3 + 1;
            r->runs++;
          }
        },
        150, 2000, 48);
    const int T = 64, R = 20;
    std::vector<std::thread> th;
    std::atomic<int> bad{0};
    std::atomic<int> go{0};
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t] {
        while (!go.load()) std::this_thread::yield();
        for (int r = 0; r < R; r++) {
          Req q;
          q.in = t * 1000 + r;
          co.submit(&q);
          if (q.out != q.in * 3 + 1 || q.runs != 1) bad++;
        }
      });
    go = 1;
    for (auto& x : th) x.join();
    CHECK(bad.load() == 0);
    const auto st = co.stats();
    CHECK(st.items == (uint64_t)T * R);
    CHECK(st.launches == batches.load());
    CHECK(st.max_batch <= 48);
    CHECK(st.launches < (uint64_t)T * R / 4);  // bursts were coalesced
    // a lone request waits for the gap only, not the whole window
    Req q;
    q.in = 7;
    const auto t0 = std::chrono::steady_clock::now();
    co.submit(&q);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    CHECK(q.out == 22);
    CHECK(us < 1900);
  }  // destructor joins
  CHECK(seen.load() == 64 * 20 + 1);
  // run() throwing (a std::bad_alloc of a large batch): every caller of that batch returns, marked
  // failed by the fail hook, and the dispatcher serves the next batch
  {
    std::atomic<int> calls{0};
    Coalescer<Req> co(
        [&](std::vector<Req*>& b) {
          if (calls++ == 0) throw std::bad_alloc();
          for (Req* r : b) r->out = r->in + 1;
        },
        100, 1000, 64, [](Req* r) { r->out = -2; });
    std::vector<std::thread> th;
    std::vector<Req> qs(16);
    for (int t = 0; t < 16; t++) {
      qs[t].in = t;
      th.emplace_back([&, t] { co.submit(&qs[t]); });
    }
    for (auto& x : th) x.join();
    int failed = 0, served = 0;
    for (int t = 0; t < 16; t++) {
      failed += qs[t].out == -2;
      served += qs[t].out == t + 1;
    }
    CHECK(failed >= 1 && failed + served == 16);
    Req q;
    q.in = 41;
    co.submit(&q);
    CHECK(q.out == 42);
    // with_idle runs between batches
    int v = co.with_idle([&] { return 5; });
    CHECK(v == 5);
  }
  printf("{\"coalesce\": {\"batches\": %llu, \"items\": %llu, \"largest\": %zu}}\n",
         (unsigned long long)batches.load(), (unsigned long long)seen.load(), largest.load());
  return 0;
}

std::vector<uint8_t> slurp(const char* path) {
  std::vector<uint8_t> v;
  FILE* f = fopen(path, "rb");
  if (!f) return v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}

void spit(const std::string& path, const std::vector<uint8_t>& v) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f) return;
  fwrite(v.data(), 1, v.size(), f);
  fclose(f);
}

// one open/count/load/close cycle; returns rows loaded or -1
long long load_all(const char* path) {
  dl_db* db = nullptr;
  if (dl_open(path, &db) != 0) {
    if (db) dl_close(db);
    return -1;
  }
  const int64_t n = dl_count(db);
  long long rows = -1;
  if (n >= 0 && n < (1 << 22)) {
    const size_t m = (size_t)n + 1;
    std::vector<uint64_t> rounds(m);
    std::vector<uint8_t> prev(m * 96), sig(m * 96), v2(m * 96), plen(m), slen(m), vlen(m);
    size_t got = 0;
    if (dl_load(db, 0, (size_t)n, rounds.data(), prev.data(), plen.data(), sig.data(), slen.data(), v2.data(),
                vlen.data(), &got) == 0)
      rows = (long long)got;
  }
  dl_close(db);
  return rows;
}

int test_boltload(int argc, char** argv) {
  unsigned long long tried = 0;
  for (int a = 0; a < argc; a++) {
    const long long good = load_all(argv[a]);
    CHECK(good > 0);
    const std::vector<uint8_t> raw = slurp(argv[a]);
    const std::string tmp = std::string(argv[a]) + ".fuzz";
    uint64_t s = 0x9e3779b97f4a7c15ull ^ raw.size();
    auto rnd = [&]() {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      return s;
    };
    for (int k = 0; k < 200; k++) {
      std::vector<uint8_t> v = raw;
      if (k % 4 == 0) {
        v.resize(rnd() % (raw.size() + 1));  // truncated
      } else {
        const int flips = 1 + (int)(rnd() % 8);
        for (int f = 0; f < flips && !v.empty(); f++) v[rnd() % v.size()] ^= (uint8_t)(1u << (rnd() % 8));
        if (k % 4 == 1) {  // aim at the first pages (meta, freelist, root): the offsets live there
          for (int f = 0; f < 4; f++) v[rnd() % std::min<size_t>(v.size(), 3 * 4096)] = (uint8_t)rnd();
        }
      }
      spit(tmp, v);
      (void)load_all(tmp.c_str());  // may fail; must not fault (ASan/UBSan report otherwise)
      tried++;
    }
    remove(tmp.c_str());
  }
  printf("{\"boltload\": {\"files\": %d, \"mutants\": %llu}}\n", argc, tried);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && !strcmp(argv[1], "coalesce")) test_coalesce();
  else if (argc >= 3 && !strcmp(argv[1], "boltload")) test_boltload(argc - 2, argv + 2);
  else {
    fprintf(stderr, "usage: %s coalesce | boltload file.db...\n", argv[0]);
    return 2;
  }
  if (fails) fprintf(stderr, "%d checks failed\n", fails);
  return fails ? 1 : 0;
}

// Request coalescer of the thread-safe service (include/blsverify.h blsv_service_*): any number of
// threads submit() one request each and block; ONE dispatcher thread gathers the requests that arrive
// close together and hands them to run(batch) in a single call, then wakes their callers.
//
// Gathering rule: after the first waiting request the dispatcher keeps collecting while requests keep
// arriving within `gap` of the previous one, for at most `max_wait` after the first, or until
// `max_batch` are waiting. Requests that arrive while run() executes form the next batch; if their
// window has already passed by then (a burst that arrived during a launch) they launch at once.
//
// Pure C++ (no HIP): tools/hosttest.cpp runs it with a stand-in run() under ASan/UBSan and TSan.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace blsv_detail {

template <typename Req>
class Coalescer {
 public:
  using Clock = std::chrono::steady_clock;
  using Run = std::function<void(std::vector<Req*>&)>;
  using Fail = std::function<void(Req*)>;  // marks one request failed (run() could not process it)
  struct Stats {
    uint64_t launches = 0, items = 0, max_batch = 0;
  };

  Coalescer(Run run, uint32_t gap_us, uint32_t max_wait_us, size_t max_batch, Fail fail = nullptr)
      : run_(std::move(run)),
        fail_(std::move(fail)),
        gap_(std::chrono::microseconds(gap_us)),
        max_wait_(std::chrono::microseconds(max_wait_us)),
        max_batch_(max_batch ? max_batch : 1) {
    th_ = std::thread([this] { loop(); });
  }
  Coalescer(const Coalescer&) = delete;
  Coalescer& operator=(const Coalescer&) = delete;

  // Drains what was submitted, then joins the dispatcher.
  ~Coalescer() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    work_.notify_one();
    th_.join();
  }

  // Blocks until run() has processed r (run() fills r's outputs).
  void submit(Req* r) {
    Slot s{r, false};
    std::unique_lock<std::mutex> g(mu_);
    const auto now = Clock::now();
    if (q_.empty()) first_ = now;
    last_ = now;
    q_.push_back(&s);
    work_.notify_one();
    done_.wait(g, [&] { return s.done; });
  }

  // Runs f() on the calling thread while the dispatcher is between batches (it holds no batch and
  // starts none until f returns): for reconfiguring what run() reads.
  template <typename F>
  auto with_idle(F f) -> decltype(f()) {
    std::unique_lock<std::mutex> g(mu_);
    idle_.wait(g, [&] { return !busy_; });
    return f();
  }

  Stats stats() {
    std::lock_guard<std::mutex> g(mu_);
    return st_;
  }

 private:
  struct Slot {
    Req* r;
    bool done;
  };

  void loop() {
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      work_.wait(g, [&] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stopping, nothing left
      while (q_.size() < max_batch_ && !stop_) {
        const auto dl = std::min(first_ + max_wait_, last_ + gap_);
        if (Clock::now() >= dl) break;
        work_.wait_until(g, dl);
      }
      const size_t n = std::min(q_.size(), max_batch_);
      std::vector<Slot*> slots;
      bool ran = false;
      try {
        slots.assign(q_.begin(), q_.begin() + (ptrdiff_t)n);
      } catch (...) {
        // not even the batch list fits in host memory: fail the oldest request alone
        Slot* s = q_.front();
        q_.pop_front();
        if (fail_) fail_(s->r);
        s->done = true;
        done_.notify_all();
        continue;
      }
      q_.erase(q_.begin(), q_.begin() + (ptrdiff_t)n);
      // an overflow beyond max_batch has waited its window already: it launches right after this one
      if (!q_.empty()) first_ = last_ = Clock::now() - max_wait_ - gap_;
      busy_ = true;
      g.unlock();
      try {
        std::vector<Req*> batch;
        batch.reserve(n);
        for (Slot* s : slots) batch.push_back(s->r);
        run_(batch);
        ran = true;
      } catch (...) {
        // run() threw (host allocation of a large batch): every caller of the batch still returns
      }
      g.lock();
      busy_ = false;
      idle_.notify_all();
      for (Slot* s : slots) {
        if (!ran && fail_) fail_(s->r);
        s->done = true;
      }
      st_.launches++;
      st_.items += n;
      st_.max_batch = std::max<uint64_t>(st_.max_batch, n);
      done_.notify_all();
    }
  }

  Run run_;
  Fail fail_;
  const Clock::duration gap_, max_wait_;
  const size_t max_batch_;
  std::mutex mu_;
  std::condition_variable work_, done_, idle_;
  std::deque<Slot*> q_;
  Clock::time_point first_{}, last_{};
  bool stop_ = false;
  bool busy_ = false;  // run() executing (with_idle waits it out)
  Stats st_;
  std::thread th_;
};

}  // namespace blsv_detail

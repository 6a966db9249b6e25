// A few persistent host worker threads for the per-call host passes of a handle (the BA's edge
// staging): run(fn, ctx) calls fn(ctx, part) for part in [0, parts()), part 0 on the calling thread.
// Between calls a worker spins for a short while (50 us: a longer spin kept three workers busy between
// the calls of a pipelined BA, against the box's 16-CPU quota), then sleeps on a condition
// variable.  Not re-entrant: one run at a time per pool, as a handle serves one call at a time.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

namespace rspl {

class HostPool {
 public:
  using Fn = void (*)(void* ctx, int part);

  explicit HostPool(int workers) {
    for (int w = 0; w < workers; w++) th_.emplace_back([this, w] { loop(w + 1); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_.store(true, std::memory_order_release);
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int parts() const { return (int)th_.size() + 1; }

  void run(Fn fn, void* ctx) {
    fn_ = fn;
    ctx_ = ctx;
    left_.store((int)th_.size(), std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);  // pairs with a worker's check-then-wait
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    fn(ctx, 0);
    while (left_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }

 private:
  void loop(int part) {
    unsigned seen = 0;
    for (;;) {
      // spin (yielding) up to kSpin after the last job, then sleep until the next
      const auto t0 = std::chrono::steady_clock::now();
      unsigned g;
      while ((g = gen_.load(std::memory_order_acquire)) == seen && !quit_.load(std::memory_order_acquire) &&
             std::chrono::steady_clock::now() - t0 < kSpin)
        std::this_thread::yield();
      if (g == seen && !quit_.load(std::memory_order_acquire)) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          return gen_.load(std::memory_order_acquire) != seen || quit_.load(std::memory_order_acquire);
        });
        g = gen_.load(std::memory_order_acquire);
      }
      if (quit_.load(std::memory_order_acquire)) return;
      seen = g;
      fn_(ctx_, part);
      left_.fetch_sub(1, std::memory_order_release);
    }
  }

  static constexpr std::chrono::microseconds kSpin{50};
  std::vector<std::thread> th_;
  std::atomic<unsigned> gen_{0};
  std::atomic<int> left_{0};
  std::atomic<bool> quit_{false};
  Fn fn_ = nullptr;
  void* ctx_ = nullptr;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace rspl

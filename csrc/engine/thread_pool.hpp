// Persistent worker pool shared by the search (csrc/mcts/search.hpp) and the batched feature /
// ladder entry points (bindings.cpp): threads start once, and run(n, fn) hands out indices
// 0..n-1 through an atomic counter, so a call costs a wake-up instead of n thread creations.
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace rag {

// Persistent worker pool (thread start-up is not paid per call).
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size(); }
  void run(int n, const std::function<void(int)>& fn) {
    if (n <= 0) return;
    std::lock_guard<std::mutex> serial(run_mu_);  // one job at a time per pool
    if (th_.empty() || n == 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::unique_lock<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_ = 0;
    active_ = (int)th_.size();
    ++gen_;
    cv_.notify_all();
    done_.wait(lk, [this] { return active_ == 0; });
    fn_ = nullptr;
  }

 private:
  void loop() {
    uint64_t seen = 0;
    while (true) {
      const std::function<void(int)>* fn;
      int n;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
        fn = fn_;
        n = n_;
      }
      for (int i = next_++; i < n; i = next_++) (*fn)(i);
      std::lock_guard<std::mutex> g(mu_);
      if (--active_ == 0) done_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, active_ = 0;
  std::atomic<int> next_{0};
  uint64_t gen_ = 0;
  bool stop_ = false;
};


// Process-wide pool of `n` workers (created on first use, kept for the process lifetime).
inline Pool& shared_pool(int n) {
  static std::mutex mu;
  static std::map<int, std::unique_ptr<Pool>> pools;
  std::lock_guard<std::mutex> g(mu);
  auto& p = pools[n];
  if (!p) p = std::make_unique<Pool>(n);
  return *p;
}

}  // namespace rag

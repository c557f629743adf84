/*
 * host_pool.h — persistent host worker threads (shared by engine.hip and
 * burst_engine.hip): one task at a time, fn(t, T) run for t in [0, T).
 */
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace aero {

// Persistent host workers for the per-frame SU/ACARS work.  One task at a
// time: the previous pass's frames are finished before the next pass's are
// started, so a channel's frames keep their order.  submit() returns at
// once, so while a task runs the caller goes on launching GPU work (frames
// of step k are parsed while step k+1 demodulates).
class HostPool {
 public:
  explicit HostPool(int n) : n_(std::max(1, n)) {
    for (int t = 0; t < n_; t++) th_.emplace_back([this, t] { loop(t); });
  }
  ~HostPool() {
    wait();
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &x : th_) x.join();
  }
  int size() const { return n_; }
  // runs fn(t, T) for t in [0, T) on the pool's threads
  void submit(std::function<void(int, int)> fn, int T) {
    wait();
    {
      std::lock_guard<std::mutex> g(m_);
      fn_ = std::move(fn);
      tn_ = std::max(1, std::min(T, n_));
      left_ = tn_;
      gen_++;
    }
    cv_.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> g(m_);
    done_cv_.wait(g, [this] { return left_ == 0; });
  }

 private:
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      int T;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        T = tn_;
      }
      if (t >= T) continue;
      fn_(t, T);  // fn_ is only replaced after every worker of this task is done
      std::lock_guard<std::mutex> g(m_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  int n_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  std::function<void(int, int)> fn_;
  int tn_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace aero

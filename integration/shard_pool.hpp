// shard_pool.hpp -- one worker thread per device shard of XorecBenchmarkHipMulti
// (plain C++, no reference or HIP header: compiled into the plugin in both builds).
//
// run(fn) calls fn(i) for every shard i at once -- shard 0 on the calling
// thread, shard i > 0 on worker i -- and returns when all calls have.  Used
// for decode(), whose xec_decode scans each shard's bitmap slice on the host
// before it launches (~1.1 ns per stripe): on one thread device i would launch
// only after the scans of devices 0..i-1 (config 4 over 8 devices: ~65 us of
// skew against a ~180 us kernel).  The workers live as long as the plugin and
// sleep on a condition variable between calls.
#pragma once

#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace xec_hip {

class ShardPool {
 public:
  // A thread that cannot be started leaves none running: the ones already
  // started are stopped and joined before the exception leaves (a throwing
  // constructor runs no destructor, and a joinable std::thread would
  // terminate the process).
  explicit ShardPool(size_t shards) : n_(shards) {
    try {
      for (size_t i = 1; i < n_; ++i) threads_.emplace_back([this, i] { worker(i); });
    } catch (...) {
      stop_all();
      throw;
    }
  }
  ~ShardPool() { stop_all(); }
  ShardPool(const ShardPool&) = delete;
  ShardPool& operator=(const ShardPool&) = delete;

  // fn must not throw (the plugin's callbacks are noexcept C-ABI calls).  One
  // caller at a time: run() is not reentrant (the plugin calls it from
  // decode() only).
  void run(const std::function<void(size_t)>& fn) {
    if (n_ == 0) return;
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = &fn;
      pending_ = n_ - 1;
      ++gen_;
    }
    go_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [this] { return pending_ == 0; });
    job_ = nullptr;
  }

 private:
  void stop_all() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    go_.notify_all();
    for (std::thread& t : threads_) t.join();
    threads_.clear();
  }

  void worker(size_t i) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      go_.wait(lk, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(size_t)>* job = job_;
      lk.unlock();
      (*job)(i);
      lk.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }

  size_t n_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable go_, done_;
  const std::function<void(size_t)>* job_ = nullptr;
  uint64_t gen_ = 0;
  size_t pending_ = 0;
  bool stop_ = false;
};

// A one-shot barrier for the n calls of one ShardPool::run: arrive(ok) blocks
// until all n have arrived and returns whether every one brought ok == true.
// decode() checks every shard's bitmap slice first and launches only when all
// are recoverable (all-or-nothing over the whole batch), inside one run().
class Rendezvous {
 public:
  explicit Rendezvous(size_t n) : n_(n) {}
  bool arrive(bool ok) {
    std::unique_lock<std::mutex> lk(mu_);
    all_ok_ = all_ok_ && ok;
    if (++arrived_ == n_) {
      cv_.notify_all();
    } else {
      cv_.wait(lk, [this] { return arrived_ == n_; });
    }
    return all_ok_;
  }

 private:
  size_t n_, arrived_ = 0;
  bool all_ok_ = true;
  std::mutex mu_;
  std::condition_variable cv_;
};

}  // namespace xec_hip

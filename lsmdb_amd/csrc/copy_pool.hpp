// copy_pool.hpp -- the parallel memcpy behind the library's host staging (host_io.hpp).
// Host-only C++ (no HIP types): tests/test_copy_pool.py compiles it into a CPU harness.
#pragma once
#include <algorithm>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

namespace lsmgpu {

// Parallel memcpy for the staging copies (host DRAM to / from page-locked buffers).  Threads are
// started on the first large copy and joined by the destructor.  One copy at a time (a context
// is driven by one thread at a time, include/lsmgpu.h).
class CopyPool {
 public:
  explicit CopyPool(unsigned threads) : want_(threads) {}
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  CopyPool(const CopyPool&) = delete;
  CopyPool& operator=(const CopyPool&) = delete;

  void copy(void* dst, const void* src, size_t n) {
    constexpr size_t kMinPart = 1u << 20;
    if (n < 2 * kMinPart || want_ <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    start();
    const size_t parts = std::min<size_t>(th_.size() + 1, n / kMinPart);
    const size_t step = (n / parts + 4095) / 4096 * 4096;
    std::unique_lock<std::mutex> g(m_);
    jobs_.clear();
    for (size_t o = step; o < n; o += step)
      jobs_.push_back({static_cast<uint8_t*>(dst) + o, static_cast<const uint8_t*>(src) + o,
                       std::min(step, n - o)});
    next_ = 0;
    left_ = jobs_.size();
    g.unlock();
    cv_.notify_all();
    std::memcpy(dst, src, std::min(step, n));  // part 0 on the calling thread
    g.lock();
    while (next_ < jobs_.size()) {  // then help with the rest
      const Job j = jobs_[next_++];
      g.unlock();
      std::memcpy(j.d, j.s, j.n);
      g.lock();
      left_--;
    }
    done_.wait(g, [&] { return left_ == 0; });
  }

 private:
  struct Job {
    uint8_t* d;
    const uint8_t* s;
    size_t n;
  };
  void start() {
    if (!th_.empty()) return;
    for (unsigned i = 0; i + 1 < want_; i++) th_.emplace_back([this] { run(); });
  }
  void run() {
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      cv_.wait(g, [&] { return stop_ || next_ < jobs_.size(); });
      if (stop_) return;
      const Job j = jobs_[next_++];
      g.unlock();
      std::memcpy(j.d, j.s, j.n);
      g.lock();
      if (--left_ == 0) done_.notify_all();
    }
  }
  unsigned want_;
  std::vector<std::thread> th_;
  std::mutex m_;
  std::condition_variable cv_, done_;
  std::vector<Job> jobs_;
  size_t next_ = 0, left_ = 0;
  bool stop_ = false;
};

}  // namespace lsmgpu

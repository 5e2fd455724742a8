// Host thread pool of the drop-in upload path (staging.h).  Kept free of HIP headers so that
// tests/test_host_pool.py can stress it on the host (g++ with ThreadSanitizer).
#pragma once

#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace bh {

// Fixed set of worker threads; parallel_for(n, fn) runs fn(0..n-1) on them and the caller.
class HostPool {
 public:
  explicit HostPool(int workers);
  ~HostPool();
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;
  void parallel_for(int n, const std::function<void(int)>& fn);
  int size() const { return (int)threads_.size() + 1; }

 private:
  void run();
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, active_ = 0;
  size_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace bh

// HostPool (host_pool.h): fixed worker threads running parallel_for(n, fn) with the caller.
#include "host_pool.h"

namespace bh {

HostPool::HostPool(int workers) {
  for (int i = 0; i < workers; i++) threads_.emplace_back([this] { run(); });
}

HostPool::~HostPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : threads_) t.join();
}

// Every claim is tied to the generation the worker woke for: an index is taken, and fn_ read,
// under the lock only while gen_ is still that generation.  A worker that wakes late (after
// its generation's parallel_for returned, possibly after the next one started) therefore never
// runs a stale or null function on another generation's index; it either joins the current
// generation on its next wait or finds nothing left to claim.  fn_ stays valid while any
// claimed index runs: parallel_for returns only once active_ is 0.
void HostPool::run() {
  size_t seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
    if (stop_) return;
    seen = gen_;
    active_++;
    while (gen_ == seen && next_ < n_ && fn_) {
      const int i = next_++;
      const std::function<void(int)>* fn = fn_;
      lk.unlock();
      (*fn)(i);
      lk.lock();
    }
    if (--active_ == 0) done_cv_.notify_all();
  }
}

void HostPool::parallel_for(int n, const std::function<void(int)>& fn) {
  if (n <= 0) return;
  if (threads_.empty() || n == 1) {
    for (int i = 0; i < n; i++) fn(i);
    return;
  }
  {
    std::lock_guard<std::mutex> lk(mu_);
    fn_ = &fn;
    n_ = n;
    next_ = 0;
    gen_++;
  }
  cv_.notify_all();
  for (;;) {  // the caller works too
    int i;
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (next_ >= n_) break;
      i = next_++;
    }
    fn(i);
  }
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return active_ == 0 && next_ >= n_; });
  fn_ = nullptr;
}

}  // namespace bh

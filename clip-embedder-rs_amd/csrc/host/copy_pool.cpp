// Persistent host copy workers (copy_pool.hpp).
#include "copy_pool.hpp"

#include <sched.h>

#include <algorithm>
#include <cstring>

namespace clipgpu {

CopyPool& CopyPool::instance() {
  static CopyPool pool([] {
    int cpus = (int)std::thread::hardware_concurrency();
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) cpus = CPU_COUNT(&set);
    return std::max(0, std::min(16, cpus) - 1);
  }());
  return pool;
}

CopyPool::CopyPool(int workers) {
  for (int i = 0; i < workers; ++i) th_.emplace_back([this] { worker(); });
}

CopyPool::~CopyPool() {
  {
    std::lock_guard<std::mutex> lk(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_) t.join();
}

// A worker joins the current job under mu_ (so the job cannot end and be cleared between reading cur_
// and counting itself in), claims indices until none are left, then leaves under mu_; run() clears
// cur_ only once every joined worker has left, so no worker touches a finished job.
void CopyPool::worker() {
  unsigned seen = 0;
  std::unique_lock<std::mutex> lk(mu_);
  for (;;) {
    cv_.wait(lk, [&] { return stop_ || (cur_ != nullptr && gen_ != seen); });
    if (stop_) return;
    seen = gen_;
    Job* j = cur_;
    ++j->active;
    lk.unlock();
    for (int i; (i = j->next.fetch_add(1)) < j->n;) (*j->f)(i);
    lk.lock();
    if (--j->active == 0) done_cv_.notify_all();
  }
}

void CopyPool::run(int n, const std::function<void(int)>& f) {
  if (n <= 0) return;
  if (n == 1 || th_.empty()) {
    for (int i = 0; i < n; ++i) f(i);
    return;
  }
  std::lock_guard<std::mutex> job(job_mu_);
  Job j;
  j.f = &f;
  j.n = n;
  {
    std::lock_guard<std::mutex> lk(mu_);
    cur_ = &j;
    ++gen_;
  }
  cv_.notify_all();
  for (int i; (i = j.next.fetch_add(1)) < n;) f(i);
  std::unique_lock<std::mutex> lk(mu_);
  done_cv_.wait(lk, [&] { return j.active == 0; });
  cur_ = nullptr;
}

void add_copy_tasks(std::vector<CopyTask>& t, void* dst, const void* src, size_t n) {
  for (size_t o = 0; o < n; o += kCopyTask)
    t.push_back({(char*)dst + o, (const char*)src + o, std::min(kCopyTask, n - o), 1, 0});
}

void add_copy_tasks_2d(std::vector<CopyTask>& t, void* dst, const void* src, size_t row_bytes, size_t rows,
                       size_t sstride) {
  if (sstride == row_bytes) {
    add_copy_tasks(t, dst, src, row_bytes * rows);
    return;
  }
  const size_t per = std::max<size_t>(1, kCopyTask / std::max<size_t>(row_bytes, 1));
  for (size_t r = 0; r < rows; r += per)
    t.push_back({(char*)dst + r * row_bytes, (const char*)src + r * sstride, row_bytes, std::min(per, rows - r),
                 sstride});
}

void pool_copy(const std::vector<CopyTask>& t) {
  CopyPool::instance().run((int)t.size(), [&](int i) {
    const CopyTask& c = t[i];
    for (size_t r = 0; r < c.rows; ++r)
      std::memcpy((char*)c.dst + r * c.n, (const char*)c.src + r * c.sstride, c.n);
  });
}

void pool_memcpy(void* dst, const void* src, size_t n) {
  if (n < 2 * kCopyTask) {
    std::memcpy(dst, src, n);
    return;
  }
  std::vector<CopyTask> t;
  add_copy_tasks(t, dst, src, n);
  pool_copy(t);
}

void pool_gather(void* dst, const void* const* rows, size_t row, int n) {
  std::vector<CopyTask> t;
  for (int i = 0; i < n; ++i) add_copy_tasks(t, (char*)dst + (size_t)i * row, rows[i], row);
  pool_copy(t);
}

}  // namespace clipgpu

// Persistent host copy workers for the host entry points' pinned staging (engine.hip run_host_shard and
// the decoded-image path): one pool per process, its workers parked on a condition variable between jobs,
// so a call pays no thread creation (round 5 spawned up to 8 std::threads per chunk).  One host thread moves
// ~10 GB/s; the staging copies of a 256-image u8 batch (38.5 MB) or of 640x480 RGB8 images (236 MB) need
// several.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace clipgpu {

class CopyPool {
 public:
  // The process's pool: min(16, the CPUs in this process's affinity) threads, the caller counted.
  static CopyPool& instance();
  int threads() const { return (int)th_.size() + 1; }
  // f(i) for every i in [0, n), spread over the workers and the calling thread; returns once all n are
  // done.  Jobs submitted from several threads run one after another.
  void run(int n, const std::function<void(int)>& f);
  ~CopyPool();

 private:
  explicit CopyPool(int workers);
  struct Job {
    const std::function<void(int)>* f;
    int n;
    std::atomic<int> next{0};
    int active = 0;
  };
  void worker();
  std::mutex job_mu_;  // one job at a time
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  Job* cur_ = nullptr;
  unsigned gen_ = 0;
  bool stop_ = false;
  std::vector<std::thread> th_;
};

// memcpy split into 1 MiB pieces over the pool (a plain memcpy below 2 MiB).
void pool_memcpy(void* dst, const void* src, size_t n);
// dst[i * row .. +row) = rows[i][0 .. row) for i < n, over the pool.
void pool_gather(void* dst, const void* const* rows, size_t row, int n);

}  // namespace clipgpu

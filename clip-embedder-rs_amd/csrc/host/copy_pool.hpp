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

// Copies are cut into tasks of at most kCopyTask bytes (enough tasks to keep every worker busy on a
// 4 MiB staging piece; round 6 first used 1 MiB tasks, which left 12 of 16 workers idle there).
constexpr size_t kCopyTask = 256u << 10;
// `rows` rows of n bytes: source rows `sstride` bytes apart, destination rows packed (n apart).
struct CopyTask {
  void* dst;
  const void* src;
  size_t n;
  size_t rows = 1, sstride = 0;
};
// Appends dst[0 .. n) = src[0 .. n) as tasks of <= kCopyTask bytes.
void add_copy_tasks(std::vector<CopyTask>& t, void* dst, const void* src, size_t n);
// Appends a 2-D copy (rows of row_bytes, source rows sstride bytes apart, packed destination) as tasks
// of whole rows, <= kCopyTask bytes each where a row allows.
void add_copy_tasks_2d(std::vector<CopyTask>& t, void* dst, const void* src, size_t row_bytes, size_t rows,
                       size_t sstride);
// Runs the tasks over the pool (inline when there is only one).
void pool_copy(const std::vector<CopyTask>& t);
// memcpy over the pool (a plain memcpy below 2 tasks' worth).
void pool_memcpy(void* dst, const void* src, size_t n);
// dst[i * row .. +row) = rows[i][0 .. row) for i < n, over the pool.
void pool_gather(void* dst, const void* const* rows, size_t row, int n);

}  // namespace clipgpu

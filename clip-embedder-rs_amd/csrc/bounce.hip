// Pinned bounce buffer for synchronous pageable copies (bounce.hpp).
#include "bounce.hpp"

#include <algorithm>
#include <cstring>
#include <mutex>

#include "host/copy_pool.hpp"

namespace clipgpu {
namespace {

constexpr size_t kBounce = 32u << 20;  // two halves: one is filled while the other's DMA runs

struct Bounce {
  std::mutex mu;
  char* pin = nullptr;  // hipHostMallocPortable: any device
  hipError_t ensure() {
    if (pin) return hipSuccess;
    return hipHostMalloc((void**)&pin, kBounce, hipHostMallocPortable);
  }
};
Bounce& bounce() {
  static Bounce b;  // lives for the process (pinned memory is released at exit)
  return b;
}

}  // namespace

hipError_t copy_h2d(void* dst_dev, const void* src_host, size_t n) {
  if (n == 0) return hipSuccess;
  Bounce& b = bounce();
  std::lock_guard<std::mutex> lk(b.mu);
  hipError_t err = b.ensure();
  if (err != hipSuccess) return err;
  hipStream_t s = nullptr;
  err = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (err != hipSuccess) return err;
  hipEvent_t used[2] = {nullptr, nullptr};
  for (int i = 0; i < 2 && err == hipSuccess; ++i) err = hipEventCreateWithFlags(&used[i], hipEventDisableTiming);
  const size_t half = kBounce / 2;
  bool pending[2] = {false, false};
  for (size_t o = 0, i = 0; o < n && err == hipSuccess; o += half, ++i) {
    const int h = (int)(i & 1);
    const size_t len = std::min(half, n - o);
    if (pending[h]) err = hipEventSynchronize(used[h]);  // that half's previous DMA has read it
    if (err != hipSuccess) break;
    pool_memcpy(b.pin + h * half, (const char*)src_host + o, len);
    err = hipMemcpyAsync((char*)dst_dev + o, b.pin + h * half, len, hipMemcpyHostToDevice, s);
    if (err == hipSuccess) err = hipEventRecord(used[h], s);
    pending[h] = true;
  }
  const hipError_t e2 = hipStreamSynchronize(s);
  if (err == hipSuccess) err = e2;
  for (hipEvent_t ev : used)
    if (ev) (void)hipEventDestroy(ev);
  (void)hipStreamDestroy(s);
  return err;
}

hipError_t copy_d2h(void* dst_host, const void* src_dev, size_t n) {
  if (n == 0) return hipSuccess;
  Bounce& b = bounce();
  std::lock_guard<std::mutex> lk(b.mu);
  hipError_t err = b.ensure();
  for (size_t o = 0; o < n && err == hipSuccess; o += kBounce) {
    const size_t len = std::min(kBounce, n - o);
    err = hipMemcpy(b.pin, (const char*)src_dev + o, len, hipMemcpyDeviceToHost);
    if (err == hipSuccess) pool_memcpy((char*)dst_host + o, b.pin, len);
  }
  return err;
}

}  // namespace clipgpu

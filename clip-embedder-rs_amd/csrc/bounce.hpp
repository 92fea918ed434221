// Synchronous copies between device memory and pageable host memory (loader vectors, caller arrays),
// staged through a process-wide pinned bounce buffer, so the HIP runtime never pins or looks up a
// pageable range itself.  Round 6: engine creations right after host-buffer tests faulted inside the
// weight upload's pageable hipMemcpy (hipErrorIllegalAddress, no shader fault; never with
// AMD_SERIALIZE_COPY=3) -- a transfer through a host range the runtime believed pinned after the
// allocator had reused it.  Every synchronous pageable copy of the library goes through these.
#pragma once
#include <hip/hip_runtime.h>
#include <cstddef>

namespace clipgpu {

hipError_t copy_h2d(void* dst_dev, const void* src_host, size_t n);
hipError_t copy_d2h(void* dst_host, const void* src_dev, size_t n);

}  // namespace clipgpu

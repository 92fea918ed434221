// Error plumbing for the C ABI: every entry point runs its body through
// guarded(), which converts exceptions to a status code and records the
// message for clipgpu_last_error() (thread-local).  Status codes map onto the
// reference's ClipError variants (src/error.rs:9-41), see include/clipgpu.h.
#pragma once
#include <new>
#include <stdexcept>
#include <string>

namespace clipgpu {

struct ClipErr : std::runtime_error {
  int code;
  ClipErr(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

void set_last_error(const std::string& msg);

template <typename F>
int guarded(F&& body) {
  try {
    set_last_error("");
    body();
    return 0;
  } catch (const ClipErr& e) {
    set_last_error(e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    set_last_error("out of host memory");
    return 4;
  } catch (const std::exception& e) {
    set_last_error(e.what());
    return 1;
  }
}

}  // namespace clipgpu

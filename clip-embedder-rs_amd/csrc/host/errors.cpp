// Thread-local last-error storage behind clipgpu_last_error() (include/clipgpu.h).
#include <string>
#include "../../../include/clipgpu.h"
#include "api_util.hpp"

namespace clipgpu {
static thread_local std::string g_last_error;
void set_last_error(const std::string& msg) { g_last_error = msg; }
}  // namespace clipgpu

extern "C" const char* clipgpu_last_error(void) { return clipgpu::g_last_error.c_str(); }

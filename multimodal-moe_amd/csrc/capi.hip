// Error plumbing and identification for the C-ABI (include/moe_hip.h).
#include "moe_common.h"

namespace moe {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(const std::string& msg) {
  set_error(msg);
  return -1;
}

int check_launch(const char* what) {
  const hipError_t err = hipGetLastError();
  if (err != hipSuccess) {
    set_error(std::string(what) + ": " + hipGetErrorString(err));
    return -(1000 + (int)err);
  }
  return 0;
}

}  // namespace moe

extern "C" const char* moe_last_error(void) { return moe::g_last_error.c_str(); }

extern "C" const char* moe_version(void) { return "moe_hip 0.1.0 gfx950"; }

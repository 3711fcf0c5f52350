// Error plumbing of the C ABI (include/dro_amd.h).
#include <hip/hip_runtime.h>

#include "dro_common.hpp"

namespace dro {

static thread_local const char* g_last_error = "";

void set_error(const char* msg) { g_last_error = msg; }

// After a launch: surface a launch-configuration failure as a positive
// hipError_t (never synchronises, so it stays graph-capturable).
int launch_status(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = what;
    return (int)e;
  }
  return DRO_OK;
}

}  // namespace dro

extern "C" const char* dro_last_error(void) { return dro::g_last_error; }

extern "C" int dro_abi_version(void) { return 1; }

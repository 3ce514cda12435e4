// api.cpp -- ABI version, thread-local error text, HIP error mapping.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "../../include/mpcqp.h"

namespace mpcqp {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int hip_fail(hipError_t e, const char* where) {
  set_error("%s: HIP error %d (%s)", where, (int)e, hipGetErrorString(e));
  return MPCQP_EHIP;
}

}  // namespace mpcqp

extern "C" int mpcqp_abi_version(void) { return MPCQP_ABI_VERSION; }

extern "C" const char* mpcqp_last_error(void) { return mpcqp::g_err; }

// Error plumbing and version query for the lcq C ABI.
#include "lcq_common.h"

namespace lcq {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  set_error(msg);
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(LCQ_ELAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  return LCQ_OK;
}

}  // namespace lcq

extern "C" int lcq_version(void) { return 1; }

extern "C" const char* lcq_last_error(void) { return lcq::g_last_error.c_str(); }

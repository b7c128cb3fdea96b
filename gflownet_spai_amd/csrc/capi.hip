// ABI version + thread-local last error for libspai_hip.so.
#include <string>

#include "spai_status.h"

namespace spai {
static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}
}  // namespace spai

extern "C" int spai_abi_version(void) { return 17; }

extern "C" const char* spai_last_error(void) { return spai::g_last_error.c_str(); }

// ABI bookkeeping: version and per-thread error text.
#include <cstring>
#include <string>

#include "common.h"

namespace lea {
namespace {
thread_local char g_err[512] = {0};
}

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

void clear_error() { g_err[0] = 0; }

}  // namespace lea

extern "C" int lea_abi_version(void) { return LEA_ABI_VERSION; }

extern "C" const char* lea_last_error(void) { return lea::g_err; }

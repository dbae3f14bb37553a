// C-ABI bookkeeping: version and per-thread error message (include/kwhisper.h).
#include <stdio.h>
#include <string.h>

#include "kw_common.h"

static thread_local char g_err[512] = "";

int kw_set_error(hipError_t e) {
  snprintf(g_err, sizeof(g_err), "HIP error %d: %s", (int)e, hipGetErrorString(e));
  return KW_EHIP;
}

int kw_set_error_msg(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

extern "C" int kw_version(void) { return 110; }

extern "C" const char* kw_last_error(void) { return g_err; }

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

extern "C" int kw_version(void) { return 112; }

extern "C" int kw_stream_create(kw_stream_t* out) {
  if (!out) return kw_set_error_msg(KW_EINVAL, "kw_stream_create: null out");
  hipStream_t s = nullptr;
  const hipError_t e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  if (e != hipSuccess) return kw_set_error(e);
  *out = (kw_stream_t)s;
  return KW_OK;
}

extern "C" int kw_stream_destroy(kw_stream_t stream) {
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? KW_OK : kw_set_error(e);
}

extern "C" const char* kw_last_error(void) { return g_err; }

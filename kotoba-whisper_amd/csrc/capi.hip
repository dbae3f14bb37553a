// C-ABI bookkeeping: version and per-thread error message (include/kwhisper.h).
#include <stdio.h>
#include <string.h>

#include <hip/hip_ext.h>

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

extern "C" int kw_version(void) { return 103; }

extern "C" const char* kw_last_error(void) { return g_err; }

// A stream restricted to CUs [cu_begin, cu_end) (hipExtStreamCreateWithCUMask): the pipelined generate
// runs the next batch's log-mel / encoder / cross-K/V there while the current batch's latency-bound
// decode steps replay on the whole chip.
extern "C" int kw_stream_create_cu_range(int cu_begin, int cu_end, kw_stream_t* out) {
  if (!out || cu_begin < 0 || cu_end <= cu_begin) return kw_set_error_msg(KW_EINVAL, "kw_stream_create_cu_range: bad range");
  int dev = 0, ncu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess) return kw_set_error(e);
  if (cu_end > ncu) cu_end = ncu;
  if (cu_end <= cu_begin) return kw_set_error_msg(KW_EINVAL, "kw_stream_create_cu_range: range beyond the device's CUs");
  uint32_t mask[32] = {0};
  const int words = (ncu + 31) / 32;
  if (words > 32) return kw_set_error_msg(KW_EUNSUPPORTED, "kw_stream_create_cu_range: more than 1024 CUs");
  for (int c = cu_begin; c < cu_end; ++c) mask[c / 32] |= 1u << (c % 32);
  hipStream_t st = nullptr;
  e = hipExtStreamCreateWithCUMask(&st, (uint32_t)words, mask);
  if (e != hipSuccess) return kw_set_error(e);
  *out = (kw_stream_t)st;
  return KW_OK;
}

extern "C" int kw_stream_destroy(kw_stream_t stream) {
  const hipError_t e = hipStreamDestroy((hipStream_t)stream);
  return e == hipSuccess ? KW_OK : kw_set_error(e);
}

// Process-level entry points of libgmat_hip: version, devices, error text.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>

#include "common.h"

namespace gmat {
static thread_local char g_err[1024] = "";
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
}  // namespace gmat

extern "C" const char *gmat_last_error(void) { return gmat::g_err; }

extern "C" int gmat_version(void) { return 1; }

extern "C" int gmat_device_count(int *n) {
  GMAT_CHECK(n, GMAT_E_ARG, "gmat_device_count: null");
  int c = 0;
  hipError_t e = hipGetDeviceCount(&c);
  if (e != hipSuccess) c = 0;
  *n = c;
  return GMAT_OK;
}

extern "C" int gmat_set_device(int device) {
  GMAT_HIP(hipSetDevice(device));
  return GMAT_OK;
}

extern "C" int gmat_device_synchronize(void) {
  GMAT_HIP(hipDeviceSynchronize());
  return GMAT_OK;
}

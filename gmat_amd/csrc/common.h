// Shared plumbing for libgmat_hip: error reporting, device buffers, MFMA vector types.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/gmat_hip.h"

namespace gmat {

void set_error(const char *fmt, ...);

// Device memory through a process-wide cache (capi.cpp): freed blocks stay reserved per device and
// size class and are handed out again, so a plan created and destroyed per call (remma_epiAA end to
// end) does not pay hipMalloc / hipFree each time.  pool_alloc returns the block and its real size
// (>= n) or nullptr with the error set; pool_free synchronises the device first (the implicit
// synchronisation of hipFree that callers rely on) and returns the block to the cache.
// pool_free files the block under the device it was allocated on (dev); pool_cached_bytes is what the
// cache holds for the current device (free for the taking: callers sizing buffers from hipMemGetInfo add it)
void *pool_alloc(size_t n, size_t *got);
void pool_free(void *p, size_t bytes, int dev);
size_t pool_cached_bytes();
// the same for pinned host staging buffers (hipHostMalloc / hipHostFree take about a millisecond each)
void *pinned_alloc(size_t n, size_t *got);
void pinned_free(void *p, size_t bytes);
// non-blocking HIP streams from a process-wide cache (stream creation / destruction cost milliseconds);
// stream_release synchronises the stream and keeps it for the next stream_acquire on its device
int stream_acquire(hipStream_t *out);
// the scan pipeline's fixed streams per device, in creation order: 0 the screen (and plan setup), 1 the
// even launches' prefilter, 2 pair screen and refine, 3 the odd launches' prefilter, 4 the refine's side
// terms -- shared by every plan, never released (capi.cpp)
int pipeline_stream(int role, hipStream_t *out);
void stream_release(hipStream_t s);

#define GMAT_HIP(x)                                                                        \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      ::gmat::set_error("%s:%d %s -> %s", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return GMAT_E_HIP;                                                                   \
    }                                                                                      \
  } while (0)

#define GMAT_CHECK(cond, code, ...)    \
  do {                                 \
    if (!(cond)) {                     \
      ::gmat::set_error(__VA_ARGS__);  \
      return (code);                   \
    }                                  \
  } while (0)

#define GMAT_TRY(x)          \
  do {                       \
    int rc_ = (x);           \
    if (rc_ != GMAT_OK) return rc_; \
  } while (0)

// Owning device allocation (hipMalloc'd, freed on destruction).
struct DBuf {
  void *p = nullptr;
  size_t bytes = 0;  // the size asked for (kernels and the plan state use it as the buffer's size)
  size_t cap = 0;    // the block's real size (the cache's size class)
  int dev = 0;       // the device it was allocated on
  DBuf() = default;
  DBuf(const DBuf &) = delete;
  DBuf &operator=(const DBuf &) = delete;
  ~DBuf() { release(); }
  void release() {
    if (p) pool_free(p, cap, dev);
    p = nullptr;
    bytes = cap = 0;
  }
  int alloc(size_t n) {
    if (n <= bytes && p) return GMAT_OK;
    release();
    if (n == 0) n = 16;
    (void)hipGetDevice(&dev);
    p = pool_alloc(n, &cap);
    if (!p) return GMAT_E_NOMEM;
    bytes = n;
    return GMAT_OK;
  }
  template <class T> T *as() const { return reinterpret_cast<T *>(p); }
};

inline int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
inline int64_t cdiv(int64_t x, int64_t m) { return (x + m - 1) / m; }

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef double v4d __attribute__((ext_vector_type(4)));

}  // namespace gmat

// Process-level entry points of libgmat_hip: version, devices, error text.
#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "common.h"

namespace gmat {
static thread_local char g_err[1024] = "";
void set_error(const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

// ---- device memory cache behind DBuf (common.h)
namespace {
struct Pool {
  std::mutex mu;
  std::multimap<std::pair<int, size_t>, void *> free_blocks;  // (device, bytes) -> block
  size_t cached = 0;
  size_t limit() const {  // bytes kept cached at most (GMAT_POOL_MAX_GB, default 32)
    const char *e = getenv("GMAT_POOL_MAX_GB");
    return (size_t)((e ? atof(e) : 32.0) * (double)(1ull << 30));
  }
  void trim_all() {  // caller holds mu
    for (auto &kv : free_blocks) (void)hipFree(kv.second);
    free_blocks.clear();
    cached = 0;
  }
};
Pool &pool() {
  static Pool *p = new Pool;  // never destroyed: blocks may be released during static destruction
  return *p;
}
// size classes: 256 B granules below 1 MiB, 2 MiB granules above
size_t size_class(size_t n) {
  return n < (1u << 20) ? (n + 255) / 256 * 256 : (n + (2u << 20) - 1) / (2u << 20) * (2u << 20);
}
}  // namespace

void *pool_alloc(size_t n, size_t *got) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  const size_t c = size_class(n);
  Pool &pl = pool();
  {
    std::lock_guard<std::mutex> lk(pl.mu);
    // the smallest cached block of this device that fits and wastes at most an eighth
    auto it = pl.free_blocks.lower_bound({dev, c});
    if (it != pl.free_blocks.end() && it->first.first == dev && it->first.second <= c + c / 8) {
      void *p = it->second;
      *got = it->first.second;
      pl.cached -= it->first.second;
      pl.free_blocks.erase(it);
      return p;
    }
  }
  void *p = nullptr;
  hipError_t e = hipMalloc(&p, c);
  if (e != hipSuccess) {  // out of memory: give the cached blocks back and try once more
    (void)hipGetLastError();
    {
      std::lock_guard<std::mutex> lk(pl.mu);
      (void)hipDeviceSynchronize();
      pl.trim_all();
    }
    e = hipMalloc(&p, c);
    if (e != hipSuccess) {
      set_error("hipMalloc(%zu bytes): %s", c, hipGetErrorString(e));
      return nullptr;
    }
  }
  *got = c;
  return p;
}

void pool_free(void *p, size_t bytes, int dev) {
  if (!p) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  (void)hipDeviceSynchronize();  // no kernel still uses the block when it is handed out again
  if (cur != dev) (void)hipSetDevice(cur);
  Pool &pl = pool();
  std::lock_guard<std::mutex> lk(pl.mu);
  if (pl.cached + bytes > pl.limit()) {
    (void)hipFree(p);
    return;
  }
  pl.free_blocks.insert({{dev, bytes}, p});
  pl.cached += bytes;
}

size_t pool_cached_bytes() {
  int dev = 0;
  (void)hipGetDevice(&dev);
  Pool &pl = pool();
  std::lock_guard<std::mutex> lk(pl.mu);
  size_t c = 0;
  for (auto it = pl.free_blocks.lower_bound({dev, 0}); it != pl.free_blocks.end() && it->first.first == dev; ++it)
    c += it->first.second;
  return c;
}

namespace {
struct PinnedPool {
  std::mutex mu;
  std::multimap<size_t, void *> free_blocks;
  size_t cached = 0;
};
PinnedPool &pinned_pool() {
  static PinnedPool *p = new PinnedPool;
  return *p;
}
}  // namespace

void *pinned_alloc(size_t n, size_t *got) {
  const size_t c = n < 4096 ? 4096 : (n + 65535) / 65536 * 65536;
  PinnedPool &pl = pinned_pool();
  {
    std::lock_guard<std::mutex> lk(pl.mu);
    auto it = pl.free_blocks.lower_bound(c);
    if (it != pl.free_blocks.end() && it->first <= 2 * c) {
      void *p = it->second;
      *got = it->first;
      pl.cached -= it->first;
      pl.free_blocks.erase(it);
      return p;
    }
  }
  void *p = nullptr;
  hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
  if (e != hipSuccess) {
    set_error("hipHostMalloc(%zu bytes): %s", c, hipGetErrorString(e));
    return nullptr;
  }
  *got = c;
  return p;
}

// non-blocking streams, kept per device once created (hipStreamCreate / hipStreamDestroy take ~3 ms
// each: a plan's five streams cost ~30 ms of every remma_epiAA call end to end)
namespace {
struct StreamPool {
  std::mutex mu;
  std::multimap<int, hipStream_t> free_streams;  // device -> stream
};
StreamPool &stream_pool() {
  static StreamPool *p = new StreamPool;
  return *p;
}
}  // namespace

int stream_acquire(hipStream_t *out) {
  int dev = 0;
  GMAT_HIP(hipGetDevice(&dev));
  StreamPool &pl = stream_pool();
  {
    std::lock_guard<std::mutex> lk(pl.mu);
    auto it = pl.free_streams.find(dev);
    if (it != pl.free_streams.end()) {
      *out = it->second;
      pl.free_streams.erase(it);
      return GMAT_OK;
    }
  }
  GMAT_HIP(hipStreamCreateWithFlags(out, hipStreamNonBlocking));
  return GMAT_OK;
}

// The scan pipeline's streams, one fixed set per device shared by every plan (round 5).  HIP maps a
// process's streams onto GPU_MAX_HW_QUEUES (4) hardware queues as they are created, and streams that
// share a queue wait for each other's kernels; the pipeline was tuned on the set a first plan creates
// (the screen stream, then the even / odd prefilter streams, the pair-screen / refine stream and the
// refine's side stream).  Taken from a pool, later plans got those roles on other queues: the
// covariate leg of the bench ran 38.5 instead of 32.0 ms per step with the intercept plan alive.  The
// set is created once, in that order, on the first request; plans do not release it.
int pipeline_stream(int role, hipStream_t *out) {
  constexpr int NR = 5;
  static std::mutex mu;
  static std::map<int, std::vector<hipStream_t>> sets;
  if (role < 0 || role >= NR) {
    set_error("pipeline_stream: role %d", role);
    return GMAT_E_ARG;
  }
  int dev = 0;
  GMAT_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  std::vector<hipStream_t> &v = sets[dev];
  if (v.empty()) {
    // created into a local set, committed only when all five exist (a partial set would hand later
    // plans the null stream for the missing roles)
    hipStream_t made[NR] = {};
    for (int k = 0; k < NR; ++k) {
      const hipError_t err = hipStreamCreateWithFlags(&made[k], hipStreamNonBlocking);
      if (err != hipSuccess) {
        for (int q = 0; q < k; ++q) (void)hipStreamDestroy(made[q]);
        set_error("pipeline_stream: hipStreamCreateWithFlags: %s", hipGetErrorString(err));
        return GMAT_E_HIP;
      }
    }
    v.assign(made, made + NR);
  }
  *out = v[role];
  return GMAT_OK;
}

void stream_release(hipStream_t s) {
  if (!s) return;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return;
  (void)hipStreamSynchronize(s);  // its work is done before another user queues behind it
  StreamPool &pl = stream_pool();
  std::lock_guard<std::mutex> lk(pl.mu);
  pl.free_streams.insert({dev, s});
}

void pinned_free(void *p, size_t bytes) {
  if (!p) return;
  PinnedPool &pl = pinned_pool();
  std::lock_guard<std::mutex> lk(pl.mu);
  if (pl.cached + bytes > (size_t)1 << 30) {  // keep at most 1 GiB of pinned memory cached
    (void)hipHostFree(p);
    return;
  }
  pl.free_blocks.insert({bytes, p});
  pl.cached += bytes;
}

}  // namespace gmat

extern "C" const char *gmat_last_error(void) { return gmat::g_err; }

extern "C" int gmat_empty_cache(void) {
  gmat::Pool &pl = gmat::pool();
  std::lock_guard<std::mutex> lk(pl.mu);
  GMAT_HIP(hipDeviceSynchronize());
  pl.trim_all();
  gmat::PinnedPool &pp = gmat::pinned_pool();
  std::lock_guard<std::mutex> lk2(pp.mu);
  for (auto &kv : pp.free_blocks) (void)hipHostFree(kv.second);
  pp.free_blocks.clear();
  pp.cached = 0;
  return GMAT_OK;
}

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

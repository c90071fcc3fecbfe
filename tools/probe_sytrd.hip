// Timing probe (GPU box): rocSOLVER dsytrd/dormtr against ssytrd/sormtr at n = 2,000 (the plan's
// eigensolver front end), warm calls.  Build: hipcc --offload-arch=gfx950 -O2 -o /tmp/probe_sytrd
//   tools/probe_sytrd.hip -L/opt/rocm/lib -lrocsolver -lrocblas
#include <hip/hip_runtime.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

template <class T>
static void run(rocblas_handle hb, int n, int ne, const std::vector<double> &h) {
  std::vector<T> ht(h.begin(), h.end());
  T *A, *A0, *d, *e, *tau, *Z;
  hipMalloc(&A, sizeof(T) * n * n);
  hipMalloc(&A0, sizeof(T) * n * n);
  hipMalloc(&d, sizeof(T) * n);
  hipMalloc(&e, sizeof(T) * n);
  hipMalloc(&tau, sizeof(T) * n);
  hipMalloc(&Z, sizeof(T) * n * ne);
  hipMemcpy(A0, ht.data(), sizeof(T) * n * n, hipMemcpyHostToDevice);
  hipMemset(Z, 0, sizeof(T) * n * ne);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(A, A0, sizeof(T) * n * n, hipMemcpyDeviceToDevice);
    hipDeviceSynchronize();
    const double t0 = now();
    if constexpr (sizeof(T) == 8)
      rocsolver_dsytrd(hb, rocblas_fill_lower, n, A, n, d, e, tau);
    else
      rocsolver_ssytrd(hb, rocblas_fill_lower, n, A, n, d, e, tau);
    hipDeviceSynchronize();
    const double t1 = now();
    if constexpr (sizeof(T) == 8)
      rocsolver_dormtr(hb, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, n, ne, A, n, tau, Z, n);
    else
      rocsolver_sormtr(hb, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none, n, ne, A, n, tau, Z, n);
    hipDeviceSynchronize();
    const double t2 = now();
    printf("%s n %d: sytrd %.2f ms, ormtr(%d) %.2f ms\n", sizeof(T) == 8 ? "fp64" : "fp32", n, 1e3 * (t1 - t0), ne,
           1e3 * (t2 - t1));
  }
  hipFree(A);
  hipFree(A0);
  hipFree(d);
  hipFree(e);
  hipFree(tau);
  hipFree(Z);
}

int main() {
  rocblas_handle hb;
  rocblas_create_handle(&hb);
  const int n = 2000, ne = 129;
  std::vector<double> h((size_t)n * n);
  std::mt19937_64 g(1);
  std::normal_distribution<double> nd;
  std::vector<double> b((size_t)n * 64);
  for (auto &v : b) v = nd(g);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j <= i; ++j) {
      double s = (i == j) ? n * 0.05 : 0.0;
      for (int k = 0; k < 64; ++k) s += b[(size_t)i * 64 + k] * b[(size_t)j * 64 + k] * 0.01;
      h[(size_t)i * n + j] = h[(size_t)j * n + i] = s;
    }
  run<double>(hb, n, ne, h);
  run<float>(hb, n, ne, h);
  return 0;
}

// Timing probe (GPU box): rocSOLVER symmetric eigensolvers at the plan's sizes, and the library's
// own fp64 dgemm / Cholesky (linked from libgmat_hip.so).  Build:
//   hipcc --offload-arch=gfx950 -O2 -o tools/probe_eig tools/probe_eig.hip -Lgmat_amd -lgmat_hip \
//         -L/opt/rocm/lib -lrocsolver -lrocblas -Wl,-rpath,$PWD/gmat_amd
#include <hip/hip_runtime.h>
#include <rocsolver/rocsolver.h>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include "../gmat_amd/csrc/dla.h"

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  rocblas_handle hb;
  rocblas_create_handle(&hb);
  for (int n : {2000, 5000}) {
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
    double *A, *A0, *W, *E, *Z, *res;
    int *info, *nev, *sweeps;
    hipMalloc(&A, (size_t)n * n * 8);
    hipMalloc(&A0, (size_t)n * n * 8);
    hipMalloc(&Z, (size_t)n * n * 8);
    hipMalloc(&W, n * 8);
    hipMalloc(&E, n * 8);
    hipMalloc(&res, (size_t)n * 8);
    hipMalloc(&info, 4);
    hipMalloc(&nev, 4);
    hipMalloc(&sweeps, 4);
    hipMemcpy(A0, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
      hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
      hipDeviceSynchronize();
      double t0 = now();
      rocsolver_dsyevd(hb, rocblas_evect_original, rocblas_fill_lower, n, A, n, W, E, info);
      hipDeviceSynchronize();
      double t1 = now();
      // fp32 variants and the tridiagonal reduction alone
      float *Af = (float *)Z, *Wf = (float *)W, *Ef = (float *)E;
      {
        std::vector<float> hf(h.begin(), h.end());
        hipMemcpy(Af, hf.data(), (size_t)n * n * 4, hipMemcpyHostToDevice);
      }
      hipDeviceSynchronize();
      double t2 = now();
      rocsolver_ssyevd(hb, rocblas_evect_original, rocblas_fill_lower, n, Af, n, Wf, Ef, info);
      hipDeviceSynchronize();
      double t3 = now();
      hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
      hipDeviceSynchronize();
      double t4 = now();
      rocsolver_dsytrd(hb, rocblas_fill_lower, n, A, n, W, E, res == nullptr ? W : (double *)Z);
      hipDeviceSynchronize();
      double t5 = now();
      {
        std::vector<float> hf(h.begin(), h.end());
        hipMemcpy(Af, hf.data(), (size_t)n * n * 4, hipMemcpyHostToDevice);
      }
      hipDeviceSynchronize();
      double t6 = now();
      rocsolver_ssytrd(hb, rocblas_fill_lower, n, Af, n, Wf, Ef, (float *)res);
      hipDeviceSynchronize();
      double t7 = now();
      // rocSOLVER Cholesky + inverse from the factor (the REML's V^-1)
      hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
      hipDeviceSynchronize();
      double tp0 = now();
      rocsolver_dpotrf(hb, rocblas_fill_lower, n, A, n, info);
      hipDeviceSynchronize();
      double tp1 = now();
      rocsolver_dpotri(hb, rocblas_fill_lower, n, A, n, info);
      hipDeviceSynchronize();
      double tp2 = now();
      if (rep) printf("n %d: rocsolver dpotrf %.2f ms, dpotri %.2f ms\n", n, (tp1 - tp0) * 1e3, (tp2 - tp1) * 1e3);
      // library dgemm n x n x 416 and Cholesky
      double *dinv, *ld;
      int *ci;
      hipMalloc(&dinv, (size_t)n * 64 * 8);
      hipMalloc(&ld, 8);
      hipMalloc(&ci, 4);
      hipDeviceSynchronize();
      double t8 = now();
      gmat::dgemm(0, n, 416, n, 1.0, gmat::DView{A0, n, 0}, gmat::DView{Z, 416, 0}, 0.0, E == nullptr ? A : A, 416);
      hipDeviceSynchronize();
      double t9 = now();
      hipMemcpy(A, A0, (size_t)n * n * 8, hipMemcpyDeviceToDevice);
      hipDeviceSynchronize();
      double t10 = now();
      gmat::cholesky(0, n, A, n, dinv, ld, ci);
      hipDeviceSynchronize();
      double t11 = now();
      gmat::dgemm(0, n, n, n, 1.0, gmat::DView{A0, n, 0}, gmat::DView{A0, n, 0}, 0.0, A, n);
      hipDeviceSynchronize();
      double t12 = now();
      if (rep)
        printf("n %d: dsyevd %.1f ms, ssyevd %.1f ms, dsytrd %.1f ms, ssytrd %.1f ms | dgemm nx416xn %.2f ms (%.1f TF) "
               "chol %.2f ms, dgemm n^3 %.2f ms (%.1f TF)\n",
               n, (t1 - t0) * 1e3, (t3 - t2) * 1e3, (t5 - t4) * 1e3, (t7 - t6) * 1e3, (t9 - t8) * 1e3,
               2.0 * n * n * 416 / (t9 - t8) / 1e12, (t11 - t10) * 1e3, (t12 - t11) * 1e3,
               2.0 * n * n * n / (t12 - t11) / 1e12);
      hipFree(dinv);
      hipFree(ld);
      hipFree(ci);
    }
    hipFree(A); hipFree(A0); hipFree(Z); hipFree(W); hipFree(E); hipFree(res); hipFree(info); hipFree(nev); hipFree(sweeps);
  }
  return 0;
}

// Bottom eigenpairs of a dense symmetric fp64 matrix (the scan plan's spectral setup, epi.hip).
//
// A full divide-and-conquer decomposition (rocSOLVER syevd) spends most of its time in the
// tridiagonal merge steps when the spectrum is spread, as P's is; the plan needs only the ne
// smallest pairs (ne ~ 385 of n = 2,000).  So:
//   1. Householder tridiagonalisation A = Q T Q' (rocSOLVER dsytrd, latency bound, ~35 ms at n = 2,000);
//   2. the ne smallest eigenvalues of T by Sturm-count multisection: one wave per eigenvalue, its
//      64 lanes evaluate 64 interior points of the current bracket per round (65x narrower per
//      round, 12 rounds reach the fp64 resolution), d and e^2 staged in LDS;
//   3. their eigenvectors by inverse iteration: one workgroup per eigenvalue factors T - lam I
//      with partial pivoting in LDS (the recurrence is serial; the rest of the group normalises)
//      and runs three solves from a fixed pseudo-random start;
//   4. vectors of eigenvalue clusters orthonormalised by two-pass modified Gram-Schmidt, one
//      workgroup per cluster.  Inverse iteration leaves an eigenvector with gap g to the rest of
//      the spectrum off by ~ u |T| / g, so only gaps below 1e-7 |T| (exact repeats such as P's null
//      directions, near-degenerate pairs) need it; for those the span is what the iteration
//      delivers accurately, and which basis of it comes out does not matter to the plan;
//   5. back-transformation Z = Q Y (rocSOLVER dormtr).
// The plan certifies everything it derives from these pairs with fp64 Cholesky factorisations,
// so their accuracy affects only how tight the certificates are, never correctness.
#include <rocsolver/rocsolver.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <mutex>

#include "dla.h"

namespace gmat {

namespace {

constexpr int EIG_NMAX = 10000;  // d, e^2 LDS-resident in the bisection (160 KB)
constexpr size_t LDS_MAX = 160 * 1024 - 256;  // dynamic LDS (the kernels keep a few static words)

__global__ __launch_bounds__(64) void sturm_bisect_kernel(int n, const double *__restrict__ d, const double *__restrict__ e2,
                                                          double lo0, double hi0, double pivmin, double *__restrict__ w) {
  extern __shared__ double sb[];
  double *sd = sb, *se = sb + n;
  const int lane = threadIdx.x, k = blockIdx.x;  // k-th smallest (0-based)
  for (int i = lane; i < n; i += 64) {
    sd[i] = d[i];
    se[i] = i > 0 ? e2[i - 1] : 0.0;
  }
  __syncthreads();
  double lo = lo0, hi = hi0;
  for (int round = 0; round < 12; ++round) {
    const double x = lo + (hi - lo) * (double)(lane + 1) / 65.0;
    int cnt = 0;
    double q = sd[0] - x;
    if (fabs(q) < pivmin) q = -pivmin;
    cnt += q < 0.0;
    for (int i = 1; i < n; ++i) {
      q = (sd[i] - x) - se[i] / q;
      if (fabs(q) < pivmin) q = -pivmin;
      cnt += q < 0.0;
    }
    // first lane whose point has more than k eigenvalues below it brackets lam_k from above
    const uint64_t above = __ballot(cnt > k);
    const int j = above ? __ffsll((unsigned long long)above) - 1 : 64;
    const double xl = __shfl(x, j > 0 ? j - 1 : 0), xh = __shfl(x, j < 64 ? j : 63);
    const double nlo = j > 0 ? xl : lo, nhi = j < 64 ? xh : hi;
    lo = nlo;
    hi = nhi;
  }
  if (lane == 0) w[k] = 0.5 * (lo + hi);
}

// Inverse iteration for eigenvalue w[k]: LU of T - w I with partial pivoting (in LDS, or in a
// per-eigenvalue global scratch of 5n doubles + n bytes when that exceeds the LDS), three solves
// from a fixed pseudo-random start, normalised column k of y (n x ne, column-major).
__global__ __launch_bounds__(256) void inv_iter_kernel(int n, const double *__restrict__ d, const double *__restrict__ e,
                                                       const double *__restrict__ w, double tiny, double *scratch,
                                                       double *__restrict__ y) {
  extern __shared__ double lds[];
  const int t = threadIdx.x, k = blockIdx.x;
  double *sm = scratch ? scratch + (size_t)k * (5 * (size_t)n + (n + 7) / 8) : lds;
  double *ud = sm, *u1 = sm + n, *u2 = sm + 2 * n, *lm = sm + 3 * n, *b = sm + 4 * n;
  __shared__ double red[4];
  uint8_t *piv = reinterpret_cast<uint8_t *>(sm + 5 * n);
  const double lam = w[k];
  for (int i = t; i < n; i += 256) {
    ud[i] = d[i] - lam;
    u1[i] = i + 1 < n ? e[i] : 0.0;
    lm[i] = i + 1 < n ? e[i] : 0.0;  // sub-diagonal, becomes the multipliers
    u2[i] = 0.0;
    // start vector: a fixed hash of (k, i) in [0.5, 1.5) with alternating signs
    uint32_t h = (uint32_t)i * 2654435761u ^ ((uint32_t)k * 2246822519u + 0x9e3779b9u);
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    b[i] = (0.5 + (double)(h >> 8) * (1.0 / 16777216.0)) * ((h & 1) ? -1.0 : 1.0);
  }
  __syncthreads();
  if (t == 0) {
    for (int i = 0; i + 1 < n; ++i) {
      const double sub = lm[i];
      if (fabs(ud[i]) >= fabs(sub)) {
        piv[i] = 0;
        const double dv = fabs(ud[i]) < tiny ? (ud[i] < 0.0 ? -tiny : tiny) : ud[i];
        ud[i] = dv;
        const double f = sub / dv;
        lm[i] = f;
        ud[i + 1] -= f * u1[i];
        // u2[i] stays 0
      } else {  // swap rows i and i+1
        piv[i] = 1;
        const double f = ud[i] / sub;
        ud[i] = sub;
        lm[i] = f;
        const double tmp = u1[i];
        u1[i] = ud[i + 1];
        ud[i + 1] = tmp - f * ud[i + 1];
        if (i + 2 < n) {
          u2[i] = u1[i + 1];
          u1[i + 1] = -f * u1[i + 1];
        }
      }
    }
    if (fabs(ud[n - 1]) < tiny) ud[n - 1] = ud[n - 1] < 0.0 ? -tiny : tiny;
  }
  __syncthreads();
  for (int it = 0; it < 3; ++it) {
    if (t == 0) {
      for (int i = 0; i + 1 < n; ++i) {  // L^-1 (P) b
        if (piv[i]) {
          const double tmp = b[i];
          b[i] = b[i + 1];
          b[i + 1] = tmp - lm[i] * b[i + 1];
        } else {
          b[i + 1] -= lm[i] * b[i];
        }
      }
      b[n - 1] /= ud[n - 1];  // U^-1 b
      if (n > 1) b[n - 2] = (b[n - 2] - u1[n - 2] * b[n - 1]) / ud[n - 2];
      for (int i = n - 3; i >= 0; --i) b[i] = (b[i] - u1[i] * b[i + 1] - u2[i] * b[i + 2]) / ud[i];
    }
    __syncthreads();
    double s = 0.0, mx = 0.0;
    for (int i = t; i < n; i += 256) mx = fmax(mx, fabs(b[i]));
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    const double sc = mx > 0.0 ? 1.0 / mx : 1.0;
    for (int i = t; i < n; i += 256) {
      const double v = b[i] * sc;
      b[i] = v;
      s += v * v;
    }
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if ((t & 63) == 0) red[t >> 6] = s;
    __syncthreads();
    s = red[0] + red[1] + red[2] + red[3];
    __syncthreads();
    const double r = 1.0 / sqrt(s);
    for (int i = t; i < n; i += 256) b[i] *= r;
    __syncthreads();
  }
  for (int i = t; i < n; i += 256) y[(size_t)k * n + i] = b[i];
}

__device__ double block_sum256(double v, double *red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  const double s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

// Two-pass modified Gram-Schmidt over the columns [c0, c0 + len) of y, one workgroup per cluster.
__global__ __launch_bounds__(256) void cluster_mgs_kernel(int n, const int *__restrict__ start, const int *__restrict__ len,
                                                          double *__restrict__ y) {
  __shared__ double red[4];
  const int c0 = start[blockIdx.x], L = len[blockIdx.x], t = threadIdx.x;
  for (int a = 1; a < L; ++a) {
    double *v = y + (size_t)(c0 + a) * n;
    for (int pass = 0; pass < 2; ++pass)
      for (int b = 0; b < a; ++b) {
        const double *u = y + (size_t)(c0 + b) * n;
        double p = 0.0;
        for (int i = t; i < n; i += 256) p += u[i] * v[i];
        p = block_sum256(p, red);
        for (int i = t; i < n; i += 256) v[i] -= p * u[i];
        __syncthreads();
      }
    double s = 0.0;
    for (int i = t; i < n; i += 256) s += v[i] * v[i];
    s = block_sum256(s, red);
    const double r = s > 0.0 ? 1.0 / sqrt(s) : 0.0;
    for (int i = t; i < n; i += 256) v[i] *= r;
    __syncthreads();
  }
}

}  // namespace

rocblas_handle solver_handle() {
  // created once per device and kept: creating one costs more than a decomposition at n = 2,000
  static rocblas_handle handles[64] = {nullptr};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!handles[dev] && rocblas_create_handle(&handles[dev]) != rocblas_status_success) handles[dev] = nullptr;
  return handles[dev];
}

std::mutex &solver_mutex() {
  static std::mutex mu;
  return mu;
}

int sym_eig_bottom(int64_t n, double *a, int ne, double *w_host, double *z) {
  GMAT_CHECK(n >= 2 && n <= EIG_NMAX && ne >= 1 && ne <= n, GMAT_E_ARG, "sym_eig_bottom: n %lld ne %d",
             (long long)n, ne);
  std::lock_guard<std::mutex> lock(solver_mutex());
  rocblas_handle h = solver_handle();
  GMAT_CHECK(h != nullptr, GMAT_E_HIP, "sym_eig_bottom: rocBLAS handle");
  GMAT_CHECK(rocblas_set_stream(h, 0) == rocblas_status_success, GMAT_E_HIP, "sym_eig_bottom: set stream");
  if (getenv("GMAT_EIG_SYEVD")) {  // the full divide-and-conquer decomposition (comparison path)
    DBuf W, E, info;
    GMAT_TRY(W.alloc(n * sizeof(double)));
    GMAT_TRY(E.alloc(n * sizeof(double)));
    GMAT_TRY(info.alloc(sizeof(int)));
    const rocblas_status st = rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, (rocblas_int)n, a,
                                               (rocblas_int)n, W.as<double>(), E.as<double>(), info.as<rocblas_int>());
    GMAT_CHECK(st == rocblas_status_success, GMAT_E_HIP, "sym_eig_bottom: dsyevd status %d", (int)st);
    int hinfo = 0;
    GMAT_HIP(hipMemcpy(&hinfo, info.p, sizeof(int), hipMemcpyDeviceToHost));
    GMAT_CHECK(hinfo == 0, GMAT_E_HIP, "sym_eig_bottom: dsyevd info %d", hinfo);
    GMAT_HIP(hipMemcpy(w_host, W.p, ne * sizeof(double), hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(z, a, (size_t)n * ne * sizeof(double), hipMemcpyDeviceToDevice));
    return GMAT_OK;
  }
  DBuf dd, de, dtau, de2, dw, dcl;
  GMAT_TRY(dd.alloc(n * sizeof(double)));
  GMAT_TRY(de.alloc(n * sizeof(double)));
  GMAT_TRY(dtau.alloc(n * sizeof(double)));
  GMAT_TRY(de2.alloc(n * sizeof(double)));
  GMAT_TRY(dw.alloc(ne * sizeof(double)));
  const bool dbg = getenv("GMAT_DEBUG") != nullptr;
  double tm[6] = {0, 0, 0, 0, 0, 0};
  auto mark = [&](int i) {
    if (dbg) {
      (void)hipDeviceSynchronize();
      tm[i] = std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    }
  };
  mark(0);
  const rocblas_status st = rocsolver_dsytrd(h, rocblas_fill_lower, (rocblas_int)n, a, (rocblas_int)n, dd.as<double>(),
                                             de.as<double>(), dtau.as<double>());
  GMAT_CHECK(st == rocblas_status_success, GMAT_E_HIP, "sym_eig_bottom: dsytrd status %d", (int)st);
  mark(1);
  std::vector<double> hd(n), he(n, 0.0), he2(n, 0.0);
  GMAT_HIP(hipMemcpy(hd.data(), dd.p, n * sizeof(double), hipMemcpyDeviceToHost));
  GMAT_HIP(hipMemcpy(he.data(), de.p, (n - 1) * sizeof(double), hipMemcpyDeviceToHost));
  double lo = INFINITY, hi = -INFINITY, tnorm = 0.0, emax2 = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    const double r = (i > 0 ? std::fabs(he[i - 1]) : 0.0) + (i + 1 < n ? std::fabs(he[i]) : 0.0);
    lo = std::min(lo, hd[i] - r);
    hi = std::max(hi, hd[i] + r);
    tnorm = std::max(tnorm, std::fabs(hd[i]) + r);
    if (i + 1 < n) {
      he2[i] = he[i] * he[i];
      emax2 = std::max(emax2, he2[i]);
    }
  }
  const double ulp = std::ldexp(1.0, -52);
  const double pivmin = std::max(1e-300, 1e-300 * std::max(1.0, emax2));
  lo -= 2.0 * ulp * tnorm + pivmin;
  hi += 2.0 * ulp * tnorm + pivmin;
  GMAT_HIP(hipMemcpy(de2.p, he2.data(), n * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipFuncSetAttribute((const void *)sturm_bisect_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)LDS_MAX));
  GMAT_HIP(hipFuncSetAttribute((const void *)inv_iter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX));
  hipLaunchKernelGGL(sturm_bisect_kernel, dim3(ne), dim3(64), 2 * n * sizeof(double), 0, (int)n, dd.as<double>(), de2.as<double>(), lo, hi,
                     pivmin, dw.as<double>());
  GMAT_HIP(hipGetLastError());
  mark(2);
  const size_t per = (5 * (size_t)n + (n + 7) / 8) * sizeof(double);
  DBuf scr;
  if (per > LDS_MAX) GMAT_TRY(scr.alloc(per * ne));
  hipLaunchKernelGGL(inv_iter_kernel, dim3(ne), dim3(256), per > LDS_MAX ? 0 : per, 0, (int)n, dd.as<double>(),
                     de.as<double>(), dw.as<double>(), ulp * tnorm, scr.as<double>(), z);
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpy(w_host, dw.p, ne * sizeof(double), hipMemcpyDeviceToHost));
  mark(3);
  // clusters: consecutive eigenvalues closer than 1e-7 |T|
  std::vector<int> cs, cl;
  for (int i = 0; i < ne;) {
    int j = i + 1;
    while (j < ne && w_host[j] - w_host[j - 1] <= 1e-7 * tnorm) ++j;
    if (j - i > 1) {
      cs.push_back(i);
      cl.push_back(j - i);
    }
    i = j;
  }
  if (!cs.empty()) {
    GMAT_TRY(dcl.alloc(cs.size() * 2 * sizeof(int)));
    GMAT_HIP(hipMemcpy(dcl.p, cs.data(), cs.size() * sizeof(int), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(dcl.as<int>() + cs.size(), cl.data(), cl.size() * sizeof(int), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(cluster_mgs_kernel, dim3((unsigned)cs.size()), dim3(256), 0, 0, (int)n, dcl.as<int>(),
                       dcl.as<int>() + cs.size(), z);
    GMAT_HIP(hipGetLastError());
  }
  mark(4);
  const rocblas_status so = rocsolver_dormtr(h, rocblas_side_left, rocblas_fill_lower, rocblas_operation_none,
                                             (rocblas_int)n, (rocblas_int)ne, a, (rocblas_int)n, dtau.as<double>(), z,
                                             (rocblas_int)n);
  GMAT_CHECK(so == rocblas_status_success, GMAT_E_HIP, "sym_eig_bottom: dormtr status %d", (int)so);
  GMAT_HIP(hipDeviceSynchronize());
  mark(5);
  if (dbg)
    fprintf(stderr, "sym_eig_bottom n %lld ne %d: sytrd %.1f ms, bisection %.1f, inverse iteration %.1f, clusters %zu (%.1f), "
                    "ormtr %.1f\n", (long long)n, ne, 1e3 * (tm[1] - tm[0]), 1e3 * (tm[2] - tm[1]), 1e3 * (tm[3] - tm[2]),
            cs.size(), 1e3 * (tm[4] - tm[3]), 1e3 * (tm[5] - tm[4]));
  return GMAT_OK;
}

}  // namespace gmat

// Blocked Cholesky factorisation and SPD inverse (fp64), the O(n^3) core of the REML
// iteration (replaces np.linalg.slogdet + np.linalg.inv of V at uvlmm_varcom.py:47-48 and
// scipy.linalg.inv at remma_epiAA.py:39 / gmatrix.py:84: V is symmetric positive
// definite, so L L' factorisation gives the same inverse and log-determinant).
//
// Right-looking, 64-wide panels: a one-workgroup LDS kernel factors the diagonal block
// and inverts its factor; the panel solve and the trailing update are MFMA dgemm calls.
#include "dla.h"

namespace gmat {

namespace {
constexpr int NB = 64;

// Factor the kb x kb diagonal block at a (lda) in LDS; write L back, write inv(L) to dinv
// (kb rows of NB doubles), add 2*sum(log diag) to *logdet, flag a bad pivot in *info.
__global__ __launch_bounds__(256) void potf2_kernel(int kb, double *a, int64_t lda, double *dinv,
                                                    double *logdet, int *info, int64_t k0) {
  __shared__ double s[NB][NB + 1];
  __shared__ double x[NB][NB + 1];
  __shared__ int bad;
  const int tid = threadIdx.x;
  if (tid == 0) bad = 0;
  for (int e = tid; e < NB * NB; e += 256) {
    int r = e / NB, c = e % NB;
    s[r][c] = (r < kb && c < kb && c <= r) ? a[r * lda + c] : 0.0;
    x[r][c] = 0.0;
  }
  __syncthreads();
  for (int j = 0; j < kb; ++j) {
    if (tid == 0) {
      double d = s[j][j];
      if (!(d > 0.0)) {
        bad = 1;
        d = 1.0;
      }
      s[j][j] = sqrt(d);
    }
    __syncthreads();
    const double ljj = s[j][j];
    for (int i = j + 1 + tid; i < kb; i += 256) s[i][j] /= ljj;
    __syncthreads();
    const int m = kb - j - 1;  // trailing (m x m) lower update
    for (int e = tid; e < m * m; e += 256) {
      int i = j + 1 + e / m, k = j + 1 + e % m;
      if (k <= i) s[i][k] -= s[i][j] * s[k][j];
    }
    __syncthreads();
  }
  // inverse of the lower-triangular factor, one column per thread
  if (tid < kb) {
    const int c = tid;
    x[c][c] = 1.0 / s[c][c];
    for (int i = c + 1; i < kb; ++i) {
      double acc = 0.0;
      for (int k = c; k < i; ++k) acc += s[i][k] * x[k][c];
      x[i][c] = -acc / s[i][i];
    }
  }
  __syncthreads();
  for (int e = tid; e < kb * NB; e += 256) {
    int r = e / NB, c = e % NB;
    if (c < kb) {
      a[r * lda + c] = (c <= r) ? s[r][c] : 0.0;
      dinv[r * NB + c] = x[r][c];
    } else {
      dinv[r * NB + c] = 0.0;
    }
  }
  if (tid == 0) {
    double ld = 0.0;
    for (int j = 0; j < kb; ++j) ld += log(s[j][j]);
    *logdet += 2.0 * ld;
    if (bad && *info == 0) *info = (int)(k0 + 1);
  }
}

__global__ void zero_kernel(double *p, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.0;
}

__global__ void copy_block_kernel(int kb, const double *src, double *dst, int64_t ldd) {
  int r = blockIdx.x, c = threadIdx.x;
  if (r < kb && c < kb) dst[r * ldd + c] = src[r * NB + c];
}
}  // namespace

int cholesky(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev) {
  GMAT_HIP(hipMemsetAsync(logdet_dev, 0, sizeof(double), s));
  GMAT_HIP(hipMemsetAsync(info_dev, 0, sizeof(int), s));
  for (int64_t k0 = 0; k0 < n; k0 += NB) {
    const int kb = (int)std::min<int64_t>(NB, n - k0);
    double *akk = a + k0 * lda + k0;
    hipLaunchKernelGGL(potf2_kernel, dim3(1), dim3(256), 0, s, kb, akk, lda, dinv + k0 * NB, logdet_dev, info_dev,
                       k0);
    GMAT_HIP(hipGetLastError());
    const int64_t rem = n - k0 - kb;
    if (rem <= 0) continue;
    double *panel = a + (k0 + kb) * lda + k0;
    // L21 = A21 * inv(L11)'   (in place: one 64-wide column tile per row block)
    GMAT_TRY(dgemm(s, rem, kb, kb, 1.0, DView{panel, lda, 0}, DView{dinv + k0 * NB, NB, 1}, 0.0, panel, lda));
    // A22 -= L21 L21'  (lower tiles)
    double *a22 = a + (k0 + kb) * lda + (k0 + kb);
    GMAT_TRY(dgemm(s, rem, rem, kb, -1.0, DView{panel, lda, 0}, DView{panel, lda, 1}, 1.0, a22, lda, 1));
  }
  return GMAT_OK;
}

int spd_inverse_from_chol(hipStream_t s, int64_t n, const double *l, int64_t ldl, const double *dinv, double *work,
                          double *ainv) {
  // work: n*n (Linv, lower) + NB*n (row-panel scratch)
  double *linv = work, *t = work + n * n;
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, linv, n * n);
  GMAT_HIP(hipGetLastError());
  for (int64_t i0 = 0; i0 < n; i0 += NB) {
    const int kb = (int)std::min<int64_t>(NB, n - i0);
    hipLaunchKernelGGL(copy_block_kernel, dim3(kb), dim3(NB), 0, s, kb, dinv + i0 * NB, linv + i0 * n + i0, n);
    GMAT_HIP(hipGetLastError());
    if (i0 == 0) continue;
    // T = L[i, 0:i0] * Linv[0:i0, 0:i0]
    GMAT_TRY(dgemm(s, kb, i0, i0, 1.0, DView{l + i0 * ldl, ldl, 0}, DView{linv, n, 0}, 0.0, t, i0));
    // Linv[i, 0:i0] = -inv(L_ii) * T
    GMAT_TRY(dgemm(s, kb, i0, kb, -1.0, DView{dinv + i0 * NB, NB, 0}, DView{t, i0, 0}, 0.0, linv + i0 * n, n));
  }
  // ainv = Linv' Linv (lower tiles, then mirror)
  GMAT_TRY(dgemm(s, n, n, n, 1.0, DView{linv, n, 1}, DView{linv, n, 0}, 0.0, ainv, n, 1));
  GMAT_TRY(fill_sym_upper(s, n, ainv, n));
  return GMAT_OK;
}

}  // namespace gmat

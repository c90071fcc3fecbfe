// fp64 GEMM on v_mfma_f64_16x16x4_f64 (CDNA4), LDS-staged, 64x64 tile per 256-thread
// workgroup, 4 waves each owning a 32x32 sub-tile (2 x 2 MFMA tiles), K-step 16, register
// prefetch of the next K-step while the current one is multiplied.
//
// f64 MFMA lane maps (gfx950, verified by tools/probe_mfma.hip): A: lane l holds
// A[l&15][k = l>>4]; B: B[k = l>>4][l&15]; C/D: 4 doubles per lane, element i at
// row (l>>4) + 4*i, col l&15.
#include "dla.h"

namespace gmat {

namespace {

constexpr int TM = 64, TN = 64, TK = 16;

// Loader: logical operand element (x, k) where x runs over M (for A) or N (for B).
template <class T>
struct Ld {
  const T *p;
  int64_t ld;
  int contig_k;  // storage is contiguous along k: element (x, k) at p[x*ld + k]; else p[k*ld + x]
  int64_t X, K;
  __device__ __forceinline__ double at(int64_t x, int64_t k) const {
    if (x >= X || k >= K) return 0.0;
    return contig_k ? (double)p[x * ld + k] : (double)p[k * ld + x];
  }
};

// Each thread fetches 4 elements of the 64 x 16 (x, k) tile.
template <class L>
__device__ __forceinline__ void fetch(const L &l, int64_t x0, int64_t k0, int tid, double r[4]) {
  if (l.contig_k) {
    int k = tid & 15, x = tid >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = l.at(x0 + x + 16 * q, k0 + k);
  } else {
    int x = tid & 63, k = tid >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = l.at(x0 + x, k0 + k + 4 * q);
  }
}
template <class L>
__device__ __forceinline__ void store(const L &l, double (*s)[TM + 1], int tid, const double r[4]) {
  if (l.contig_k) {
    int k = tid & 15, x = tid >> 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) s[k][x + 16 * q] = r[q];
  } else {
    int x = tid & 63, k = tid >> 6;
#pragma unroll
    for (int q = 0; q < 4; ++q) s[k + 4 * q][x] = r[q];
  }
}

template <class LA, class LB>
__global__ __launch_bounds__(256) void dgemm_kernel(int64_t M, int64_t N, int64_t K, double alpha, LA la,
                                                    LB lb, double beta, double *__restrict__ C, int64_t ldc,
                                                    int mask) {
  const int64_t bm = (int64_t)blockIdx.y * TM, bn = (int64_t)blockIdx.x * TN;
  if (mask >= 1 && blockIdx.y < blockIdx.x) return;
  __shared__ double As[2][TK][TM + 1];
  __shared__ double Bs[2][TK][TN + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  v4d acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4d{0, 0, 0, 0};

  // mask 2: both operands vanish for k < row (A' A with A lower triangular): start at the tile row
  const int kt0 = mask == 2 ? (int)(bm / TK) : 0;
  double ra[4], rb[4];
  fetch(la, bm, (int64_t)kt0 * TK, tid, ra);
  fetch(lb, bn, (int64_t)kt0 * TK, tid, rb);
  store(la, As[0], tid, ra);
  store(lb, Bs[0], tid, rb);
  __syncthreads();
  const int nk = (int)((K + TK - 1) / TK);
  for (int kt = kt0; kt < nk; ++kt) {
    const int cur = (kt - kt0) & 1;
    if (kt + 1 < nk) {
      fetch(la, bm, (int64_t)(kt + 1) * TK, tid, ra);
      fetch(lb, bn, (int64_t)(kt + 1) * TK, tid, rb);
    }
#pragma unroll
    for (int ks = 0; ks < TK / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      double a0 = As[cur][kk][wm * 32 + (lane & 15)];
      double a1 = As[cur][kk][wm * 32 + 16 + (lane & 15)];
      double b0 = Bs[cur][kk][wn * 32 + (lane & 15)];
      double b1 = Bs[cur][kk][wn * 32 + 16 + (lane & 15)];
      acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (kt + 1 < nk) {
      store(la, As[cur ^ 1], tid, ra);
      store(lb, Bs[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int64_t row = bm + wm * 32 + i * 16 + (lane >> 4) + 4 * r;
        int64_t col = bn + wn * 32 + j * 16 + (lane & 15);
        if (row < M && col < N) {
          double v = alpha * acc[i][j][r];
          if (beta != 0.0) v += beta * C[row * ldc + col];
          C[row * ldc + col] = v;
        }
      }
}

// Skinny products (N <= 8 with K >= 256, or M * N <= 64): the 64 x 64 tile grid would leave most
// of the chip idle and read A at a few hundred GB/s.  One wave per output row (A contiguous along
// k: coalesced row reads, B's N columns shared through the cache) or one thread per row (A stored
// k-major), fixed reduction order (deterministic).
template <int NC, class LA, class LB>
__global__ __launch_bounds__(256) void gemv_rows_kernel(int64_t M, int64_t K, double alpha, LA la, LB lb, double beta,
                                                        double *__restrict__ C, int64_t ldc, int64_t N) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= M) return;
  double acc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = 0.0;
  for (int64_t k = lane; k < K; k += 64) {
    const double a = la.p[r * la.ld + k];
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (j < N) acc[j] = fma(a, lb.at(j, k), acc[j]);
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    double v = acc[j];
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
    if (lane == 0 && j < N) {
      double o = alpha * v;
      if (beta != 0.0) o += beta * C[r * ldc + j];
      C[r * ldc + j] = o;
    }
  }
}
template <int NC, class LA, class LB>
__global__ __launch_bounds__(256) void gemv_cols_kernel(int64_t M, int64_t K, double alpha, LA la, LB lb, double beta,
                                                        double *__restrict__ C, int64_t ldc, int64_t N) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= M) return;
  double acc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = 0.0;
  for (int64_t k = 0; k < K; ++k) {
    const double a = la.p[k * la.ld + r];
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (j < N) acc[j] = fma(a, lb.at(j, k), acc[j]);
  }
#pragma unroll
  for (int j = 0; j < NC; ++j)
    if (j < N) {
      double o = alpha * acc[j];
      if (beta != 0.0) o += beta * C[r * ldc + j];
      C[r * ldc + j] = o;
    }
}
// M * N <= 64 outputs, long K: one workgroup per output, 256-way split of k, fixed tree.
template <class LA, class LB>
__global__ __launch_bounds__(256) void dot_kernel(int64_t M, int64_t N, int64_t K, double alpha, LA la, LB lb,
                                                  double beta, double *__restrict__ C, int64_t ldc) {
  __shared__ double red[4];
  const int64_t i = blockIdx.x / N, j = blockIdx.x % N;
  double v = 0.0;
  for (int64_t k = threadIdx.x; k < K; k += 256) v = fma(la.at(i, k), lb.at(j, k), v);
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double o = alpha * ((red[0] + red[1]) + (red[2] + red[3]));
    if (beta != 0.0) o += beta * C[i * ldc + j];
    C[i * ldc + j] = o;
  }
}

template <class LA, class LB>
int launch(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, LA la, LB lb, double beta, double *C,
           int64_t ldc, int mask) {
  if (M <= 0 || N <= 0) return GMAT_OK;
  if (mask == 0 && K >= 256 && M * N <= 64) {
    hipLaunchKernelGGL((dot_kernel<LA, LB>), dim3((unsigned)(M * N)), dim3(256), 0, s, M, N, K, alpha, la, lb, beta, C,
                       ldc);
    GMAT_HIP(hipGetLastError());
    return GMAT_OK;
  }
  if (mask == 0 && K >= 256 && N <= 8) {
    if (la.contig_k)
      hipLaunchKernelGGL((gemv_rows_kernel<8, LA, LB>), dim3((unsigned)cdiv(M, 4)), dim3(256), 0, s, M, K, alpha, la, lb,
                         beta, C, ldc, N);
    else
      hipLaunchKernelGGL((gemv_cols_kernel<8, LA, LB>), dim3((unsigned)cdiv(M, 256)), dim3(256), 0, s, M, K, alpha, la,
                         lb, beta, C, ldc, N);
    GMAT_HIP(hipGetLastError());
    return GMAT_OK;
  }
  dim3 grid((unsigned)cdiv(N, TN), (unsigned)cdiv(M, TM));
  hipLaunchKernelGGL((dgemm_kernel<LA, LB>), grid, dim3(256), 0, s, M, N, K, alpha, la, lb, beta, C, ldc, mask);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

// A logical (M x K): storage row-major unless trans.  contig along k iff !trans.
template <class T, class V>
Ld<T> loaderA(V v, int64_t M, int64_t K) { return Ld<T>{v.p, v.ld, v.trans ? 0 : 1, M, K}; }
// B logical (K x N): element (k, n) at p[k*ld + n] unless trans.  Loader indexes (n, k):
// contiguous along k iff trans.
template <class T, class V>
Ld<T> loaderB(V v, int64_t K, int64_t N) { return Ld<T>{v.p, v.ld, v.trans ? 1 : 0, N, K}; }

}  // namespace

int dgemm(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, DView A, DView B, double beta, double *C,
          int64_t ldc, int mask) {
  return launch(s, M, N, K, alpha, loaderA<double>(A, M, K), loaderB<double>(B, K, N), beta, C, ldc, mask);
}
int dgemm_i8a(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, I8View A, DView B, double beta,
              double *C, int64_t ldc) {
  return launch(s, M, N, K, alpha, loaderA<int8_t>(A, M, K), loaderB<double>(B, K, N), beta, C, ldc, 0);
}
int dgemm_i8b(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, DView A, I8View B, double beta,
              double *C, int64_t ldc) {
  return launch(s, M, N, K, alpha, loaderA<double>(A, M, K), loaderB<int8_t>(B, K, N), beta, C, ldc, 0);
}

// ------------------------------------------------------------------ small helpers

namespace {
__global__ void fill_upper_kernel(int64_t n, double *a, int64_t lda) {
  int64_t r = blockIdx.y * 16 + threadIdx.y, c = blockIdx.x * 16 + threadIdx.x;
  if (r < n && c < n && c > r) a[r * lda + c] = a[c * lda + r];
}

// out[r] = sum_k a[r,k] * b[r,k]; one wave per row, fixed lane order -> deterministic.
__global__ void dot_rows_kernel(int64_t rows, int64_t n, const double *a, int64_t lda, const double *b,
                                int64_t ldb, double *out) {
  int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  int lane = threadIdx.x & 63;
  if (r >= rows) return;
  double s = 0.0;
  for (int64_t k = lane; k < n; k += 64) s += a[r * lda + k] * (b ? b[r * ldb + k] : 1.0);
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) out[r] = s;
}
}  // namespace

int fill_sym_upper(hipStream_t s, int64_t n, double *a, int64_t lda) {
  dim3 grid((unsigned)cdiv(n, 16), (unsigned)cdiv(n, 16));
  hipLaunchKernelGGL(fill_upper_kernel, grid, dim3(16, 16), 0, s, n, a, lda);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

int dot_rows(hipStream_t s, int64_t rows, int64_t n, const double *a, int64_t lda, const double *b, int64_t ldb,
             double *out) {
  if (rows <= 0) return GMAT_OK;
  hipLaunchKernelGGL(dot_rows_kernel, dim3((unsigned)cdiv(rows, 4)), dim3(256), 0, s, rows, n, a, lda, b, ldb,
                     out);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

}  // namespace gmat

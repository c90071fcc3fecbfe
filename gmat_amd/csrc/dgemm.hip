// fp64 GEMM on v_mfma_f64_16x16x4_f64 (CDNA4), LDS-staged, 64x64 tile per 256-thread
// workgroup, 4 waves each owning a 32x32 sub-tile (2 x 2 MFMA tiles), K-step 16, register
// prefetch of the next K-step while the current one is multiplied.
//
// f64 MFMA lane maps (gfx950, verified by tools/probe_mfma.hip): A: lane l holds
// A[l&15][k = l>>4]; B: B[k = l>>4][l&15]; C/D: 4 doubles per lane, element i at
// row (l>>4) + 4*i, col l&15.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>

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

// Each thread fetches X / 16 elements of the X x 16 (x, k) tile (X = 64 or 32 rows of A, 64 of B).
template <int X, class L>
__device__ __forceinline__ void fetch(const L &l, int64_t x0, int64_t k0, int tid, double r[X / 16]) {
  if (l.contig_k) {
    int k = tid & 15, x = tid >> 4;
#pragma unroll
    for (int q = 0; q < X / 16; ++q) r[q] = l.at(x0 + x + 16 * q, k0 + k);
  } else {
    int x = tid % X, k = tid / X;
#pragma unroll
    for (int q = 0; q < X / 16; ++q) r[q] = l.at(x0 + x, k0 + k + (256 / X) * q);
  }
}
template <int X, class L>
__device__ __forceinline__ void store(const L &l, double (*s)[TM + 1], int tid, const double r[X / 16]) {
  if (l.contig_k) {
    int k = tid & 15, x = tid >> 4;
#pragma unroll
    for (int q = 0; q < X / 16; ++q) s[k][x + 16 * q] = r[q];
  } else {
    int x = tid % X, k = tid / X;
#pragma unroll
    for (int q = 0; q < X / 16; ++q) s[k + (256 / X) * q][x] = r[q];
  }
}

// TMv = 64: 64 x 64 tiles, 4 waves of 32 x 32 (2 x 2 MFMA tiles); TMv = 32: 32 x 64 tiles, 4 waves of
// 16 x 32 -- twice the workgroups for shapes whose 64 x 64 grid leaves most CUs idle (the tall-skinny
// products of the eigensolver, n x n x k with k ~ 192: 96 tiles on 256 CUs).
template <int TMv, class LA, class LB>
__global__ __launch_bounds__(256) void dgemm_kernel(int64_t M, int64_t N, int64_t K, double alpha, LA la,
                                                    LB lb, double beta, double *__restrict__ C, int64_t ldc,
                                                    int mask) {
  constexpr int MI = TMv / 32;  // 16-row MFMA blocks per wave
  const int64_t bm = (int64_t)blockIdx.y * TMv, bn = (int64_t)blockIdx.x * TN;
  if (mask >= 1 && bm + TMv - 1 < bn) return;
  // mask < 0: split-K part blockIdx.z over k in [z * kq, (z + 1) * kq), kq = -mask, written to the
  // z-th M x N partial product (C + z M ldc)
  int64_t kbeg = 0, kend = K;
  if (mask < 0) {
    kbeg = (int64_t)blockIdx.z * (int64_t)(-mask);
    kend = kbeg - mask < K ? kbeg - mask : K;
    C += (int64_t)blockIdx.z * M * ldc;
  }
  __shared__ double As[2][TK][TM + 1];
  __shared__ double Bs[2][TK][TN + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 1, wn = w & 1;
  v4d acc[MI][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = v4d{0, 0, 0, 0};

  // mask 2: both operands vanish for k < row (A' A with A lower triangular): start at the tile row
  const int kt0 = mask == 2 ? (int)(bm / TK) : (int)(kbeg / TK);
  double ra[TMv / 16], rb[4];
  fetch<TMv>(la, bm, (int64_t)kt0 * TK, tid, ra);
  fetch<64>(lb, bn, (int64_t)kt0 * TK, tid, rb);
  store<TMv>(la, As[0], tid, ra);
  store<64>(lb, Bs[0], tid, rb);
  __syncthreads();
  const int nk = (int)((kend + TK - 1) / TK);
  for (int kt = kt0; kt < nk; ++kt) {
    const int cur = (kt - kt0) & 1;
    if (kt + 1 < nk) {
      fetch<TMv>(la, bm, (int64_t)(kt + 1) * TK, tid, ra);
      fetch<64>(lb, bn, (int64_t)(kt + 1) * TK, tid, rb);
    }
#pragma unroll
    for (int ks = 0; ks < TK / 4; ++ks) {
      const int kk = ks * 4 + (lane >> 4);
      double av[MI];
#pragma unroll
      for (int i = 0; i < MI; ++i) av[i] = As[cur][kk][wm * (TMv / 2) + 16 * i + (lane & 15)];
      double b0 = Bs[cur][kk][wn * 32 + (lane & 15)];
      double b1 = Bs[cur][kk][wn * 32 + 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        acc[i][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], b0, acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[i], b1, acc[i][1], 0, 0, 0);
      }
    }
    if (kt + 1 < nk) {
      store<TMv>(la, As[cur ^ 1], tid, ra);
      store<64>(lb, Bs[cur ^ 1], tid, rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int64_t row = bm + wm * (TMv / 2) + i * 16 + (lane >> 4) + 4 * r;
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

// C = alpha sum_z P_z + beta C over the split-K partial products (fixed order: deterministic).
__global__ void splitk_sum_kernel(int64_t M, int64_t N, int splits, const double *__restrict__ ws, double alpha,
                                  double beta, double *__restrict__ C, int64_t ldc) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t r = idx / N, c = idx % N;
  double acc = 0.0;
  for (int z = 0; z < splits; ++z) acc += ws[(int64_t)z * M * N + idx];
  double v = alpha * acc;
  if (beta != 0.0) v += beta * C[r * ldc + c];
  C[r * ldc + c] = v;
}

// Split-K scratch: one grow-only buffer per (device, stream), so the partial products of successive
// products on a stream reuse it in stream order and concurrent streams never share one.  (A
// stream-ordered hipMallocAsync / hipFreeAsync pair per product on the null stream handed out
// memory that a later product's partial kernel overwrote while it was still being summed.)
int splitk_workspace(hipStream_t s, size_t bytes, double **out) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> bufs;
  int dev = 0;
  GMAT_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lock(mu);
  auto &b = bufs[{dev, s}];
  if (b.second < bytes) {
    if (b.first) {
      GMAT_HIP(hipStreamSynchronize(s));  // the old buffer may still be read by queued work
      pool_free(b.first, b.second, dev);
      b.first = nullptr;
      b.second = 0;
    }
    // through the device-memory cache (an allocation failure there trims the cache and retries)
    size_t got = 0;
    b.first = pool_alloc(std::max(bytes, (size_t)64 << 20), &got);
    if (!b.first) return GMAT_E_NOMEM;
    b.second = got;
  }
  *out = static_cast<double *>(b.first);
  return GMAT_OK;
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
  const int64_t tiles = cdiv(N, TN) * cdiv(M, TM);
  static const bool nosplit = getenv("GMAT_DGEMM_NOSPLIT") != nullptr;  // A/B diagnostics
  if (mask == 0 && tiles < 256 && K >= 1024 && !nosplit) {
    // split-K: a 64 x 64 grid that leaves most CUs idle is latency bound (one K-step of loads in
    // flight per workgroup); `splits` workgroups per tile each take a contiguous K range into their
    // own partial product (stream-ordered scratch), summed in a fixed order (deterministic)
    const int splits = (int)std::min<int64_t>(8, std::max<int64_t>(2, 768 / tiles));
    const int64_t kq = round_up(cdiv(K, splits), TK);
    const int64_t per = M * N;
    double *ws = nullptr;
    GMAT_TRY(splitk_workspace(s, (size_t)per * splits * sizeof(double), &ws));
    dim3 grid((unsigned)cdiv(N, TN), (unsigned)cdiv(M, TM), (unsigned)splits);
    hipLaunchKernelGGL((dgemm_kernel<64, LA, LB>), grid, dim3(256), 0, s, M, N, K, 1.0, la, lb, 0.0, ws, N, -(int)kq);
    hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)cdiv(per, 256)), dim3(256), 0, s, M, N, splits, ws, alpha, beta,
                       C, ldc);
    GMAT_HIP(hipGetLastError());
    return GMAT_OK;
  }
  {
    dim3 grid((unsigned)cdiv(N, TN), (unsigned)cdiv(M, TM));
    hipLaunchKernelGGL((dgemm_kernel<64, LA, LB>), grid, dim3(256), 0, s, M, N, K, alpha, la, lb, beta, C, ldc, mask);
  }
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

// Bottom eigenpairs of a dense symmetric fp64 matrix (the scan plan's spectral setup, epi.hip),
// hand-written on this library's fp64 MFMA GEMM (dgemm.hip) and Cholesky (chol.hip).
//
// The plan needs only the ne smallest pairs (ne = R + 1 = 129 of n = 2,000 by default) and
// certifies everything it derives from them with its own fp64 Cholesky factorisations, so the
// pairs' accuracy affects how tight the screens are, never correctness.  A full reduction to
// tridiagonal form is latency bound (n dependent rank-2 steps); instead, Chebyshev-filtered
// subspace iteration on a block of k ~ 4/3 ne vectors, where the n^3-class work is k-wide GEMMs:
//   1. spectrum bounds: Gershgorin's upper bound b (a true bound: the filter must damp all of
//      [cut, b]); the first cut is the mean eigenvalue trace/n;
//   2. filter: Y = T_deg((A - c)/e) X with c, e centring [cut, b] on [-1, 1] (three-term
//      recurrence, one n x n x k GEMM per degree): the eigen-directions below the cut grow by
//      T_deg(1 + 2 (cut - lam)/(b - cut)) against at most 1 for the ones above it;
//   3. orthonormalisation by Cholesky QR, twice (G = Y'Y, Y L^-T), with a shifted retry when G
//      is numerically singular;
//   4. Rayleigh-Ritz: H = Y'AY (k x k) decomposed on the device -- one workgroup reduces H to
//      tridiagonal form in LDS (Householder, packed lower triangle), Sturm multisection for its
//      eigenvalues (one wave each), inverse iteration for its eigenvectors (one workgroup each),
//      Gram-Schmidt inside clusters of near-equal eigenvalues, back-transformation by the stored
//      reflectors (one wave per vector); X = Y S;
//   5. residuals |A x_r - theta_r x_r| of the wanted pairs from W S - X Theta (W = AY); stop when
//      the largest is <= tol * b, else the next cut is the largest Ritz value (the first
//      direction the block does not hold).
// Eigenvalues come out as the Ritz values theta_r (>= the true ones), eigenvectors orthonormal.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <mutex>

#include "dla.h"

namespace gmat {

namespace {

constexpr size_t LDS_MAX = 160 * 1024 - 256;  // dynamic LDS (the kernels keep a few static words)
constexpr int TRI_LDS_K = 192;  // packed lower triangle of H (k (k+1)/2 doubles) LDS-resident up to k = 192
constexpr int TRI_THREADS = 512;
constexpr int TRI_WAVES = TRI_THREADS / 64;

__device__ __forceinline__ double wave_sum(double v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Sum over a workgroup of `waves` waves (red: >= waves doubles; two barriers).
__device__ __forceinline__ double block_sum(double v, double *red, int waves) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < waves; ++w) s += red[w];
  __syncthreads();
  return s;
}

// Gershgorin discs, one wave per row: lo[i] = a_ii - sum_j!=i |a_ij|, hi[i] = a_ii + ...
__global__ __launch_bounds__(256) void gersh_kernel(int64_t n, const double *__restrict__ a, double *__restrict__ lo,
                                                    double *__restrict__ hi) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  double s = 0.0;
  for (int64_t j = lane; j < n; j += 64)
    if (j != i) s += fabs(a[i * n + j]);
  s = wave_sum(s);
  if (lane == 0) {
    lo[i] = a[i * n + i] - s;
    hi[i] = a[i * n + i] + s;
  }
}

// Start block: a fixed hash of (row, column) in [-1, 1).
__global__ void init_block_kernel(int64_t cnt, double *__restrict__ x) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= cnt) return;
  uint64_t h = (uint64_t)idx * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;
  h ^= h >> 31;
  h *= 0xBF58476D1CE4E5B9ull;
  h ^= h >> 29;
  x[idx] = (double)(h >> 11) * (2.0 / 9007199254740992.0) - 1.0;
}

// out = alpha x + beta y (y may be null)
__global__ void axpby_kernel(int64_t cnt, double alpha, const double *__restrict__ x, double beta,
                             const double *__restrict__ y, double *__restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= cnt) return;
  out[idx] = alpha * x[idx] + (y ? beta * y[idx] : 0.0);
}

// G += shift I (k x k)
__global__ void shift_diag_kernel(int k, double *g, const double *shift) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k) g[(int64_t)i * k + i] += *shift;
}
// *shift = f * trace(G), one workgroup
__global__ __launch_bounds__(256) void trace_kernel(int k, const double *g, double f, double *shift) {
  __shared__ double red[4];
  double s = 0.0;
  for (int i = threadIdx.x; i < k; i += 256) s += g[(int64_t)i * k + i];
  s = block_sum(s, red, 4);
  if (threadIdx.x == 0) *shift = f * s;
}

__device__ __forceinline__ int pk(int i, int l) { return i * (i + 1) / 2 + l; }  // packed lower, i >= l

// Householder reduction of the symmetric k x k matrix (H + H')/2 to tridiagonal form Q T Q' in one
// workgroup.  The packed lower triangle lives in LDS (IN_LDS, k <= 192) or in global scratch.
// Step j: x = A[j+1:, j], v = x - alpha e1 (alpha = -sign(x0)|x|), tau = 2 / v'v; p = tau A22 v,
// w = p - (tau/2)(p'v) v, A22 -= v w' + w v' (one wave per row: the packed row of A22 is read along
// the row up to the diagonal and down the column after it).  Reflector j is stored as row j of V
// (v over rows j+1..k-1) with tau[j] (0: no reflection).  d, e: T's diagonal and sub-diagonal.
template <bool IN_LDS>
__global__ __launch_bounds__(TRI_THREADS) void tridiag_small_kernel(int k, const double *__restrict__ H, double *gA,
                                                                    double *__restrict__ d, double *__restrict__ e,
                                                                    double *__restrict__ V, double *__restrict__ tv) {
  extern __shared__ double lds[];
  __shared__ double red[TRI_WAVES];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double *A = IN_LDS ? lds : gA;
  double *sv = IN_LDS ? lds + (size_t)k * (k + 1) / 2 : lds, *sp = sv + k;
  for (int i = wv; i < k; i += TRI_WAVES)
    for (int l = lane; l <= i; l += 64) A[pk(i, l)] = 0.5 * (H[(int64_t)i * k + l] + H[(int64_t)l * k + i]);
  __syncthreads();
  for (int j = 0; j + 2 < k; ++j) {
    const int m = k - j - 1, r0 = j + 1;
    double s = 0.0;
    for (int q = t; q < m; q += TRI_THREADS) {
      const double x = A[pk(r0 + q, j)];
      sv[q] = x;
      s += x * x;
    }
    s = block_sum(s, red, TRI_WAVES);
    const double x0 = sv[0];
    const double sigma = s - x0 * x0;
    double tau = 0.0, alpha = x0;
    if (sigma > 0.0) {
      alpha = x0 >= 0.0 ? -sqrt(s) : sqrt(s);
      const double v0 = x0 - alpha;
      tau = 2.0 / (sigma + v0 * v0);
      __syncthreads();  // every thread has read sv[0]
      if (t == 0) sv[0] = v0;
    }
    if (t == 0) {
      d[j] = A[pk(j, j)];
      e[j] = alpha;
      tv[j] = tau;
    }
    __syncthreads();
    for (int q = t; q < m; q += TRI_THREADS) V[(int64_t)j * k + q] = tau != 0.0 ? sv[q] : 0.0;
    if (tau == 0.0) continue;
    // p = tau A22 v
    for (int r = wv; r < m; r += TRI_WAVES) {
      double acc = 0.0;
      const int gr = r0 + r;
      for (int c = lane; c < m; c += 64) {
        const int gc = r0 + c;
        acc += (c <= r ? A[pk(gr, gc)] : A[pk(gc, gr)]) * sv[c];
      }
      acc = wave_sum(acc);
      if (lane == 0) sp[r] = tau * acc;
    }
    __syncthreads();
    double pv = 0.0;
    for (int q = t; q < m; q += TRI_THREADS) pv += sp[q] * sv[q];
    pv = block_sum(pv, red, TRI_WAVES);
    const double K = 0.5 * tau * pv;
    for (int q = t; q < m; q += TRI_THREADS) sp[q] -= K * sv[q];
    __syncthreads();
    for (int r = wv; r < m; r += TRI_WAVES) {
      const double vr = sv[r], wr = sp[r];
      const int base = pk(r0 + r, r0);
      for (int c = lane; c <= r; c += 64) A[base + c] -= vr * sp[c] + wr * sv[c];
    }
    __syncthreads();
  }
  if (t == 0) {
    if (k >= 2) {
      d[k - 2] = A[pk(k - 2, k - 2)];
      e[k - 2] = A[pk(k - 1, k - 2)];
      tv[k - 2] = 0.0;
    }
    d[k - 1] = A[pk(k - 1, k - 1)];
    tv[k - 1] = 0.0;
  }
}

// The same reduction for k <= 192 with the whole (zero-padded) 192 x 192 matrix in registers: wave w
// holds columns c = w + 8 cc (cc < 24), lane l rows r = l + 64 rr (rr < 3), 72 doubles per lane, so a
// step costs straight-line FMAs and three barriers instead of packed-triangle LDS traffic.  Step j:
// the owner wave of column j (j mod 8) builds v and tau from its registers (wave reduction) and
// publishes v; every wave forms its columns' share of A v for its rows and publishes it; every lane
// then sums the eight shares of its three rows (all waves redundantly: p, K = tau/2 p'v and w = p - K v
// need no further barrier), wave 0 publishes w, and every lane applies A -= v w' + w v' to its 72
// entries.  Rows / columns <= j pick up garbage from the full-matrix update; they are never read again
// (step j + 1 reads column j + 1 below the diagonal and the diagonal entry).  v and w are double
// buffered by step parity (a wave may still be reading step j's while the owner of j + 1 writes).
constexpr int TRR_K = 192, TRR_CC = TRR_K / 8, TRR_RR = TRR_K / 64;
__global__ __launch_bounds__(512) void tridiag_reg_kernel(int k, const double *__restrict__ H, double *__restrict__ d,
                                                          double *__restrict__ e, double *__restrict__ V,
                                                          double *__restrict__ tv) {
  __shared__ double sv[2][TRR_K], sw[2][TRR_K], pp[8][TRR_K];
  __shared__ double stau[2];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double a[TRR_CC][TRR_RR];
#pragma unroll
  for (int cc = 0; cc < TRR_CC; ++cc)
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) {
      const int r = lane + 64 * rr, c = wv + 8 * cc;
      a[cc][rr] = (r < k && c < k) ? 0.5 * (H[(int64_t)r * k + c] + H[(int64_t)c * k + r]) : 0.0;
    }
  for (int j = 0; j + 2 < k; ++j) {
    const int par = j & 1, cj = j >> 3;
    double *v = sv[par], *wq = sw[par];
    if (wv == (j & 7)) {  // owner of column j: x = A[j+1:, j], v = x - alpha e_{j+1}
      double x[TRR_RR];
#pragma unroll
      for (int rr = 0; rr < TRR_RR; ++rr) x[rr] = 0.0;
#pragma unroll
      for (int cc = 0; cc < TRR_CC; ++cc)
        if (cc == cj)
#pragma unroll
          for (int rr = 0; rr < TRR_RR; ++rr) x[rr] = a[cc][rr];
      double djj = 0.0, x0 = 0.0, s = 0.0;
#pragma unroll
      for (int rr = 0; rr < TRR_RR; ++rr) {
        const int r = lane + 64 * rr;
        if (r == j) djj = x[rr];
        if (r == j + 1) x0 = x[rr];
        if (r <= j) x[rr] = 0.0;
        s += x[rr] * x[rr];
      }
      s = wave_sum(s);
      x0 = wave_sum(x0);
      djj = wave_sum(djj);
      const double sigma = s - x0 * x0;
      double tau = 0.0, alpha = x0, v0 = x0;
      if (sigma > 0.0) {
        alpha = x0 >= 0.0 ? -sqrt(s) : sqrt(s);
        v0 = x0 - alpha;
        tau = 2.0 / (sigma + v0 * v0);
      }
#pragma unroll
      for (int rr = 0; rr < TRR_RR; ++rr) {
        const int r = lane + 64 * rr;
        const double vr = tau != 0.0 ? (r == j + 1 ? v0 : x[rr]) : 0.0;
        v[r] = vr;
        if (r > j && r < k) V[(int64_t)j * k + (r - j - 1)] = vr;
      }
      if (lane == 0) {
        stau[par] = tau;
        d[j] = djj;
        e[j] = alpha;
        tv[j] = tau;
      }
    }
    __syncthreads();
    const double tau = stau[par];
    if (tau == 0.0) continue;  // uniform: nothing to reflect
    // this wave's columns' share of A v for my three rows
    double part[TRR_RR];
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) part[rr] = 0.0;
#pragma unroll
    for (int cc = 0; cc < TRR_CC; ++cc) {
      if (wv + 8 * cc <= j) continue;  // v_c = 0 (uniform)
      const double vc = v[wv + 8 * cc];
#pragma unroll
      for (int rr = 0; rr < TRR_RR; ++rr)
        if (64 * rr + 63 > j) part[rr] = fma(a[cc][rr], vc, part[rr]);
    }
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) pp[wv][lane + 64 * rr] = part[rr];
    __syncthreads();
    double pr[TRR_RR], vr[TRR_RR], pv = 0.0;
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) {
      const int r = lane + 64 * rr;
      double q = 0.0;
#pragma unroll
      for (int u = 0; u < 8; ++u) q += pp[u][r];
      pr[rr] = tau * q;
      vr[rr] = v[r];
      pv = fma(pr[rr], vr[rr], pv);
    }
    const double K = 0.5 * tau * wave_sum(pv);
    double wr[TRR_RR];
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) {
      wr[rr] = fma(-K, vr[rr], pr[rr]);
      if (wv == 0) wq[lane + 64 * rr] = wr[rr];
    }
    __syncthreads();
#pragma unroll
    for (int cc = 0; cc < TRR_CC; ++cc) {
      const int c = wv + 8 * cc;
      if (c <= j) continue;  // columns already reduced (uniform)
      const double vc = v[c], wc = wq[c];
#pragma unroll
      for (int rr = 0; rr < TRR_RR; ++rr)
        if (64 * rr + 63 > j) a[cc][rr] -= fma(vr[rr], wc, wr[rr] * vc);
    }
  }
  // the trailing 2 x 2 block: d[k-2], d[k-1], e[k-2] from their owners
#pragma unroll
  for (int cc = 0; cc < TRR_CC; ++cc)
#pragma unroll
    for (int rr = 0; rr < TRR_RR; ++rr) {
      const int r = lane + 64 * rr, c = wv + 8 * cc;
      if (k >= 2 && c == k - 2 && r == k - 2) {
        d[k - 2] = a[cc][rr];
        tv[k - 2] = 0.0;
      }
      if (k >= 2 && c == k - 2 && r == k - 1) e[k - 2] = a[cc][rr];
      if (c == k - 1 && r == k - 1) {
        d[k - 1] = a[cc][rr];
        tv[k - 1] = 0.0;
      }
    }
}

// Back-transformation for k <= 192, one wave per column: the next reflector is fetched into
// registers (3 entries per lane) while the current one is applied, and the column lives in LDS
// (a single wave: program order, no barrier).
__global__ __launch_bounds__(64) void tri_back_reg_kernel(int k, const double *__restrict__ V, const double *__restrict__ tv,
                                                          double *__restrict__ S) {
  __shared__ double col[2 * TRR_K];  // reads run up to j + 1 + 191 (masked by v = 0 past the column)
  const int lane = threadIdx.x;
  double *s = S + (int64_t)blockIdx.x * k;
  for (int i = lane; i < 2 * TRR_K; i += 64) col[i] = i < k ? s[i] : 0.0;
  double vn[TRR_RR];
  int j = k - 3;
#pragma unroll
  for (int u = 0; u < TRR_RR; ++u) vn[u] = (j >= 0 && lane + 64 * u < k - j - 1) ? V[(int64_t)j * k + lane + 64 * u] : 0.0;
  for (; j >= 0; --j) {
    double vc[TRR_RR];
#pragma unroll
    for (int u = 0; u < TRR_RR; ++u) {
      vc[u] = vn[u];
      vn[u] = (j >= 1 && lane + 64 * u < k - j) ? V[(int64_t)(j - 1) * k + lane + 64 * u] : 0.0;
    }
    const double tau = tv[j];
    double dt = 0.0;
#pragma unroll
    for (int u = 0; u < TRR_RR; ++u) dt = fma(vc[u], col[j + 1 + lane + 64 * u], dt);
    dt = tau * wave_sum(dt);
#pragma unroll
    for (int u = 0; u < TRR_RR; ++u) col[j + 1 + lane + 64 * u] -= dt * vc[u];
  }
  for (int i = lane; i < k; i += 64) s[i] = col[i];
}

// Back-transformation S := Q S for the first ncol columns (column r at S[r k ..]): reflectors
// applied last to first, one wave per column, the column in LDS.
__global__ __launch_bounds__(64) void tri_back_kernel(int k, const double *__restrict__ V, const double *__restrict__ tv,
                                                      double *__restrict__ S) {
  extern __shared__ double col[];
  const int lane = threadIdx.x;
  double *s = S + (int64_t)blockIdx.x * k;
  for (int i = lane; i < k; i += 64) col[i] = s[i];
  __syncthreads();
  for (int j = k - 3; j >= 0; --j) {
    const double tau = tv[j];
    if (tau == 0.0) continue;
    const int m = k - j - 1;
    const double *v = V + (int64_t)j * k;
    double dt = 0.0;
    for (int q = lane; q < m; q += 64) dt += v[q] * col[j + 1 + q];
    dt = tau * wave_sum(dt);
    for (int q = lane; q < m; q += 64) col[j + 1 + q] -= dt * v[q];
    __syncthreads();
  }
  for (int i = lane; i < k; i += 64) s[i] = col[i];
}

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

// Inverse iteration for eigenvalue w[k] of T: LU of T - w I with partial pivoting (in LDS, or in a
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
    double mx = 0.0;
    for (int i = t; i < n; i += 256) mx = fmax(mx, fabs(b[i]));
    for (int o = 32; o > 0; o >>= 1) mx = fmax(mx, __shfl_xor(mx, o));
    if ((t & 63) == 0) red[t >> 6] = mx;
    __syncthreads();
    mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    __syncthreads();
    const double sc = mx > 0.0 ? 1.0 / mx : 1.0;
    double s = 0.0;
    for (int i = t; i < n; i += 256) {
      const double v = b[i] * sc;
      b[i] = v;
      s += v * v;
    }
    s = block_sum(s, red, 4);
    const double r = 1.0 / sqrt(s);
    for (int i = t; i < n; i += 256) b[i] *= r;
    __syncthreads();
  }
  for (int i = t; i < n; i += 256) y[(size_t)k * n + i] = b[i];
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
        p = block_sum(p, red, 4);
        for (int i = t; i < n; i += 256) v[i] -= p * u[i];
        __syncthreads();
      }
    double s = 0.0;
    for (int i = t; i < n; i += 256) s += v[i] * v[i];
    s = block_sum(s, red, 4);
    const double r = s > 0.0 ? 1.0 / sqrt(s) : 0.0;
    for (int i = t; i < n; i += 256) v[i] *= r;
    __syncthreads();
  }
}

// res[r] = |WS[:, r] - theta_r X[:, r]| for r < ne (WS: n x ne, X: n x k, row-major), one workgroup per r.
__global__ __launch_bounds__(256) void ritz_res_kernel(int64_t n, int k, int ne, const double *__restrict__ WS,
                                                       const double *__restrict__ X, const double *__restrict__ theta,
                                                       double *__restrict__ res) {
  __shared__ double red[4];
  const int r = blockIdx.x;
  const double th = theta[r];
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const double q = WS[i * ne + r] - th * X[i * k + r];
    s += q * q;
  }
  s = block_sum(s, red, 4);
  if (threadIdx.x == 0) res[r] = sqrt(s);
}

std::mutex &eig_mutex() {
  static std::mutex mu;
  return mu;
}

// Work area of one decomposition, carved from one allocation.
struct EigWork {
  DBuf arena;
  double *X, *Y0, *Y1, *Y2, *W, *G, *Li, *dinv, *H, *V, *S, *WS, *gA;
  double *tv, *dd, *de, *de2, *th, *res, *scal;
  int *info, *cl;
  int alloc(int64_t n, int k, int ne) {
    const size_t nk = (size_t)n * k, kk = (size_t)k * k;
    const size_t doubles = 5 * nk + 5 * kk + (size_t)k * 64 + (size_t)n * ne + (k > TRI_LDS_K ? kk : 0) + 6 * (size_t)k +
                           (size_t)ne + 8;
    GMAT_TRY(arena.alloc(doubles * sizeof(double) + (2 * (size_t)k + 2) * sizeof(int) + 256));
    double *p = arena.as<double>();
    auto take = [&](size_t c) {
      double *q = p;
      p += c;
      return q;
    };
    X = take(nk), Y0 = take(nk), Y1 = take(nk), Y2 = take(nk), W = take(nk);
    G = take(kk), Li = take(kk), H = take(kk), V = take(kk), S = take(kk);
    dinv = take((size_t)k * 64);
    WS = take((size_t)n * ne);
    gA = k > TRI_LDS_K ? take(kk) : nullptr;
    tv = take(k), dd = take(k), de = take(k), de2 = take(k), th = take(k), res = take(ne + (size_t)k);
    scal = take(8);
    info = reinterpret_cast<int *>(p);
    cl = info + 2;
    return GMAT_OK;
  }
};

// Y -> Yout with orthonormal columns spanning the same space: G = Y'Y = LL', Yout = Y L^-T.  A
// numerically singular G (Cholesky breakdown) is retried with G + 1e-13 trace(G) I; the second
// pass of the caller restores orthonormality.
int chol_qr(EigWork &w, int64_t n, int k, const double *Y, double *Yout) {
  GMAT_TRY(dgemm(0, k, k, n, 1.0, DView{Y, k, 1}, DView{Y, k, 0}, 0.0, w.G, k));
  for (int attempt = 0; attempt < 3; ++attempt) {
    if (attempt > 0) {
      GMAT_TRY(dgemm(0, k, k, n, 1.0, DView{Y, k, 1}, DView{Y, k, 0}, 0.0, w.G, k));
      hipLaunchKernelGGL(trace_kernel, dim3(1), dim3(256), 0, 0, k, w.G, attempt == 1 ? 1e-13 : 1e-10, w.scal);
      hipLaunchKernelGGL(shift_diag_kernel, dim3((unsigned)cdiv(k, 256)), dim3(256), 0, 0, k, w.G, w.scal);
      GMAT_HIP(hipGetLastError());
    }
    GMAT_TRY(cholesky(0, k, w.G, k, w.dinv, w.scal + 1, w.info));
    int hinfo = 1;
    GMAT_HIP(hipMemcpy(&hinfo, w.info, sizeof(int), hipMemcpyDeviceToHost));
    if (hinfo == 0) {
      GMAT_TRY(chol_lower_inverse(0, k, w.G, k, w.dinv, w.Li));
      return dgemm(0, n, k, k, 1.0, DView{Y, k, 0}, DView{w.Li, k, 1}, 0.0, Yout, k);
    }
  }
  set_error("sym_eig_bottom: Cholesky QR of the filtered block failed");
  return GMAT_E_HIP;
}

// All eigenpairs of the symmetric k x k matrix H (device): eigenvalues ascending to th (device) and
// th_host, eigenvector r to S[r k .. r k + k).
int small_eig(EigWork &w, int k, const double *H, double *th_host) {
  const size_t tri_lds = (size_t)k * (k + 1) / 2 * sizeof(double) + 2 * (size_t)k * sizeof(double);
  if (k <= TRR_K) {
    hipLaunchKernelGGL(tridiag_reg_kernel, dim3(1), dim3(512), 0, 0, k, H, w.dd, w.de, w.V, w.tv);
  } else if (k <= TRI_LDS_K) {
    GMAT_HIP(hipFuncSetAttribute((const void *)tridiag_small_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 (int)LDS_MAX));
    hipLaunchKernelGGL(tridiag_small_kernel<true>, dim3(1), dim3(TRI_THREADS), tri_lds, 0, k, H, nullptr, w.dd, w.de,
                       w.V, w.tv);
  } else {
    hipLaunchKernelGGL(tridiag_small_kernel<false>, dim3(1), dim3(TRI_THREADS), 2 * (size_t)k * sizeof(double), 0, k, H,
                       w.gA, w.dd, w.de, w.V, w.tv);
  }
  GMAT_HIP(hipGetLastError());
  std::vector<double> hd(k), he(k, 0.0), he2(k, 0.0);
  GMAT_HIP(hipMemcpy(hd.data(), w.dd, k * sizeof(double), hipMemcpyDeviceToHost));
  if (k > 1) GMAT_HIP(hipMemcpy(he.data(), w.de, (k - 1) * sizeof(double), hipMemcpyDeviceToHost));
  double lo = INFINITY, hi = -INFINITY, tnorm = 0.0, emax2 = 0.0;
  for (int i = 0; i < k; ++i) {
    const double r = (i > 0 ? std::fabs(he[i - 1]) : 0.0) + (i + 1 < k ? std::fabs(he[i]) : 0.0);
    lo = std::min(lo, hd[i] - r);
    hi = std::max(hi, hd[i] + r);
    tnorm = std::max(tnorm, std::fabs(hd[i]) + r);
    if (i + 1 < k) {
      he2[i] = he[i] * he[i];
      emax2 = std::max(emax2, he2[i]);
    }
  }
  const double ulp = std::ldexp(1.0, -52);
  const double pivmin = std::max(1e-300, 1e-300 * std::max(1.0, emax2));
  lo -= 2.0 * ulp * tnorm + pivmin;
  hi += 2.0 * ulp * tnorm + pivmin;
  GMAT_HIP(hipMemcpy(w.de2, he2.data(), k * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(sturm_bisect_kernel, dim3(k), dim3(64), 2 * (size_t)k * sizeof(double), 0, k, w.dd, w.de2, lo, hi,
                     pivmin, w.th);
  GMAT_HIP(hipGetLastError());
  const size_t per = (5 * (size_t)k + (k + 7) / 8) * sizeof(double);
  GMAT_CHECK(per <= LDS_MAX, GMAT_E_ARG, "sym_eig_bottom: block of %d vectors too wide", k);
  GMAT_HIP(hipFuncSetAttribute((const void *)inv_iter_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_MAX));
  hipLaunchKernelGGL(inv_iter_kernel, dim3(k), dim3(256), per, 0, k, w.dd, w.de, w.th, ulp * tnorm, nullptr, w.S);
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpy(th_host, w.th, k * sizeof(double), hipMemcpyDeviceToHost));
  // clusters: consecutive eigenvalues closer than 1e-7 |T| (exact repeats: P's null directions)
  std::vector<int> cs, cl;
  for (int i = 0; i < k;) {
    int j = i + 1;
    while (j < k && th_host[j] - th_host[j - 1] <= 1e-7 * tnorm) ++j;
    if (j - i > 1) {
      cs.push_back(i);
      cl.push_back(j - i);
    }
    i = j;
  }
  if (!cs.empty()) {
    DBuf dcl;
    GMAT_TRY(dcl.alloc(cs.size() * 2 * sizeof(int)));
    GMAT_HIP(hipMemcpy(dcl.p, cs.data(), cs.size() * sizeof(int), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(dcl.as<int>() + cs.size(), cl.data(), cl.size() * sizeof(int), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(cluster_mgs_kernel, dim3((unsigned)cs.size()), dim3(256), 0, 0, k, dcl.as<int>(),
                       dcl.as<int>() + cs.size(), w.S);
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipDeviceSynchronize());
  }
  if (k <= TRR_K)
    hipLaunchKernelGGL(tri_back_reg_kernel, dim3(k), dim3(64), 0, 0, k, w.V, w.tv, w.S);
  else
    hipLaunchKernelGGL(tri_back_kernel, dim3(k), dim3(64), (size_t)k * sizeof(double), 0, k, w.V, w.tv, w.S);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

}  // namespace

int sym_eig_bottom(int64_t n, const double *a, int ne, double tol, int maxit, double *w_host, double *z, double *res_host,
                   int *iters) {
  GMAT_CHECK(n >= 2 && ne >= 1 && ne <= n && maxit >= 1, GMAT_E_ARG, "sym_eig_bottom: n %lld ne %d", (long long)n, ne);
  std::lock_guard<std::mutex> lock(eig_mutex());
  const int k = (int)std::min<int64_t>(n, round_up(ne + std::max(ne / 3, 16), 64));
  const int deg = 12;
  EigWork w;
  GMAT_TRY(w.alloc(n, k, ne));
  const bool dbg = getenv("GMAT_DEBUG") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  // spectrum bounds
  {
    hipLaunchKernelGGL(gersh_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, 0, n, a, w.Y0, w.Y1);
    GMAT_HIP(hipGetLastError());
  }
  std::vector<double> glo(n), ghi(n);
  GMAT_HIP(hipMemcpy(glo.data(), w.Y0, n * sizeof(double), hipMemcpyDeviceToHost));
  GMAT_HIP(hipMemcpy(ghi.data(), w.Y1, n * sizeof(double), hipMemcpyDeviceToHost));
  double b = -INFINITY, lo = INFINITY, tr = 0.0;
  for (int64_t i = 0; i < n; ++i) {
    b = std::max(b, ghi[i]);
    lo = std::min(lo, glo[i]);
    tr += 0.5 * (glo[i] + ghi[i]);
  }
  GMAT_CHECK(std::isfinite(b) && std::isfinite(lo), GMAT_E_ARG, "sym_eig_bottom: non-finite matrix");
  b += 1e-12 * std::max(std::fabs(b), std::fabs(lo));
  double cut = tr / (double)n;
  const int64_t nk = n * (int64_t)k;
  const unsigned gb = (unsigned)cdiv(nk, 256);
  hipLaunchKernelGGL(init_block_kernel, dim3(gb), dim3(256), 0, 0, nk, w.X);
  GMAT_HIP(hipGetLastError());
  std::vector<double> th(k), res(ne);
  // Schedule: a Rayleigh-Ritz step after the first filter pass (it sets the cut at the block's
  // largest Ritz value), then groups of RR_EVERY passes of which only the last ends in a
  // Rayleigh-Ritz step and the convergence test; the other passes only re-orthonormalise (one
  // Cholesky QR: the next filter pass and its QR absorb the loss of orthogonality).
  constexpr int RR_EVERY = 5;
  int it = 0;
  double rmax = INFINITY;
  double tm[4] = {0, 0, 0, 0};  // GMAT_DEBUG: filter, QR, Rayleigh-Ritz, residual seconds
  auto mark = [&](int ph, double t_ph) {
    if (dbg) {
      (void)hipDeviceSynchronize();
      tm[ph] += std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count() - t_ph;
    }
  };
  auto clock_now = [&]() {
    if (dbg) (void)hipDeviceSynchronize();
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
  };
  for (it = 0; it < maxit;) {
    const bool rr = it == 0 || (it % RR_EVERY) == 0 || it + 1 == maxit || k == n;
    double t_ph = clock_now();
    const double *Yf = w.X;
    if (k < n && cut < b) {  // Chebyshev filter of degree deg on [cut, b]: Y_1 = (A - c) X / e, ...
      const double c = 0.5 * (b + cut), e = 0.5 * (b - cut);
      double *buf[3] = {w.X, w.Y0, w.Y1};  // Y_{q-2}, Y_{q-1}, Y_q rotate through X, Y0, Y1
      hipLaunchKernelGGL(axpby_kernel, dim3(gb), dim3(256), 0, 0, nk, -c / e, w.X, 0.0, nullptr, buf[1]);
      GMAT_TRY(dgemm(0, n, k, n, 1.0 / e, DView{a, n, 0}, DView{w.X, k, 0}, 1.0, buf[1], k));
      for (int q = 2; q <= deg; ++q) {  // Y_q = 2 (A - c) Y_{q-1} / e - Y_{q-2}
        hipLaunchKernelGGL(axpby_kernel, dim3(gb), dim3(256), 0, 0, nk, -2.0 * c / e, buf[1], -1.0, buf[0], buf[2]);
        GMAT_TRY(dgemm(0, n, k, n, 2.0 / e, DView{a, n, 0}, DView{buf[1], k, 0}, 1.0, buf[2], k));
        double *old = buf[0];
        buf[0] = buf[1];
        buf[1] = buf[2];
        buf[2] = old;
      }
      GMAT_HIP(hipGetLastError());
      Yf = buf[1];
    }
    mark(0, t_ph);
    t_ph = clock_now();
    ++it;
    if (!rr) {  // orthonormal basis for the next pass, back in X
      GMAT_TRY(chol_qr(w, n, k, Yf, w.W));
      GMAT_HIP(hipMemcpyAsync(w.X, w.W, (size_t)nk * sizeof(double), hipMemcpyDeviceToDevice, 0));
      mark(1, t_ph);
      continue;
    }
    // orthonormal basis Yo = Y2 (Cholesky QR twice, through W), Rayleigh-Ritz
    double *Yo = w.Y2;
    GMAT_TRY(chol_qr(w, n, k, Yf, w.W));
    GMAT_TRY(chol_qr(w, n, k, w.W, Yo));
    mark(1, t_ph);
    t_ph = clock_now();
    GMAT_TRY(dgemm(0, n, k, n, 1.0, DView{a, n, 0}, DView{Yo, k, 0}, 0.0, w.W, k));
    GMAT_TRY(dgemm(0, k, k, n, 1.0, DView{Yo, k, 1}, DView{w.W, k, 0}, 0.0, w.H, k));
    GMAT_TRY(small_eig(w, k, w.H, th.data()));
    GMAT_TRY(dgemm(0, n, k, k, 1.0, DView{Yo, k, 0}, DView{w.S, k, 1}, 0.0, w.X, k));
    mark(2, t_ph);
    t_ph = clock_now();
    GMAT_TRY(dgemm(0, n, ne, k, 1.0, DView{w.W, k, 0}, DView{w.S, k, 1}, 0.0, w.WS, ne));
    hipLaunchKernelGGL(ritz_res_kernel, dim3(ne), dim3(256), 0, 0, n, k, ne, w.WS, w.X, w.th, w.res);
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpy(res.data(), w.res, ne * sizeof(double), hipMemcpyDeviceToHost));
    mark(3, t_ph);
    rmax = 0.0;
    for (int r = 0; r < ne; ++r) rmax = std::max(rmax, res[r]);
    if (dbg)
      fprintf(stderr, "sym_eig_bottom n %lld ne %d k %d: iteration %d cut %.6g b %.6g theta[ne-1] %.6g max res %.3g\n",
              (long long)n, ne, k, it, cut, b, th[ne - 1], rmax);
    if (rmax <= tol * b || k == n) break;
    cut = th[k - 1];
  }
  // z (ne x n, eigenvector r as row r) = X[:, :ne]' = S[:, :ne]' Y2'
  GMAT_TRY(dgemm(0, ne, n, k, 1.0, DView{w.S, k, 0}, DView{w.Y2, k, 1}, 0.0, z, n));
  for (int r = 0; r < ne; ++r) w_host[r] = th[r];
  if (res_host)
    for (int r = 0; r < ne; ++r) res_host[r] = res[r];
  if (iters) *iters = it;
  GMAT_HIP(hipDeviceSynchronize());
  if (dbg)
    fprintf(stderr, "sym_eig_bottom n %lld ne %d k %d: %d iterations, max res %.3g, %.1f ms (filter %.1f, QR %.1f, "
                    "Rayleigh-Ritz %.1f, residuals %.1f)\n", (long long)n, ne, k, it, rmax,
            1e3 * std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(), 1e3 * tm[0], 1e3 * tm[1],
            1e3 * tm[2], 1e3 * tm[3]);
  return GMAT_OK;
}

}  // namespace gmat

// Blocked Cholesky factorisation and SPD inverse (fp64), the O(n^3) core of the REML
// iteration (replaces np.linalg.slogdet + np.linalg.inv of V at uvlmm_varcom.py:47-48 and
// scipy.linalg.inv at remma_epiAA.py:39 / gmatrix.py:84: V is symmetric positive
// definite, so L L' factorisation gives the same inverse and log-determinant).
//
// Right-looking, 64-wide panels: a one-workgroup kernel factors the diagonal block (16-wide
// sub-panels in registers) and inverts its factor; the panel solve and the trailing update are
// MFMA dgemm calls.
#include <mutex>
#include <vector>

#include "dla.h"

namespace gmat {

namespace {
constexpr int NB = 64;

__device__ __forceinline__ double readlane_d(double v, int l) {
  union {
    double d;
    int w[2];
  } u;
  u.d = v;
  u.w[0] = __builtin_amdgcn_readlane(u.w[0], l);
  u.w[1] = __builtin_amdgcn_readlane(u.w[1], l);
  return u.d;
}

// Factor the kb x kb (kb <= 64) diagonal block at a (lda) in LDS with 4 barrier-separated
// 16-column panels (instead of one barrier group per column): wave 0 factors a panel with its rows
// in registers (pivot and the panel's column entries broadcast by readlane, no LDS round trips),
// then the four waves apply the panel to the trailing lower 16 x 16 blocks on fp64 MFMA.  inv(L)
// is blocked the same way: the four 16 x 16 diagonal inverses by forward substitution (one thread
// per column, the column in registers), then the off-diagonal blocks by distance d = i - j as two
// small MFMA products, X_ij = -X_ii (sum_{j<=k<i} L_ik X_kj).  Rows / columns >= kb are an uncoupled identity.  Writes
// L back, inv(L) to dinv (kb rows of NB doubles), adds 2 sum(log diag) to *logdet, flags a bad
// pivot's block in *info.
__global__ __launch_bounds__(256) void potf2_kernel(int kb, double *a, int64_t lda, double *dinv, double *logdet,
                                                    int *info, int64_t k0) {
  constexpr int PW = 16, NP = NB / PW;
  __shared__ double Ls[NB][NB + 1];
  __shared__ double Xs[NB][NB + 1];
  __shared__ double Ts[NP - 1][PW][PW + 1];
  __shared__ double piv[NB];  // L_jj (log-determinant summed at the end, off the pivot chain)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  {  // the block's 16 values per thread: all loads issued before the first LDS store (a load-store loop
     // waited for each load in turn: ~16 memory latencies per launch)
    double v[NB * NB / 256];
#pragma unroll
    for (int u = 0; u < NB * NB / 256; ++u) {
      const int e = tid + 256 * u, rr = e / NB, cc = e % NB;
      v[u] = (rr < kb && cc < kb) ? a[(int64_t)rr * lda + cc] : (rr == cc ? 1.0 : 0.0);
    }
#pragma unroll
    for (int u = 0; u < NB * NB / 256; ++u) {
      const int e = tid + 256 * u, rr = e / NB, cc = e % NB;
      Ls[rr][cc] = v[u];
      Xs[rr][cc] = 0.0;
    }
  }
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int c0 = PW * p;
    if (w == 0) {
      const int i = lane;
      double r[PW];
#pragma unroll
      for (int q = 0; q < PW; ++q) r[q] = Ls[i][c0 + q];
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        double d = readlane_d(r[j], c0 + j);
        if (!(d > 0.0)) {
          if (c0 + j < kb) bad = true;
          d = 1.0;
        }
        // 1/sqrt(d) from v_rsq_f64 and two Newton steps (to ~1 ulp), L_jj = d / sqrt(d)
        double inv = __builtin_amdgcn_rsq(d);
        inv = inv * fma(-0.5 * d * inv, inv, 1.5);
        inv = inv * fma(-0.5 * d * inv, inv, 1.5);
        const double ljj = d * inv;
        if (i == 0) piv[c0 + j] = (c0 + j < kb) ? ljj : 1.0;
        r[j] = (i > c0 + j) ? r[j] * inv : (i == c0 + j ? ljj : r[j]);
#pragma unroll
        for (int k = j + 1; k < PW; ++k) r[k] = fma(-r[j], readlane_d(r[j], c0 + k), r[k]);
      }
      if (i >= c0)
#pragma unroll
        for (int q = 0; q < PW; ++q) Ls[i][c0 + q] = (c0 + q <= i) ? r[q] : 0.0;
    }
    __syncthreads();
    // trailing lower blocks (bi >= bk > p) -= L_i,p L_k,p' on v_mfma_f64_16x16x4, one wave per block
    {
      const int nb = NP - 1 - p;  // block rows below the panel
      for (int blk = w; blk < nb * (nb + 1) / 2; blk += 4) {
        int bi = 0;
        while ((bi + 1) * (bi + 2) / 2 <= blk) ++bi;
        const int bk = blk - bi * (bi + 1) / 2;
        const int ri = PW * (p + 1 + bi), rk = PW * (p + 1 + bk);
        v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s4 = 0; s4 < PW / 4; ++s4) {
          const double av = Ls[ri + (lane & 15)][c0 + 4 * s4 + (lane >> 4)];
          const double bv = Ls[rk + (lane & 15)][c0 + 4 * s4 + (lane >> 4)];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) Ls[ri + (lane >> 4) + 4 * q][rk + (lane & 15)] -= acc[q];
      }
    }
    __syncthreads();
  }
  // inv(L): diagonal blocks (thread t < 64: block t / 16, column t % 16)
  if (tid < NB) {
    const int o = PW * (tid / PW), c = tid % PW;
    double x[PW];
#pragma unroll
    for (int q = 0; q < PW; ++q) {
      double sacc = 0.0;
#pragma unroll
      for (int k = 0; k < q; ++k) sacc = fma(Ls[o + q][o + k], x[k], sacc);
      const double v = (q == c) ? 1.0 : -sacc;
      // (a division, not a multiplication by 1 / L_qq: the bits of P = V^-1 .. are pinned by the
      // recorded exhaustive hit set's cohort fingerprint; the multiplication measured no faster)
      x[q] = (q >= c) ? v / Ls[o + q][o + q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < PW; ++q) Xs[o + q][o + c] = x[q];
  }
  __syncthreads();
  // off-diagonal blocks by distance d = i - j on v_mfma_f64_16x16x4 (wave j of the level):
  // T_j = sum_{k=j}^{i-1} L_ik X_kj, then X_ij = -X_ii T_j
#pragma unroll
  for (int d = 1; d < NP; ++d) {
    const int j = w, i = j + d;
    if (i < NP) {
      v4d acc = {0.0, 0.0, 0.0, 0.0};
      for (int k = j; k < i; ++k)
#pragma unroll
        for (int s4 = 0; s4 < PW / 4; ++s4) {
          const double av = Ls[PW * i + (lane & 15)][PW * k + 4 * s4 + (lane >> 4)];
          const double bv = Xs[PW * k + 4 * s4 + (lane >> 4)][PW * j + (lane & 15)];
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
        }
#pragma unroll
      for (int q = 0; q < 4; ++q) Ts[j][(lane >> 4) + 4 * q][lane & 15] = acc[q];
    }
    __syncthreads();
    if (i < NP) {
      v4d acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < PW / 4; ++s4) {
        const double av = Xs[PW * i + (lane & 15)][PW * i + 4 * s4 + (lane >> 4)];
        const double bv = Ts[j][4 * s4 + (lane >> 4)][lane & 15];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Xs[PW * i + (lane >> 4) + 4 * q][PW * j + (lane & 15)] = -acc[q];
    }
    __syncthreads();
  }
  for (int e = tid; e < kb * NB; e += 256) {
    const int r2 = e / NB, c2 = e % NB;
    if (c2 < kb) a[(int64_t)r2 * lda + c2] = Ls[r2][c2];
    dinv[r2 * NB + c2] = (c2 < kb) ? Xs[r2][c2] : 0.0;
  }
  if (w == 0) {  // sum of log L_jj over the block, one log per lane, fixed shuffle tree
    double lg = log(piv[lane]);
    for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off);
    if (lane == 0) {
      *logdet += 2.0 * lg;
      if (bad && *info == 0) *info = (int)(k0 + 1);
    }
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

// cholesky() and chol_lower_inverse() overlapped: block row i of L^-1 needs only panel i of L (its
// diagonal block's inverse and the panel below it, final once the panel solve of step i is done), so
// the inverse's step i runs on a second stream as soon as that panel is out, beside the factorisation's
// trailing update and later panels.  Both chains are dozens of small dependent launches that leave most
// CUs idle; side by side they take about the time of the longer one.  The inverse is computed even if
// a pivot fails (the caller checks *info_dev).
int cholesky_inverse(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev,
                     double *linv) {
  // Optional look-ahead (GMAT_CHOL_LOOKAHEAD): after panel k is solved, the main stream updates only
  // block column k + 1 of the trailing matrix ("narrow") and goes on to factor it, while the rest of the trailing update
  // (block columns k + 2 ..) runs on a third stream; the narrow update of step k + 1 waits for that
  // rest (both write block column k + 2).  The factorisation's critical path per step becomes potf2 +
  // panel solve + the narrow update instead of potf2 + panel solve + the whole trailing update.
  static std::mutex mu;
  static hipStream_t side[64] = {nullptr}, rest_s[64] = {nullptr};
  static std::vector<hipEvent_t> evs[64];
  int dev = 0;
  GMAT_HIP(hipGetDevice(&dev));
  GMAT_CHECK(dev >= 0 && dev < 64, GMAT_E_ARG, "cholesky_inverse: device %d", dev);
  std::lock_guard<std::mutex> lock(mu);
  if (!side[dev]) GMAT_HIP(hipStreamCreateWithFlags(&side[dev], hipStreamNonBlocking));
  if (!rest_s[dev]) GMAT_HIP(hipStreamCreateWithFlags(&rest_s[dev], hipStreamNonBlocking));
  const hipStream_t s2 = side[dev], s3 = rest_s[dev];
  const int64_t nb = cdiv(n, NB);
  // ev[0]: start, ev[1 + i]: panel i solved, ev[nb + 1]: inverse done, ev[nb + 2 + i]: rest update i done,
  // ev[2 nb + 2]: all rest updates done
  while ((int64_t)evs[dev].size() < 2 * nb + 3) {
    hipEvent_t e;
    GMAT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    evs[dev].push_back(e);
  }
  hipEvent_t *ev = evs[dev].data();
  hipEvent_t *ev_rest = ev + nb + 2;
  // (one-box A/B at n = 2,000: 2.77 ms per REML iteration with the look-ahead against 2.33 without --
  // the narrow update is as latency-bound as the whole one and the cross-stream waits add their own;
  // kept behind GMAT_CHOL_LOOKAHEAD)
  const bool lookahead = getenv("GMAT_CHOL_LOOKAHEAD") != nullptr;
  GMAT_HIP(hipMemsetAsync(logdet_dev, 0, sizeof(double), s));
  GMAT_HIP(hipMemsetAsync(info_dev, 0, sizeof(int), s));
  GMAT_HIP(hipEventRecord(ev[0], s));
  GMAT_HIP(hipStreamWaitEvent(s2, ev[0], 0));  // after the caller's earlier work on s
  GMAT_HIP(hipStreamWaitEvent(s3, ev[0], 0));
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s2, linv, n * n);
  GMAT_HIP(hipGetLastError());
  for (int64_t k0 = 0, i = 0; k0 < n; k0 += NB, ++i) {
    const int kb = (int)std::min<int64_t>(NB, n - k0);
    double *akk = a + k0 * lda + k0;
    hipLaunchKernelGGL(potf2_kernel, dim3(1), dim3(256), 0, s, kb, akk, lda, dinv + k0 * NB, logdet_dev, info_dev, k0);
    GMAT_HIP(hipGetLastError());
    const int64_t rem = n - k0 - kb;
    double *panel = a + (k0 + kb) * lda + k0;
    if (rem > 0)  // L21 = A21 * inv(L11)'
      GMAT_TRY(dgemm(s, rem, kb, kb, 1.0, DView{panel, lda, 0}, DView{dinv + k0 * NB, NB, 1}, 0.0, panel, lda));
    GMAT_HIP(hipEventRecord(ev[1 + i], s));
    // inverse step i on the side stream (chol_lower_inverse's loop body)
    GMAT_HIP(hipStreamWaitEvent(s2, ev[1 + i], 0));
    double *xi = linv + k0 * n;
    if (k0 > 0) GMAT_TRY(dgemm(s2, kb, k0, kb, 1.0, DView{dinv + k0 * NB, NB, 0}, DView{xi, n, 0}, 0.0, xi, n));
    hipLaunchKernelGGL(copy_block_kernel, dim3(kb), dim3(NB), 0, s2, kb, dinv + k0 * NB, xi + k0, n);
    GMAT_HIP(hipGetLastError());
    if (rem > 0) {
      GMAT_TRY(dgemm(s2, rem, k0 + kb, kb, -1.0, DView{a + (k0 + kb) * lda + k0, lda, 0}, DView{xi, n, 0}, 1.0,
                     linv + (k0 + kb) * n, n));
      double *a22 = a + (k0 + kb) * lda + (k0 + kb);
      const int64_t kb1 = std::min<int64_t>(NB, rem), rest = rem - kb1;
      if (!lookahead || rest <= 0) {  // A22 -= L21 L21'  (lower tiles), all on the main stream
        if (i > 0 && lookahead) GMAT_HIP(hipStreamWaitEvent(s, ev_rest[i - 1], 0));
        GMAT_TRY(dgemm(s, rem, rem, kb, -1.0, DView{panel, lda, 0}, DView{panel, lda, 1}, 1.0, a22, lda, 1));
      } else {
        // rest: block columns k + 2 .. (rows k + 2 ..) on the third stream, after panel k
        GMAT_HIP(hipStreamWaitEvent(s3, ev[1 + i], 0));
        GMAT_TRY(dgemm(s3, rest, rest, kb, -1.0, DView{panel + kb1 * lda, lda, 0}, DView{panel + kb1 * lda, lda, 1}, 1.0,
                       a22 + kb1 * lda + kb1, lda, 1));
        GMAT_HIP(hipEventRecord(ev_rest[i], s3));
        // narrow: block column k + 1 (rows k + 1 ..) on the main stream, after the previous rest (which
        // wrote this block column)
        if (i > 0) GMAT_HIP(hipStreamWaitEvent(s, ev_rest[i - 1], 0));
        GMAT_TRY(dgemm(s, rem, kb1, kb, -1.0, DView{panel, lda, 0}, DView{panel, lda, 1}, 1.0, a22, lda));
      }
    }
  }
  GMAT_HIP(hipEventRecord(ev[2 * nb + 2], s3));
  GMAT_HIP(hipStreamWaitEvent(s, ev[2 * nb + 2], 0));
  GMAT_HIP(hipEventRecord(ev[nb + 1], s2));
  GMAT_HIP(hipStreamWaitEvent(s, ev[nb + 1], 0));
  return GMAT_OK;
}

int chol_lower_inverse(hipStream_t s, int64_t n, const double *l, int64_t ldl, const double *dinv, double *linv) {
  // X = L^-1 by right-looking block forward substitution (linv: n*n, lower): block row i of X is
  // inv(L_ii) times the accumulated right-hand side, then every later block row j subtracts
  // L_ji X_i in one wide product ((n - i0) x (i0 + 64) x 64) -- the large GEMMs carry the n^3/3
  // flops instead of 64-row strips.
  hipLaunchKernelGGL(zero_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, linv, n * n);
  GMAT_HIP(hipGetLastError());
  for (int64_t i0 = 0; i0 < n; i0 += NB) {
    const int kb = (int)std::min<int64_t>(NB, n - i0);
    double *xi = linv + i0 * n;
    // X_i[:, 0:i0] = inv(L_ii) B_i[:, 0:i0]  (in place: each output tile reads only its own columns)
    if (i0 > 0) GMAT_TRY(dgemm(s, kb, i0, kb, 1.0, DView{dinv + i0 * NB, NB, 0}, DView{xi, n, 0}, 0.0, xi, n));
    hipLaunchKernelGGL(copy_block_kernel, dim3(kb), dim3(NB), 0, s, kb, dinv + i0 * NB, xi + i0, n);
    GMAT_HIP(hipGetLastError());
    const int64_t rem = n - i0 - kb;
    if (rem > 0)  // B_j -= L_ji X_i for the block rows below
      GMAT_TRY(dgemm(s, rem, i0 + kb, kb, -1.0, DView{l + (i0 + kb) * ldl + i0, ldl, 0}, DView{xi, n, 0}, 1.0,
                     linv + (i0 + kb) * n, n));
  }
  return GMAT_OK;
}

int spd_inverse_from_chol(hipStream_t s, int64_t n, const double *l, int64_t ldl, const double *dinv, double *work,
                          double *ainv) {
  double *linv = work;
  GMAT_TRY(chol_lower_inverse(s, n, l, ldl, dinv, linv));
  // ainv = Linv' Linv (lower tiles, then mirror)
  GMAT_TRY(dgemm(s, n, n, n, 1.0, DView{linv, n, 1}, DView{linv, n, 0}, 0.0, ainv, n, 2));
  GMAT_TRY(fill_sym_upper(s, n, ainv, n));
  return GMAT_OK;
}

}  // namespace gmat

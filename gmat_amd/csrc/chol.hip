// Blocked Cholesky factorisation and SPD inverse (fp64), the O(n^3) core of the REML
// iteration (replaces np.linalg.slogdet + np.linalg.inv of V at uvlmm_varcom.py:47-48 and
// scipy.linalg.inv at remma_epiAA.py:39 / gmatrix.py:84: V is symmetric positive
// definite, so L L' factorisation gives the same inverse and log-determinant).
//
// Right-looking, 64-wide panels: a one-workgroup kernel factors the diagonal block (16-wide
// sub-panels in registers) and inverts its factor; the panel solve and the trailing update are
// MFMA dgemm calls.
#include <map>
#include <mutex>
#include <vector>

#include "dla.h"

// stage timestamps for tools/chol_micro.hip (defines CHOL_STAMP before including this file)
#ifndef CHOL_STAMP
#define CHOL_STAMP(i)
#endif
#ifndef CHOL_TASK_BEGIN
#define CHOL_TASK_BEGIN
#define CHOL_TASK_END(task)
#endif

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

// v's value on lane k (0..15) of each row of 16 lanes (v_mov_b64_dpp row_newbcast; k a constant after
// unrolling)
template <int K>
__device__ __forceinline__ double bcast16_c(double v) {
  return __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xF, 0xF, true);
}
__device__ __forceinline__ double bcast16(double v, int k) {
  switch (k) {
    case 0: return bcast16_c<0>(v);
    case 1: return bcast16_c<1>(v);
    case 2: return bcast16_c<2>(v);
    case 3: return bcast16_c<3>(v);
    case 4: return bcast16_c<4>(v);
    case 5: return bcast16_c<5>(v);
    case 6: return bcast16_c<6>(v);
    case 7: return bcast16_c<7>(v);
    case 8: return bcast16_c<8>(v);
    case 9: return bcast16_c<9>(v);
    case 10: return bcast16_c<10>(v);
    case 11: return bcast16_c<11>(v);
    case 12: return bcast16_c<12>(v);
    case 13: return bcast16_c<13>(v);
    case 14: return bcast16_c<14>(v);
    default: return bcast16_c<15>(v);
  }
}

// Row block q of X = inv(L) for the 16 x 16 blocks of the NB x NB factor in Ls (L_qk, k <= q, final;
// X_kj, j <= k < q, already in Xs), computed by one wave: the diagonal block X_qq by forward substitution
// in registers -- lane (g = lane / 16, i = lane % 16) row i, columns 4c + g (c = 0..3), which is the
// v_mfma_f64_16x16x4 A-operand layout of X_qq, rows of X broadcast by row_newbcast -- then, for j = jq
// < q, X_qj = -X_qq T_j with T_j = sum_{j<=k<q} L_qk X_kj (T_j's accumulator is already the B operand of
// the second product).  Stores X_qq when diag, X_qj when jq < q.
__device__ __forceinline__ void x_row_block(const double (*Ls)[NB + 1], double (*Xs)[NB + 1], const double *ipiv, int q,
                                            int jq, bool diag) {
  constexpr int PW = 16;
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15, o = PW * q;
  double lo[PW], t[4];
#pragma unroll
  for (int m = 0; m < PW; ++m) lo[m] = (m < li) ? Ls[o + li][o + m] : 0.0;  // strictly lower row of L_qq
  const double id = ipiv[o + li];
#pragma unroll
  for (int c = 0; c < 4; ++c) t[c] = (li == 4 * c + g) ? 1.0 : 0.0;
  // row m of X_qq is t / L_mm on lane m once rows < m are subtracted; later rows subtract L_im X_m,c
  // (rows above m and the diagonal are untouched: lo is strictly lower)
#pragma unroll
  for (int m = 0; m < PW; ++m)
#pragma unroll
    for (int c = 0; c < 4; ++c) t[c] = fma(-lo[m], bcast16(t[c] * id, m), t[c]);
#pragma unroll
  for (int c = 0; c < 4; ++c) t[c] *= id;  // X_qq[li][4c + g]
  if (diag)
#pragma unroll
    for (int c = 0; c < 4; ++c) Xs[o + li][o + 4 * c + g] = t[c];
  if (jq < q) {
    const int j = jq;
    v4d acc = {0.0, 0.0, 0.0, 0.0};
    for (int k = j; k < q; ++k)
#pragma unroll
      for (int s4 = 0; s4 < PW / 4; ++s4) {
        const double av = Ls[o + li][PW * k + 4 * s4 + g];
        const double bv = Xs[PW * k + 4 * s4 + g][PW * j + li];
        acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
      }
    v4d x = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < PW / 4; ++s4) x = __builtin_amdgcn_mfma_f64_16x16x4f64(t[s4], acc[s4], x, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) Xs[o + g + 4 * r][PW * j + li] = -x[r];
  }
}

// The factor and its inverse of the NB x NB block in Ls (rows / columns >= kb already an identity), in
// place: Ls := L (lower; upper zero), Xs := inv(L), piv[j] := L_jj (1 past kb).  Returns whether a pivot
// within kb was not positive (then replaced by 1).  All 256 threads of the workgroup; ends with a barrier.
//   4 barrier-separated 16-column panels.  Wave 0 factors the whole 64-row panel in registers: lane l
//   holds its row of the panel and, in every row of 16 lanes, a copy of the panel's diagonal-block row
//   l % 16, so each pivot and each L_c0+k,j a rank-1 update needs is one row_newbcast DPP move (no
//   readlane / SGPR round trips).  Meanwhile waves 1..3 compute row block p - 1 of inv(L)
//   (x_row_block).  Then the four waves apply the panel to the trailing lower 16 x 16 blocks on fp64
//   MFMA.  Row block 3 of inv(L) after the last panel.
__device__ __forceinline__ bool factor_invert_block(double (*Ls)[NB + 1], double (*Xs)[NB + 1], double *piv, int kb) {
  constexpr int PW = 16, NP = NB / PW;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, li = lane & 15;
  bool bad = false;
  __shared__ double ipiv[NB];  // 1 / L_jj
#pragma unroll 1
  for (int p = 0; p < NP; ++p) {
    const int c0 = PW * p;
    if (w == 0) {
      double r[PW], dr[PW];
#pragma unroll
      for (int q = 0; q < PW; ++q) {
        r[q] = Ls[lane][c0 + q];
        dr[q] = Ls[c0 + li][c0 + q];
      }
      double pv = 1.0, ipv = 1.0;
#pragma unroll
      for (int j = 0; j < PW; ++j) {
        double d = bcast16(dr[j], j);
        if (!(d > 0.0)) {
          if (c0 + j < kb) bad = true;
          d = 1.0;
        }
        // 1/sqrt(d) from v_rsq_f64 and two Newton steps (to ~1 ulp), L_jj = d / sqrt(d)
        double inv = __builtin_amdgcn_rsq(d);
        inv = inv * fma(-0.5 * d * inv, inv, 1.5);
        inv = inv * fma(-0.5 * d * inv, inv, 1.5);
        if (li == j) {
          pv = d * inv;
          ipv = inv;
        }
        dr[j] *= inv;
        r[j] *= inv;
#pragma unroll
        for (int k = j + 1; k < PW; ++k) {
          const double t = bcast16(dr[j], k);  // L_c0+k,j
          dr[k] = fma(-dr[j], t, dr[k]);
          r[k] = fma(-r[j], t, r[k]);
        }
      }
      if (lane >= c0)
#pragma unroll
        for (int q = 0; q < PW; ++q) Ls[lane][c0 + q] = (c0 + q <= lane) ? r[q] : 0.0;
      if (lane < PW) {
        piv[c0 + lane] = (c0 + lane < kb) ? pv : 1.0;
        ipiv[c0 + lane] = ipv;
      }
    } else if (p > 0) {
      x_row_block(Ls, Xs, ipiv, p - 1, w - 1, w == 1);
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
    CHOL_STAMP(1 + p);
  }
  x_row_block(Ls, Xs, ipiv, NP - 1, w, w == NP - 1);
  __syncthreads();
  CHOL_STAMP(5);
  return bad;
}

// ---- One launch per 64-column step (cholesky_steps): the factorisation, the inverses of its diagonal
// blocks and optionally X = L^-1 and V^-1 = X'X, without cholesky_inverse()'s chain of small dependent
// launches (potf2, panel solve, trailing update and the inverse's two products per step, each a few
// microseconds of work behind its own launch latency).  Launch k (every task independent of the others
// in it):
//   D  (block d = k + 1): its last trailing update A_dd - L_dk L_dk', then its factor and inverse in LDS
//      (factor_invert_block): L_dd into A_dd, inv(L_dd) into dinv, 2 sum log L_jj, the pivot check;
//      launch -1 factors block 0 as it stands.  Block k + 1's factor is ready when launch k + 1 starts.
//   T1 (k < j <= i, (i, j) != (k + 1, k + 1)): A_ij -= L_ik L_jk'
//   T3 (j <= k < i, with X):                   B_ij -= L_ik X_kj     (right-looking L^-1 = X, B = I at first)
//   W  (the in-place writes of step k - 1, which launch k - 1's readers must not see):
//      L_i,k-1 = A_i,k-1 inv(L_k-1,k-1)' for i >= k, and X_k-1,j = inv(L_k-1,k-1) B_k-1,j for j <= k - 1.
//   T5 (with V^-1, row q = k - 2 of X final): V_ab += X_qa' X_qb for b <= a <= q (stored at q = a, the
//      first term; mirrored into V_ba at q = K - 1, the last).
// T1 and T3 derive the panel blocks they need, L_ik = A_ik inv(L_kk)' and X_kj = inv(L_kk) B_kj, in the
// workgroup (the same products as cholesky_inverse's panel solve and inverse step); launches K and K + 1
// do the last W and T5.  Products are 64 x 64 x 64 on v_mfma_f64_16x16x4f64 from two LDS tiles (two
// workgroups per CU); a task's global loads are all issued at its start (register-staged tiles); tiles
// past n are zero (identity on a diagonal block).
struct StepArgs {
  int64_t n, lda;
  int K, k;  // blocks; the step (-1: block 0's factor only; K, K + 1: the last writes only)
  int nD, nT1, nT3, nWL, nWX, nT5;
  bool keep_l;  // L into a (else a is scratch: the W_L tasks and D's write of L_dd are skipped)
  double *a, *linv, *dinv, *logdet, *vinv;
  int *info;
  // split steps: the panel L_ik (i > k) and X_kj (j <= k) of step k precomputed by chol_step_kernel<3>
  // into 64 x 64 tiles (tile b at b NB^2, row-major), so that a product task does one product, not three
  double *lp, *xr;
  int nPL, nPX;
};

// acc (+)= A B' for NB x NB operands in LDS (row-major, pitch NB + 1): wave w the 32 x 32 quadrant at rows
// 32 (w >> 1), columns 32 (w & 1); acc[bi][bj][q] = element (acc_row(bi, q), acc_col(bj))
__device__ __forceinline__ void mm_abt(const double (*A)[NB + 1], const double (*B)[NB + 1], v4d acc[2][2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = 32 * (w >> 1), c0 = 32 * (w & 1);
#pragma unroll 4
  for (int s4 = 0; s4 < NB / 4; ++s4) {
    const int kk = 4 * s4 + (lane >> 4);
    const double a0 = A[r0 + (lane & 15)][kk], a1 = A[r0 + 16 + (lane & 15)][kk];
    const double b0 = B[c0 + (lane & 15)][kk], b1 = B[c0 + 16 + (lane & 15)][kk];
    acc[0][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0][0], 0, 0, 0);
    acc[0][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[0][1], 0, 0, 0);
    acc[1][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[1][0], 0, 0, 0);
    acc[1][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[1][1], 0, 0, 0);
  }
}
__device__ __forceinline__ void acc_zero(v4d acc[2][2]) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) acc[bi][bj] = v4d{0.0, 0.0, 0.0, 0.0};
}
__device__ __forceinline__ int acc_row(int bi, int q) {
  return 32 * ((threadIdx.x >> 6) >> 1) + 16 * bi + ((threadIdx.x & 63) >> 4) + 4 * q;
}
__device__ __forceinline__ int acc_col(int bj) { return 32 * ((threadIdx.x >> 6) & 1) + 16 * bj + (threadIdx.x & 15); }

// an NB x NB tile staged in registers: element e = threadIdx.x + 256 u is (e / NB, e % NB)
struct TileRegs {
  double v[NB * NB / 256];
};
// the block of src at (r0, c0) (ld), rows < nr and columns < nc; elsewhere 0, or 1 on the diagonal when ident
__device__ __forceinline__ void tile_load(TileRegs &t, const double *src, int64_t ld, int64_t r0, int64_t c0, int64_t nr,
                                          int64_t nc, bool ident) {
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = threadIdx.x + 256 * u, rr = e / NB, cc = e % NB;
    t.v[u] = (rr < nr && cc < nc) ? src[(r0 + rr) * ld + c0 + cc] : ((ident && rr == cc) ? 1.0 : 0.0);
  }
}
// S = the tile (transposed when trans)
__device__ __forceinline__ void tile_to_lds(double (*S)[NB + 1], const TileRegs &t, bool trans) {
#pragma unroll
  for (int u = 0; u < NB * NB / 256; ++u) {
    const int e = threadIdx.x + 256 * u, rr = e / NB, cc = e % NB;
    if (trans)
      S[cc][rr] = t.v[u];
    else
      S[rr][cc] = t.v[u];
  }
}
// the block of src at (r0, c0) in the accumulator layout (rows < nr, columns < nc; else 0)
__device__ __forceinline__ void acc_load(v4d c[2][2], const double *src, int64_t ld, int64_t r0, int64_t c0, int64_t nr,
                                         int64_t nc) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = acc_row(bi, q), cc = acc_col(bj);
        c[bi][bj][q] = (r < nr && cc < nc) ? src[(r0 + r) * ld + c0 + cc] : 0.0;
      }
}
// S = acc (transposed when trans); the caller synchronises before and after
__device__ __forceinline__ void acc_to_lds(double (*S)[NB + 1], const v4d acc[2][2], bool trans) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = acc_row(bi, q), c = acc_col(bj);
        if (trans)
          S[c][r] = acc[bi][bj][q];
        else
          S[r][c] = acc[bi][bj][q];
      }
}
// the block of dst at (r0, c0) (ld), rows < nr, columns < nc := acc (transposed: dst at (c0, r0) gets
// element (r, c) at (c, r))
__device__ __forceinline__ void acc_store(double *dst, int64_t ld, int64_t r0, int64_t c0, int64_t nr, int64_t nc,
                                          const v4d acc[2][2], bool trans = false) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = acc_row(bi, q), c = acc_col(bj);
        if (r < nr && c < nc) {
          if (trans)
            dst[(c0 + c) * ld + r0 + r] = acc[bi][bj][q];
          else
            dst[(r0 + r) * ld + c0 + c] = acc[bi][bj][q];
        }
      }
}
__device__ __forceinline__ void acc_axpy(v4d y[2][2], double alpha, const v4d x[2][2]) {
#pragma unroll
  for (int bi = 0; bi < 2; ++bi)
#pragma unroll
    for (int bj = 0; bj < 2; ++bj) y[bi][bj] += alpha * x[bi][bj];
}

// the D task of launch k (block d = k + 1)
__device__ __forceinline__ void step_d(const StepArgs &x, double (*P0)[NB + 1], double (*P1)[NB + 1], double *piv) {
  const int64_t n = x.n, lda = x.lda;
  const int k = x.k;
  const int64_t k0 = (int64_t)k * NB;
  auto bsize = [n](int b) { return std::min<int64_t>(NB, n - (int64_t)b * NB); };
  TileRegs t0, t1;
  v4d acc[2][2], cc[2][2];
  {  // D: block d = k + 1
    const int64_t d0 = k0 + NB, nd = bsize(k + 1);
    if (k >= 0) {
      tile_load(t1, x.dinv + k0 * NB, NB, 0, 0, NB, NB, false);  // inv(L_kk), a full block (k + 1 < K)
      tile_load(t0, x.a, lda, d0, k0, nd, NB, false);            // A_dk
      acc_load(cc, x.a, lda, d0, d0, nd, nd);                    // A_dd
      tile_to_lds(P1, t1, false);
      tile_to_lds(P0, t0, false);
      __syncthreads();
      acc_zero(acc);
      mm_abt(P0, P1, acc);  // L_dk
      __syncthreads();
      acc_to_lds(P0, acc, false);
      __syncthreads();
      acc_zero(acc);
      mm_abt(P0, P0, acc);  // L_dk L_dk'
      __syncthreads();
#pragma unroll
      for (int bi = 0; bi < 2; ++bi)
#pragma unroll
        for (int bj = 0; bj < 2; ++bj)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int r = acc_row(bi, q), c = acc_col(bj);
            P0[r][c] = (r < nd && c < nd) ? cc[bi][bj][q] - acc[bi][bj][q] : (r == c ? 1.0 : 0.0);
          }
    } else {
      tile_load(t0, x.a, lda, 0, 0, nd, nd, true);
      tile_to_lds(P0, t0, false);
    }
    for (int e = threadIdx.x; e < NB * NB; e += 256) P1[e / NB][e % NB] = 0.0;
    __syncthreads();
    const bool bad = factor_invert_block(P0, P1, piv, (int)nd);
    for (int e = threadIdx.x; e < nd * NB; e += 256) {
      const int r2 = e / NB, c2 = e % NB;
      if (c2 < nd && x.keep_l) x.a[(d0 + r2) * lda + d0 + c2] = P0[r2][c2];
      x.dinv[(d0 + r2) * NB + c2] = (c2 < nd) ? P1[r2][c2] : 0.0;
    }
    if (threadIdx.x < 64) {  // 2 sum log L_jj, one log per lane, fixed shuffle tree
      double lg = log(piv[threadIdx.x]);
      for (int off = 32; off > 0; off >>= 1) lg += __shfl_xor(lg, off);
      if (threadIdx.x == 0) {
        *x.logdet += 2.0 * lg;
        if (bad && *x.info == 0) *x.info = (int)(d0 + 1);
      }
    }
  }
}

// the other tasks of launch k (T1, T3, W, T5)
__device__ __forceinline__ void step_t(const StepArgs &x, double (*P0)[NB + 1], double (*P1)[NB + 1], int task) {
  const int64_t n = x.n, lda = x.lda;
  const int k = x.k;
  const int64_t k0 = (int64_t)k * NB;
  auto bsize = [n](int b) { return std::min<int64_t>(NB, n - (int64_t)b * NB); };
  TileRegs t0, t1, t2;
  v4d acc[2][2], acc2[2][2], cc[2][2];
  if (task < x.nT1 + x.nT3) {
    int bi, bj;
    const bool t1t = task < x.nT1;
    if (t1t) {  // lower-triangle index t of the trailing blocks, row-major; t = 0 is D's block
      const int t = task + 1;
      int i = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while (i * (i + 1) / 2 > t) --i;
      while ((i + 1) * (i + 2) / 2 <= t) ++i;
      bi = k + 1 + i;
      bj = k + 1 + (t - i * (i + 1) / 2);
    } else {
      const int t = task - x.nT1;
      bi = k + 1 + t / (k + 1);
      bj = t % (k + 1);
    }
    const int64_t i0 = (int64_t)bi * NB, j0 = (int64_t)bj * NB, ni = bsize(bi), nj = bsize(bj);
    const bool two = !t1t || bj != bi;
    double *dst = t1t ? x.a : x.linv;
    const int64_t ldd = t1t ? lda : n;
    if (x.lp) {  // the panel tiles precomputed: one product
      tile_load(t0, x.lp + (int64_t)bi * NB * NB, NB, 0, 0, ni, NB, false);  // L_ik
      if (t1t) {
        if (two) tile_load(t2, x.lp + (int64_t)bj * NB * NB, NB, 0, 0, nj, NB, false);  // L_jk
      } else {
        tile_load(t2, x.xr + (int64_t)bj * NB * NB, NB, 0, 0, NB, nj, false);  // X_kj
      }
      acc_load(cc, dst, ldd, i0, j0, ni, nj);
      tile_to_lds(P0, t0, false);
      if (two) tile_to_lds(P1, t2, !t1t);  // L_jk, or X_kj'
      __syncthreads();
      acc_zero(acc);
      mm_abt(P0, two ? P1 : P0, acc);
      acc_axpy(cc, -1.0, acc);
      acc_store(dst, ldd, i0, j0, ni, nj, cc);
      return;
    }
    tile_load(t1, x.dinv + k0 * NB, NB, 0, 0, NB, NB, false);  // inv(L_kk) (k < K - 1)
    tile_load(t0, x.a, lda, i0, k0, ni, NB, false);            // A_ik
    if (t1t) {
      if (two) tile_load(t2, x.a, lda, j0, k0, nj, NB, false);  // A_jk
    } else {
      tile_load(t2, x.linv, n, k0, j0, NB, nj, false);  // B_kj
    }
    acc_load(cc, dst, ldd, i0, j0, ni, nj);  // the tile updated
    tile_to_lds(P1, t1, false);
    tile_to_lds(P0, t0, false);
    __syncthreads();
    acc_zero(acc);
    mm_abt(P0, P1, acc);  // L_ik
    if (two) {
      __syncthreads();
      tile_to_lds(P0, t2, !t1t);  // A_jk, or B_kj'
      __syncthreads();
      acc_zero(acc2);
      if (t1t)
        mm_abt(P0, P1, acc2);  // L_jk = A_jk inv(L_kk)'
      else
        mm_abt(P1, P0, acc2);  // X_kj = inv(L_kk) B_kj
    }
    __syncthreads();
    acc_to_lds(P0, acc, false);
    if (two) acc_to_lds(P1, acc2, !t1t);  // L_jk, or X_kj'
    __syncthreads();
    acc_zero(acc);
    mm_abt(P0, two ? P1 : P0, acc);
    acc_axpy(cc, -1.0, acc);
    acc_store(dst, ldd, i0, j0, ni, nj, cc);
    return;
  }
  task -= x.nT1 + x.nT3;
  if (task < x.nWL + x.nWX) {  // W: block k - 1's panel column and row of X
    const int64_t p0 = k0 - NB, np = bsize(k - 1);
    tile_load(t1, x.dinv + p0 * NB, NB, 0, 0, np, np, false);  // inv(L_k-1,k-1)
    acc_zero(acc);
    if (task < x.nWL) {  // L_i,k-1 = A_i,k-1 inv(L_k-1,k-1)', i = k + task
      const int64_t i0 = (int64_t)(k + task) * NB, ni = bsize(k + task);
      tile_load(t0, x.a, lda, i0, p0, ni, NB, false);
      tile_to_lds(P1, t1, false);
      tile_to_lds(P0, t0, false);
      __syncthreads();
      mm_abt(P0, P1, acc);
      acc_store(x.a, lda, i0, p0, ni, NB, acc);
    } else {  // X_k-1,j = inv(L_k-1,k-1) B_k-1,j
      const int j = task - x.nWL;
      const int64_t j0 = (int64_t)j * NB, nj = bsize(j);
      tile_load(t0, x.linv, n, p0, j0, np, nj, false);
      tile_to_lds(P1, t1, false);
      tile_to_lds(P0, t0, true);
      __syncthreads();
      mm_abt(P1, P0, acc);
      acc_store(x.linv, n, p0, j0, np, nj, acc);
    }
    return;
  }
  task -= x.nWL + x.nWX;
  {  // T5: V_ab += X_qa' X_qb, q = k - 2, lower-triangle index (a, b) over blocks <= q
    const int q = k - 2, K = x.K;
    int a = (int)((sqrt(8.0 * task + 1.0) - 1.0) * 0.5);
    while (a * (a + 1) / 2 > task) --a;
    while ((a + 1) * (a + 2) / 2 <= task) ++a;
    const int b = task - a * (a + 1) / 2;
    const int64_t q0 = (int64_t)q * NB, a0 = (int64_t)a * NB, b0 = (int64_t)b * NB;
    const int64_t nq = bsize(q), na = bsize(a), nb = bsize(b);
    tile_load(t0, x.linv, n, q0, a0, nq, na, false);
    tile_load(t1, x.linv, n, q0, b0, nq, nb, false);
    if (q > a)
      acc_load(cc, x.vinv, n, a0, b0, na, nb);
    else
      acc_zero(cc);
    tile_to_lds(P0, t0, true);
    tile_to_lds(P1, t1, true);
    __syncthreads();
    acc_zero(acc);
    mm_abt(P0, P1, acc);
    acc_axpy(cc, 1.0, acc);
    acc_store(x.vinv, n, a0, b0, na, nb, cc);
    if (q == K - 1 && a != b) acc_store(x.vinv, n, a0, b0, na, nb, cc, true);
  }
}

// the panel of split step k: task p < nPL: L_ik = A_ik inv(L_kk)' (i = k + 1 + p) into lp tile i; else
// X_kj = inv(L_kk) B_kj (j = p - nPL) into xr tile j -- the products the self-contained tasks derive
__device__ __forceinline__ void step_p(const StepArgs &x, double (*P0)[NB + 1], double (*P1)[NB + 1], int p) {
  const int64_t n = x.n;
  const int k = x.k;
  const int64_t k0 = (int64_t)k * NB;
  auto bsize = [n](int b) { return std::min<int64_t>(NB, n - (int64_t)b * NB); };
  TileRegs t0, t1;
  v4d acc[2][2];
  tile_load(t1, x.dinv + k0 * NB, NB, 0, 0, NB, NB, false);  // inv(L_kk)
  if (p < x.nPL) {
    const int i = k + 1 + p;
    const int64_t ni = bsize(i);
    tile_load(t0, x.a, x.lda, (int64_t)i * NB, k0, ni, NB, false);  // A_ik
    tile_to_lds(P1, t1, false);
    tile_to_lds(P0, t0, false);
    __syncthreads();
    acc_zero(acc);
    mm_abt(P0, P1, acc);
    acc_store(x.lp + (int64_t)i * NB * NB, NB, 0, 0, ni, NB, acc);
  } else {
    const int j = p - x.nPL;
    const int64_t nj = bsize(j);
    tile_load(t0, x.linv, n, k0, (int64_t)j * NB, NB, nj, false);  // B_kj
    tile_to_lds(P1, t1, false);
    tile_to_lds(P0, t0, true);
    __syncthreads();
    acc_zero(acc);
    mm_abt(P1, P0, acc);
    acc_store(x.xr + (int64_t)j * NB * NB, NB, 0, 0, NB, nj, acc);
  }
}

// ROLE 0: the D task alone (one workgroup; the 64 x 64 factor takes ~340 registers); ROLE 1: the
// product tasks alone, two workgroups per CU (188 registers); ROLE 2: both in one launch (task 0 the D
// task), one workgroup per CU.  cholesky_steps runs 0 and 1 side by side on two streams for the steps
// with many product tasks, 2 for the others; ROLE 3: the split step's panel (step_p).
template <int ROLE>
__global__ __launch_bounds__(256, ROLE == 1 || ROLE == 3 ? 2 : 1) void chol_step_kernel(StepArgs x) {
  __shared__ double P0[NB][NB + 1];
  __shared__ double P1[NB][NB + 1];
  __shared__ double piv[NB];
  CHOL_TASK_BEGIN;
  const int task = ROLE == 1 ? x.nD + (int)blockIdx.x : (int)blockIdx.x;
  if (ROLE == 3)
    step_p(x, P0, P1, task);
  else if (ROLE == 0 || (ROLE == 2 && task < x.nD))
    step_d(x, P0, P1, piv);
  else
    step_t(x, P0, P1, task - x.nD);
  CHOL_TASK_END(task);
}

__global__ void identity_kernel(double *p, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n * n) p[i] = (i / n == i % n) ? 1.0 : 0.0;
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

// The factorisation, X = L^-1 into linv (n x n) when given and V^-1 = X'X into vinv (n x n, full; needs
// linv) when given.  Step k's D task and product tasks touch disjoint blocks; D(k) needs T(k - 1) (its
// block's last updates) and T(k) needs D(k - 1) (inv(L_kk)).  A step with at least CHOL_SPLIT product
// tasks runs D (chol_step_kernel<0>) on a side stream beside its panel (<3>: L_ik and X_kj once, into
// scratch tiles) and its product tasks (<1>, two workgroups per CU, one product each instead of
// deriving their panel tiles), two events carrying the edges; the others run as one launch (<2>, or
// <1> without a D task) on s: a cross-stream edge costs ~10 us per step, which only a long product
// launch repays (REML at n = 2,000 split at every step: 1.33 -> 1.72 ms per iteration).  REML at
// n = 5,000 (5 GRMs): 11.7 ms per iteration as one launch per step, 10.3 with D beside the
// self-deriving products, 8.0 with the panel launch (same bits).
// (Threshold A/B at n = 5,000: 384 / 768 / 1,536 tasks 8.02-8.32 / 8.10-8.66 / 7.92-8.01 ms per iteration;
// at n = 2,000, 384 splits its first steps: 1.49-1.56 against 1.32-1.34 ms.)
constexpr int CHOL_SPLIT = 1536;
namespace {
// the D stream: one per device, created on first use and kept (a pooled stream would be synchronised
// by the host on release, after the whole factorisation)
int chol_side_stream(hipStream_t *out) {
  static std::mutex mu;
  static std::map<int, hipStream_t> side;
  int dev = 0;
  GMAT_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(mu);
  auto it = side.find(dev);
  if (it == side.end()) {
    hipStream_t st = nullptr;
    GMAT_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    it = side.emplace(dev, st).first;
  }
  *out = it->second;
  return GMAT_OK;
}
struct StepEvents {  // the two events of one call (per call: concurrent callers share the D stream)
  hipEvent_t ed = nullptr, et = nullptr;
  ~StepEvents() {
    if (ed) (void)hipEventDestroy(ed);
    if (et) (void)hipEventDestroy(et);
  }
};
}  // namespace

int cholesky_steps(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev,
                   double *linv, bool keep_l, double *vinv) {
  GMAT_CHECK(!vinv || linv, GMAT_E_ARG, "cholesky_steps: V^-1 needs L^-1");
  GMAT_HIP(hipMemsetAsync(logdet_dev, 0, sizeof(double), s));
  GMAT_HIP(hipMemsetAsync(info_dev, 0, sizeof(int), s));
  if (linv) {
    hipLaunchKernelGGL(identity_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, linv, n);
    GMAT_HIP(hipGetLastError());
  }
  const int K = (int)cdiv(n, NB);
  GMAT_CHECK((int64_t)K * (K + 1) / 2 < (1ll << 31), GMAT_E_ARG, "cholesky_steps: n = %lld", (long long)n);
  struct {
    hipStream_t s2 = nullptr;
    StepEvents ev;
  } ss;
  DBuf lp, xr;  // split steps' panel tiles (declared after ss: freed first, after the synchronise)
  bool d_pending = false;              // ed holds a D launch that s has not waited for
  for (int k = -1; k <= K + (vinv ? 1 : 0); ++k) {
    StepArgs x{};
    x.n = n;
    x.lda = lda;
    x.K = K;
    x.k = k;
    x.a = a;
    x.linv = linv;
    x.dinv = dinv;
    x.logdet = logdet_dev;
    x.info = info_dev;
    x.vinv = vinv;
    x.keep_l = keep_l;
    const int r = K - 1 - k;  // trailing blocks below block k
    if (k >= 0 && k < K) {
      x.nT1 = r >= 1 ? r * (r + 1) / 2 - 1 : 0;
      x.nT3 = linv ? r * (k + 1) : 0;
    }
    x.nD = k + 1 < K ? 1 : 0;
    x.nWL = (k >= 1 && k <= K && keep_l) ? K - k : 0;
    x.nWX = (k >= 1 && k <= K && linv) ? k : 0;
    const int q = k - 2;
    x.nT5 = (vinv && q >= 0 && q < K) ? (q + 1) * (q + 2) / 2 : 0;
    const int64_t grid = (int64_t)x.nT1 + x.nT3 + x.nWL + x.nWX + x.nT5;
    if (x.nD && grid >= CHOL_SPLIT) {
      // D(k) after T(k - 1) (et: everything queued on s so far) on the side stream, T(k) after D(k - 1)
      // (ed) on s; the stream and events are set up at the first split step (none at small n)
      if (!ss.s2) {
        GMAT_TRY(chol_side_stream(&ss.s2));
        GMAT_HIP(hipEventCreateWithFlags(&ss.ev.ed, hipEventDisableTiming));
        GMAT_HIP(hipEventCreateWithFlags(&ss.ev.et, hipEventDisableTiming));
      }
      GMAT_HIP(hipEventRecord(ss.ev.et, s));
      GMAT_HIP(hipStreamWaitEvent(ss.s2, ss.ev.et, 0));
      hipLaunchKernelGGL(chol_step_kernel<0>, dim3(1), dim3(256), 0, ss.s2, x);
      GMAT_HIP(hipGetLastError());
      if (d_pending) GMAT_HIP(hipStreamWaitEvent(s, ss.ev.ed, 0));
      // the panel of step k, then its product tasks with one product each
      if (!lp.p) {
        GMAT_TRY(lp.alloc((size_t)K * NB * NB * sizeof(double)));
        if (linv) GMAT_TRY(xr.alloc((size_t)K * NB * NB * sizeof(double)));
      }
      x.lp = lp.as<double>();
      x.xr = linv ? xr.as<double>() : nullptr;
      x.nPL = K - 1 - k;
      x.nPX = linv ? k + 1 : 0;
      hipLaunchKernelGGL(chol_step_kernel<3>, dim3((unsigned)(x.nPL + x.nPX)), dim3(256), 0, s, x);
      GMAT_HIP(hipGetLastError());
      hipLaunchKernelGGL(chol_step_kernel<1>, dim3((unsigned)grid), dim3(256), 0, s, x);
      GMAT_HIP(hipGetLastError());
      GMAT_HIP(hipEventRecord(ss.ev.ed, ss.s2));
      d_pending = true;
    } else if (x.nD + grid > 0) {  // one launch on s
      if (d_pending) GMAT_HIP(hipStreamWaitEvent(s, ss.ev.ed, 0));
      d_pending = false;
      if (x.nD)
        hipLaunchKernelGGL(chol_step_kernel<2>, dim3((unsigned)(x.nD + grid)), dim3(256), 0, s, x);
      else
        hipLaunchKernelGGL(chol_step_kernel<1>, dim3((unsigned)grid), dim3(256), 0, s, x);
      GMAT_HIP(hipGetLastError());
    }
  }
  if (d_pending) GMAT_HIP(hipStreamWaitEvent(s, ss.ev.ed, 0));  // the last D before s's later work
  if (lp.p) GMAT_HIP(hipStreamSynchronize(s));  // the panel scratch goes back to the pool below
  return GMAT_OK;
}

int cholesky(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev) {
  return cholesky_steps(s, n, a, lda, dinv, logdet_dev, info_dev, nullptr, true, nullptr);
}

// The factorisation and L^-1 (linv, n x n, lower) by cholesky_steps; a is scratch.  The inverse is computed
// even if a pivot fails (the caller checks *info_dev).
int cholesky_inverse(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev,
                     double *linv, double *vinv) {
  return cholesky_steps(s, n, a, lda, dinv, logdet_dev, info_dev, linv, false, vinv);
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

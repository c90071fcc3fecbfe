// fp64 dense linear algebra building blocks (device side), used by the REML, the GRM
// epilogue and the scan's exact (refine) and side-term passes.
#pragma once
#include "common.h"

namespace gmat {

// Operand views.  Element (r, c) of a logical matrix; `trans` means the storage holds the
// transpose (element (r, c) at p[c*ld + r]).
struct DView {
  const double *p;
  int64_t ld;
  int trans;
};
struct I8View {
  const int8_t *p;
  int64_t ld;
  int trans;
};

// C[M x N] = alpha * op(A)[M x K] * op(B)[K x N] + beta * C  (row-major C, ldc).
// mask: 0 = every tile, 1 = only 64x64 tiles with tile_row >= tile_col (lower half), 2 = as 1 and
// the k loop starts at the tile's first row (op(A)[r, k] = 0 for k < r: A' A with A lower).
int dgemm(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, DView A, DView B, double beta,
          double *C, int64_t ldc, int mask = 0);
// Same with an int8 A (values converted exactly to fp64).
int dgemm_i8a(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, I8View A, DView B, double beta,
              double *C, int64_t ldc);
// Same with an int8 B.
int dgemm_i8b(hipStream_t s, int64_t M, int64_t N, int64_t K, double alpha, DView A, I8View B, double beta,
              double *C, int64_t ldc);

// In-place blocked Cholesky of the lower triangle of a (n x n, ld = lda): a = L L'.
// On return the lower triangle holds L, the upper triangle is unspecified.  The inverses of
// the diagonal blocks are written to dinv (n x 64 doubles).  *logdet_dev (device double)
// receives sum(log(diag(L)))*2; *info_dev (device int) > 0 marks a non-positive pivot.
int cholesky(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev);
// cholesky() and, when linv is given, L^-1 (n x n, lower; upper zero) as one launch per 64-column step
// (chol.hip chol_step_kernel).  keep_l: L into a's lower triangle (upper unspecified), else a is scratch.
// vinv (needs linv): V^-1 = L^-T L^-1, n x n, both triangles.
int cholesky_steps(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev,
                   double *linv, bool keep_l = true, double *vinv = nullptr);
// L^-1 into linv, optionally A^-1 into vinv (both triangles), log|A| and the pivot check, a used as
// scratch (cholesky_steps); ordered after the caller's earlier work on s.
int cholesky_inverse(hipStream_t s, int64_t n, double *a, int64_t lda, double *dinv, double *logdet_dev, int *info_dev,
                     double *linv, double *vinv = nullptr);
// linv = L^-1 (n x n, lower triangle; the upper triangle is zeroed) from the factor and its
// diagonal-block inverses.
int chol_lower_inverse(hipStream_t s, int64_t n, const double *l, int64_t ldl, const double *dinv, double *linv);
// ainv = (L L')^-1 from the factor (lower triangle of l) and its diagonal-block inverses;
// work is n*n doubles of scratch.  ainv is fully populated (symmetric).
int spd_inverse_from_chol(hipStream_t s, int64_t n, const double *l, int64_t ldl, const double *dinv,
                          double *work, double *ainv);

// The ne smallest eigenpairs of the symmetric n x n matrix a (device, both triangles, row-major,
// not modified), by Chebyshev-filtered subspace iteration (eig.hip): Ritz values ascending to
// w_host, Ritz vector r to z[r*n .. r*n+n) (device, orthonormal); iterates until every pair's
// residual |a z_r - w_r z_r| is <= tol * (Gershgorin bound of |a|) or maxit block iterations.
// res_host (ne residual norms) and iters may be null.  Synchronous.
int sym_eig_bottom(int64_t n, const double *a, int ne, double tol, int maxit, double *w_host, double *z,
                   double *res_host, int *iters);

// Small device helpers.
int fill_sym_upper(hipStream_t s, int64_t n, double *a, int64_t lda);           // upper := lower'
int dot_rows(hipStream_t s, int64_t rows, int64_t n, const double *a, int64_t lda, const double *b,
             int64_t ldb, double *out);  // out[r] = sum_k a[r,k] * b[r,k]  (b==NULL -> vector of ones)

}  // namespace gmat

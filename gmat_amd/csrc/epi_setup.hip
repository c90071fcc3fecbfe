// Plan-setup and coding kernels (see epi.h for the stage files).
#include "epi.h"

namespace gmat {
namespace epi {

// P_store[q][q'] = P[nat(q)][nat(q')], zero padded; z = P_store 1 computed later.
__global__ void permute_p_kernel(int64_t n, int64_t n_pad, const double *P, double *Ps) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t q = idx / n_pad, q2 = idx % n_pad;
  const int64_t r = (q & ~31LL) + perm_nat((int)(q & 31)), c = (q2 & ~31LL) + perm_nat((int)(q2 & 31));
  Ps[idx] = (r < n && c < n) ? P[r * n + c] : 0.0;
}

__global__ void permute_vec_kernel(int64_t n, int64_t n_pad, const double *v, double *vs) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_pad) return;
  const int64_t r = (q & ~31LL) + perm_nat((int)(q & 31));
  vs[q] = (r < n) ? v[r] : 0.0;
}

// slices A_s[rho][t] (rho natural row, t storage column) of P_off*127/qmax (zero diagonal:
// the diagonal enters the screen exactly, as a side term)
__global__ void slice_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                             int8_t *slices) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t rho = idx / n_pad, t = idx % n_pad;
  const int64_t c = (t & ~31LL) + perm_nat((int)(t & 31));
  double r = (rho < n && c < n && rho != c) ? P[rho * n + c] * inv_unit : 0.0;
  for (int s = 0; s < n_slice; ++s) {
    const double q = rint(r);
    slices[(int64_t)s * n_pad * n_pad + idx] = (int8_t)q;
    r = (r - q) * 128.0;
  }
}

// residual of the slicing, R = P_off - P~ (natural order, zero padded and zero diagonal), scaled
__global__ void residual_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                                double out_scale, double *R) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t r0 = idx / n_pad, c0 = idx % n_pad;
  double r = (r0 < n && c0 < n && r0 != c0) ? P[r0 * n + c0] * inv_unit : 0.0;
  for (int s = 0; s < n_slice; ++s) r = (r - rint(r)) * 128.0;
  R[idx] = r * out_scale;
}

// per-SNP side vectors for the left coding: L' = a o (u - alpha z), L3 = a o py,
// Ld = diag(P) o a o a, and scalars qa = a.u, ra = a.z, sa = a.py.  One workgroup per SNP.
__global__ __launch_bounds__(256) void left_side_kernel(int64_t n_pad, const int8_t *panel, const double *U,
                                                        const double *z, const double *py, const double *dg,
                                                        const double *alpha, double *Lp, double *L3, double *Ld,
                                                        double *qa, double *ra, double *sa) {
  const int64_t j = blockIdx.x;
  const double al = alpha[j];
  double s1 = 0, s2 = 0, s3 = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const double av = (double)panel[j * n_pad + q];
    const double u = U[j * n_pad + q];
    if (Lp) Lp[j * n_pad + q] = av * (u - al * z[q]);  // Lp, Ld: the block-granular screens only
    if (L3) L3[j * n_pad + q] = av * py[q];
    if (Ld) Ld[j * n_pad + q] = av * av * dg[q];
    s1 += av * u;
    s2 += av * z[q];
    s3 += av * py[q];
  }
  __shared__ double red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    s3 += __shfl_xor(s3, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
    red[2][threadIdx.x >> 6] = s3;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    qa[j] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    ra[j] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    sa[j] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
  }
}

// right coding: R' = (b - beta) o v, qb = b.v, rb = b.z, sb = b.py
__global__ __launch_bounds__(256) void right_side_kernel(int64_t n_pad, const int8_t *panel, const double *V,
                                                         const double *z, const double *py, const double *beta,
                                                         double *Rp, double *qb, double *rb, double *sb) {
  const int64_t j = blockIdx.x;
  const double be = beta[j];
  double s1 = 0, s2 = 0, s3 = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const double bv = (double)panel[j * n_pad + q];
    const double v = V[j * n_pad + q];
    if (Rp) Rp[j * n_pad + q] = (bv - be) * v;
    s1 += bv * v;
    s2 += bv * z[q];
    s3 += bv * py[q];
  }
  __shared__ double red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    s3 += __shfl_xor(s3, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
    red[2][threadIdx.x >> 6] = s3;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    qb[j] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    rb[j] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    sb[j] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
  }
}

// Per-row int8 slices of an fp64 [rows][n_pad] matrix: v = s (sum_{t<T} 128^-t Q_t + r) with
// s = max|v|/127, |Q_0| <= 127, |Q_t| <= 64, |r| <= 0.5 * 128^-(T-1) (+ fp64 rounding).
__global__ __launch_bounds__(256) void quantize_rows_kernel(int64_t n_pad, int64_t slice_stride, const double *v,
                                                            int8_t *q, double *scale) {
  const int64_t j = blockIdx.x;
  const double *row = v + j * n_pad;
  double mx = 0.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) mx = fmax(mx, fabs(row[k]));
  for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double s = mx / 127.0, inv = mx > 0.0 ? 127.0 / mx : 0.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) {
    double r = row[k] * inv;
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t) {
      const double qv = rint(r);
      q[t * slice_stride + j * n_pad + k] = (int8_t)qv;
      r = (r - qv) * 128.0;
    }
  }
  if (threadIdx.x == 0) scale[j] = s;
}

// gather band rows of the int8 side slices: BL[t][r] = Lq[t][rows[r]], BL[t][R+r] = L3q[t][rows[r]],
// BL[t][2R+r] = Ldq[t][rows[r]], BA[r] = panel[rows[r]], BA[R+r] = sqpanel[rows[r]] (squared codes)
__global__ void gather_band_kernel(int64_t n_pad, int R, int64_t slice_stride, const int64_t *rows, const int8_t *Lq,
                                   const int8_t *L3q, const int8_t *Ldq, const int8_t *panel, const int8_t *sqpanel,
                                   int8_t *BL, int8_t *BA) {
  const int r = blockIdx.x;
  const int64_t src = rows[r];
  for (int64_t q = threadIdx.x * 16; q < n_pad; q += blockDim.x * 16) {
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t) {
      const int64_t o = (int64_t)t * SIDE_P * R + r, so = t * slice_stride + src * n_pad + q;
      *(v4i *)&BL[o * n_pad + q] = *(const v4i *)&Lq[so];
      *(v4i *)&BL[(o + R) * n_pad + q] = *(const v4i *)&L3q[so];
      *(v4i *)&BL[(o + 2 * R) * n_pad + q] = *(const v4i *)&Ldq[so];
    }
    *(v4i *)&BA[(int64_t)r * n_pad + q] = *(const v4i *)&panel[src * n_pad + q];
    *(v4i *)&BA[(int64_t)(R + r) * n_pad + q] = *(const v4i *)&sqpanel[src * n_pad + q];
  }
}

__global__ __launch_bounds__(256) void i8gemm_nt_kernel(int M, int N, int K, const int8_t *__restrict__ A, int64_t lda,
                                                        int64_t za, const int8_t *__restrict__ B, int64_t ldb,
                                                        int64_t zb, int *__restrict__ C, int64_t ldc, int64_t zc) {
  A += blockIdx.z * za;
  B += blockIdx.z * zb;
  C += blockIdx.z * zc;
  const int m0 = blockIdx.y * GM, n0 = blockIdx.x * GN;
  __shared__ __attribute__((aligned(16))) int8_t sa[GM * GPI];
  __shared__ __attribute__((aligned(16))) int8_t sb[GN * GPI];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
  v16i acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0;
  const int ar = tid >> 2, c16 = (tid & 3) * 16;
  const v4i zero = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += GKK) {
    *(v4i *)&sa[ar * GPI + c16] = (m0 + ar < M) ? *(const v4i *)&A[(int64_t)(m0 + ar) * lda + k0 + c16] : zero;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int br = ar + 64 * u;
      *(v4i *)&sb[br * GPI + c16] = (n0 + br < N) ? *(const v4i *)&B[(int64_t)(n0 + br) * ldb + k0 + c16] : zero;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i fa = *(const v4i *)&sa[(wr * 32 + (lane & 31)) * GPI + kk * 32 + (lane >> 5) * 16];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const v4i fb = *(const v4i *)&sb[(wc * 64 + t * 32 + (lane & 31)) * GPI + kk * 32 + (lane >> 5) * 16];
        acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = m0 + wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int col = n0 + wc * 64 + t * 32 + (lane & 31);
      if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[t][e];
    }
}

// screen panel of the additive coding: minor-allele dosage a~ = flip ? 2 - a : a (padding stays
// 0), and its square a~^2 in {0, 1, 4}
__global__ void flip_panel_kernel(int64_t n, int64_t n_pad, int64_t m, const int8_t *src, const uint8_t *flip,
                                  int8_t *dst, int8_t *sq) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * n_pad) return;
  const int64_t j = idx / n_pad, q = idx % n_pad;
  const int64_t nat = (q & ~31LL) + perm_nat((int)(q & 31));
  const int a = src[idx];
  const int v = (flip[j] && nat < n) ? 2 - a : a;
  dst[idx] = (int8_t)v;
  sq[idx] = (int8_t)(v * v);
}

__global__ void diag_kernel(int64_t n_pad, const double *Ps, double *dg) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n_pad) dg[q] = Ps[q * n_pad + q];
}

__global__ void zsum_kernel(int64_t n_pad, const double *Ps, double *z) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= n_pad) return;
  double s = 0.0;
  for (int64_t k = lane; k < n_pad; k += 64) s += Ps[q * n_pad + k];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) z[q] = s;
}

__global__ void mx_quant_kernel(int64_t n, int64_t n_pad, int nK, const double *P, uint32_t *tiles, double *Qn) {
  const int64_t nblk = n_pad / 32;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * nblk) return;
  const int64_t rho = idx / nblk, bI = idx % nblk;
  double v[32], dq[32];
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    v[j] = (rho < n && c < n && rho != c) ? P[rho * n + c] : 0.0;
  }
  uint32_t wds[8];
  fp6_block(v, wds, dq);
  for (int j = 0; j < 32; ++j) Qn[rho * n_pad + bI * 32 + perm_nat(j)] = dq[j];
  fp6_store(tiles, nK, rho, bI, wds);
}

// R = (P_off - E) * out_scale with E the symmetric matrix the MX screen actually evaluates
// (block-upper visit over 128-row K-blocks: off-diagonal blocks from the upper row's scales,
// diagonal blocks symmetrised), natural order; rowabs[k] = sum_l |E_kl|.  One workgroup per row.
__global__ __launch_bounds__(256) void mx_residual_kernel(int64_t n, int64_t n_pad, const double *P, const double *Qn,
                                                          double out_scale, double *R, double *rowabs) {
  const int64_t k = blockIdx.x, bk = k / MXK;
  double s = 0.0;
  for (int64_t l = threadIdx.x; l < n_pad; l += 256) {
    const int64_t bl = l / MXK;
    const double E = bl == bk ? 0.5 * (Qn[k * n_pad + l] + Qn[l * n_pad + k])
                              : (bl > bk ? Qn[k * n_pad + l] : Qn[l * n_pad + k]);
    const double po = (k < n && l < n && k != l) ? P[k * n + l] : 0.0;
    R[k * n_pad + l] = (po - E) * out_scale;
    s += fabs(E);
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) rowabs[k] = (red[0] + red[1]) + (red[2] + red[3]);
}

// nibble planes of a screen panel (storage order, codes 0..2): record (SNP, stage) = two 64-byte
// planes, individual q of the stage at nibble q & 1 of byte q >> 1.  i side: M1 = [a==1] 0xF,
// M2 = [a==2] 0xF; j side: S1 = b, S2 = 2b (fp4 codes of w/2 for w = 1*b, 2*b).
__global__ void nibble_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *nib_i,
                              uint32_t *nib_j) {
  const int64_t per = n_pad / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * per) return;
  const int64_t j = idx / per, d = idx % per;
  const int64_t stage = d / 16, dd = d % 16;
  const int8_t *src = panel + j * n_pad + 8 * d;
  uint32_t m1 = 0, m2 = 0, s1 = 0, s2 = 0;
  for (int e = 0; e < 8; ++e) {
    const uint32_t a = (uint32_t)src[e];
    m1 |= (a == 1 ? 0xFu : 0u) << (4 * e);
    m2 |= (a == 2 ? 0xFu : 0u) << (4 * e);
    s1 |= a << (4 * e);
    s2 |= (2 * a) << (4 * e);
  }
  const int64_t rec = (j * nK + stage) * (NB_REC / 4);
  nib_i[rec + dd] = m1;
  nib_i[rec + 16 + dd] = m2;
  nib_j[rec + dd] = s1;
  nib_j[rec + 16 + dd] = s2;
}

// the j side's S1 planes (nibble_kernel: nibble e of dword dd = code of individual 8 dd + e) at 2 bits
// for the compacted low-rank screen: per (SNP, 128-individual stage) 32 bytes, 8-byte piece k packing
// the plane's dwords 4k .. 4k + 3 as D0 | D1 << 2, D2 | D3 << 2 (codes 0..2 fit two bits)
__global__ void s1_code2_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *out) {
  const int64_t per = n_pad / 16;  // one output dword per 16 individuals
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * per) return;
  const int64_t j = idx / per, g = idx % per;  // g: output dword (16 individuals: plane dwords 2g, 2g + 1)
  const int8_t *src = panel + j * n_pad + 16 * g;
  uint32_t d = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) d |= ((uint32_t)(src[e] & 3) | ((uint32_t)(src[8 + e] & 3) << 2)) << (4 * e);
  out[j * (n_pad / 16) + g] = d;
}

// per row i of P (n x n, natural order): max |P_ik| off the diagonal, |P_ii| and the sum (mod 2^64)
// of a 64-bit mix of every element's bits with its index (the plan's fingerprint of P, order-free)
__global__ __launch_bounds__(256) void p_scan_kernel(int64_t n, const double *P, double *out) {
  const int64_t i = blockIdx.x;
  const double *row = P + i * n;
  double q = 0.0;
  uint64_t h = 0;
  for (int64_t k = threadIdx.x; k < n; k += 256) {
    const double v = row[k];
    if (k != i) q = fmax(q, fabs(v));
    uint64_t z = (uint64_t)__double_as_longlong(v) ^ ((uint64_t)(i * n + k) * 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    h += z ^ (z >> 31);
  }
  __shared__ double sq[256];
  __shared__ uint64_t sh[256];
  sq[threadIdx.x] = q;
  sh[threadIdx.x] = h;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
      sq[threadIdx.x] = fmax(sq[threadIdx.x], sq[threadIdx.x + off]);
      sh[threadIdx.x] += sh[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[i] = sq[0];
    out[n + i] = fabs(row[i]);
    out[2 * n + i] = __longlong_as_double((long long)sh[0]);
  }
}

// A = P + (mu + tau) 11'/n - mu I (natural order, n x n) for the prefilter's Cholesky certificate
__global__ void pf_shift_kernel(int64_t n, const double *P, double mu, double tau, double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  const int64_t r = idx / n, c = idx % n;
  A[idx] = P[idx] + (mu + tau) / (double)n - (r == c ? mu : 0.0);
}

// fp4 e2m1 copy of a screen panel (codes 0, 1, 2 -> 0x0, 0x2, 0x4; the prefilter derives the
// squares' codes in registers, sq4); individual 2q at the low nibble of byte q (the MFMA's packing)
// A = P + (mu + tau) 11'/n + ku C - mu I  (C = U U', or none)
__global__ void pf_shift_u_kernel(int64_t n, const double *P, const double *C, double mu, double tau, double ku,
                                  double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  double v = P[idx] + (mu + tau) / (double)n;
  if (C) v += ku * C[idx];
  if (idx / n == idx % n) v -= mu;
  A[idx] = v;
}

// covariate direction dots of a coding: dot[j] = sum_t code[j][t] u[t] (fixed-order reduction)
__global__ __launch_bounds__(256) void cov_dot_kernel(int64_t n_pad, const int8_t *panel, const double *u, double *dot) {
  const int64_t j = blockIdx.x;
  const int8_t *pj = panel + j * n_pad;
  __shared__ double rsum[256];
  double sm = 0.0;
  for (int64_t t = threadIdx.x; t < n_pad; t += 256) sm += (double)pj[t] * u[t];
  rsum[threadIdx.x] = sm;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) rsum[threadIdx.x] += rsum[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) dot[j] = rsum[0];
}

// stage-blocked copy of an SNP-major int8 panel (dst[(st m + snp) w + b] = src[snp W + st w + b] for
// stages st of w bytes, W bytes per SNP, 16 bytes per thread), each 8 bytes reordered to individuals
// 0 2 4 6 1 3 5 7 (the K slot order of i8x2_of_fp4_eo)
__global__ void block_panel_perm8_kernel(int64_t m, int64_t W, int64_t w, const uint8_t *__restrict__ src,
                                         uint8_t *__restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, per = W / 16;
  if (t >= m * per) return;
  const int64_t snp = t / per, o = (t % per) * 16, st = o / w, b = o % w;
  v4i v = *(const v4i *)(src + snp * W + o);
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // bytes 0..7 of dwords (2h, 2h + 1): even ones first, then odd
    const unsigned lo = (unsigned)v[2 * h], hi = (unsigned)v[2 * h + 1];
    v[2 * h] = (int)__builtin_amdgcn_perm(hi, lo, 0x06040200u);
    v[2 * h + 1] = (int)__builtin_amdgcn_perm(hi, lo, 0x07050301u);
  }
  *(v4i *)(dst + (st * m + snp) * w + b) = v;
}

// prefilter test records (prefilter_pass_kernel's epilogue, 32 bytes per SNP, fetched by LDS-DMA with
// the first stage): fp64 per-SNP sums rounded once to fp32, exactly the values the test used to derive
// itself.  Row role: [i (int bits; -1 = monomorphic), alpha, csum, R1 = csq - 2 alpha csum, sL3, sa,
// (2 + alpha)^2, 0]; column role: [beta, csum, C1n = csq - 2 beta csum + n beta^2, n beta - csum,
// beta spy - sb, sum_k (b + beta)^2, monomorphic, 0]
__global__ void pf_rec_kernel(int64_t m, double n, double spy, const double *__restrict__ soff,
                              const double *__restrict__ csum, const double *__restrict__ csq,
                              const double *__restrict__ sL3, const double *__restrict__ sa,
                              const double *__restrict__ sb, const uint8_t *__restrict__ mono, float *recL,
                              float *recR) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const double al = soff[j], c = csum[j], c2 = csq[j];
  float *l = recL + j * PF_REC, *r = recR + j * PF_REC;
  l[0] = __int_as_float(mono[j] ? -1 : (int)j);
  l[1] = (float)al;
  l[2] = (float)c;
  l[3] = (float)(c2 - 2.0 * al * c);
  l[4] = (float)sL3[j];
  l[5] = (float)sa[j];
  l[6] = (float)((2.0 + al) * (2.0 + al));
  l[7] = 0.0f;
  r[0] = (float)al;
  r[1] = (float)c;
  r[2] = (float)(c2 - 2.0 * al * c + n * al * al);
  r[3] = (float)(n * al - c);
  r[4] = (float)(al * spy - sb[j]);
  r[5] = (float)(c2 + 2.0 * al * c + n * al * al);
  r[6] = mono[j] ? 1.0f : 0.0f;
  r[7] = 0.0f;
}

__global__ void fp4_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint8_t *p4) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * (n_pad / 2)) return;
  const int v0 = panel[2 * idx], v1 = panel[2 * idx + 1];
  auto code = [](int v) { return v == 0 ? 0 : v == 1 ? 2 : 4; };
  p4[idx] = (uint8_t)(code(v0) | (code(v1) << 4));
}

__global__ void u8_unit_kernel(int64_t n_pad, const double *__restrict__ Ps, double *__restrict__ unit) {
  const int64_t q = blockIdx.x;
  double mx = 0.0;
  for (int64_t r = threadIdx.x; r < n_pad; r += blockDim.x) mx = fmax(mx, fabs(Ps[q * n_pad + r]));
  for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double m4 = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    unit[q] = m4 > 0.0 ? m4 / 127.0 : 1.0;
  }
}

__global__ void u8_slice_kernel(int64_t n_pad, const double *__restrict__ Ps, const double *__restrict__ unit,
                                int8_t *__restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t q = idx / n_pad, r = idx % n_pad;
  const int64_t st = r / 64;
  const int rr = (int)(r % 64), chunk = rr >> 4, pos = u8_pos(rr & 15);
  const int phys = chunk ^ u8_swz((int)(q & 31));
  double v = Ps[idx] / unit[q];
  int8_t *o = out + (st * U8_S * n_pad + q) * 64 + phys * 16 + pos;
  for (int sl = 0; sl < U8_S; ++sl) {
    const double t = rint(v);
    o[(int64_t)sl * n_pad * 64] = (int8_t)t;
    v = (v - t) * 128.0;
  }
}

__global__ __launch_bounds__(512, 1) void u8_gemm_kernel(int64_t m, int64_t n_pad, const uint8_t *__restrict__ p2b,
                                                         const int8_t *__restrict__ slices, const double *__restrict__ unit,
                                                         double *__restrict__ U) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[U8_NS][U8_ST];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t j0 = (int64_t)blockIdx.x * U8_J, q0 = (int64_t)blockIdx.y * U8_Q;
  const int S = (int)(n_pad / SG_K);
  // DMAs per stage: wave w the two 1-KB pieces of slice w (q rows 0-15, 16-31); waves 0-3 also the
  // codes of SNPs j0 + 64 w .. + 63 (16 B each)
  const int nq = w < 4 ? 3 : 2;
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]);
  const int8_t *bsrc = slices + ((int64_t)w * n_pad + q0) * 64 + lane * 16;
  const uint8_t *asrc = p2b + std::min<int64_t>(j0 + 64 * w + lane, m - 1) * 16;
  auto issue = [&](int st, int slot) __attribute__((always_inline)) {
    const unsigned base = ring_m0 + slot * U8_ST;
    const int8_t *b = bsrc + (int64_t)st * U8_S * n_pad * 64;
    lds_dma16_m0(b, base + U8_AB + w * 2048);
    lds_dma16_m0(b + 1024, base + U8_AB + w * 2048 + 1024);
    if (w < 4) lds_dma16_m0(asrc + (int64_t)st * m * 16, base + w * 1024);
  };
  static_assert(U8_NS == 4, "wait_for's vmcnt values");
  auto wait_for = [&](int ahead) __attribute__((always_inline)) {
    if (nq == 3) {
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };
  const int pre = min(S, U8_NS - 1);
  for (int st = 0; st < pre; ++st) issue(st, st);
  v16i acc[U8_S];
#pragma unroll
  for (int sl = 0; sl < U8_S; ++sl)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[sl][e] = 0;
  const int sw = u8_swz(c);
  for (int st = 0; st < S; ++st) {
    // stage st landed (the younger stages issued may be in flight), then every wave has left stage
    // st - 1, whose slot the stage issued next reuses
    wait_for(min(st + U8_NS - 2, S - 1) - st);
    if (st + U8_NS - 1 < S) issue(st + U8_NS - 1, (st + U8_NS - 1) % U8_NS);
    const uint8_t *bf = ring[st % U8_NS];
    const v4i ad = *(const v4i *)&bf[(32 * w + c) * 16];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i a8 = i8_of_code2((unsigned)ad[2 * kk + h]);
#pragma unroll
      for (int sl = 0; sl < U8_S; ++sl) {
        const v4i b8 = *(const v4i *)&bf[U8_AB + sl * 2048 + c * 64 + 16 * ((2 * kk + h) ^ sw)];
        acc[sl] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a8, b8, acc[sl], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int64_t q = q0 + c;
  const double uq = unit[q];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t j = j0 + 32 * w + (e & 3) + 8 * (e >> 2) + 4 * h;
    double sum = (double)acc[U8_S - 1][e];
#pragma unroll
    for (int sl = U8_S - 2; sl >= 0; --sl) sum = sum * (1.0 / 128.0) + (double)acc[sl][e];
    if (j < m) U[j * n_pad + q] = uq * sum;
  }
}

__global__ void code2_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint32_t *dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, per = n_pad / 16;
  if (idx >= m * per) return;
  const int64_t snp = idx / per, g = idx % per, st = g >> 2;
  const int8_t *p = panel + snp * n_pad + 16 * g;
  unsigned d = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) d |= (unsigned)((p[k] & 3) | ((p[8 + k] & 3) << 2)) << (4 * k);
  dst[(st * m + snp) * 4 + (g & 3)] = d;
}

// A = P + C + (lam + tau) 11'/n - lam I (natural order) for the low-rank screen's certificate
__global__ void lr_shift_kernel(int64_t n, const double *P, const double *C, double lam, double tau, double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  const int64_t r = idx / n, c = idx % n;
  A[idx] = P[idx] + C[idx] + (lam + tau) / (double)n - (r == c ? lam : 0.0);
}

// G'[j][r] = G[j][r] - soff[j] q1[r] (fp64, rounded once to fp32)
__global__ void lr_adjust_kernel(int64_t m, int64_t R, const double *G, const double *soff, const double *q1, float *out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < m * R) out[idx] = (float)(G[idx] - soff[idx / R] * q1[idx % R]);
}

__global__ void f64_to_f16_kernel(int64_t count, const double *src, _Float16 *dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < count) dst[t] = (_Float16)src[t];  // |U| << 65504 (P entries ~ 1 / sigma, codes <= 2)
}

__global__ void f64_to_f32_kernel(int64_t count, const double *src, float *dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < count) dst[idx] = (float)src[idx];
}

// Q(lam) on the device: block (r, bI) of sqrt(d_r) u_r quantised to fp6 (fp6_block), dequantised
// into Bn (natural [k][r]) and Bs (storage [q][r]), and the tile images when img is given.
__global__ void lr_quant_kernel(int64_t n, int64_t n_pad, int nK, int Rp, const double *__restrict__ Z,
                                const double *__restrict__ sd, double *__restrict__ Bn, double *__restrict__ Bs,
                                uint32_t *__restrict__ img) {
  const int64_t nblk = n_pad / 32;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)Rp * nblk) return;
  const int r = (int)(idx / nblk);
  const int64_t bI = idx % nblk;
  const double s = sd[r];
  double v[32], dq[32];
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    v[j] = (s > 0.0 && c < n) ? s * Z[(size_t)r * n + c] : 0.0;
  }
  uint32_t wds[8];
  fp6_block(v, wds, dq);
  if (img) fp6_store(img, nK, r, bI, wds);
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    if (c < n) Bn[(size_t)c * Rp + r] = dq[j];
    Bs[(size_t)(bI * 32 + j) * Rp + r] = dq[j];
  }
}

__global__ __launch_bounds__(AUD_T) void audit_kernel(int64_t n, int64_t n_pad, int R, int ncov, const int8_t *left,
                                                      const int8_t *right, const double *alpha, const double *beta,
                                                      const int64_t *pi, const int64_t *pj, const double *Q,
                                                      const double *U, double pf_mu, double pf_tau, double pf_eps,
                                                      double pf_ku, double lr_lam, double lr_tau, double lr_eps,
                                                      double *out) {
  __shared__ double es[AUD_T];
  __shared__ double red[AUD_T / 64][8];
  const int tid = threadIdx.x;
  const int64_t t = blockIdx.x, i = pi[t], j = pj[t];
  const int8_t *a = left + i * n_pad, *b = right + j * n_pad;
  const double al = alpha[i], be = beta[j];
  double ee = 0, se = 0, cr = 0, cu[4] = {0, 0, 0, 0};
  for (int64_t s0 = 0; s0 < n_pad; s0 += AUD_T) {
    const int64_t s = s0 + tid;
    const int64_t nat = (s & ~31LL) + perm_nat((int)(s & 31));
    const double e = (nat < n) ? ((double)a[s] - al) * ((double)b[s] - be) : 0.0;
    ee += e * e;
    se += e;
    for (int k = 0; k < ncov; ++k) cu[k] += U[k * n_pad + s] * e;
    es[tid] = e;
    __syncthreads();
    if (tid < R)
      for (int q = 0; q < AUD_T; ++q) cr += Q[(s0 + q) * R + tid] * es[q];
    __syncthreads();
  }
  double v[7] = {ee, se, tid < R ? cr * cr : 0.0, cu[0], cu[1], cu[2], cu[3]};
  for (int q = 0; q < 7; ++q)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o);
  if ((tid & 63) == 0)
    for (int q = 0; q < 7; ++q) red[tid >> 6][q] = v[q];
  __syncthreads();
  if (tid == 0) {
    double s7[7];
    for (int q = 0; q < 7; ++q) s7[q] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
    const double EE = s7[0], SE = s7[1], QQ = s7[2], dn = (double)n;
    double uu = 0.0;
    for (int k = 0; k < ncov; ++k) uu += s7[3 + k] * s7[3 + k];
    out[5 * t + 0] = pf_mu > 0 ? (pf_mu - pf_eps) * EE - (pf_mu + pf_tau) * SE * SE / dn - pf_ku * uu : -INFINITY;
    out[5 * t + 1] = R > 0 ? lr_lam * (EE - SE * SE / dn) - lr_tau * SE * SE / dn - lr_eps * EE - QQ : -INFINITY;
    out[5 * t + 2] = EE;
    out[5 * t + 3] = SE;
    out[5 * t + 4] = QQ;
  }
}


// host launcher of i8gemm_nt_kernel (the block-granular scans' side GEMMs)
int i8gemm_nt(hipStream_t st, int Z, int M, int N, int K, const int8_t *A, int64_t lda, int64_t za, const int8_t *B,
              int64_t ldb, int64_t zb, int *C, int64_t ldc, int64_t zc) {
  if (M <= 0 || N <= 0) return GMAT_OK;
  hipLaunchKernelGGL(i8gemm_nt_kernel, dim3((unsigned)cdiv(N, GN), (unsigned)cdiv(M, GM), (unsigned)Z), dim3(256), 0,
                     st, M, N, K, A, lda, za, B, ldb, zb, C, ldc, zc);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

}  // namespace epi
}  // namespace gmat

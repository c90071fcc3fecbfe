// PLINK .bed decoding into device panels, and the genomic relationship matrices.
//
// Decode semantics follow process_plink/_read_plink_bed.c:17-44 (2-bit code c of
// individual k at bits 2*(k%4) of byte k/4 of the SNP's ceil(n/4)-byte row; dosage
// (c^2+c)/6 with code 01 = missing).  The GRM replaces the fp64 GEMM np.dot(X, X.T) of
// gmatrix.py:63 (additive) / :127 (dominance) by an EXACT integer product of the
// uncentred 0/1/2 (or 0/1) codes on int8 MFMA, then applies the centring as fp64
// rank-one corrections:  (G - 1c')(G - 1c')' = GG' - r1' - 1r' + (c'c) 11',  r = Gc.
#include "dla.h"
#include "geno.h"

using namespace gmat;

namespace {

// one workgroup per SNP: decode, permute into storage order, count
__global__ __launch_bounds__(256) void decode_kernel(const uint8_t *__restrict__ packed, int64_t nb, int64_t n,
                                                     int64_t n_pad, int8_t *__restrict__ dose,
                                                     int8_t *__restrict__ het, int64_t *__restrict__ cnt) {
  const int64_t snp = blockIdx.x;
  const uint8_t *row = packed + snp * nb;
  int s_dose = 0, s_het = 0, s_miss = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const int64_t k = (q & ~31LL) + perm_nat((int)(q & 31));
    int d = 0, h = 0;
    if (k < n) {
      const int c = (row[k >> 2] >> (2 * (k & 3))) & 3;
      if (c == 1) {
        s_miss++;
      } else {
        d = (c == 0) ? 0 : c - 1;  // 00->0, 10->1, 11->2
        h = (c == 2);
      }
    }
    dose[snp * n_pad + q] = (int8_t)d;
    het[snp * n_pad + q] = (int8_t)h;
    s_dose += d;
    s_het += h;
  }
  __shared__ int red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s_dose += __shfl_xor(s_dose, off);
    s_het += __shfl_xor(s_het, off);
    s_miss += __shfl_xor(s_miss, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s_dose;
    red[1][threadIdx.x >> 6] = s_het;
    red[2][threadIdx.x >> 6] = s_miss;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int64_t t = 0;
    for (int w = 0; w < 4; ++w) t += red[threadIdx.x][w];
    cnt[snp * 3 + threadIdx.x] = t;
  }
}

// individual-major natural-order code matrix for the GRM: out[a][j] (ld = m_pad),
// kind 0 -> dosage, 1 -> het indicator.  64 SNPs x 64 individuals per block.
__global__ __launch_bounds__(256) void transpose_codes_kernel(const uint8_t *__restrict__ packed, int64_t nb,
                                                              int64_t n, int64_t m, int64_t m_pad, int kind,
                                                              int8_t *__restrict__ out) {
  __shared__ int8_t t[64][65];
  const int64_t j0 = (int64_t)blockIdx.x * 64, a0 = (int64_t)blockIdx.y * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int jj = e >> 6, aa = e & 63;
    const int64_t j = j0 + jj, a = a0 + aa;
    int v = 0;
    if (j < m && a < n) {
      const int c = (packed[j * nb + (a >> 2)] >> (2 * (a & 3))) & 3;
      v = kind == 0 ? (c == 0 ? 0 : (c == 1 ? 0 : c - 1)) : (c == 2);
    }
    t[jj][aa] = (int8_t)v;
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int aa = e >> 6, jj = e & 63;
    const int64_t a = a0 + aa, j = j0 + jj;
    if (j < m_pad) out[a * m_pad + j] = t[jj][aa];
  }
}

// r[a] = sum_j code[a][j] * c[j]
__global__ __launch_bounds__(256) void rowdot_i8_kernel(const int8_t *__restrict__ gt, int64_t m_pad, int64_t m,
                                                        const double *__restrict__ c, int64_t n,
                                                        double *__restrict__ r) {
  const int64_t a = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (a >= n) return;
  double s = 0.0;
  for (int64_t j = lane; j < m; j += 64) s += (double)gt[a * m_pad + j] * c[j];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) r[a] = s;
}

// Lower-triangle SYRK C = Gt Gt' on v_mfma_i32_32x32x32_i8: 128 x 128 tile per workgroup,
// 4 waves of 64 x 64 (2 x 2 MFMA tiles), 64-deep K stages staged through LDS with an
// 80-byte row pitch (conflict-free ds_read_b128), fp64 centring/scaling epilogue.
constexpr int GT = 128, GK = 64, GP = 80;

__global__ __launch_bounds__(256) void grm_kernel(const int8_t *__restrict__ gt, int64_t m_pad, int64_t n,
                                                  const double *__restrict__ r, double cc, double scale,
                                                  double small_val, double *__restrict__ kin) {
  const int tb = blockIdx.x, ta = blockIdx.y;
  if (ta < tb) return;
  __shared__ __attribute__((aligned(16))) int8_t sa[GT * GP];
  __shared__ __attribute__((aligned(16))) int8_t sb[GT * GP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 1, wc = w & 1;
  const int64_t a0 = (int64_t)ta * GT, b0 = (int64_t)tb * GT;
  v16i acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
  for (int64_t j0 = 0; j0 < m_pad; j0 += GK) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ch = tid + 256 * q, row = ch >> 2, c16 = ch & 3;
      *(v4i *)&sa[row * GP + c16 * 16] = *(const v4i *)&gt[(a0 + row) * m_pad + j0 + c16 * 16];
      *(v4i *)&sb[row * GP + c16 * 16] = *(const v4i *)&gt[(b0 + row) * m_pad + j0 + c16 * 16];
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4i fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        fa[t] = *(const v4i *)&sa[(wr * 64 + t * 32 + (lane & 31)) * GP + kk * 32 + (lane >> 5) * 16];
        fb[t] = *(const v4i *)&sb[(wc * 64 + t * 32 + (lane & 31)) * GP + kk * 32 + (lane >> 5) * 16];
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t a = a0 + wr * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
        const int64_t b = b0 + wc * 64 + j * 32 + (lane & 31);
        if (a < n && b < n && b <= a) {
          double v = ((double)acc[i][j][e] - r[a] - r[b] + cc) / scale;
          if (a == b) v = v + v * small_val;
          kin[a * n + b] = v;
          kin[b * n + a] = v;
        }
      }
}

}  // namespace

extern "C" int gmat_geno_create(gmat_geno **out, const uint8_t *bed_body, int64_t body_bytes, int64_t n_id,
                                int64_t n_snp) {
  GMAT_CHECK(out && bed_body && n_id > 0 && n_snp > 0, GMAT_E_ARG, "gmat_geno_create: bad arguments");
  const int64_t nb = (n_id + 3) / 4;
  GMAT_CHECK(body_bytes >= nb * n_snp, GMAT_E_ARG,
             "gmat_geno_create: .bed body has %lld bytes, %lld x %lld individuals/SNPs need %lld",
             (long long)body_bytes, (long long)n_snp, (long long)n_id, (long long)(nb * n_snp));
  auto *g = new gmat_geno();
  g->n = n_id;
  g->m = n_snp;
  g->nb = nb;
  g->n_pad = round_up(n_id, 256);
  int rc = g->packed.alloc(nb * n_snp);
  if (rc == GMAT_OK) rc = g->panels.alloc(2 * g->n_pad * n_snp);
  DBuf cnt;
  if (rc == GMAT_OK) rc = cnt.alloc(3 * n_snp * sizeof(int64_t));
  if (rc != GMAT_OK) {
    delete g;
    return rc;
  }
  hipError_t e = hipMemcpy(g->packed.p, bed_body, nb * n_snp, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(decode_kernel, dim3((unsigned)n_snp), dim3(256), 0, 0, g->packed.as<uint8_t>(), nb, n_id,
                       g->n_pad, g->dose_ptr(), g->het_ptr(), cnt.as<int64_t>());
    e = hipGetLastError();
  }
  std::vector<int64_t> h(3 * n_snp);
  if (e == hipSuccess) e = hipMemcpy(h.data(), cnt.p, h.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    set_error("gmat_geno_create: %s", hipGetErrorString(e));
    delete g;
    return GMAT_E_HIP;
  }
  g->sum_dose.resize(n_snp);
  g->n_het.resize(n_snp);
  g->n_miss.resize(n_snp);
  for (int64_t j = 0; j < n_snp; ++j) {
    g->sum_dose[j] = h[3 * j];
    g->n_het[j] = h[3 * j + 1];
    g->n_miss[j] = h[3 * j + 2];
    g->total_missing += h[3 * j + 2];
  }
  *out = g;
  return GMAT_OK;
}

extern "C" int gmat_geno_counts(const gmat_geno *g, int64_t *sum_dose, int64_t *n_het, int64_t *n_miss) {
  GMAT_CHECK(g, GMAT_E_ARG, "gmat_geno_counts: null handle");
  if (sum_dose) memcpy(sum_dose, g->sum_dose.data(), g->m * sizeof(int64_t));
  if (n_het) memcpy(n_het, g->n_het.data(), g->m * sizeof(int64_t));
  if (n_miss) memcpy(n_miss, g->n_miss.data(), g->m * sizeof(int64_t));
  return GMAT_OK;
}

extern "C" int gmat_geno_destroy(gmat_geno *g) {
  delete g;
  return GMAT_OK;
}

static double g_grm_stats[4] = {0, 0, 0, 0};

extern "C" int gmat_grm_stats(double *out4) {
  GMAT_CHECK(out4, GMAT_E_ARG, "gmat_grm_stats: null");
  for (int k = 0; k < 4; ++k) out4[k] = g_grm_stats[k];
  return GMAT_OK;
}

extern "C" int gmat_grm(gmat_geno *g, int kind, double small_val, double *kin, double *scale_out) {
  GMAT_CHECK(g && kin, GMAT_E_ARG, "gmat_grm: bad arguments");
  GMAT_CHECK(kind == GMAT_GRM_ADD || kind == GMAT_GRM_DOM, GMAT_E_ARG, "gmat_grm: unknown kind %d", kind);
  GMAT_CHECK(g->total_missing == 0, GMAT_E_ARG, "gmat_grm: panel has %lld missing genotypes (impute first)",
             (long long)g->total_missing);
  const int64_t n = g->n, m = g->m, m_pad = round_up(m, 64), n_pad = round_up(n, GT);
  // centring vector and scale exactly as gmatrix.py:53-57 (additive) / :116-120 (dominance)
  std::vector<double> c(m);
  double scale = 0.0, cc = 0.0;
  for (int64_t j = 0; j < m; ++j) {
    const double freq = (double)g->sum_dose[j] / (2.0 * (double)n);
    const double s = 2.0 * freq * (1.0 - freq);
    if (kind == GMAT_GRM_ADD) {
      c[j] = 2.0 * freq;
      scale += s;
    } else {
      c[j] = s;
      scale += s * (1.0 - s);
    }
    cc += c[j] * c[j];
  }
  if (scale_out) *scale_out = scale;
  DBuf gt, dc, dr, dk;
  GMAT_TRY(gt.alloc(n_pad * m_pad));
  GMAT_TRY(dc.alloc(m * sizeof(double)));
  GMAT_TRY(dr.alloc(n_pad * sizeof(double)));
  GMAT_TRY(dk.alloc(n * n * sizeof(double)));
  GMAT_HIP(hipMemset(gt.p, 0, n_pad * m_pad));
  GMAT_HIP(hipMemcpy(dc.p, c.data(), m * sizeof(double), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(transpose_codes_kernel, dim3((unsigned)cdiv(m_pad, 64), (unsigned)cdiv(n, 64)), dim3(256), 0, 0,
                     g->packed.as<uint8_t>(), g->nb, n, m, m_pad, kind, gt.as<int8_t>());
  GMAT_HIP(hipGetLastError());
  hipLaunchKernelGGL(rowdot_i8_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, 0, gt.as<int8_t>(), m_pad, m,
                     dc.as<double>(), n, dr.as<double>());
  GMAT_HIP(hipGetLastError());
  const unsigned nt = (unsigned)(n_pad / GT);
  hipEvent_t e0, e1;
  GMAT_HIP(hipEventCreate(&e0));
  GMAT_HIP(hipEventCreate(&e1));
  GMAT_HIP(hipEventRecord(e0, 0));
  hipLaunchKernelGGL(grm_kernel, dim3(nt, nt), dim3(256), 0, 0, gt.as<int8_t>(), m_pad, n, dr.as<double>(), cc,
                     scale, small_val, dk.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(e1, 0));
  GMAT_HIP(hipEventSynchronize(e1));
  float ms = 0;
  GMAT_HIP(hipEventElapsedTime(&ms, e0, e1));
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  g_grm_stats[0] = ms * 1e-3;
  g_grm_stats[1] = (double)nt * (nt + 1) / 2 * 2.0 * GT * GT * (double)m_pad;  // int8 ops issued (lower tiles)
  g_grm_stats[2] = 2.0 * (double)n * n * m;                                      // dense-equivalent flop 2n^2m
  GMAT_HIP(hipMemcpy(kin, dk.p, n * n * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

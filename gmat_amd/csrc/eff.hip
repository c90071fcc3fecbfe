// Effect-only epistasis screen (the reference's C kernels remma_epi{AA,AD,DD}(_maf)_eff_cpu,
// _remma_epi_eff_cpu.c:61-574) and the plain .bed decoder read_plink_bed (:10-56).
//
// eff(i, j) = sum_k x_ik x_jk py_k over pairs j > i of the listed first SNPs i, where x is the
// reference's fp64 coding of the 2-bit PLINK code c: v = (c^2 + c)/6 (0, 1/3 missing, 1, 2),
// additive x = v - 2p, dominance x = [v != 2] v - 2p(1-p), with p accumulated exactly as the
// reference does (p += v/(2n) over individuals in .fam order, :103-112 / :277-285 / :459-464),
// so the centring is bit-identical.  A pair is kept when |eff| > eff_cut (AD: >= for the
// (i, j) orientation, > for (j, i), :238/:245), eff_cut from one value or, for the _maf
// forms, from the 111-entry table at freq_i*10 + freq_j (:152, :338, :525).
//
// Device layout: X (m x n fp64, natural individual order) for each coding the kind needs,
// built once per call from the resident packed panel.  A chunk of R listed rows becomes the
// band A = X1[rows] o py (R x n); E = A X2[j0:]^T is an fp64 MFMA GEMM (dgemm, ~2n flop per
// pair); an ordered compaction (one workgroup per row, block prefix sums) emits the kept
// pairs in the reference's single-thread order: rows in list order, j ascending, for AD
// (i, j) before (j, i).  The hit records are written as "%lld %lld %g" text on the host.
#include <chrono>
#include <cmath>

#include "dla.h"
#include "geno.h"

namespace {
using namespace gmat;

// One thread per SNP: the reference's sequential frequency accumulation (bit-exact), then
// the centring constants of both codings.
__global__ void eff_freq_kernel(const uint8_t *packed, int64_t nb, int64_t n, int64_t m, double *c_add,
                                double *c_dom) {
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (j >= m) return;
  const uint8_t *p = packed + j * nb;
  const double two_n = 2.0 * (double)n;
  double f = 0.0;
  for (int64_t k = 0; k < n; ++k) {
    const int c = (p[k >> 2] >> (2 * (k & 3))) & 3;
    f += ((double)(c * c + c) / 6.0) / two_n;
  }
  c_add[j] = 2.0 * f;
  c_dom[j] = 2.0 * f * (1.0 - f);
}

// X[j][k] for one coding (dom = 0 additive, 1 dominance); one workgroup per SNP.
__global__ void eff_x_kernel(const uint8_t *packed, int64_t nb, int64_t n, const double *centre, int dom,
                             double *x) {
  const int64_t j = blockIdx.x;
  const uint8_t *p = packed + j * nb;
  const double c0 = centre[j];
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int c = (p[k >> 2] >> (2 * (k & 3))) & 3;
    double v = (double)(c * c + c) / 6.0;
    if (dom && fabs(v - 2.0) < 0.0001) v = 0.0;
    x[j * n + k] = v - c0;
  }
}

// A[r][k] = X[rows[r]][k] * py[k]
__global__ void eff_band_kernel(const double *x, int64_t n, const int64_t *rows, const double *py, double *a) {
  const int64_t r = blockIdx.y;
  const int64_t k = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (k >= n) return;
  a[r * n + k] = x[rows[r] * n + k] * py[k];
}

// The plain .bed decoder (_read_plink_bed.c:5-51): marker[j*n + k] = (c^2 + c)/6; one
// workgroup per SNP.
__global__ void decode_f64_kernel(const uint8_t *packed, int64_t nb, int64_t n, double *out) {
  const int64_t j = blockIdx.x;
  for (int64_t k = threadIdx.x; k < n; k += blockDim.x) {
    const int c = (packed[j * nb + (k >> 2)] >> (2 * (k & 3))) & 3;
    out[j * n + k] = (double)(c * c + c) / 6.0;
  }
}

struct EffCut {
  const double *cut;     // 1 or 111 entries (device)
  const int64_t *fi;     // freq of the first SNP's coding (device), null: single cut
  const int64_t *fj;     // freq of the second SNP's coding (device)
};

// Per-thread hit count (0..2) of pair column t of row r.
__device__ __forceinline__ int eff_keep(int kind, const double *e1, const double *e2, int64_t r, int64_t ld,
                                        int64_t t, int64_t i, int64_t j, EffCut ec, bool *k1, bool *k2) {
  const double cut = ec.fi ? ec.cut[ec.fi[i] * 10 + ec.fj[j]] : ec.cut[0];
  const double a = fabs(e1[r * ld + t]);
  if (kind == GMAT_AD) {
    *k1 = a >= cut;
    *k2 = fabs(e2[r * ld + t]) > cut;
  } else {
    *k1 = a > cut;
    *k2 = false;
  }
  return (int)*k1 + (int)*k2;
}

constexpr int CT = 256;  // compaction threads

__device__ __forceinline__ int block_excl_scan(int v, int *sh, int *total) {
  // inclusive wave scan, then across the 4 waves
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(s, o);
    if (lane >= o) s += u;
  }
  if (lane == 63) sh[w] = s;
  __syncthreads();
  int base = 0, tot = 0;
#pragma unroll
  for (int q = 0; q < CT / 64; ++q) {
    if (q < w) base += sh[q];
    tot += sh[q];
  }
  __syncthreads();
  *total = tot;
  return base + s - v;
}

// Pass 1 (write == false): hits of row r -> counts[r].  Pass 2: records at offsets[r], in
// j order, (i, j) before (j, i).
template <bool WRITE>
__global__ __launch_bounds__(CT) void eff_compact_kernel(int kind, const double *e1, const double *e2, int64_t ld,
                                                         int64_t j0, int64_t m, const int64_t *rows, EffCut ec,
                                                         int64_t *counts, const int64_t *offsets, int64_t *hi,
                                                         int64_t *hj, double *he) {
  __shared__ int sh[CT / 64];
  const int64_t r = blockIdx.x;
  const int64_t i = rows[r];
  int64_t pos = WRITE ? offsets[r] : 0;
  int64_t cnt = 0;
  for (int64_t jb = i + 1; jb < m; jb += CT) {
    const int64_t j = jb + threadIdx.x;
    bool k1 = false, k2 = false;
    int c = 0;
    if (j < m) c = eff_keep(kind, e1, e2, r, ld, j - j0, i, j, ec, &k1, &k2);
    int total;
    const int off = block_excl_scan(c, sh, &total);
    if (WRITE) {
      int64_t q = pos + off;
      if (k1) {
        hi[q] = i;
        hj[q] = j;
        he[q] = e1[r * ld + (j - j0)];
        ++q;
      }
      if (k2) {
        hi[q] = j;
        hj[q] = i;
        he[q] = e2[r * ld + (j - j0)];
      }
    }
    pos += total;
    cnt += total;
  }
  if (!WRITE && threadIdx.x == 0) counts[r] = cnt;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// "%lld %lld %g\n" for every record.
int write_records(FILE *f, const std::vector<int64_t> &hi, const std::vector<int64_t> &hj,
                  const std::vector<double> &he, int64_t k) {
  std::vector<char> buf;
  buf.reserve(1 << 20);
  char line[96];
  for (int64_t t = 0; t < k; ++t) {
    const int len = snprintf(line, sizeof(line), "%lld %lld %g\n", (long long)hi[t], (long long)hj[t], he[t]);
    buf.insert(buf.end(), line, line + len);
    if (buf.size() > (1u << 20) - 128) {
      if (fwrite(buf.data(), 1, buf.size(), f) != buf.size()) return GMAT_E_ARG;
      buf.clear();
    }
  }
  if (!buf.empty() && fwrite(buf.data(), 1, buf.size(), f) != buf.size()) return GMAT_E_ARG;
  return GMAT_OK;
}

double g_eff_stats[4] = {0, 0, 0, 0};

}  // namespace

extern "C" int gmat_eff_stats(double *out4) {
  GMAT_CHECK(out4, GMAT_E_ARG, "gmat_eff_stats: null");
  for (int k = 0; k < 4; ++k) out4[k] = g_eff_stats[k];
  return GMAT_OK;
}

extern "C" int gmat_eff_scan(gmat_geno *g, int kind, const double *py, const int64_t *rows, int64_t n_rows,
                             const double *eff_cut, const int64_t *freq_i, const int64_t *freq_j,
                             const char *out_file, int64_t *n_hits) {
  GMAT_CHECK(g && py && eff_cut && out_file && (rows || n_rows == 0) && n_rows >= 0, GMAT_E_ARG,
             "gmat_eff_scan: bad arguments");
  GMAT_CHECK(kind == GMAT_AA || kind == GMAT_AD || kind == GMAT_DD, GMAT_E_ARG, "gmat_eff_scan: kind %d", kind);
  GMAT_CHECK(!freq_i == !freq_j, GMAT_E_ARG, "gmat_eff_scan: freq_i and freq_j go together");
  const int64_t n = g->n, m = g->m;
  for (int64_t r = 0; r < n_rows; ++r)
    GMAT_CHECK(rows[r] >= 0 && rows[r] < m, GMAT_E_ARG, "gmat_eff_scan: row %lld outside [0, %lld)",
               (long long)rows[r], (long long)m);
  if (freq_i)
    for (int64_t j = 0; j < m; ++j)
      GMAT_CHECK(freq_i[j] >= 0 && freq_i[j] <= 10 && freq_j[j] >= 0 && freq_j[j] <= 10, GMAT_E_ARG,
                 "gmat_eff_scan: frequency class of SNP %lld outside 0..10", (long long)j);
  const double t0 = now_s();
  FILE *f = fopen(out_file, "w");
  GMAT_CHECK(f, GMAT_E_ARG, "gmat_eff_scan: cannot open %s for writing", out_file);
  struct Closer {
    FILE *f;
    ~Closer() { fclose(f); }
  } closer{f};
  fprintf(f, "%s %s %s\n", "snp_0", "snp_1", "eff");

  const bool need_add = kind != GMAT_DD, need_dom = kind != GMAT_AA;
  DBuf cen, xa, xd, dpy, drows, dcut, dfi, dfj;
  GMAT_TRY(cen.alloc(2 * m * sizeof(double)));
  GMAT_TRY(dpy.alloc(n * sizeof(double)));
  const int n_cut = freq_i ? 111 : 1;
  GMAT_TRY(dcut.alloc(n_cut * sizeof(double)));
  GMAT_HIP(hipMemcpy(dpy.p, py, n * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dcut.p, eff_cut, n_cut * sizeof(double), hipMemcpyHostToDevice));
  if (freq_i) {
    GMAT_TRY(dfi.alloc(m * sizeof(int64_t)));
    GMAT_TRY(dfj.alloc(m * sizeof(int64_t)));
    GMAT_HIP(hipMemcpy(dfi.p, freq_i, m * sizeof(int64_t), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(dfj.p, freq_j, m * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  double *c_add = cen.as<double>(), *c_dom = c_add + m;
  hipLaunchKernelGGL(eff_freq_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, 0, g->packed.as<uint8_t>(), g->nb,
                     n, m, c_add, c_dom);
  GMAT_HIP(hipGetLastError());
  if (need_add) {
    GMAT_TRY(xa.alloc(m * n * sizeof(double)));
    hipLaunchKernelGGL(eff_x_kernel, dim3((unsigned)m), dim3(256), 0, 0, g->packed.as<uint8_t>(), g->nb, n, c_add, 0,
                       xa.as<double>());
    GMAT_HIP(hipGetLastError());
  }
  if (need_dom) {
    GMAT_TRY(xd.alloc(m * n * sizeof(double)));
    hipLaunchKernelGGL(eff_x_kernel, dim3((unsigned)m), dim3(256), 0, 0, g->packed.as<uint8_t>(), g->nb, n, c_dom, 1,
                       xd.as<double>());
    GMAT_HIP(hipGetLastError());
  }
  // first-SNP coding / second-SNP coding of each GEMM
  const double *x1 = kind == GMAT_DD ? xd.as<double>() : xa.as<double>();
  const double *x2 = kind == GMAT_AA ? xa.as<double>() : xd.as<double>();
  const EffCut ec{dcut.as<double>(), dfi.as<int64_t>(), dfj.as<int64_t>()};

  // chunk of R rows: E is R x (m - j0) doubles per orientation, bounded to ~1 GiB
  const int64_t R = std::max<int64_t>(1, std::min<int64_t>(1024, (int64_t)(1ll << 27) / std::max<int64_t>(m, 1)));
  DBuf band, e1, e2, dcnt, doff, bhi, bhj, bhe;
  GMAT_TRY(drows.alloc(R * sizeof(int64_t)));
  GMAT_TRY(band.alloc(R * n * sizeof(double)));
  GMAT_TRY(e1.alloc(R * m * sizeof(double)));
  if (kind == GMAT_AD) GMAT_TRY(e2.alloc(R * m * sizeof(double)));
  GMAT_TRY(dcnt.alloc(R * sizeof(int64_t)));
  GMAT_TRY(doff.alloc(R * sizeof(int64_t)));
  std::vector<int64_t> hcnt(R), hoff(R), hi, hj;
  std::vector<double> he;
  double dev_s = 0.0, write_s = 0.0, pairs = 0.0;
  int64_t total = 0;
  for (int64_t r0 = 0; r0 < n_rows; r0 += R) {
    const double c0 = now_s();
    const int64_t nr = std::min(R, n_rows - r0);
    int64_t imin = m;
    for (int64_t r = 0; r < nr; ++r) {
      imin = std::min(imin, rows[r0 + r]);
      pairs += (double)(m - 1 - rows[r0 + r]) * (kind == GMAT_AD ? 2.0 : 1.0);
    }
    const int64_t j0 = imin + 1, nj = m - j0;
    GMAT_HIP(hipMemcpy(drows.p, rows + r0, nr * sizeof(int64_t), hipMemcpyHostToDevice));
    if (nj > 0) {
      const int64_t ld = nj;
      hipLaunchKernelGGL(eff_band_kernel, dim3((unsigned)cdiv(n, 256), (unsigned)nr), dim3(256), 0, 0, x1, n,
                         drows.as<int64_t>(), dpy.as<double>(), band.as<double>());
      GMAT_HIP(hipGetLastError());
      GMAT_TRY(dgemm(0, nr, nj, n, 1.0, DView{band.as<double>(), n, 0}, DView{x2 + j0 * n, n, 1}, 0.0,
                     e1.as<double>(), ld));
      if (kind == GMAT_AD) {  // (d_i o py) . a_j for the (j, i) orientation
        hipLaunchKernelGGL(eff_band_kernel, dim3((unsigned)cdiv(n, 256), (unsigned)nr), dim3(256), 0, 0,
                           xd.as<double>(), n, drows.as<int64_t>(), dpy.as<double>(), band.as<double>());
        GMAT_HIP(hipGetLastError());
        GMAT_TRY(dgemm(0, nr, nj, n, 1.0, DView{band.as<double>(), n, 0}, DView{xa.as<double>() + j0 * n, n, 1},
                       0.0, e2.as<double>(), ld));
      }
      hipLaunchKernelGGL(eff_compact_kernel<false>, dim3((unsigned)nr), dim3(CT), 0, 0, kind, e1.as<double>(),
                         e2.as<double>(), ld, j0, m, drows.as<int64_t>(), ec, dcnt.as<int64_t>(), nullptr, nullptr,
                         nullptr, nullptr);
      GMAT_HIP(hipGetLastError());
      GMAT_HIP(hipMemcpy(hcnt.data(), dcnt.p, nr * sizeof(int64_t), hipMemcpyDeviceToHost));
      int64_t k = 0;
      for (int64_t r = 0; r < nr; ++r) {
        hoff[r] = k;
        k += hcnt[r];
      }
      if (k > 0) {
        if ((int64_t)(bhi.bytes / sizeof(int64_t)) < k) {
          GMAT_TRY(bhi.alloc(k * sizeof(int64_t)));
          GMAT_TRY(bhj.alloc(k * sizeof(int64_t)));
          GMAT_TRY(bhe.alloc(k * sizeof(double)));
        }
        GMAT_HIP(hipMemcpy(doff.p, hoff.data(), nr * sizeof(int64_t), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(eff_compact_kernel<true>, dim3((unsigned)nr), dim3(CT), 0, 0, kind, e1.as<double>(),
                           e2.as<double>(), ld, j0, m, drows.as<int64_t>(), ec, nullptr, doff.as<int64_t>(),
                           bhi.as<int64_t>(), bhj.as<int64_t>(), bhe.as<double>());
        GMAT_HIP(hipGetLastError());
        hi.resize(k);
        hj.resize(k);
        he.resize(k);
        GMAT_HIP(hipMemcpy(hi.data(), bhi.p, k * sizeof(int64_t), hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(hj.data(), bhj.p, k * sizeof(int64_t), hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(he.data(), bhe.p, k * sizeof(double), hipMemcpyDeviceToHost));
      }
      const double c1 = now_s();
      dev_s += c1 - c0;
      if (k > 0) GMAT_CHECK(write_records(f, hi, hj, he, k) == GMAT_OK, GMAT_E_ARG, "gmat_eff_scan: write to %s failed",
                            out_file);
      write_s += now_s() - c1;
      total += k;
    }
  }
  GMAT_HIP(hipDeviceSynchronize());
  if (n_hits) *n_hits = total;
  g_eff_stats[0] = pairs;
  g_eff_stats[1] = (double)total;
  g_eff_stats[2] = dev_s;
  g_eff_stats[3] = write_s;
  (void)t0;
  return GMAT_OK;
}

extern "C" int gmat_geno_decode(const gmat_geno *g, double *marker_mat) {
  GMAT_CHECK(g && marker_mat, GMAT_E_ARG, "gmat_geno_decode: bad arguments");
  DBuf out;
  GMAT_TRY(out.alloc(g->m * g->n * sizeof(double)));
  hipLaunchKernelGGL(decode_f64_kernel, dim3((unsigned)g->m), dim3(256), 0, 0,
                     g->packed.as<uint8_t>(), g->nb, g->n, out.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpy(marker_mat, out.p, g->m * g->n * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// Single-SNP random SNP-BLUP test quantities (remma_add.py:49-60, remma_dom.py:49-62): for every
// SNP j, x_j = additive (g - 2p) or dominance ([g != 2] g - 2p(1-p)) coding with p = sum/(2n)
// from the exact integer dosage sums; xpy[j] = x_j' py, xpx[j] = x_j' P x_j.  Chunks of SNPs:
// X (C x n fp64, .fam order) from the packed panel, Y = X P (fp64 MFMA dgemm), row dots.
extern "C" int gmat_snp_test(gmat_geno *g, int kind, const double *pvp, const double *py, double *xpy,
                             double *xpx) {
  GMAT_CHECK(g && pvp && py && xpy && xpx, GMAT_E_ARG, "gmat_snp_test: bad arguments");
  GMAT_CHECK(kind == GMAT_GRM_ADD || kind == GMAT_GRM_DOM, GMAT_E_ARG, "gmat_snp_test: unknown kind %d", kind);
  GMAT_CHECK(g->total_missing == 0, GMAT_E_ARG, "gmat_snp_test: panel has %lld missing genotypes (impute first)",
             (long long)g->total_missing);
  const int64_t n = g->n, m = g->m;
  std::vector<double> c(m);
  for (int64_t j = 0; j < m; ++j) {
    const double freq = (double)g->sum_dose[j] / (double)(2 * n);
    c[j] = kind == GMAT_GRM_ADD ? 2 * freq : 2 * freq * (1 - freq);
  }
  const int64_t C = std::max<int64_t>(64, std::min<int64_t>(m, (int64_t)(1ll << 26) / std::max<int64_t>(n, 1)));
  DBuf dc, dp, dpy, x, y, o1, o2;
  GMAT_TRY(dc.alloc(m * sizeof(double)));
  GMAT_TRY(dp.alloc(n * n * sizeof(double)));
  GMAT_TRY(dpy.alloc(n * sizeof(double)));
  GMAT_TRY(x.alloc(C * n * sizeof(double)));
  GMAT_TRY(y.alloc(C * n * sizeof(double)));
  GMAT_TRY(o1.alloc(m * sizeof(double)));
  GMAT_TRY(o2.alloc(m * sizeof(double)));
  GMAT_HIP(hipMemcpy(dc.p, c.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dp.p, pvp, n * n * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dpy.p, py, n * sizeof(double), hipMemcpyHostToDevice));
  for (int64_t j0 = 0; j0 < m; j0 += C) {
    const int64_t nc = std::min(C, m - j0);
    hipLaunchKernelGGL(eff_x_kernel, dim3((unsigned)nc), dim3(256), 0, 0, g->packed.as<uint8_t>() + j0 * g->nb, g->nb,
                       n, dc.as<double>() + j0, kind == GMAT_GRM_DOM ? 1 : 0, x.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(dgemm(0, nc, n, n, 1.0, DView{x.as<double>(), n, 0}, DView{dp.as<double>(), n, 0}, 0.0, y.as<double>(),
                   n));
    GMAT_TRY(dot_rows(0, nc, n, x.as<double>(), n, y.as<double>(), n, o2.as<double>() + j0));
    GMAT_TRY(dot_rows(0, nc, n, x.as<double>(), n, dpy.as<double>(), 0, o1.as<double>() + j0));
  }
  GMAT_HIP(hipMemcpy(xpy, o1.p, m * sizeof(double), hipMemcpyDeviceToHost));
  GMAT_HIP(hipMemcpy(xpx, o2.p, m * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

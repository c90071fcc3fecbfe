// Effect-only epistasis screen (the reference's C kernels remma_epi{AA,AD,DD}(_maf)_eff_cpu,
// _remma_epi_eff_cpu.c:61-574) and the plain .bed decoder read_plink_bed (:10-56).
//
// eff(i, j) = sum_k x_ik x_jk py_k over pairs j > i of the listed first SNPs i, where x is the
// reference's fp64 coding of the 2-bit PLINK code c: v = (c^2 + c)/6 (0, 1/3 missing, 1, 2),
// additive x = v - 2p, dominance x = [v != 2] v - 2p(1-p), with p accumulated exactly as the
// reference does (p += v/(2n) over individuals in .fam order, :103-112 / :277-285 / :459-464).
// A pair is kept when |eff| > eff_cut (AD: >= for the (i, j) orientation, > for (j, i),
// :238/:245), eff_cut from one value or, for the _maf forms, from the 111-entry table at
// freq_i*10 + freq_j (:152, :338, :525).
//
// Two passes, the exact scan's machinery (epi.hip) on the effect alone:
//  1. SCREEN (eff_screen_kernel).  With integer codes c3 = 3v in {0, 1, 3, 6} (dominance {0, 1, 3}),
//     eff = (T - 3 beta_j U_i - 3 alpha_i V_j + 9 alpha_i beta_j 1'py) / 9 with T = (c3_i o py) . c3_j,
//     U_i = c3_i . py, V_j = c3_j . py.  T comes from S = 2 int8 slices of the row image c3_i o py on
//     v_mfma_i32_32x32x32_i8 (exact int32) with the slice-remainder bound
//     |T - T~| <= 128^-(S-1) s_i / 2 sum_k c3_jk, so every pair whose |eff| can reach the cut
//     becomes a candidate (~1 % above the hits at the bench threshold).  64 x 64 (row, column)
//     tiles, 4 waves of 32 x 32, LDS double buffer; candidates appended with one atomic each.
//  2. EXACT (eff_exact_kernel).  Every candidate is recomputed the way the reference's loop does it:
//     sequential over individuals in .fam order, eff += (x_i * x_j) * py_k with separate roundings
//     (no FMA contraction) -- the same fp64 value bit for bit -- and kept with the reference's test.
// Records are ordered as the reference's single-thread loop writes them (rows in list order, j
// ascending, AD (i, j) before (j, i)) and written as "%lld %lld %g" text on the host.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>

#include "dla.h"
#include "geno.h"

namespace {
using namespace gmat;

constexpr int ES = 2;                        // int8 slices of the screen's row images
constexpr int ET = 64, EK = 64, EP = 80;     // tile edge, individuals per stage, LDS pitch

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

// X[j][k] for one coding (dom = 0 additive, 1 dominance); one workgroup per SNP (gmat_snp_test).
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

// Integer codes c3 = 3v of both codings ([m][n_pad], .fam order, zero padding), their sums and
// their py products U = c3 . py (fixed-order reduction); one workgroup per SNP.
__global__ __launch_bounds__(256) void eff_codes_kernel(const uint8_t *packed, int64_t nb, int64_t n, int64_t n_pad,
                                                        const double *py, int8_t *ca, int8_t *cd, double *sa, double *sd,
                                                        double *ua, double *ud) {
  const int64_t j = blockIdx.x;
  const uint8_t *p = packed + j * nb;
  __shared__ double r[4][256];
  double s1 = 0, s2 = 0, u1 = 0, u2 = 0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) {
    int a = 0;
    if (k < n) {
      const int c = (p[k >> 2] >> (2 * (k & 3))) & 3;
      a = (c * c + c) / 2;  // 0, 1 (missing), 3, 6
    }
    const int d = a == 6 ? 0 : a;
    ca[j * n_pad + k] = (int8_t)a;
    cd[j * n_pad + k] = (int8_t)d;
    const double pk = k < n ? py[k] : 0.0;
    s1 += a;
    s2 += d;
    u1 += a * pk;
    u2 += d * pk;
  }
  r[0][threadIdx.x] = s1;
  r[1][threadIdx.x] = s2;
  r[2][threadIdx.x] = u1;
  r[3][threadIdx.x] = u2;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off)
      for (int q = 0; q < 4; ++q) r[q][threadIdx.x] += r[q][threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    sa[j] = r[0][0];
    sd[j] = r[1][0];
    ua[j] = r[2][0];
    ud[j] = r[3][0];
  }
}

// Row images of the listed rows: L = c3 o py quantised to ES int8 slices with scale s = max|L|/127;
// one workgroup per listed row (rows[r]), slices at stride ss.
__global__ __launch_bounds__(256) void eff_rowimg_kernel(int64_t n_pad, const int8_t *codes, const int64_t *rows,
                                                         const double *py, int64_t ss, int8_t *img, double *scale) {
  const int64_t r = blockIdx.x, j = rows[r];
  const int8_t *c = codes + j * n_pad;
  __shared__ double red[256];
  double mx = 0.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) mx = fmax(mx, fabs((double)c[k] * py[k]));
  red[threadIdx.x] = mx;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + off]);
    __syncthreads();
  }
  const double sc = red[0] > 0.0 ? red[0] / 127.0 : 1.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) {
    double v = (double)c[k] * py[k] / sc;
    for (int t = 0; t < ES; ++t) {
      const double q = fmin(127.0, fmax(-127.0, rint(v)));
      img[t * ss + r * n_pad + k] = (int8_t)q;
      v = (v - q) * 128.0;
    }
  }
  if (threadIdx.x == 0) scale[r] = sc;
}

struct EffArgs {
  int kind;
  int64_t n_pad, m, n_rows;   // listed (unique, ascending) rows of this launch
  const int64_t *rows;
  const int8_t *img1, *img2;  // row images (slices at stride ss): orientation 0 (and 1 for AD)
  int64_t ss;
  const double *sc1, *sc2;    // their scales [n_rows]
  const int8_t *col1, *col2;  // column codes [m][n_pad]: orientation 0 (and 1)
  const double *cen1, *cen2;  // row-side centring (alpha) of orientation 0 / 1, by SNP
  const double *cenc1, *cenc2;  // column-side centring (beta)
  const double *u1, *u2;      // row-side c3 . py, by SNP
  const double *v1, *v2;      // column-side c3 . py
  const double *cs1, *cs2;    // column-side code sums
  double spy;
  const double *cut;          // 1 or 111 entries
  const int64_t *fi, *fj;     // frequency classes (null: single cut)
  unsigned long long *counter;
  int64_t cap;
  int64_t *cand;              // (row index << 32) | (j << 1) | orientation
  int n_rt;
};

template <int NO>  // orientations (1: AA / DD, 2: AD)
__global__ __launch_bounds__(256, 2) void eff_screen_kernel(EffArgs x) {
  const int nwg = (int)gridDim.x, xq = nwg / 8, xr = nwg % 8, xcd = (int)blockIdx.x % 8;
  const int tile = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (int)blockIdx.x / 8;
  const int rt = tile % x.n_rt, ct = tile / x.n_rt;
  const int r0 = rt * ET;
  const int64_t jlo = x.rows[0] + 1;
  const int64_t c0 = (jlo / 32) * 32 + (int64_t)ct * ET;
  if (r0 >= x.n_rows || c0 >= x.m) return;
  if (c0 + ET - 1 <= x.rows[r0]) return;  // left of the diagonal: no pair j > i
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1, h = lane >> 5, c = lane & 31;
  constexpr int NR = ES * NO, NC = NO;
  __shared__ __attribute__((aligned(16))) int8_t sR[2][NR][ET * EP];
  __shared__ __attribute__((aligned(16))) int8_t sC[2][NC][ET * EP];
  const int srow = tid >> 2, spc = (tid & 3) * 16;
  const int64_t rr = min(r0 + srow, (int)x.n_rows - 1);
  const int64_t sj = min(c0 + srow, x.m - 1);
  const int8_t *rsrc[NR];
  const int8_t *csrc[NC];
#pragma unroll
  for (int o = 0; o < NO; ++o) {
#pragma unroll
    for (int t = 0; t < ES; ++t) rsrc[o * ES + t] = (o ? x.img2 : x.img1) + t * x.ss + rr * x.n_pad;
    csrc[o] = (o ? x.col2 : x.col1) + sj * x.n_pad;
  }
  v16i acc[NR];
#pragma unroll
  for (int p = 0; p < NR; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0;
  // per-row epilogue operands staged in LDS while the K loop runs (the candidate stores would
  // otherwise force a reload of every operand per element): [o][r] scale, centring, c3 . py, and
  // the row's SNP index and frequency class
  __shared__ double eR[NO][3][ET];
  __shared__ int64_t eI[ET];
  __shared__ int64_t eF[ET];
  if (tid < ET) {
    const int r = min(r0 + tid, (int)x.n_rows - 1);
    const int64_t i = x.rows[r];
    eI[tid] = i;
    eF[tid] = x.fi ? x.fi[i] : 0;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      eR[o][0][tid] = (o ? x.sc2 : x.sc1)[r];
      eR[o][1][tid] = (o ? x.cen2 : x.cen1)[i];
      eR[o][2][tid] = (o ? x.u2 : x.u1)[i];
    }
  }
  v4i rv[NR], cv[NC];
  auto load = [&](int64_t k0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NR; ++u) rv[u] = *(const v4i *)(rsrc[u] + k0 + spc);
#pragma unroll
    for (int u = 0; u < NC; ++u) cv[u] = *(const v4i *)(csrc[u] + k0 + spc);
  };
  auto store = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NR; ++u) *(v4i *)&sR[b][u][srow * EP + spc] = rv[u];
#pragma unroll
    for (int u = 0; u < NC; ++u) *(v4i *)&sC[b][u][srow * EP + spc] = cv[u];
  };
  load(0);
  store(0);
  __syncthreads();
  int b = 0;
  for (int64_t k0 = 0; k0 < x.n_pad; k0 += EK) {
    const bool more = k0 + EK < x.n_pad;
    if (more) load(k0 + EK);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4i fc[NC];
#pragma unroll
      for (int u = 0; u < NC; ++u) fc[u] = *(const v4i *)&sC[b][u][(32 * wc + c) * EP + 32 * kk + 16 * h];
#pragma unroll
      for (int u = 0; u < NR; ++u) {
        const v4i fr = *(const v4i *)&sR[b][u][(32 * wr + c) * EP + 32 * kk + 16 * h];
        acc[u] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fr, fc[u / ES], acc[u], 0, 0, 0);
      }
    }
    if (more) store(b ^ 1);
    __syncthreads();
    b ^= 1;
  }
  // epilogue: lane (c, h) holds rows 32 wr + (e & 3) + 8 (e >> 2) + 4h, column 32 wc + c
  const int64_t j = c0 + 32 * wc + c;
  if (j >= x.m) return;
  constexpr double rem = (ES == 1 ? 0.5 : ES == 2 ? 0.5 / 128.0 : 0.5 / 16384.0) * (1.0 + 1e-9);
  // per-column operands in registers (the lane's column is fixed)
  double cbe[NO], cv3[NO], ccs[NO];
#pragma unroll
  for (int o = 0; o < NO; ++o) {
    cbe[o] = (o ? x.cenc2 : x.cenc1)[j];
    cv3[o] = (o ? x.v2 : x.v1)[j];
    ccs[o] = (o ? x.cs2 : x.cs1)[j];
  }
  const int64_t fjj = x.fi ? x.fj[j] : 0;
  const double cut0 = x.cut[0];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int rl = 32 * wr + (e & 3) + 8 * (e >> 2) + 4 * h, r = r0 + rl;
    if (r >= x.n_rows) continue;
    const int64_t i = eI[rl];
    if (j <= i) continue;
    const double cut = x.fi ? x.cut[eF[rl] * 10 + fjj] : cut0;
#pragma unroll
    for (int o = 0; o < NO; ++o) {
      double t = 0.0;
#pragma unroll
      for (int q = ES - 1; q >= 0; --q) t = t * (1.0 / 128.0) + (double)acc[o * ES + q][e];
      const double s = eR[o][0][rl], al = eR[o][1][rl], be = cbe[o];
      const double T = s * t, t2 = 3.0 * be * eR[o][2][rl], t3 = 3.0 * al * cv3[o], t4 = 9.0 * al * be * x.spy;
      const double eff = (T - t2 - t3 + t4) / 9.0;
      const double bnd = (rem * s * ccs[o] + 1e-9 * (fabs(T) + fabs(t2) + fabs(t3) + fabs(t4))) / 9.0;
      if (fabs(eff) + bnd >= cut * (1.0 - 1e-12)) {
        const unsigned long long k = atomicAdd(x.counter, 1ULL);
        if ((int64_t)k < x.cap) x.cand[k] = ((int64_t)r << 32) | ((int64_t)j << 1) | o;
      }
    }
  }
}

// The reference's arithmetic for each candidate: x = v - centre, eff += (x_i * x_j) * py_k in .fam
// order with separate roundings; keep[t] = the reference's threshold test.
__global__ void eff_exact_kernel(int kind, int64_t count, const int64_t *cand, const int64_t *rows, int64_t n,
                                 int64_t n_pad, const int8_t *ca, const int8_t *cd, const double *c_add,
                                 const double *c_dom, const double *py, const double *cut, const int64_t *fi,
                                 const int64_t *fj, double *eff, uint8_t *keep) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= count) return;
  const int64_t code = cand[t];
  const int64_t i = rows[code >> 32], j = (code & 0xFFFFFFFFll) >> 1;
  const int o = (int)(code & 1);
  // first factor: the row SNP's coding (AA: A, DD: D, AD: A for o = 0, D for o = 1)
  const bool left_dom = kind == GMAT_DD || (kind == GMAT_AD && o == 1);
  const bool right_dom = kind == GMAT_DD || (kind == GMAT_AD && o == 0);
  const int8_t *pi = (left_dom ? cd : ca) + i * n_pad, *pj = (right_dom ? cd : ca) + j * n_pad;
  const double ci = left_dom ? c_dom[i] : c_add[i], cj = right_dom ? c_dom[j] : c_add[j];
  // x = v - centre takes one of four values per SNP (c3 = 3v in {0, 1, 3, 6}): each is the same
  // correctly rounded __dsub_rn((double)c3 / 3.0, centre) the loop computed per individual, so the
  // sum below is bit-identical; the codes are read 16 per load (rows are 16-byte aligned)
  const double i0 = __dsub_rn(0.0, ci), i1 = __dsub_rn(1.0 / 3.0, ci), i3 = __dsub_rn(1.0, ci), i6 = __dsub_rn(2.0, ci);
  const double j0 = __dsub_rn(0.0, cj), j1 = __dsub_rn(1.0 / 3.0, cj), j3 = __dsub_rn(1.0, cj), j6 = __dsub_rn(2.0, cj);
  auto xv = [](int c3, double v0, double v1, double v3, double v6) __attribute__((always_inline)) {
    return c3 == 0 ? v0 : c3 == 1 ? v1 : c3 == 3 ? v3 : v6;
  };
  double e = 0.0;
  for (int64_t k0 = 0; k0 < n; k0 += 16) {
    const v4i a4 = *(const v4i *)(pi + k0), b4 = *(const v4i *)(pj + k0);
    const int kn = (int)min((int64_t)16, n - k0);
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      if (q >= kn) break;
      const int ca3 = (int)(int8_t)(a4[q >> 2] >> (8 * (q & 3))), cb3 = (int)(int8_t)(b4[q >> 2] >> (8 * (q & 3)));
      const double xi = xv(ca3, i0, i1, i3, i6), xj = xv(cb3, j0, j1, j3, j6);
      e = __dadd_rn(e, __dmul_rn(__dmul_rn(xi, xj), py[k0 + q]));
    }
  }
  const double c = fi ? cut[fi[i] * 10 + fj[j]] : cut[0];
  eff[t] = e;
  keep[t] = (kind == GMAT_AD && o == 0) ? (fabs(e) >= c) : (fabs(e) > c);
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
  GMAT_CHECK(m < (1ll << 30), GMAT_E_ARG, "gmat_eff_scan: at most 2^30 SNPs");
  for (int64_t r = 0; r < n_rows; ++r)
    GMAT_CHECK(rows[r] >= 0 && rows[r] < m, GMAT_E_ARG, "gmat_eff_scan: row %lld outside [0, %lld)",
               (long long)rows[r], (long long)m);
  if (freq_i)
    for (int64_t j = 0; j < m; ++j)
      GMAT_CHECK(freq_i[j] >= 0 && freq_i[j] <= 10 && freq_j[j] >= 0 && freq_j[j] <= 10, GMAT_E_ARG,
                 "gmat_eff_scan: frequency class of SNP %lld outside 0..10", (long long)j);
  FILE *f = fopen(out_file, "w");
  GMAT_CHECK(f, GMAT_E_ARG, "gmat_eff_scan: cannot open %s for writing", out_file);
  struct Closer {
    FILE *f;
    ~Closer() { fclose(f); }
  } closer{f};
  fprintf(f, "%s %s %s\n", "snp_0", "snp_1", "eff");
  const double t_dev0 = now_s();
  // unique ascending rows (the list may be unsorted or hold duplicates; records are replayed in
  // list order at the end)
  std::vector<int64_t> urows(rows, rows + n_rows);
  std::sort(urows.begin(), urows.end());
  urows.erase(std::unique(urows.begin(), urows.end()), urows.end());
  const int64_t nu = (int64_t)urows.size();
  const int64_t n_pad = round_up(n, EK);
  DBuf cen, dpy, ca, cd, sums, dcut, dfi, dfj;
  GMAT_TRY(cen.alloc(2 * m * sizeof(double)));
  GMAT_TRY(dpy.alloc(n_pad * sizeof(double)));
  GMAT_TRY(ca.alloc((size_t)m * n_pad));
  GMAT_TRY(cd.alloc((size_t)m * n_pad));
  GMAT_TRY(sums.alloc(4 * m * sizeof(double)));
  const int n_cut = freq_i ? 111 : 1;
  GMAT_TRY(dcut.alloc(n_cut * sizeof(double)));
  GMAT_HIP(hipMemset(dpy.p, 0, n_pad * sizeof(double)));
  GMAT_HIP(hipMemcpy(dpy.p, py, n * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dcut.p, eff_cut, n_cut * sizeof(double), hipMemcpyHostToDevice));
  if (freq_i) {
    GMAT_TRY(dfi.alloc(m * sizeof(int64_t)));
    GMAT_TRY(dfj.alloc(m * sizeof(int64_t)));
    GMAT_HIP(hipMemcpy(dfi.p, freq_i, m * sizeof(int64_t), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(dfj.p, freq_j, m * sizeof(int64_t), hipMemcpyHostToDevice));
  }
  double *c_add = cen.as<double>(), *c_dom = c_add + m;
  double *s_a = sums.as<double>(), *s_d = s_a + m, *u_a = s_d + m, *u_d = u_a + m;
  hipLaunchKernelGGL(eff_freq_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, 0, g->packed.as<uint8_t>(), g->nb,
                     n, m, c_add, c_dom);
  hipLaunchKernelGGL(eff_codes_kernel, dim3((unsigned)m), dim3(256), 0, 0, g->packed.as<uint8_t>(), g->nb, n, n_pad,
                     dpy.as<double>(), ca.as<int8_t>(), cd.as<int8_t>(), s_a, s_d, u_a, u_d);
  GMAT_HIP(hipGetLastError());
  double spy = 0.0;
  for (int64_t k = 0; k < n; ++k) spy += py[k];
  // orientation 0: (row coding, column coding) = AA (A, A), DD (D, D), AD (A, D); AD orientation 1 = (D, A)
  const bool r0dom = kind == GMAT_DD, c0dom = kind != GMAT_AA;
  const int NO = kind == GMAT_AD ? 2 : 1;
  // listed rows per launch (GMAT_EFF_RL): large launches keep the GPU full as j > i shrinks the
  // column range of the later ones, and cost fewer host round trips
  const int64_t RL = getenv("GMAT_EFF_RL") ? std::max<int64_t>(64, atoll(getenv("GMAT_EFF_RL"))) : 2048;
  DBuf drows, img, sc, cnt, cand, deff, dkeep;
  GMAT_TRY(drows.alloc(RL * sizeof(int64_t)));
  GMAT_TRY(img.alloc((size_t)NO * ES * RL * n_pad));
  GMAT_TRY(sc.alloc(2 * RL * sizeof(double)));
  GMAT_TRY(cnt.alloc(8));
  int64_t cap = 1 << 20;
  GMAT_TRY(cand.alloc(cap * 8));
  GMAT_TRY(deff.alloc(cap * 8));
  GMAT_TRY(dkeep.alloc(cap));
  // kept records: unique-row index, j, orientation, eff
  std::vector<int64_t> rec_u, rec_j;
  std::vector<uint8_t> rec_o;
  std::vector<double> rec_e;
  std::vector<int64_t> hcand;
  std::vector<double> heff;
  std::vector<uint8_t> hkeep;
  double pairs = 0.0;
  for (int64_t u0 = 0; u0 < nu; u0 += RL) {
    const int64_t nr = std::min(RL, nu - u0);
    if (urows[u0] + 1 >= m) break;  // no pair j > i left
    for (int64_t r = 0; r < nr; ++r) pairs += (double)(m - 1 - urows[u0 + r]) * NO;
    GMAT_HIP(hipMemcpy(drows.p, urows.data() + u0, nr * sizeof(int64_t), hipMemcpyHostToDevice));
    const int64_t ss = RL * n_pad;
    for (int o = 0; o < NO; ++o) {
      const bool rdom = o ? true : r0dom;
      hipLaunchKernelGGL(eff_rowimg_kernel, dim3((unsigned)nr), dim3(256), 0, 0, n_pad, rdom ? cd.as<int8_t>() : ca.as<int8_t>(),
                         drows.as<int64_t>(), dpy.as<double>(), ss, img.as<int8_t>() + (int64_t)o * ES * ss,
                         sc.as<double>() + o * RL);
    }
    GMAT_HIP(hipGetLastError());
    EffArgs x;
    x.kind = kind;
    x.n_pad = n_pad;
    x.m = m;
    x.n_rows = nr;
    x.rows = drows.as<int64_t>();
    x.ss = ss;
    x.img1 = img.as<int8_t>();
    x.img2 = img.as<int8_t>() + ES * ss;
    x.sc1 = sc.as<double>();
    x.sc2 = sc.as<double>() + RL;
    x.col1 = c0dom ? cd.as<int8_t>() : ca.as<int8_t>();
    x.col2 = ca.as<int8_t>();
    x.cen1 = r0dom ? c_dom : c_add;
    x.cen2 = c_dom;
    x.cenc1 = c0dom ? c_dom : c_add;
    x.cenc2 = c_add;
    x.u1 = r0dom ? u_d : u_a;
    x.u2 = u_d;
    x.v1 = c0dom ? u_d : u_a;
    x.v2 = u_a;
    x.cs1 = c0dom ? s_d : s_a;
    x.cs2 = s_a;
    x.spy = spy;
    x.cut = dcut.as<double>();
    x.fi = freq_i ? dfi.as<int64_t>() : nullptr;
    x.fj = freq_i ? dfj.as<int64_t>() : nullptr;
    x.counter = cnt.as<unsigned long long>();
    x.n_rt = (int)cdiv(nr, ET);
    const int64_t jlo = urows[u0] + 1, ncols = m - (jlo / 32) * 32;
    const unsigned grid = (unsigned)(x.n_rt * cdiv(ncols, ET));
    unsigned long long count = 0;
    for (;;) {
      x.cap = cap;
      x.cand = cand.as<int64_t>();
      GMAT_HIP(hipMemset(cnt.p, 0, 8));
      if (NO == 2)
        hipLaunchKernelGGL(eff_screen_kernel<2>, dim3(grid), dim3(256), 0, 0, x);
      else
        hipLaunchKernelGGL(eff_screen_kernel<1>, dim3(grid), dim3(256), 0, 0, x);
      GMAT_HIP(hipGetLastError());
      GMAT_HIP(hipMemcpy(&count, cnt.p, 8, hipMemcpyDeviceToHost));
      if ((int64_t)count <= cap) break;
      cap = (int64_t)(1.25 * (double)count) + 1024;  // a small eff_cut: grow and redo the launch
      GMAT_TRY(cand.alloc(cap * 8));
      GMAT_TRY(deff.alloc(cap * 8));
      GMAT_TRY(dkeep.alloc(cap));
    }
    if (count == 0) continue;
    const int64_t k = (int64_t)count;
    hipLaunchKernelGGL(eff_exact_kernel, dim3((unsigned)cdiv(k, 128)), dim3(128), 0, 0, kind, k, cand.as<int64_t>(),
                       drows.as<int64_t>(), n, n_pad, ca.as<int8_t>(), cd.as<int8_t>(), c_add, c_dom, dpy.as<double>(),
                       dcut.as<double>(), x.fi, x.fj, deff.as<double>(), dkeep.as<uint8_t>());
    GMAT_HIP(hipGetLastError());
    hcand.resize(k);
    heff.resize(k);
    hkeep.resize(k);
    GMAT_HIP(hipMemcpy(hcand.data(), cand.p, k * 8, hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(heff.data(), deff.p, k * 8, hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(hkeep.data(), dkeep.p, k, hipMemcpyDeviceToHost));
    for (int64_t t = 0; t < k; ++t) {
      if (!hkeep[t]) continue;
      rec_u.push_back(u0 + (hcand[t] >> 32));
      rec_j.push_back((hcand[t] & 0xFFFFFFFFll) >> 1);
      rec_o.push_back((uint8_t)(hcand[t] & 1));
      rec_e.push_back(heff[t]);
    }
  }
  // the reference's single-thread order: per listed row (list order, duplicates replayed), j
  // ascending, (i, j) before (j, i)
  std::vector<int64_t> ord(rec_u.size());
  for (size_t t = 0; t < ord.size(); ++t) ord[t] = (int64_t)t;
  std::sort(ord.begin(), ord.end(), [&](int64_t a, int64_t b) {
    if (rec_u[a] != rec_u[b]) return rec_u[a] < rec_u[b];
    if (rec_j[a] != rec_j[b]) return rec_j[a] < rec_j[b];
    return rec_o[a] < rec_o[b];
  });
  std::vector<int64_t> start(nu + 1, 0);
  for (int64_t t : ord) start[rec_u[t] + 1]++;
  for (int64_t u = 0; u < nu; ++u) start[u + 1] += start[u];
  std::vector<int64_t> hi, hj;
  std::vector<double> he;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t u = std::lower_bound(urows.begin(), urows.end(), rows[r]) - urows.begin();
    for (int64_t q = start[u]; q < start[u + 1]; ++q) {
      const int64_t t = ord[q];
      const int64_t i = urows[u], j = rec_j[t];
      hi.push_back(rec_o[t] ? j : i);
      hj.push_back(rec_o[t] ? i : j);
      he.push_back(rec_e[t]);
    }
  }
  GMAT_HIP(hipDeviceSynchronize());
  const double t_dev = now_s() - t_dev0;
  const double t_w0 = now_s();
  GMAT_CHECK(write_records(f, hi, hj, he, (int64_t)hi.size()) == GMAT_OK, GMAT_E_ARG,
             "gmat_eff_scan: write to %s failed", out_file);
  if (n_hits) *n_hits = (int64_t)hi.size();
  g_eff_stats[0] = pairs;
  g_eff_stats[1] = (double)hi.size();
  g_eff_stats[2] = t_dev;
  g_eff_stats[3] = now_s() - t_w0;
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

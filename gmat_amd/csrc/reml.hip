// Weighted EM-AI REML (the loop of _wemai_multi_gmat, uvlmm_varcom.py:41-99) with every
// O(n^2)/O(n^3) step on the device, and the P / Py projection used by the scans
// (remma_epiAA.py:33-49).
//
// Per iteration: V = s_e I + sum_k s_k ZG_kZ' (combine kernel), V = LL' (blocked
// Cholesky; log|V| from diag L), V^-1 = L^-T L^-1, P = V^-1 - V^-1X (X'V^-1X)^-1 X'V^-1,
// Py, the traces tr(P ZG_kZ') as elementwise sums sum_ab P_ab (ZG_kZ')_ab (O(n^2) instead of
// the reference's O(n^3) np.trace(np.dot(P, ZGZ)) at :66), W = [ZG_kZ'Py..., Py] and
// AI = W'PW/2.  The (c+1)-sized EM/AI weight search and the convergence test run on the
// host exactly as :78-99.
#include <chrono>
#include <cmath>

#include "dla.h"

using namespace gmat;

namespace {

constexpr int MAXG = 16;
struct Coefs {
  const double *g[MAXG];
  double s[MAXG];
  int c;
  double diag;
};

__global__ void combine_kernel(int64_t n, Coefs k, double *v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * n) return;
  double acc = (i / n == i % n) ? k.diag : 0.0;
  for (int t = 0; t < k.c; ++t) acc += k.g[t][i] * k.s[t];
  v[i] = acc;
}

// out[r][s] = g[col[r]][col[s]]  (Z G Z' for an incidence Z)
__global__ void zgz_kernel(int64_t n, int64_t n_id, const int64_t *col, const double *g, double *out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * n) return;
  out[i] = g[col[i / n] * n_id + col[i % n]];
}

// pvp[a][b] = sum_{r in rec(a)} sum_{s in rec(b)} P[r][s];  py[a] = sum_{r in rec(a)} Py[r]
__global__ void ztpz_kernel(int64_t n, int64_t n_id, const int64_t *off, const int64_t *rec, const double *p,
                            double *pvp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_id * n_id) return;
  const int64_t a = i / n_id, b = i % n_id;
  double acc = 0.0;
  for (int64_t u = off[a]; u < off[a + 1]; ++u)
    for (int64_t v = off[b]; v < off[b + 1]; ++v) acc += p[rec[u] * n + rec[v]];
  pvp[i] = acc;
}

// sum of the diagonal in a fixed order (one wave)
__global__ void trace_kernel(int64_t n, const double *a, double *out) {
  double s = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 64) s += a[i * n + i];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (threadIdx.x == 0) *out = s;
}

__global__ void copy_kernel(int64_t n, const double *src, double *dst) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// host Gauss-Jordan inverse with partial pivoting (sizes here are the covariate count and
// the number of variance components); returns log|det| through *logabsdet.
bool small_inverse(int n, const double *a, double *inv, double *logabsdet) {
  std::vector<double> m(a, a + n * n);
  for (int i = 0; i < n * n; ++i) inv[i] = 0.0;
  for (int i = 0; i < n; ++i) inv[i * n + i] = 1.0;
  double ld = 0.0;
  for (int c = 0; c < n; ++c) {
    int piv = c;
    for (int r = c + 1; r < n; ++r)
      if (std::fabs(m[r * n + c]) > std::fabs(m[piv * n + c])) piv = r;
    if (m[piv * n + c] == 0.0) return false;
    if (piv != c)
      for (int k = 0; k < n; ++k) {
        std::swap(m[c * n + k], m[piv * n + k]);
        std::swap(inv[c * n + k], inv[piv * n + k]);
      }
    const double d = m[c * n + c];
    ld += std::log(std::fabs(d));
    for (int k = 0; k < n; ++k) {
      m[c * n + k] /= d;
      inv[c * n + k] /= d;
    }
    for (int r = 0; r < n; ++r) {
      if (r == c) continue;
      const double f = m[r * n + c];
      if (f == 0.0) continue;
      for (int k = 0; k < n; ++k) {
        m[r * n + k] -= f * m[c * n + k];
        inv[r * n + k] -= f * inv[c * n + k];
      }
    }
  }
  if (logabsdet) *logabsdet = ld;
  return true;
}

struct Model {
  int64_t n = 0, p = 0, n_id = 0;
  int c = 0;
  hipStream_t s = 0;
  std::vector<DBuf> zg;
  DBuf v, dinv, work, vi, x, vx, t, pm, y, py, w, pw, small, rowbuf, col;
  std::vector<double> h_trace;

  int setup(int64_t n_rec, int64_t n_fix, int64_t nid, int n_gmat, const double *hy, const double *hx,
            const int64_t *z_col, const double *const *gmat) {
    n = n_rec;
    p = n_fix;
    n_id = nid;
    c = n_gmat;
    GMAT_CHECK(c >= 0 && c <= MAXG, GMAT_E_ARG, "REML: at most %d relationship matrices", MAXG);
    GMAT_CHECK(n > 0 && p > 0 && n_id > 0, GMAT_E_ARG, "REML: bad sizes");
    zg = std::vector<DBuf>(c);
    const size_t nn = (size_t)n * n * sizeof(double);
    GMAT_TRY(v.alloc(nn));
    GMAT_TRY(vi.alloc(nn));
    GMAT_TRY(pm.alloc(nn));
    GMAT_TRY(dinv.alloc((size_t)n * 64 * sizeof(double)));
    GMAT_TRY(work.alloc(((size_t)n * n + 64 * (size_t)n) * sizeof(double)));
    GMAT_TRY(x.alloc((size_t)n * p * sizeof(double)));
    GMAT_TRY(vx.alloc((size_t)n * p * sizeof(double)));
    GMAT_TRY(t.alloc((size_t)n * p * sizeof(double)));
    GMAT_TRY(y.alloc((size_t)n * sizeof(double)));
    GMAT_TRY(py.alloc((size_t)n * sizeof(double)));
    GMAT_TRY(w.alloc((size_t)n * (c + 1) * sizeof(double)));
    GMAT_TRY(pw.alloc((size_t)n * (c + 1) * sizeof(double)));
    GMAT_TRY(small.alloc(4096 * sizeof(double)));
    GMAT_TRY(rowbuf.alloc((size_t)n * (c + 1) * sizeof(double)));
    GMAT_TRY(col.alloc((size_t)n * sizeof(int64_t)));
    GMAT_HIP(hipMemcpy(x.p, hx, (size_t)n * p * sizeof(double), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(y.p, hy, (size_t)n * sizeof(double), hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(col.p, z_col, (size_t)n * sizeof(int64_t), hipMemcpyHostToDevice));
    DBuf g;
    GMAT_TRY(g.alloc((size_t)n_id * n_id * sizeof(double)));
    for (int k = 0; k < c; ++k) {
      GMAT_TRY(zg[k].alloc(nn));
      GMAT_HIP(hipMemcpy(g.p, gmat[k], (size_t)n_id * n_id * sizeof(double), hipMemcpyHostToDevice));
      hipLaunchKernelGGL(zgz_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, n, n_id, col.as<int64_t>(),
                         g.as<double>(), zg[k].as<double>());
      GMAT_HIP(hipGetLastError());
    }
    return GMAT_OK;
  }

  // P and Py for variance vector var (c+1 entries).  *ll_v = log|V|.
  int projection(const double *var, double *ll_v) {
    Coefs k{};
    k.c = c;
    k.diag = var[c];
    for (int t2 = 0; t2 < c; ++t2) {
      k.g[t2] = zg[t2].as<double>();
      k.s[t2] = var[t2];
    }
    hipLaunchKernelGGL(combine_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, n, k, v.as<double>());
    GMAT_HIP(hipGetLastError());
    double *dl = small.as<double>();
    int *info = reinterpret_cast<int *>(small.as<double>() + 1);
    // V = LL' with L^-1 (work) and V^-1 = L^-T L^-1 (vi) built beside the factorisation
    GMAT_TRY(cholesky_inverse(s, n, v.as<double>(), n, dinv.as<double>(), dl, info, work.as<double>(), vi.as<double>()));
    double hdl[2];
    GMAT_HIP(hipMemcpyAsync(hdl, small.p, 2 * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipStreamSynchronize(s));
    int hinfo;
    memcpy(&hinfo, &hdl[1], sizeof(int));
    GMAT_CHECK(hinfo == 0, GMAT_E_NOTPD, "V is not positive definite (pivot %d)", hinfo);
    if (ll_v) *ll_v = hdl[0];
    // VX = V^-1 X ; XVX = X' VX
    GMAT_TRY(dgemm(s, n, p, n, 1.0, DView{vi.as<double>(), n, 0}, DView{x.as<double>(), p, 0}, 0.0, vx.as<double>(), p));
    double *dxvx = small.as<double>() + 8;
    GMAT_CHECK(p * p <= 1024, GMAT_E_ARG, "too many fixed effects (%lld)", (long long)p);
    GMAT_TRY(dgemm(s, p, p, n, 1.0, DView{x.as<double>(), p, 1}, DView{vx.as<double>(), p, 0}, 0.0, dxvx, p));
    std::vector<double> xvx(p * p), xvxi(p * p);
    GMAT_HIP(hipMemcpyAsync(xvx.data(), dxvx, p * p * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipStreamSynchronize(s));
    GMAT_CHECK(small_inverse((int)p, xvx.data(), xvxi.data(), nullptr), GMAT_E_NOTPD, "X'V^-1X is singular");
    double *dxi = small.as<double>() + 8 + 1024;
    GMAT_HIP(hipMemcpyAsync(dxi, xvxi.data(), p * p * sizeof(double), hipMemcpyHostToDevice, s));
    // T = VX * XVX^-1 ; P = V^-1 - T VX'
    GMAT_TRY(dgemm(s, n, p, p, 1.0, DView{vx.as<double>(), p, 0}, DView{dxi, p, 0}, 0.0, t.as<double>(), p));
    hipLaunchKernelGGL(copy_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, n * n, vi.as<double>(),
                       pm.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(dgemm(s, n, n, p, -1.0, DView{t.as<double>(), p, 0}, DView{vx.as<double>(), p, 1}, 1.0, pm.as<double>(), n));
    // Py
    GMAT_TRY(dgemm(s, n, 1, n, 1.0, DView{pm.as<double>(), n, 0}, DView{y.as<double>(), 1, 0}, 0.0, py.as<double>(), 1));
    return GMAT_OK;
  }

  // gradient fd (c+1) and AI matrix ((c+1)^2) at the current P, Py: every device product is queued
  // first and the results come back in one transfer (one host synchronisation per call).
  int derivatives(double *fd, double *ai) {
    const int c1 = c + 1;
    for (int k = 0; k < c; ++k) {
      // tr(P ZGZ') = sum_ab P_ab (ZGZ')_ab   (both symmetric): row sums into rowbuf[k]
      GMAT_TRY(dot_rows(s, n, n, pm.as<double>(), n, zg[k].as<double>(), n, rowbuf.as<double>() + k * n));
      // W[:,k] = ZGZ' Py
      GMAT_TRY(dgemm(s, n, 1, n, 1.0, DView{zg[k].as<double>(), n, 0}, DView{py.as<double>(), 1, 0}, 0.0,
                     w.as<double>() + k, c1));
    }
    hipLaunchKernelGGL(trace_kernel, dim3(1), dim3(64), 0, s, n, pm.as<double>(), rowbuf.as<double>() + c * n);
    GMAT_HIP(hipGetLastError());
    // W[:,c] = Py
    GMAT_TRY(dgemm(s, n, 1, 1, 1.0, DView{py.as<double>(), 1, 0}, DView{small.as<double>() + 3000, 1, 0}, 0.0,
                   w.as<double>() + c, c1));
    // AI = 0.5 W' P W
    GMAT_TRY(dgemm(s, n, c1, n, 1.0, DView{pm.as<double>(), n, 0}, DView{w.as<double>(), c1, 0}, 0.0,
                   pw.as<double>(), c1));
    double *dai = small.as<double>() + 2200;
    GMAT_TRY(dgemm(s, c1, c1, n, 0.5, DView{w.as<double>(), c1, 1}, DView{pw.as<double>(), c1, 0}, 0.0, dai, c1));
    std::vector<double> rows((size_t)n * c + 1), hw((size_t)n * c1);
    GMAT_HIP(hipMemcpyAsync(rows.data(), rowbuf.p, ((size_t)n * c + 1) * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipMemcpyAsync(hw.data(), w.p, hw.size() * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipMemcpyAsync(ai, dai, c1 * c1 * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipStreamSynchronize(s));
    // W[:,c] is Py itself
    for (int k = 0; k < c; ++k) {
      double tr = 0.0, q = 0.0;
      for (int64_t r = 0; r < n; ++r) tr += rows[(size_t)k * n + r];
      for (int64_t r = 0; r < n; ++r) q += hw[r * c1 + c] * hw[r * c1 + k];
      fd[k] = 0.5 * (-tr + q);
    }
    double pp = 0.0;  // residual: -tr(P) + Py'Py
    for (int64_t r = 0; r < n; ++r) pp += hw[r * c1 + c] * hw[r * c1 + c];
    fd[c] = 0.5 * (-rows[(size_t)n * c] + pp);
    return GMAT_OK;
  }
};

double wall_now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
double g_reml_stats[4] = {0, 0, 0, 0};
// per iteration of the last gmat_reml call: gradient norm, update norm, EM weight
std::vector<double> g_reml_trace[3];

}  // namespace

extern "C" int gmat_reml_stats(double *out4) {
  GMAT_CHECK(out4, GMAT_E_ARG, "gmat_reml_stats: null");
  for (int k = 0; k < 4; ++k) out4[k] = g_reml_stats[k];
  return GMAT_OK;
}

extern "C" int gmat_reml_trace(int cap, double *grad_norm, double *update_norm, double *em_weight, int *count) {
  GMAT_CHECK(cap >= 0 && count, GMAT_E_ARG, "gmat_reml_trace: bad arguments");
  const int k = (int)g_reml_trace[0].size();
  *count = k;
  double *out[3] = {grad_norm, update_norm, em_weight};
  for (int t = 0; t < 3; ++t)
    if (out[t])
      for (int i = 0; i < std::min(cap, k); ++i) out[t][i] = g_reml_trace[t][i];
  return GMAT_OK;
}

extern "C" int gmat_reml(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y, const double *xmat,
                         const int64_t *z_col, const double *const *gmat, const double *init, int maxiter,
                         double cc_par, double cc_gra, double *var_out, int *n_iter, double *history) {
  GMAT_CHECK(y && xmat && z_col && var_out && (n_gmat == 0 || gmat), GMAT_E_ARG, "gmat_reml: bad arguments");
  const double t_start = wall_now();
  Model md;
  GMAT_TRY(md.setup(n_rec, n_fix, n_id, n_gmat, y, xmat, z_col, gmat));
  const int c1 = n_gmat + 1;
  GMAT_HIP(hipDeviceSynchronize());
  const double t_loop = wall_now();
  {  // ones vector used to copy Py into W
    double one = 1.0;
    GMAT_HIP(hipMemcpy(md.small.as<double>() + 3000, &one, sizeof(double), hipMemcpyHostToDevice));
  }
  std::vector<double> var(c1, 1.0), fd(c1), ai(c1 * c1), em(c1 * c1), wm(c1 * c1), wi(c1 * c1), delta(c1),
      nv(c1);
  if (init)
    for (int k = 0; k < c1; ++k) var[k] = init[k];
  int it = 0;
  double cc_gra_val = 1000.0, cc_par_val = 1000.0;
  for (auto &v : g_reml_trace) v.clear();
  while (it < maxiter) {
    ++it;
    GMAT_TRY(md.projection(var.data(), nullptr));
    GMAT_TRY(md.derivatives(fd.data(), ai.data()));
    for (int a = 0; a < c1; ++a)
      for (int b = 0; b < c1; ++b) em[a * c1 + b] = (a == b) ? (double)n_rec / (var[a] * var[a]) : 0.0;
    // EM weight grid (uvlmm_varcom.py:82-89): first weight giving all-positive variances
    double wt = 0.0;
    for (int j = 0; j <= 100; ++j) {
      wt = j * 0.01;
      for (int e = 0; e < c1 * c1; ++e) wm[e] = (1.0 - wt) * ai[e] + wt * em[e];
      GMAT_CHECK(small_inverse(c1, wm.data(), wi.data(), nullptr), GMAT_E_NOTPD, "singular EM/AI matrix");
      double mn = 1e300;
      for (int a = 0; a < c1; ++a) {
        double d = 0.0;
        for (int b = 0; b < c1; ++b) d += wi[a * c1 + b] * fd[b];
        delta[a] = d;
        nv[a] = var[a] + d;
        mn = std::min(mn, nv[a]);
      }
      if (mn > 0) break;
    }
    double dd = 0.0, vv = 0.0, gg = 0.0;
    for (int a = 0; a < c1; ++a) {
      dd += delta[a] * delta[a];
      vv += nv[a] * nv[a];
      gg += fd[a] * fd[a];
    }
    cc_par_val = std::sqrt(dd / vv);
    var = nv;
    cc_gra_val = std::sqrt(gg);
    g_reml_trace[0].push_back(cc_gra_val);
    g_reml_trace[1].push_back(cc_par_val);
    g_reml_trace[2].push_back(wt);
    if (history)
      for (int a = 0; a < c1; ++a) history[(int64_t)(it - 1) * c1 + a] = var[a];
    if (cc_gra_val < cc_gra && cc_par_val < cc_par) break;
  }
  for (int a = 0; a < c1; ++a) var_out[a] = var[a];
  if (n_iter) *n_iter = it;
  GMAT_HIP(hipDeviceSynchronize());
  const double t_end = wall_now(), nn = (double)n_rec;
  g_reml_stats[0] = t_end - t_start;
  g_reml_stats[1] = it;
  g_reml_stats[2] = it ? (t_end - t_loop) / it : 0.0;
  // algorithmic flop per iteration: potrf n^3/3, inverse 2n^3/3, traces/AI
  g_reml_stats[3] = nn * nn * nn + 2.0 * nn * nn * (2 * n_gmat + 1);
  return GMAT_OK;
}

extern "C" int gmat_projection(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y,
                               const double *xmat, const int64_t *z_col, const double *const *gmat,
                               const double *var_com, double *pvp, double *py) {
  GMAT_CHECK(y && xmat && z_col && var_com && pvp && py, GMAT_E_ARG, "gmat_projection: bad arguments");
  Model md;
  GMAT_TRY(md.setup(n_rec, n_fix, n_id, n_gmat, y, xmat, z_col, gmat));
  GMAT_TRY(md.projection(var_com, nullptr));
  const int64_t n = n_rec;
  bool identity = (n_id == n);
  for (int64_t r = 0; identity && r < n; ++r) identity = (z_col[r] == r);
  std::vector<double> hpy(n);
  GMAT_HIP(hipMemcpy(hpy.data(), md.py.p, n * sizeof(double), hipMemcpyDeviceToHost));
  if (identity) {
    GMAT_HIP(hipMemcpy(pvp, md.pm.p, n * n * sizeof(double), hipMemcpyDeviceToHost));
    memcpy(py, hpy.data(), n * sizeof(double));
    return GMAT_OK;
  }
  // CSR of records per individual (records in ascending order: deterministic sums)
  std::vector<int64_t> off(n_id + 1, 0), rec(n);
  for (int64_t r = 0; r < n; ++r) off[z_col[r] + 1]++;
  for (int64_t a = 0; a < n_id; ++a) off[a + 1] += off[a];
  std::vector<int64_t> fill(off.begin(), off.end() - 1);
  for (int64_t r = 0; r < n; ++r) rec[fill[z_col[r]]++] = r;
  for (int64_t a = 0; a < n_id; ++a) {
    double acc = 0.0;
    for (int64_t u = off[a]; u < off[a + 1]; ++u) acc += hpy[rec[u]];
    py[a] = acc;
  }
  DBuf doff, drec, dout;
  GMAT_TRY(doff.alloc((n_id + 1) * sizeof(int64_t)));
  GMAT_TRY(drec.alloc(n * sizeof(int64_t)));
  GMAT_TRY(dout.alloc(n_id * n_id * sizeof(double)));
  GMAT_HIP(hipMemcpy(doff.p, off.data(), (n_id + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(drec.p, rec.data(), n * sizeof(int64_t), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(ztpz_kernel, dim3((unsigned)cdiv(n_id * n_id, 256)), dim3(256), 0, 0, n, n_id,
                     doff.as<int64_t>(), drec.as<int64_t>(), md.pm.as<double>(), dout.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpy(pvp, dout.p, n_id * n_id * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// Random-effect prediction of wemai_multi_gmat_pred (uvlmm_varcom.py:147-166), reproduced as
// written there: the projection is built from V itself (vxmat = V X, pmat = V - VX (X'VX)^-1
// X'V, :152-156) rather than from V^-1, then zpy = Z' pmat y and rand_eff[:, k] =
// (G_k zpy) var_com[k].  rand_eff is n_id x n_gmat, row-major.
extern "C" int gmat_blup(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y,
                         const double *xmat, const int64_t *z_col, const double *const *gmat, const double *var_com,
                         double *rand_eff) {
  GMAT_CHECK(y && xmat && z_col && var_com && rand_eff && (gmat || n_gmat == 0), GMAT_E_ARG,
             "gmat_blup: bad arguments");
  Model md;
  GMAT_TRY(md.setup(n_rec, n_fix, n_id, n_gmat, y, xmat, z_col, gmat));
  const int64_t n = n_rec, p = n_fix;
  const hipStream_t s = md.s;
  Coefs k{};
  k.c = n_gmat;
  k.diag = var_com[n_gmat];
  for (int t = 0; t < n_gmat; ++t) {
    k.g[t] = md.zg[t].as<double>();
    k.s[t] = var_com[t];
  }
  hipLaunchKernelGGL(combine_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, s, n, k, md.v.as<double>());
  GMAT_HIP(hipGetLastError());
  // VX = V X ; XVX = X' VX (p x p, inverted on the host)
  GMAT_TRY(dgemm(s, n, p, n, 1.0, DView{md.v.as<double>(), n, 0}, DView{md.x.as<double>(), p, 0}, 0.0,
                 md.vx.as<double>(), p));
  GMAT_CHECK(p * p <= 1024, GMAT_E_ARG, "too many fixed effects (%lld)", (long long)p);
  double *dxvx = md.small.as<double>() + 8;
  GMAT_TRY(dgemm(s, p, p, n, 1.0, DView{md.x.as<double>(), p, 1}, DView{md.vx.as<double>(), p, 0}, 0.0, dxvx, p));
  std::vector<double> xvx(p * p), xvxi(p * p);
  GMAT_HIP(hipMemcpyAsync(xvx.data(), dxvx, p * p * sizeof(double), hipMemcpyDeviceToHost, s));
  GMAT_HIP(hipStreamSynchronize(s));
  GMAT_CHECK(small_inverse((int)p, xvx.data(), xvxi.data(), nullptr), GMAT_E_NOTPD, "X'VX is singular");
  double *dxi = md.small.as<double>() + 8 + 1024;
  GMAT_HIP(hipMemcpyAsync(dxi, xvxi.data(), p * p * sizeof(double), hipMemcpyHostToDevice, s));
  // pmat = V - (VX XVX^-1) VX' ; py = pmat y
  GMAT_TRY(dgemm(s, n, p, p, 1.0, DView{md.vx.as<double>(), p, 0}, DView{dxi, p, 0}, 0.0, md.t.as<double>(), p));
  GMAT_TRY(dgemm(s, n, n, p, -1.0, DView{md.t.as<double>(), p, 0}, DView{md.vx.as<double>(), p, 1}, 1.0,
                 md.v.as<double>(), n));
  GMAT_TRY(dgemm(s, n, 1, n, 1.0, DView{md.v.as<double>(), n, 0}, DView{md.y.as<double>(), 1, 0}, 0.0,
                 md.py.as<double>(), 1));
  std::vector<double> hpy(n), zpy(n_id, 0.0);
  GMAT_HIP(hipMemcpyAsync(hpy.data(), md.py.p, n * sizeof(double), hipMemcpyDeviceToHost, s));
  GMAT_HIP(hipStreamSynchronize(s));
  for (int64_t r = 0; r < n; ++r) zpy[z_col[r]] += hpy[r];  // Z' (records in order)
  DBuf g, dz, de;
  GMAT_TRY(g.alloc((size_t)n_id * n_id * sizeof(double)));
  GMAT_TRY(dz.alloc((size_t)n_id * sizeof(double)));
  GMAT_TRY(de.alloc((size_t)n_id * sizeof(double)));
  GMAT_HIP(hipMemcpyAsync(dz.p, zpy.data(), n_id * sizeof(double), hipMemcpyHostToDevice, s));
  std::vector<double> he(n_id);
  for (int t = 0; t < n_gmat; ++t) {
    GMAT_HIP(hipMemcpyAsync(g.p, gmat[t], (size_t)n_id * n_id * sizeof(double), hipMemcpyHostToDevice, s));
    GMAT_TRY(dgemm(s, n_id, 1, n_id, 1.0, DView{g.as<double>(), n_id, 0}, DView{dz.as<double>(), 1, 0}, 0.0,
                   de.as<double>(), 1));
    GMAT_HIP(hipMemcpyAsync(he.data(), de.p, n_id * sizeof(double), hipMemcpyDeviceToHost, s));
    GMAT_HIP(hipStreamSynchronize(s));
    for (int64_t a = 0; a < n_id; ++a) rand_eff[a * n_gmat + t] = he[a] * var_com[t];
  }
  return GMAT_OK;
}

extern "C" int gmat_spd_inverse(int64_t n, const double *a, double *ainv, double *logdet) {
  GMAT_CHECK(n > 0 && a && ainv, GMAT_E_ARG, "gmat_spd_inverse: bad arguments");
  DBuf da, dinv, work, out, sm;
  GMAT_TRY(da.alloc(n * n * sizeof(double)));
  GMAT_TRY(dinv.alloc(n * 64 * sizeof(double)));
  GMAT_TRY(work.alloc((n * n + 64 * n) * sizeof(double)));
  GMAT_TRY(out.alloc(n * n * sizeof(double)));
  GMAT_TRY(sm.alloc(2 * sizeof(double)));
  GMAT_HIP(hipMemcpy(da.p, a, n * n * sizeof(double), hipMemcpyHostToDevice));
  int *info = reinterpret_cast<int *>(sm.as<double>() + 1);
  GMAT_TRY(cholesky_inverse(0, n, da.as<double>(), n, dinv.as<double>(), sm.as<double>(), info, work.as<double>(),
                            out.as<double>()));
  double h[2];
  GMAT_HIP(hipMemcpy(h, sm.p, 2 * sizeof(double), hipMemcpyDeviceToHost));
  int hinfo;
  memcpy(&hinfo, &h[1], sizeof(int));
  GMAT_CHECK(hinfo == 0, GMAT_E_NOTPD, "matrix is not positive definite (pivot %d)", hinfo);
  if (logdet) *logdet = h[0];
  GMAT_HIP(hipMemcpy(ainv, out.p, n * n * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

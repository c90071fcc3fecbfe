// CPU restatement of the reference's effect-only screen -- TEST INFRASTRUCTURE ONLY (the checker
// of the GPU effect screen and the timed CPU baseline of bench.py's eff_screen leg; the product
// package never loads it).  Restates, in this repository's own C++ with OpenMP:
//   read_plink_bed            _read_plink_bed.c:5-51 / _remma_epi_eff_cpu.c:10-56 (v = (c^2+c)/6)
//   centring                  _remma_epi_eff_cpu.c:103-112 (AA), :277-285 (AD), :459-464 (DD)
//   print_outAA / AD / DD     :61-81, :226-257, :415-438 (eff += x_i x_j py, sequential over
//                             individuals, |eff| > cut; AD: >= for (i, j), > for (j, i))
//   the _maf forms            :141-166, :318-348, :500-522 (cut = table[freq_i[i]*10 + freq_j[j]])
// with the same fp64 operation order (no FMA contraction: built with -ffp-contract=off), so its
// numbers are the reference's bit for bit (checked against the reference's own C in this
// container by tests/test_oracle_golden.py).  Records come out in the reference's single-thread
// order (rows in list order, j ascending, AD (i, j) before (j, i)) instead of the reference's
// OpenMP interleaving.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

namespace {

struct Rec {
  int64_t i, j;
  double e;
};

void decode(const uint8_t *body, int64_t n, int64_t m, std::vector<double> &v) {
  const int64_t nb = (n + 3) / 4;
  v.assign((size_t)n * m, 0.0);
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < m; ++s)
    for (int64_t k = 0; k < n; ++k) {
      const int c = (body[s * nb + k / 4] >> (2 * (k % 4))) & 3;
      v[(size_t)s * n + k] = (double)(c * c + c) / 6.0;
    }
}

// kind 0 AA, 1 AD, 2 DD.  xa / xd: the centred codings (either may be empty when unused).
void centre(int64_t n, int64_t m, const std::vector<double> &v, bool need_a, bool need_d, std::vector<double> &xa,
            std::vector<double> &xd) {
  if (need_a) xa.assign((size_t)n * m, 0.0);
  if (need_d) xd.assign((size_t)n * m, 0.0);
#pragma omp parallel for schedule(static)
  for (int64_t s = 0; s < m; ++s) {
    double p = 0.0;
    for (int64_t k = 0; k < n; ++k) p += v[(size_t)s * n + k] / (double)(2 * n);
    for (int64_t k = 0; k < n; ++k) {
      const double x = v[(size_t)s * n + k];
      if (need_a) xa[(size_t)s * n + k] = x - 2 * p;
      if (need_d) xd[(size_t)s * n + k] = (std::fabs(x - 2.0) < 0.0001 ? 0.0 : x) - 2 * p * (1 - p);
    }
  }
}

inline double dot3(const double *a, const double *b, const double *py, int64_t n) {
  double e = 0.0;
  for (int64_t k = 0; k < n; ++k) e += a[k] * b[k] * py[k];
  return e;
}

}  // namespace

// Returns the number of records (written to out_i / out_j / out_e up to cap; call again with a
// larger buffer when the return value exceeds cap).  freq_i / freq_j may be null (single cut).
extern "C" int64_t oracle_eff_screen(int kind, const uint8_t *body, int64_t n, int64_t m, const int64_t *rows,
                                     int64_t n_rows, const double *py, const double *cut, const int64_t *freq_i,
                                     const int64_t *freq_j, int64_t cap, int64_t *out_i, int64_t *out_j,
                                     double *out_e) {
  std::vector<double> v, xa, xd;
  decode(body, n, m, v);
  centre(n, m, v, kind != 2, kind != 0, xa, xd);
  const double *X1 = kind == 2 ? xd.data() : xa.data();  // first SNP's coding
  const double *X2 = kind == 0 ? xa.data() : xd.data();  // second SNP's coding
  std::vector<std::vector<Rec>> per(n_rows);
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t i = rows[r];
    auto &out = per[r];
    for (int64_t j = i + 1; j < m; ++j) {
      const double c = freq_i ? cut[freq_i[i] * 10 + freq_j[j]] : cut[0];
      const double e1 = dot3(X1 + i * n, X2 + j * n, py, n);
      if (kind == 1 ? std::fabs(e1) >= c : std::fabs(e1) > c) out.push_back({i, j, e1});
      if (kind == 1) {
        const double e2 = dot3(xd.data() + i * n, xa.data() + j * n, py, n);
        if (std::fabs(e2) > c) out.push_back({j, i, e2});
      }
    }
  }
  int64_t k = 0;
  for (int64_t r = 0; r < n_rows; ++r)
    for (const Rec &q : per[r]) {
      if (k < cap) {
        out_i[k] = q.i;
        out_j[k] = q.j;
        out_e[k] = q.e;
      }
      ++k;
    }
  return k;
}

// Multi-threaded writers of the relationship-matrix text formats (gmatrix.py:10-31), and the scans'
// hit rows (DataFrame.to_csv of remma_epiAA.py:84-86 / remma_epiAA_pair.py: ints, then float reprs).
//
// 'mat' is np.savetxt's default ("%.18e", ' ' between values, '\n' per row): glibc's
// printf and CPython's '%' formatting both round correctly, so the bytes are identical.
// 'row_col_val' / 'id_id_val' are pandas DataFrame.to_csv rows whose float column is the
// shortest round-trip repr of each value (CPython float_repr_style 'short'): digits from
// std::to_chars (shortest round trip), laid out with CPython's rules -- fixed notation for
// decimal exponents -4 <= e < 16, otherwise d[.ddd]e(+|-)XX.
#include <algorithm>
#include <charconv>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <atomic>
#include <thread>
#include <vector>

#include "common.h"

namespace {

// CPython repr(float) of v into out; returns the length.
int py_repr(double v, char *out) {
  if (std::isnan(v)) return (int)(strcpy(out, "nan"), 3);
  if (std::isinf(v)) {
    if (v < 0) return (int)(strcpy(out, "-inf"), 4);
    return (int)(strcpy(out, "inf"), 3);
  }
  char sci[64];
  auto r = std::to_chars(sci, sci + sizeof(sci), v, std::chars_format::scientific);
  *r.ptr = 0;
  // sci = [-]d[.ddd]e(+|-)XX
  const char *p = sci;
  int len = 0;
  if (*p == '-') {
    out[len++] = '-';
    ++p;
  }
  char dig[32];
  int nd = 0;
  for (; *p && *p != 'e'; ++p)
    if (*p != '.') dig[nd++] = *p;
  const int e10 = atoi(p + 1);  // value = d.ddd x 10^e10
  if (nd == 1 && dig[0] == '0') {
    memcpy(out + len, "0.0", 3);
    return len + 3;
  }
  const int decpt = e10 + 1;  // value = 0.ddd x 10^decpt
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      out[len++] = '0';
      out[len++] = '.';
      for (int k = 0; k < -decpt; ++k) out[len++] = '0';
      memcpy(out + len, dig, nd);
      len += nd;
    } else if (decpt >= nd) {
      memcpy(out + len, dig, nd);
      len += nd;
      for (int k = nd; k < decpt; ++k) out[len++] = '0';
      out[len++] = '.';
      out[len++] = '0';
    } else {
      memcpy(out + len, dig, decpt);
      len += decpt;
      out[len++] = '.';
      memcpy(out + len, dig + decpt, nd - decpt);
      len += nd - decpt;
    }
    return len;
  }
  out[len++] = dig[0];
  if (nd > 1) {
    out[len++] = '.';
    memcpy(out + len, dig + 1, nd - 1);
    len += nd - 1;
  }
  len += snprintf(out + len, 16, "e%c%02d", e10 < 0 ? '-' : '+', e10 < 0 ? -e10 : e10);
  return len;
}

// Format rows [r0, r1) of the chosen layout into buf.
void format_rows(int fmt, const double *mat, int64_t n, const std::vector<std::string> &ids, int64_t r0, int64_t r1,
                 std::string *buf) {
  char tmp[96];
  for (int64_t r = r0; r < r1; ++r) {
    if (fmt == 0) {
      for (int64_t c = 0; c < n; ++c) {
        const int l = snprintf(tmp, sizeof(tmp), c + 1 < n ? "%.18e " : "%.18e\n", mat[r * n + c]);
        buf->append(tmp, l);
      }
    } else {
      for (int64_t c = 0; c <= r; ++c) {
        if (fmt == 1) {
          buf->append(std::to_string(r + 1)).push_back(' ');
          buf->append(std::to_string(c + 1)).push_back(' ');
        } else {
          buf->append(ids[r]).push_back(' ');
          buf->append(ids[c]).push_back(' ');
        }
        const int l = py_repr(mat[r * n + c], tmp);
        buf->append(tmp, l).push_back('\n');
      }
    }
  }
}

}  // namespace

extern "C" int gmat_float_repr(double v, char *out, int cap) {
  GMAT_CHECK(out && cap >= 32, GMAT_E_ARG, "gmat_float_repr: buffer");
  const int l = py_repr(v, out);
  out[l] = 0;
  return l;
}

// Append n hit rows "i j v_0 .. v_{nf-1}\n" (values as CPython repr) to path: the scans' result
// files, byte-identical to the reference's DataFrame.to_csv(sep=' ', header=False, index=False)
// rows (remma_epiAA.py:84-86) and to gmat_amd.remma._scan.format_rows.
extern "C" int gmat_append_hit_rows(const char *path, int64_t n, const int64_t *i, const int64_t *j, int nf,
                                    const double *f0, const double *f1, const double *f2, const double *f3) {
  const double *fv[4] = {f0, f1, f2, f3};
  GMAT_CHECK(path && n >= 0 && nf >= 1 && nf <= 4 && (n == 0 || (i && j)), GMAT_E_ARG,
             "gmat_append_hit_rows: bad arguments");
  for (int k = 0; k < nf; ++k) GMAT_CHECK(n == 0 || fv[k], GMAT_E_ARG, "gmat_append_hit_rows: column %d missing", k);
  FILE *f = fopen(path, "ab");
  GMAT_CHECK(f, GMAT_E_ARG, "gmat_append_hit_rows: cannot open %s", path);
  // rows formatted by up to 16 threads in contiguous chunks of >= 2,048 (the shortest-repr formatting is
  // ~250 ns a row: 2.8 ms for a configs[2] step's 10,932 hits on one thread), written in order in
  // blocks of at most 1M rows
  // a formatting thread that runs out of memory records it here instead of taking the process down
  std::atomic<bool> oom{false};
  auto fmt_rows = [&](int64_t r0, int64_t r1, std::string *out) {
    out->clear();
    out->reserve((size_t)(r1 - r0) * (16 + 25 * nf));
    char tmp[96];
    for (int64_t r = r0; r < r1; ++r) {
      const int l = snprintf(tmp, sizeof(tmp), "%lld %lld", (long long)i[r], (long long)j[r]);
      out->append(tmp, l);
      for (int k = 0; k < nf; ++k) {
        out->push_back(' ');
        out->append(tmp, py_repr(fv[k][r], tmp));
      }
      out->push_back('\n');
    }
  };
  auto fmt = [&](int64_t r0, int64_t r1, std::string *out) {
    try {
      fmt_rows(r0, r1, out);
    } catch (...) {
      oom = true;
      std::string().swap(*out);
    }
  };
  const int64_t blk = 1 << 20;
  const int hw = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  int rc = GMAT_OK;
  for (int64_t b0 = 0; b0 < n && rc == GMAT_OK; b0 += blk) {
    const int64_t b1 = std::min(n, b0 + blk);
    const int T = (int)std::max<int64_t>(1, std::min<int64_t>(hw, (b1 - b0) / 2048));
    std::vector<std::string> bufs(T);
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t)
      th.emplace_back(fmt, b0 + (b1 - b0) * t / T, b0 + (b1 - b0) * (t + 1) / T, &bufs[t]);
    fmt(b0, b0 + (b1 - b0) / T, &bufs[0]);
    for (auto &x : th) x.join();
    if (oom) {
      fclose(f);
      GMAT_CHECK(false, GMAT_E_NOMEM, "gmat_append_hit_rows: out of host memory formatting %lld rows", (long long)n);
    }
    for (auto &s : bufs)
      if (!s.empty() && fwrite(s.data(), 1, s.size(), f) != s.size()) rc = GMAT_E_ARG;
  }
  if (fclose(f) != 0) rc = GMAT_E_ARG;
  GMAT_CHECK(rc == GMAT_OK, rc, "gmat_append_hit_rows: write to %s failed", path);
  return GMAT_OK;
}

extern "C" int gmat_write_grm_text(const char *path, const double *mat, int64_t n, int fmt, const char *ids_blob,
                                   int n_threads) {
  GMAT_CHECK(path && mat && n > 0 && fmt >= 0 && fmt <= 2 && (fmt != 2 || ids_blob), GMAT_E_ARG,
             "gmat_write_grm_text: bad arguments");
  std::vector<std::string> ids;
  if (fmt == 2) {  // n NUL-terminated strings back to back
    const char *p = ids_blob;
    for (int64_t k = 0; k < n; ++k) {
      ids.emplace_back(p);
      p += ids.back().size() + 1;
    }
  }
  FILE *f = fopen(path, "wb");
  GMAT_CHECK(f, GMAT_E_ARG, "gmat_write_grm_text: cannot open %s", path);
  const int T = n_threads > 0 ? n_threads : std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // row blocks of roughly equal output size, written in order
  const int64_t R = 64;
  int rc = GMAT_OK;
  std::atomic<bool> oom{false};
  for (int64_t base = 0; base < n && rc == GMAT_OK; base += R * T) {
    std::vector<std::string> bufs(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
      const int64_t r0 = std::min(n, base + t * R), r1 = std::min(n, r0 + R);
      if (r0 >= r1) break;
      th.emplace_back(
          [&, r0, r1, t]() {
            try {
              format_rows(fmt, mat, n, ids, r0, r1, &bufs[t]);
            } catch (...) {
              oom = true;
              std::string().swap(bufs[t]);
            }
          });
    }
    for (auto &x : th) x.join();
    if (oom) {
      fclose(f);
      GMAT_CHECK(false, GMAT_E_NOMEM, "gmat_write_grm_text: out of host memory");
    }
    for (auto &b : bufs)
      if (!b.empty() && fwrite(b.data(), 1, b.size(), f) != b.size()) rc = GMAT_E_ARG;
  }
  if (fclose(f) != 0) rc = GMAT_E_ARG;
  GMAT_CHECK(rc == GMAT_OK, rc, "gmat_write_grm_text: write to %s failed", path);
  return GMAT_OK;
}

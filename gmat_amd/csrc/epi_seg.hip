// Scan plans past the single-plan limits (see epi.h).
//
// The scan kernels address the panels and their stage-blocked copies with 32-bit lane offsets from a
// 64-bit wave-uniform base (LDS-DMA and buffer loads), so one plan holds at most 2 m n_pad < 2^32 bytes
// of int8 panel (m SNPs of n_pad individuals: ~1.05 M SNPs at 2,000 individuals, ~419 k at 5,000).  The
// reference's loop (remma_epiAA.py:35-82 and siblings) has no such limit; a larger panel is cut here into
// k SNP segments A_0 .. A_{k-1} of equal size such that any two of them fit one plan, and a scan runs
//   * for each segment A with listed rows: a plan on [A] (pairs inside A), and
//   * for each other segment B (B after A for the triangular kinds AA / DD, every B != A for AD): a
//     plan on the concatenated panel [A, B] scanning A's rows against B's columns only (the plan's col_lo
//     = |A|, so no pair is tested twice),
// each sub-plan importing the spectral state (certificates, low-rank basis: properties of P alone) of
// the plan on segment 0, so every pair sees the same screens and the same exact refine as in one plan:
// the hits and their values are those of an unsegmented scan, byte for byte.  Pair lists are grouped by
// the segments of their two SNPs.  GMAT_SEG_SNPS=s forces segments of s SNPs (tests, at sizes one plan
// could hold).
#include "epi.h"

#include <map>
#include <utility>

namespace gmat {
namespace epi {

struct SegPlan {
  gmat_geno *g = nullptr;     // the whole panel (the caller's)
  std::vector<int64_t> lo;    // segment t = SNPs [lo[t], lo[t + 1])
  std::vector<double> pvp, py;
  std::vector<uint8_t> state;  // the spectral state of base (imported by every sub-plan)
  int n_slice = 3;
  gmat_geno *base_g = nullptr;  // segment 0 and its plan
  gmat_epi *base = nullptr;
  ~SegPlan() {
    delete base;
    gmat_geno_destroy(base_g);
  }
  int k() const { return (int)lo.size() - 1; }
  int64_t size(int t) const { return lo[t + 1] - lo[t]; }
  int of(int64_t j) const { return (int)(std::upper_bound(lo.begin(), lo.end(), j) - lo.begin()) - 1; }
};

void seg_free(SegPlan *sp) { delete sp; }

const gmat_epi *seg_base(const gmat_epi *e) { return e->seg->base; }

int64_t seg_snps(const gmat_geno *g) {
  // the largest segment of which two fit one plan: 2 (2 s) n_pad < 2^32
  const int64_t s_max = ((((int64_t)1 << 31) - 1) / g->n_pad - 1) / 2;
  int64_t s = s_max;
  const char *v = getenv("GMAT_SEG_SNPS");
  if (v) s = std::min(s_max, std::max<int64_t>(64, atoll(v)));
  // one plan holds the panel: segments only past 2 m n_pad >= 2^32, or at a forced size (tests)
  if (2 * g->m * g->n_pad < ((int64_t)1 << 32) && (!v || g->m <= s)) return 0;
  const int64_t k = cdiv(g->m, s);
  return cdiv(g->m, k);  // equal segments
}

namespace {

// a sub-plan on the segments [a] (a == b) or [a, b], with the shared spectral state
struct SubPlan {
  gmat_geno *g = nullptr;
  gmat_epi *e = nullptr;
  ~SubPlan() {
    delete e;
    gmat_geno_destroy(g);
  }
};

int sub_plan(SegPlan &sp, int a, int b, SubPlan *out) {
  const int64_t lo[2] = {sp.lo[a], sp.lo[b]}, hi[2] = {sp.lo[a + 1], sp.lo[b + 1]};
  GMAT_TRY(geno_subset(sp.g, lo, hi, a == b ? 1 : 2, &out->g));
  return epi_create_impl(&out->e, out->g, sp.pvp.data(), sp.py.data(), sp.n_slice, sp.state.data(),
                         (int64_t)sp.state.size(), false);
}

// a sub-plan's local SNP index -> the whole panel's
inline int64_t global_of(const SegPlan &sp, int a, int b, int64_t local) {
  return local < sp.size(a) ? sp.lo[a] + local : sp.lo[b] + (local - sp.size(a));
}

}  // namespace

int seg_create(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice, const uint8_t *state,
               int64_t state_bytes) {
  const double t0 = now();
  const int64_t s = seg_snps(g);
  GMAT_CHECK(s > 0, GMAT_E_ARG, "seg_create: the panel fits one plan");
  auto *sp = new SegPlan();
  auto *e = new gmat_epi();
  e->seg = sp;  // owned: deleted with e
  e->g = g;
  e->n = g->n;
  e->n_pad = g->n_pad;
  e->m = g->m;
  e->n_slice = n_slice;
  e->nK = (int)(g->n_pad / MXK);
  sp->g = g;
  sp->n_slice = n_slice;
  for (int64_t j = 0; j < g->m; j += s) sp->lo.push_back(j);
  sp->lo.push_back(g->m);
  sp->pvp.assign(pvp, pvp + g->n * g->n);
  sp->py.assign(py, py + g->n);
  auto fail = [&](int rc) {
    delete e;
    return rc;
  };
  // segment 0's plan computes (or imports) the spectral state every sub-plan shares
  const int64_t lo0 = 0, hi0 = sp->size(0);
  int rc = geno_subset(g, &lo0, &hi0, 1, &sp->base_g);
  if (rc == GMAT_OK) rc = epi_create_impl(&sp->base, sp->base_g, pvp, py, n_slice, state, state_bytes, false);
  if (rc != GMAT_OK) return fail(rc);
  int64_t need = 0;
  if ((rc = gmat_epi_export(sp->base, nullptr, 0, &need)) != GMAT_OK) return fail(rc);
  sp->state.resize((size_t)need);
  if ((rc = gmat_epi_export(sp->base, sp->state.data(), need, &need)) != GMAT_OK) return fail(rc);
  e->exh_only = sp->base->exh_only;
  e->lr_R = sp->base->lr_R;
  e->pf_mu = sp->base->pf_mu;
  e->setup[0] = now() - t0;
  if (getenv("GMAT_DEBUG"))
    fprintf(stderr, "gmat_epi_create: %lld SNPs x %lld individuals in %d segments of %lld SNPs\n", (long long)g->m,
            (long long)g->n_pad, sp->k(), (long long)s);
  *out = e;
  return GMAT_OK;
}

int seg_scan(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut, int n_slice,
             int64_t *n_hits) {
  SegPlan &sp = *e->seg;
  const double t0 = now();
  const bool tri = kind != GMAT_AD;
  for (auto *v : {&e->hit_i, &e->hit_j}) v->clear();
  for (auto *v : {&e->hit_eff, &e->hit_var, &e->hit_chi, &e->hit_p}) v->clear();
  double stats[10] = {0}, kstats[8] = {0};
  int level = 0;
  double bound = 0.0;
  for (int a = 0; a < sp.k(); ++a) {
    // this segment's rows, as local indices (rows ascend)
    const int64_t *r0 = std::lower_bound(rows, rows + n_rows, sp.lo[a]);
    const int64_t *r1 = std::lower_bound(rows, rows + n_rows, sp.lo[a + 1]);
    if (r0 == r1) continue;
    std::vector<int64_t> loc(r0, r1);
    for (int64_t &r : loc) r -= sp.lo[a];
    for (int b = tri ? a : 0; b < sp.k(); ++b) {
      SubPlan sub;
      GMAT_TRY(sub_plan(sp, a, b, &sub));
      sub.e->col_lo = a == b ? 0 : sp.size(a);  // [A, B]: A's rows against B's columns only
      int64_t nh = 0;
      if (getenv("GMAT_DEBUG"))
        fprintf(stderr, "seg_scan: kind %d segments (%d, %d): %zu rows, sub-plan %lld SNPs, col_lo %lld\n", kind, a, b,
                loc.size(), (long long)sub.e->m, (long long)sub.e->col_lo);
      GMAT_TRY(scan_dispatch(sub.e, kind, loc.data(), (int64_t)loc.size(), p_cut, chi_cut, n_slice, &nh));
      if (getenv("GMAT_DEBUG")) GMAT_HIP(hipDeviceSynchronize());
      for (int64_t t = 0; t < nh; ++t) {
        e->hit_i.push_back(global_of(sp, a, b, sub.e->hit_i[t]));
        e->hit_j.push_back(global_of(sp, a, b, sub.e->hit_j[t]));
      }
      e->hit_eff.insert(e->hit_eff.end(), sub.e->hit_eff.begin(), sub.e->hit_eff.end());
      e->hit_var.insert(e->hit_var.end(), sub.e->hit_var.begin(), sub.e->hit_var.end());
      e->hit_chi.insert(e->hit_chi.end(), sub.e->hit_chi.begin(), sub.e->hit_chi.end());
      e->hit_p.insert(e->hit_p.end(), sub.e->hit_p.begin(), sub.e->hit_p.end());
      for (int q = 0; q < 8; ++q) stats[q] += sub.e->stats[q];  // pairs, candidates, times, launches
      for (int q = 0; q < 7; ++q) kstats[q] += sub.e->kstats[q];
      level = (int)sub.e->stats[8];
      bound = sub.e->stats[9];
    }
  }
  // (i, j) order, as one plan's scan returns them
  std::vector<int64_t> ord(e->hit_i.size());
  for (size_t q = 0; q < ord.size(); ++q) ord[q] = (int64_t)q;
  std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) {
    return e->hit_i[x] != e->hit_i[y] ? e->hit_i[x] < e->hit_i[y] : e->hit_j[x] < e->hit_j[y];
  });
  auto apply = [&](auto &v) {
    auto c = v;
    for (size_t q = 0; q < ord.size(); ++q) v[q] = c[ord[q]];
  };
  apply(e->hit_i);
  apply(e->hit_j);
  apply(e->hit_eff);
  apply(e->hit_var);
  apply(e->hit_chi);
  apply(e->hit_p);
  for (int q = 0; q < 8; ++q) e->stats[q] = stats[q];
  e->stats[6] = now() - t0;
  e->stats[8] = level;
  e->stats[9] = bound;
  for (int q = 0; q < 7; ++q) e->kstats[q] = kstats[q];
  e->kstats[7] = -1;
  e->kev_used = 0;  // the sub-plans' kernel timers went with them
  e->kmarks.clear();
  *n_hits = (int64_t)e->hit_i.size();
  return GMAT_OK;
}

namespace {
// the pairs grouped by the segments of their SNPs: (a, b) with a <= b -> indices into the list
std::map<std::pair<int, int>, std::vector<int64_t>> seg_groups(const SegPlan &sp, const int64_t *pairs, int64_t n) {
  std::map<std::pair<int, int>, std::vector<int64_t>> grp;
  for (int64_t t = 0; t < n; ++t) {
    const int a = sp.of(pairs[2 * t]), b = sp.of(pairs[2 * t + 1]);
    grp[{std::min(a, b), std::max(a, b)}].push_back(t);
  }
  return grp;
}
// a SNP's index in the sub-plan [a] / [a, b]
inline int64_t local_of(const SegPlan &sp, int a, int b, int64_t j) {
  return (j >= sp.lo[a] && j < sp.lo[a + 1]) ? j - sp.lo[a] : sp.size(a) + (j - sp.lo[b]);
}
}  // namespace

int seg_pairs(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *eff, double *var, double *chi,
              double *p) {
  SegPlan &sp = *e->seg;
  for (int64_t t = 0; t < n_pairs; ++t)
    GMAT_CHECK(pairs[2 * t] >= 0 && pairs[2 * t] < e->m && pairs[2 * t + 1] >= 0 && pairs[2 * t + 1] < e->m, GMAT_E_ARG,
               "pair %lld out of range", (long long)t);
  for (const auto &kv : seg_groups(sp, pairs, n_pairs)) {
    const int a = kv.first.first, b = kv.first.second;
    const std::vector<int64_t> &idx = kv.second;
    SubPlan sub;
    GMAT_TRY(sub_plan(sp, a, b, &sub));
    std::vector<int64_t> loc(2 * idx.size());
    for (size_t q = 0; q < idx.size(); ++q) {
      loc[2 * q] = local_of(sp, a, b, pairs[2 * idx[q]]);
      loc[2 * q + 1] = local_of(sp, a, b, pairs[2 * idx[q] + 1]);
    }
    std::vector<double> out(4 * idx.size());
    const int64_t np = (int64_t)idx.size();
    GMAT_TRY(gmat_epi_pairs(sub.e, kind, loc.data(), np, out.data(), out.data() + np, out.data() + 2 * np,
                            out.data() + 3 * np));
    for (size_t q = 0; q < idx.size(); ++q) {
      eff[idx[q]] = out[q];
      var[idx[q]] = out[np + q];
      chi[idx[q]] = out[2 * np + q];
      p[idx[q]] = out[3 * np + q];
    }
  }
  return GMAT_OK;
}

int seg_audit(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *out5) {
  SegPlan &sp = *e->seg;
  for (int64_t t = 0; t < n_pairs; ++t)
    GMAT_CHECK(pairs[2 * t] >= 0 && pairs[2 * t] < e->m && pairs[2 * t + 1] >= 0 && pairs[2 * t + 1] < e->m, GMAT_E_ARG,
               "pair %lld out of range", (long long)t);
  for (const auto &kv : seg_groups(sp, pairs, n_pairs)) {
    const int a = kv.first.first, b = kv.first.second;
    const std::vector<int64_t> &idx = kv.second;
    SubPlan sub;
    GMAT_TRY(sub_plan(sp, a, b, &sub));
    std::vector<int64_t> loc(2 * idx.size());
    for (size_t q = 0; q < idx.size(); ++q) {
      loc[2 * q] = local_of(sp, a, b, pairs[2 * idx[q]]);
      loc[2 * q + 1] = local_of(sp, a, b, pairs[2 * idx[q] + 1]);
    }
    std::vector<double> out(5 * idx.size());
    GMAT_TRY(gmat_epi_audit(sub.e, kind, loc.data(), (int64_t)idx.size(), out.data()));
    for (size_t q = 0; q < idx.size(); ++q)
      for (int c = 0; c < 5; ++c) out5[5 * idx[q] + c] = out[5 * q + c];
  }
  return GMAT_OK;
}

}  // namespace epi
}  // namespace gmat

extern "C" int gmat_epi_layout(const gmat_epi *e, int64_t *out4) {
  GMAT_CHECK(e && out4, GMAT_E_ARG, "gmat_epi_layout: bad arguments");
  out4[0] = e->seg ? e->seg->k() : 1;
  out4[1] = e->seg ? e->seg->size(0) : e->m;
  out4[2] = e->exh_only ? 1 : 0;
  out4[3] = e->m;
  return GMAT_OK;
}

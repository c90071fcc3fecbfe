// The scans of a plan (exhaustive, compacted low-rank, block-granular) and their C API (see epi.h).
#include "epi.h"

namespace gmat {
namespace epi {

// ---- pieces shared by the three scan paths (scan_exhaustive, scan_lowrank, scan_blocks)

// the codings of one scan kind: reference codes (refine) and screen codes of both sides
struct ScanSide {
  int lc = 0, rc = 0, tri = 1;
  const Coding *L = nullptr, *R = nullptr;
  const int8_t *lp = nullptr, *rp = nullptr;    // reference codes (refine)
  const int8_t *slp = nullptr, *srp = nullptr;  // screen codes
};

// the block-granular screens' side vectors of a built coding (int8 slices of L' = a o (Pa - alpha z),
// Ld = a^2 o diag(P) and R' = (b - beta) o Pb), made when a scan first uses those screens
int block_sides(gmat_epi *e, int which) {
  Coding &cd = e->code[which];
  if (cd.side_ready) return GMAT_OK;
  const int64_t m = e->m, n_pad = e->n_pad, ss = m * n_pad;
  const size_t vb = (size_t)m * n_pad * sizeof(double);
  const int8_t *panel = screen_panel(e, which);
  DBuf Lp, Ld, Rp;
  GMAT_TRY(Lp.alloc(vb));
  GMAT_TRY(Ld.alloc(vb));
  GMAT_TRY(Rp.alloc(vb));
  for (DBuf *b : {&cd.Lq, &cd.Ldq, &cd.Rq}) GMAT_TRY(b->alloc((size_t)SIDE_T * m * n_pad));
  DBuf scratch;  // the kernels' per-SNP scalars again (discarded: the coding has them)
  GMAT_TRY(scratch.alloc((size_t)6 * m * sizeof(double)));
  double *sc = scratch.as<double>();
  hipLaunchKernelGGL(left_side_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, panel, cd.U.as<double>(),
                     e->z.as<double>(), e->py.as<double>(), e->dg.as<double>(), cd.soff.as<double>(), Lp.as<double>(),
                     nullptr, Ld.as<double>(), sc, sc + m, sc + 2 * m);
  hipLaunchKernelGGL(right_side_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, panel, cd.U.as<double>(),
                     e->z.as<double>(), e->py.as<double>(), cd.soff.as<double>(), Rp.as<double>(), sc + 3 * m,
                     sc + 4 * m, sc + 5 * m);
  hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, ss, Lp.as<double>(),
                     cd.Lq.as<int8_t>(), cd.sL.as<double>());
  hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, ss, Ld.as<double>(),
                     cd.Ldq.as<int8_t>(), cd.sLd.as<double>());
  hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, ss, Rp.as<double>(),
                     cd.Rq.as<int8_t>(), cd.sR.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipStreamSynchronize(e->s));
  cd.side_ready = true;
  return GMAT_OK;
}

// builds the codings `kind` needs and clears the previous scan's hits and counters
// the covariate directions quantised for prefilter_cov_kernel: q_k = rint(u_k / sq_k), sq_k = max |u_k| / 63
// (so a o q_k, a in {0, 1, 2}, is an exact int8 vector); from pf_U, once per plan (also after an import)
int ensure_pf_q(gmat_epi *e) {
  const int K0 = e->pf_ncov;
  if (K0 <= 0 || e->pf_q.p) return GMAT_OK;
  const int64_t n_pad = e->n_pad;
  std::vector<double> u((size_t)K0 * n_pad);
  GMAT_HIP(hipMemcpy(u.data(), e->pf_U.p, u.size() * sizeof(double), hipMemcpyDeviceToHost));
  std::vector<int8_t> q(u.size(), 0);
  for (int k = 0; k < K0; ++k) {
    double mx = 0.0;
    for (int64_t t = 0; t < n_pad; ++t) mx = std::max(mx, std::fabs(u[(size_t)k * n_pad + t]));
    const double sq = mx > 0.0 ? mx / 63.0 : 1.0;
    e->pf_sq[k] = sq;
    // stored in the stage-blocked panels' order: per 8 individuals 0 2 4 6 1 3 5 7 (block_panel_perm8_kernel)
    static const int eo[8] = {0, 2, 4, 6, 1, 3, 5, 7};
    for (int64_t t = 0; t < n_pad; ++t)
      q[(size_t)k * n_pad + t] =
          (int8_t)std::max(-63.0, std::min(63.0, std::rint(u[(size_t)k * n_pad + (t & ~7LL) + eo[t & 7]] / sq)));
  }
  GMAT_TRY(e->pf_q.alloc(q.size()));
  GMAT_HIP(hipMemcpy(e->pf_q.p, q.data(), q.size(), hipMemcpyHostToDevice));
  return GMAT_OK;
}

int scan_begin(gmat_epi *e, int kind, ScanSide *c) {
  kind_codings(kind, &c->lc, &c->rc);
  GMAT_TRY(build_coding(e, c->lc));
  GMAT_TRY(build_coding(e, c->rc));
  GMAT_TRY(ensure_pf_q(e));
  c->L = &e->code[c->lc];
  c->R = &e->code[c->rc];
  c->lp = c->lc == 0 ? e->g->dose_ptr() : e->g->het_ptr();
  c->rp = c->rc == 0 ? e->g->dose_ptr() : e->g->het_ptr();
  c->slp = screen_panel(e, c->lc);
  c->srp = screen_panel(e, c->rc);
  c->tri = kind != GMAT_AD;
  for (double &v : e->stats) v = 0.0;
  for (double &v : e->kstats) v = 0.0;
  e->kev_used = 0;
  e->kmarks.clear();
  for (auto *v : {&e->hit_i, &e->hit_j}) v->clear();
  for (auto *v : {&e->hit_eff, &e->hit_var, &e->hit_chi, &e->hit_p}) v->clear();
  return GMAT_OK;
}

// one launch of the screened scans: its first SNPs, the first column a pair of it can reach and
// (block-granular int8 screen only) its (row offset, J) tile list, built when a level needs it
struct ScanLaunch {
  std::vector<int64_t> rows;
  std::vector<int> tiles;
  int64_t j_lo = 0;
};

// launches of `rl` rows: chunk k of half that size folded with chunk NC-1-k (equal work per launch,
// as the triangle's rows shrink); launches without a pair are dropped.  *pairs = the pairs the
// launches test.
std::vector<ScanLaunch> fold_launches(const int64_t *rows, int64_t n_rows, int64_t m, int tri, double *pairs,
                                      int64_t rl = ROWS_PER_LAUNCH, int64_t col_lo = 0) {
  std::vector<ScanLaunch> plan;
  *pairs = 0;
  const int64_t half = rl / 2, nc = cdiv(n_rows, half);
  for (int64_t k = 0, l = nc - 1; k <= l; ++k, --l) {
    ScanLaunch ln;
    for (int64_t t = k * half; t < std::min(n_rows, (k + 1) * half); ++t) ln.rows.push_back(rows[t]);
    if (l != k)
      for (int64_t t = l * half; t < std::min(n_rows, (l + 1) * half); ++t) ln.rows.push_back(rows[t]);
    if (ln.rows.empty()) continue;
    ln.j_lo = std::max<int64_t>(tri ? ln.rows[0] + 1 : 0, col_lo);
    if (ln.j_lo >= m) continue;
    for (int64_t r : ln.rows) *pairs += (double)(m - std::max<int64_t>(tri ? r + 1 : 0, col_lo));
    plan.push_back(std::move(ln));
  }
  return plan;
}

// candidate buffers of the screened scans (kept by the plan): `dflt` candidates unless a previous
// scan left larger ones (GMAT_CAND_CAP: tests give a small buffer to exercise the overflow paths);
// the pair screen's survivor buffers beside them
int ensure_candidates(gmat_epi *e, int64_t dflt, bool use_ps) {
  if (e->cand_cap == 0 || e->cand_i.bytes < (size_t)e->cand_cap * 8) {
    const char *cenv = getenv("GMAT_CAND_CAP");
    e->cand_cap = cenv ? std::max<int64_t>(1024, atoll(cenv)) : std::max<int64_t>(e->cand_cap, dflt);
    for (DBuf *d : {&e->cand_i, &e->cand_j, &e->ceff, &e->cvar, &e->cchi, &e->cp}) GMAT_TRY(d->alloc(e->cand_cap * 8));
  }
  if (!e->counter.p) GMAT_TRY(e->counter.alloc(8));
  if (use_ps && e->cand2_i.bytes < (size_t)e->cand_cap * 8) {
    GMAT_TRY(e->cand2_i.alloc(e->cand_cap * 8));
    GMAT_TRY(e->cand2_j.alloc(e->cand_cap * 8));
  }
  if (use_ps && !e->counter2.p) GMAT_TRY(e->counter2.alloc(8));
  return GMAT_OK;
}

// grows the (empty) candidate buffers to `cap`
int grow_candidates(gmat_epi *e, int64_t cap, bool use_ps) {
  for (DBuf *d : {&e->cand_i, &e->cand_j, &e->ceff, &e->cvar, &e->cchi, &e->cp}) GMAT_TRY(d->alloc((size_t)cap * 8));
  if (use_ps)
    for (DBuf *d : {&e->cand2_i, &e->cand2_j}) GMAT_TRY(d->alloc((size_t)cap * 8));
  e->cand_cap = cap;
  if (getenv("GMAT_DEBUG")) fprintf(stderr, "candidate buffer grown to %lld\n", (long long)cap);
  return GMAT_OK;
}

struct RefineTally {
  double t_ref = 0, n_cand = 0, n_refined = 0;  // seconds on the refine stream, candidates, refined pairs
};


int refine_collect(gmat_epi *e, const ScanSide &c, hipStream_t st, bool use_ps, int64_t lo, int64_t hi, int64_t ps_done,
                   double chi_cut, double p_cut, hipEvent_t beg, hipEvent_t end, RefineTally *tl) {
  if (hi <= lo) return GMAT_OK;
  ps_done = std::max(ps_done, lo);
  const int64_t *fi = e->cand_i.as<int64_t>() + lo, *fj = e->cand_j.as<int64_t>() + lo;
  int64_t nf = hi - lo;
  GMAT_HIP(hipEventRecord(beg, st));
  if (use_ps) {
    GMAT_TRY(pair_screen(e, st, *c.L, *c.R, c.slp, c.srp, e->cand_i.as<int64_t>() + ps_done,
                         e->cand_j.as<int64_t>() + ps_done, hi - ps_done, chi_cut, &nf, ps_done == lo));
    fi = e->cand2_i.as<int64_t>();
    fj = e->cand2_j.as<int64_t>();
  }
  tl->n_cand += (double)(hi - lo);
  tl->n_refined += (double)nf;
  Pinned &pin = e->pins.res;
  if (nf > 0) {
    GMAT_TRY(refine(e, st, *c.L, *c.R, c.lp, c.rp, fi, fj, nf, e->ceff.as<double>(), e->cvar.as<double>(),
                    e->cchi.as<double>(), e->cp.as<double>()));
    // the hits (p < p_cut) compacted on the device and read back: their count, then their 48-byte records
    // (round 4 read back all refined candidates, ~12 MB per configs[2] step, and filtered on the host:
    // ~0.5 ms of the step between its last kernel and the next scan's first)
    if (e->cpack.bytes < (size_t)nf * 48) {
      GMAT_HIP(hipStreamSynchronize(st));
      GMAT_TRY(e->cpack.alloc((size_t)std::max<int64_t>(nf, 1 << 16) * 48));
    }
    if (!e->hcount.p) GMAT_TRY(e->hcount.alloc(8));
    GMAT_TRY(pin.reserve(4096));
    GMAT_HIP(hipMemsetAsync(e->hcount.p, 0, 8, st));
    hipLaunchKernelGGL(hit_pack_kernel, dim3((unsigned)cdiv(nf, 256)), dim3(256), 0, st, nf, fi, fj, e->ceff.as<double>(),
                       e->cvar.as<double>(), e->cchi.as<double>(), e->cp.as<double>(), p_cut, e->cpack.as<double>(),
                       e->hcount.as<unsigned long long>());
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpyAsync(pin.p, e->hcount.p, 8, hipMemcpyDeviceToHost, st));
    GMAT_HIP(hipEventRecord(end, st));
    GMAT_HIP(hipStreamSynchronize(st));
    const int64_t nh = (int64_t)*pin.as<unsigned long long>();
    if (nh > 0) {
      GMAT_TRY(pin.reserve((size_t)nh * 48));
      GMAT_HIP(hipMemcpyAsync(pin.p, e->cpack.p, (size_t)nh * 48, hipMemcpyDeviceToHost, st));
      GMAT_HIP(hipStreamSynchronize(st));
      std::vector<double> hb((size_t)nh * 6);  // one bulk copy out of the pinned block
      std::memcpy(hb.data(), pin.p, (size_t)nh * 48);
      const size_t h0 = e->hit_i.size();
      for (auto *v : {&e->hit_eff, &e->hit_var, &e->hit_chi, &e->hit_p}) v->resize(h0 + nh);
      e->hit_i.resize(h0 + nh);
      e->hit_j.resize(h0 + nh);
      for (int64_t k = 0; k < nh; ++k) {
        const double *r = &hb[(size_t)k * 6];
        std::memcpy(&e->hit_i[h0 + k], &r[0], 8);
        std::memcpy(&e->hit_j[h0 + k], &r[1], 8);
        e->hit_eff[h0 + k] = r[2];
        e->hit_var[h0 + k] = r[3];
        e->hit_chi[h0 + k] = r[4];
        e->hit_p[h0 + k] = r[5];
      }
    }
  } else {
    GMAT_HIP(hipEventRecord(end, st));
    GMAT_HIP(hipStreamSynchronize(st));
  }
  float ms;
  GMAT_HIP(hipEventElapsedTime(&ms, beg, end));
  tl->t_ref += ms * 1e-3;
  return GMAT_OK;
}

// hits in (i, j) order, as the reference's row loop emits them: an LSD radix sort (11-bit digits, passes
// whose digit is the same for every hit skipped) of the keys i m + j with the hits' positions, then the
// six arrays permuted through a reused scratch block (the comparison sort of the positions took ~0.4 ms
// of host time per configs[2] step)
int64_t sort_hits(gmat_epi *e) {
  const size_t n = e->hit_i.size();
  if (n < 2) return (int64_t)n;
  thread_local std::vector<uint64_t> key, key2, tmp;
  thread_local std::vector<uint32_t> pos, pos2;
  key.resize(n);
  key2.resize(n);
  pos.resize(n);
  pos2.resize(n);
  tmp.resize(n);
  const uint64_t mm = (uint64_t)e->m;
  uint64_t kmax = 0;
  for (size_t k = 0; k < n; ++k) {
    key[k] = (uint64_t)e->hit_i[k] * mm + (uint64_t)e->hit_j[k];
    pos[k] = (uint32_t)k;
    kmax = std::max(kmax, key[k]);
  }
  constexpr int DB = 11, ND = 1 << DB;
  std::vector<uint32_t> cnt(ND + 1);
  for (int sh = 0; sh < 64 && (kmax >> sh) != 0; sh += DB) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    for (size_t k = 0; k < n; ++k) ++cnt[((key[k] >> sh) & (ND - 1)) + 1];
    if (cnt[((key[0] >> sh) & (ND - 1)) + 1] == n) continue;  // one digit value: the pass keeps the order
    for (int d = 0; d < ND; ++d) cnt[d + 1] += cnt[d];
    for (size_t k = 0; k < n; ++k) {
      const uint32_t q = cnt[(key[k] >> sh) & (ND - 1)]++;
      key2[q] = key[k];
      pos2[q] = pos[k];
    }
    key.swap(key2);
    pos.swap(pos2);
  }
  auto apply = [&](auto &v) {
    static_assert(sizeof(v[0]) == 8, "64-bit hit fields");
    for (size_t k = 0; k < n; ++k) std::memcpy(&tmp[k], &v[pos[k]], 8);
    std::memcpy(v.data(), tmp.data(), n * 8);
  };
  apply(e->hit_i);
  apply(e->hit_j);
  apply(e->hit_eff);
  apply(e->hit_var);
  apply(e->hit_chi);
  apply(e->hit_p);
  return (int64_t)n;
}

// owner of the events a scan creates
// a scan's pipeline events, handed out from the plan's pool (event creation costs ~10 us each: ~0.2 ms
// of host time per scan when the compacted scan created its 20 per call)
struct ScanEvents {
  gmat_epi *e;
  size_t used = 0;
  int make(hipEvent_t *x) {
    if (used == e->sev.size()) {
      hipEvent_t ev;
      GMAT_HIP(hipEventCreate(&ev));
      e->sev.push_back(ev);
    }
    *x = e->sev[used++];
    return GMAT_OK;
  }
};

int scan_exhaustive(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, int64_t *n_hits) {
  const double t_start = now();
  const int64_t m = e->m;
  ScanSide c;
  GMAT_TRY(scan_begin(e, kind, &c));
  const int tri = c.tri;
  // chunks of whole rows of at most `cap` pairs (one row holds at most m)
  // (the wide int8 refine keeps R8_S integer partial sums per pair and square of stages: chunks of at
  // most ~2 GB of them)
  const int64_t nQ = cdiv(e->n_pad / 64, R8_NC), nseg_w = e->n_pad > 64 * R8_NC ? nQ * (nQ + 1) / 2 : 1;
  const int64_t dflt = std::min<int64_t>(1 << 24, ((int64_t)1 << 31) / (8 * (1 + R8_S * nseg_w)));
  const int64_t cap = std::max<int64_t>(m, getenv("GMAT_EXH_CHUNK") ? atoll(getenv("GMAT_EXH_CHUNK")) : dflt);
  if (!e->s3) GMAT_TRY(pipeline_stream(2, &e->s3));
  const hipStream_t st = e->s3;
  DBuf di, dj, de, dv, dc, dp, hi, hj, he, hv, hc, hp, cnt, drows, doffs;
  for (DBuf *b : {&di, &dj, &de, &dv, &dc, &dp, &hi, &hj, &he, &hv, &hc, &hp}) GMAT_TRY(b->alloc((size_t)cap * 8));
  GMAT_TRY(cnt.alloc(8));
  GMAT_TRY(drows.alloc((size_t)std::max<int64_t>(n_rows, 1) * 8));
  GMAT_TRY(doffs.alloc((size_t)std::max<int64_t>(n_rows, 1) * 8));
  GMAT_HIP(hipStreamSynchronize(e->s));  // the codings were built on the plan's stream
  ScanEvents evs{e};
  hipEvent_t ev0, ev1;
  GMAT_TRY(evs.make(&ev0));
  GMAT_TRY(evs.make(&ev1));
  double pairs = 0, t_ref = 0;
  std::vector<int64_t> offs;
  std::vector<int64_t> hbuf;
  std::vector<double> dbuf;
  for (int64_t r0 = 0; r0 < n_rows;) {
    offs.clear();
    int64_t np = 0, r1 = r0;
    while (r1 < n_rows && r1 - r0 < 65535) {
      const int64_t c = m - std::max<int64_t>(tri ? rows[r1] + 1 : 0, e->col_lo);
      if (np + c > cap) break;
      offs.push_back(np);
      np += c;
      ++r1;
    }
    const int64_t nr = r1 - r0;
    pairs += (double)np;
    if (np > 0) {
      GMAT_HIP(hipMemcpyAsync(drows.p, rows + r0, nr * 8, hipMemcpyHostToDevice, st));
      GMAT_HIP(hipMemcpyAsync(doffs.p, offs.data(), nr * 8, hipMemcpyHostToDevice, st));
      // the longest row of the chunk (rows increase)
      const int64_t per_row = m - std::max<int64_t>(tri ? rows[r0] + 1 : 0, e->col_lo);
      hipLaunchKernelGGL(all_pairs_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(per_row, 256), 64)),
                                                (unsigned)nr),
                         dim3(256), 0, st, drows.as<int64_t>(), doffs.as<int64_t>(), m, tri, e->col_lo, di.as<int64_t>(),
                         dj.as<int64_t>());
      GMAT_HIP(hipGetLastError());
      GMAT_HIP(hipEventRecord(ev0, st));
      GMAT_TRY(refine(e, st, *c.L, *c.R, c.lp, c.rp, di.as<int64_t>(), dj.as<int64_t>(), np, de.as<double>(),
                      dv.as<double>(), dc.as<double>(), dp.as<double>()));
      GMAT_HIP(hipEventRecord(ev1, st));
      GMAT_HIP(hipMemsetAsync(cnt.p, 0, 8, st));
      hipLaunchKernelGGL(hit_compact_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, np, di.as<int64_t>(),
                         dj.as<int64_t>(), de.as<double>(), dv.as<double>(), dc.as<double>(), dp.as<double>(), p_cut,
                         cnt.as<unsigned long long>(), hi.as<int64_t>(), hj.as<int64_t>(), he.as<double>(),
                         hv.as<double>(), hc.as<double>(), hp.as<double>());
      GMAT_HIP(hipGetLastError());
      unsigned long long k = 0;
      GMAT_HIP(hipMemcpyAsync(&k, cnt.p, 8, hipMemcpyDeviceToHost, st));
      GMAT_HIP(hipStreamSynchronize(st));
      float ms;
      GMAT_HIP(hipEventElapsedTime(&ms, ev0, ev1));
      t_ref += ms * 1e-3;
      if (k) {
        const size_t o = e->hit_i.size();
        for (auto *v : {&e->hit_i, &e->hit_j}) v->resize(o + k);
        for (auto *v : {&e->hit_eff, &e->hit_var, &e->hit_chi, &e->hit_p}) v->resize(o + k);
        GMAT_HIP(hipMemcpy(e->hit_i.data() + o, hi.p, k * 8, hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(e->hit_j.data() + o, hj.p, k * 8, hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(e->hit_eff.data() + o, he.p, k * 8, hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(e->hit_var.data() + o, hv.p, k * 8, hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(e->hit_chi.data() + o, hc.p, k * 8, hipMemcpyDeviceToHost));
        GMAT_HIP(hipMemcpy(e->hit_p.data() + o, hp.p, k * 8, hipMemcpyDeviceToHost));
      }
    }
    r0 = r1;
  }
  *n_hits = sort_hits(e);
  e->stats[0] = pairs;
  e->stats[1] = pairs;  // every pair is refined
  e->stats[4] = t_ref;
  e->stats[6] = now() - t_start;
  e->stats[8] = GMAT_SCREEN_NONE;
  return GMAT_OK;
}

// ---- the compacted low-rank scan (default level for p_cut <= 1e-4 when the plan has the low-rank
// certificate): per launch of 4,096 first SNPs (two folded 2,048-row chunks, equal work; fewer rows
// when the scan would have fewer than eight launches)
//   S2: prefilter (live-pair masks, E3 slices and code products of live blocks) -> slot lists (lc_*)
//   sm: compacted low-rank screen of the launch's slots (candidates appended to cand)
//   S3: pair screen of the candidates in chunks beside the later launches, the exact refine at flush
// The prefilters of launches L + 1 and L + 2 are queued beside launch L's screen (three buffer sets,
// even and odd launches on two streams); the host reads a
// launch's slot count (pinned) to reserve candidate room before queueing its screen, so the
// candidate buffer can never overflow (a screen adds at most 32 per slot).
int scan_lowrank(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut,
                 int64_t *n_hits) {
  const double t_start = now();
  const int64_t m = e->m, n_pad = e->n_pad;
  ScanSide c;
  GMAT_TRY(scan_begin(e, kind, &c));
  const Coding &L = *c.L, &R = *c.R;
  const int8_t *slp = c.slp, *srp = c.srp;
  const int tri = c.tri;
  const int64_t nJ = cdiv(m, BJ);
  auto &B = e->lrc;
  constexpr int NBUF = 3;  // buffer sets: launch L uses set L % 3
  // first SNPs per launch: LRC_ROWS_PER_LAUNCH (7,168: configs[2] in 7 launches, 15.57-15.81 ms per step
  // against 15.99-16.12 at 4,096 in 13, 15.78-15.81 at 6,144, 15.65-16.02 at 8,192 on one box; each launch
  // costs its pipeline turn), but at least GMAT_LRC_MIN_LAUNCHES (6) launches down to
  // 512 rows (a rank's part of a multi-GPU split keeps the prefilter-ahead pipeline filled: rank 0's
  // 8-way part 2.62 ms at 1,024 rows per launch against 2.75 at 1,536, 2.72 at 768, 2.82 at 512), and no more
  // than the three sets' live masks and record bases (8 bytes per (row, 32-column block)) fit in an
  // eighth of the free HBM; GMAT_LRC_ROWS forces it for A/B runs (a multiple of 128, at most 8192)
  int64_t RL = 0;
  {
    const int64_t min_launches = getenv("GMAT_LRC_MIN_LAUNCHES") ? std::max(1, atoi(getenv("GMAT_LRC_MIN_LAUNCHES"))) : 6;
    RL = getenv("GMAT_LRC_ROWS")
             ? std::min<int64_t>(8192, std::max<int64_t>(128, atoll(getenv("GMAT_LRC_ROWS")) / 128 * 128))
             : std::min<int64_t>(LRC_ROWS_PER_LAUNCH, std::max<int64_t>(512, n_rows / min_launches / 128 * 128));
    if (RL > B.rl) {  // buffers sized for fewer rows than this scan wants: is there room?
      size_t free_b = 0, total_b = 0;
      GMAT_HIP(hipMemGetInfo(&free_b, &total_b));
      free_b += pool_cached_bytes();  // blocks the device-memory cache holds are free for the sets
      const int64_t room = (int64_t)((free_b + (size_t)NBUF * 8 * B.rl * nJ) / 8 / (NBUF * 8 * nJ)) / 128 * 128;
      RL = std::max<int64_t>(std::max<int64_t>(B.rl, 128), std::min(RL, room));
    }
  }
  double pairs_tested = 0;
  // Scans of fewer than ten launches (a rank's part of a multi-GPU split) fold into the same number of
  // launches of equal rows (an even number of equal chunks, none left alone) instead of RL-row launches
  // plus a short lone middle chunk.  One-box A/Bs (bench split rehearsal, twice): 2 / 4 / 8-way parts
  // 8.62-8.69 / 4.29-4.34 / 2.42-2.48 ms against 8.78-8.85 / 4.42-4.60 / 2.47-2.52; the configs[2] step
  // (13 launches) keeps the RL-row launches and its half-size last launch (16.05-16.14 against
  // 16.35-16.43 ms; an odd number of equal chunks, the last launch one lone chunk, was no better)
  int64_t fold_rl = RL;
  if (cdiv(n_rows, RL) < 10 && n_rows > RL) fold_rl = 2 * cdiv(n_rows, 2 * cdiv(n_rows, RL));
  const std::vector<ScanLaunch> plan = fold_launches(rows, n_rows, m, tri, &pairs_tested, fold_rl, e->col_lo);
  // live-pair records per launch: an initial capacity of 1/128 of a launch's pairs (at least 2^20; the
  // configs[2] prefilter keeps 1/250), grown (and the launch rerun) when a launch keeps more
  const int64_t rl_sets = std::max(RL, B.rl);
  auto alloc_sets = [&](int64_t rl, int64_t cap) -> int {
    GMAT_CHECK(cap <= ((int64_t)1 << LM_BASE_BITS), GMAT_E_ARG, "compacted scan: %lld live-pair records in one launch "
               "exceed the entries' 2^%d", (long long)cap, LM_BASE_BITS);
    const int64_t max_slots = cap / 32 + rl + 2 * LC_SLOTS;  // a row's last slot may be partial
    for (int b = 0; b < NBUF; ++b) {
      GMAT_TRY(B.drows[b].alloc(rl * 8));
      // a grown entry buffer can be the same block again (the cache hands back what it just took):
      // its rows past the old size hold stale entries, so any change of size forces the full clear
      const size_t lm_before = B.lmask[b].bytes;
      GMAT_TRY(B.lmask[b].alloc((size_t)rl * nJ * sizeof(uint64_t)));
      if (B.lmask[b].bytes != lm_before) B.lm_ptr[b] = nullptr;
      GMAT_TRY(B.ops[b].alloc((size_t)cap * OPS_REC * sizeof(int)));
      GMAT_TRY(B.opc[b].alloc(16));
      GMAT_TRY(B.slot_ops[b].alloc((size_t)max_slots * 32 * OPS_REC * sizeof(int)));
      GMAT_TRY(B.slot_row[b].alloc((size_t)max_slots * sizeof(int)));
      GMAT_TRY(B.slot_j[b].alloc((size_t)max_slots * 32 * sizeof(int)));
      GMAT_TRY(B.cnt[b].alloc(rl * sizeof(int)));
      GMAT_TRY(B.soff[b].alloc(rl * sizeof(int)));
      GMAT_TRY(B.info[b].alloc(4 * sizeof(int)));
      GMAT_TRY(B.tlist[b].alloc((size_t)cdiv(rl, PC_TR) * (cdiv(m, 128) + 1) * sizeof(int)));  // PC tiles: the most
      GMAT_TRY(e->pins.tl[b].reserve((size_t)cdiv(rl, PC_TR) * (cdiv(m, 128) + 1) * sizeof(int)));
      GMAT_TRY(e->pins.rows[b].reserve(rl * 8));
      GMAT_TRY(e->pins.cnt[b].reserve(8));
      GMAT_TRY(e->pins.t2[b].reserve(32));
    }
    B.rl = rl;
    B.ops_cap = cap;
    B.slot_cap = max_slots;
    return GMAT_OK;
  };
  // (GMAT_LRC_OPS_CAP: a smaller logical capacity for this scan -- tests of the grow-and-rerun path)
  GMAT_TRY(alloc_sets(rl_sets, getenv("GMAT_LRC_OPS_CAP")
                                   ? std::max<int64_t>(32, atoll(getenv("GMAT_LRC_OPS_CAP")))
                                   : std::max(B.ops_cap, std::min<int64_t>(1 << 23, std::max<int64_t>(1 << 20, RL * m / 128)))));
  const bool use_ps = pair_screen_fits(e) && !getenv("GMAT_NO_PAIR_SCREEN");
  GMAT_TRY(ensure_candidates(e, 1 << 24, use_ps));
  DBuf live_cnt;  // GMAT_LIVE_COUNT: pairs the prefilter keeps (diagnostics, printed at the end)
  if (getenv("GMAT_LIVE_COUNT")) {
    GMAT_TRY(live_cnt.alloc(8));
    GMAT_HIP(hipMemset(live_cnt.p, 0, 8));
  }
  DBuf pf_st;  // GMAT_PF_STAMPS: per-workgroup phase stamps of the prefilter of launch 5
  const size_t stamp_launch = 5;
  int64_t stamp_grid = 0;
  // the prefilter as a persistent grid over each launch's tile list (GMAT_PF_NOLIST: one workgroup
  // per tile, as the per-tile phase stamps need)
  const bool pf_list = !getenv("GMAT_PF_NOLIST") && !getenv("GMAT_PF_STAMPS");
  // GMAT_PF_WG caps the persistent grid (tests: many tiles per workgroup at small cohorts)
  if (!e->n_cu) {
    int dev = 0, cus = 0;
    GMAT_HIP(hipGetDevice(&dev));
    GMAT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    e->n_cu = std::max(cus, 8);
  }
  // by default 7/8 of the CUs (28 of an XCD's 32): the slot lists and the low-rank screens of the
  // launches before run on the rest instead of waiting for a whole prefilter launch (one-box A/Bs,
  // configs[2]: 18.4 against 19.2 ms per step at 224 against 256 workgroups; 240 and 232 were slower)
  // 32 x 256 tiles of four waves, two workgroups on every CU (round 5; configs[2] one-box A/B: 16.7-16.9
  // against 17.7 ms per step for the former 64 x 256 tiles of eight waves on 7/8 of the CUs, 17.0-17.4 ms
  // for the 32-row tiles on 7/8 of the CUs, 16.6-17.1 on 480 workgroups; a six-slot ring 16.9-17.0 ms)
  constexpr int pf_tr = 32;
  const int pf_wg = getenv("GMAT_PF_WG") ? std::max(8, atoi(getenv("GMAT_PF_WG"))) : std::max(8, 2 * e->n_cu);
  // covariate designs: 32 x 128 tiles of four waves, two workgroups on every CU (covariate configs[2]
  // 32.0 against 33.5 ms per step for 32 x 256 tiles of eight waves on 7/8 of the CUs)
  constexpr int pc_tc = 128;
  const int pc_wg = pf_wg;
  constexpr int pf_rg = 8;  // row tiles per tile-list block (256 rows)
  if (getenv("GMAT_PF_STAMPS")) {
    GMAT_TRY(pf_st.alloc((size_t)PF_NSTAMP * 8 * 1 << 20));
    GMAT_HIP(hipMemset(pf_st.p, 0, (size_t)PF_NSTAMP * 8 * 1 << 20));
  }
  if (!e->s1) GMAT_TRY(pipeline_stream(0, &e->s1));
  if (!e->s2) GMAT_TRY(pipeline_stream(1, &e->s2));
  if (!e->s3) GMAT_TRY(pipeline_stream(2, &e->s3));
  if (!e->s4) GMAT_TRY(pipeline_stream(3, &e->s4));
  // the prefilter passes of even / odd launches on two streams: launch L + 1 (other buffer set) can
  // start on the CUs that the tail of launch L leaves idle (a launch's ~800 equal tiles fill its last
  // round of 256 CUs only partly; on one stream the next launch would wait for the whole tail)
  const hipStream_t sm = e->s1, S3 = e->s3;
  const hipStream_t S2b[2] = {e->s2, e->s4};
  // (the slot lists: after each prefilter on its stream, below; round 5 put those of launches of 4,096 rows or
  // more on the screen stream, where the former workgroup-per-row list kernels measured faster)
  GMAT_HIP(hipStreamSynchronize(e->s));  // the codings were built on the plan's stream
  ScanEvents evs{e};
  hipEvent_t side_beg[NBUF], side_end[NBUF], scr_beg[NBUF], scr_end[NBUF], pf_beg[NBUF], pf_end[NBUF], ref_beg, ref_end;
  double t_pf = 0, pf_ops = 0;
  std::vector<double> pf_ops_of(plan.size(), 0.0);
  for (int b = 0; b < NBUF; ++b) {
    GMAT_TRY(evs.make(&pf_beg[b]));
    GMAT_TRY(evs.make(&pf_end[b]));
    GMAT_TRY(evs.make(&side_beg[b]));
    GMAT_TRY(evs.make(&side_end[b]));
    GMAT_TRY(evs.make(&scr_beg[b]));
    GMAT_TRY(evs.make(&scr_end[b]));
    GMAT_HIP(hipEventRecord(scr_end[b], sm));  // buffer sets free at the start
  }
  GMAT_TRY(evs.make(&ref_beg));
  GMAT_TRY(evs.make(&ref_end));
  GMAT_HIP(hipMemsetAsync(e->counter.p, 0, 8, sm));
  double t_screen = 0, t_side = 0, ops = 0;
  RefineTally tally;
  // candidates pair-screened beside the launches once at least ps_chunk are pending (one-box A/Bs,
  // configs[2] at ~60 k candidates per launch: 17.6-17.8 ms per step at 32 k, 48 k and 128 k against
  // 18.3-18.5 at 64 k and 96 k; rank 0's 8-way part 2.78-2.84 ms at 48 k against 2.76-2.82 at 64 k and
  // 2.84-2.94 at 32 k, 96 k and 128 k)
  const int64_t ps_chunk = getenv("GMAT_PS_CHUNK") ? atoll(getenv("GMAT_PS_CHUNK")) : 49152;
  int64_t ps_done = 0;  // candidates [0, ps_done) already pair-screened (queued on S3)
  // candidate room: known_count (exact, after the last screen whose count was read) + inflight (32 per
  // slot of the screen queued since) bounds the buffer's fill
  int64_t known_count = 0, inflight = 0;
  // the prefilter pass and the slot lists of launch li into buffer set b (stream S2)
  auto enqueue_side = [&](size_t li, int b) -> int {
    const hipStream_t S2 = S2b[li & 1];
    const ScanLaunch &ln = plan[li];
    const int Rn = (int)ln.rows.size();
    GMAT_HIP(hipStreamWaitEvent(S2, scr_end[b], 0));  // buffer set b free (screen three launches back)
    std::memcpy(e->pins.rows[b].p, ln.rows.data(), Rn * 8);
    GMAT_HIP(hipMemcpyAsync(B.drows[b].p, e->pins.rows[b].p, Rn * 8, hipMemcpyHostToDevice, S2));
    GMAT_HIP(hipEventRecord(side_beg[b], S2));
    // the set's live-block entries: a fresh tag per launch (1..63); a new buffer or a spent tag range
    // clears the whole buffer first (every 63rd launch of the set, instead of a launch's masks each time)
    if (B.lm_ptr[b] != B.lmask[b].p || B.ltag[b] >= 63) {
      GMAT_HIP(hipMemsetAsync(B.lmask[b].p, 0, B.lmask[b].bytes, S2));
      B.lm_ptr[b] = B.lmask[b].p;
      B.ltag[b] = 0;
    }
    const unsigned tag = ++B.ltag[b];
    GMAT_HIP(hipMemsetAsync(B.opc[b].p, 0, 16, S2));
    SideArgs x{};
    ScreenArgs &a = x.a;
    std::memset(&a, 0, sizeof(a));
    a.n_pad = n_pad;
    a.left = slp;
    a.right = srp;
    a.m = m;
    a.rows = B.drows[b].as<int64_t>();
    a.n_rows = Rn;
    a.tri = tri;
    a.sL3 = L.sL3.as<double>();
    a.csum_l = L.csum.as<double>();
    a.csum_r = R.csum.as<double>();
    a.csq_l = L.csq.as<double>();
    a.csq_r = R.csq.as<double>();
    a.ops = B.ops[b].as<int>();  // one record per live pair (no dense per-pair arrays)
    a.ops_count = B.opc[b].as<unsigned>();
    a.ops_cap = B.ops_cap;
    a.pf_mu = e->pf_mu;
    a.pf_eps = e->pf_eps;
    a.pf_tau = e->pf_tau;
    a.pf_ncov = e->pf_ncov;
    a.pf_ku = e->pf_ku;
    for (int k = 0; k < 4; ++k) a.pf_su[k] = e->pf_su[k];
    for (int k = 0; k < 4; ++k) a.pf_sq[k] = e->pf_sq[k];
    a.pf_ua = e->pf_ncov ? L.uc.as<double>() : nullptr;
    a.pf_ub = e->pf_ncov ? R.uc.as<double>() : nullptr;
    x.qimg = e->pf_q.as<uint8_t>();
    a.n_id = (double)e->n;
    a.flags = nullptr;
    a.lmask = B.lmask[b].as<uint64_t>();
    a.ltag = tag;
    a.live_count = live_cnt.p ? live_cnt.as<unsigned long long>() : nullptr;
    a.pf_stamp = (pf_st.p && li == stamp_launch) ? pf_st.as<unsigned long long>() : nullptr;
    a.nJ = (int)nJ;
    a.e3_t = E3_PF;
    a.e3_eps = 0.5 * std::pow(128.0, -(E3_PF - 1)) + 1e-12;
    a.ld_e = m;
    a.j_lo = ln.j_lo;
    a.alpha = L.soff.as<double>();
    a.sa = L.sa.as<double>();
    a.beta = R.soff.as<double>();
    a.sb = R.sb.as<double>();
    a.mono_l = L.mono.as<uint8_t>();
    a.mono_r = R.mono.as<uint8_t>();
    a.spy = e->spy;
    a.chi_cut = chi_cut;
    x.n_pad = n_pad;
    const int64_t ss = m * n_pad;
    const int64_t ncols = m - (ln.j_lo / 32) * 32;
    for (int t = 0; t < E3_PF; ++t) x.rs[t] = L.L3q.as<int8_t>() + t * ss;
    x.cs[0] = srp;
    x.rs4 = L.p4.as<uint8_t>();
    x.cs4 = R.p4.as<uint8_t>();
    x.blocked = 0;
    x.tile_list = nullptr;
    x.n_list = 0;
    x.recL = L.pfRecL.as<float>();
    x.recR = R.pfRecR.as<float>();
    if (e->pf_ncov == 0) {  // prefilter_pass_kernel reads stage-blocked operands
      x.blocked = 1;
      for (int t = 0; t < E3_PF; ++t) x.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;
      x.rs2 = L.p2b.as<uint8_t>();
      x.cs2 = R.p2b.as<uint8_t>();
      x.n_rt = (int)cdiv(Rn, pf_tr);
      // the tiles that run (a tile entirely left of the diagonal has no pair), in tile order
      // rt + n_rt ct; MFMA work per pair: 4 fp4 code products + 2 int8 E3 slices over n_pad
      // individuals = 16 n_pad fp4-equivalent ops
      int *tl = e->pins.tl[b].as<int>();
      int run = 0;
      const int64_t n_ct = cdiv(ncols, PF_TC);
      auto runs = [&](int rt, int64_t ct) {
        const int64_t c0 = (ln.j_lo / 32) * 32 + ct * PF_TC;
        return c0 < m && !(tri && c0 + PF_TC - 1 <= ln.rows[rt * pf_tr]);
      };
      // blocks of 4 row tiles x 8 column tiles (the 32 workgroups of an XCD run one block at a time:
      // 4 row and 8 column panels per stage instead of 32 + 1), blocks of a row group consecutive
      // (its rows stay in L2 while the columns stream), row groups dealt to the XCDs in eighths
      // (round 3 A/B: 23.8 against 24.2 ms per configs[2] step for the column-tile-major list)
      const int rgs = pf_rg;  // row tiles per block (default 256 rows)
      for (int rg = 0; rg < x.n_rt; rg += rgs)
        for (int64_t cg = 0; cg < n_ct; cg += 8)
          for (int64_t ct = cg; ct < std::min(n_ct, cg + 8); ++ct)
            for (int rt = rg; rt < std::min(x.n_rt, rg + rgs); ++rt)
              if (runs(rt, ct)) tl[run++] = rt + x.n_rt * (int)ct;
      pf_ops_of[li] = (double)run * pf_tr * PF_TC * 16.0 * (double)n_pad;
      GMAT_HIP(hipEventRecord(pf_beg[b], S2));
      // persistent grid over the list: one workgroup per CU (a multiple of 8).  (Same-box A/B: 27.6
      // against 27.7 ms per configs[2] step for as few workgroups as finish in the same number of
      // tile rounds, and 28.0 against 28.2 for one workgroup per tile, GMAT_PF_NOLIST: a grid of as many
      // workgroups as tiles, which the per-tile phase stamps use.)
      GMAT_HIP(hipMemcpyAsync(B.tlist[b].p, tl, (size_t)run * sizeof(int), hipMemcpyHostToDevice, S2));
      x.tile_list = B.tlist[b].as<int>();
      x.n_list = run;
      const int g = 8 * (int)(pf_list ? std::min<int64_t>(cdiv(pf_wg, 8), cdiv(run, 8)) : cdiv(run, 8));
      if (!pf_list && li == stamp_launch) stamp_grid = g;
      if (run > 0) {
        if (x.a.pf_stamp)  // the phase-stamped build (GMAT_PF_STAMPS)
          hipLaunchKernelGGL((prefilter_pass_kernel<true, true, true, 32, 5>), dim3((unsigned)g), dim3(256), 0, S2, x);
        else
          hipLaunchKernelGGL((prefilter_pass_kernel<true, true, false, 32, 5>), dim3((unsigned)g), dim3(256), 0, S2, x);
      }
      GMAT_HIP(hipEventRecord(pf_end[b], S2));
    } else {
      for (int t = 0; t < E3_PF; ++t) x.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;  // stage-blocked operands
      x.rs2 = L.p2b.as<uint8_t>();
      x.cs2 = R.p2b.as<uint8_t>();
      x.n_rt = (int)cdiv(Rn, PC_TR);
      // the running 32 x pc_tc tiles in blocks of 8 row x (2048 / pc_tc) column tiles (256 x 2,048, as the
      // intercept-only prefilter's list), a persistent grid over them (GMAT_PF_NOLIST: one per tile)
      int *tl = e->pins.tl[b].as<int>();
      int run = 0;
      const int64_t n_ct = cdiv(ncols, pc_tc), cgs = 2048 / pc_tc;
      for (int rg = 0; rg < x.n_rt; rg += 8)
        for (int64_t cg = 0; cg < n_ct; cg += cgs)
          for (int64_t ct = cg; ct < std::min(n_ct, cg + cgs); ++ct)
            for (int rt = rg; rt < std::min(x.n_rt, rg + 8); ++rt) {
              const int64_t c0 = (ln.j_lo / 32) * 32 + ct * pc_tc;
              if (c0 < m && !(tri && c0 + pc_tc - 1 <= ln.rows[rt * PC_TR])) tl[run++] = rt + x.n_rt * (int)ct;
            }
      // MFMA work per pair: 4 fp4 code products + (2 + K0) int8 products over n_pad individuals
      pf_ops_of[li] = (double)run * PC_TR * pc_tc * (8.0 + 4.0 * (2 + e->pf_ncov)) * (double)n_pad;
      GMAT_HIP(hipEventRecord(pf_beg[b], S2));
      // persistent (one-box A/B, covariate configs[2] step: 35.8 against 41.9 ms for one workgroup per
      // tile, GMAT_PF_NOLIST; the persistent variant spills a few registers at three or four directions)
      if (run > 0 && pf_list) {
        GMAT_HIP(hipMemcpyAsync(B.tlist[b].p, tl, (size_t)run * sizeof(int), hipMemcpyHostToDevice, S2));
        x.tile_list = B.tlist[b].as<int>();
        x.n_list = run;
        const dim3 gp((unsigned)(8 * (int)std::min<int64_t>(cdiv(pc_wg, 8), cdiv(run, 8))));
        const dim3 bd((unsigned)(2 * pc_tc));
#define PC_LAUNCH(NC_, L_) hipLaunchKernelGGL((prefilter_cov_kernel<NC_, L_, pc_tc>), gp, bd, 0, S2, x)
        switch (e->pf_ncov) {
          case 1: PC_LAUNCH(1, true); break;
          case 2: PC_LAUNCH(2, true); break;
          case 3: PC_LAUNCH(3, true); break;
          default: PC_LAUNCH(4, true); break;
        }
      } else if (run > 0) {
        const dim3 gp((unsigned)(x.n_rt * n_ct));
        const dim3 bd((unsigned)(2 * pc_tc));
        if (li == stamp_launch) stamp_grid = x.n_rt * n_ct;
        switch (e->pf_ncov) {
          case 1: PC_LAUNCH(1, false); break;
          case 2: PC_LAUNCH(2, false); break;
          case 3: PC_LAUNCH(3, false); break;
          default: PC_LAUNCH(4, false); break;
        }
#undef PC_LAUNCH
      }
      GMAT_HIP(hipEventRecord(pf_end[b], S2));
    }
    GMAT_HIP(hipGetLastError());
    // the slot lists after the prefilter on its stream (round 6, with the one-wave-per-row list kernels:
    // configs[2] 14.95-14.96 against 15.00-15.01 ms per step on the screen stream, one box; a prefilter
    // also waiting for the screen two launches back: 18.5 ms)
    const hipStream_t SL = S2;
    hipLaunchKernelGGL(lc_count_kernel, dim3((unsigned)cdiv(Rn, LC_T / 64)), dim3(LC_T), 0, SL, B.lmask[b].as<uint64_t>(), tag,
                       (int)nJ, Rn,
                       B.cnt[b].as<int>());
    hipLaunchKernelGGL(lc_scan_kernel, dim3(1), dim3(1024), 0, SL, B.cnt[b].as<int>(), Rn, B.soff[b].as<int>(),
                       B.info[b].as<int>(), B.slot_row[b].as<int>(), B.slot_cap);
    hipLaunchKernelGGL(lc_fill_kernel, dim3((unsigned)cdiv(Rn, LC_T / 64)), dim3(LC_T), 0, SL, B.lmask[b].as<uint64_t>(), tag,
                       (int)nJ, Rn,
                       B.cnt[b].as<int>(), B.soff[b].as<int>(), B.slot_row[b].as<int>(), B.slot_j[b].as<int>(),
                       B.ops[b].as<int>(), B.ops_cap, B.slot_ops[b].as<int>(), B.slot_cap);
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpyAsync(e->pins.t2[b].p, B.info[b].p, 4 * sizeof(int), hipMemcpyDeviceToHost, SL));
    GMAT_HIP(hipMemcpyAsync(e->pins.t2[b].as<int>() + 4, B.opc[b].p, sizeof(int), hipMemcpyDeviceToHost, SL));
    GMAT_HIP(hipEventRecord(side_end[b], SL));
    return GMAT_OK;
  };
  // (Refining each pair-screen chunk's survivors beside the later launches instead of all of them at
  // flush time was measured slower: 32.7 vs 28.4 ms per configs[2] step -- refine workgroups hold
  // CUs that the whole-CU prefilter workgroups then wait for.)
  // pair screen of what is left, refine of candidates [0, count), hits collected.  (Refining what
  // the earlier launches left beside the last launch's screen, so that the refine does not run alone
  // at the end, was measured slower too: 24.4 vs 22.7 ms per configs[2] step on one box.)
  auto flush = [&](int64_t count) -> int {
    const int64_t done = ps_done;
    ps_done = 0;
    return refine_collect(e, c, S3, use_ps, 0, count, done, chi_cut, p_cut, ref_beg, ref_end, &tally);
  };
  auto read_count = [&](int b) -> int64_t { return (int64_t)*e->pins.cnt[b].as<unsigned long long>(); };
  ScreenArgs sa;
  std::memset(&sa, 0, sizeof(sa));
  sa.m = m;
  sa.tri = tri;
  sa.n_id = (double)e->n;
  sa.e3_t = E3_PF;
  sa.e3_eps = 0.5 * std::pow(128.0, -(E3_PF - 1)) + 1e-12;
  sa.ld_e = m;
  sa.spy = e->spy;
  sa.chi_cut = chi_cut;
  sa.counter = e->counter.as<unsigned long long>();
  LrcArgs lx;
  lx.tiles = e->lr_tiles.as<uint8_t>();
  lx.nib_i = L.nibI.as<uint8_t>();
  lx.nib_j = R.nibJ.as<uint8_t>();
  lx.s1c2 = R.s1c2.as<uint8_t>();
  lx.nK = e->nK;
  lx.nC = e->lr_R / MXK;
  lx.R = e->lr_R;
  lx.G = L.lrGa.as<float>();
  lx.H = R.lrG.as<float>();
  lx.recL = L.lrRecL.as<double>();
  lx.recR = R.lrRecR.as<double>();
  lx.lam = e->lr_lam;
  lx.tau = e->lr_tau;
  lx.eps = e->lr_eps;
  lx.E = e->lr_E;
  int64_t prev_count = 0;  // candidates after the previous launch's screen (known once it completed)
  // the prefilters of the next launch(es) queued ahead of the screen being launched (the prefilter
  // streams never wait for a host round trip between launches).  Round 3, every CU in the prefilter
  // grid: 28.0 ms per configs[2] step two launches ahead against 28.6 one ahead; round 4
  // (one-box A/Bs with the 7/8 prefilter grid: 18.25 against 18.41 ms per configs[2] step one launch
  // ahead against two; 3.12 against 3.14-3.19 ms for rank 0's part of an 8-way split)
  const size_t ahead = 1;
  const double t_setup = now();
  for (size_t li = 0; li < std::min<size_t>(ahead, plan.size()); ++li) GMAT_TRY(enqueue_side(li, (int)li));
  const double t_enq0 = now();
  for (size_t li = 0; li < plan.size(); ++li) {
    const int b = (int)(li % NBUF);
    const ScanLaunch &ln = plan[li];
    if (li + ahead < plan.size()) GMAT_TRY(enqueue_side(li + ahead, (int)((li + ahead) % NBUF)));
    GMAT_HIP(hipEventSynchronize(side_end[b]));
    // the prefilter kept more pairs than the record buffers hold: grow them and rerun the launches
    // whose side passes are queued (none of their records can be trusted; the screens before are done)
    while ((int64_t)e->pins.t2[b].as<unsigned>()[4] > B.ops_cap) {
      const int64_t need = (int64_t)e->pins.t2[b].as<unsigned>()[4];
      GMAT_HIP(hipDeviceSynchronize());
      GMAT_TRY(alloc_sets(B.rl, std::max<int64_t>(2 * B.ops_cap, need + need / 4)));
      if (getenv("GMAT_DEBUG")) fprintf(stderr, "live-pair records grown to %lld\n", (long long)B.ops_cap);
      for (size_t lj = li; lj < std::min(plan.size(), li + ahead + 1); ++lj) GMAT_TRY(enqueue_side(lj, (int)(lj % NBUF)));
      GMAT_HIP(hipEventSynchronize(side_end[b]));
    }
    const int *info = e->pins.t2[b].as<int>();
    const int64_t slots = info[0], tiles = info[1];
    float ms_side;
    GMAT_HIP(hipEventElapsedTime(&ms_side, side_beg[b], side_end[b]));
    t_side += ms_side * 1e-3;
    if (pf_ops_of[li] > 0) {
      float ms_pf;
      GMAT_HIP(hipEventElapsedTime(&ms_pf, pf_beg[b], pf_end[b]));
      t_pf += ms_pf * 1e-3;
      pf_ops += pf_ops_of[li];
    }
    // candidate room: a screen adds at most 32 per slot
    bool flushed = false;  // the candidates of the earlier launches were refined just now
    if (known_count + inflight + 32 * slots > e->cand_cap) {
      flushed = true;
      GMAT_HIP(hipStreamSynchronize(sm));
      GMAT_HIP(hipMemcpy(e->pins.cnt[b].p, e->counter.p, 8, hipMemcpyDeviceToHost));
      GMAT_TRY(flush(read_count(b)));
      GMAT_HIP(hipMemsetAsync(e->counter.p, 0, 8, sm));
      known_count = inflight = 0;
      prev_count = 0;
      if (32 * slots > e->cand_cap) GMAT_TRY(grow_candidates(e, 2 * 32 * slots, use_ps));  // nothing pending
    }
    sa.rows = B.drows[b].as<int64_t>();
    sa.n_rows = (int)ln.rows.size();
    sa.j_lo = ln.j_lo;
    sa.cap = e->cand_cap;
    sa.cand_i = e->cand_i.as<int64_t>();
    sa.cand_j = e->cand_j.as<int64_t>();
    lx.slot_row = B.slot_row[b].as<int>();
    lx.slot_j = B.slot_j[b].as<int>();
    lx.slot_ops = B.slot_ops[b].as<int>();
    GMAT_HIP(hipStreamWaitEvent(sm, side_end[b], 0));
    GMAT_HIP(hipEventRecord(scr_beg[b], sm));
    if (tiles > 0) {
      // (one-box A/Bs: 18.3 against 19.3 ms per configs[2] step for the 2-bit j side against the nibble
      // plane; a four-slot ring with it measured 18.4 against 18.2 ms)
      hipLaunchKernelGGL((lrc_screen_kernel<3>), dim3((unsigned)tiles), dim3(512), 0, sm, sa, lx);
    }
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpyAsync(e->pins.cnt[b].p, e->counter.p, 8, hipMemcpyDeviceToHost, sm));
    GMAT_HIP(hipEventRecord(scr_end[b], sm));
    ops += (double)tiles * 2.0 * (double)e->lr_R * (double)n_pad * LC_SLOTS * 32;  // incl. empty slots
    inflight = 32 * slots;
    // the previous launch's screen has completed (or is about to): pair-screen its candidates on S3
    if (li > 0) {
      const int pb = (int)((li - 1) % NBUF);
      GMAT_HIP(hipEventSynchronize(scr_end[pb]));
      float ms;
      GMAT_HIP(hipEventElapsedTime(&ms, scr_beg[pb], scr_end[pb]));
      t_screen += ms * 1e-3;
      prev_count = flushed ? 0 : read_count(pb);
      known_count = prev_count;  // exact after screen li - 1
      if (use_ps && !flushed && prev_count - ps_done >= ps_chunk) {
        GMAT_HIP(hipStreamWaitEvent(S3, scr_end[pb], 0));
        GMAT_TRY(pair_screen(e, S3, L, R, slp, srp, e->cand_i.as<int64_t>() + ps_done, e->cand_j.as<int64_t>() + ps_done,
                             prev_count - ps_done, chi_cut, nullptr, ps_done == 0));
        ps_done = prev_count;
      }
    }
  }
  GMAT_HIP(hipStreamSynchronize(sm));
  const double t_loop = now();
  if (!plan.empty()) {
    const int lb = (int)((plan.size() - 1) % NBUF);
    float ms;
    GMAT_HIP(hipEventElapsedTime(&ms, scr_beg[lb], scr_end[lb]));
    t_screen += ms * 1e-3;
    GMAT_TRY(flush(read_count(lb)));
  }
  const double t_flush = now();
  *n_hits = sort_hits(e);
  if (getenv("GMAT_HOST_T"))  // host-side phases of the scan (diagnostics)
    fprintf(stderr, "scan host: setup %.1f us, first enqueue %.1f, launches %.1f, flush %.1f, sort %.1f (%lld hits)\n",
            (t_setup - t_start) * 1e6, (t_enq0 - t_setup) * 1e6, (t_loop - t_enq0) * 1e6, (t_flush - t_loop) * 1e6,
            (now() - t_flush) * 1e6, (long long)*n_hits);
  e->stats[0] = pairs_tested;
  e->stats[1] = tally.n_cand;
  e->stats[2] = ops;
  e->stats[3] = t_screen;
  e->stats[4] = tally.t_ref;
  e->stats[5] = t_side;
  e->stats[6] = now() - t_start;
  e->stats[7] = (double)plan.size();
  e->stats[8] = -1;
  e->stats[9] = e->lr_lam;
  e->kstats[0] = t_pf;
  e->kstats[1] = pf_ops > 0 ? (double)plan.size() : 0.0;
  e->kstats[2] = pf_ops;
  e->kstats[3] = t_screen;
  e->kstats[4] = (double)plan.size();
  e->kstats[5] = ops;
  e->kstats[6] = tally.t_ref;
  e->kstats[7] = -1;
  if (pf_st.p && stamp_grid > 0 && stamp_grid <= (1 << 20)) {  // phase times of the stamped launch
    std::vector<unsigned long long> hs((size_t)PF_NSTAMP * stamp_grid);
    GMAT_HIP(hipMemcpy(hs.data(), pf_st.p, hs.size() * 8, hipMemcpyDeviceToHost));
    double d[PF_NPHASE - 1] = {0, 0, 0, 0, 0, 0}, clk = 0.0;
    unsigned long long t_min = ~0ull, t_max = 0;
    int64_t nw = 0;
    for (int64_t g = 0; g < stamp_grid; ++g) {
      const unsigned long long *q = &hs[PF_NSTAMP * g];
      if (!q[0] || !q[PF_NPHASE - 1]) continue;  // tiles that exit at once
      ++nw;
      for (int k = 0; k + 1 < PF_NPHASE; ++k) d[k] += (double)(q[k + 1] - q[k]) * 0.01;  // 100 MHz ticks -> us
      // the shader clock over the tile: s_memtime ticks per s_memrealtime tick (100 MHz)
      clk += (double)(q[PF_NPHASE + 1] - q[PF_NPHASE]) / (double)std::max<unsigned long long>(q[PF_NPHASE - 1] - q[0], 1) * 0.1;
      t_min = std::min(t_min, q[0]);
      t_max = std::max(t_max, q[PF_NPHASE - 1]);
    }
    const double nn = (double)std::max<int64_t>(nw, 1);
    fprintf(stderr, "prefilter launch %zu: %lld tiles run, per tile: prologue %.2f us, main loop %.2f us, epilogue "
            "%.2f us (column records %.2f, tests %.2f, stores %.2f, masks %.2f); launch span %.1f us; s_memtime "
            "clock %.3f GHz\n", stamp_launch, (long long)nw, d[0] / nn, d[1] / nn, (d[2] + d[3] + d[4] + d[5]) / nn,
            d[2] / nn, d[3] / nn, d[4] / nn, d[5] / nn, (double)(t_max - t_min) * 0.01, clk / nn);
  }
  if (live_cnt.p) {
    unsigned long long lcnt = 0;
    GMAT_HIP(hipMemcpy(&lcnt, live_cnt.p, 8, hipMemcpyDeviceToHost));
    e->kstats[7] = (double)lcnt;
    fprintf(stderr, "gmat_epi_scan (compacted): %.0f pairs, prefilter keeps %llu pairs (%.4f%%), %.0f low-rank candidates, "
            "%.0f refined\n", pairs_tested, lcnt, 100.0 * (double)lcnt / std::max(pairs_tested, 1.0), tally.n_cand,
            tally.n_refined);
  }
  if (getenv("GMAT_DEBUG"))
    fprintf(stderr, "gmat_epi_scan (compacted): %zu launches, %.0f candidates, %.0f refined, screen %.3f s, side %.3f s\n",
            plan.size(), tally.n_cand, tally.n_refined, t_screen, t_side);
  return GMAT_OK;
}


// ---- the block-granular scan: the int8 slice screens (p_cut > 1e-4), the MX quadratic form
// (n_slice -1) and the low-rank screen when the compacted scan cannot serve it (n_pad > 8064: the pair
// screen does not fit in LDS; GMAT_LR_BLOCKS=1 for A/B runs).  Per launch of 512 first SNPs:
//   S2: side terms (prefilter flags + E3, or the int8 side GEMMs E1 / Ed / E2) into buffer set L % 2
//   sm: the screen over the launch's tile list (candidates appended to cand)
//   S3: pair screen + exact refine when the candidate buffer is flushed
int scan_blocks(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut, int n_slice,
                int64_t *n_hits) {
  const double t_start = now();
  const int64_t m = e->m, n_pad = e->n_pad;
  ScanSide c;
  GMAT_TRY(scan_begin(e, kind, &c));
  const int lc = c.lc, rc = c.rc;
  {
    const double t0 = now();
    GMAT_TRY(block_sides(e, lc));
    GMAT_TRY(block_sides(e, rc));
    e->setup[5] += now() - t0;
  }
  const Coding &L = *c.L, &R = *c.R;
  const int8_t *slp = c.slp, *srp = c.srp, *srq = screen_sq(e, rc), *slq = screen_sq(e, lc);  // screen codes
  const int tri = c.tri;
  // tile shape of the int8 screen: Shape<SCREEN_SHAPE>
  // screen level S: 0 = MX (fp6 x fp4, one pass, tighter than one int8 slice), 1..n_slice = int8
  // slices.  Automatic: MX when the candidate band stays thin (p_cut <= 1e-4), 2 slices up to
  // p_cut 1e-2, else all; n_slice > 0 forces S slices, n_slice < 0 forces MX.  A launch whose
  // candidates overflow the buffer is redone one level finer (and the scan keeps that level).
  // Level 0 runs the low-rank screen when the plan has one (n_slice -1 forces the MX quadratic
  // form, -2 the low-rank screen).
  GMAT_CHECK(n_slice >= -2, GMAT_E_ARG, "n_slice %d < -2", n_slice);
  GMAT_CHECK(n_slice != -2 || e->lr_R > 0, GMAT_E_ARG, "n_slice -2: this plan has no low-rank screen certificate");
  int S = n_slice > 0 ? n_slice
                      : (n_slice < 0 ? 0 : (p_cut <= 1e-4 ? 0 : std::min(e->n_slice, p_cut <= 1e-2 ? 2 : 4)));
  GMAT_CHECK(S >= 0 && S <= e->n_slice, GMAT_E_ARG, "n_slice %d not in [1, %d]", S, e->n_slice);
  int S_max_used = S;
  constexpr int BI = Shape<SCREEN_SHAPE>::BI, MT = Shape<SCREEN_SHAPE>::MT;
  GMAT_CHECK(n_pad % MT == 0, GMAT_E_ARG, "n_pad %lld is not a multiple of the K-block %d", (long long)n_pad, MT);
  double pairs_tested = 0;
  std::vector<ScanLaunch> plan = fold_launches(rows, n_rows, m, tri, &pairs_tested, ROWS_PER_LAUNCH, e->col_lo);

  // Two buffer sets: the side GEMMs of launch L+1 (stream s2) run while the screen of launch
  // L (stream sm) is in flight; each buffer set is rewritten only after the screen that
  // read it has completed (event wait).
  const int64_t max_tiles = (ROWS_PER_LAUNCH / BI) * cdiv(m, BJ);
  auto &drows = e->sb.drows, &dtiles = e->sb.dtiles, &bl = e->sb.bl, &ba = e->sb.ba, &e13 = e->sb.e13, &e2 = e->sb.e2,
       &pfc = e->sb.pfc, &flags = e->sb.flags, &mxt = e->sb.mxt, &mxr = e->sb.mxr;
  bool side_full[2] = {false, false};  // band arrays hold E1 / Ed / E2 too (int8 screens need them)
  int e3_slices[2] = {SIDE_T, SIDE_T};  // E3 slices in the band arrays of each buffer set
  const int64_t nJ = cdiv(m, BJ), max_mx = (ROWS_PER_LAUNCH / MX_BI) * nJ + 16;
  const bool use_pf = e->pf_mu > 0.0 && !getenv("GMAT_NO_PREFILTER");
  const bool use_lr = use_pf && e->lr_R > 0 && n_slice != -1;  // level 0 = low-rank screen
  // low-rank screen tile lists built on the device right behind the prefilter (tl_*_kernel): the
  // host waits only for the tile count, not for the flags and a host-side build
  DBuf tl_cnt, tl_h, tl_info;
  DBuf live_cnt;  // GMAT_LIVE_COUNT: pairs the prefilter keeps (diagnostics, printed at the end)
  if (getenv("GMAT_LIVE_COUNT")) {
    GMAT_TRY(live_cnt.alloc(8));
    GMAT_HIP(hipMemset(live_cnt.p, 0, 8));
  }
  if (use_lr) {
    GMAT_TRY(tl_cnt.alloc((size_t)TL_G * nJ * sizeof(int)));
    GMAT_TRY(tl_h.alloc((size_t)nJ * sizeof(int)));
    GMAT_TRY(tl_info.alloc(2 * 4 * sizeof(int)));
  }
  for (int b = 0; b < 2; ++b) {
    GMAT_TRY(drows[b].alloc(ROWS_PER_LAUNCH * 8));
    GMAT_TRY(dtiles[b].alloc((size_t)max_tiles * 2 * sizeof(int)));
    GMAT_TRY(bl[b].alloc((size_t)SIDE_T * SIDE_P * ROWS_PER_LAUNCH * n_pad));
    GMAT_TRY(ba[b].alloc((size_t)2 * ROWS_PER_LAUNCH * n_pad));
    GMAT_TRY(mxt[b].alloc((size_t)max_mx * MX_TE * sizeof(int)));
    GMAT_TRY(mxr[b].alloc((size_t)max_mx * MX_BI * sizeof(int)));
    if (use_pf) {
      GMAT_TRY(pfc[b].alloc((size_t)4 * ROWS_PER_LAUNCH * m * sizeof(int)));
      GMAT_TRY(flags[b].alloc((size_t)ROWS_PER_LAUNCH * nJ));
    }
    GMAT_TRY(e13[b].alloc((size_t)SIDE_T * SIDE_P * ROWS_PER_LAUNCH * m * sizeof(int)));
    GMAT_TRY(e2[b].alloc((size_t)SIDE_T * ROWS_PER_LAUNCH * m * sizeof(int)));
  }
  // pair screen between the screens and the refine (GMAT_NO_PAIR_SCREEN: off, for A/B runs)
  const bool use_ps = pair_screen_fits(e) && !getenv("GMAT_NO_PAIR_SCREEN");
  GMAT_TRY(ensure_candidates(e, 1 << 22, use_ps));
  // scan-private streams (the null stream would serialise them): screen on sm, side terms on S2,
  // pair screen + refine on S3; ordered after the coding setup by a device synchronisation
  // (Refining launch by launch beside the screens was measured 2.7x slower overall: refine waves
  // occupy CUs that a screen workgroup, which needs a whole CU, then waits for.)
  if (!e->s1) GMAT_TRY(pipeline_stream(0, &e->s1));
  if (!e->s2) GMAT_TRY(pipeline_stream(1, &e->s2));
  if (!e->s3) GMAT_TRY(pipeline_stream(2, &e->s3));
  const hipStream_t sm = e->s1, S2 = e->s2, S3 = e->s3;
  GMAT_HIP(hipDeviceSynchronize());
  ScanEvents evs{e};
  // per buffer set: side pass begin / end, screen begin / end (+ its count copy); refine begin / end
  hipEvent_t side_beg[2], side_end[2], scr_beg[2], scr_end[2], screen_end[2], ref_beg, ref_end;
  for (int b = 0; b < 2; ++b)
    for (hipEvent_t *x : {&side_beg[b], &side_end[b], &scr_beg[b], &scr_end[b], &screen_end[b]}) GMAT_TRY(evs.make(x));
  GMAT_TRY(evs.make(&ref_beg));
  GMAT_TRY(evs.make(&ref_end));
  double t_screen = 0, t_side = 0, ops = 0;
  RefineTally tally;
  int64_t launches_done = 0;
  int64_t pending = 0;  // candidates waiting in the device buffer
  GMAT_HIP(hipMemsetAsync(e->counter.p, 0, 8, sm));
  // pair screen of the candidates [0, ps_done) already queued on S3 beside the screens (chunks of
  // GMAT_PS_CHUNK, default 65,536 candidates); the flush screens the rest and refines the survivors
  int64_t ps_done = 0;
  const int64_t ps_chunk = getenv("GMAT_PS_CHUNK") ? atoll(getenv("GMAT_PS_CHUNK")) : 65536;
  auto flush = [&](int64_t count) -> int {
    const int64_t done = ps_done;
    ps_done = 0;
    return refine_collect(e, c, S3, use_ps, 0, count, done, chi_cut, p_cut, ref_beg, ref_end, &tally);
  };

  // the int8 screen's (row offset, J) tile list of a launch, built when a level >= 1 needs it
  auto ensure_tiles = [&](size_t li) {
    ScanLaunch &ln = plan[li];
    if (!ln.tiles.empty()) return;
    const int Rn = (int)ln.rows.size();
    for (int r0 = 0; r0 < Rn; r0 += BI) {
      const int64_t jb0 = std::max<int64_t>(tri ? ln.rows[r0] + 1 : 0, ln.j_lo) / BJ;
      for (int64_t J = jb0; J * BJ < m; ++J) {
        ln.tiles.push_back(r0);
        ln.tiles.push_back((int)J);
      }
    }
  };
  // kernel arguments of launch li on buffer set b
  auto make_args = [&](size_t li, int b) -> ScreenArgs {
    ScreenArgs sa{};  // value-initialised: unset pointers (lmask, ops, ...) are null
    const ScanLaunch &ln = plan[li];
    const int Rn = (int)ln.rows.size();
    sa.slices = e->slices.as<int8_t>();
    sa.slices_bytes = (int64_t)e->n_slice * n_pad * n_pad;
    sa.panels = e->spanels.as<int8_t>();
    sa.panels_bytes = 2 * m * n_pad;
    sa.left_off = lc == 0 ? 0 : m * n_pad;
    sa.right_off = rc == 0 ? 0 : m * n_pad;
    sa.n_pad = n_pad;
    sa.left = slp;
    sa.right = srp;
    sa.m = m;
    sa.rows = drows[b].as<int64_t>();
    sa.n_rows = Rn;
    sa.tiles = dtiles[b].as<int>();
    sa.tri = tri;
    sa.c13 = e13[b].as<int>();
    sa.c2 = e2[b].as<int>();
    sa.c13_stride = (int64_t)SIDE_P * Rn * m;
    sa.c2_stride = (int64_t)Rn * m;
    sa.sL = L.sL.as<double>();
    sa.sL3 = L.sL3.as<double>();
    sa.sLd = L.sLd.as<double>();
    sa.sR = R.sR.as<double>();
    sa.csum_l = L.csum.as<double>();
    sa.csum_r = R.csum.as<double>();
    sa.csq_l = L.csq.as<double>();
    sa.csq_r = R.csq.as<double>();
    sa.tile_rows = mxr[b].as<int>();
    sa.tile_side = nullptr;
    sa.pf_store = use_lr && S == 0;
    sa.lmask = nullptr;
    sa.pf_stamp = nullptr;
    sa.live_count = live_cnt.p ? live_cnt.as<unsigned long long>() : nullptr;
    sa.pfc = use_pf ? pfc[b].as<int>() : nullptr;
    sa.pfc_stride = (int64_t)Rn * m;
    sa.pf_mu = e->pf_mu;
    sa.pf_eps = e->pf_eps;
    sa.pf_tau = e->pf_tau;
    sa.pf_ncov = e->pf_ncov;
    sa.pf_ku = e->pf_ku;
    for (int k = 0; k < 4; ++k) sa.pf_su[k] = e->pf_su[k];
    for (int k = 0; k < 4; ++k) sa.pf_sq[k] = e->pf_sq[k];
    sa.pf_ua = e->pf_ncov ? L.uc.as<double>() : nullptr;
    sa.pf_ub = e->pf_ncov ? R.uc.as<double>() : nullptr;
    sa.n_id = (double)e->n;
    sa.flags = use_pf ? flags[b].as<uint8_t>() : nullptr;
    sa.nJ = (int)nJ;
    // per element |v - s sum_t 128^-t Q_t| <= s (0.5 * 128^-(T-1) + fp64 rounding)
    sa.side_eps = 0.5 * std::pow(128.0, -(SIDE_T - 1)) + 1e-12;
    sa.e3_t = e3_slices[b];
    sa.e3_eps = 0.5 * std::pow(128.0, -(sa.e3_t - 1)) + 1e-12;
    sa.ld_e = m;
    sa.j_lo = ln.j_lo;
    sa.alpha = L.soff.as<double>();
    sa.qa = L.qa.as<double>();
    sa.ra = L.ra.as<double>();
    sa.sa = L.sa.as<double>();
    sa.beta = R.soff.as<double>();
    sa.qb = R.qb.as<double>();
    sa.rb = R.rb.as<double>();
    sa.sb = R.sb.as<double>();
    sa.mono_l = L.mono.as<uint8_t>();
    sa.mono_r = R.mono.as<uint8_t>();
    sa.zz = e->zz;
    sa.spy = e->spy;
    sa.chi_cut = chi_cut;
    sa.counter = e->counter.as<unsigned long long>();
    sa.cap = e->cand_cap;
    sa.cand_i = e->cand_i.as<int64_t>();
    sa.cand_j = e->cand_j.as<int64_t>();
    sa.n_slice = 0;
    sa.scale_main = 0.0;
    sa.delta = 0.0;
    return sa;
  };
  // side terms of launch `li` into buffer set b (stream s2)
  // pinned host staging: asynchronous copies from / to pageable memory block the host until the
  // stream drains, which would serialise the side passes of launch li+1 behind screen li
  auto &pin_rows = e->pins.rows, &pin_flags = e->pins.flags, &pin_mxt = e->pins.mxt, &pin_mxr = e->pins.mxr;
  auto stage_rows = [&](const ScanLaunch &ln, int b) -> int {
    GMAT_TRY(pin_rows[b].reserve(ln.rows.size() * 8));
    std::memcpy(pin_rows[b].p, ln.rows.data(), ln.rows.size() * 8);
    return GMAT_OK;
  };
  auto enqueue_side = [&](size_t li, int b, bool full) -> int {
    side_full[b] = full;
    e3_slices[b] = (!full && use_pf) ? E3_PF : SIDE_T;
    if (!full && use_pf) {  // fused passes: prefilter flags + E3, then E1 / Ed / E2 for flagged blocks
      const ScanLaunch &ln = plan[li];
      const int Rn = (int)ln.rows.size();
      GMAT_HIP(hipStreamWaitEvent(S2, screen_end[b], 0));  // buffer b free (screen two launches back)
      GMAT_TRY(stage_rows(ln, b));
      GMAT_HIP(hipMemcpyAsync(drows[b].p, pin_rows[b].p, Rn * 8, hipMemcpyHostToDevice, S2));
      GMAT_HIP(hipEventRecord(side_beg[b], S2));
      GMAT_HIP(hipMemsetAsync(flags[b].p, 0, (size_t)Rn * nJ, S2));
      SideArgs x{};
      x.a = make_args(li, b);
      x.n_pad = n_pad;
      x.blocked = 0;
      x.tile_list = nullptr;
      x.n_list = 0;
      x.recL = L.pfRecL.as<float>();
      x.recR = R.pfRecR.as<float>();
      x.n_rt = (int)cdiv(Rn, SG_T);
      const int64_t ss = m * n_pad;
      const int64_t ncols = m - (ln.j_lo / 32) * 32;
      const unsigned grid = (unsigned)(x.n_rt * cdiv(ncols, SG_T));
      for (int t = 0; t < E3_PF; ++t) x.rs[t] = L.L3q.as<int8_t>() + t * ss;
      x.cs[0] = srp;
      x.rs4 = L.p4.as<uint8_t>();
      x.cs4 = R.p4.as<uint8_t>();
      if (e->pf_ncov == 0) {  // prefilter pass (stage-blocked operands)
        SideArgs xp = x;
        xp.blocked = 1;
        for (int t = 0; t < E3_PF; ++t) xp.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;
        xp.rs2 = L.p2b.as<uint8_t>();
        xp.cs2 = R.p2b.as<uint8_t>();
        xp.n_rt = (int)cdiv(Rn, PF_TR);
        const unsigned gp = (unsigned)(xp.n_rt * cdiv(ncols, PF_TC));
        hipLaunchKernelGGL((prefilter_pass_kernel<false, false, false, PF_TR, PF_NS>), dim3(gp), dim3(512), 0, S2, xp);
      } else {  // covariate designs: 64 x 128 tiles with the direction products
        SideArgs xp = x;
        xp.qimg = e->pf_q.as<uint8_t>();
        for (int t = 0; t < E3_PF; ++t) xp.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;  // stage-blocked
        xp.rs2 = L.p2b.as<uint8_t>();
        xp.cs2 = R.p2b.as<uint8_t>();
        xp.n_rt = (int)cdiv(Rn, PC_TR);
        const unsigned gp = (unsigned)(xp.n_rt * cdiv(ncols, PC_TC));
        switch (e->pf_ncov) {
          case 1: hipLaunchKernelGGL((prefilter_cov_kernel<1, false, PC_TC>), dim3(gp), dim3(512), 0, S2, xp); break;
          case 2: hipLaunchKernelGGL((prefilter_cov_kernel<2, false, PC_TC>), dim3(gp), dim3(512), 0, S2, xp); break;
          case 3: hipLaunchKernelGGL((prefilter_cov_kernel<3, false, PC_TC>), dim3(gp), dim3(512), 0, S2, xp); break;
          default: hipLaunchKernelGGL((prefilter_cov_kernel<4, false, PC_TC>), dim3(gp), dim3(512), 0, S2, xp); break;
        }
      }
      GMAT_HIP(hipGetLastError());
      if (x.a.pf_store) {  // the low-rank screen needs nothing else
        const unsigned gj = (unsigned)cdiv(nJ, 64);
        int *info = tl_info.as<int>() + 4 * b;
        hipLaunchKernelGGL(tl_count_kernel, dim3(gj), dim3(1024), 0, S2, flags[b].as<uint8_t>(), Rn, (int)nJ,
                           tl_cnt.as<int>());
        hipLaunchKernelGGL(tl_scan_kernel, dim3(1), dim3(1024), 0, S2, tl_cnt.as<int>(), (int)nJ, tl_h.as<int>(), info,
                           mxt[b].as<int>(), mxr[b].as<int>());
        hipLaunchKernelGGL(tl_fill_kernel, dim3(gj), dim3(1024), 0, S2, flags[b].as<uint8_t>(), Rn, (int)nJ,
                           tl_cnt.as<int>(), tl_h.as<int>(), info, mxt[b].as<int>(), mxr[b].as<int>());
        GMAT_HIP(hipGetLastError());
        GMAT_TRY(pin_flags[b].reserve(16));
        GMAT_HIP(hipMemcpyAsync(pin_flags[b].p, info, 4 * sizeof(int), hipMemcpyDeviceToHost, S2));
        GMAT_HIP(hipEventRecord(side_end[b], S2));
        return GMAT_OK;
      }
      for (int t = 0; t < SIDE_T; ++t) x.rs[t] = L.Lq.as<int8_t>() + t * ss;  // E1
      x.cs[0] = srp;
      hipLaunchKernelGGL(side_gemm_kernel<2>, dim3(grid), dim3(256), 0, S2, x);
      for (int t = 0; t < SIDE_T; ++t) x.rs[t] = L.Ldq.as<int8_t>() + t * ss;  // Ed
      x.cs[0] = srq;
      hipLaunchKernelGGL(side_gemm_kernel<3>, dim3(grid), dim3(256), 0, S2, x);
      x.rs[0] = slp;  // E2
      for (int t = 0; t < SIDE_T; ++t) x.cs[t] = R.Rq.as<int8_t>() + t * ss;
      hipLaunchKernelGGL(side_gemm_kernel<4>, dim3(grid), dim3(256), 0, S2, x);
      GMAT_HIP(hipGetLastError());
      GMAT_TRY(pin_flags[b].reserve((size_t)Rn * nJ));
      GMAT_HIP(hipMemcpyAsync(pin_flags[b].p, flags[b].p, (size_t)Rn * nJ, hipMemcpyDeviceToHost, S2));
      GMAT_HIP(hipEventRecord(side_end[b], S2));
      return GMAT_OK;
    }
    ensure_tiles(li);
    const ScanLaunch &ln = plan[li];
    const int Rn = (int)ln.rows.size();
    GMAT_HIP(hipStreamWaitEvent(S2, screen_end[b], 0));  // buffer b free (screen two launches back)
    GMAT_TRY(stage_rows(ln, b));
    GMAT_HIP(hipMemcpyAsync(drows[b].p, pin_rows[b].p, Rn * 8, hipMemcpyHostToDevice, S2));
    GMAT_HIP(hipMemcpyAsync(dtiles[b].p, ln.tiles.data(), ln.tiles.size() * sizeof(int), hipMemcpyHostToDevice,
                            S2));
    GMAT_HIP(hipEventRecord(side_beg[b], S2));
    const int64_t ss = m * n_pad;  // slice stride of the side vectors
    hipLaunchKernelGGL(gather_band_kernel, dim3(Rn), dim3(256), 0, S2, n_pad, Rn, ss, drows[b].as<int64_t>(),
                       L.Lq.as<int8_t>(), L.L3q.as<int8_t>(), L.Ldq.as<int8_t>(), slp, slq, bl[b].as<int8_t>(),
                       ba[b].as<int8_t>());
    GMAT_HIP(hipGetLastError());
    // int32 slice products (int8 MFMA, exact): C13[t] = [L'q_t; L3q_t]_band . b_j and
    // Ldq_t,band . b_j^2, C2[t] = a_band . R'q_t,j; per group of 64 rows from the group's first
    // needed column (a folded launch's second chunk needs far fewer columns than its first)
    const int64_t z13 = (int64_t)SIDE_P * Rn * m, z2 = (int64_t)Rn * m;
    for (int g0 = 0; g0 < Rn; g0 += 64) {
      const int gn = std::min(64, Rn - g0);
      const int64_t jg = tri ? std::max<int64_t>(ln.j_lo, ln.rows[g0] + 1) : ln.j_lo;
      const int64_t nc = m - jg, coff = jg - ln.j_lo;
      if (nc <= 0) continue;
      for (int part = 0; part < SIDE_P; ++part)  // L' rows, L3 rows (x b), Ld rows (x b^2)
        if (full || part == 1)
          GMAT_TRY(i8gemm_nt(S2, SIDE_T, gn, (int)nc, (int)n_pad, bl[b].as<int8_t>() + (int64_t)(part * Rn + g0) * n_pad,
                             n_pad, (int64_t)SIDE_P * Rn * n_pad, (part == 2 ? srq : srp) + jg * n_pad, n_pad, 0,
                             e13[b].as<int>() + (int64_t)(part * Rn + g0) * m + coff, m, z13));
      if (full)
        GMAT_TRY(i8gemm_nt(S2, SIDE_T, gn, (int)nc, (int)n_pad, ba[b].as<int8_t>() + (int64_t)g0 * n_pad, n_pad, 0,
                           R.Rq.as<int8_t>() + jg * n_pad, n_pad, ss, e2[b].as<int>() + (int64_t)g0 * m + coff, m, z2));
    }
    GMAT_HIP(hipEventRecord(side_end[b], S2));
    return GMAT_OK;
  };
    // MX tiles: per 32-column block J the band rows with work in it (all rows whose block holds
    // a pair j > i; with the prefilter only flagged (row, block) pairs), MX_BI rows per tile,
    // J-major, dealt to the 8 XCDs (workgroup b runs on XCD b mod 8) in contiguous chunks so a
    // J's j-side records are re-read from one L2; padding entries (-1) exit at once
  std::vector<int> mxT[2], mxR[2];
  int64_t nMX[2] = {0, 0}, gT[2] = {0, 0};  // tiles, tile entries (= workgroups, padding included)
  size_t built_for[2] = {SIZE_MAX, SIZE_MAX};
  double t_build = 0.0;  // host seconds spent building MX / low-rank tile lists (diagnostics)
  auto build_mx = [&](size_t li, int b) -> int {
    const double tb0 = now();
    struct Acc {
      double &t;
      double t0;
      ~Acc() { t += now() - t0; }
    } acc_guard{t_build, tb0};
    const ScanLaunch &ln = plan[li];
    const int Rn = (int)ln.rows.size();
    std::vector<int> &mx_tiles = mxT[b], &mx_rows = mxR[b];
    int64_t &n_mx = nMX[b];
    built_for[b] = li;
    if (use_lr) {  // the lists are on the device already: the tile count is all the host needs
      GMAT_HIP(hipEventSynchronize(side_end[b]));
      const int *info = pin_flags[b].as<int>();
      n_mx = info[1];
      gT[b] = info[2];
      return GMAT_OK;
    }
    {
      const uint8_t *fl = nullptr;  // flags of launch li (copied to pinned memory by its side pass)
      if (use_pf) {
        GMAT_HIP(hipEventSynchronize(side_end[b]));
        fl = pin_flags[b].as<uint8_t>();
      }
      // half-tiles: up to MX_BI/2 rows of one column block; consecutive half-tiles pair up
      std::vector<int> lst, rl;  // lst: (row-list index, J0, J1) per tile
      int halves = 0;
      // live rows per column block, bucketed in one row-major sweep of the flags
      std::vector<int> jcnt(nJ + 1, 0), jrow;
      auto live = [&](int r, int64_t J) {
        return use_pf ? fl[(size_t)r * nJ + J] != 0 : (!tri || J * BJ + BJ - 1 > ln.rows[r]);
      };
      // (r, J) with a set flag, in row-major order: the flags are sparse, scan 8 at a time
      std::vector<std::pair<int, int>> set_rj;
      if (use_pf) {
        set_rj.reserve((size_t)Rn * nJ / 8);
        for (int r = 0; r < Rn; ++r) {
          const uint8_t *f = fl + (size_t)r * nJ;
          int64_t J = 0;
          for (; J + 8 <= nJ; J += 8) {
            uint64_t wd;
            std::memcpy(&wd, f + J, 8);
            while (wd) {
              const int bit = __builtin_ctzll(wd);
              set_rj.push_back({r, (int)(J + bit / 8)});
              wd &= ~(0xFFull << (bit & ~7));
            }
          }
          for (; J < nJ; ++J)
            if (f[J]) set_rj.push_back({r, (int)J});
        }
      } else {
        for (int r = 0; r < Rn; ++r)
          for (int64_t J = 0; J < nJ; ++J)
            if (live(r, J)) set_rj.push_back({r, (int)J});
      }
      for (const auto &q : set_rj) ++jcnt[q.second + 1];
      for (int64_t J = 0; J < nJ; ++J) jcnt[J + 1] += jcnt[J];
      jrow.resize(jcnt[nJ]);
      {
        std::vector<int> fill(jcnt.begin(), jcnt.end() - 1);
        for (const auto &q : set_rj) jrow[fill[q.second]++] = q.first;
      }
      for (int64_t J = 0; J < nJ; ++J) {
        int cnt = 0;
        for (int q = jcnt[J]; q < jcnt[J + 1]; ++q) {
          const int r = jrow[q];
          if (cnt % (MX_BI / 2) == 0) {  // open a half-tile
            if (halves % 2 == 0) {
              lst.push_back((int)(rl.size() / MX_BI));
              lst.push_back((int)J);
              lst.push_back(-1);
              rl.insert(rl.end(), MX_BI, -1);
            } else {
              lst.back() = (int)J;
            }
            ++halves;
          }
          rl[rl.size() - MX_BI + ((halves - 1) % 2) * (MX_BI / 2) + cnt % (MX_BI / 2)] = r;
          ++cnt;
        }
      }
      n_mx = (int64_t)lst.size() / MX_TE;
      if (getenv("GMAT_DEBUG") && li < 3) {
        int64_t live = 0;
        for (int64_t q = 0; fl && q < (int64_t)Rn * nJ; ++q) live += fl[q];
        fprintf(stderr, "launch %zu: %lld MX tiles, flagged blocks %lld of %lld\n", li, (long long)n_mx, (long long)live,
                (long long)Rn * nJ);
      }
      const int64_t C = cdiv(n_mx, 8);
      mx_tiles.assign((size_t)MX_TE * 8 * C, -1);
      for (int64_t p = 0; p < n_mx; ++p) {
        const int64_t bb = 8 * (p % C) + p / C;
        for (int k = 0; k < MX_TE; ++k) mx_tiles[MX_TE * bb + k] = lst[MX_TE * p + k];
      }
      mx_rows.swap(rl);
      gT[b] = (int64_t)(mx_tiles.size() / MX_TE);
      if (!mx_tiles.empty()) {  // sm is past screen li-1, the last reader of mxt[b] / mxr[b]
        GMAT_TRY(pin_mxt[b].reserve(mx_tiles.size() * sizeof(int)));
        GMAT_TRY(pin_mxr[b].reserve(mx_rows.size() * sizeof(int)));
        std::memcpy(pin_mxt[b].p, mx_tiles.data(), mx_tiles.size() * sizeof(int));
        std::memcpy(pin_mxr[b].p, mx_rows.data(), mx_rows.size() * sizeof(int));
        GMAT_HIP(hipMemcpyAsync(mxt[b].p, pin_mxt[b].p, mx_tiles.size() * sizeof(int), hipMemcpyHostToDevice, sm));
        GMAT_HIP(hipMemcpyAsync(mxr[b].p, pin_mxr[b].p, mx_rows.size() * sizeof(int), hipMemcpyHostToDevice, sm));
      }
    }
    return GMAT_OK;
  };
  // the first screen launches wait on never-recorded events: record them once up front
  GMAT_HIP(hipEventRecord(screen_end[0], sm));
  GMAT_HIP(hipEventRecord(screen_end[1], sm));
  if (!plan.empty()) GMAT_TRY(enqueue_side(0, 0, S != 0));
  // The next launch's low-rank screen is queued on sm right behind the current one (its side
  // pass and tile list are ready by then), so the host's per-launch bookkeeping no longer leaves
  // the GPU idle; a launch that overflows the candidate buffer discards the queued one.
  const bool pipe_next = use_lr;
  std::vector<char> queued(plan.size(), 0);
  auto &pin_cnt = e->pins.cnt;
  GMAT_TRY(pin_cnt[0].reserve(8));
  GMAT_TRY(pin_cnt[1].reserve(8));
  // 256-deep stages when the K extent allows (an even number of 128-deep MX K blocks), else 128
  const int lr_sk = (e->nK % 2) ? 1 : 2;
  auto launch_lr_kernel = [&](unsigned g, const ScreenArgs &sa_, LrArgs lx_) {
    lx_.n_tiles = (int)g;  // one tile entry per workgroup
    if (lr_sk == 2)
      hipLaunchKernelGGL((lr_screen_kernel<2, 2>), dim3(g), dim3(MxShape<1>::T), 0, sm, sa_, lx_);
    else
      hipLaunchKernelGGL((lr_screen_kernel<1, 2>), dim3(g), dim3(MxShape<1>::T), 0, sm, sa_, lx_);
  };

  auto lr_args = [&](size_t li) {
    LrArgs lx;
    lx.tiles = e->lr_tiles.as<uint8_t>();
    lx.nib_i = L.nibI.as<uint8_t>();
    lx.nib_j = R.nibJ.as<uint8_t>();
    lx.tiles_bytes = (int64_t)e->lr_tiles.bytes;
    lx.nib_bytes = m * n_pad;
    lx.nK = e->nK;
    lx.nC = e->lr_R / MXK;
    lx.R = e->lr_R;
    lx.G = L.lrGa.as<float>();
    lx.H = R.lrG.as<float>();
    lx.E = e->lr_E;
    lx.lam = e->lr_lam;
    lx.tau = e->lr_tau;
    lx.eps = e->lr_eps;
    lx.recL = L.lrRecL.as<double>();
    lx.recR = R.lrRecR.as<double>();
    lx.n_tiles = 0;
    return lx;
  };
  // queue the low-rank screen of launch li (level 0) on sm: waits for its side pass, counts after it
  auto queue_lr = [&](size_t li, int b) -> int {
    ScreenArgs sa = make_args(li, b);
    sa.n_slice = 0;
    sa.delta = e->rho_mx;
    sa.tiles = mxt[b].as<int>();
    const LrArgs lx = lr_args(li);
    GMAT_HIP(hipStreamWaitEvent(sm, side_end[b], 0));
    GMAT_HIP(hipEventRecord(scr_beg[b], sm));
    if (gT[b] > 0) launch_lr_kernel((unsigned)gT[b], sa, lx);
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipEventRecord(scr_end[b], sm));
    GMAT_HIP(hipMemcpyAsync(pin_cnt[b].p, e->counter.p, 8, hipMemcpyDeviceToHost, sm));
    GMAT_HIP(hipEventRecord(screen_end[b], sm));
    return GMAT_OK;
  };
  for (size_t li = 0; li < plan.size(); ++li) {
    const ScanLaunch &ln = plan[li];
    const int b = (int)(li & 1);
    const int Rn = (int)ln.rows.size();
    int64_t ntiles = 0;  // int8 screen workgroups (tile lists are built lazily)
    ScreenArgs sa = make_args(li, b);
    unsigned long long count = 0;
    MxArgs mx;
    mx.tiles = e->mx_tiles.as<uint8_t>();
    mx.nib_i = L.nibI.as<uint8_t>();
    mx.nib_j = R.nibJ.as<uint8_t>();
    mx.tiles_bytes = (int64_t)e->mx_tiles.bytes;
    mx.nib_bytes = m * n_pad;
    mx.nK = e->nK;
    const LrArgs lx = lr_args(li);
    if (S == 0 && built_for[b] != li) GMAT_TRY(build_mx(li, b));
    const std::vector<int> &mx_tiles = mxT[b];
    const int64_t n_mx = nMX[b];
    for (int attempt = 0;; ++attempt) {
      sa.n_slice = S;
      sa.scale_main = e->qmax / 127.0 * std::pow(128.0, -(S - 1));
      if (S > 0) GMAT_TRY(ensure_rho(e, S));
      sa.delta = S == 0 ? e->rho_mx : e->rho[S];
      if (queued[li] && S == 0) {  // queued behind the previous launch
        queued[li] = 0;
      } else {
      queued[li] = 0;
      GMAT_HIP(hipStreamWaitEvent(sm, side_end[b], 0));
      GMAT_HIP(hipEventRecord(scr_beg[b], sm));
      sa.tiles = S == 0 ? mxt[b].as<int>() : dtiles[b].as<int>();
      if (S != 0 && !side_full[b]) {  // escalated from the MX screen: the int8 screen needs E1 / Ed / E2
        GMAT_HIP(hipStreamSynchronize(S2));
        GMAT_TRY(enqueue_side(li, b, true));
        GMAT_HIP(hipStreamSynchronize(S2));
        sa.e3_t = e3_slices[b];
        sa.e3_eps = 0.5 * std::pow(128.0, -(sa.e3_t - 1)) + 1e-12;
      }
      ntiles = (int64_t)plan[li].tiles.size() / 2;
      if (S == 0 && use_lr && gT[b] > 0) {
        launch_lr_kernel((unsigned)gT[b], sa, lx);
      } else if (S == 0 && !mx_tiles.empty()) {
        const unsigned g = (unsigned)(mx_tiles.size() / MX_TE);
        hipLaunchKernelGGL(mx_screen_kernel<1>, dim3(g), dim3(MxShape<1>::T), 0, sm, sa, mx);
      }
      else if (S != 0)
        hipLaunchKernelGGL(screen_kernel<SCREEN_SHAPE>, dim3((unsigned)ntiles), dim3(256), 0, sm, sa);
      GMAT_HIP(hipGetLastError());
      GMAT_HIP(hipEventRecord(scr_end[b], sm));
      GMAT_HIP(hipMemcpyAsync(pin_cnt[b].p, e->counter.p, 8, hipMemcpyDeviceToHost, sm));
      GMAT_HIP(hipEventRecord(screen_end[b], sm));
      }
      // next launch's side terms overlap this screen; its tile list is built on the host
      // meanwhile, and its low-rank screen queued behind this one
      if (attempt == 0 && li + 1 < plan.size() && !queued[li + 1]) {
        GMAT_TRY(enqueue_side(li + 1, b ^ 1, S != 0));
        if (S == 0) GMAT_TRY(build_mx(li + 1, b ^ 1));
        if (S == 0 && pipe_next) {
          GMAT_TRY(queue_lr(li + 1, b ^ 1));
          queued[li + 1] = 1;
        }
      }
      GMAT_HIP(hipEventSynchronize(screen_end[b]));
      count = *pin_cnt[b].as<unsigned long long>();
      if ((int64_t)count <= e->cand_cap) break;
      // overflow in this launch: refine what earlier launches left and redo this one; if it
      // overflowed on its own, redo it with one more slice (thinner candidate band).  A queued
      // next launch appended behind the overflow: drain it and run it again later.
      GMAT_HIP(hipStreamSynchronize(sm));
      if (li + 1 < plan.size()) queued[li + 1] = 0;
      if (pending == 0) {
        if (S < e->n_slice) {  // thinner candidate band first
          S = S == 0 ? std::min(2, e->n_slice) : S + 1;
          S_max_used = std::max(S_max_used, S);
        } else {  // the finest screen still overflows on one launch (large p_cut): grow the buffer
          GMAT_TRY(grow_candidates(e, std::max<int64_t>(2 * e->cand_cap, (int64_t)(1.25 * (double)count) + 1024), use_ps));
          sa.cap = e->cand_cap;
          sa.cand_i = e->cand_i.as<int64_t>();
          sa.cand_j = e->cand_j.as<int64_t>();
        }
      }
      GMAT_TRY(flush(pending));
      pending = 0;
      GMAT_HIP(hipMemsetAsync(e->counter.p, 0, 8, sm));
    }
    pending = (int64_t)count;
    if (use_ps && ps_chunk > 0 && pending - ps_done >= ps_chunk) {
      // the screen of this launch has finished (its count was read): screen its candidates now
      GMAT_TRY(pair_screen(e, S3, L, R, slp, srp, e->cand_i.as<int64_t>() + ps_done, e->cand_j.as<int64_t>() + ps_done,
                           pending - ps_done, chi_cut, nullptr, ps_done == 0));
      ps_done = pending;
    }
    float ms_side, ms_screen;
    GMAT_HIP(hipEventSynchronize(side_end[b]));
    GMAT_HIP(hipEventElapsedTime(&ms_side, side_beg[b], side_end[b]));
    GMAT_HIP(hipEventElapsedTime(&ms_screen, scr_beg[b], scr_end[b]));
    t_side += ms_side * 1e-3;
    t_screen += ms_screen * 1e-3;
    // int8 MFMA ops issued: per tile and slice, sum over K-blocks of (n_pad - K) x MT MACs per
    // pair = n_pad (n_pad + MT) / 2, x (BI x BJ) pairs x 2
    if (S == 0 && use_lr)
      ops += (double)n_mx * 2.0 * (double)e->lr_R * (double)n_pad * MX_BI * BJ;  // incl. empty slots
    else if (S == 0)
      ops += (double)n_mx * (double)n_pad * (double)(n_pad + MXK) * MX_BI * BJ;  // incl. empty slots
    else
      ops += (double)ntiles * S * (double)n_pad * (double)(n_pad + MT) * BI * BJ;
    ++launches_done;
    if (pending > e->cand_cap / 2) {
      GMAT_HIP(hipStreamSynchronize(sm));  // a queued next launch is discarded: the counter restarts
      if (li + 1 < plan.size()) queued[li + 1] = 0;
      GMAT_TRY(flush(pending));
      pending = 0;
      GMAT_HIP(hipMemsetAsync(e->counter.p, 0, 8, sm));
    }
  }
  GMAT_HIP(hipStreamSynchronize(S2));
  GMAT_TRY(flush(pending));
  *n_hits = sort_hits(e);
  e->stats[0] = pairs_tested;
  e->stats[1] = tally.n_cand;
  e->stats[2] = ops;
  e->stats[3] = t_screen;
  e->stats[4] = tally.t_ref;
  e->stats[5] = t_side;
  e->stats[6] = now() - t_start;
  e->stats[7] = (double)launches_done;
  if (getenv("GMAT_DEBUG"))
    fprintf(stderr, "gmat_epi_scan: %lld launches, tile-list building %.3f s on the host, total %.3f s, %.0f screen "
            "candidates, %.0f refined%s\n", (long long)launches_done, t_build, e->stats[6], tally.n_cand,
            tally.n_refined, use_ps ? " (pair screen)" : "");
  if (live_cnt.p) {
    unsigned long long lcnt = 0;
    GMAT_HIP(hipMemcpy(&lcnt, live_cnt.p, 8, hipMemcpyDeviceToHost));
    fprintf(stderr, "gmat_epi_scan: %.0f pairs, prefilter keeps %llu pairs (%.4f%%), %.0f low-rank candidates\n",
            pairs_tested, lcnt, 100.0 * (double)lcnt / std::max(pairs_tested, 1.0), tally.n_cand);
  }
  const bool lr_only = use_lr && S_max_used == 0;
  e->stats[8] = lr_only ? -1 : S_max_used;
  e->stats[9] = lr_only ? e->lr_lam : (S_max_used == 0 ? e->rho_mx : e->rho[S_max_used]);
  return GMAT_OK;
}

}  // namespace epi
}  // namespace gmat

int gmat::epi::scan_dispatch(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut,
                             int n_slice, int64_t *n_hits) {
  GMAT_CHECK(!e->seg, GMAT_E_ARG, "scan_dispatch: a segmented plan (seg_scan runs its sub-plans)");
  // no screen asked for, or none available (a plan past EXH_ONLY_NPAD individuals): every pair refined
  if (n_slice == GMAT_SCREEN_NONE || e->exh_only) return scan_exhaustive(e, kind, rows, n_rows, p_cut, n_hits);
  // the compacted low-rank scan serves the low-rank level (automatic at p_cut <= 1e-4, or forced by
  // n_slice -2); GMAT_LR_BLOCKS=1 keeps the block-granular path below (A/B runs)
  const bool lr_level = e->lr_R > 0 && e->pf_mu > 0.0 && (n_slice == -2 || (n_slice == 0 && p_cut <= 1e-4));
  if (lr_level && pair_screen_fits(e) && !getenv("GMAT_LR_BLOCKS") && !getenv("GMAT_NO_PREFILTER"))
    return scan_lowrank(e, kind, rows, n_rows, p_cut, chi_cut, n_hits);
  return scan_blocks(e, kind, rows, n_rows, p_cut, chi_cut, n_slice, n_hits);
}

extern "C" int gmat_epi_scan(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut,
                             int n_slice, int64_t *n_hits) {
  GMAT_CHECK(e && rows && n_hits, GMAT_E_ARG, "gmat_epi_scan: bad arguments");
  GMAT_CHECK(kind >= 0 && kind <= 2, GMAT_E_ARG, "gmat_epi_scan: bad kind");
  const int64_t m = e->m;
  for (int64_t t = 0; t < n_rows; ++t) {
    GMAT_CHECK(rows[t] >= 0 && rows[t] < m, GMAT_E_ARG, "row %lld out of range", (long long)rows[t]);
    GMAT_CHECK(t == 0 || rows[t] > rows[t - 1], GMAT_E_ARG, "rows must be strictly increasing");
  }
  if (e->seg) return seg_scan(e, kind, rows, n_rows, p_cut, chi_cut, n_slice, n_hits);
  return scan_dispatch(e, kind, rows, n_rows, p_cut, chi_cut, n_slice, n_hits);
}

extern "C" int gmat_epi_hits(gmat_epi *e, int64_t cap, int64_t *i, int64_t *j, double *eff, double *var, double *chi,
                             double *p) {
  GMAT_CHECK(e, GMAT_E_ARG, "gmat_epi_hits: null handle");
  const int64_t n = (int64_t)e->hit_i.size();
  GMAT_CHECK(cap >= n, GMAT_E_OVERFLOW, "gmat_epi_hits: capacity %lld < %lld hits", (long long)cap, (long long)n);
  for (int64_t k = 0; k < n; ++k) {
    if (i) i[k] = e->hit_i[k];
    if (j) j[k] = e->hit_j[k];
    if (eff) eff[k] = e->hit_eff[k];
    if (var) var[k] = e->hit_var[k];
    if (chi) chi[k] = e->hit_chi[k];
    if (p) p[k] = e->hit_p[k];
  }
  return GMAT_OK;
}

extern "C" int gmat_epi_kernel_stats(const gmat_epi *e, double *out8) {
  GMAT_CHECK(e && out8, GMAT_E_ARG, "gmat_epi_kernel_stats: bad arguments");
  for (int k = 0; k < 8; ++k) out8[k] = e->kstats[k];
  return GMAT_OK;
}

extern "C" int gmat_epi_kernel_stats_ext(const gmat_epi *e, double *out, int cap, int *count) {
  GMAT_CHECK(e && out && count && cap >= 0, GMAT_E_ARG, "gmat_epi_kernel_stats_ext: bad arguments");
  double v[3 * KT_N] = {0};
  for (size_t k = 0; k + 1 < e->kmarks.size(); k += 2) {
    const auto &b = e->kmarks[k], &en = e->kmarks[k + 1];
    float ms = 0.f;
    GMAT_HIP(hipEventSynchronize(e->kev[en.ev]));
    GMAT_HIP(hipEventElapsedTime(&ms, e->kev[b.ev], e->kev[en.ev]));
    v[3 * b.kernel] += ms * 1e-3;
    v[3 * b.kernel + 1] += 1.0;
    v[3 * b.kernel + 2] += b.pairs;
  }
  *count = 3 * KT_N;
  for (int k = 0; k < std::min(cap, 3 * KT_N); ++k) out[k] = v[k];
  return GMAT_OK;
}

extern "C" int gmat_epi_stats(const gmat_epi *e, double *out10) {
  GMAT_CHECK(e && out10, GMAT_E_ARG, "gmat_epi_stats: bad arguments");
  for (int k = 0; k < 10; ++k) out10[k] = e->stats[k];
  return GMAT_OK;
}


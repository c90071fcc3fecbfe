// The scan plan: codings, certificates and spectral state, the refine / pair-screen drivers, pairs and audit (see epi.h).
#include "epi.h"

namespace gmat {
namespace epi {

// screen panel of a coding (inside e->spanels) and its squared codes (B operand of the Ld term)
const int8_t *screen_panel(const gmat_epi *e, int which) { return e->spanels.as<int8_t>() + which * e->m * e->n_pad; }

// kernel timers: kt_begin records the start event of a launch on st, kt_end its end event
int kt_event(gmat_epi *e, hipStream_t st, size_t *idx) {
  if (e->kev_used == e->kev.size()) {
    hipEvent_t ev;
    GMAT_HIP(hipEventCreate(&ev));
    e->kev.push_back(ev);
  }
  *idx = e->kev_used++;
  GMAT_HIP(hipEventRecord(e->kev[*idx], st));
  return GMAT_OK;
}
int kt_begin(gmat_epi *e, hipStream_t st, size_t *idx) { return kt_event(e, st, idx); }
int kt_end(gmat_epi *e, hipStream_t st, int kernel, size_t beg, double pairs) {
  size_t end;
  GMAT_TRY(kt_event(e, st, &end));
  e->kmarks.push_back({kernel, beg, pairs});  // marks come in (start, end) pairs
  e->kmarks.push_back({-1, end, 0.0});
  return GMAT_OK;
}
const int8_t *screen_sq(const gmat_epi *e, int which) {
  return which == 0 ? e->code[0].sq.as<int8_t>() : screen_panel(e, 1);  // 0/1 codes: a^2 = a
}

int build_coding_impl(gmat_epi *e, int which);
int build_coding(gmat_epi *e, int which) {
  if (e->code[which].ready) return GMAT_OK;
  const double t0 = now();
  const int rc = build_coding_impl(e, which);
  e->setup[5] += now() - t0;
  return rc;
}
int build_coding_impl(gmat_epi *e, int which) {
  Coding &cd = e->code[which];
  const int64_t m = e->m, n_pad = e->n_pad, n = e->n;
  // centring offsets exactly as the reference (for the refine): freq = sum/(2n); A: 2*freq,
  // D: 2*freq*(1-freq).  Screen codes: the additive coding counts the minor allele
  // (a~ = 2 - a, offset 2(1 - freq), when freq > 1/2); the heterozygote coding is unchanged.
  std::vector<double> off(m), soff(m), csum(m), csq(m);
  std::vector<uint8_t> mono(m), flip(m);
  for (int64_t j = 0; j < m; ++j) {
    const int64_t sd = e->g->sum_dose[j], nh = e->g->n_het[j], n2 = (sd - nh) / 2, n0 = n - nh - n2;
    const double freq = (double)sd / (2.0 * (double)n);
    off[j] = which == 0 ? 2.0 * freq : 2.0 * freq * (1.0 - freq);
    mono[j] = which == 0 ? (sd == 0 || sd == 2 * n || nh == n) : (sd == 0 || sd == 2 * n);
    if (which == 0) {
      flip[j] = sd > n;
      soff[j] = flip[j] ? 2.0 * ((double)(2 * n - sd) / (2.0 * (double)n)) : off[j];
      csum[j] = (double)(flip[j] ? 2 * n - sd : sd);
      csq[j] = (double)(nh + 4 * (flip[j] ? n0 : n2));
    } else {
      soff[j] = off[j];
      csum[j] = csq[j] = (double)nh;
    }
  }
  int8_t *panel = e->spanels.as<int8_t>() + which * m * n_pad;
  if (which == 0) {
    DBuf dflip;
    GMAT_TRY(dflip.alloc(m));
    GMAT_TRY(cd.sq.alloc((size_t)m * n_pad));
    GMAT_HIP(hipMemcpy(dflip.p, flip.data(), m, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(flip_panel_kernel, dim3((unsigned)cdiv(m * n_pad, 256)), dim3(256), 0, e->s, n, n_pad, m,
                       e->g->dose_ptr(), dflip.as<uint8_t>(), panel, cd.sq.as<int8_t>());
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipStreamSynchronize(e->s));
  } else {
    GMAT_HIP(hipMemcpyAsync(panel, e->g->het_ptr(), (size_t)m * n_pad, hipMemcpyDeviceToDevice, e->s));
  }
  const size_t vb = (size_t)m * n_pad * sizeof(double);
  DBuf L3;  // fp64 side vector L3 = a o Py, sliced to int8 below (L', Ld, R' of the block-granular
            // screens: block_sides, when a scan first needs them)
  GMAT_TRY(cd.U.alloc(vb));
  GMAT_TRY(L3.alloc(vb));
  for (DBuf *b : {&cd.off, &cd.soff, &cd.qa, &cd.ra, &cd.sa, &cd.qb, &cd.rb, &cd.sb, &cd.sL, &cd.sL3, &cd.sLd, &cd.sR,
                  &cd.csum, &cd.csq})
    GMAT_TRY(b->alloc(m * sizeof(double)));
  if (!e->exh_only) GMAT_TRY(cd.L3q.alloc((size_t)SIDE_T * m * n_pad));
  GMAT_HIP(hipMemcpy(cd.csum.p, csum.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(cd.csq.p, csq.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_TRY(cd.mono.alloc(m));
  GMAT_HIP(hipMemcpy(cd.off.p, off.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(cd.soff.p, soff.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(cd.mono.p, mono.data(), m, hipMemcpyHostToDevice));
  // the 2-bit stage-blocked codes (the prefilter's operand; also the int8 U GEMM's)
  GMAT_TRY(cd.p2b.alloc((size_t)m * n_pad / 4));
  hipLaunchKernelGGL(code2_panel_kernel, dim3((unsigned)cdiv(m * (n_pad / 16), 256)), dim3(256), 0, e->s, m, n_pad, panel,
                     cd.p2b.as<uint32_t>());
  GMAT_HIP(hipGetLastError());
  // U[j][q] = sum_q' panel[j][q'] P[q'][q]: on int8 slices of P (u8_gemm_kernel), or as an fp64 GEMM
  // (GMAT_U_DGEMM, A/B and checks)
  if (!getenv("GMAT_U_DGEMM") && n_pad % SG_K == 0) {
    if (!e->u8_slices.p) {
      GMAT_TRY(e->u8_unit.alloc((size_t)n_pad * sizeof(double)));
      GMAT_TRY(e->u8_slices.alloc((size_t)U8_S * n_pad * n_pad));
      hipLaunchKernelGGL(u8_unit_kernel, dim3((unsigned)n_pad), dim3(256), 0, e->s, n_pad, e->Ps.as<double>(),
                         e->u8_unit.as<double>());
      hipLaunchKernelGGL(u8_slice_kernel, dim3((unsigned)cdiv(n_pad * n_pad, 256)), dim3(256), 0, e->s, n_pad,
                         e->Ps.as<double>(), e->u8_unit.as<double>(), e->u8_slices.as<int8_t>());
      GMAT_HIP(hipGetLastError());
    }
    hipLaunchKernelGGL(u8_gemm_kernel, dim3((unsigned)cdiv(m, U8_J), (unsigned)(n_pad / U8_Q)), dim3(512), 0, e->s, m, n_pad,
                       cd.p2b.as<uint8_t>(), e->u8_slices.as<int8_t>(), e->u8_unit.as<double>(), cd.U.as<double>());
    GMAT_HIP(hipGetLastError());
  } else {
    GMAT_TRY(dgemm_i8a(e->s, m, n_pad, n_pad, 1.0, I8View{panel, n_pad, 0}, DView{e->Ps.as<double>(), n_pad, 0}, 0.0,
                       cd.U.as<double>(), n_pad));
  }
  hipLaunchKernelGGL(left_side_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, panel, cd.U.as<double>(),
                     e->z.as<double>(), e->py.as<double>(), e->dg.as<double>(), cd.soff.as<double>(), nullptr,
                     L3.as<double>(), nullptr, cd.qa.as<double>(), cd.ra.as<double>(), cd.sa.as<double>());
  GMAT_HIP(hipGetLastError());
  hipLaunchKernelGGL(right_side_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, panel, cd.U.as<double>(),
                     e->z.as<double>(), e->py.as<double>(), cd.soff.as<double>(), nullptr, cd.qb.as<double>(),
                     cd.rb.as<double>(), cd.sb.as<double>());
  GMAT_HIP(hipGetLastError());
  if (e->exh_only) {  // the exact refine's operands only (U, the offsets and per-SNP scalars above)
    GMAT_HIP(hipStreamSynchronize(e->s));
    cd.ready = true;
    return GMAT_OK;
  }
  const int64_t ss = m * n_pad;
  hipLaunchKernelGGL(quantize_rows_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, ss, L3.as<double>(),
                     cd.L3q.as<int8_t>(), cd.sL3.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(cd.p4.alloc((size_t)m * n_pad / 2));
  hipLaunchKernelGGL(fp4_panel_kernel, dim3((unsigned)cdiv(m * (n_pad / 2), 256)), dim3(256), 0, e->s, m, n_pad, panel,
                     cd.p4.as<uint8_t>());
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(cd.L3b.alloc((size_t)E3_PF * m * n_pad));
  for (int t = 0; t < E3_PF; ++t)
    hipLaunchKernelGGL(block_panel_perm8_kernel, dim3((unsigned)cdiv(m * (n_pad / 16), 256)), dim3(256), 0, e->s, m,
                       n_pad, (int64_t)SG_K, (const uint8_t *)cd.L3q.as<int8_t>() + (int64_t)t * m * n_pad,
                       cd.L3b.as<uint8_t>() + (int64_t)t * m * n_pad);
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(cd.pfRecL.alloc((size_t)m * PF_REC * sizeof(float)));
  GMAT_TRY(cd.pfRecR.alloc((size_t)m * PF_REC * sizeof(float)));
  hipLaunchKernelGGL(pf_rec_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, e->s, m, (double)n, e->spy,
                     cd.soff.as<double>(), cd.csum.as<double>(), cd.csq.as<double>(), cd.sL3.as<double>(),
                     cd.sa.as<double>(), cd.sb.as<double>(), cd.mono.as<uint8_t>(), cd.pfRecL.as<float>(),
                     cd.pfRecR.as<float>());
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(cd.nibI.alloc((size_t)m * n_pad));
  GMAT_TRY(cd.nibJ.alloc((size_t)m * n_pad));
  hipLaunchKernelGGL(nibble_kernel, dim3((unsigned)cdiv(m * (n_pad / 8), 256)), dim3(256), 0, e->s, m, n_pad, e->nK,
                     panel, cd.nibI.as<uint32_t>(), cd.nibJ.as<uint32_t>());
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(cd.s1c2.alloc((size_t)m * n_pad / 4));
  hipLaunchKernelGGL(s1_code2_kernel, dim3((unsigned)cdiv(m * (n_pad / 16), 256)), dim3(256), 0, e->s, m, n_pad, e->nK,
                     panel, cd.s1c2.as<uint32_t>());
  GMAT_HIP(hipGetLastError());
  if (e->pf_ncov > 0) {  // covariate directions: u_k . code per SNP (the prefilter forms the images on chip)
    const int K0 = e->pf_ncov;
    GMAT_TRY(cd.uc.alloc((size_t)K0 * m * sizeof(double)));
    for (int k = 0; k < K0; ++k)
      hipLaunchKernelGGL(cov_dot_kernel, dim3((unsigned)m), dim3(256), 0, e->s, n_pad, panel,
                         e->pf_U.as<double>() + k * n_pad, cd.uc.as<double>() + k * m);
    GMAT_HIP(hipGetLastError());
  }
  if (e->lr_R) {  // G = screen codes x B (exact in fp64: fp6 x small integers), kept in fp32
    DBuf g64;
    const int64_t Rp = e->lr_R;
    GMAT_TRY(g64.alloc((size_t)m * Rp * sizeof(double)));
    GMAT_TRY(cd.lrG.alloc((size_t)m * Rp * sizeof(float)));
    GMAT_TRY(dgemm_i8a(e->s, m, Rp, n_pad, 1.0, I8View{panel, n_pad, 0}, DView{e->lr_Bs.as<double>(), Rp, 0}, 0.0,
                       g64.as<double>(), Rp));
    hipLaunchKernelGGL(f64_to_f32_kernel, dim3((unsigned)cdiv(m * Rp, 256)), dim3(256), 0, e->s, m * Rp,
                       g64.as<double>(), cd.lrG.as<float>());
    GMAT_TRY(cd.lrGa.alloc((size_t)m * Rp * sizeof(float)));
    hipLaunchKernelGGL(lr_adjust_kernel, dim3((unsigned)cdiv(m * Rp, 256)), dim3(256), 0, e->s, m, Rp, g64.as<double>(),
                       cd.soff.as<double>(), e->lr_q1.as<double>(), cd.lrGa.as<float>());
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(cd.lrRecL.alloc((size_t)m * LR_REC * sizeof(double)));
    GMAT_TRY(cd.lrRecR.alloc((size_t)m * LR_REC * sizeof(double)));
    hipLaunchKernelGGL(lr_rec_kernel, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, e->s, m, cd.soff.as<double>(),
                       cd.csum.as<double>(), cd.csq.as<double>(), cd.sL3.as<double>(), cd.sa.as<double>(),
                       cd.sb.as<double>(), cd.mono.as<uint8_t>(), cd.lrRecL.as<double>(), cd.lrRecR.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipStreamSynchronize(e->s));
  }
  GMAT_TRY(cd.U16.alloc((size_t)m * n_pad * sizeof(_Float16)));
  hipLaunchKernelGGL(f64_to_f16_kernel, dim3((unsigned)cdiv(m * n_pad, 256)), dim3(256), 0, e->s, m * n_pad,
                     cd.U.as<double>(), cd.U16.as<_Float16>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipStreamSynchronize(e->s));
  // (U = P x codes stays in fp64: the int8 refine's O(n) terms, refine8_side_kernel)
  cd.ready = true;
  return GMAT_OK;
}

// the int8 refine serves plans with n_pad <= 64 R8_NC (w in registers) and a nonzero P_off;
// GMAT_REFINE64 selects the fp64 MFMA refine (refine_kernel) for A/B runs
// (n_pad > 64 R8_NC: refine8w_kernel, by squares of stages)
bool refine8_fits(const gmat_epi *e) { return e->n_pad % 64 == 0 && e->qmax > 0 && !getenv("GMAT_REFINE64"); }
int refine8_setup(gmat_epi *e) {
  if (e->r8_tiles.p) return GMAT_OK;
  const int64_t n_pad = e->n_pad, NS = n_pad / 64, N = r8_toff(n_pad / 32, NS);
  GMAT_TRY(e->r8_tiles.alloc((size_t)N * R8_TILE));
  e->r8_unit = 2.0 * e->qmax / 127.0;
  hipLaunchKernelGGL(r8_image_kernel, dim3((unsigned)cdiv(n_pad * n_pad, 256)), dim3(256), 0, e->s, n_pad,
                     e->Ps.as<double>(), 1.0 / e->r8_unit, e->r8_tiles.as<int8_t>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipStreamSynchronize(e->s));
  return GMAT_OK;
}

// exact statistics for device pair lists (pi, pj) of length np -> device eff/var/chi/p
int refine(gmat_epi *e, hipStream_t st, const Coding &L, const Coding &R, const int8_t *lp, const int8_t *rp,
           const int64_t *pi, const int64_t *pj, int64_t np, double *eff, double *var, double *chi, double *p) {
  if (np <= 0) return GMAT_OK;
  if (refine8_fits(e) && L.U.p && R.U.p) {
    GMAT_TRY(refine8_setup(e));
    // segments: short lists spread over more workgroups (one workgroup per CU holds its LDS ring)
    if (!e->n_cu) {
      int dev = 0, cus = 0;
      GMAT_HIP(hipGetDevice(&dev));
      GMAT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      e->n_cu = std::max(cus, 8);
    }
    const bool wide = e->n_pad > 64 * R8_NC;  // w by squares of stages (refine8w_kernel)
    const int64_t wgs = cdiv(np, wide ? R8_PP : R8_PP2);
    const int nQ = (int)cdiv(e->n_pad / 64, R8_NC);
    const int nseg = wide ? nQ * (nQ + 1) / 2 : (int)std::max<int64_t>(1, std::min<int64_t>(seg_max(), e->n_cu / wgs));
    const size_t need = (size_t)np * sizeof(double) * (nseg > 1 ? 1 + R8_S * nseg : 1);
    if (e->r8_varw.bytes < need) {
      GMAT_HIP(hipStreamSynchronize(st));  // an earlier refine queued on st may still use the old buffer
      GMAT_TRY(e->r8_varw.alloc(std::max(need, (size_t)np * sizeof(double) * (1 + R8_S * 8))));
    }
    double *tpart = e->r8_varw.as<double>() + np;
    const int li = (int)(&L - e->code), ri = (int)(&R - e->code);
    const int8_t *sl = screen_panel(e, li), *sr = screen_panel(e, ri);
    // the O(n) terms on a second stream beside refine8_kernel (round 5: 0.27 ms less at the end of a
    // configs[2] step, where refine8_side_kernel ran alone after it), joined before refine8_fin_kernel
    if (e->r8_terms.bytes < (size_t)R8_NT * np * sizeof(double)) {
      GMAT_HIP(hipStreamSynchronize(st));
      if (e->s5) GMAT_HIP(hipStreamSynchronize(e->s5));
      GMAT_TRY(e->r8_terms.alloc((size_t)R8_NT * std::max<int64_t>(np, 1 << 16) * sizeof(double)));
    }
    if (!e->s5) GMAT_TRY(pipeline_stream(4, &e->s5));
    for (auto &ev : e->r8ev)
      if (!ev) GMAT_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const hipStream_t s5 = e->s5;
    GMAT_HIP(hipEventRecord(e->r8ev[0], st));  // the pair list is ready
    GMAT_HIP(hipStreamWaitEvent(s5, e->r8ev[0], 0));
    size_t kt0;
    GMAT_TRY(kt_begin(e, s5, &kt0));
    hipLaunchKernelGGL(refine8_side_kernel, dim3((unsigned)cdiv(np, 4)), dim3(256), 0, s5, e->n_pad, sl, sr,
                       L.U.as<double>(), R.U.as<double>(), e->z.as<double>(), e->dg.as<double>(), e->py.as<double>(), lp,
                       rp, L.soff.as<double>(), R.soff.as<double>(), L.off.as<double>(), R.off.as<double>(),
                       L.qa.as<double>(), L.ra.as<double>(), R.qb.as<double>(), R.rb.as<double>(), e->zz, pi, pj, np,
                       e->r8_terms.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(kt_end(e, s5, KT_REFINE_SIDE, kt0, (double)np));
    GMAT_HIP(hipEventRecord(e->r8ev[1], s5));
    GMAT_TRY(kt_begin(e, st, &kt0));
    if (wide)
      hipLaunchKernelGGL(refine8w_kernel, dim3((unsigned)wgs, (unsigned)nseg), dim3(512), 0, st, e->n_pad,
                         e->r8_tiles.as<int8_t>(), sl, sr, pi, pj, np, tpart);
    else
      hipLaunchKernelGGL(refine8_kernel, dim3((unsigned)wgs, (unsigned)nseg), dim3(512), 0, st, e->n_pad,
                         e->r8_tiles.as<int8_t>(), sl, sr, pi, pj, np, e->r8_unit, e->r8_varw.as<double>(), tpart);
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(kt_end(e, st, KT_REFINE, kt0, (double)np));
    // the segments' combination, the O(n) terms and the p-values in one launch
    GMAT_HIP(hipStreamWaitEvent(st, e->r8ev[1], 0));
    hipLaunchKernelGGL(refine8_fin_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, np, e->r8_terms.as<double>(),
                       L.soff.as<double>(), R.soff.as<double>(), L.qa.as<double>(), L.ra.as<double>(),
                       R.qb.as<double>(), R.rb.as<double>(), e->zz, L.mono.as<uint8_t>(), R.mono.as<uint8_t>(), pi, pj,
                       e->r8_varw.as<double>(), nseg, tpart, e->r8_unit, eff, var, chi, p);
    GMAT_HIP(hipGetLastError());
    return GMAT_OK;
  }
  // a fixed number of segments per pair tile (not one chosen from np: a pair's numbers must not
  // depend on the length of the list it came in, scan vs pairs); 4 segments fill >= 90 % of the
  // last round of resident workgroups (two per CU) from about 1,000 tiles up
  const int64_t tiles = cdiv(np, RP);
  const int nseg = RF_SEG;
  if (nseg > 1 && e->rf_part.bytes < (size_t)2 * nseg * np * sizeof(double)) {
    GMAT_HIP(hipStreamSynchronize(st));  // an earlier refine queued on st may still use the old buffer
    GMAT_TRY(e->rf_part.alloc((size_t)2 * nseg * np * sizeof(double)));
  }
  double *epart = nseg > 1 ? e->rf_part.as<double>() : nullptr, *vpart = nseg > 1 ? epart + nseg * np : nullptr;
  hipLaunchKernelGGL(refine_kernel, dim3((unsigned)tiles, (unsigned)nseg), dim3(RT), 0, st, e->n_pad, e->Ps.as<double>(),
                     e->py.as<double>(), lp, rp, L.off.as<double>(), R.off.as<double>(), pi, pj, np, eff, var, epart,
                     vpart);
  GMAT_HIP(hipGetLastError());
  if (nseg > 1) {
    hipLaunchKernelGGL(refine_sum_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, np, nseg, epart, vpart, eff,
                       var);
    GMAT_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(pvalue_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, np, eff, var, chi, p);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

// pair screen of np candidates (pi, pj) on stream st: the survivors go to e->cand2_i / cand2_j,
// their number to *n_out (the stream is synchronised).  Needs the w planes of a workgroup's pairs
// in LDS: nK <= 63 (n_pad <= 8064); the caller checks pair_screen_fits.
bool pair_screen_fits(const gmat_epi *e) { return e->nK <= 63; }
// Rank of the low-rank screen: with the pair screen behind it a looser, cheaper bound pays (one
// 128-deep basis chunk: 4.5x the candidates of rank 384, 0.55x the screen time at the bench
// configuration); without it the refine of those candidates would dominate.
int default_lr_rank(const gmat_epi *e) { return pair_screen_fits(e) && !getenv("GMAT_NO_PAIR_SCREEN") ? 128 : 384; }
// Survivors are appended to cand2 at counter2: `reset` zeroes the counter first, `n_out` (when given)
// receives its value after a stream synchronisation; without it the call only enqueues (the scan
// screens candidate ranges in chunks beside the later launches and reads the total at flush time).
int pair_screen(gmat_epi *e, hipStream_t st, const Coding &L, const Coding &R, const int8_t *slp, const int8_t *srp,
                const int64_t *pi, const int64_t *pj, int64_t np, double chi_cut, int64_t *n_out, bool reset) {
  if (n_out) *n_out = 0;
  if (np <= 0 && !n_out) return GMAT_OK;
  if (np <= 0 && reset) return GMAT_OK;
  const int nK = e->nK;
  GMAT_CHECK(nK <= 63, GMAT_E_ARG, "pair screen: %d stages (at most 63: pair_mxw_kernel's squares)", nK);
  GMAT_CHECK(L.U16.p && R.U16.p && L.nibI.p && R.nibJ.p && e->mx_tiles.p && e->z.p && e->dg.p && e->py.p && L.qa.p &&
                 R.qb.p && e->cand2_i.p && e->cand2_j.p && e->counter2.p &&
                 e->cand2_i.bytes >= (size_t)np * 8 && L.U16.bytes >= (size_t)e->m * e->n_pad * 2 &&
                 R.U16.bytes >= (size_t)e->m * e->n_pad * 2 && e->mx_tiles.bytes >= (size_t)nK * nK * MX_TILE,
             GMAT_E_ARG, "pair screen: plan buffers missing (U16 %d %d nib %d %d mx %zu z %d cand2 %zu / %lld counter2 %d)",
             L.U16.p != nullptr, R.U16.p != nullptr, L.nibI.p != nullptr, R.nibJ.p != nullptr, e->mx_tiles.bytes,
             e->z.p != nullptr, e->cand2_i.bytes, (long long)np, e->counter2.p != nullptr);
  // the side-term buffer is sized for the largest call once (calls queued on one stream share it)
  if (e->ps_side.bytes < (size_t)5 * np * sizeof(double)) {
    GMAT_HIP(hipStreamSynchronize(st));
    GMAT_TRY(e->ps_side.alloc((size_t)5 * std::max<int64_t>(np, e->cand_cap) * sizeof(double)));
  }
  GMAT_TRY(e->pins.count2.reserve(8));
  PairArgs x;
  x.ci = pi;
  x.cj = pj;
  x.np = np;
  x.n_pad = e->n_pad;
  x.a = slp;
  x.b = srp;
  x.Ua = L.U16.as<_Float16>();
  x.Ub = R.U16.as<_Float16>();
  x.alpha = L.soff.as<double>();
  x.beta = R.soff.as<double>();
  x.qa = L.qa.as<double>();
  x.ra = L.ra.as<double>();
  x.qb = R.qb.as<double>();
  x.rb = R.rb.as<double>();
  x.z = e->z.as<double>();
  x.dg = e->dg.as<double>();
  x.py = e->py.as<double>();
  x.zz = e->zz;
  x.side = e->ps_side.as<double>();
  x.tiles = e->mx_tiles.as<uint8_t>();
  x.nib_i = L.nibI.as<uint8_t>();
  x.nib_j = R.nibJ.as<uint8_t>();
  x.tiles_bytes = (int64_t)e->mx_tiles.bytes;
  x.nK = nK;
  x.rho = e->rho_mx;
  x.chi_cut = chi_cut;
  x.counter = e->counter2.as<unsigned long long>();
  x.oi = e->cand2_i.as<int64_t>();
  x.oj = e->cand2_j.as<int64_t>();
  if (reset) GMAT_HIP(hipMemsetAsync(e->counter2.p, 0, 8, st));
  if (np > 0) {
  static bool attr = false;
  if (!attr) {
    GMAT_HIP(hipFuncSetAttribute((const void *)pair_side_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 256));
    attr = true;
  }
  size_t kt0;
  GMAT_TRY(kt_begin(e, st, &kt0));
  hipLaunchKernelGGL(pair_side_kernel, dim3((unsigned)cdiv(np, 4 * PS_PPW)), dim3(256),
                     (size_t)3 * e->n_pad * sizeof(float), st, x);
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(kt_end(e, st, KT_PAIR_SIDE, kt0, (double)np));
  GMAT_TRY(kt_begin(e, st, &kt0));
  if (nK <= PXR_NK) {  // w in registers: 256 pairs per workgroup
    // a short list in row-block segments over more workgroups (one per CU holds its LDS ring)
    if (!e->n_cu) {
      int dev = 0, cus = 0;
      GMAT_HIP(hipGetDevice(&dev));
      GMAT_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
      e->n_cu = std::max(cus, 8);
    }
    const int64_t wgs = cdiv(np, 256);
    const int nseg = (int)std::max<int64_t>(1, std::min<int64_t>(std::min(seg_max(), nK), e->n_cu / wgs));
    if (nseg > 1 && e->ps_mpart.bytes < (size_t)nseg * np * sizeof(double)) {
      GMAT_HIP(hipStreamSynchronize(st));
      GMAT_TRY(e->ps_mpart.alloc((size_t)std::max(8, nseg) * std::max<int64_t>(np, 1 << 16) * sizeof(double)));
    }
    x.mpart = e->ps_mpart.as<double>();
    hipLaunchKernelGGL(pair_mxr_kernel, dim3((unsigned)wgs, (unsigned)nseg), dim3(512), 0, st, x);
    if (nseg > 1) {
      GMAT_HIP(hipGetLastError());
      hipLaunchKernelGGL(pair_test_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, x, nseg);
    }
  } else {  // w in registers by squares of stages (pair_mxw_kernel)
    const int nQ = cdiv(nK, PXR_NK), nseg = nQ * (nQ + 1) / 2;
    if (e->ps_mpart.bytes < (size_t)nseg * np * sizeof(double)) {
      GMAT_HIP(hipStreamSynchronize(st));
      GMAT_TRY(e->ps_mpart.alloc((size_t)std::max(8, nseg) * std::max<int64_t>(np, 1 << 16) * sizeof(double)));
    }
    x.mpart = e->ps_mpart.as<double>();
    hipLaunchKernelGGL(pair_mxw_kernel, dim3((unsigned)cdiv(np, 256), (unsigned)nseg), dim3(512), 0, st, x);
    GMAT_HIP(hipGetLastError());
    hipLaunchKernelGGL(pair_test_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, x, nseg);
  }
  GMAT_HIP(hipGetLastError());
  GMAT_TRY(kt_end(e, st, KT_PAIR_MX, kt0, (double)np));
  }
  if (!n_out) return GMAT_OK;
  GMAT_HIP(hipMemcpyAsync(e->pins.count2.p, e->counter2.p, 8, hipMemcpyDeviceToHost, st));
  GMAT_HIP(hipStreamSynchronize(st));
  *n_out = (int64_t)*e->pins.count2.as<unsigned long long>();
  return GMAT_OK;
}

void kind_codings(int kind, int *lc, int *rc) {
  *lc = (kind == GMAT_DD) ? 1 : 0;
  *rc = (kind == GMAT_AA) ? 0 : 1;
}


// Low-rank screen setup: bottom eigenpairs of P (eig.hip, the intercept direction lifted
// out of the bottom by s 11'/n), fp6 quantisation of B (the exact values the MFMA multiplies),
// and the certificate: the largest lam (bisection) for which an fp64 Cholesky of
//   A = P - lam I + (lam + tau) 11'/n + B D(lam) B',  d_r = (lam - lam_r)_+ (1 + kappa)
// completes.  As for the prefilter, A + E = LL' with ||E||_2 <= gamma_{n+1} trace(A); the fp64
// rounding of A itself (at most (R + 4) u per entry of |P| + lam + 2(lam + tau)/n + |B|D|B'| <=
// cmax) adds n (R + 4) u (...) in the spectral norm.  Returns GMAT_OK with lr_R = 0 when the
// screen is disabled (GMAT_LR_RANK=0 / GMAT_NO_LR) or not applicable.
// Bottom eigenpairs of P with the intercept direction lifted out of the bottom (P + 4 tr(P)/n
// 11'/n): Ritz pairs of eig.hip's filtered subspace iteration (ascending); lam[r], r < ne, and eigenvector r as row r of Z (natural
// order).  The screens only need SOME basis and bounds -- every certificate below is checked by its
// own Cholesky -- so the eigenvectors' accuracy affects tightness, never correctness.
struct Eigen {
  int ne = 0, iters = 0;
  std::vector<double> lam, Z;
  DBuf dZ;  // Z on the device (ne x n)
};
int eigen_bottom(gmat_epi *e, const double *dP, double trP, int ne, Eigen *eg) {
  const int64_t n = e->n;
  DBuf A;
  DBuf &Z = eg->dZ;
  GMAT_TRY(A.alloc(n * n * sizeof(double)));
  GMAT_TRY(Z.alloc((size_t)n * ne * sizeof(double)));
  hipLaunchKernelGGL(pf_shift_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, 0, n, dP, 0.0, 4.0 * trP / (double)n,
                     A.as<double>());
  GMAT_HIP(hipGetLastError());
  eg->ne = ne;
  eg->lam.resize(ne);
  eg->Z.resize((size_t)n * ne);
  // residual tolerance 3e-4 of the Gershgorin bound (two Rayleigh-Ritz steps on the bench cohort);
  // lam_r = theta_r - |residual_r| (a Ritz value lies within its residual of an eigenvalue): with
  // these the certificates reach within ~0.3 % of those of exact eigenpairs (tighter costs block
  // iterations, not hits)
  const char *tenv = getenv("GMAT_EIG_TOL");
  std::vector<double> res(ne);
  GMAT_TRY(sym_eig_bottom(n, A.as<double>(), ne, tenv ? atof(tenv) : 3e-4, 16, eg->lam.data(), Z.as<double>(),
                          res.data(), &eg->iters));
  for (int r = 0; r < ne; ++r) eg->lam[r] -= res[r];
  GMAT_HIP(hipMemcpy(eg->Z.data(), Z.p, eg->Z.size() * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// Certificate search: the largest x in (0, top] for which ok(x) holds, trying a few candidates just
// below the eigenvalue estimate first (one Cholesky each; the first success is kept) and bisecting
// only when all of them fail.  ok returns 1 (certified), 0 (not), < 0 (error).
template <class F>
int certify_below(double top, F &&ok, double *best) {
  static const double fr[] = {1.0 - 2e-3, 1.0 - 2e-2, 0.9, 0.7};
  double hi = top;
  for (double f : fr) {
    const int r = ok(f * top);
    if (r < 0) return r;
    if (r) {  // certified; when a higher candidate failed, bisect a few steps between the two
      double lo = f * top;
      if (hi < top)
        for (int it = 0; it < 4; ++it) {
          const double mid = 0.5 * (lo + hi);
          const int q = ok(mid);
          if (q < 0) return q;
          (q ? lo : hi) = mid;
        }
      *best = lo;
      return GMAT_OK;
    }
    hi = f * top;
  }
  double lo = 0.0;
  for (int it = 0; it < 14; ++it) {
    const double mid = 0.5 * (lo + hi);
    const int r = ok(mid);
    if (r < 0) return r;
    (r ? lo : hi) = mid;
  }
  *best = lo;
  return GMAT_OK;
}


int lr_setup(gmat_epi *e, const double *dP, const double *pvp, double pmax, const Eigen &eg) {
  const int64_t n = e->n, n_pad = e->n_pad;
  const char *renv = getenv("GMAT_LR_RANK"), *kenv = getenv("GMAT_LR_KAPPA");
  const int R_req = renv ? atoi(renv) : default_lr_rank(e);
  if (R_req <= 0 || getenv("GMAT_NO_LR") || n < 8) return GMAT_OK;
  const int Re = (int)std::min<int64_t>(std::min<int64_t>(R_req, n - 1), eg.ne - 1);
  if (Re < 1) return GMAT_OK;
  const int Rp = (int)cdiv(Re, MXK) * MXK;
  const int ne = Re + 1;
  const double kap = kenv ? atof(kenv) : 0.45;
  double trP = 0.0;
  for (int64_t i = 0; i < n; ++i) trP += pvp[i * n + i];
  const std::vector<double> &lam_r = eg.lam, &Zh = eg.Z;
  const double t1 = now();
  // Q(lam) = fp6(sqrt(d_r(lam)) u_r), d_r = (lam - lam_r)_+ (1 + kappa): the rows of Q' are the
  // A operand of the screen (tile images) and Q Q' = B D B' enters the certificate exactly.
  const int nK = e->nK, nC = Rp / MXK;
  const double lam_top = lam_r[ne - 1];
  const char *tenv = getenv("GMAT_LR_TAU");
  const double tau = (tenv ? atof(tenv) : 0.5) * lam_top;
  const size_t img_words = (size_t)nC * nK * MX_TILE / 4;
  std::vector<double> Bn((size_t)n * Rp, 0.0);  // natural [k][r] (host copy of the certified Q)
  DBuf A, dBn, dBs, dsd, C, dinv, ld, cinfo;
  GMAT_TRY(A.alloc(n * n * sizeof(double)));
  GMAT_TRY(dBn.alloc(Bn.size() * sizeof(double)));
  GMAT_TRY(dBs.alloc((size_t)n_pad * Rp * sizeof(double)));
  GMAT_TRY(dsd.alloc(Rp * sizeof(double)));
  GMAT_TRY(C.alloc(n * n * sizeof(double)));
  GMAT_TRY(dinv.alloc(n * 64 * sizeof(double)));
  GMAT_TRY(ld.alloc(sizeof(double)));
  GMAT_TRY(cinfo.alloc(sizeof(int)));
  GMAT_TRY(e->lr_tiles.alloc(img_words * 4));
  GMAT_HIP(hipMemset(dBn.p, 0, Bn.size() * sizeof(double)));
  GMAT_HIP(hipMemset(dBs.p, 0, (size_t)n_pad * Rp * sizeof(double)));
  GMAT_HIP(hipMemset(e->lr_tiles.p, 0, img_words * 4));
  auto quantise = [&](double lam, bool images) -> int {
    std::vector<double> sd(Rp, 0.0);
    for (int r = 0; r < Re; ++r) sd[r] = std::sqrt(std::max(lam - lam_r[r], 0.0) * (1.0 + kap));
    GMAT_HIP(hipMemcpy(dsd.p, sd.data(), Rp * sizeof(double), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(lr_quant_kernel, dim3((unsigned)cdiv((int64_t)Rp * (n_pad / 32), 256)), dim3(256), 0, 0, n, n_pad,
                       nK, Rp, eg.dZ.as<double>(), dsd.as<double>(), dBn.as<double>(), dBs.as<double>(),
                       images ? e->lr_tiles.as<uint32_t>() : nullptr);
    GMAT_HIP(hipGetLastError());
    return GMAT_OK;
  };
  auto eps_of = [&](double lam) {  // Bn must be quantise(lam)
    double trC = 0.0, cmax = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      double ck = 0.0;
      for (int r = 0; r < Rp; ++r) ck += Bn[(size_t)k * Rp + r] * Bn[(size_t)k * Rp + r];
      trC += ck;
      cmax = std::max(cmax, ck);
    }
    const double u = std::ldexp(1.0, -53);
    const double trA = trP + trC + (lam + tau) - (double)n * lam;
    return 2.0 * (double)(n + 1) * u * std::fabs(trA) * 1.01 +
           (double)n * (Rp + 4) * u * (pmax + 2.0 * lam + 2.0 * (lam + tau) / (double)n + cmax);
  };
  auto ok = [&](double lam) -> int {
    GMAT_TRY(quantise(lam, false));
    GMAT_TRY(dgemm(0, n, n, Rp, 1.0, DView{dBn.as<double>(), Rp, 0}, DView{dBn.as<double>(), Rp, 1}, 0.0,
                   C.as<double>(), n));
    hipLaunchKernelGGL(lr_shift_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, 0, n, dP, C.as<double>(), lam,
                       tau, A.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(cholesky(0, n, A.as<double>(), n, dinv.as<double>(), ld.as<double>(), cinfo.as<int>()));
    e->setup[6] += 1;
    int hi = 1;
    GMAT_HIP(hipMemcpy(&hi, cinfo.p, sizeof(int), hipMemcpyDeviceToHost));
    return hi == 0 ? 1 : 0;
  };
  double lo = 0.0;
  GMAT_TRY(certify_below(lam_top, ok, &lo));
  GMAT_TRY(quantise(lo, true));  // the certified Q (quantise is deterministic)
  GMAT_HIP(hipMemcpy(Bn.data(), dBn.p, Bn.size() * sizeof(double), hipMemcpyDeviceToHost));
  e->setup[3] = now() - t1;
  const double eps = eps_of(lo);
  if (getenv("GMAT_DEBUG"))
    fprintf(stderr, "lr_setup: R %d (padded %d) lam_0 %.4g lam_R %.4g -> lam %.4g tau %.3g eps %.3g (pf_mu %.4g); "
                    "certificate %.3f s\n",
            Re, Rp, lam_r[0], lam_top, lo, tau, eps, e->pf_mu, now() - t1);
  if (!(lo > 0.0) || lo <= e->pf_mu || lo < 1e3 * eps) return GMAT_OK;  // no better than the prefilter
  // |c~_r - c_r| <= eta_r = u32 |Q_r|_1 (8 n_pad + 400): fp32 accumulation over n_pad products
  // (w <= 4, one rounding per product, x2 for the MFMA's internal order), the fp32 G' / H and the
  // 2-term combination; the kernel bounds sum_r c_r^2 <= (|c~| + |eta|)^2 with E = |eta|^2
  std::vector<double> q1(Rp, 0.0);
  double Esum = 0.0;
  const double u32 = std::ldexp(1.0, -24);
  for (int r = 0; r < Rp; ++r) {
    double l1 = 0.0;
    for (int64_t k = 0; k < n; ++k) {
      l1 += std::fabs(Bn[(size_t)k * Rp + r]);
      q1[r] += Bn[(size_t)k * Rp + r];
    }
    const double eta = u32 * l1 * (8.0 * (double)n_pad + 400.0) * 1.01;
    Esum += eta * eta;
  }
  GMAT_TRY(e->lr_Bs.alloc((size_t)n_pad * Rp * sizeof(double)));
  GMAT_TRY(e->lr_q1.alloc(Rp * sizeof(double)));
  GMAT_HIP(hipMemcpy(e->lr_Bs.p, dBs.p, (size_t)n_pad * Rp * sizeof(double), hipMemcpyDeviceToDevice));
  GMAT_HIP(hipMemcpy(e->lr_q1.p, q1.data(), Rp * sizeof(double), hipMemcpyHostToDevice));
  e->lr_lam = lo;
  e->lr_tau = tau;
  e->lr_eps = eps + 1e-15 * lo;
  e->lr_E = Esum * 1.001;
  e->lr_R = Rp;
  return GMAT_OK;
}
}  // namespace epi
}  // namespace gmat

namespace gmat {
namespace epi {
constexpr uint64_t EPI_STATE_MAGIC = 0x31495045544d4147ULL;  // "GMATEPI1"
int import_state(gmat_epi *e, const uint8_t *st, int64_t bytes);
}  // namespace epi
}  // namespace gmat

// ||R^16||_F^(1/16) >= ||R||_2 (R symmetric) from a residual in r1 scaled to entries of order one:
// four fp64 MFMA squarings (r1, r2 are overwritten)
// the device part on stream st (row sums of squares of R^16 land in rrows)
static int fro16_enqueue(hipStream_t st, int64_t n_pad, DBuf &r1, DBuf &r2, DBuf &rrows) {
  double *src = r1.as<double>(), *dst = r2.as<double>();
  for (int q = 0; q < 4; ++q) {
    GMAT_TRY(dgemm(st, n_pad, n_pad, n_pad, 1.0, DView{src, n_pad, 0}, DView{src, n_pad, 0}, 0.0, dst, n_pad));
    std::swap(src, dst);
  }
  return dot_rows(st, n_pad, n_pad, src, n_pad, src, n_pad, rrows.as<double>());
}
static int fro16_finish(int64_t n_pad, DBuf &rrows, double *fro_root) {
  std::vector<double> hr(n_pad);
  GMAT_HIP(hipMemcpy(hr.data(), rrows.p, n_pad * sizeof(double), hipMemcpyDeviceToHost));
  double fro2 = 0.0;
  for (double v : hr) fro2 += v;
  *fro_root = std::pow(std::sqrt(fro2), 1.0 / 16.0);
  return GMAT_OK;
}

// rho[S], the int8 screen's bound ||P_off - sum_{s<S} A_s 128^-s qmax/127||_2 for S slices, computed
// when a scan first uses that level (the low-rank and MX levels never do): the residual of the
// slicing of P in storage order (a symmetric permutation of the natural one: same spectrum)
int gmat::epi::ensure_rho(gmat_epi *e, int S) {
  if (S < 1 || S > e->n_slice || e->rho[S] > 0.0) return GMAT_OK;
  const int64_t n_pad = e->n_pad;
  DBuf r1, r2, rrows;
  GMAT_TRY(r1.alloc(n_pad * n_pad * sizeof(double)));
  GMAT_TRY(r2.alloc(n_pad * n_pad * sizeof(double)));
  GMAT_TRY(rrows.alloc(n_pad * sizeof(double)));
  const double unit = e->qmax > 0 ? 127.0 / e->qmax : 1.0;
  const double rmax = 0.5 * std::pow(128.0, -(S - 1)) / unit;
  hipLaunchKernelGGL(residual_kernel, dim3((unsigned)cdiv(n_pad * n_pad, 256)), dim3(256), 0, 0, n_pad, n_pad,
                     e->Ps.as<double>(), unit, S, 1.0 / 64.0, r1.as<double>());  // residual in [-64, 64] units
  GMAT_HIP(hipGetLastError());
  double fr;
  GMAT_TRY(fro16_enqueue(0, n_pad, r1, r2, rrows));
  GMAT_TRY(fro16_finish(n_pad, rrows, &fr));
  // 5% margin for the fp64 rounding of the squarings, plus the rounding of P*unit itself
  e->rho[S] = 1.05 * rmax * fr + 1e-15 * e->pmax * (double)e->n;
  return GMAT_OK;
}

int gmat::epi::epi_create_impl(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                               const uint8_t *state, int64_t state_bytes, bool allow_seg) {
  GMAT_CHECK(out && g && pvp && py, GMAT_E_ARG, "gmat_epi_create: bad arguments");
  GMAT_CHECK(n_slice >= 1 && n_slice <= 4, GMAT_E_ARG, "gmat_epi_create: n_slice must be 1..4");
  GMAT_CHECK(g->total_missing == 0, GMAT_E_ARG, "gmat_epi_create: panel has missing genotypes (impute first)");
  // panels whose byte offsets would reach 2^32 (the kernels' 32-bit lane offsets from a 64-bit base):
  // a plan of SNP segments, each sub-plan within the limit (epi_seg.hip)
  if (allow_seg && seg_snps(g) > 0) return seg_create(out, g, pvp, py, n_slice, state, state_bytes);
  GMAT_CHECK(2 * g->m * g->n_pad < ((int64_t)1 << 32), GMAT_E_ARG, "gmat_epi_create: a single-panel plan of %lld SNPs "
             "x %lld individuals (2 m n_pad >= 2^32)", (long long)g->m, (long long)g->n_pad);
  const double t_create = now();
  auto *e = new gmat_epi();
  // past EXH_ONLY_NPAD individuals no screen applies (the int8 slice screen's 24-bit epilogue sums, the
  // pair screen's LDS-resident planes): every pair is refined exactly (GMAT_EXH_ONLY: the same below it)
  e->exh_only = g->n_pad > EXH_ONLY_NPAD || getenv("GMAT_EXH_ONLY") != nullptr;
  e->g = g;
  e->n = g->n;
  e->n_pad = g->n_pad;
  e->m = g->m;
  e->n_slice = n_slice;
  e->nK = (int)(g->n_pad / MXK);
  const int64_t n = e->n, n_pad = e->n_pad;
  // max |P|, max |P_kl| off the diagonal and the fingerprint of P: on the device after the upload
  // (p_scan_kernel; the host scan took ~3 ms of every plan at n = 2,000)
  double pmax = 0.0, qmax = 0.0, dmax = 0.0;
  uint64_t ph = 0;
  double spy = 0.0;
  for (int64_t i = 0; i < n; ++i) spy += py[i];
  e->spy = spy;
  DBuf dp, dv;
  int rc = GMAT_OK;
  auto fail = [&](int code) {
    (void)hipDeviceSynchronize();  // nothing in flight (the MX bound's stream) still uses the plan
    delete e;
    return code;
  };
  if ((rc = dp.alloc(n * n * sizeof(double))) || (rc = dv.alloc(n * sizeof(double))) ||
      (rc = e->Ps.alloc(n_pad * n_pad * sizeof(double))) || (rc = e->py.alloc(n_pad * sizeof(double))) ||
      (rc = e->z.alloc(n_pad * sizeof(double))) || (rc = e->dg.alloc(n_pad * sizeof(double))) ||
      (!e->exh_only && (rc = e->slices.alloc((size_t)n_slice * n_pad * n_pad))) ||
      (rc = e->spanels.alloc((size_t)2 * e->m * n_pad)))
    return fail(rc);
  if (hipMemcpy(dp.p, pvp, n * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(dv.p, py, n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    set_error("gmat_epi_create: upload failed");
    return fail(GMAT_E_HIP);
  }
  {
    DBuf scan;
    if ((rc = scan.alloc((size_t)3 * n * sizeof(double)))) return fail(rc);
    hipLaunchKernelGGL(p_scan_kernel, dim3((unsigned)n), dim3(256), 0, 0, n, dp.as<double>(), scan.as<double>());
    std::vector<double> hs((size_t)3 * n);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpy(hs.data(), scan.p, hs.size() * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
      set_error("gmat_epi_create: scan of P failed");
      return fail(GMAT_E_HIP);
    }
    ph = 0x9e3779b97f4a7c15ULL ^ (uint64_t)n;
    for (int64_t i = 0; i < n; ++i) {
      qmax = std::max(qmax, hs[i]);
      dmax = std::max(dmax, hs[n + i]);
      uint64_t h;
      memcpy(&h, &hs[2 * n + i], 8);
      ph += h;  // a sum of per-element mixes: independent of the reduction order
    }
    pmax = std::max(qmax, dmax);
  }
  e->qmax = qmax;
  e->p_hash = ph;
  const unsigned gb = (unsigned)cdiv(n_pad * n_pad, 256);
  hipLaunchKernelGGL(permute_p_kernel, dim3(gb), dim3(256), 0, 0, n, n_pad, dp.as<double>(), e->Ps.as<double>());
  hipLaunchKernelGGL(permute_vec_kernel, dim3((unsigned)cdiv(n_pad, 256)), dim3(256), 0, 0, n, n_pad, dv.as<double>(),
                     e->py.as<double>());
  const double unit = qmax > 0 ? 127.0 / qmax : 1.0;
  if (!e->exh_only)
    hipLaunchKernelGGL(slice_kernel, dim3(gb), dim3(256), 0, 0, n, n_pad, dp.as<double>(), unit, n_slice,
                       e->slices.as<int8_t>());
  hipLaunchKernelGGL(zsum_kernel, dim3((unsigned)cdiv(n_pad, 4)), dim3(256), 0, 0, n_pad, e->Ps.as<double>(),
                     e->z.as<double>());
  hipLaunchKernelGGL(diag_kernel, dim3((unsigned)cdiv(n_pad, 256)), dim3(256), 0, 0, n_pad, e->Ps.as<double>(),
                     e->dg.as<double>());
  if (hipGetLastError() != hipSuccess) {
    set_error("gmat_epi_create: setup kernels failed");
    return fail(GMAT_E_HIP);
  }
  // the int8 levels' bounds rho[S] are computed on first use (ensure_rho)
  e->pmax = pmax;
  // the plan's last step: 1'P1 (z summed on the host)
  auto finish_plan = [&]() -> int {
    std::vector<double> hz(n_pad);
    if (hipMemcpy(hz.data(), e->z.p, n_pad * sizeof(double), hipMemcpyDeviceToHost) != hipSuccess) {
      set_error("gmat_epi_create: z download failed");
      return fail(GMAT_E_HIP);
    }
    double zz = 0.0;
    for (double v : hz) zz += v;
    e->zz = zz;
    e->setup[0] = now() - t_create;
    *out = e;
    return GMAT_OK;
  };
  if (e->exh_only) {  // no screens: P, z, diag(P) and Py are all the exact refine reads
    if (state && (rc = import_state(e, state, state_bytes)) != GMAT_OK) return fail(rc);
    e->pf_mu = 0.0;
    e->lr_R = 0;
    return finish_plan();
  }
  DBuf r1, r2, rrows;
  if ((rc = r1.alloc(n_pad * n_pad * sizeof(double))) || (rc = r2.alloc(n_pad * n_pad * sizeof(double))) ||
      (rc = rrows.alloc(n_pad * sizeof(double))))
    return fail(rc);
  // MX screen: fp6 records + scales, the residual of the matrix it evaluates, and the fp32
  // accumulation bound: every acc_k is a sum of at most n_pad products (each exact in fp32)
  // accumulated with at most one rounding per product (x2 margin for the MFMA's internal
  // order), the epilogue adds 32 roundings; all are bounded by u * w'|E|w <= u * max_k
  // sum_l |E_kl| * |w|^2 (|E| symmetric non-negative).
  // The bound's four fp64 squarings run on a stream of their own beside the eigendecomposition
  // below (whose small Rayleigh-Ritz steps leave most CUs idle); rho_mx is finished after it.
  DBuf qn, rabs;
  if ((rc = e->mx_tiles.alloc((size_t)e->nK * e->nK * MX_TILE)) || (rc = qn.alloc(n_pad * n_pad * sizeof(double))) ||
      (rc = rabs.alloc(n_pad * sizeof(double))))
    return fail(rc);
  hipStream_t sx = nullptr;
  if ((rc = pipeline_stream(0, &sx)) != GMAT_OK) return fail(rc);
  struct StreamGuard {  // the squarings are done before the plan is (or fails)
    hipStream_t s;
    ~StreamGuard() { (void)hipStreamSynchronize(s); }
  } sx_guard{sx};
  (void)hipDeviceSynchronize();  // P, the slices and z / dg are ready for both streams
  const double os = qmax > 0 ? 15.0 / qmax : 1.0;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((unsigned)cdiv(n_pad * (n_pad / 32), 256)), dim3(256), 0, sx, n, n_pad,
                     e->nK, dp.as<double>(), e->mx_tiles.as<uint32_t>(), qn.as<double>());
  hipLaunchKernelGGL(mx_residual_kernel, dim3((unsigned)n_pad), dim3(256), 0, sx, n, n_pad, dp.as<double>(),
                     qn.as<double>(), os, r1.as<double>(), rabs.as<double>());
  if (hipGetLastError() != hipSuccess) {
    set_error("gmat_epi_create: MX setup kernels failed");
    return fail(GMAT_E_HIP);
  }
  if ((rc = fro16_enqueue(sx, n_pad, r1, r2, rrows))) return fail(rc);
  auto finish_mx = [&]() -> int {
    GMAT_HIP(hipStreamSynchronize(sx));
    double fr;
    GMAT_TRY(fro16_finish(n_pad, rrows, &fr));
    std::vector<double> ha(n_pad);
    GMAT_HIP(hipMemcpy(ha.data(), rabs.p, n_pad * sizeof(double), hipMemcpyDeviceToHost));
    double amax = 0.0;
    for (double v : ha) amax = std::max(amax, v);
    const double u = std::ldexp(1.0, -24);
    e->rho_mx = 1.05 * fr / os + 1e-15 * pmax * (double)n + 1.01 * (2.0 * (double)n_pad + 64.0) * u * amax;
    return GMAT_OK;
  };
  e->setup[4] = now() - t_create;
  if (state) {  // the spectral state (eigenpairs, certificates, Q images) of another rank's plan
    if ((rc = import_state(e, state, state_bytes)) != GMAT_OK) return fail(rc);
  } else {
    double trP = 0.0;
    for (int64_t i = 0; i < n; ++i) trP += pvp[i * n + i];
    // Bottom eigenpairs of P (intercept lifted): the prefilter's covariate directions (P's other null
    // directions: eigenvalues ~ 0), its mu estimate, and the low-rank screen's basis.
    Eigen eg;
    bool have_eig = false;
    {
      const double t_eig = now();
      const char *renv = getenv("GMAT_LR_RANK");
      const int R_req = renv ? std::max(0, atoi(renv)) : default_lr_rank(e);
      const int ne = (int)std::min<int64_t>(std::max(R_req, 16) + 1, n);
      have_eig = n >= 8 && !getenv("GMAT_NO_PREFILTER") && eigen_bottom(e, dp.as<double>(), trP, ne, &eg) == GMAT_OK;
      if (!have_eig && getenv("GMAT_DEBUG")) fprintf(stderr, "gmat_epi_create: no eigendecomposition (%s)\n", gmat_last_error());
      e->setup[2] = now() - t_eig;
    }
    int K0 = 0;
    if (have_eig)
      while (K0 < eg.ne && eg.lam[K0] < 1e-9 * trP / (double)n) ++K0;
    // Spectral prefilter certificate.  If the fp64 Cholesky of
    //   A = P + (mu + tau) 11'/n + ku U U' - mu I      (U: the K0 null directions, ku = mu + tau)
    // completes with positive pivots, A + E = LL' with |E| <= gamma_{n+1} |L||L'|, so lambda_min(A)
    // >= -||E||_2 >= -gamma_{n+1} trace(A) (||L||_F^2 = trace(LL')), i.e. for every e
    //   e'Pe >= mu |e|^2 - (mu + tau)(1'e)^2/n - ku |U'e|^2 - eps |e|^2,
    // eps = 2 gamma_{n+1} trace(A) (x2 margin for the blocked MFMA order) + the rounding of forming A.
    // tau (a small lift) keeps the directions P annihilates definite; mu starts just below the
    // smallest eigenvalue off those directions.
    const double t_pf = now();
    if (have_eig && K0 <= PF_NCOV_MAX && K0 < eg.ne) {
      DBuf A, dinv, ld, info, dU, C;
      if ((rc = A.alloc(n * n * sizeof(double))) || (rc = dinv.alloc(n * 64 * sizeof(double))) ||
          (rc = ld.alloc(sizeof(double))) || (rc = info.alloc(sizeof(int))))
        return fail(rc);
      double cmax = 0.0;
      if (K0 > 0) {  // C = U'U (n x n) from the eigenvectors, exactly as stored
        if ((rc = dU.alloc((size_t)K0 * n * sizeof(double))) || (rc = C.alloc(n * n * sizeof(double)))) return fail(rc);
        if (hipMemcpy(dU.p, eg.Z.data(), (size_t)K0 * n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
          set_error("gmat_epi_create: direction upload failed");
          return fail(GMAT_E_HIP);
        }
        if ((rc = dgemm(0, n, n, K0, 1.0, DView{dU.as<double>(), n, 1}, DView{dU.as<double>(), n, 0}, 0.0, C.as<double>(),
                        n)))
          return fail(rc);
        for (int64_t i = 0; i < n; ++i) {
          double cii = 0.0;
          for (int k = 0; k < K0; ++k) cii += eg.Z[(size_t)k * n + i] * eg.Z[(size_t)k * n + i];
          cmax = std::max(cmax, cii);
        }
      }
      const double tau0 = 1e-8 * trP / (double)n;
      auto ok = [&](double mu) -> int {  // 1 = certified, 0 = not, < 0 error
        const double tau = tau0 + 1e-6 * mu;
        hipLaunchKernelGGL(pf_shift_u_kernel, dim3((unsigned)cdiv(n * n, 256)), dim3(256), 0, 0, n, dp.as<double>(),
                           K0 ? C.as<double>() : nullptr, mu, tau, mu + tau, A.as<double>());
        if (hipGetLastError() != hipSuccess) return -1;
        if (cholesky(0, n, A.as<double>(), n, dinv.as<double>(), ld.as<double>(), info.as<int>()) != GMAT_OK) return -1;
        e->setup[6] += 1;
        int hinfo = 1;
        if (hipMemcpy(&hinfo, info.p, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) return -1;
        return hinfo == 0 ? 1 : 0;
      };
      double lo = 0.0;
      if (certify_below(eg.lam[K0], ok, &lo) != GMAT_OK) {
        set_error("gmat_epi_create: prefilter certificate failed");
        return fail(GMAT_E_HIP);
      }
      const double tau = tau0 + 1e-6 * lo, u = std::ldexp(1.0, -53);
      const double trA = trP + (lo + tau) + (lo + tau) * K0 - (double)n * lo;
      const double eps = 2.0 * (double)(n + 1) * u * std::fabs(trA) * 1.01 +
                         (double)n * (K0 + 4) * u * (pmax + lo + 2.0 * (lo + tau) / (double)n + (lo + tau) * cmax);
      if (lo > 0.0 && lo > 1e3 * eps) {
        e->pf_mu = lo;
        e->pf_tau = tau;
        e->pf_eps = eps + 1e-15 * lo;
        e->pf_ku = lo + tau;
        e->pf_ncov = K0;
        if (K0 > 0) {  // the directions in storage order for the codings' images
          std::vector<double> Us((size_t)K0 * n_pad, 0.0);
          for (int k = 0; k < K0; ++k) {
            double su = 0.0;
            for (int64_t c = 0; c < n; ++c) su += eg.Z[(size_t)k * n + c];
            e->pf_su[k] = su;
            for (int64_t q = 0; q < n_pad; ++q) {
              const int64_t c = (q & ~31LL) + perm_nat((int)(q & 31));
              if (c < n) Us[(size_t)k * n_pad + q] = eg.Z[(size_t)k * n + c];
            }
          }
          if ((rc = e->pf_U.alloc(Us.size() * sizeof(double)))) return fail(rc);
          if (hipMemcpy(e->pf_U.p, Us.data(), Us.size() * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
            set_error("gmat_epi_create: direction upload failed");
            return fail(GMAT_E_HIP);
          }
        }
      }
      if (getenv("GMAT_DEBUG"))
        fprintf(stderr, "gmat_epi_create: prefilter mu %.6g (lam %.6g) eps %.3g, %d covariate directions (trace/n %.4g)\n", lo,
                eg.lam[K0], eps, K0, trP / n);
    } else if (getenv("GMAT_DEBUG")) {
      fprintf(stderr, "gmat_epi_create: prefilter off (%d null directions, eigen %d)\n", K0, (int)have_eig);
    }
    e->setup[1] = now() - t_pf;
    if (e->pf_mu > 0.0 && (rc = lr_setup(e, dp.as<double>(), pvp, pmax, eg)) != GMAT_OK) {
      // the low-rank screen is an accelerator: without it the MX screen runs
      if (getenv("GMAT_DEBUG")) fprintf(stderr, "gmat_epi_create: low-rank screen unavailable: %s\n", gmat_last_error());
      e->lr_R = 0;
      rc = GMAT_OK;
    }
  }  // spectral state computed here
  if ((rc = finish_mx()) != GMAT_OK) return fail(rc);
  return finish_plan();
}

extern "C" int gmat_epi_create(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice) {
  return epi_create_impl(out, g, pvp, py, n_slice, nullptr, 0);
}

extern "C" int gmat_epi_create_with(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                                    const uint8_t *state, int64_t state_bytes) {
  GMAT_CHECK(state && state_bytes > 0, GMAT_E_ARG, "gmat_epi_create_with: no state");
  return epi_create_impl(out, g, pvp, py, n_slice, state, state_bytes);
}

namespace gmat {
namespace epi {
struct StateHead {
  uint64_t magic, n, n_pad, p_hash;
  double d[12];  // pf_mu, pf_tau, pf_eps, pf_ku, pf_su[4], lr_lam, lr_tau, lr_eps, lr_E
  int64_t pf_ncov, lr_R, tiles_bytes, pad;
};
int64_t state_size(const gmat_epi *e) {
  return (int64_t)sizeof(StateHead) + (int64_t)e->pf_ncov * e->n_pad * 8 + (e->lr_R ? (int64_t)e->lr_tiles.bytes : 0) +
         (int64_t)e->n_pad * e->lr_R * 8 + (int64_t)e->lr_R * 8;
}
int import_state(gmat_epi *e, const uint8_t *st, int64_t bytes) {
  StateHead h;
  GMAT_CHECK(bytes >= (int64_t)sizeof(h), GMAT_E_ARG, "plan state: %lld bytes", (long long)bytes);
  memcpy(&h, st, sizeof(h));
  GMAT_CHECK(h.magic == EPI_STATE_MAGIC && (int64_t)h.n == e->n && (int64_t)h.n_pad == e->n_pad, GMAT_E_ARG,
             "plan state: not a state of an n = %lld plan", (long long)e->n);
  GMAT_CHECK(h.p_hash == e->p_hash, GMAT_E_ARG, "plan state: computed for a different P");
  GMAT_CHECK(h.pf_ncov >= 0 && h.pf_ncov <= PF_NCOV_MAX && h.lr_R >= 0 && h.tiles_bytes >= 0, GMAT_E_ARG,
             "plan state: corrupt header");
  // the low-rank screen's rank is whole 128-deep basis chunks below n_pad, and its tile images are
  // exactly nC x nK tiles (the kernel derives nC = lr_R / MXK from the rank, not from the payload)
  GMAT_CHECK(h.lr_R % MXK == 0 && h.lr_R < e->n_pad, GMAT_E_ARG, "plan state: low-rank rank %lld is not a multiple "
             "of %d below n_pad %lld", (long long)h.lr_R, MXK, (long long)e->n_pad);
  GMAT_CHECK(h.lr_R == 0 || h.tiles_bytes == (h.lr_R / MXK) * (int64_t)e->nK * MX_TILE, GMAT_E_ARG,
             "plan state: %lld tile bytes for rank %lld (%lld expected)", (long long)h.tiles_bytes, (long long)h.lr_R,
             (long long)((h.lr_R / MXK) * (int64_t)e->nK * MX_TILE));
  e->pf_mu = h.d[0];
  e->pf_tau = h.d[1];
  e->pf_eps = h.d[2];
  e->pf_ku = h.d[3];
  for (int k = 0; k < 4; ++k) e->pf_su[k] = h.d[4 + k];
  e->lr_lam = h.d[8];
  e->lr_tau = h.d[9];
  e->lr_eps = h.d[10];
  e->lr_E = h.d[11];
  e->pf_ncov = (int)h.pf_ncov;
  e->lr_R = (int)h.lr_R;
  int64_t off = sizeof(h);
  const int64_t nU = (int64_t)e->pf_ncov * e->n_pad * 8, nB = e->n_pad * (int64_t)e->lr_R * 8, nq = e->lr_R * 8LL;
  GMAT_CHECK(bytes == off + nU + (e->lr_R ? h.tiles_bytes : 0) + nB + nq, GMAT_E_ARG, "plan state: %lld bytes, "
             "header describes %lld", (long long)bytes, (long long)(off + nU + h.tiles_bytes + nB + nq));
  if (nU) {
    GMAT_TRY(e->pf_U.alloc(nU));
    GMAT_HIP(hipMemcpy(e->pf_U.p, st + off, nU, hipMemcpyHostToDevice));
    off += nU;
  }
  if (e->lr_R) {
    GMAT_TRY(e->lr_tiles.alloc(h.tiles_bytes));
    GMAT_HIP(hipMemcpy(e->lr_tiles.p, st + off, h.tiles_bytes, hipMemcpyHostToDevice));
    off += h.tiles_bytes;
    GMAT_TRY(e->lr_Bs.alloc(nB));
    GMAT_HIP(hipMemcpy(e->lr_Bs.p, st + off, nB, hipMemcpyHostToDevice));
    off += nB;
    GMAT_TRY(e->lr_q1.alloc(nq));
    GMAT_HIP(hipMemcpy(e->lr_q1.p, st + off, nq, hipMemcpyHostToDevice));
  }
  e->imported = 1;
  return GMAT_OK;
}
}  // namespace epi
}  // namespace gmat

// The plan's spectral state -- the prefilter and low-rank certificates (P's covariate directions,
// mu, lam, tau, eps and the certified Q's tile images and fp64 copy) -- serialised so that one
// rank computes it and every other rank imports it (gmat_epi_create_with): the eigendecomposition
// and the certificate searches run once per job.  *needed = the size; buf may be null.
extern "C" int gmat_epi_export(const gmat_epi *e, uint8_t *buf, int64_t cap, int64_t *needed) {
  GMAT_CHECK(e && needed, GMAT_E_ARG, "gmat_epi_export: bad arguments");
  if (e->seg) return gmat_epi_export(seg_base(e), buf, cap, needed);  // the state of the segments' plans
  const int64_t sz = state_size(e);
  *needed = sz;
  if (!buf) return GMAT_OK;
  GMAT_CHECK(cap >= sz, GMAT_E_OVERFLOW, "gmat_epi_export: %lld bytes needed", (long long)sz);
  StateHead h{};
  h.magic = EPI_STATE_MAGIC;
  h.n = e->n;
  h.n_pad = e->n_pad;
  h.p_hash = e->p_hash;
  const double d[12] = {e->pf_mu, e->pf_tau, e->pf_eps, e->pf_ku, e->pf_su[0], e->pf_su[1],
                        e->pf_su[2], e->pf_su[3], e->lr_lam, e->lr_tau, e->lr_eps, e->lr_E};
  memcpy(h.d, d, sizeof(d));
  h.pf_ncov = e->pf_ncov;
  h.lr_R = e->lr_R;
  h.tiles_bytes = e->lr_R ? (int64_t)e->lr_tiles.bytes : 0;
  memcpy(buf, &h, sizeof(h));
  int64_t off = sizeof(h);
  const int64_t nU = (int64_t)e->pf_ncov * e->n_pad * 8;
  if (nU) {
    GMAT_HIP(hipMemcpy(buf + off, e->pf_U.p, nU, hipMemcpyDeviceToHost));
    off += nU;
  }
  if (e->lr_R) {
    GMAT_HIP(hipMemcpy(buf + off, e->lr_tiles.p, h.tiles_bytes, hipMemcpyDeviceToHost));
    off += h.tiles_bytes;
    GMAT_HIP(hipMemcpy(buf + off, e->lr_Bs.p, e->n_pad * (int64_t)e->lr_R * 8, hipMemcpyDeviceToHost));
    off += e->n_pad * (int64_t)e->lr_R * 8;
    GMAT_HIP(hipMemcpy(buf + off, e->lr_q1.p, e->lr_R * 8LL, hipMemcpyDeviceToHost));
  }
  return GMAT_OK;
}

extern "C" int gmat_epi_setup_stats(const gmat_epi *e, double *out8) {
  GMAT_CHECK(e && out8, GMAT_E_ARG, "gmat_epi_setup_stats: bad arguments");
  if (e->seg) return gmat_epi_setup_stats(seg_base(e), out8);
  for (int k = 0; k < 7; ++k) out8[k] = e->setup[k];
  out8[7] = e->pf_ncov;
  return GMAT_OK;
}

extern "C" int gmat_epi_info(const gmat_epi *e, double *out8) {
  GMAT_CHECK(e && out8, GMAT_E_ARG, "gmat_epi_info: bad arguments");
  if (e->seg) return gmat_epi_info(seg_base(e), out8);
  out8[0] = e->lr_R;
  out8[1] = e->lr_lam;
  out8[2] = e->pf_mu;
  out8[3] = (double)e->n_pad;
  // prefilter_pass_kernel<.., 32, 5> (epi_prefilter.hip): per stage four 1 KB DMAs of the two int8 L3
  // slices, four of the 256 columns' 2-bit codes and one of the 32 rows' codes (twice); per tile the
  // 32-byte test records of its 32 rows and 256 columns
  out8[4] = 32;
  out8[5] = PF_TC;
  out8[6] = 9 * 1024;
  out8[7] = (32 + PF_TC) * PF_REC * sizeof(float);
  return GMAT_OK;
}

extern "C" int gmat_epi_destroy(gmat_epi *e) {
  delete e;
  return GMAT_OK;
}

extern "C" int gmat_epi_pairs(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *eff, double *var,
                              double *chi, double *p) {
  GMAT_CHECK(e && (n_pairs == 0 || (pairs && eff && var && chi && p)), GMAT_E_ARG, "gmat_epi_pairs: bad arguments");
  GMAT_CHECK(kind >= 0 && kind <= 2, GMAT_E_ARG, "gmat_epi_pairs: bad kind");
  if (n_pairs == 0) return GMAT_OK;
  if (e->seg) return seg_pairs(e, kind, pairs, n_pairs, eff, var, chi, p);
  int lc, rc;
  kind_codings(kind, &lc, &rc);
  GMAT_TRY(build_coding(e, lc));
  GMAT_TRY(build_coding(e, rc));
  // the kernel timers record the calls since the last scan or pairs call only (refine() marks every
  // chunk's launches: without the reset repeated pairs calls would grow them without bound)
  e->kev_used = 0;
  e->kmarks.clear();
  std::vector<int64_t> hi(n_pairs), hj(n_pairs);
  for (int64_t t = 0; t < n_pairs; ++t) {
    hi[t] = pairs[2 * t];
    hj[t] = pairs[2 * t + 1];
    GMAT_CHECK(hi[t] >= 0 && hi[t] < e->m && hj[t] >= 0 && hj[t] < e->m, GMAT_E_ARG, "pair %lld out of range",
               (long long)t);
  }
  const int8_t *lp = lc == 0 ? e->g->dose_ptr() : e->g->het_ptr();
  const int8_t *rp = rc == 0 ? e->g->dose_ptr() : e->g->het_ptr();
  const int64_t chunk = 1 << 16;
  DBuf di, dj, de, dv, dc, dpv;
  GMAT_TRY(di.alloc(chunk * 8));
  GMAT_TRY(dj.alloc(chunk * 8));
  GMAT_TRY(de.alloc(chunk * 8));
  GMAT_TRY(dv.alloc(chunk * 8));
  GMAT_TRY(dc.alloc(chunk * 8));
  GMAT_TRY(dpv.alloc(chunk * 8));
  for (int64_t t0 = 0; t0 < n_pairs; t0 += chunk) {
    const int64_t np = std::min(chunk, n_pairs - t0);
    GMAT_HIP(hipMemcpy(di.p, hi.data() + t0, np * 8, hipMemcpyHostToDevice));
    GMAT_HIP(hipMemcpy(dj.p, hj.data() + t0, np * 8, hipMemcpyHostToDevice));
    GMAT_TRY(refine(e, e->s, e->code[lc], e->code[rc], lp, rp, di.as<int64_t>(), dj.as<int64_t>(), np, de.as<double>(),
                    dv.as<double>(), dc.as<double>(), dpv.as<double>()));
    GMAT_HIP(hipMemcpy(eff + t0, de.p, np * 8, hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(var + t0, dv.p, np * 8, hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(chi + t0, dc.p, np * 8, hipMemcpyDeviceToHost));
    GMAT_HIP(hipMemcpy(p + t0, dpv.p, np * 8, hipMemcpyDeviceToHost));
  }
  return GMAT_OK;
}

// ------------------------------------------------------------------ exhaustive mode
// Every pair of the listed rows refined exactly, no screen: the reference's computation
// (remma_epiAA.py:71-82, remma_epiAD.py:68-80, remma_epiDD.py:68-79) on refine_kernel.  It audits
// the certified screens (a screened scan must return the same hits, byte for byte: the refine of
// a pair does not depend on the list it comes in) and is the fallback when no screen is wanted.



// ------------------------------------------------------------------ bound audit (diagnostic)
// The certified lower bounds of e'Pe the screens test with, evaluated exactly (fp64, no screen
// arithmetic) for listed pairs, e = (a - alpha)(b - beta) of the screen codes over the real
// individuals: the prefilter's mu |e|^2 - (mu + tau)(1'e)^2/n - ku |U'e|^2 - eps |e|^2 and the
// low-rank screen's lam |Pi e|^2 - tau (1'e)^2/n - eps |e|^2 - |Q'e|^2 (Q = the certified fp6 basis).
// The caller compares them with the exact e'Pe (gmat_epi_pairs): every ratio must be >= 1.
// One workgroup per pair; out[5 t + ..] = {lb_prefilter, lb_lowrank, |e|^2, 1'e, |Q'e|^2}.

extern "C" int gmat_epi_audit(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *out5) {
  GMAT_CHECK(e && (n_pairs == 0 || (pairs && out5)), GMAT_E_ARG, "gmat_epi_audit: bad arguments");
  GMAT_CHECK(kind >= 0 && kind <= 2, GMAT_E_ARG, "gmat_epi_audit: bad kind");
  if (n_pairs == 0) return GMAT_OK;
  if (e->seg) return seg_audit(e, kind, pairs, n_pairs, out5);
  int lc, rc;
  kind_codings(kind, &lc, &rc);
  GMAT_TRY(build_coding(e, lc));
  GMAT_TRY(build_coding(e, rc));
  for (int64_t t = 0; t < n_pairs; ++t)
    GMAT_CHECK(pairs[2 * t] >= 0 && pairs[2 * t] < e->m && pairs[2 * t + 1] >= 0 && pairs[2 * t + 1] < e->m,
               GMAT_E_ARG, "pair %lld out of range", (long long)t);
  std::vector<int64_t> hi(n_pairs), hj(n_pairs);
  for (int64_t t = 0; t < n_pairs; ++t) {
    hi[t] = pairs[2 * t];
    hj[t] = pairs[2 * t + 1];
  }
  DBuf di, dj, dout;
  GMAT_TRY(di.alloc(n_pairs * 8));
  GMAT_TRY(dj.alloc(n_pairs * 8));
  GMAT_TRY(dout.alloc(n_pairs * 5 * 8));
  GMAT_HIP(hipMemcpy(di.p, hi.data(), n_pairs * 8, hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dj.p, hj.data(), n_pairs * 8, hipMemcpyHostToDevice));
  const int R = e->lr_R > 0 && e->lr_Bs.p ? e->lr_R : 0;
  GMAT_CHECK(R <= AUD_T, GMAT_E_ARG, "gmat_epi_audit: rank %d > %d", R, AUD_T);
  hipLaunchKernelGGL(audit_kernel, dim3((unsigned)n_pairs), dim3(AUD_T), 0, e->s, e->n, e->n_pad, R, e->pf_ncov,
                     screen_panel(e, lc), screen_panel(e, rc), e->code[lc].soff.as<double>(),
                     e->code[rc].soff.as<double>(), di.as<int64_t>(), dj.as<int64_t>(), e->lr_Bs.as<double>(),
                     e->pf_U.as<double>(), e->pf_mu, e->pf_tau, e->pf_eps, e->pf_ku, e->lr_lam, e->lr_tau, e->lr_eps,
                     dout.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpyAsync(out5, dout.p, n_pairs * 5 * 8, hipMemcpyDeviceToHost, e->s));
  GMAT_HIP(hipStreamSynchronize(e->s));
  return GMAT_OK;
}

/*
 * gmat_hip.h -- C ABI of libgmat_hip.so, the MI355X (gfx950) implementation of GMAT's
 * dense-linear-algebra hot path.  Plain pointers and sizes only; every function returns
 * GMAT_OK (0) or a negative GMAT_E_* code and never exits the process (the reference's C
 * code calls exit(1) on I/O errors: _remma_epi_eff_cpu.c:19-20,116-117).  The message of
 * the last failure on the calling thread is available from gmat_last_error().
 *
 * Host arrays are row-major.  Genotype input is the body of a PLINK .bed file (the bytes
 * after the 3-byte magic), SNP-major, ceil(n_id/4) bytes per SNP, decoded with the
 * reference's convention (process_plink/_read_plink_bed.c:37): code 00->0, 10->1, 11->2,
 * 01->missing.
 *
 * Which reference interface each entry point replaces is noted per function; the
 * Python host layer (gmat_amd/) keeps the reference's Python signatures on top of it.
 */
#ifndef GMAT_HIP_H
#define GMAT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  GMAT_OK = 0,
  GMAT_E_ARG = -1,      /* invalid argument */
  GMAT_E_HIP = -2,      /* HIP runtime error */
  GMAT_E_NOMEM = -3,    /* device allocation failed */
  GMAT_E_NOTPD = -4,    /* matrix not positive definite */
  GMAT_E_OVERFLOW = -5, /* an output buffer was too small (see the *_needed argument) */
  GMAT_E_STATE = -6     /* call sequence error */
};

enum { GMAT_AA = 0, GMAT_AD = 1, GMAT_DD = 2 };         /* epistasis kinds */
enum { GMAT_GRM_ADD = 0, GMAT_GRM_DOM = 1 };             /* relationship matrices */

const char *gmat_last_error(void);
int gmat_version(void);
int gmat_device_count(int *n);
int gmat_set_device(int device);
/* wait for all work queued by this process on the current device (hipDeviceSynchronize) */
int gmat_device_synchronize(void);
/* device memory freed by the library stays cached for reuse (up to GMAT_POOL_MAX_GB, default 64);
 * this returns every cached block to the device */
int gmat_empty_cache(void);

/* ---------------------------------------------------------------- genotype panel
 * Uploads the packed .bed body once and decodes it on the device into SNP-major int8
 * panels (dosage and heterozygote indicator).  Replaces the decode done by
 * read_plink (process_plink.py:7-9 / pandas_plink) and read_plink_bed
 * (_read_plink_bed.c:5-51) for every consumer below.  Missing genotypes must have been
 * imputed by the caller (as gmatrix.py:47-49 / remma_epiAA.py:57-59 do); a panel that
 * still contains missing codes is rejected by the consumers. */
typedef struct gmat_geno gmat_geno;
int gmat_geno_create(gmat_geno **out, const uint8_t *bed_body, int64_t body_bytes, int64_t n_id,
                     int64_t n_snp);
/* per-SNP sum of dosages, heterozygote count and missing count (each n_snp long; any may be NULL) */
int gmat_geno_counts(const gmat_geno *g, int64_t *sum_dose, int64_t *n_het, int64_t *n_miss);
int gmat_geno_destroy(gmat_geno *g);

/* ---------------------------------------------------------------- relationship matrices
 * kin (n_id x n_id, host) = additive GRM of agmat (gmatrix.py:52-66) for GMAT_GRM_ADD or the
 * dominance GRM of dgmat_as (gmatrix.py:115-130) for GMAT_GRM_DOM, diagonal scaled by
 * (1 + small_val).  *scale_out receives the scale factor. */
int gmat_grm(gmat_geno *g, int kind, double small_val, double *kin, double *scale_out);
/* last gmat_grm call: [0] seconds of the product (fp4 fragment images + the block-scaled fp4 MFMA
 * SYRK), [1] fp4 MFMA ops it issued, [2] dense-equivalent flop 2 n^2 m, [3] seconds of every kernel
 * of the call (row sums, product, centring epilogue) */
int gmat_grm_stats(double *out4);

/* ainv = a^-1 for a symmetric positive-definite n x n matrix (scipy.linalg.inv at
 * gmatrix.py:84); *logdet = log|a| (may be NULL). */
int gmat_spd_inverse(int64_t n, const double *a, double *ainv, double *logdet);

/* ---------------------------------------------------------------- REML
 * Weighted EM-AI REML of _wemai_multi_gmat (uvlmm_varcom.py:8-104).  z_col[r] is the
 * individual (column of Z) of record r; gmat[k] points to an n_id x n_id matrix.
 * var_out has n_gmat+1 entries (residual last); history (may be NULL) receives maxiter x
 * (n_gmat+1) values (the variances after each iteration). */
int gmat_reml(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y,
              const double *xmat, const int64_t *z_col, const double *const *gmat, const double *init,
              int maxiter, double cc_par, double cc_gra, double *var_out, int *n_iter, double *history);

/* last gmat_reml call on this process: [0] seconds (setup + iterations), [1] iterations,
 * [2] seconds per iteration, [3] algorithmic flop per iteration (n^3/3 potrf + 2n^3/3 inverse
 * + 2n^2(2c+1) traces / AI) */
int gmat_reml_stats(double *out4);

/* per iteration of the last gmat_reml call on this process (the quantities the reference logs,
 * uvlmm_varcom.py:90-96): norm of the gradient vector, norm of the update vector, and the EM weight
 * the step used; up to cap values each into the non-NULL arrays, *count = iterations run. */
int gmat_reml_trace(int cap, double *grad_norm, double *update_norm, double *em_weight, int *count);

/* pvp = Z'PZ (n_id x n_id) and py = Z'Py (n_id) of the scans' setup (remma_epiAA.py:33-49). */
int gmat_projection(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y,
                    const double *xmat, const int64_t *z_col, const double *const *gmat,
                    const double *var_com, double *pvp, double *py);

/* ---------------------------------------------------------------- epistasis scans
 * A scan plan keeps the genotype panel, P (= Z'PZ) and Py resident in HBM. */
typedef struct gmat_epi gmat_epi;
/* n_slice (1..4): int8 slices of P (off the diagonal) kept for the screen (see gmat_epi_scan). */
int gmat_epi_create(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice);
/* Multi-GPU: the plan's spectral state (P's covariate directions, the certified prefilter and
 * low-rank bounds, the low-rank basis' tile images) computed once and shared.  gmat_epi_export
 * writes it to buf (cap bytes; *needed = its size, buf may be NULL to query); gmat_epi_create_with
 * builds a plan for the same P from it (checked against a fingerprint of P) instead of
 * recomputing the eigendecomposition and the certificate searches. */
int gmat_epi_export(const gmat_epi *e, uint8_t *buf, int64_t cap, int64_t *needed);
int gmat_epi_create_with(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                         const uint8_t *state, int64_t state_bytes);
/* Exhaustive exact scan over first-SNP rows `rows` (sorted ascending): AA/DD test pairs
 * (i, j>i) (remma_epiAA.py:71-82, remma_epiDD.py:75-86), AD tests (i, all j) including i==j
 * (remma_epiAD.py:76-87).  A pair is a hit when p < p_cut with p = chi2.sf(eff^2/var, 1);
 * chi_cut must be chi2.isf(p_cut, 1).  n_slice selects the certified screen in front of the exact
 * fp64 refine: 0 = automatic (the low-rank spectral screen when the plan has one and p_cut <= 1e-4,
 * else int8 slices of P: 2 up to p_cut 1e-2, then all kept), S > 0 = S int8 slices, -1 = the fp6
 * quadratic form, -2 = the low-rank screen, GMAT_SCREEN_NONE = no screen (every pair refined, the
 * reference's computation; audits the screens).  A launch whose candidates overflow is redone one
 * level finer.  The hit set and its numbers do not depend on the level.  *n_hits receives the
 * number of hits, retrieved with gmat_epi_hits (sorted by (i, j)). */
#define GMAT_SCREEN_NONE (-9)
int gmat_epi_scan(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut,
                  int n_slice, int64_t *n_hits);
int gmat_epi_hits(gmat_epi *e, int64_t cap, int64_t *i, int64_t *j, double *eff, double *var, double *chi,
                  double *p);
/* Exact statistics of an explicit pair list (remma_epiAA_pair.py:79-84 and siblings). */
int gmat_epi_pairs(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *eff, double *var,
                   double *chi, double *p);
/* counters of the last scan: [0] pairs tested, [1] candidates refined, [2] int8 MFMA ops,
 * [3] screen kernel seconds, [4] refine kernel seconds, [5] side-term kernel seconds,
 * [6] total seconds, [7] screen kernel launches, [8] screen level (-1 low-rank, 0 MX, k int8 slices),
 * [9] bound coefficient */
int gmat_epi_stats(const gmat_epi *e, double *out10);
/* per-kernel accounting of the last scan at the low-rank level (compacted path): [0] prefilter kernel
 * seconds (HIP events on its stream), [1] its launches, [2] its MFMA ops in fp4-equivalents (fp4 ops +
 * 2 x int8 ops), [3] low-rank screen seconds, [4] its launches, [5] its fp6 x fp4 ops, [6] pair screen
 * + refine seconds at flush, [7] pairs kept by the prefilter (GMAT_LIVE_COUNT set) or -1 */
int gmat_epi_kernel_stats(const gmat_epi *e, double *out8);
/* the candidate kernels of the last scan, timed with HIP events on their streams: per kernel
 * (pair_side, pair_mx, refine, refine_side) seconds, launches and pairs, in that order; up to cap
 * values, *count = 12 */
int gmat_epi_kernel_stats_ext(const gmat_epi *e, double *out, int cap, int *count);
/* Diagnostic: the certified lower bounds of e'Pe that the screens test with, evaluated exactly in
 * fp64 for listed pairs (i, j) (e = the screen codes' centred product over the real individuals):
 * out5[5 t ..] = {prefilter bound, low-rank bound, |e|^2, 1'e, |Q'e|^2} (-inf where the plan has no
 * such screen).  Compared with the exact e'Pe of gmat_epi_pairs, every ratio must be >= 1. */
int gmat_epi_audit(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *out5);
/* screen certificates of the plan: [0] rank of the low-rank spectral screen (padded to 128; 0 =
 * none, scans use the fp6 quadratic form), [1] its lam, [2] the prefilter's mu, [3] n_pad; the
 * compacted scan's prefilter (prefilter_pass_kernel): [4] tile rows, [5] tile columns, [6] bytes one
 * tile streams into LDS by LDS-DMA per 64-individual stage, [7] bytes of a tile's test records.  In
 * gmat_epi_stats, [8] = -1 marks a scan screened by the low-rank bound. */
int gmat_epi_info(const gmat_epi *e, double *out8);
/* plan setup seconds: [0] gmat_epi_create total, [1] prefilter certificate, [2] eigendecomposition
 * of P, [3] low-rank certificate, [4] slices and residual bounds, [5] coding builds (side vectors;
 * done lazily by the first scan of each coding), [6] Cholesky factorisations the certificates ran,
 * [7] covariate directions in the prefilter certificate (null directions of P besides 1) */
int gmat_epi_setup_stats(const gmat_epi *e, double *out8);
/* how the plan holds its panel: [0] SNP segments (1: one plan; more when 2 n_snp n_pad would reach
 * 2^32 bytes, or GMAT_SEG_SNPS asks for them: scans run on sub-plans of one or two segments), [1]
 * SNPs per segment, [2] 1 when the plan has no screens (n_pad > 8,192: every pair refined exactly),
 * [3] n_snp */
int gmat_epi_layout(const gmat_epi *e, int64_t *out4);
int gmat_epi_destroy(gmat_epi *e);

/* Random-effect prediction of wemai_multi_gmat_pred (uvlmm_varcom.py:147-166) at var_com, as
 * the reference computes it (its projection uses V, not V^-1: vxmat = V X, pmat = V -
 * VX (X'VX)^-1 X'V).  rand_eff[a * n_gmat + k] = (G_k Z' pmat y)[a] * var_com[k]. */
int gmat_blup(int64_t n_rec, int64_t n_fix, int64_t n_id, int n_gmat, const double *y, const double *xmat,
              const int64_t *z_col, const double *const *gmat, const double *var_com, double *rand_eff);

/* ---- effect-only screen (the approximate pipeline's first pass) ----
 * Replaces the OpenMP row loops of _remma_epi_eff_cpu.c (AA :61-137, AA maf :141-219,
 * AD :226-314, AD maf :318-410, DD :415-496, DD maf :500-574).  eff(i, j) =
 * sum_k x_ik x_jk py_k with the reference's fp64 codings and centring (freq accumulated as
 * the reference does, missing = 1/3) for j > i over the listed first SNPs `rows` (in list
 * order), keeping |eff| > cut (AD: >= for (i, j), > for (j, i)).  cut = eff_cut[0] when
 * freq_i is NULL, else eff_cut[freq_i[i]*10 + freq_j[j]] (111 entries; freq values 0..10;
 * AA/DD pass the same array twice, AD passes freqA, freqD).  Writes out_file: header
 * "snp_0 snp_1 eff" then "%lld %lld %g" rows (rows in list order, j ascending, AD (i, j)
 * before (j, i)); py is Z'Py in .fam order. */
int gmat_eff_scan(gmat_geno *g, int kind, const double *py, const int64_t *rows, int64_t n_rows,
                  const double *eff_cut, const int64_t *freq_i, const int64_t *freq_j, const char *out_file,
                  int64_t *n_hits);
/* Last gmat_eff_scan on this process: pairs tested, hits, device seconds, text-writing seconds. */
int gmat_eff_stats(double *out4);
/* ---- relationship-matrix text output (gmatrix.py:10-31), multi-threaded ----
 * fmt 0 'mat': np.savetxt layout ("%.18e", ' ', '\n'); fmt 1 'row_col_val' and fmt 2
 * 'id_id_val': lower triangle row by row, "<row> <col> <value>" with 1-based indices or the
 * ids (ids_blob: n NUL-terminated strings back to back) and the value as CPython
 * repr(float), as pandas to_csv writes it.  n_threads <= 0: up to 16. */
int gmat_write_grm_text(const char *path, const double *mat, int64_t n, int fmt, const char *ids_blob, int n_threads);
/* CPython repr(float) of v (the value text of fmt 1/2); returns its length (cap >= 32). */
int gmat_float_repr(double v, char *out, int cap);
/* Append n scan result rows "i j v_0 .. v_{nf-1}\n" (1 <= nf <= 4 value columns f0..f3, CPython
 * float repr) to the file at path: the reference's DataFrame.to_csv rows (remma_epiAA.py:84-86). */
int gmat_append_hit_rows(const char *path, int64_t n, const int64_t *i, const int64_t *j, int nf, const double *f0,
                         const double *f1, const double *f2, const double *f3);

/* ---- single-SNP tests (remma_add / remma_dom) ----
 * For every SNP j of the (imputed) panel: x_j = g_j - 2p_j (kind GMAT_GRM_ADD) or
 * [g_j != 2] g_j - 2p_j(1-p_j) (GMAT_GRM_DOM), p_j = sum/(2n); xpy[j] = x_j' py and
 * xpx[j] = x_j' P x_j with P (pvp, n x n) and py in .fam order.  Replaces the two dense
 * products of remma_add.py:58-59 / remma_dom.py:60-61; the scaling by var_com and the
 * chi2 test stay on the host. */
int gmat_snp_test(gmat_geno *g, int kind, const double *pvp, const double *py, double *xpy, double *xpx);
/* Decoded fp64 dosage (m x n, SNP-major, .fam order; (c^2+c)/6: missing = 1/3) -- the
 * reference's read_plink_bed (_read_plink_bed.c:5-51). */
int gmat_geno_decode(const gmat_geno *g, double *marker_mat);

/* ---- multi-GPU exchange (RCCL over xGMI; one process per GPU) ----
 * The sharded scans need one-off exchanges only: the all-gather of the packed
 * genotype shards, the broadcast of P / Py from rank 0 and the gather of the hit records (the
 * reference runs separate parallel=[N,k] processes that each write out_file.k,
 * remma_epiAA.py:109-161).  Host buffers in and out; every call returns when its result is on
 * the host.  Rank 0 creates the 128-byte unique id, the launcher shares it (gmat_amd/dist.py). */
typedef struct gmat_comm gmat_comm;
int gmat_comm_unique_id(uint8_t *out128);
int gmat_comm_init(gmat_comm **out, int nranks, int rank, const uint8_t *id128);
int gmat_comm_destroy(gmat_comm *c);
/* recv (nranks x bytes, rank order) = every rank's send (bytes) */
int gmat_comm_allgather(gmat_comm *c, const void *send, void *recv, int64_t bytes);
/* buf (bytes) from root to every rank, in place */
int gmat_comm_broadcast(gmat_comm *c, void *buf, int64_t bytes, int root);
/* in place over ranks: op 0 = sum, 1 = max (fp64) */
int gmat_comm_allreduce_f64(gmat_comm *c, double *v, int64_t count, int op);
/* variable-length byte records to root: counts[nranks] on every rank; root's recv gets the payloads
 * back to back in rank order.  When root's recv_cap is too small every rank returns GMAT_E_OVERFLOW
 * (with *needed) before any send is posted (the check is collective). */
int gmat_comm_gatherv(gmat_comm *c, const void *send, int64_t bytes, int root, int64_t *counts, void *recv,
                      int64_t recv_cap, int64_t *needed);
int gmat_comm_barrier(gmat_comm *c);

/* ---- diagnostics ----
 * The low-rank screen's accumulation (lr_screen_kernel) on one wave: a chain of n_steps
 * v_mfma_scale_f32_32x32x64_f8f6f4 (A fp6 e2m3 codes[n_steps][32 rows][2 halves][32] with e8m0
 * scales[n_steps][32][2], one per (row, half); B = the screen's worst case w = 4 everywhere)
 * accumulated in fp32; out[32 x 32] (every column = 4 sum_k A[r][k]).  Lets tests check the
 * screen's fp32 accumulation bound (eta_r) on the hardware. */
int gmat_probe_mx_accum(int n_steps, const uint8_t *codes, const uint8_t *scales, float *out);
/* The scan plan's partial symmetric eigensolver on a host matrix (n x n, symmetric): the ne
 * smallest Ritz values ascending to w_out, Ritz vector r to z_out[r*n .. r*n+n), iterating until
 * every residual is <= tol x the Gershgorin bound of |a| or maxit block iterations; res_out (ne
 * residual norms) and iters_out may be NULL.  Test support. */
int gmat_probe_eig_bottom(int64_t n, const double *a_host, int ne, double tol, int maxit, double *w_out,
                          double *z_out, double *res_out, int *iters_out);

#ifdef __cplusplus
}
#endif
#endif /* GMAT_HIP_H */

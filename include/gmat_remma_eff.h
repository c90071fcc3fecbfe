/*
 * gmat_remma_eff.h -- drop-in exports with the exact prototypes of the reference's cffi
 * modules _cremma_epi_eff_cpu (gmat/remma/_build.py:8-53) and _cread_plink_bed
 * (gmat/process_plink/_build.py:8-14), implemented on the GPU by libgmat_hip.so.
 *
 * File semantics follow the reference: bed_file is the PLINK prefix (".bed" is appended),
 * out_file receives "snp_0 snp_1 eff" and "%lld %lld %g" rows.  Differences, by design:
 * the .bed magic and size are checked; rows come out in list order (the reference's
 * OpenMP order is nondeterministic); errors return a negative GMAT_E_* code with the text
 * in gmat_last_error() instead of exit(1); no progress bar is printed.  Success returns 1
 * like the reference.
 */
#ifndef GMAT_REMMA_EFF_H
#define GMAT_REMMA_EFF_H

#ifdef __cplusplus
extern "C" {
#endif

/* _read_plink_bed.c:5-51 (copy at _remma_epi_eff_cpu.c:10-56): marker_mat[snp*num_id + id]. */
int read_plink_bed(char *bed_file, long long num_id, long long num_snp, double *marker_mat);

/* _remma_epi_eff_cpu.c:91-137 */
int remma_epiAA_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                        long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file);
/* _remma_epi_eff_cpu.c:171-219 */
int remma_epiAA_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                            long long len_snp_lst_0, double *pymat, long long *freq, double *eff_cut,
                            char *out_file);
/* _remma_epi_eff_cpu.c:260-314 */
int remma_epiAD_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                        long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file);
/* _remma_epi_eff_cpu.c:354-410 */
int remma_epiAD_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                            long long len_snp_lst_0, double *pymat, long long *freqA, long long *freqD,
                            double *eff_cut, char *out_file);
/* _remma_epi_eff_cpu.c:443-496 */
int remma_epiDD_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                        long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file);
/* _remma_epi_eff_cpu.c:526-574 */
int remma_epiDD_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                            long long len_snp_lst_0, double *pymat, long long *freq, double *eff_cut,
                            char *out_file);

#ifdef __cplusplus
}
#endif
#endif /* GMAT_REMMA_EFF_H */

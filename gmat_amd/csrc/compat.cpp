// Drop-in exports with the reference's cffi prototypes (include/gmat_remma_eff.h): each
// reads <bed_file>.bed, uploads it as a genotype panel and runs the device effect screen
// (gmat_eff_scan) or decoder (gmat_geno_decode).
#include <cstdio>
#include <vector>

#include "../../include/gmat_remma_eff.h"
#include "common.h"

namespace {

// The .bed body (after the 3-byte magic) of <prefix>.bed, checked for magic and size.
int read_bed_body(const char *prefix, long long num_id, long long num_snp, std::vector<uint8_t> *body) {
  GMAT_CHECK(prefix && num_id > 0 && num_snp > 0, GMAT_E_ARG, "bad arguments");
  std::string path = std::string(prefix) + ".bed";
  FILE *f = fopen(path.c_str(), "rb");
  GMAT_CHECK(f, GMAT_E_ARG, "Fail to open the plink bed file: %s.", path.c_str());
  unsigned char magic[3] = {0, 0, 0};
  const size_t got = fread(magic, 1, 3, f);
  const long long nb = (num_id + 3) / 4;
  body->resize((size_t)(nb * num_snp));
  const size_t want = body->size();
  const size_t read = got == 3 ? fread(body->data(), 1, want, f) : 0;
  fclose(f);
  GMAT_CHECK(got == 3 && magic[0] == 0x6c && magic[1] == 0x1b && magic[2] == 0x01, GMAT_E_ARG,
             "%s is not a SNP-major PLINK .bed file", path.c_str());
  GMAT_CHECK(read == want, GMAT_E_ARG, "%s: %zu body bytes, %lld SNPs x %lld individuals need %zu", path.c_str(),
             read, num_snp, num_id, want);
  return GMAT_OK;
}

int eff_entry(const char *name, int kind, char *bed_file, long long num_id, long long num_snp, long long *rows,
              long long n_rows, double *py, const double *cut, const long long *fi, const long long *fj,
              char *out_file) {
  std::vector<uint8_t> body;
  int rc = read_bed_body(bed_file, num_id, num_snp, &body);
  gmat_geno *g = nullptr;
  if (rc == GMAT_OK) rc = gmat_geno_create(&g, body.data(), (int64_t)body.size(), num_id, num_snp);
  if (rc == GMAT_OK) {
    static_assert(sizeof(long long) == sizeof(int64_t), "long long is 64-bit");
    int64_t hits = 0;
    rc = gmat_eff_scan(g, kind, py, (const int64_t *)rows, n_rows, cut, (const int64_t *)fi, (const int64_t *)fj,
                       out_file, &hits);
  }
  if (g) gmat_geno_destroy(g);
  if (rc != GMAT_OK) {
    fprintf(stderr, "%s: %s\n", name, gmat_last_error());
    return rc;
  }
  return 1;
}

}  // namespace

extern "C" int read_plink_bed(char *bed_file, long long num_id, long long num_snp, double *marker_mat) {
  std::vector<uint8_t> body;
  int rc = read_bed_body(bed_file, num_id, num_snp, &body);
  gmat_geno *g = nullptr;
  if (rc == GMAT_OK) rc = gmat_geno_create(&g, body.data(), (int64_t)body.size(), num_id, num_snp);
  if (rc == GMAT_OK) rc = gmat_geno_decode(g, marker_mat);
  if (g) gmat_geno_destroy(g);
  if (rc != GMAT_OK) {
    fprintf(stderr, "read_plink_bed: %s\n", gmat_last_error());
    return rc;
  }
  return 1;
}

extern "C" int remma_epiAA_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                   long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file) {
  return eff_entry("remma_epiAA_eff_cpu", GMAT_AA, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   &eff_cut, nullptr, nullptr, out_file);
}

extern "C" int remma_epiAA_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                       long long len_snp_lst_0, double *pymat, long long *freq, double *eff_cut,
                                       char *out_file) {
  return eff_entry("remma_epiAA_maf_eff_cpu", GMAT_AA, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   eff_cut, freq, freq, out_file);
}

extern "C" int remma_epiAD_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                   long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file) {
  return eff_entry("remma_epiAD_eff_cpu", GMAT_AD, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   &eff_cut, nullptr, nullptr, out_file);
}

extern "C" int remma_epiAD_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                       long long len_snp_lst_0, double *pymat, long long *freqA, long long *freqD,
                                       double *eff_cut, char *out_file) {
  return eff_entry("remma_epiAD_maf_eff_cpu", GMAT_AD, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   eff_cut, freqA, freqD, out_file);
}

extern "C" int remma_epiDD_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                   long long len_snp_lst_0, double *pymat, double eff_cut, char *out_file) {
  return eff_entry("remma_epiDD_eff_cpu", GMAT_DD, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   &eff_cut, nullptr, nullptr, out_file);
}

extern "C" int remma_epiDD_maf_eff_cpu(char *bed_file, long long num_id, long long num_snp, long long *snp_lst_0,
                                       long long len_snp_lst_0, double *pymat, long long *freq, double *eff_cut,
                                       char *out_file) {
  return eff_entry("remma_epiDD_maf_eff_cpu", GMAT_DD, bed_file, num_id, num_snp, snp_lst_0, len_snp_lst_0, pymat,
                   eff_cut, freq, freq, out_file);
}

// Device-resident genotype panel (internal definition of the opaque gmat_geno handle).
#pragma once
#include "common.h"

// Individuals are stored in 32-blocks with the within-block order of perm_nat(): storage
// slot q of a block holds natural individual perm_nat(q).  This puts, in every lane of a
// v_mfma_i32_32x32x32_i8 B fragment, exactly the 16 individuals whose accumulator rows the
// same lane owns (rows (r&3) + 8(r>>2) + 4(lane>>5)), so the scan's epilogue weights come
// from the same contiguous 16 bytes (see epi.hip).  Every consumer of the panels works
// in this order; P and Py are permuted identically when a scan plan is built.
__host__ __device__ inline int perm_nat(int q) { return (q & 3) + 8 * ((q & 15) >> 2) + 4 * (q >> 4); }

struct gmat_geno {
  int64_t n = 0, m = 0;  // individuals, SNPs
  int64_t n_pad = 0;     // individuals padded to a multiple of 256 (zero genotypes)
  int64_t nb = 0;        // packed bytes per SNP (ceil(n/4))
  gmat::DBuf packed;     // m * nb, PLINK order
  gmat::DBuf panels;     // int8 [2][m][n_pad]: dosage 0/1/2 (missing stored as 0), then the
                         // heterozygote indicator; individuals in storage order
  int8_t *dose_ptr() const { return panels.as<int8_t>(); }
  int8_t *het_ptr() const { return panels.as<int8_t>() + m * n_pad; }
  std::vector<int64_t> sum_dose, n_het, n_miss;
  int64_t total_missing = 0;
};

// A panel of the SNP ranges [lo[r], hi[r]) of g, in that order (device copies of the dosage and
// heterozygote rows, the per-SNP counts): the sub-panels of a segmented scan plan (epi_seg.hip).  The
// packed .bed rows are not copied (the scans never read them).
int geno_subset(const gmat_geno *g, const int64_t *lo, const int64_t *hi, int nr, gmat_geno **out);

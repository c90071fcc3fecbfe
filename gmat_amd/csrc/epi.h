// Internal interface of the exhaustive epistasis scans (remma_epiAA.py:71-82, remma_epiAD.py:76-87,
// remma_epiDD.py:75-86) and the pair-list test (remma_epiAA_pair.py:79-84), shared by the stage files:
//   epi_prefilter.hip  spectral prefilter (prefilter_pass_kernel, prefilter_cov_kernel, side GEMMs)
//   epi_screen.hip     int8 / MX / low-rank screens and the device-built tile and slot lists
//   epi_refine.hip     exact refine (int8 slices, fp64), pair screen, hit compaction
//   epi_setup.hip      plan-setup and coding kernels (P slices, tile images, code panels, records)
//   epi_plan.hip       the plan: codings, certificates, spectral state, refine / pair-screen drivers
//   epi_scan.hip       the scans (exhaustive, compacted low-rank, block-granular) and their C API
//   epi_seg.hip        plans past the single-plan size limits (SNP segments, exhaustive-only plans)
//
// For a pair (i, j) with centred codes x_i = a_i - alpha_i, x_j = b_j - beta_j (a, b the
// integer 0/1/2 dosage or 0/1 heterozygote codes), the reference computes
//     e = x_i o x_j,  eff = e'Py,  var = e'Pe  (2n^2 fp64 flop per pair),
// chi = eff^2/var, p = chi2.sf(chi, 1), and keeps p < p_cut.
//
// Here the scan runs in two passes:
//  1. SCREEN.  The screen codes count the MINOR allele (a~ = 2 - a when 2p > 1, which only
//     flips the sign of x and leaves e'Pe unchanged), so w = a~_i o b~_j (integers 0..4)
//     stays small.  Every pair passes through a cascade of certified lower bounds of e'Pe
//     (DESIGN.md 5.3): a pair is dropped only when its p-value provably is >= p_cut.
//  2. REFINE.  Candidates are re-evaluated exactly as the reference does (var = e'Pe from
//     seven int8 slices of P with exact integer sums plus fp64 O(n) terms, eff = e'Py in fp64,
//     p = erfc(sqrt(chi/2))) and the hits are kept.
// The reported statistics therefore come from the reference's formula; the screens only decide
// which pairs need it.
#pragma once
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "dla.h"
#include "geno.h"

namespace gmat {
namespace epi {


typedef int v2i_ __attribute__((ext_vector_type(2)));
typedef int v8i_ __attribute__((ext_vector_type(8)));
typedef float v16f_ __attribute__((ext_vector_type(16)));
typedef float v2f_ __attribute__((ext_vector_type(2)));

constexpr int LK = 64;   // inner (individual) depth per LDS stage
constexpr int AP = 80;   // LDS pitch of a 64-byte row (conflict-free ds_read_b128)
constexpr int BJ = 32;   // second-SNP columns per screen tile
constexpr int ROWS_PER_LAUNCH = 512;       // first SNPs per launch of the block-granular scan
constexpr int LRC_ROWS_PER_LAUNCH = 7168;  // ... and of the compacted low-rank scan
constexpr int SIDE_T = 3;        // int8 slices of the O(n)-per-pair side vectors (21 bits)
constexpr int E3_PF = 2;         // L3 slices of the prefilter pass (eff to ~2^-14: enough to screen)
constexpr int SIDE_P = 3;        // left side-vector parts per band row: L', L3, Ld
constexpr int SCREEN_SHAPE = 0;  // default tile shape of the screen kernel (Shape<SH> below)

// w = a*b via one v_perm_b32 per 4 bytes: the i-side byte holds o(a) = {0,2,5}[a], the
// j-side byte b in {0,1,2}; T[o(a)+b] = a*b with T = {0,0,0,1,2,0,2,4}.  Off-diagonal
// blocks of the symmetric quadratic form count twice: table 2T.
constexpr unsigned T_LO = 0x01000000u, T_HI = 0x04020002u;
constexpr unsigned T2_LO = 0x02000000u, T2_HI = 0x08040004u;

__device__ __forceinline__ unsigned to_offset(unsigned v) { return (v << 1) + ((v >> 1) & 0x7f7f7f7fu); }

struct ScreenArgs {
  const int8_t *slices;
  int64_t slices_bytes;
  const int8_t *panels;  // dosage then heterozygote panels, one allocation
  int64_t panels_bytes, left_off, right_off;
  int64_t n_pad;
  int n_slice;
  const int8_t *left, *right;  // panels [m][n_pad]
  int64_t m;
  const int64_t *rows;
  int n_rows;
  const int *tiles;  // (row offset, J) pairs; MX screens: (row-list index, J)
  const int *tile_rows;  // MX screens: MX_BI band rows per tile (-1 = none)
  const int *tile_side;  // MX screens: per tile [3][SIDE_T][MX_TS] E1 / Ed / E2 slice products
  int tri;           // 1: only j > i
  // side terms as int32 products of int8 slices (SIDE_T slices, slice stride in elements):
  // E1 = sL[i] sum_t 128^-t c13[t][ri], E3 = sL3[i] sum_t 128^-t c13[t][R+ri],
  // Ed = sLd[i] sum_t 128^-t c13[t][2R+ri] (= sum_q P_qq a_q^2 b_q^2),
  // E2 = sR[j] sum_t 128^-t c2[t][ri]; slicing error bounds side_eps * scale * code sum
  const int *c13, *c2;
  int64_t c13_stride, c2_stride;
  const double *sL, *sL3, *sLd, *sR, *csum_l, *csum_r, *csq_l, *csq_r;
  double side_eps;
  int e3_t;       // slices of E3 in c13 (E3_PF from the prefilter pass, SIDE_T from the full side path)
  double e3_eps;  // their slicing bound (as side_eps)
  int64_t ld_e, j_lo;
  const double *alpha, *qa, *ra, *sa;
  const double *beta, *qb, *rb, *sb;
  const uint8_t *mono_l, *mono_r;
  double zz, spy, scale_main, delta, chi_cut;
  unsigned long long *counter;
  int64_t cap;
  int64_t *cand_i, *cand_j;
  // spectral prefilter: exact code products Sab, Sa2b, Sab2, Sa2b2 ([4][R][ld_e] int32, z-stride
  // pfc_stride), the certificate (pf_mu, pf_eps), n, and per (band row, 32-column block) flags
  const int *pfc;
  int64_t pfc_stride;
  double pf_mu, pf_tau, pf_eps, n_id;
  uint8_t *flags;
  int nJ;
  int pf_store;  // side pass 1 also writes the code products of flagged blocks to pfc
  // covariate directions of the prefilter certificate (P's null space besides 1, pf_ncov of them):
  // direction k quantised to int8 q_k = rint(u_k / pf_sq[k]) (SideArgs qimg); pf_ua[k][i] = u_k . a_i
  // (left screen codes), pf_ub[k][j] = u_k . b_j (right); pf_su[k] = 1'u_k; the certificate's
  // coefficient of |U'e|^2 is pf_ku
  const double *pf_ua, *pf_ub;
  double pf_sq[4], pf_su[4];
  double pf_ku;
  int pf_ncov;
  unsigned long long *live_count;  // diagnostics (GMAT_LIVE_COUNT): pairs the prefilter keeps, or null
  unsigned long long *pf_stamp;    // diagnostics (GMAT_PF_STAMPS): 4 s_memrealtime stamps per workgroup, or null
  // compacted low-rank path, per (band row, 32-column block) with a live pair: one 64-bit entry (lm_*)
  // {live mask (bit c = column 32 J + c), index of the block's first record, launch tag}, or null.  Only
  // live blocks are written; a reader takes an entry whose tag is not ltag as an empty block, so the
  // entries need no clearing between launches (the host zeroes a buffer set once per 63 launches)
  uint64_t *lmask;
  unsigned ltag;
  // compacted low-rank path: the live pairs' test operands as OPS_REC-int records {E3 slice 0, E3
  // slice 1, Sab, Sa2b, Sab2, Sa2b2, j, 0} appended at ops (a wave reserves its records with one
  // atomic on ops_count, a persistent one in chunks of PF_CHUNK or more; nothing is stored past
  // ops_cap: the host sees the count (records reserved, a little above those written), grows the buffer
  // and reruns the launch); a live block's pairs' records are consecutive, ascending j
  int *ops;
  unsigned *ops_count;
  int64_t ops_cap;
};
// the live-block entries of the compacted path: mask | first record << 32 | tag << 58 (records < 2^26)
constexpr int LM_BASE_BITS = 26;
__host__ __device__ inline uint64_t lm_entry(uint32_t mask, uint32_t base, unsigned tag) {
  return (uint64_t)mask | ((uint64_t)(base & ((1u << LM_BASE_BITS) - 1)) << 32) | ((uint64_t)tag << 58);
}
__device__ inline uint32_t lm_mask(uint64_t e, unsigned tag) { return (unsigned)(e >> 58) == tag ? (uint32_t)e : 0u; }
__device__ inline uint32_t lm_base(uint64_t e) { return (uint32_t)(e >> 32) & ((1u << LM_BASE_BITS) - 1); }
constexpr int OPS_REC = 8;  // ints per live-pair record (32 bytes: two 16-byte stores / loads)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void *base, int64_t bytes) {
  const uint64_t b = (uint64_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b), hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const unsigned nb = __builtin_amdgcn_readfirstlane((unsigned)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)nb, 0x00020000);
}

// Candidate test of pair (i, j) (band row ri of the launch) given M = w'P~w (P~ the screen's
// approximation of P_off) and sum w^2: every pair whose p-value could be below p_cut is kept.
// ts (MX screens): the tile's E1 / Ed / E2 slice products ([3][SIDE_T][MX_TS] int32 at slot * 32 +
// col, tile_side_kernel); otherwise they come from the launch's band arrays like E3.
constexpr int MX_TS = 16 * 32;
__device__ __forceinline__ void cand_test(const ScreenArgs &a, int ri, int64_t i, int64_t j, double M, double sumw2,
                                          const int *ts = nullptr, int slot = 0, int col = 0) {
  if (j >= a.m || j < a.j_lo || (a.tri && j <= i)) return;  // j_lo: a launch's (or segment's) first column
  if (a.mono_l[i] || a.mono_r[j]) return;  // x == 0: the reference's statistic is NaN
  const int64_t o1 = (int64_t)ri * a.ld_e + (j - a.j_lo), o3 = o1 + (int64_t)a.n_rows * a.ld_e,
                od = o3 + (int64_t)a.n_rows * a.ld_e;
  double c1 = 0.0, c3 = 0.0, cd = 0.0, c2 = 0.0;
  const int so = slot * 32 + col;
#pragma unroll
  for (int t = a.e3_t - 1; t >= 0; --t) c3 = c3 * (1.0 / 128.0) + (double)a.c13[t * a.c13_stride + o3];
#pragma unroll
  for (int t = SIDE_T - 1; t >= 0; --t) {  // exact: |c| < 2^22, powers of two
    if (ts) {
      c1 = c1 * (1.0 / 128.0) + (double)ts[(0 * SIDE_T + t) * MX_TS + so];
      cd = cd * (1.0 / 128.0) + (double)ts[(1 * SIDE_T + t) * MX_TS + so];
      c2 = c2 * (1.0 / 128.0) + (double)ts[(2 * SIDE_T + t) * MX_TS + so];
    } else {
      c1 = c1 * (1.0 / 128.0) + (double)a.c13[t * a.c13_stride + o1];
      cd = cd * (1.0 / 128.0) + (double)a.c13[t * a.c13_stride + od];
      c2 = c2 * (1.0 / 128.0) + (double)a.c2[t * a.c2_stride + o1];
    }
  }
  const double E1 = a.sL[i] * c1, E3 = a.sL3[i] * c3, Ed = a.sLd[i] * cd, E2 = a.sR[j] * c2;
  const double dE1 = a.side_eps * a.sL[i] * a.csum_r[j], dE3 = a.e3_eps * a.sL3[i] * a.csum_r[j],
               dEd = a.side_eps * a.sLd[i] * a.csq_r[j], dE2 = a.side_eps * a.sR[j] * a.csum_l[i];
  const double al = a.alpha[i], be = a.beta[j];
  const double t1 = -2.0 * be * E1, t2 = -2.0 * al * E2, t3 = be * be * a.qa[i], t4 = -2.0 * al * be * be * a.ra[i],
               t5 = al * al * a.qb[j], t6 = -2.0 * al * al * be * a.rb[j], t7 = al * al * be * be * a.zz;
  const double var = M + Ed + t1 + t2 + t3 + t4 + t5 + t6 + t7;
  const double eff = E3 - be * a.sa[i] - al * a.sb[j] + al * be * a.spy;
  const double slack =
      1e-12 * (fabs(M) + fabs(Ed) + fabs(t1) + fabs(t2) + fabs(t3) + fabs(t4) + fabs(t5) + fabs(t6) + fabs(t7));
  // |w'(P_off - P~)w| <= a.delta * |w|^2 (a.delta: rigorous bound of the approximation error)
  const double var_lo = var - a.delta * sumw2 - slack - 2.0 * fabs(be) * dE1 - 2.0 * fabs(al) * dE2 - dEd;
  const double eff_hi = fabs(eff) + dE3;
  const bool cand = !(var_lo > 0.0) || eff_hi * eff_hi * (1.0 + 1e-9) >= a.chi_cut * var_lo;
  if (cand) {
    const unsigned long long k = atomicAdd(a.counter, 1ULL);
    if ((int64_t)k < a.cap) {
      a.cand_i[k] = i;
      a.cand_j[k] = j;
    }
  }
}

// ------------------------------------------------------------------ fused side pass
// Multi-product int8 GEMMs over a launch's band rows x all columns, 64 x 64 (band row, column)
// tiles, exact int32 on v_mfma_i32_32x32x32_i8 from double-buffered LDS stages of 64 individuals.
// Row-side operand sets are read straight from the per-SNP arrays through rows[] (no band
// gather), column-side sets by column.
//   PASS 1 (prefilter_pass_kernel below): E3 and the code products, the spectral prefilter in the
//           epilogue, flags per (band row, 32-column block), E3 (and the code products) of flagged blocks.
//   PASS 2..4: E1_t = L'q_t[i].b_j, Ed_t = Ldq_t[i].b_j^2, E2_t = a_i.R'q_t[j], written only for
//           flagged blocks (the MX screen's side terms; the low-rank screen needs none).
constexpr int SG_T = 64, SG_K = 64, SG_P = 80;  // tile edge, individuals per stage, LDS pitch
struct SideArgs {
  ScreenArgs a;  // rows, tri, j_lo, ld_e, scalars, prefilter constants, flags, c13 / c2 outputs
  const int8_t *rs[7];  // row-side sets [m][n_pad] (slices: stride slice_stride)
  const int8_t *cs[5];  // column-side sets
  const uint8_t *rs4, *cs4;  // prefilter: fp4 code panels (a | b) [m][n_pad / 2]
  const uint8_t *rs2, *cs2;  // prefilter: stage-blocked 2-bit code panels (a | b) [n_pad / 64][m][16 B]
  int64_t n_pad;
  int n_rt;             // row tiles
  int blocked;          // prefilter_pass_kernel: rs[0..E3_PF), rs4, cs4 are stage-blocked panels
                        // ([n_pad / 64][m][64 B] int8, block_panel_perm8_kernel; the codes: rs2 / cs2)
  const float *recL, *recR;  // prefilter_pass_kernel: test records, row / column role (pf_rec_kernel)
  const int *tile_list;      // prefilter_pass_kernel: the launch's running tiles (rt + n_rt ct, ascending),
  int n_list;                // dealt to the XCDs in contiguous eighths; null: one tile per workgroup
  const uint8_t *qimg;       // prefilter_cov_kernel: the quantised covariate directions [ncov][n_pad] int8
};

// LDS-DMA of 16 bytes per lane (global_load_lds_dwordx4: lane i's bytes land at lds + 16 i) issued
// through inline asm.  With the builtin the compiler tracks the DMA as an LDS write and, unable to
// tell the ring slot being filled from the one being read, puts an s_waitcnt vmcnt(0) before the
// next ds_read: every stage then waits for its own prefetch.  Here the kernels count vmcnt
// themselves (the compiler's own loads stay safe: vmcnt retires in order, so its waits can only
// over-wait on these).
__device__ __forceinline__ void lds_dma16(const void *g, const void *lds) {
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "{m0}"(m) : "memory");
}

// ------------------------------------------------------------------ prefilter pass
// The prefilter of the low-rank / MX screens (the PASS 1 products of side_gemm_kernel) on 64 x 256
// (band row, column) tiles, 8 waves of 32 x 64 (2 row x 4 column waves).  The pass is bound by the
// chip's L2 -> LDS fabric (~6.4 TB/s of LDS-DMA with every CU streaming), so the tile shape minimises
// the bytes per pair at the register file's limit of 16,384 pairs (six accumulators each): a row
// brings 160 B per stage (two int8 L3 slices + fp4 codes), a column 32 B, so 64 x 256 streams 18 KB
// per stage where 128 x 128 streamed 24 KB.  Stage image (64 individuals), five-slot LDS-DMA ring
// (65 KB), four stages in flight: int8 L3 slices 0, 1 (64 rows x 64 B each), then the genotype codes
// of a (64 rows) and b (256 columns) at 2 bits each (16 B per SNP and stage, code2_panel_kernel: the
// codes take 0, 1, 2; round 3 streamed them as fp4, 32 B, so that a stage is 13 instead of 18 KB).  The
// fp4 codes (fp4_of_code2: two VALU per dword), their squares (sq4) and the int8 b of the E3 products
// (i8x2_of_fp4_eo) come from them in registers.  The int8 16-byte chunks XOR-swizzled through the
// DMA source address (chunk ^ (row >> 2) & 3); the image holds DMA instruction q (1 KB) at q KB, wave w
// issuing q = w + 8u (u < 2; waves 0-4 two, 5-7 one).  Round 5: by default 32 x 256 tiles of four
// waves (1 row x 4 column waves, a 9 KB stage), two workgroups per CU (prefilter_pass_kernel<.., 32, 5>);
// the constants below are the 64-row shape's (eight waves: the block-granular path).
constexpr int PF_TR = 64, PF_TC = 256, PF_ST = 13 * 1024, PF_NS = 5, PF_NQ = 13;
constexpr int PF_REC = 8;  // floats per prefilter test record (pf_rec_kernel)
constexpr int PF_CHUNK = 128;  // live-pair records a persistent prefilter wave reserves at a time
constexpr int PF_NSTAMP = 9;  // GMAT_PF_STAMPS: start, prologue, main loop, column records, tests, stores, end
                               // (s_memrealtime), then s_memtime (shader clock) at start and end
constexpr int PF_NPHASE = 7;
// fp4 codes of c^2 from those of c in {0, 1, 2} (0x0, 0x2, 0x4 -> 0x0, 0x2, 0x6): nibble bit 2 -> bit 1
__device__ __forceinline__ v8i_ sq4(v4i x) {
  v8i_ r = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < 4; ++q) r[q] = x[q] | ((x[q] >> 1) & 0x22222222);
  return r;
}
// fp4 codes (e2m1 nibble 2c: 0, 1, 2 -> 0x0, 0x2, 0x4) of 32 genotype codes c stored at 2 bits
// (code2_panel_kernel: per 16 individuals a dword whose nibble k holds c[k] | c[8 + k] << 2), as the
// four nibble-per-individual dwords of individuals 0-7, 8-15, 16-23, 24-31
__device__ __forceinline__ v4i fp4_of_code2(v2i_ d) {
  const unsigned d0 = (unsigned)d[0], d1 = (unsigned)d[1];
  return v4i{(int)((d0 << 1) & 0x66666666u), (int)((d0 >> 1) & 0x66666666u), (int)((d1 << 1) & 0x66666666u),
             (int)((d1 >> 1) & 0x66666666u)};
}
// int8 values of 16 fp4 codes (two dwords, individual i at nibble i): code >> 1, in order
__device__ __forceinline__ v4i i8_of_fp4(unsigned x0, unsigned x1) {
  const unsigned l0 = (x0 >> 1) & 0x07070707u, h0 = (x0 >> 5) & 0x07070707u;
  const unsigned l1 = (x1 >> 1) & 0x07070707u, h1 = (x1 >> 5) & 0x07070707u;
  v4i r;
  r[0] = (int)__builtin_amdgcn_perm(h0, l0, 0x05010400u);
  r[1] = (int)__builtin_amdgcn_perm(h0, l0, 0x07030602u);
  r[2] = (int)__builtin_amdgcn_perm(h1, l1, 0x05010400u);
  r[3] = (int)__builtin_amdgcn_perm(h1, l1, 0x07030602u);
  return r;
}
// int8 values 2b of 16 fp4 codes (code = 2b for b in {0, 1, 2}) WITHOUT the interleave: even
// individuals of the first dword, odd ones, then the same for the second (K slot order 0 2 4 6 1 3 5 7
// per 8 individuals).  The prefilter's stage-blocked int8 L3 panels are stored in that order
// (block_panel_perm8_kernel), so A and B agree slot by slot: three VALU per dword, no v_perm.  The
// products come out doubled (exactly: every term is even) and are halved where they are used.
__device__ __forceinline__ v4i i8x2_of_fp4_eo(unsigned x0, unsigned x1) {
  v4i r;
  r[0] = (int)(x0 & 0x0f0f0f0fu);
  r[1] = (int)((x0 >> 4) & 0x0f0f0f0fu);
  r[2] = (int)(x1 & 0x0f0f0f0fu);
  r[3] = (int)((x1 >> 4) & 0x0f0f0f0fu);
  return r;
}
// LDS-DMA from a wave-uniform 64-bit base (SGPRs) + a 32-bit per-lane byte offset (one VGPR per
// source instead of two), LDS destination m0
__device__ __forceinline__ void lds_dma16_sv(unsigned voff, const void *sbase, unsigned m0) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}
// LDS-DMA with the LDS destination given as a wave-uniform byte address (m0), no per-call
// generic -> LDS address conversion
__device__ __forceinline__ void lds_dma16_m0(const void *g, unsigned m0) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(g), "{m0}"(m0) : "memory");
}

// ------------------------------------------------------------------ prefilter pass, covariate designs
// The same prefilter when P has null directions besides 1 (covariate columns of X): the certificate
// (gmat_epi_create) is  e'Pe >= mu |e|^2 - (mu + tau)(1'e)^2/n - ku |U'e|^2 - eps |e|^2  with U the
// orthonormal null directions, so every pair also needs u_k'e = (a o u_k).b - beta u_k.a - alpha
// u_k.b + alpha beta 1'u_k for k < NC.  u_k is quantised once per plan to q_k = rint(u_k / sq_k),
// sq_k = max |u_k| / 63 (ensure_pf_q), so that a o q_k is an exact int8 vector (|a q| <= 126) and
// |(a o u_k).b - sq_k (a o q_k).b| <= sq_k / 2 sum_t a_t b_t = sq_k Sab / 2 (Sab: the exact code product
// the kernel computes anyway).  The images a o q_k are formed ON CHIP, once per stage and workgroup,
// from the streamed fp4 codes of a and a 64-byte q slice per direction (round 3 streamed per-row int8
// images a o u_k from HBM: 64 B per row, stage and direction, 2.1x the bytes per pair of the
// intercept-only prefilter).  32 x 256 (row, column) tiles, 8 waves of 32 x 32 (one row band, wave w
// the columns 32 w ..) at two waves per SIMD (the NC extra int32 accumulator sets keep a wave at 1,024
// pairs).  Stage slot (64 individuals), all from stage-blocked panels: DMA instruction q (1 KB) at q KB:
// L3 slices 0, 1 (q 0-3, 32 rows x 64 B each), the 2-bit codes of a (q 4, 32 rows x 16 B; lanes 32-63
// load a copy into the unused half) and b (q 5-8, 256 columns x 16 B), the q slices (q 9: direction k at
// 64 k).  The NC direction images (32 rows x 64 B each, same swizzle as
// the L3 slices) are written by the workgroup into a double buffer: the image of stage s + 1 is formed
// while stage s multiplies.  Eight-slot ring: stage s + 7 streams while stage s multiplies (stages up
// to s + 2 have landed at its closing barrier, five more in flight: the loop is bound by the latency of
// the LDS-DMA stream as much as by its rate).
// Round 5: by default 32 x 128 tiles of four waves, two workgroups per CU (TC = 128: b's codes at q 5-6,
// the q slices at q 7; a seven-slot ring), as the intercept-only prefilter's 32-row tiles.
constexpr int PC_TR = 32, PC_TC = 256, PC_NS = 8, PF_NCOV_MAX = 4;
template <int NC, int TC = PC_TC>
struct PcShape {
  static constexpr int O_A2 = 4096, O_B2 = 5120, O_Q = O_B2 + TC * 16;
  static constexpr int QT = 6 + TC / 64;               // DMA instructions per stage
  static constexpr int ST = O_Q + 1024;                // slot bytes
  static constexpr int NS = TC == PC_TC ? PC_NS : 7;   // ring slots
};
// s_waitcnt vmcnt(n) lgkmcnt(0) + s_barrier as ONE asm statement (see prefilter_pass_kernel)
__device__ __forceinline__ void vm_wait_barrier(int n) {
#define VMW(k) \
  case k:      \
    asm volatile("s_waitcnt vmcnt(" #k ") lgkmcnt(0)\n\ts_barrier" ::: "memory"); \
    break;
  switch (n) {
    VMW(1) VMW(2) VMW(3) VMW(4) VMW(5) VMW(6) VMW(7) VMW(8) VMW(9) VMW(10) VMW(11) VMW(12) VMW(13) VMW(14)
    VMW(15) VMW(16) VMW(17) VMW(18) VMW(19) VMW(20) VMW(21) VMW(22) VMW(23) VMW(24) VMW(25) VMW(26) VMW(27)
    VMW(28) VMW(29) VMW(30) VMW(31) VMW(32)
    default:
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
#undef VMW
}
// a o q for 16 individuals in the stage-blocked panels' even/odd order (i8x2_of_fp4_eo): a from two
// dwords of fp4 codes (0, 1, 2 as e2m1: nibble = 2a), q as int8 (|q| <= 63, the same order): bytes q
// where a = 1, 2q where a = 2, 0 where a = 0 (byte-table v_perm masks on 2a + bit select)
__device__ __forceinline__ v4i aq_of_fp4_eo(unsigned x0, unsigned x1, v4i q) {
  const v4i av = i8x2_of_fp4_eo(x0, x1);  // 2a: 0, 2, 4
  v4i r;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const unsigned a = (unsigned)av[d], qd = (unsigned)q[d];
    const unsigned nz = __builtin_amdgcn_perm(0x000000FFu, 0x00FF0000u, a), two = __builtin_amdgcn_perm(0x000000FFu, 0u, a);
    const unsigned q2 = (qd & 0x7F7F7F7Fu) << 1;  // 2q per byte (|2q| <= 126: the dropped bit is a sign copy)
    r[d] = (int)((q2 & two) | (qd & nz & ~two));
  }
  return r;
}

// Tile shapes (SH): the K-block height MT (rows of A_s per accumulator set) and the pair blocks
// PB per wave.  SH 0: MT 128, PB 2 -> 8 first SNPs x 32 second SNPs per workgroup; each
//   generated B fragment feeds 4 MFMAs.
// SH 1: MT 256, PB 1 -> 4 x 32 per workgroup; each B fragment feeds 8 MFMAs (half the
//   B-generation VALU per MFMA), same 128 accumulator registers.
template <int SH>
struct Shape {
  static constexpr int MT = SH ? 256 : 128;
  static constexpr int PB = SH ? 1 : 2;
  static constexpr int BI = 4 * PB;      // first-SNP rows per tile
  static constexpr int RB = MT / 32;     // 32-row accumulator blocks per wave
  static constexpr int EP = MT + 16;     // epilogue-region pitch
  static constexpr int NA = MT / 64;     // 16-byte A chunks per thread per stage
  static constexpr int DS = MT / LK;     // diagonal-block stages per K-block
};


// ------------------------------------------------------------------ MX screen (fp6 x fp4)
// The same screen on the block-scaled v_mfma_scale_f32_32x32x64_f8f6f4 (fp6 e2m3 x fp4 e2m1,
// twice the int8 rate).  A = P_off in fp6 with one e8m0 scale per (row, 32 storage columns)
// (residual ~0.46x that of one int8 slice on relationship matrices: the per-block scale follows
// the many small entries); B = w/2 in fp4 (w in {0,1,2,4} -> codes 0,1,2,4, so the code IS the
// integer w), generated per 8 individuals with one v_and + one v_and_or from nibble planes:
//   i side  M1 = [a == 1] 0xF, M2 = [a == 2] 0xF;  j side  S1 = b, S2 = 2b;
//   code(w) = (M1 & S1) | (M2 & S2).
// The B scale restores w (x2) on the diagonal block and 2w (x4) beyond it.  Accumulation is
// fp32; its rounding is bounded rigorously (gmat_epi_create) and folded into delta.  The
// epilogue sums w[row] * acc[row] with v_cvt_scalef32_pk_f32_fp4 (two w per instruction, from the
// same nibble codes) and v_pk_fma_f32; sum w^2 comes from v_dot8_u32_u4.
//
// A is stored as tile images, one per (K-block of 128 natural rows, 128-column stage), laid out
// exactly as the LDS stage: four planes (block (kk, h) = columns 64kk + 32h .. +32) of 128 rows x
// a 32-byte slot = 6 dwords of fp6 codes (code j at bits 6j), the row's e8m0 scale in dword 6,
// dword 7 zero; rows with (row >> 3) & 1 store the two 16-byte halves swapped, which makes the
// two ds_read_b128 per fragment bank-conflict-free.  Genotype nibble records per (SNP, stage) =
// two 64-byte planes (individual 2q + e at nibble e of byte q); in LDS the j side's 16-byte slots
// are XOR-swizzled with (snp >> 1) & 7 (conflict-free), the i side is read as a broadcast.
constexpr int MXK = 128;          // individuals per MX stage (= K-block height)
constexpr int MX_TILE = 16384;    // bytes per A tile image
constexpr int NB_REC = 128;       // nibble bytes per (SNP, stage): two planes
constexpr int NB_E = 136;         // LDS pitch of the epilogue copies (8-byte reads)
constexpr int MX_BI = 16, MX_RB = MXK / 32;  // first SNPs per workgroup; 32-row tiles per K-block
// workgroup shape (MxShape<1>): 8 waves x 2 pair blocks, two waves per SIMD (a 4-wave x 4-block
// shape with 256 accumulator registers per wave measured slower: one wave per SIMD exposes the
// LDS and barrier latency)
template <int V>
struct MxShape {
  static_assert(V == 1, "only the 8-wave shape is built");
  static constexpr int NW = 8, PB = MX_BI / NW, T = 64 * NW, MINB = 1;
};


struct MxArgs {
  const uint8_t *tiles;    // [nK][nK] A tile images (upper ones used)
  const uint8_t *nib_i;    // i-side planes (M1, M2) of the left coding [m][nK][NB_REC]
  const uint8_t *nib_j;    // j-side planes (S1, S2) of the right coding
  int64_t tiles_bytes, nib_bytes;
  int nK;
};

__device__ __forceinline__ v16f_ mfma_mx(v8i_ fa, v8i_ fb, v16f_ c, int sa, int sb) {
  return __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, c, 2, 4, 0, sa, 0, sb);  // fp6 x fp4
}
template <int BB>
__device__ __forceinline__ v2f_ fp4_pair(unsigned wd) {
  return __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(wd, 2.0f, BB);
}

// One workgroup = MX_BI (band row, 32-column block) slots in two halves: slots 0 .. MX_BI/2-1
// pair with column block J0 of the tile, the rest with J1 (rows flagged by the prefilter are
// packed in half-tiles, so partly filled column blocks share a workgroup).  Wave w owns slots
// PB*w .. +PB (one half, so its column block is wave-uniform): MX_RB row tiles x PB column
// tiles of 32 x 32 per K-block.  Loop nest: K-block kb -> column stage cs >= kb (one 128-deep
// stage = two 64-deep k-steps), LDS double buffer, one barrier per stage; the next stage is
// fetched into registers while this one multiplies.  The diagonal stage's genotype records are
// also copied to eI/eJ for the K-block's epilogue.  Tile entries are (row-list index, J0, J1).
constexpr int MX_TE = 3;  // ints per tile entry

// ------------------------------------------------------------------ low-rank screen (LR)
// A certified lower bound of var = e'Pe from the bottom of P's spectrum.  With B (n x R) the
// fp6-quantised bottom eigenvectors of P (as the MFMA reads them) and D = diag(d) >= 0,
// gmat_epi_create certifies by an fp64 Cholesky that
//   P - lam (I - 11'/n) + tau 11'/n + B D B' - eps I  is positive semi-definite,
// so for every e
//   e'Pe >= lam (|e|^2 - (1'e)^2/n) - tau (1'e)^2/n - eps |e|^2 - sum_r d_r (B_r'e)^2.
// The per-pair cost is R x n MACs instead of the quadratic form's n^2/2: for relationship-
// structured P the few hundred smallest eigen-directions carry the bound (lam approaches the
// (R+1)-th eigenvalue).  c_r = B_r'e expands with e = (a - alpha) o (b - beta) (screen codes):
//   c_r = B_r'w - beta G_r(i) - alpha H_r(j) + alpha beta q1_r,   w = a o b,
// B_r'w on v_mfma_scale_f32_32x32x64_f8f6f4 (A = B' in fp6 tile images, B = w/2 in fp4, the
// MX screen's operands), G = panel x B per coding (fp32), q1 = B'1.  eta_r bounds the fp32
// accumulation and the fp32 G / H / combination rounding, |c_r - c~_r| <= eta_r, so
//   sum_r d_r c_r^2 <= sum_r d_r (|c~_r| + eta_r)^2.
// |e|^2 and 1'e are exact from the prefilter pass's int8 code products (pfc), eff from E3.
struct LrArgs {
  const uint8_t *tiles;    // [nC][nK] B' tile images (MX_TILE bytes each)
  const uint8_t *nib_i, *nib_j;
  int64_t tiles_bytes, nib_bytes;
  int nK, nC, R;           // stages, 128-row chunks, padded rank
  int n_tiles;             // tile entries of the launch: workgroup b takes entries b, b + grid, ...
  const float *G, *H;      // [m][R]: left G' = Q'a - alpha Q'1, right H = Q'b
  const double *recL, *recR;  // per-SNP test records (LR_REC doubles each, lr_rec_kernel)
  double lam, tau, eps, E;  // E = sum_r eta_r^2
};
// Test records: left {alpha, csum, csq, sL3, sa, mono}, right {beta, csum, csq, sb, mono}, padded to
// 64 bytes (four 16-byte DMA chunks)
constexpr int LR_REC = 8;
// Test operands staged in LDS while a tile's stages run: planes [LR_NPL][16 slots][32 columns] of
// int32 (the E3 slices c13_0 .. c13_{SIDE_T-1}, then the code products Sab, Sa2b, Sab2, Sa2b2), the
// 16 slots' left records and the 64 columns' right records.
constexpr int LR_NPL = SIDE_T + 4, LR_PLANE = MX_BI * BJ * 4;
constexpr int LR_OFF_RL = LR_NPL * LR_PLANE, LR_OFF_RR = LR_OFF_RL + MX_BI * LR_REC * 8;
constexpr int LR_ST_BYTES = LR_OFF_RR + 2 * BJ * LR_REC * 8;

__device__ __forceinline__ void lds_dma4(const void *g, const void *lds) {
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned m = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)lds);
  asm volatile("s_nop 0\n\tglobal_load_lds_dword %0, off" : : "v"(g), "{m0}"(m) : "memory");
}

// Candidate test of the lane's pair (slot s, column col of column block `half`) from the operands
// staged in sT: every pair whose p-value could be below p_cut is kept.
__device__ __forceinline__ void lr_test(const ScreenArgs &a, const LrArgs &x, const uint8_t *sT, int s, int col,
                                        int half, bool ok, int64_t i, int64_t j, double lowrank) {
  const int *pl = (const int *)sT + s * BJ + col;
  const double *rl = (const double *)(sT + LR_OFF_RL) + s * LR_REC;
  const double *rr = (const double *)(sT + LR_OFF_RR) + (half * BJ + col) * LR_REC;
  double c3 = 0.0;
#pragma unroll
  for (int t = SIDE_T - 1; t >= 0; --t) c3 = c3 * (1.0 / 128.0) + (t < a.e3_t ? (double)pl[t * MX_BI * BJ] : 0.0);
  const double sab = (double)pl[SIDE_T * MX_BI * BJ], sa2b = (double)pl[(SIDE_T + 1) * MX_BI * BJ],
               sab2 = (double)pl[(SIDE_T + 2) * MX_BI * BJ], sa2b2 = (double)pl[(SIDE_T + 3) * MX_BI * BJ];
  const double al = rl[0], ca = rl[1], ca2 = rl[2], sl3 = rl[3], sai = rl[4];
  const double be = rr[0], cb = rr[1], cb2 = rr[2], sbj = rr[3];
  const bool mono = rl[5] != 0.0 || rr[4] != 0.0;
  const double n = a.n_id;
  const double eff = sl3 * c3 - be * sai - al * sbj + al * be * a.spy;
  const double eff_hi = fabs(eff) + a.e3_eps * sl3 * cb;
  const double t_ee[9] = {sa2b2, -2.0 * be * sa2b, be * be * ca2, -2.0 * al * sab2, 4.0 * al * be * sab,
                          -2.0 * al * be * be * ca, al * al * cb2, -2.0 * al * al * be * cb, n * al * al * be * be};
  double ee = 0.0, mag = 0.0;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    ee += t_ee[q];
    mag += fabs(t_ee[q]);
  }
  const double se = sab - be * ca - al * cb + n * al * be;
  // |Q'e|^2 <= (|c~| + |eta|)^2; fp32 sums of squares: relative error < 1e-4
  const double qb = sqrt(lowrank * (1.0 + 1e-4)) + sqrt(x.E);
  const double vlo = x.lam * (ee - se * se / n) - x.tau * se * se / n - x.eps * ee - qb * qb -
                     1e-12 * (x.lam + x.tau) * (mag + se * se / n);
  if (ok && !mono && (!(vlo > 0.0) || eff_hi * eff_hi * (1.0 + 1e-9) >= a.chi_cut * vlo)) {
    const unsigned long long k = atomicAdd(a.counter, 1ULL);
    if ((int64_t)k < a.cap) {
      a.cand_i[k] = i;
      a.cand_j[k] = j;
    }
  }
}


// ------------------------------------------------------------------ compacted low-rank screen
// The low-rank screen of lr_screen_kernel on the prefilter's live PAIRS instead of its flagged
// (band row, 32-column block) slots: at configs[2] 0.40 % of the pairs survive the prefilter but
// 8.5 % of the 32-pair blocks hold one, so testing whole blocks multiplies ~21x the necessary work.
// A slot is (band row r, 32 live second SNPs of r in ascending order: slot lists, lc_* kernels); a
// tile is 16 slots (8 waves x 2 slots, the MX shape), one tile per workgroup.  Per 128-individual
// stage the A tile image (Q' fp6, shared by every slot) and the slots' i-side nibble records come
// through LDS-DMA as in lr_screen_kernel, and so do the 512 columns' j-side S1 planes (each column
// its own SNP: 32 KB per stage), in an NSL-slot ring.  The chunk epilogue reads G' of the slot
// rows and H of the columns from memory, the test reads the prefilter's stored operands (E3
// slices, code products) and the per-SNP records; the bound and the test are lr_screen_kernel's.
struct LrcArgs {
  const uint8_t *tiles;  // [nC][nK] Q' tile images
  const uint8_t *nib_i, *nib_j;
  const uint8_t *s1c2;           // the j side's S1 planes at 2 bits (s1_code2_kernel) [m][nK][32 B]
  int nK, nC, R;
  const int *slot_row, *slot_j;  // slot lists of the launch
  const int *slot_ops;           // the slot pairs' records (OPS_REC ints each, lc_fill)
  const float *G, *H;            // [m][R]: left G' = Q'a - alpha Q'1, right H = Q'b
  const double *recL, *recR;     // per-SNP test records (LR_REC doubles each)
  double lam, tau, eps, E;
};
constexpr int LRC_J2B = 32;  // j-side bytes per column and stage of the compacted screen (2-bit S1 planes)

// slot pair p's record (lc_fill: the prefilter's E3 slices and code products of the pair)
__device__ __forceinline__ bool lrc_cand(const ScreenArgs &a, const LrcArgs &x, int64_t p, int64_t i, int64_t j,
                                         double lowrank) {
  static_assert(E3_PF == 2, "record layout");
  const v4i r0v = *(const v4i *)(x.slot_ops + p * OPS_REC), r1v = *(const v4i *)(x.slot_ops + p * OPS_REC + 4);
  const double c3 = (double)r0v[0] + (double)r0v[1] * (1.0 / 128.0);
  const double sab = (double)r0v[2], sa2b = (double)r0v[3], sab2 = (double)r1v[0], sa2b2 = (double)r1v[1];
  const double *rl = x.recL + i * LR_REC, *rr = x.recR + j * LR_REC;
  const double al = rl[0], ca = rl[1], ca2 = rl[2], sl3 = rl[3], sai = rl[4];
  const double be = rr[0], cb = rr[1], cb2 = rr[2], sbj = rr[3];
  const double n = a.n_id;
  const double eff = sl3 * c3 - be * sai - al * sbj + al * be * a.spy;
  const double eff_hi = fabs(eff) + a.e3_eps * sl3 * cb;
  const double t_ee[9] = {sa2b2, -2.0 * be * sa2b, be * be * ca2, -2.0 * al * sab2, 4.0 * al * be * sab,
                          -2.0 * al * be * be * ca, al * al * cb2, -2.0 * al * al * be * cb, n * al * al * be * be};
  double ee = 0.0, mag = 0.0;
#pragma unroll
  for (int q = 0; q < 9; ++q) {
    ee += t_ee[q];
    mag += fabs(t_ee[q]);
  }
  const double se = sab - be * ca - al * cb + n * al * be;
  // |Q'e|^2 <= (|c~| + |eta|)^2; fp32 sums of squares: relative error < 1e-4
  const double qb = sqrt(lowrank * (1.0 + 1e-4)) + sqrt(x.E);
  const double vlo = x.lam * (ee - se * se / n) - x.tau * se * se / n - x.eps * ee - qb * qb -
                     1e-12 * (x.lam + x.tau) * (mag + se * se / n);
  return !(vlo > 0.0) || eff_hi * eff_hi * (1.0 + 1e-9) >= a.chi_cut * vlo;
}





// ------------------------------------------------------------------ exact fp64 refine
// For pairs (pi[t], pj[t]): e = (a - alpha)(b - beta) in fp64 (storage order), var = e'Pe,
// eff = e'Py.  RP pairs per workgroup (P, 32 MB in fp64, is streamed once per workgroup from
// the MALL/HBM, so more pairs per workgroup = less traffic); for every RM-row block of P the f64
// MFMA tile C = P[rows, k >= rows] E (off-diagonal blocks x2, exact) is formed in RK-deep stages
// (the next stage's P rows and code bytes fetched into registers while this one multiplies) and
// folded into var.  Waves: 4 (rows) x 2 (64-pair halves), each 32 x 64 of 16x16x4 f64 MFMA tiles.
// The (row block, column stage) sequence of a pair tile splits into gridDim.y segments of equal
// work (blockIdx.y = segment) so that a short candidate list still fills whole rounds of the
// chip; segment partials of var / eff go to var_part / eff_part and refine_sum adds them in order.
constexpr int RP = 128, RM = 128, RK = 32, RT = 512, RF_SEG = 4;

__device__ __forceinline__ double ecode(const int8_t *l, const int8_t *r, double al, double be, int64_t q) {
  const double x = (double)l[q] - al;
  const double y = (double)r[q] - be;
  return x * y;
}

typedef double v2d_ __attribute__((ext_vector_type(2)));
typedef int v2i__ __attribute__((ext_vector_type(2)));



// ------------------------------------------------------------------ exact refine on int8 slices
// var = e'Pe for the candidates with the O(n^2) part on the int8 matrix cores.  With the screen codes
// a, b (integers), w = a o b and v = -beta a - alpha b + alpha beta 1 (the pair screen's expansion):
//   e'Pe = w'P_off w + sum_q P_qq w_q^2 + 2 v'Pw + v'Pv.
// w'P_off w: P_off in storage order is cut into R8_S int8 slices of one unit u = 2 qmax / 127,
//   P' = u sum_s 128^-s A_s + R,  |R_kl| <= u 128^-(R8_S-1) / 2  (~1e-15 qmax),
// of the block-upper form at 32-row granularity (diagonal blocks as they are, blocks right of the
// diagonal doubled -- hence 2 qmax in the unit --, blocks left of it zero), so that w'P_off w = w'P'w
// and w'A_s w is an exact integer: int32 MFMA accumulation per row (|sum| < 2^21), int32 fold with w
// per row tile, fp64 sums of integers (< 2^53) per slice; the only roundings are the final fp64
// combination sum_s 2^-7s T_s and R (|w'Rw| <= 8e-16 qmax |w|_1^2).  The O(n) terms are fp64 dot
// products with U = P x codes (refine8_side_kernel), eff = e'Py in fp64 from the reference codes.
// Tiles: (32-row block kb, 64-column stage cs >= kb / 2), R8_S slices x 2 row tiles x 16 rows x 64
// bytes, 16-byte chunks XOR-swizzled by row (r8_swz); a workgroup = 8 waves x 16 pairs (v_mfma_i32_16x16x64_i8,
// w as the B fragments in registers: n_pad <= 64 R8_NC), the tiles stream through an eight-slot
// LDS-DMA ring (six in flight) in the order kb, then cs from the last stage down to kb / 2 (whose visit
// folds the row block).
constexpr int R8_S = 7, R8_TB = 2048, R8_TILE = R8_S * R8_TB, R8_NC = 32, R8_PP = 128;
constexpr int R8_PP2 = 256;  // pairs per workgroup of refine8_kernel (w held as 2-bit codes; refine8w_kernel: R8_PP)
constexpr int R8_NT = 4;  // O(n) sums per pair stored by refine8_side_kernel for refine8_fin_kernel
__host__ __device__ inline int64_t r8_toff(int64_t kb, int64_t NS) {  // tiles of the row blocks before kb
  const int64_t h = kb >> 1;
  return kb * NS - ((kb & 1) ? h * h : h * (h - 1));
}
// the 16-byte chunk swizzle of a tile row (row & 15): chunk k of row r sits at k ^ r8_swz(r), so that
// each 16-lane group of refine8_kernel's ds_read_b128 (rows c, chunks g) covers all 64 banks (k ^ (r & 3)
// alone left rows r and r + 4 on the same banks: 2-way conflicts, ~20 % of the kernel's cycles)
__host__ __device__ inline int r8_swz(int r) { return (r & 3) ^ ((r >> 1) & 2); }

// the most row-block segments a short refine8 / pair_mxr list is split into (GMAT_SEG_MAX, default 8)
inline int seg_max() {
  const char *s = getenv("GMAT_SEG_MAX");
  return s ? std::max(1, std::min(16, atoi(s))) : 8;
}


// ------------------------------------------------------------------ pair screen
// The screens' candidates re-tested one pair at a time before the fp64 refine (the low-rank
// screen's bound is loose by design: most of its candidates fail a sharper test).  With screen
// codes a, b, offsets alpha, beta, w = a o b and v = -beta a - alpha b + alpha beta 1, e = w + v and
//   e'Pe = w'P_off w + sum_q P_qq w_q^2 + 2 v'Pw + v'Pv,
//   v'Pw = w.(-beta Pa - alpha Pb + alpha beta z),
//   v'Pv = beta^2 a'Pa + alpha^2 b'Pb + alpha^2 beta^2 1'P1 + 2 alpha beta a'Pb - 2 alpha beta^2 a'P1
//          - 2 alpha^2 beta b'P1.
// pair_side_kernel forms every term but the first in fp64 from U = P x codes (the side vectors of
// the screens), and eff = e'Py; pair_mxr_kernel / pair_mxw_kernel evaluate w'P_off w on the MX screen's fp6 tile
// images with w in fp4 (the error bound rho_mx |w|^2 of mx_screen_kernel: the same operands,
// stage order and fp32 accumulation) and keeps the pair unless its p-value is certainly >= p_cut.
struct PairArgs {
  const int64_t *ci, *cj;  // candidates [np]
  int64_t np, n_pad;
  const int8_t *a, *b;        // screen panels (left, right coding) [m][n_pad]
  const _Float16 *Ua, *Ub;    // P x panel rounded to fp16 [m][n_pad]
  const double *alpha, *beta;  // screen-code offsets
  const double *qa, *ra, *qb, *rb;
  const double *z, *dg, *py;
  double zz;
  double *side;  // [5][np]: v-terms of var, their rounding slack, eff, sum |e py|, sum w^2
  const uint8_t *tiles, *nib_i, *nib_j;
  int64_t tiles_bytes;
  int nK;
  double rho, chi_cut;
  unsigned long long *counter;
  int64_t *oi, *oj;  // surviving pairs
  double *mpart;     // pair_mxr_kernel with segments: w'P~w per (segment, pair), added by pair_test_kernel
};

// the pair screen's test of pair p given M = w'P~w: kept unless its p-value is certainly >= p_cut
__device__ __forceinline__ void pair_test(const PairArgs &x, int64_t p, double M) {
  const double var = M + x.side[p], sw = x.side[4 * x.np + p];
  const double var_lo = var - x.rho * sw - x.side[x.np + p] - 1e-12 * fabs(M);
  const double eff_hi = fabs(x.side[2 * x.np + p]) + x.side[3 * x.np + p];
  if (!(var_lo > 0.0) || eff_hi * eff_hi * (1.0 + 1e-9) >= x.chi_cut * var_lo) {
    const unsigned long long k = atomicAdd(x.counter, 1ULL);
    x.oi[k] = x.ci[p];
    x.oj[k] = x.cj[p];
  }
}

// One wave per pair, PS_PPW pairs per wave; z, diag(P) and Py staged once per workgroup in LDS as
// fp32.  The sums run in fp32 with a certified slack: each lane adds its n_pad / 64 terms per
// quantity and the wave reduces the lane partials in fp64; the inputs' fp32 rounding (U = P x
// codes, z, diag(P), Py: 2^-24 relative each) adds a few 2^-24 per term (the bound is below; it is
// carried to the pair screen's variance bound, side[np + p], and to its eff bound, side[3 np + p]).
constexpr int PS_PPW = 8;


// The same quadratic form with each pair's w held in REGISTERS (n_pad <= 128 PXR_NK): a wave owns 32
// pairs, lane (c, h) holds pair c's fp4 w for 32 individuals of every 64-individual chunk (the MFMA
// B fragments, 4 registers per chunk), so 8 waves carry 256 pairs and the P tile images stream
// through LDS once per 256 pairs (round 3's LDS-resident w planes: once per 96) in an
// eight-slot LDS-DMA ring, six tiles in flight (the tiles compete for L2 with the pairs' record
// gathers).  Visit order: row block kb, then column stage cs from
// the last down to kb (the inner loop is unrolled so that every register index is static; its last
// visit, the diagonal tile, folds the row block's accumulators with w of block kb, fetched from the
// lane half that holds them).  Same operands, scales and bound as mx_screen_kernel.
constexpr int PXR_NK = 16, PXR_NSL = 8;  // w chunks in registers (n_pad <= 2048); LDS ring slots

// ------------------------------------------------------------------ setup kernels






// C[z] (M x N int32, ldc) = A[z] (M x K int8, lda) . B[z]^T (N x K int8, ldb) for z = blockIdx.z;
// K a multiple of 64.  64 x 128 tile per workgroup, each wave 32 x 64 (two 32x32x32 i8 MFMAs
// per k-step), 64-deep LDS stages with the 80-byte pitch.  Exact int32 accumulation.
constexpr int GM = 64, GN = 128, GKK = 64, GPI = 80;





// ---- MX setup.  fp6 e2m3 quantisation of P_off, one e8m0 scale per (natural row, 32 storage
// columns): scale 2^e with e the least exponent giving |v| / 2^e <= 7.5, round to nearest even
// on the e2m3 grid (steps 1/8 below 2, 1/4 below 4, 1/2 up to 7.5).  Also writes the dequantised
// matrix Qn (natural order) for the rigorous residual bound.
__host__ __device__ inline void fp6_block(const double *v, uint32_t wds[8], double *dq) {
  double mx = 0.0;
  for (int j = 0; j < 32; ++j) mx = fmax(mx, fabs(v[j]));
  int e = -127;
  if (mx > 0.0) {
    e = (int)ceil(log2(mx / 7.5));
    while (ldexp(7.5, e) < mx) ++e;
    while (e > -127 && ldexp(7.5, e - 1) >= mx) --e;
    e = e < -127 ? -127 : e;
  }
  for (int k = 0; k < 8; ++k) wds[k] = 0;
  wds[6] = (uint32_t)(e + 127);
  for (int j = 0; j < 32; ++j) {
    const double y = ldexp(v[j], -e), ay = fabs(y);
    double q;
    uint32_t code;
    if (ay < 2.0) {
      q = rint(ay * 8.0) / 8.0;
      code = (uint32_t)(q * 8.0);  // 0..16 (16 = 2.0)
    } else if (ay < 4.0) {
      q = rint(ay * 4.0) / 4.0;
      code = 16u + (uint32_t)((q - 2.0) * 4.0);
    } else {
      q = rint(ay * 2.0) / 2.0;
      code = 24u + (uint32_t)((q - 4.0) * 2.0);
    }
    if (y < 0.0 && code) code |= 32u;
    const int bit = 6 * j;
    wds[bit >> 5] |= code << (bit & 31);
    if ((bit & 31) > 26) wds[(bit >> 5) + 1] |= code >> (32 - (bit & 31));
    dq[j] = ldexp(y < 0.0 ? -q : q, e);
  }
}
// tile image slot of (matrix row rho, 32-column storage block bI): tile (rho / MXK, bI / 4), plane
// bI & 3, 32-byte slot of the row, halves swapped on rows with (row >> 3) & 1
__host__ __device__ inline void fp6_store(uint32_t *tiles, int nK, int64_t rho, int64_t bI, const uint32_t wds[8]) {
  const int64_t kb = rho / MXK, row = rho % MXK, cs = bI >> 2, plane = bI & 3;
  uint32_t *dst = tiles + ((kb * nK + cs) * MX_TILE + plane * 4096 + row * 32) / 4;
  const int sw = (int)((row >> 3) & 1) * 4;
  for (int k = 0; k < 8; ++k) dst[(k + sw) & 7] = wds[k];
}







// stage-blocked 2-bit genotype codes (the prefilters' code stream): per SNP and 16 individuals a dword
// whose nibble k holds c[k] | c[8 + k] << 2 (fp4_of_code2 expands it with two VALU per fp4 dword);
// dst[(st m + snp) 16 B + 4 g] for the stage st's 16-individual group g
// ---- U = codes x P on the int8 matrix cores (the codings' side vectors; fp64 GEMM: 10.5 ms per coding
// at configs[2], this 2-3 ms).  P in U8_S int8 slices per row q with the row's unit u_q = max_r |P_qr| / 127:
//   P_qr = u_q sum_s 128^-s B_s[q][r] + R_qr,  |R_qr| <= u_q 128^-(U8_S-1) / 2 = u_q 2^-50,
// so T_s = codes x B_s' is an exact int32 sum (|T_s| <= 254 n_pad) and U[j][q] = u_q sum_s 128^-s T_s[j][q]
// is off by at most 2 n_pad u_q 2^-50 (below the fp64 GEMM's own rounding bound, 2 n_pad 2^-53 max |P|
// per row, times 8 n_pad / 127 -- ~2^-46 relative to the row's largest |P| at n_pad = 2048).  P is
// symmetric: row q is column q.
// Operands per stage of 64 individuals (SG_K): the codes from the 2-bit stage-blocked panel (p2b, 16 B per
// SNP and stage, code2_panel_kernel) expanded to int8 in registers; the slices stage-blocked as
// [stage][slice][q][64 B] with the 16-byte chunks XOR-swizzled by q & 31 (u8_swz: conflict-free
// ds_read_b128 of the B fragments) and the bytes of a chunk in the expansion's individual order
// (0 2 4 6 1 3 5 7 8 10 12 14 9 11 13 15).  A workgroup: 256 SNPs x 32 columns q, 8 waves of 32 SNPs
// (v_mfma_i32_32x32x32_i8, one accumulator per slice), a four-slot LDS-DMA ring (three stages in
// flight).
constexpr int U8_S = 8, U8_J = 256, U8_Q = 32, U8_NS = 4, U8_AB = U8_J * 16, U8_ST = U8_AB + U8_S * U8_Q * 64;
__host__ __device__ inline int u8_swz(int q) { return (q & 3) ^ ((q >> 3) & 3); }
__host__ __device__ inline int u8_pos(int t16) {  // byte position of individual t16 (0..15) in its chunk
  return (t16 & 8) + ((t16 & 1) ? 4 : 0) + ((t16 & 7) >> 1);
}
// int8 values of the 16 genotype codes of one dword of the 2-bit panel (nibble k = c[k] | c[8 + k] << 2),
// in the order 0 2 4 6 | 1 3 5 7 | 8 10 12 14 | 9 11 13 15
__device__ __forceinline__ v4i i8_of_code2(unsigned d) {
  const unsigned lo = d & 0x33333333u, hi = (d >> 2) & 0x33333333u;
  return v4i{(int)(lo & 0x0f0f0f0fu), (int)((lo >> 4) & 0x0f0f0f0fu), (int)(hi & 0x0f0f0f0fu), (int)((hi >> 4) & 0x0f0f0f0fu)};
}



inline double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}


// ------------------------------------------------------------------ plan object

// ---- tile lists of the low-rank screen built on the device from the prefilter's flags (the host
// builder of build_mx, restated): per 32-column block J the flagged band rows in row order, packed
// into half-tiles of MX_BI/2 rows, consecutive half-tiles (J-major) paired into MX tiles, tile t
// dealt to entry 8 (t mod C) + t / C (C = ceil(tiles / 8): the 8 XCDs get contiguous chunks),
// padding entries -1.  Thread (jl, rg) of a 1024-thread workgroup: column block 64 b + jl, rows
// [TL_R rg, TL_R rg + TL_R) (16 row groups: short load chains, 16 waves per column group).
constexpr int TL_G = 16, TL_R = ROWS_PER_LAUNCH / TL_G;  // row groups, band rows per thread
__device__ __forceinline__ int tl_total(const int *cnt, int J) {
  int c = 0;
#pragma unroll
  for (int g = 0; g < TL_G; ++g) c += cnt[TL_G * J + g];
  return c;
}

// ---- slot lists of the compacted low-rank screen (lrc_screen_kernel), built on the device from the
// prefilter's live-pair masks: band row r's live pairs, in ascending j, are cut into slots of 32
// (the last one padded with -1); slot s = (slot_row[s], slot_j[32 s .. 32 s + 31]).  Slots are
// numbered row by row and grouped 16 to a tile; the padding slots of the last tile have row -1.
// lc_count: live pairs per band row (one workgroup per row).
constexpr int LC_T = 256, LC_SLOTS = MX_BI;  // threads per row; slots per tile


}  // namespace epi
}  // namespace gmat

using namespace gmat;
using namespace gmat::epi;

struct Coding {
  bool ready = false;
  bool side_ready = false;        // Lq / Ldq / Rq built (block_sides)
  DBuf U;                         // P * screen code panel  [m][n_pad] (fp64, while the coding is built)
  DBuf U16;                       // the same rounded to fp16 (pair screen side terms)
  DBuf off;                       // alpha/beta of the reference codes (refine) [m]
  DBuf soff;                      // centring offsets of the screen codes [m]
  DBuf sq;                        // squared screen codes (additive coding only) [m][n_pad]
  DBuf Lq, L3q, Ldq, Rq;          // side vectors L', L3, Ld, R' as int8 slices [SIDE_T][m][n_pad]
  DBuf sL, sL3, sLd, sR, csum, csq;  // their per-SNP scales; per-SNP sums of codes / squared codes
  DBuf qa, ra, sa, qb, rb, sb;    // per-SNP scalars
  DBuf mono;                      // uint8 [m]
  DBuf nibI, nibJ;                // MX screen nibble planes (i side M1/M2, j side S1/S2) [m][nK][128]
  DBuf s1c2;                      // the S1 planes at 2 bits (compacted low-rank screen) [m][nK][32]
  DBuf p4;                        // screen codes as fp4 e2m1 [m][n_pad / 2] (prefilter)
  DBuf p2b, L3b;                  // stage-blocked copies for the prefilters: 2-bit codes [n_pad/64][m][16 B]
                                  // (code2_panel_kernel), L3q slices 0 .. E3_PF-1 [E3_PF][n_pad/64][m][64 B]
  DBuf pfRecL, pfRecR;            // prefilter test records, row / column role [m][PF_REC] fp32
  DBuf uc;                        // covariate directions: u_k . code [ncov][m]
  DBuf lrG, lrGa;                 // low-rank screen: Q' x screen codes, fp32 [m][lr_R]; the same minus
                                  // soff x Q'1 (left side: folds the alpha beta q1 term)
  DBuf lrRecL, lrRecR;            // low-rank screen test records [m][LR_REC] (left / right roles)
};

// pinned host staging buffer (grown on demand, kept by the plan across scans)
struct Pinned {
  void *p = nullptr;
  size_t cap = 0;
  ~Pinned() { pinned_free(p, cap); }
  int reserve(size_t n) {
    if (n <= cap) return GMAT_OK;
    pinned_free(p, cap);
    p = nullptr;
    cap = 0;
    size_t got = 0;
    p = pinned_alloc(n, &got);
    if (!p) return GMAT_E_NOMEM;
    cap = got;
    return GMAT_OK;
  }
  template <class T>
  T *as() const {
    return (T *)p;
  }
};

namespace gmat {
namespace epi {
struct SegPlan;               // a plan cut into SNP segments (epi_seg.hip)
void seg_free(SegPlan *sp);
}  // namespace epi
}  // namespace gmat

struct gmat_epi {
  gmat_geno *g = nullptr;
  int64_t n = 0, n_pad = 0, m = 0;
  int n_slice = 3;
  // Past the single-plan limits (epi_seg.hip): a plan whose panels would need byte offsets of 2^32 or
  // more (2 m n_pad) is cut into SNP segments, each scan running on sub-plans of one or two segments
  // (seg); a plan with n_pad > EXH_ONLY_NPAD individuals has no screens (the int8 screen's 24-bit
  // epilogue sums and the pair screen's LDS planes stop there) and scans every pair exactly
  // (exh_only).  col_lo: the first second SNP a scan of this plan tests (a segment pair's sub-plan
  // [A, B] scans rows of A against columns of B only); 0 otherwise.
  gmat::epi::SegPlan *seg = nullptr;
  bool exh_only = false;
  int64_t col_lo = 0;
  double qmax = 0, zz = 0, spy = 0;
  double rho[5] = {0, 0, 0, 0, 0};  // rho[S]: upper bound of ||P_off - sum_{s<S} A_s 128^-s qmax/127||_2
                                    // (0: not computed yet, ensure_rho)
  double pmax = 0;                  // max |P|
  double rho_mx = 0;                // the MX screen's bound: ||P_off - E||_2 + fp32 accumulation term
  // spectral prefilter: e'Pe >= pf_mu * (|e|^2 - (1'e)^2 / n) - pf_eps * |e|^2 for every e,
  // certified by a Cholesky factorisation of P + pf_mu (11'/n - I); pf_mu = 0: disabled
  double pf_mu = 0, pf_tau = 0, pf_eps = 0;
  // covariate designs: pf_ncov null directions of P besides 1 enter the certificate with weight pf_ku
  int pf_ncov = 0;
  double pf_ku = 0, pf_su[4] = {0, 0, 0, 0};
  DBuf pf_U;  // [pf_ncov][n_pad] the directions in storage order
  DBuf pf_q;  // [pf_ncov][n_pad] int8: rint(u_k / pf_sq[k]), |q| <= 63 (ensure_pf_q)
  double pf_sq[4] = {0, 0, 0, 0};
  // low-rank screen (lr_screen_kernel): e'Pe >= lam |Pi e|^2 - tau (1'e)^2/n - eps |e|^2 - |Q'e|^2
  // with Q = fp6(bottom eigenvectors x sqrt(d)); lr_R = padded rank (0: disabled)
  int lr_R = 0;
  double lr_lam = 0, lr_tau = 0, lr_eps = 0;
  double lr_E = 0;                  // sum_r eta_r^2 (the screen's fp32 error budget)
  DBuf lr_tiles, lr_Bs, lr_q1;      // Q' tile images; Q fp64 [n_pad][lr_R] storage order; Q'1 (fp64)
  int nK = 0;                       // 128-individual stages
  DBuf rf_part;                     // refine segment partials [2][nseg][np]
  DBuf r8_tiles, r8_varw;           // refine8: int8 slice tiles of the block-upper P_off; w'P_off w per pair
  DBuf u8_slices, u8_unit;          // U = codes x P on int8 MFMA: the slices of P by row, their units
  double r8_unit = 0;               // their unit (2 qmax / 127)
  DBuf Ps, py, z, dg, slices;
  DBuf mx_tiles;                    // fp6 P_off tile images with e8m0 scales (MX screen)
  DBuf spanels;  // screen codes, one allocation: [0] minor-allele dosage, [1] heterozygote [m][n_pad]
  Coding code[2];  // 0 = additive (dosage), 1 = dominance (het)
  // scan state
  DBuf cand_i, cand_j, counter, ceff, cvar, cchi, cp;
  DBuf cand2_i, cand2_j, counter2, ps_side;  // pair screen survivors; its per-pair side terms
  DBuf cpack;                                 // the refined candidates' hits packed for the read-back
  DBuf hcount;                                // their count (hit_pack_kernel)
  DBuf ps_mpart;                              // pair_mxr_kernel's segment partials
  int64_t cand_cap = 0;
  std::vector<int64_t> hit_i, hit_j;
  std::vector<double> hit_eff, hit_var, hit_chi, hit_p;
  double stats[10] = {0};
  // per-kernel accounting of the last compacted low-rank scan (gmat_epi_kernel_stats): [0] prefilter
  // kernel seconds (HIP events on its stream), [1] its launches, [2] its MFMA ops (fp4-equivalent:
  // fp4 ops + 2 x int8 ops, the rate ratio), [3] low-rank screen seconds, [4] its launches,
  // [5] its fp6 x fp4 ops (R n_pad MACs x 2 per slot pair, empty slots included), [6] pair screen +
  // refine seconds at flush, [7] live pairs (GMAT_LIVE_COUNT) or -1
  double kstats[8] = {0};
  // per-kernel timers of the candidate kernels (gmat_epi_kernel_stats_ext): HIP event pairs recorded on
  // the kernel's stream around each launch, read after the scan; kernel ids KT_*
  std::vector<hipEvent_t> kev;
  size_t kev_used = 0;
  std::vector<hipEvent_t> sev;  // the scans' pipeline events (ScanEvents), created once
  struct KMark {
    int kernel;
    size_t ev;
    double pairs;
  };
  std::vector<KMark> kmarks;
  // plan setup seconds: [0] gmat_epi_create total, [1] prefilter certificate, [2] eigendecomposition,
  // [3] low-rank certificate, [4] slices + residual bounds, [5] coding builds (side vectors, lazily
  // in the first scan of a kind), [6] Cholesky factorisations run by the certificates
  double setup[8] = {0};
  uint64_t p_hash = 0;  // fingerprint of P (guards imported spectral state)
  int imported = 0;     // spectral state imported from another plan (gmat_epi_create_with)
  int n_cu = 0;         // compute units of the device (persistent prefilter grid), queried on first use
  hipStream_t s = 0;
  // scan work buffers, two sets (kept across scans of the plan: allocation is not free)
  struct ScanBufs {
    DBuf drows[2], dtiles[2], bl[2], ba[2], e13[2], e2[2], pfc[2], flags[2], mxt[2], mxr[2];
  } sb;
  // pinned host staging of the scan pipeline (hipHostMalloc is slow: allocated once per plan)
  struct ScanPins {
    Pinned res, rows[3], flags[3], mxt[3], mxr[3], t2[3], cnt[3], count2, tl[3];
  } pins;
  hipStream_t s1 = nullptr, s2 = nullptr, s3 = nullptr;  // scan pipeline: screen / side terms / refine
  hipStream_t s4 = nullptr;  // the compacted scan's second prefilter stream (odd launches)
  hipStream_t s5 = nullptr;  // the int8 refine's O(n) terms beside refine8_kernel
  hipEvent_t r8ev[2] = {nullptr, nullptr};  // refine(): fork / join of that stream
  DBuf r8_terms;                            // refine8_side_kernel's terms [R8_NT][np]
  struct LrcBuffers {  // three sets: the prefilters of launches L + 1 and L + 2 are queued while L screens
    DBuf drows[3], lmask[3], ops[3], opc[3], slot_ops[3], slot_row[3], slot_j[3], cnt[3], soff[3], info[3], tlist[3];
    int64_t rl = 0, ops_cap = 0, slot_cap = 0;  // the sets' rows per launch, record and slot capacities
                                                // (grown, never shrunk)
    unsigned ltag[3] = {0, 0, 0};               // the live-block entries' tag of each set's last launch
    void *lm_ptr[3] = {nullptr, nullptr, nullptr};  // the entry buffer that tag refers to
  } lrc;  // compacted low-rank scan buffers (scan_lowrank)
  ~gmat_epi() {
    gmat::epi::seg_free(seg);
    for (auto ev : kev) (void)hipEventDestroy(ev);
    for (auto ev : sev) (void)hipEventDestroy(ev);
    for (hipStream_t st : {s1, s2, s3, s4, s5})  // the device's pipeline streams (shared): drained, kept
      if (st) (void)hipStreamSynchronize(st);
    for (auto ev : r8ev)
      if (ev) (void)hipEventDestroy(ev);
  }
};


namespace gmat {
namespace epi {

// ---- kernels (defined in the stage files)
template <int PASS>
__global__ void side_gemm_kernel(SideArgs x);
template <bool LIST, bool COMPACT, bool STAMP, int TR, int NS>
__global__ void prefilter_pass_kernel(SideArgs x);
template <int NC, bool LIST, int TC>
__global__ void prefilter_cov_kernel(SideArgs x);
template <int SH>
__global__ void screen_kernel(ScreenArgs a);
template <int V>
__global__ void mx_screen_kernel(ScreenArgs a, MxArgs x);
template <int SK, int NSL>
__global__ void lr_screen_kernel(ScreenArgs a, LrArgs x);
template <int NSL>
__global__ void lrc_screen_kernel(ScreenArgs a, LrcArgs x);
__global__ void lr_rec_kernel(int64_t m, const double *soff, const double *csum, const double *csq, const double *sL3,
                              const double *sa, const double *sb, const uint8_t *mono, double *recL, double *recR);
__global__ void refine_kernel(int64_t n_pad, const double *__restrict__ P,
                                                       const double *__restrict__ py, const int8_t *left,
                                                       const int8_t *right, const double *alpha, const double *beta,
                                                       const int64_t *pi, const int64_t *pj, int64_t np, double *eff,
                                                       double *var, double *eff_part, double *var_part);
__global__ void refine_sum_kernel(int64_t np, int nseg, const double *eff_part, const double *var_part, double *eff,
                                  double *var);
__global__ void pvalue_kernel(int64_t np, const double *eff, const double *var, double *chi, double *p);
__global__ void r8_image_kernel(int64_t n_pad, const double *__restrict__ Ps, double inv_unit, int8_t *__restrict__ tiles);
__global__ void refine8_kernel(int64_t n_pad, const int8_t *__restrict__ tiles,
                                                         const int8_t *__restrict__ sl, const int8_t *__restrict__ sr,
                                                         const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                         int64_t np, double unit, double *__restrict__ varw,
                                                         double *__restrict__ tpart);
__global__ void refine8w_kernel(int64_t n_pad, const int8_t *__restrict__ tiles,
                                                          const int8_t *__restrict__ sl, const int8_t *__restrict__ sr,
                                                          const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                          int64_t np, double *__restrict__ tpart);
__global__ void refine8_side_kernel(int64_t n_pad, const int8_t *__restrict__ sl,
                                                           const int8_t *__restrict__ sr, const double *__restrict__ Ua,
                                                           const double *__restrict__ Ub, const double *__restrict__ z,
                                                           const double *__restrict__ dg, const double *__restrict__ py,
                                                           const int8_t *__restrict__ lp, const int8_t *__restrict__ rp,
                                                           const double *soff_l, const double *soff_r, const double *off_l,
                                                           const double *off_r, const double *qa, const double *ra,
                                                           const double *qb, const double *rb, double zz,
                                                           const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                           int64_t np, double *__restrict__ terms);
__global__ void refine8_fin_kernel(int64_t np, const double *__restrict__ terms, const double *soff_l,
                                   const double *soff_r, const double *qa, const double *ra, const double *qb,
                                   const double *rb, double zz, const uint8_t *mono_l, const uint8_t *mono_r,
                                   const int64_t *__restrict__ pi, const int64_t *__restrict__ pj, const double *varw,
                                   int nseg, const double *tpart, double unit, double *eff, double *var, double *chi,
                                   double *pv);
__global__ void pair_side_kernel(PairArgs x);
__global__ void pair_mxr_kernel(PairArgs x);
__global__ void pair_mxw_kernel(PairArgs x);
__global__ void pair_test_kernel(PairArgs x, int nseg);
__global__ void permute_p_kernel(int64_t n, int64_t n_pad, const double *P, double *Ps);
__global__ void permute_vec_kernel(int64_t n, int64_t n_pad, const double *v, double *vs);
__global__ void slice_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                             int8_t *slices);
__global__ void residual_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                                double out_scale, double *R);
__global__ void left_side_kernel(int64_t n_pad, const int8_t *panel, const double *U,
                                                        const double *z, const double *py, const double *dg,
                                                        const double *alpha, double *Lp, double *L3, double *Ld,
                                                        double *qa, double *ra, double *sa);
__global__ void right_side_kernel(int64_t n_pad, const int8_t *panel, const double *V,
                                                         const double *z, const double *py, const double *beta,
                                                         double *Rp, double *qb, double *rb, double *sb);
__global__ void quantize_rows_kernel(int64_t n_pad, int64_t slice_stride, const double *v,
                                                            int8_t *q, double *scale);
__global__ void gather_band_kernel(int64_t n_pad, int R, int64_t slice_stride, const int64_t *rows, const int8_t *Lq,
                                   const int8_t *L3q, const int8_t *Ldq, const int8_t *panel, const int8_t *sqpanel,
                                   int8_t *BL, int8_t *BA);
__global__ void i8gemm_nt_kernel(int M, int N, int K, const int8_t *__restrict__ A, int64_t lda,
                                                        int64_t za, const int8_t *__restrict__ B, int64_t ldb,
                                                        int64_t zb, int *__restrict__ C, int64_t ldc, int64_t zc);
__global__ void flip_panel_kernel(int64_t n, int64_t n_pad, int64_t m, const int8_t *src, const uint8_t *flip,
                                  int8_t *dst, int8_t *sq);
__global__ void diag_kernel(int64_t n_pad, const double *Ps, double *dg);
__global__ void zsum_kernel(int64_t n_pad, const double *Ps, double *z);
__global__ void mx_quant_kernel(int64_t n, int64_t n_pad, int nK, const double *P, uint32_t *tiles, double *Qn);
__global__ void mx_residual_kernel(int64_t n, int64_t n_pad, const double *P, const double *Qn,
                                                          double out_scale, double *R, double *rowabs);
__global__ void nibble_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *nib_i,
                              uint32_t *nib_j);
__global__ void s1_code2_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *out);
__global__ void p_scan_kernel(int64_t n, const double *P, double *out);
__global__ void pf_shift_kernel(int64_t n, const double *P, double mu, double tau, double *A);
__global__ void pf_shift_u_kernel(int64_t n, const double *P, const double *C, double mu, double tau, double ku,
                                  double *A);
__global__ void cov_dot_kernel(int64_t n_pad, const int8_t *panel, const double *u, double *dot);
__global__ void block_panel_perm8_kernel(int64_t m, int64_t W, int64_t w, const uint8_t *__restrict__ src,
                                         uint8_t *__restrict__ dst);
__global__ void pf_rec_kernel(int64_t m, double n, double spy, const double *__restrict__ soff,
                              const double *__restrict__ csum, const double *__restrict__ csq,
                              const double *__restrict__ sL3, const double *__restrict__ sa,
                              const double *__restrict__ sb, const uint8_t *__restrict__ mono, float *recL,
                              float *recR);
__global__ void fp4_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint8_t *p4);
__global__ void u8_unit_kernel(int64_t n_pad, const double *__restrict__ Ps, double *__restrict__ unit);
__global__ void u8_slice_kernel(int64_t n_pad, const double *__restrict__ Ps, const double *__restrict__ unit,
                                int8_t *__restrict__ out);
__global__ void u8_gemm_kernel(int64_t m, int64_t n_pad, const uint8_t *__restrict__ p2b,
                                                         const int8_t *__restrict__ slices, const double *__restrict__ unit,
                                                         double *__restrict__ U);
__global__ void code2_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint32_t *dst);
__global__ void lr_shift_kernel(int64_t n, const double *P, const double *C, double lam, double tau, double *A);
__global__ void lr_adjust_kernel(int64_t m, int64_t R, const double *G, const double *soff, const double *q1, float *out);
__global__ void f64_to_f16_kernel(int64_t count, const double *src, _Float16 *dst);
__global__ void f64_to_f32_kernel(int64_t count, const double *src, float *dst);
__global__ void tl_count_kernel(const uint8_t *__restrict__ flags, int Rn, int nJ,
                                                        int *__restrict__ cnt4);
__global__ void tl_scan_kernel(const int *__restrict__ cnt4, int nJ, int *__restrict__ H,
                                                       int *__restrict__ info, int *__restrict__ mxt,
                                                       int *__restrict__ mxr);
__global__ void tl_fill_kernel(const uint8_t *__restrict__ flags, int Rn, int nJ,
                                                      const int *__restrict__ cnt4, const int *__restrict__ H,
                                                      const int *__restrict__ info, int *__restrict__ mxt,
                                                      int *__restrict__ mxr);
__global__ void lc_count_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ, int Rn,
                                                        int *__restrict__ cnt);
__global__ void lc_scan_kernel(const int *__restrict__ cnt, int Rn, int *__restrict__ soff,
                                                       int *__restrict__ info, int *__restrict__ slot_row,
                                                       int64_t slot_cap);
__global__ void lc_fill_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ, int Rn,
                                                       const int *__restrict__ cnt, const int *__restrict__ soff,
                                                       int *__restrict__ slot_row, int *__restrict__ slot_j,
                                                       const int *__restrict__ ops, int64_t ops_cap,
                                                       int *__restrict__ slot_ops, int64_t slot_cap);
__global__ void lr_quant_kernel(int64_t n, int64_t n_pad, int nK, int Rp, const double *__restrict__ Z,
                                const double *__restrict__ sd, double *__restrict__ Bn, double *__restrict__ Bs,
                                uint32_t *__restrict__ img);
__global__ void all_pairs_kernel(const int64_t *__restrict__ rows, const int64_t *__restrict__ offs, int64_t m, int tri,
                                 int64_t col_lo, int64_t *__restrict__ pi, int64_t *__restrict__ pj);
__global__ void hit_compact_kernel(int64_t np, const int64_t *__restrict__ pi,
                                                          const int64_t *__restrict__ pj, const double *__restrict__ eff,
                                                          const double *__restrict__ var, const double *__restrict__ chi,
                                                          const double *__restrict__ p, double p_cut,
                                                          unsigned long long *count, int64_t *hi, int64_t *hj,
                                                          double *he, double *hv, double *hc, double *hp);
__global__ void audit_kernel(int64_t n, int64_t n_pad, int R, int ncov, const int8_t *left,
                                                      const int8_t *right, const double *alpha, const double *beta,
                                                      const int64_t *pi, const int64_t *pj, const double *Q,
                                                      const double *U, double pf_mu, double pf_tau, double pf_eps,
                                                      double pf_ku, double lr_lam, double lr_tau, double lr_eps,
                                                      double *out);
__global__ void hit_pack_kernel(int64_t n, const int64_t *ci, const int64_t *cj, const double *eff, const double *var,
                                const double *chi, const double *p, double p_cut, double *out, unsigned long long *count);

constexpr int AUD_T = 256;  // audit_kernel workgroup (the low-rank rank it serves at most)

// ---- host pieces shared by epi_plan.hip / epi_scan.hip / epi_seg.hip
// kernel timers (gmat_epi_kernel_stats_ext): kernel ids, a launch's start / end events on its stream
enum { KT_PAIR_SIDE = 0, KT_PAIR_MX = 1, KT_REFINE = 2, KT_REFINE_SIDE = 3, KT_N = 4 };
int kt_begin(gmat_epi *e, hipStream_t st, size_t *idx);
int kt_end(gmat_epi *e, hipStream_t st, int kernel, size_t beg, double pairs);
// screen panel of a coding (inside e->spanels) and its squared codes (B operand of the Ld term)
const int8_t *screen_panel(const gmat_epi *e, int which);
const int8_t *screen_sq(const gmat_epi *e, int which);
// codings of a scan kind (0 additive, 1 dominance) for the left / right SNP; builds one on first use
void kind_codings(int kind, int *lc, int *rc);
int build_coding(gmat_epi *e, int which);
// the int8 levels' residual bound rho[S] (computed on first use)
int ensure_rho(gmat_epi *e, int S);
// exact statistics of device pair lists (epi_plan.hip: refine8 / refine8w + refine8_side, or the fp64 refine)
int refine(gmat_epi *e, hipStream_t st, const Coding &L, const Coding &R, const int8_t *lp, const int8_t *rp,
           const int64_t *pi, const int64_t *pj, int64_t np, double *eff, double *var, double *chi, double *p);
// the pair screen between the low-rank screen and the refine (survivors to e->cand2_*)
bool pair_screen_fits(const gmat_epi *e);
int default_lr_rank(const gmat_epi *e);
int pair_screen(gmat_epi *e, hipStream_t st, const Coding &L, const Coding &R, const int8_t *slp, const int8_t *srp,
                const int64_t *pi, const int64_t *pj, int64_t np, double chi_cut, int64_t *n_out, bool reset = true);
// plan creation (epi_plan.hip): a plan of one panel (state: another plan's spectral state, or null)
// (allow_seg false: a plan of this one panel even when seg_snps() would cut it -- the segments' sub-plans)
int epi_create_impl(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                    const uint8_t *state, int64_t state_bytes, bool allow_seg = true);
constexpr int64_t EXH_ONLY_NPAD = 8192;  // plans past this many (padded) individuals scan exhaustively
// whether a plan for g is cut into SNP segments, and the segment size (epi_seg.hip)
int64_t seg_snps(const gmat_geno *g);
int seg_create(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice, const uint8_t *state,
               int64_t state_bytes);
// the scan of a validated row list on a plan of one panel (gmat_epi_scan without the checks), epi_scan.hip
int scan_dispatch(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut, int n_slice,
                  int64_t *n_hits);
// segmented plans' scan / pair statistics / bound audit (epi_seg.hip)
int seg_scan(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut, int n_slice,
             int64_t *n_hits);
int seg_pairs(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *eff, double *var, double *chi,
              double *p);
int seg_audit(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *out5);
const gmat_epi *seg_base(const gmat_epi *e);  // the plan of segment 0 (spectral state, setup statistics)
// batched int8 GEMM C = A B' (the block-granular scans' side GEMMs), epi_setup.hip
int i8gemm_nt(hipStream_t st, int Z, int M, int N, int K, const int8_t *A, int64_t lda, int64_t za, const int8_t *B,
              int64_t ldb, int64_t zb, int *C, int64_t ldc, int64_t zc);


}  // namespace epi
}  // namespace gmat

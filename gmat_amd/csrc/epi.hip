// Exhaustive epistasis scans (remma_epiAA.py:71-82, remma_epiAD.py:76-87,
// remma_epiDD.py:75-86) and the pair-list test (remma_epiAA_pair.py:79-84).
//
// For a pair (i, j) with centred codes x_i = a_i - alpha_i, x_j = b_j - beta_j (a, b the
// integer 0/1/2 dosage or 0/1 heterozygote codes), the reference computes
//     e = x_i o x_j,  eff = e'Py,  var = e'Pe  (2n^2 fp64 flop per pair),
// chi = eff^2/var, p = chi2.sf(chi, 1), and keeps p < p_cut.
//
// Here the scan runs in two passes:
//  1. SCREEN.  The screen codes count the MINOR allele (a~ = 2 - a when 2p > 1, which only
//     flips the sign of x and leaves e'Pe unchanged), so w = a~_i o b~_j (integers 0..4)
//     stays small.  The quadratic form expands into
//       e'Pe = w'P_off w + sum_q P_qq w_q^2 - 2 beta L'_i.b_j - 2 alpha a_i.R'_j + (per-SNP
//              and constant terms),
//     L'_i = a_i o (P a_i - alpha_i P1),  R'_j = x_j o (P b_j).
//     The O(n^2)-per-pair term w'P_off w (P without its diagonal) is evaluated EXACTLY for a
//     sliced P_off:
//       P_off ~ (qmax/127) sum_s 128^-s A_s,  A_s int8,  qmax = max |P_kl| (k != l),
//     as integer quadratic forms on v_mfma_i32_32x32x32_i8 (int32 accumulation, int64
//     combination -- bit-deterministic), using the symmetry of A_s to visit only the
//     block-upper half.  The O(n)-per-pair side terms (diagonal included) are int8-sliced
//     MFMA GEMMs.  The slicing error is bounded rigorously by delta * sum w^2, so every pair
//     that COULD have p < p_cut becomes a candidate.  Minor-allele codes and the diagonal
//     split make the one-slice bound tight enough for small p_cut (half the MFMA work of two).
//  2. REFINE.  Candidates are re-evaluated exactly as the reference does (fp64 e = x_i*x_j,
//     var = e'Pe on f64 MFMA, p = erfc(sqrt(chi/2))) and the hits are kept.
// The reported statistics therefore come from the same fp64 formula as the reference;
// the screen only decides which pairs need it.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <numeric>


#include "dla.h"
#include "geno.h"

using namespace gmat;

namespace {

typedef int v2i_ __attribute__((ext_vector_type(2)));
typedef int v8i_ __attribute__((ext_vector_type(8)));
typedef float v16f_ __attribute__((ext_vector_type(16)));
typedef float v2f_ __attribute__((ext_vector_type(2)));

constexpr int LK = 64;   // inner (individual) depth per LDS stage
constexpr int AP = 80;   // LDS pitch of a 64-byte row (conflict-free ds_read_b128)
constexpr int BJ = 32;   // second-SNP columns per screen tile
constexpr int ROWS_PER_LAUNCH = 512;       // first SNPs per launch of the block-granular scan
constexpr int LRC_ROWS_PER_LAUNCH = 4096;  // ... and of the compacted low-rank scan
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
  if (j >= a.m || (a.tri && j <= i)) return;
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
template <int PASS>
__global__ __launch_bounds__(256, 2) void side_gemm_kernel(SideArgs x) {
  // PASS 2: E1 (L'q_t x b), PASS 3: Ed (Ldq_t x b^2), PASS 4: E2 (a x R'q_t) -- three int8 products
  // each, written for the blocks the prefilter flagged (the MX quadratic-form screen's side terms)
  static_assert(PASS >= 2 && PASS <= 4, "PASS 1 is prefilter_pass_kernel");
  constexpr int NR = PASS == 4 ? 1 : 3, NC = PASS == 4 ? 3 : 1, NPR = 3;
  const ScreenArgs &a = x.a;
  // XCD-aware tile order: workgroup b runs on XCD b mod 8; the bijective remap gives each XCD a
  // contiguous range of tiles, so the n_rt row tiles of a column tile share one L2
  const int nwg = (int)gridDim.x, xq = nwg / 8, xr = nwg % 8, xcd = (int)blockIdx.x % 8;
  const int tile = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + (int)blockIdx.x / 8;
  const int rt = tile % x.n_rt, ct = tile / x.n_rt;
  const int r0 = rt * SG_T;
  const int64_t c0 = (a.j_lo / 32) * 32 + (int64_t)ct * SG_T;  // 32-aligned: a half-wave = one block
  if (r0 >= a.n_rows || c0 >= a.m) return;
  if (a.tri && c0 + SG_T - 1 <= a.rows[r0]) return;  // tiles left of the diagonal hold no pair
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1, h = lane >> 5, c = lane & 31;
  // product p: (row set, column set)
  constexpr int PR[3][3] = {{0, 1, 2}, {0, 1, 2}, {0, 0, 0}};
  constexpr int PC[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 1, 2}};
  v16i acc[NPR];
#pragma unroll
  for (int p = 0; p < NPR; ++p)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[p][e] = 0;
  __shared__ __attribute__((aligned(16))) int8_t sR[2][NR][SG_T * SG_P];
  __shared__ __attribute__((aligned(16))) int8_t sC[2][NC][SG_T * SG_P];
  // staging: chunk q of an int8 set = (tile row q >> 2, 16-byte piece q & 3); 256 chunks per set
  const int srow = tid >> 2, spc = (tid & 3) * 16;
  const int64_t si = a.rows[min(r0 + srow, a.n_rows - 1)];
  const int64_t sj = min(c0 + srow, a.m - 1);
  v4i rv[NR], cv[NC];
  auto load = [&](int k0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NR; ++u) rv[u] = *(const v4i *)(x.rs[u] + si * x.n_pad + k0 + spc);
#pragma unroll
    for (int u = 0; u < NC; ++u) cv[u] = *(const v4i *)(x.cs[u] + sj * x.n_pad + k0 + spc);
  };
  auto store = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NR; ++u) *(v4i *)&sR[b][u][srow * SG_P + spc] = rv[u];
#pragma unroll
    for (int u = 0; u < NC; ++u) *(v4i *)&sC[b][u][srow * SG_P + spc] = cv[u];
  };
  load(0);
  store(0);
  __syncthreads();
  int b = 0;
  for (int k0 = 0; k0 < x.n_pad; k0 += SG_K) {
    const bool more = k0 + SG_K < x.n_pad;
    if (more) load(k0 + SG_K);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v4i fr[NR], fc[NC];
#pragma unroll
      for (int u = 0; u < NR; ++u) fr[u] = *(const v4i *)&sR[b][u][(32 * wr + c) * SG_P + 32 * kk + 16 * h];
#pragma unroll
      for (int u = 0; u < NC; ++u) fc[u] = *(const v4i *)&sC[b][u][(32 * wc + c) * SG_P + 32 * kk + 16 * h];
#pragma unroll
      for (int p = 0; p < NPR; ++p)
        acc[p] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fr[PR[PASS - 2][p]], fc[PC[PASS - 2][p]], acc[p], 0, 0, 0);
    }
    if (more) store(b ^ 1);
    __syncthreads();
    b ^= 1;
  }
  // epilogue: lane (c, h) holds rows 32 wr + (e & 3) + 8 (e >> 2) + 4h, column 32 wc + c
  const int64_t j = c0 + 32 * wc + c;
  const int J = (int)(j / 32);
  const bool jok = j < a.m && j >= a.j_lo;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int r = r0 + 32 * wr + (e & 3) + 8 * (e >> 2) + 4 * h;
    if (r >= a.n_rows || !jok || !a.flags[(int64_t)r * a.nJ + J]) continue;
    const int64_t o1 = (int64_t)r * a.ld_e + (j - a.j_lo), od = o1 + 2 * (int64_t)a.n_rows * a.ld_e;
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t) {
      if (PASS == 2) ((int *)a.c13)[t * a.c13_stride + o1] = acc[t][e];
      if (PASS == 3) ((int *)a.c13)[t * a.c13_stride + od] = acc[t][e];
      if (PASS == 4) ((int *)a.c2)[t * a.c2_stride + o1] = acc[t][e];
    }
  }
}

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
// issuing q = w + 8u (u < 2; waves 0-4 two, 5-7 one).
constexpr int PF_TR = 64, PF_TC = 256, PF_ST = 13 * 1024, PF_NS = 5, PF_NQ = 13;
constexpr int PF_REC = 8;  // floats per prefilter test record (pf_rec_kernel)
constexpr int PF_CHUNK = 128;  // live-pair records a persistent prefilter wave reserves at a time
constexpr int PF_NSTAMP = 7;  // GMAT_PF_STAMPS: start, prologue, main loop, column records, tests, stores, end
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
// COMPACT: the compacted low-rank path's output (live masks + one record per live pair at a.ops); else
// the block-granular path's (flags + E3 and code products of every pair of a live block, dense)
template <bool LIST, bool COMPACT>
__global__ __launch_bounds__(512, 1) void prefilter_pass_kernel(SideArgs x) {
  const ScreenArgs &a = x.a;
  // The workgroup's tiles.  With a tile list (the launch's running tiles), XCD x (workgroup b runs on
  // XCD b mod 8) takes the list's x-th eighth and its G workgroups stride through it: a persistent
  // grid, in which the next tile's records and first stages stream into LDS while the current tile's
  // epilogue runs.  Without one, the workgroup's single tile of the XCD-aware remap, if it has a pair.
  const int xcd = (int)blockIdx.x % 8, kw = (int)blockIdx.x / 8, G = (int)gridDim.x / 8;
  const int l_lo = LIST ? (int)(((int64_t)x.n_list * xcd) / 8) : 0;
  const int l_hi = LIST ? (int)(((int64_t)x.n_list * (xcd + 1)) / 8) : 0;
  auto tile_at = [&](int i) __attribute__((always_inline)) -> int {
    if (LIST) {
      const int q = l_lo + kw + i * G;
      return q < l_hi ? __builtin_amdgcn_readfirstlane(x.tile_list[q]) : -1;
    }
    if (i > 0) return -1;
    const int nwg = (int)gridDim.x, xq = nwg / 8, xr = nwg % 8;
    const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + kw;
    const int tr0 = (t % x.n_rt) * PF_TR;
    const int64_t tc0 = (a.j_lo / 32) * 32 + (int64_t)(t / x.n_rt) * PF_TC;
    if (tr0 >= a.n_rows || tc0 >= a.m) return -1;
    if (a.tri && tc0 + PF_TC - 1 <= a.rows[tr0]) return -1;  // rows ascend within a launch
    return t;
  };
  int it = 0, tile = tile_at(0);
  if (tile < 0) return;
  int r0 = (tile % x.n_rt) * PF_TR;
  int64_t c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * PF_TC;
  auto pstamp = [&](int k) __attribute__((always_inline)) {  // the workgroup's first tile only
    if (!LIST && a.pf_stamp && threadIdx.x == 0)
      a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + k] = __builtin_amdgcn_s_memrealtime();
  };
  pstamp(0);
  // 8 waves: wave w = rows 32 (w >> 2) .. +32 x columns 64 (w & 3) .. +64 (two 32-column blocks)
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), wr = w >> 2, wc = w & 3;  // wave-uniform (SGPR)
  constexpr int O_R8 = 0, O_R8S = 4096, O_R4 = 8192, O_C4 = 9216;
  static_assert(O_C4 + PF_TC * 16 == PF_ST && PF_ST == 1024 * PF_NQ, "prefilter stage image");
  const int nq = w + 8 < PF_NQ ? 2 : 1;  // stage DMAs of this wave (q = w, w + 8)
  __shared__ __attribute__((aligned(16))) uint8_t ring[PF_NS][PF_ST];
  // stage-blocked panels: a stage's 64-byte / 16-byte pieces of consecutive SNPs are contiguous, so
  // an instruction's 1 KB comes from 8 whole 128-byte lines (int8 pieces in the even / odd
  // individual order of i8x2_of_fp4_eo).  Sources: a wave-uniform base per instruction (the panel's
  // stage st, SGPRs) + a 32-bit lane offset
  constexpr int64_t rstride = SG_K, cstride = SG_K / 4;
  const uint8_t *sbase0 = (const uint8_t *)x.rs[w >> 2];           // q = w: L3 slice w / 4
  const uint8_t *sbase1 = w == 0 ? x.rs2 : x.cs2;                  // q = w + 8: codes
  const int64_t sstep0 = a.m * SG_K, sstep1 = a.m * cstride;
  unsigned voff[2];
  auto set_src = [&](int r0, int64_t c0) __attribute__((always_inline)) {
    {  // int8 L3 slices: 16 rows x 4 chunks per instruction (q 0..3 slice 0, 4..7 slice 1)
      const int row = (w & 3) * 16 + (lane >> 2), lg = (lane & 3) ^ ((row >> 2) & 3);
      voff[0] = (unsigned)(a.rows[min(r0 + row, a.n_rows - 1)] * rstride + 16 * lg);
    }
    if (w == 0)  // q 8: 2-bit codes of the 64 rows, one per lane
      voff[1] = (unsigned)(a.rows[min(r0 + lane, a.n_rows - 1)] * cstride);
    else  // q 9..12: 2-bit codes of 64 columns per instruction
      voff[1] = (unsigned)(min(c0 + 64 * (w - 1) + lane, a.m - 1) * cstride);
  };
  set_src(r0, c0);
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]) + w * 1024;
  // stage st into ring slot `slot` (= st % PF_NS, kept by the caller)
  auto issue = [&](int st, int slot) __attribute__((always_inline)) {
    lds_dma16_sv(voff[0], sbase0 + st * sstep0, ring_m0 + slot * PF_ST);
    if (nq == 2) lds_dma16_sv(voff[1], sbase1 + st * sstep1, ring_m0 + slot * PF_ST + 8 * 1024);
  };
  // wait until stage `st` has landed given the stages issued up to `last` (nq DMAs per stage), then
  // the workgroup barrier, in ONE asm statement: the compiler does not know that the DMA asm writes
  // LDS, and the barrier builtin is no memory fence, so a separate builtin would let it hoist the next
  // stage's ds_reads above the barrier.  The counted vmcnt assumes that VMEM operations retire in order
  // (they do on gfx9 for loads).  (The record DMAs are older than any stage.)
  static_assert(PF_NS == 5, "wait_for's vmcnt values");
  auto wait_for = [&](int st, int last) __attribute__((always_inline)) {
    const int ahead = last - st;
    if (nq == 2) {
      if (ahead >= 3)
        asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (ahead == 2)
        asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (ahead >= 3)
        asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (ahead == 2)
        asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };
  v16i acc[2][E3_PF];
  v16f_ acc4[2][4];  // per column block: a.b, a^2.b, a.b^2, a^2.b^2
  const int S = (int)(x.n_pad / SG_K);
  const int pre = min(S, PF_NS - 1);
  // the epilogue's test records (32 B per row / column) by LDS-DMA ahead of the stages: wave w the
  // 32 columns 32 w .., waves 0 and 1 also the 32 rows 32 w ..; lane l half l & 1 of record l / 2.
  // They retire before stage 0 (in-order vmcnt), so the stage waits cover them.
  // Two record buffers: the next tile's land while the current tile's epilogue reads its own.
  __shared__ __attribute__((aligned(16))) float rec[2][PF_TR + PF_TC][PF_REC];
  auto issue_rec = [&](int r0, int64_t c0, int rb) __attribute__((always_inline)) {
    const int k = 32 * w + (lane >> 1);
    if (w < PF_TR / 32)
      lds_dma16(x.recL + a.rows[min(r0 + k, a.n_rows - 1)] * PF_REC + 4 * (lane & 1), &rec[rb][32 * w][0]);
    lds_dma16(x.recR + min(c0 + k, a.m - 1) * PF_REC + 4 * (lane & 1), &rec[rb][PF_TR + 32 * w][0]);
  };
  issue_rec(r0, c0, 0);
  for (int st = 0; st < pre; ++st) issue(st, st);
  // COMPACT + LIST: the wave's live-pair records are placed in chunks of at least PF_CHUNK records
  // reserved with one atomic (a tile keeps ~8 per wave at configs[2]: an atomic every ~16 tiles instead
  // of a round trip in every epilogue; the unused tails count against ops_cap)
  unsigned ch_cur = 0u, ch_end = 0u;
  for (;; ++it) {
    // per-lane values re-derived from an opaque copy of the thread index each tile: hoisted out of
    // the tile loop, the epilogue's would stay live through the main loop (256-VGPR budget)
    int tid_o = (int)threadIdx.x;
    asm volatile("" : "+v"(tid_o));
    const int lane = tid_o & 63, h = lane >> 5, c = lane & 31;
    const int rrow = 32 * wr + c;
    const int rb = it & 1;
    if (it == 0) {
      wait_for(0, pre - 1);
    } else {  // the prefetched stages, records and the previous epilogue's stores (vmcnt counts those too)
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    pstamp(1);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
#pragma unroll
      for (int p = 0; p < E3_PF; ++p)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[q][p][e] = 0;
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc4[q][p][e] = 0.f;
    }
    // (two stages per barrier, a six-slot ring, measured slower: 11.7 against 11.0 ms of prefilter per
    // configs[2] step, serialised)
    int slot = 0, slot_ahead = PF_NS - 1;  // ring slots of stage st and of stage st + 4
    for (int st = 0; st < S; ++st) {
      const uint8_t *bf = ring[slot];
      // slot (st + 4) % 5 was read in stage st - 1, which every wave has left (barrier)
      if (st + PF_NS - 1 < S) issue(st + PF_NS - 1, slot_ahead);
      slot = slot == PF_NS - 1 ? 0 : slot + 1;
      slot_ahead = slot_ahead == PF_NS - 1 ? 0 : slot_ahead + 1;
      // lane (c, h) holds the fp4 codes of individuals 32h .. 32h + 31 of the stage; the int8 E3
      // product kk sums individuals 32h + 16kk .. + 15 (A side: logical int8 chunk 2h + kk)
      v4i rb4[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) rb4[q] = fp4_of_code2(*(const v2i_ *)&bf[O_C4 + (64 * wc + 32 * q + c) * 16 + 8 * h]);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int lr = (2 * h + kk) ^ ((rrow >> 2) & 3);
        const v4i f0 = *(const v4i *)&bf[O_R8 + rrow * 64 + 16 * lr];
        const v4i f1 = *(const v4i *)&bf[O_R8S + rrow * 64 + 16 * lr];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const v4i fc = i8x2_of_fp4_eo((unsigned)rb4[q][2 * kk], (unsigned)rb4[q][2 * kk + 1]);
          acc[q][0] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f0, fc, acc[q][0], 0, 0, 0);
          acc[q][1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(f1, fc, acc[q][1], 0, 0, 0);
        }
      }
      {
        v8i_ fa[2];
        {
          const v4i ra4 = fp4_of_code2(*(const v2i_ *)&bf[O_R4 + rrow * 16 + 8 * h]);
          fa[0] = v8i_{ra4[0], ra4[1], ra4[2], ra4[3], 0, 0, 0, 0};
          fa[1] = sq4(ra4);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          v8i_ fb[2];
          fb[0] = v8i_{rb4[q][0], rb4[q][1], rb4[q][2], rb4[q][3], 0, 0, 0, 0};
          fb[1] = sq4(rb4[q]);
#pragma unroll
          for (int p = 0; p < 4; ++p)
            acc4[q][p] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[p & 1], fb[p >> 1], acc4[q][p], 4, 4, 0, 127, 0, 127);
        }
      }
      wait_for(st + 1, min(st + PF_NS - 1, S - 1));
    }
    pstamp(2);
    // every wave has passed the last stage's barrier (its vmcnt(0) wait): the ring is free, so the
    // next tile's records and first stages go out now and land while this tile's epilogue runs
    const int nxt = tile_at(it + 1);
    if (nxt >= 0) {
      const int nr0 = (nxt % x.n_rt) * PF_TR;
      const int64_t nc0 = (a.j_lo / 32) * 32 + (int64_t)(nxt / x.n_rt) * PF_TC;
      set_src(nr0, nc0);
      issue_rec(nr0, nc0, rb ^ 1);
      for (int st = 0; st < pre; ++st) issue(st, st);
    }
    // epilogue: lane (c, h) holds rows 32 wr + (e & 3) + 8 (e >> 2) + 4h, column 64 wc + 32 q + c; a
    // half-wave covers one 32-column block.  Per-row scalars staged in LDS, per-column ones in registers.
    // The test runs in fp32 with a certified slack (fp64 costs twice the issue slots and two registers
    // per value): every quantity below is a signed sum of the monomials of (a - alpha)^2 (b - beta)^2 or
    // (a - alpha)(b - beta) over the individuals, whose absolute values add up to at most
    //   M = sum_k (a_k + alpha)^2 (b_k + beta)^2 <= (2 + alpha)^2 sum_k (b_k + beta)^2   (|1'e| <= sqrt(n M)),
    // so the fp32 evaluation (about a dozen roundings of 2^-24 each, inputs rounded from fp64 included)
    // is off by at most 2^-20 M for |e|^2 and 2^-21 sqrt(n M) for 1'e, and vlo = (mu - eps)|e|^2 -
    // (mu + tau)(1'e)^2/n by at most 2^-19 (2 mu + tau) M: vlo is lowered by 2^-17 (2 mu + tau) M.  eff
    // = sL3 c3 - beta sa + alpha (beta spy - sb) is off by at most 2^-20 times the sum of the three
    // terms' magnitudes, which is added to eff_hi with the int8 slicing bound.  The final comparison's
    // three roundings are covered by the factor 1 + 2^-18.
    // per-row / per-column values: the records in rec[] (pf_rec_kernel).  Two passes: the tests of all
    // 32 (row, column block) elements of a lane as straight-line code (no branch between them, so the
    // row records' LDS reads are scheduled ahead of their use), collecting the live masks and a per-lane
    // bit per element for the stores; then the stores of the live blocks' products (a few per cent).
    const float mu_e = (float)(a.pf_mu - a.pf_eps), k1 = (float)((a.pf_mu + a.pf_tau + 1e-12 * a.pf_mu) / a.n_id);
    const float k2 = (float)(std::ldexp(1.0, -17) * (2.0 * a.pf_mu + a.pf_tau));
    const float chi_cut = (float)a.chi_cut, e3_eps = (float)a.e3_eps;
    constexpr float EFF_REL = 0x1p-20f, CMP = 1.0f + 0x1p-18f;
    const float4 *rv = (const float4 *)&rec[rb][0][0];
    int jq[2];  // SNP indices < 2^31
    bool cok[2];
    float cbe[2], ccb[2], cC1n[2], cnb[2], cbsb[2], cmag[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int cl = 64 * wc + 32 * q + c;
      jq[q] = (int)(c0 + cl);
      // beta, csum, C1n, n beta - csum | beta spy - sb, sum_k (b + beta)^2, monomorphic
      const float4 cv0 = rv[2 * (PF_TR + cl)], cv1 = rv[2 * (PF_TR + cl) + 1];
      cbe[q] = cv0.x;
      ccb[q] = cv0.y;
      cC1n[q] = cv0.z;
      cnb[q] = cv0.w;
      cbsb[q] = cv1.x;
      cmag[q] = cv1.y;
      cok[q] = (jq[q] < a.m) & (jq[q] >= a.j_lo) & (cv1.z == 0.0f);
    }
    // masks: lane t < 32 of the wave writes the word of (e = t / 2, half t % 2) of each column block
    const int te = (lane >> 1) & 15, th = lane & 1;
    unsigned mine[2] = {0u, 0u}, n_live = 0, st_bits = 0u;
    pstamp(3);
    const int rw = r0 + 32 * wr;
    const int64_t cw = c0 + 64 * wc - a.j_lo;
    const uint32_t voff = (uint32_t)(4 * h * a.ld_e + c);
    int *const b13 = (int *)a.c13 + ((int64_t)a.n_rows + rw) * a.ld_e + cw;
    int *const bpf = (int *)a.pfc + (int64_t)rw * a.ld_e + cw;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int kr = (e & 3) + 8 * (e >> 2);
      const int rl = 32 * wr + kr + 4 * h, r = r0 + rl;
      const float4 r0v = rv[2 * rl], r1v = rv[2 * rl + 1];  // i, alpha, csum, R1 | sL3, sa, (2 + alpha)^2
      const int iv = __float_as_int(r0v.x);
      const float al = r0v.y, sL3 = r1v.x, sL3h = 0.5f * sL3;
      const bool rok = (r < a.n_rows) & (iv >= 0);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const bool ok = rok & cok[q] & !(a.tri & (jq[q] <= iv));
        const float be = cbe[q];
        float c3 = 0.0f;  // twice the E3 slice sum (the doubled int8 b), halved through sL3h
#pragma unroll
        for (int t = E3_PF - 1; t >= 0; --t) c3 = c3 * (1.0f / 128.0f) + (float)acc[q][t][e];
        const float t1 = sL3h * c3, t2 = be * r1v.y, t3 = al * cbsb[q];
        const float eff = t1 - t2 + t3;
        const float eff_hi = fabsf(eff) + e3_eps * sL3 * ccb[q] + EFF_REL * (fabsf(t1) + fabsf(t2) + fabsf(t3));
        const float sab = acc4[q][0][e], sa2b = acc4[q][1][e], sab2 = acc4[q][2][e], sa2b2 = acc4[q][3][e];
        // |e|^2 = sa2b2 - 2b sa2b - 2a sab2 + 4ab sab + b^2 R1 + a^2 C1n;  1'e = sab - b ca + a (n b - cb)
        const float ee = sa2b2 + be * (be * r0v.w - 2.0f * sa2b) + al * (4.0f * be * sab - 2.0f * sab2 + al * cC1n[q]);
        const float se = sab - be * r0v.z + al * cnb[q];
        const float vlo = mu_e * ee - k1 * se * se - k2 * r1v.z * cmag[q];
        const bool lv = ok & (!(vlo > 0.0f) | (eff_hi * eff_hi * CMP >= chi_cut * vlo));
        const unsigned long long bal = __ballot(lv);
        n_live += (unsigned)__popcll(bal);
        const unsigned w0 = (unsigned)bal, w1 = (unsigned)(bal >> 32);
        mine[q] = te == e ? (th ? w1 : w0) : mine[q];
        // COMPACT: this lane's pair is live; else: a live block (its row r < n_rows: some lane of the half
        // passed rok) whose column this lane holds
        st_bits |= ((COMPACT ? lv : (((h ? w1 : w0) != 0u) & cok[q])) ? 1u : 0u) << (2 * e + q);
      }
    }
    pstamp(4);
    if (COMPACT) {
      // one record per live pair: the wave reserves its n_live records with one atomic, then each
      // (row pair, block) ballot places its pairs in lane order (h = 0 row first, ascending columns)
      unsigned base = 0u;
      if (n_live) {
        if (!LIST) {
          if (lane == 0) base = atomicAdd(a.ops_count, n_live);
          base = __builtin_amdgcn_readfirstlane(base);
        } else {
          if (ch_cur + n_live > ch_end) {
            const unsigned want = max(n_live, (unsigned)PF_CHUNK);
            unsigned b0 = 0u;
            if (lane == 0) b0 = atomicAdd(a.ops_count, want);
            ch_cur = __builtin_amdgcn_readfirstlane(b0);
            ch_end = ch_cur + want;
          }
          base = ch_cur;
          ch_cur += n_live;
        }
      }
      const bool fits = (int64_t)base + n_live <= a.ops_cap;
      unsigned run = base;
      int *const ops = a.ops;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bool lv = (st_bits >> (2 * e + q)) & 1u;
          const unsigned long long bal = __ballot(lv);
          if (bal) {
            // the first record of each live (row, block) of the ballot: lane 2 e + th writes row th's
            const unsigned word = th ? (unsigned)(bal >> 32) : (unsigned)bal;
            const int trr = r0 + 32 * wr + (e & 3) + 8 * (e >> 2) + 4 * th;
            const int J = (int)((c0 + 64 * wc + 32 * q) / 32);
            if (te == e && lane < 32 && word && trr < a.n_rows && J < a.nJ)
              a.lmask[(int64_t)trr * a.nJ + J] = lm_entry(word, run + (th ? (unsigned)__popc((unsigned)bal) : 0u), a.ltag);
            if (lv && fits) {
              const unsigned k = run + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32),
                                                                 __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
              v4i r0v = {acc[q][0][e] >> 1, acc[q][1][e] >> 1, (int)acc4[q][0][e], (int)acc4[q][1][e]};  // exact
              v4i r1v = {(int)acc4[q][2][e], (int)acc4[q][3][e], jq[q], 0};
              *(v4i *)(ops + (int64_t)k * OPS_REC) = r0v;
              *(v4i *)(ops + (int64_t)k * OPS_REC + 4) = r1v;
            }
            run += (unsigned)__popcll(bal);
          }
        }
      }
    } else {
      // a live block's E3 (and code products) for the low-rank / pair screens (cok: j in range; a
      // monomorphic j is never live).  Wave-uniform base + 32-bit lane offset.
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int kr = (e & 3) + 8 * (e >> 2);
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if ((st_bits >> (2 * e + q)) & 1u) {
            const int64_t ou = (int64_t)kr * a.ld_e + 32 * q;
#pragma unroll
            for (int t = 0; t < E3_PF; ++t) (b13 + t * a.c13_stride + ou)[voff] = acc[q][t][e] >> 1;  // exact
            if (a.pf_store)  // the low-rank screen's |e|^2 and 1'e come from these code products
#pragma unroll
              for (int p = 0; p < 4; ++p) (bpf + p * a.pfc_stride + ou)[voff] = (int)acc4[q][p][e];
          }
      }
    }
    pstamp(5);
    const int tr = r0 + 32 * wr + (te & 3) + 8 * (te >> 2) + 4 * th;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int J = (int)((c0 + 64 * wc + 32 * q) / 32);
      if (lane < 32 && tr < a.n_rows && J < a.nJ) {
        if (a.flags) a.flags[(int64_t)tr * a.nJ + J] = mine[q] != 0;
      }
    }
    if (a.live_count && lane == 0 && n_live) atomicAdd(a.live_count, (unsigned long long)n_live);
    if (!LIST && a.pf_stamp) __syncthreads();  // the phase stamps time the slowest wave
    pstamp(6);
    if (nxt < 0) break;
    r0 = (nxt % x.n_rt) * PF_TR;
    c0 = (a.j_lo / 32) * 32 + (int64_t)(nxt / x.n_rt) * PF_TC;
    set_src(r0, c0);  // again: the source addresses stay out of the epilogue's registers
  }
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
constexpr int PC_TR = 32, PC_TC = 256, PC_NS = 8, PF_NCOV_MAX = 4;
template <int NC>
struct PcShape {
  static constexpr int O_A2 = 4096, O_B2 = 5120, O_Q = 9216;
  static constexpr int QT = 10;                        // DMA instructions per stage
  static constexpr int ST = 10240;                     // slot bytes
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
// LIST: a persistent grid over the launch's tile list (as prefilter_pass_kernel<true>: XCD x takes the
// list's x-th eighth, its workgroups stride through it, and the next tile's first stages stream into
// the ring while this tile's epilogue runs); else one workgroup per tile of the XCD-aware remap.
template <int NC, bool LIST>
__global__ __launch_bounds__(512, 1) void prefilter_cov_kernel(SideArgs x) {
  using SH = PcShape<NC>;
  constexpr int NW = 8;
  const ScreenArgs &a = x.a;
  const int xcd = (int)blockIdx.x % 8, kw = (int)blockIdx.x / 8, G = (int)gridDim.x / 8;
  const int l_lo = LIST ? (int)(((int64_t)x.n_list * xcd) / 8) : 0;
  const int l_hi = LIST ? (int)(((int64_t)x.n_list * (xcd + 1)) / 8) : 0;
  auto tile_at = [&](int i) __attribute__((always_inline)) -> int {
    if (LIST) {
      const int q = l_lo + kw + i * G;
      return q < l_hi ? __builtin_amdgcn_readfirstlane(x.tile_list[q]) : -1;
    }
    if (i > 0) return -1;
    const int nwg = (int)gridDim.x, xq = nwg / 8, xr = nwg % 8;
    const int t = (xcd < xr ? xcd * (xq + 1) : xr * (xq + 1) + (xcd - xr) * xq) + kw;
    const int r0_ = (t % x.n_rt) * PC_TR;
    const int64_t c0_ = (a.j_lo / 32) * 32 + (int64_t)(t / x.n_rt) * PC_TC;
    if (r0_ >= a.n_rows || c0_ >= a.m) return -1;
    if (a.tri && c0_ + PC_TC - 1 <= a.rows[r0_]) return -1;  // rows ascend within a launch
    return t;
  };
  auto pstamp = [&](int st_) __attribute__((always_inline)) {  // GMAT_PF_STAMPS (one tile per workgroup)
    if (!LIST && a.pf_stamp && threadIdx.x == 0)
      a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + st_] = __builtin_amdgcn_s_memrealtime();
  };
  pstamp(0);
  int tile = tile_at(0);
  if (tile < 0) return;
  // 8 waves at two per SIMD: wave w = the tile's 32 rows x columns 32 w .. +32
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            c = lane & 31;
  __shared__ __attribute__((aligned(16))) uint8_t ring[PC_NS][SH::ST];
  __shared__ __attribute__((aligned(16))) uint8_t img[2][NC][2048];  // direction images, stages s % 2
  // DMA instruction q = w + 8u (u < 2): a wave-uniform base per instruction (the panel at stage st,
  // SGPRs) + a 32-bit lane offset
  const int nq = (w + NW < SH::QT) ? 2 : 1;  // DMA instructions this wave issues per stage
  auto base_of = [&](int q) __attribute__((always_inline)) -> const uint8_t * {
    return q < 4 ? (const uint8_t *)x.rs[q >> 1] : q == 4 ? x.rs2 : q < 9 ? x.cs2 : x.qimg;
  };
  auto step_of = [&](int q) __attribute__((always_inline)) -> int64_t {
    return q < 4 ? (int64_t)SG_K * a.m : q < 9 ? (int64_t)(SG_K / 4) * a.m : (int64_t)SG_K;
  };
  const uint8_t *sbase0 = base_of(w), *sbase1 = base_of(w + NW);
  const int64_t sstep0 = step_of(w), sstep1 = step_of(w + NW);
  unsigned voff[2];
  auto set_src = [&](int r0, int64_t c0) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q = w + NW * u;
      if (q < 4) {  // int8 L3 rows (stage-blocked): slice q / 2, 16 rows x 4 chunks per instruction
        const int row = (q & 1) * 16 + (lane >> 2), lg = (lane & 3) ^ ((row >> 2) & 3);
        voff[u] = (unsigned)(a.rows[min(r0 + row, a.n_rows - 1)] * SG_K + 16 * lg);
      } else if (q == 4) {  // 2-bit codes of the 32 rows (lanes 32-63: a copy)
        voff[u] = (unsigned)(a.rows[min(r0 + (lane & 31), a.n_rows - 1)] * (SG_K / 4));
      } else if (q < 9) {  // 2-bit codes of 64 columns per instruction
        voff[u] = (unsigned)(min(c0 + 64 * (q - 5) + lane, a.m - 1) * (SG_K / 4));
      } else {  // the q slices: lane l = direction min(l / 4, NC - 1), chunk l % 4
        voff[u] = (unsigned)(min(lane >> 2, NC - 1) * x.n_pad + 16 * (lane & 3));
      }
    }
  };
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]) + w * 1024;
  auto issue = [&](int st) __attribute__((always_inline)) {
    const unsigned m0 = ring_m0 + (st % PC_NS) * SH::ST;
    lds_dma16_sv(voff[0], sbase0 + st * sstep0, m0);
    if (nq == 2) lds_dma16_sv(voff[1], sbase1 + st * sstep1, m0 + NW * 1024);
  };
  // the direction images of stage st (its codes and q slices have landed): thread t < 128 NC forms
  // direction t / 128, row (t / 4) % 32, 16-individual chunk t % 4
  auto image = [&](int st) __attribute__((always_inline)) {
    if (tid < 128 * NC) {
      uint8_t *sl = ring[st % PC_NS];
      const int k = tid >> 7, row = (tid >> 2) & 31, ch = tid & 3;
      const unsigned cw = *(const unsigned *)(sl + SH::O_A2 + row * 16 + 4 * ch);  // 16 individuals, 2 bits each
      const v4i qv = *(const v4i *)(sl + SH::O_Q + 64 * k + 16 * ch);
      *(v4i *)(&img[st & 1][k][row * 64 + 16 * (ch ^ ((row >> 2) & 3))]) =
          aq_of_fp4_eo((cw << 1) & 0x66666666u, (cw >> 1) & 0x66666666u, qv);
    }
  };
  const int S = (int)(x.n_pad / SG_K);
  const int pre = min(S, PC_NS - 1);
  int r0 = (tile % x.n_rt) * PC_TR;
  int64_t c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * PC_TC;
  set_src(r0, c0);
  for (int st = 0; st < pre; ++st) issue(st);
  unsigned ch_cur = 0u, ch_end = 0u;  // LIST: record chunks (prefilter_pass_kernel)
  for (int it = 0;; ++it) {
  if (it == 0)
    vm_wait_barrier(nq * max(0, pre - 2));  // stages 0 and 1 have landed
  else  // the prefetched stages and the previous epilogue's stores (vmcnt counts those too)
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  image(0);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // (no vmcnt wait: later stages stream on)
  pstamp(1);
  v16i acc[E3_PF], accu[NC];
  v16f_ acc4[4];  // a.b, a^2.b, a.b^2, a^2.b^2
#pragma unroll
  for (int e = 0; e < 16; ++e) {
#pragma unroll
    for (int p = 0; p < E3_PF; ++p) acc[p][e] = 0;
#pragma unroll
    for (int k = 0; k < NC; ++k) accu[k][e] = 0;
#pragma unroll
    for (int p = 0; p < 4; ++p) acc4[p][e] = 0.f;
  }
  const int rrow = c;
  const int crow = 32 * w + c;
  for (int st = 0; st < S; ++st) {
    const uint8_t *bf = ring[st % PC_NS];
    if (st + PC_NS - 1 < S) issue(st + PC_NS - 1);
    if (st + 1 < S) image(st + 1);
    const v4i rb4 = fp4_of_code2(*(const v2i_ *)&bf[SH::O_B2 + crow * 16 + 8 * h]);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int lr = (2 * h + kk) ^ ((rrow >> 2) & 3);
      const v4i fc = i8x2_of_fp4_eo((unsigned)rb4[2 * kk], (unsigned)rb4[2 * kk + 1]);  // 2b: sums doubled
#pragma unroll
      for (int g = 0; g < E3_PF; ++g)
        acc[g] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const v4i *)&bf[2048 * g + rrow * 64 + 16 * lr], fc, acc[g], 0, 0, 0);
#pragma unroll
      for (int k = 0; k < NC; ++k)
        accu[k] = __builtin_amdgcn_mfma_i32_32x32x32_i8(*(const v4i *)&img[st & 1][k][rrow * 64 + 16 * lr], fc, accu[k], 0,
                                                        0, 0);
    }
    {
      const v4i ra4 = fp4_of_code2(*(const v2i_ *)&bf[SH::O_A2 + rrow * 16 + 8 * h]);
      const v8i_ fa[2] = {v8i_{ra4[0], ra4[1], ra4[2], ra4[3], 0, 0, 0, 0}, sq4(ra4)};
      const v8i_ fb[2] = {v8i_{rb4[0], rb4[1], rb4[2], rb4[3], 0, 0, 0, 0}, sq4(rb4)};
#pragma unroll
      for (int p = 0; p < 4; ++p)
        acc4[p] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[p & 1], fb[p >> 1], acc4[p], 4, 4, 0, 127, 0, 127);
    }
    // stages up to st + 2 have landed (the image of st + 2 is formed in the next iteration)
    vm_wait_barrier(nq * max(0, min(st + PC_NS - 1, S - 1) - (st + 2)));
  }
  pstamp(2);
  // epilogue as prefilter_pass_kernel's (fp32 with its certified slack, straight-line tests), plus the
  // direction terms: each c_k = t1 - t2 - t3 + t4 (t1 = sq_k / 2 x the doubled integer sum, t2 = beta
  // u_k.a, t3 = alpha u_k.b, t4 = alpha beta 1'u_k) is off by at most 2^-21 (|t1| + .. + |t4|) in fp32
  // (inputs rounded from fp64 included), to which the quantisation bound sq_k Sab / 2 is added; |U'e|^2
  // from those upper bounds carries a relative 2^-20 of its own roundings, covered by ku (1 + 2^-18).
  // (Round 3 / early round 4: fp64, 13 us of epilogue per tile.)
  __shared__ float rowf[7][PC_TR];    // i (int bits, -1 monomorphic), alpha, csum, R1, sL3, sa, (2 + alpha)^2
  __shared__ float rowu[NC][PC_TR];   // u.a per direction
  const double n = a.n_id;
  if (tid < PC_TR) {
    const int r = min(r0 + tid, a.n_rows - 1);
    const int64_t i = a.rows[r];
    const double al = a.alpha[i], ca = a.csum_l[i];
    rowf[0][tid] = __int_as_float(a.mono_l[i] ? -1 : (int)i);
    rowf[1][tid] = (float)al;
    rowf[2][tid] = (float)ca;
    rowf[3][tid] = (float)(a.csq_l[i] - 2.0 * al * ca);
    rowf[4][tid] = (float)a.sL3[i];
    rowf[5][tid] = (float)a.sa[i];
    rowf[6][tid] = (float)((2.0 + al) * (2.0 + al));
#pragma unroll
    for (int k = 0; k < NC; ++k) rowu[k][tid] = (float)a.pf_ua[k * a.m + i];
  }
  __syncthreads();
  pstamp(3);
  const float mu_e = (float)(a.pf_mu - a.pf_eps), k1 = (float)((a.pf_mu + a.pf_tau + 1e-12 * a.pf_mu) / n);
  const float k2 = (float)(std::ldexp(1.0, -17) * (2.0 * a.pf_mu + a.pf_tau));
  const float ku = (float)(a.pf_ku * (1.0 + std::ldexp(1.0, -18)));
  const float chi_cut = (float)a.chi_cut, e3_eps = (float)a.e3_eps;
  constexpr float EFF_REL = 0x1p-20f, CMP = 1.0f + 0x1p-18f, UREL = 0x1p-21f, QREL = 1.0f + 0x1p-20f;
  const int64_t j = c0 + crow;
  const int J = (int)(j / 32);
  const bool jok = j < a.m && j >= a.j_lo;
  float cbe = 0, ccb = 0, cC1n = 0, cnb = 0, cbsb = 0, cmag = 0, cub[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) cub[k] = 0.f;
  unsigned own = 0u, n_live = 0u;  // compacted path: this lane's live elements, the wave's live pairs
  bool cmono = true;
  if (jok) {
    const double be = a.beta[j], cb = a.csum_r[j], cb2 = a.csq_r[j];
    cbe = (float)be;
    ccb = (float)cb;
    cC1n = (float)(cb2 - 2.0 * be * cb + n * be * be);
    cnb = (float)(n * be - cb);
    cbsb = (float)(be * a.spy - a.sb[j]);
    cmag = (float)(cb2 + 2.0 * be * cb + n * be * be);
    cmono = a.mono_r[j];
#pragma unroll
    for (int k = 0; k < NC; ++k) cub[k] = (float)a.pf_ub[k * a.m + j];
  }
  float sqh[NC], su4[NC];
#pragma unroll
  for (int k = 0; k < NC; ++k) {
    sqh[k] = (float)(0.5 * a.pf_sq[k]);
    su4[k] = (float)a.pf_su[k];
  }
  // every wave has passed the last stage's barrier (and the records' barrier): the ring is free for the
  // next tile's first stages, which land while the tests below run.  (Issued after the per-row and
  // per-column loads have been consumed: the compiler's waits for those count the DMAs as well.)
  const int nxt = tile_at(it + 1);
  if (nxt >= 0) {
    set_src((nxt % x.n_rt) * PC_TR, (a.j_lo / 32) * 32 + (int64_t)(nxt / x.n_rt) * PC_TC);
    asm volatile("" ::"v"(cbe), "v"(ccb), "v"(cC1n), "v"(cnb), "v"(cbsb), "v"(cmag), "v"(cub[0]), "v"((int)cmono));
    for (int st = 0; st < pre; ++st) issue(st);
  }
  const bool cok = jok & !cmono;
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int rl = (e & 3) + 8 * (e >> 2) + 4 * h, r = r0 + rl;
    const bool rok = r < a.n_rows;
    const int64_t o1 = (int64_t)(rok ? r : 0) * a.ld_e + (j - a.j_lo);
    const int iv = __float_as_int(rowf[0][rl]);
    const bool ok = rok & cok & (iv >= 0) & !(a.tri & (j <= (int64_t)iv));
    const float al = rowf[1][rl], sL3 = rowf[4][rl], be = cbe;
    const float c3 = (float)acc[1][e] * (1.0f / 128.0f) + (float)acc[0][e];  // twice the E3 slice sums
    const float t1 = 0.5f * sL3 * c3, t2 = be * rowf[5][rl], t3 = al * cbsb;
    const float eff = t1 - t2 + t3;
    const float eff_hi = fabsf(eff) + e3_eps * sL3 * ccb + EFF_REL * (fabsf(t1) + fabsf(t2) + fabsf(t3));
    const float sab = acc4[0][e], sa2b = acc4[1][e], sab2 = acc4[2][e], sa2b2 = acc4[3][e];
    const float ee = sa2b2 + be * (be * rowf[3][rl] - 2.0f * sa2b) + al * (4.0f * be * sab - 2.0f * sab2 + al * cC1n);
    const float se = sab - be * rowf[2][rl] + al * cnb;
    float u2 = 0.f;
#pragma unroll
    for (int k = 0; k < NC; ++k) {
      const float u1 = sqh[k] * (float)accu[k][e], uu2 = be * rowu[k][rl], u3 = al * cub[k], u4 = al * be * su4[k];
      const float ck = fabsf(u1 - uu2 - u3 + u4) + sqh[k] * sab * QREL + UREL * (fabsf(u1) + fabsf(uu2) + fabsf(u3) + fabsf(u4));
      u2 += ck * ck;
    }
    const float vlo = mu_e * ee - k1 * se * se - ku * u2 - k2 * rowf[6][rl] * cmag;
    const bool live = ok & (!(vlo > 0.0f) | (eff_hi * eff_hi * CMP >= chi_cut * vlo));
    const unsigned long long bal = __ballot(live);
    const bool blk = ((bal >> (32 * h)) & 0xFFFFFFFFull) != 0;
    if (rok && c == 0 && J < a.nJ) {
      if (a.flags) a.flags[(int64_t)r * a.nJ + J] = blk;
    }
    if (a.ops) {  // compacted path: records below
      own |= (live ? 1u : 0u) << e;
      n_live += (unsigned)__popcll(bal);
    } else if (blk && rok && jok) {
      const int64_t o3 = o1 + (int64_t)a.n_rows * a.ld_e;
#pragma unroll
      for (int t = 0; t < E3_PF; ++t) ((int *)a.c13)[t * a.c13_stride + o3] = acc[t][e] >> 1;  // exact
      if (a.pf_store)
#pragma unroll
        for (int p = 0; p < 4; ++p) ((int *)a.pfc)[p * a.pfc_stride + o1] = (int)acc4[p][e];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  pstamp(4);
  if (a.ops) {  // one record per live pair, placed as in prefilter_pass_kernel (one atomic per wave)
    unsigned base = 0u;
    if (n_live) {
      if (!LIST) {
        if (lane == 0) base = atomicAdd(a.ops_count, n_live);
        base = __builtin_amdgcn_readfirstlane(base);
      } else {
        if (ch_cur + n_live > ch_end) {
          const unsigned want = max(n_live, (unsigned)PF_CHUNK);
          unsigned b0 = 0u;
          if (lane == 0) b0 = atomicAdd(a.ops_count, want);
          ch_cur = __builtin_amdgcn_readfirstlane(b0);
          ch_end = ch_cur + want;
        }
        base = ch_cur;
        ch_cur += n_live;
      }
    }
    const bool fits = (int64_t)base + n_live <= a.ops_cap;
    unsigned run = base;
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int r = r0 + (e & 3) + 8 * (e >> 2) + 4 * h;
      const bool lv = (own >> e) & 1u;
      const unsigned long long bal = __ballot(lv);
      const unsigned lo = (unsigned)bal, word = h ? (unsigned)(bal >> 32) : lo;
      if (word && c == 0 && r < a.n_rows && J < a.nJ)
        a.lmask[(int64_t)r * a.nJ + J] = lm_entry(word, run + (h ? (unsigned)__popc(lo) : 0u), a.ltag);
      if (bal) {
        if (lv && fits) {
          const unsigned k = run + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo(lo, 0u));
          const v4i r0v = {acc[0][e] >> 1, acc[1][e] >> 1, (int)acc4[0][e], (int)acc4[1][e]};  // exact
          const v4i r1v = {(int)acc4[2][e], (int)acc4[3][e], (int)j, 0};
          *(v4i *)(a.ops + (int64_t)k * OPS_REC) = r0v;
          *(v4i *)(a.ops + (int64_t)k * OPS_REC + 4) = r1v;
        }
        run += (unsigned)__popcll(bal);
      }
    }
  }
  pstamp(5);
  if (!LIST && a.pf_stamp) __syncthreads();
  pstamp(6);
  if (nxt < 0) break;
  tile = nxt;
  r0 = (tile % x.n_rt) * PC_TR;
  c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * PC_TC;
  }  // tile loop
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

// One workgroup = one tile of BI first-SNP rows x BJ second-SNP columns; wave w owns the 32-wide
// column tiles of first-SNP rows PB*w .. PB*w+PB-1 (RB row tiles x PB col tiles of 32 x 32).
// Loop nest per tile: slice s -> K-block (MT rows of A_s) -> stage pairs (2 x LK individuals,
// static LDS double-buffer parity).  The next stage's A band and genotype chunks are fetched
// with buffer loads (per-lane constant voffset, scalar soffset) while the current stage
// multiplies, including across K-block and slice boundaries.  The first stage pair of a K-block
// is peeled (its MFMAs start from a zero C operand); the genotype chunks of the diagonal-block
// stages are also kept in a ping-pong LDS region (eI/eJ) from which the K-block epilogue
// rebuilds w[row].
template <int SH>
__global__ __launch_bounds__(256, 2) void screen_kernel(ScreenArgs a) {
  using S_ = Shape<SH>;
  constexpr int MT = S_::MT, PB = S_::PB, BI = S_::BI, RB = S_::RB, EP = S_::EP, NA = S_::NA, DS = S_::DS;
  __shared__ __attribute__((aligned(16))) int8_t sA[2][MT * AP];
  __shared__ __attribute__((aligned(16))) int8_t sI[2][BI * AP];
  __shared__ __attribute__((aligned(16))) int8_t sJ[2][BJ * AP];
  __shared__ __attribute__((aligned(16))) int8_t eI[2][BI * EP];
  __shared__ __attribute__((aligned(16))) int8_t eJ[2][BJ * EP];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int roff = a.tiles[2 * blockIdx.x], J = a.tiles[2 * blockIdx.x + 1];
  const int64_t J0 = (int64_t)J * BJ;
  const int n_pad = (int)a.n_pad;
  const int nK = n_pad / MT;
  const int nn = n_pad * n_pad;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(a.slices, a.slices_bytes);
  const __amdgpu_buffer_rsrc_t rsP = make_rsrc(a.panels, a.panels_bytes);

  int64_t ti[PB];
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    const int r = roff + PB * w + t;
    ti[t] = (r < a.n_rows) ? a.rows[r] : -1;
  }
  // staging roles: NA 16-byte A chunks per thread (rows tid/4 + 64u), one genotype chunk for
  // the first 4*(BI+BJ) threads (i-side rows first, offset-coded when stored)
  const int arow0 = tid >> 2, acol0 = (tid & 3) * 16;
  int voffA[NA];
#pragma unroll
  for (int u = 0; u < NA; ++u) voffA[u] = (arow0 + 64 * u) * n_pad + acol0;
  int prow = 0, pcol = (tid & 3) * 16, pside = 0;  // 1 = i-panel (offset coded), 2 = j-panel
  unsigned voffP = 0xFFFFFFF0u;                     // out of range -> the buffer load returns zeros
  if (tid < 4 * BI) {
    pside = 1;
    prow = tid >> 2;
    const int r = roff + prow;
    if (r < a.n_rows) voffP = (unsigned)(a.left_off + a.rows[r] * n_pad + pcol);
  } else if (tid < 4 * (BI + BJ)) {
    pside = 2;
    prow = (tid - 4 * BI) >> 2;
    if (J0 + prow < a.m) voffP = (unsigned)(a.right_off + (J0 + prow) * n_pad + pcol);
  }

  v4i ra[NA], rp = {0, 0, 0, 0};
  // fetch stage (A band at scalar byte offset soffA, genotype chunk at individual L)
  auto load = [&](int soffA, int L) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NA; ++u) ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rsA, voffA[u], soffA, 0);
    if (pside) rp = __builtin_amdgcn_raw_buffer_load_b128(rsP, voffP, L, 0);
  };
  // write the fetched stage into buffer b; epi >= 0: also into epilogue region at column epi
  auto store = [&](int b, int epi, int region) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NA; ++u) *(v4i *)&sA[b][(arow0 + 64 * u) * AP + acol0] = ra[u];
    if (pside == 1) {
      v4i o;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q] = (int)to_offset((unsigned)rp[q]);
      *(v4i *)&sI[b][prow * AP + pcol] = o;
      if (epi >= 0) *(v4i *)&eI[region][prow * EP + epi + pcol] = o;
    } else if (pside == 2) {
      *(v4i *)&sJ[b][prow * AP + pcol] = rp;
      if (epi >= 0) *(v4i *)&eJ[region][prow * EP + epi + pcol] = rp;
    }
  };

  v16i acc[RB][PB];
  // one 32-deep k-step on buffer b: B fragments w = a_i*b_j generated from the staged
  // genotype chunks, A fragments from the staged band
  auto kstep = [&](int b, int kk, bool diag, bool zero) __attribute__((always_inline)) {
    const unsigned tlo = diag ? T_LO : T2_LO, thi = diag ? T_HI : T2_HI;
    v4i fb[PB];
    const v4i v = *(const v4i *)&sJ[b][c * AP + kk * 32 + 16 * h];
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      const v4i o = *(const v4i *)&sI[b][(PB * w + t) * AP + kk * 32 + 16 * h];
#pragma unroll
      for (int q = 0; q < 4; ++q) fb[t][q] = (int)__builtin_amdgcn_perm(thi, tlo, (unsigned)o[q] + (unsigned)v[q]);
    }
    const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const v4i fa = *(const v4i *)&sA[b][(r * 32 + c) * AP + kk * 32 + 16 * h];
#pragma unroll
      for (int t = 0; t < PB; ++t)
        acc[r][t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb[t], zero ? z : acc[r][t], 0, 0, 0);
    }
  };

  int64_t tot[PB];
  unsigned sw[PB];
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    tot[t] = 0;
    sw[t] = 0;
  }
  // epilogue: sum_rows w[row] * acc[row]; acc register e of this lane <-> storage slot 16h+e of
  // each 32-row tile, whose genotype bytes sit in the LDS epilogue region (24-bit products:
  // |acc| <= 127 * 8 * n_pad < 2^23 for n_pad <= 8192)
  auto epilogue = [&](int region, int shift, bool first_slice) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      int64_t part64 = 0;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const v4i o = *(const v4i *)&eI[region][(PB * w + t) * EP + r * 32 + 16 * h];
        const v4i v = *(const v4i *)&eJ[region][c * EP + r * 32 + 16 * h];
        int part = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const unsigned wb = __builtin_amdgcn_perm(T_HI, T_LO, (unsigned)o[q] + (unsigned)v[q]);
          part += __mul24((int)(wb & 0xff), acc[r][t][4 * q]) + __mul24((int)((wb >> 8) & 0xff), acc[r][t][4 * q + 1]) +
                  __mul24((int)((wb >> 16) & 0xff), acc[r][t][4 * q + 2]) + __mul24((int)(wb >> 24), acc[r][t][4 * q + 3]);
          if (first_slice) sw[t] = __builtin_amdgcn_udot4(wb, wb, sw[t], false);  // sum w^2
        }
        part64 += part;
      }
      tot[t] += (int64_t)((uint64_t)part64 << shift);
    }
  };

  int gk = 0;  // K-blocks done (epilogue region parity)
  load(0, 0);
  store(0, 0, 0);
  __syncthreads();
  for (int s = 0; s < a.n_slice; ++s) {
    const int shift = 7 * (a.n_slice - 1 - s);
    for (int kb = 0; kb < nK; ++kb) {
      const int K = kb * MT;
      const int row0 = s * nn + K * n_pad;  // byte offset of row K of A_s
      const int nst = (nK - kb) * DS;
      int nxtA = -1, nxtL = 0;  // first stage of the next K-block (or slice)
      if (kb + 1 < nK) {
        nxtA = row0 + MT * n_pad + K + MT;
        nxtL = K + MT;
      } else if (s + 1 < a.n_slice) {
        nxtA = (s + 1) * nn;
        nxtL = 0;
      }
      // stage pair (st, st+1): st in LDS buffer 0, st+1 in buffer 1; stages < DS are the
      // diagonal block (table T, epilogue copies), later ones count twice (table 2T)
      auto pair = [&](int st, bool diag, bool zero) __attribute__((always_inline)) {
        const int L0 = K + st * LK;
        const bool last = (st + 2 == nst);
        load(row0 + L0 + LK, L0 + LK);
        kstep(0, 0, diag, zero);
        kstep(0, 1, diag, false);
        store(1, (st + 1 < DS) ? (st + 1) * LK : -1, gk & 1);
        __syncthreads();
        if (!last) load(row0 + L0 + 2 * LK, L0 + 2 * LK);
        else if (nxtA >= 0) load(nxtA, nxtL);
        kstep(1, 0, diag, false);
        kstep(1, 1, diag, false);
        if (last) {
          epilogue(gk & 1, shift, s == 0);
          ++gk;
          if (nxtA >= 0) store(0, 0, gk & 1);
        } else {
          store(0, (st + 2 < DS) ? (st + 2) * LK : -1, gk & 1);
        }
        __syncthreads();
      };
      pair(0, true, true);
#pragma unroll
      for (int st = 2; st < DS; st += 2) pair(st, true, false);
#pragma unroll 1
      for (int st = DS; st < nst; st += 2) pair(st, false, false);
    }
  }
  // combine the two lane halves (disjoint rows of the same column), then test
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    const int64_t other = __shfl_xor(tot[t], 32);
    const unsigned osw = __shfl_xor(sw[t], 32);
    if (h != 0 || ti[t] < 0) continue;
    cand_test(a, roff + PB * w + t, ti[t], J0 + c, (double)(tot[t] + other) * a.scale_main, (double)(sw[t] + osw));
  }
}

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
template <int V>
__global__ __launch_bounds__(MxShape<V>::T, MxShape<V>::MINB) void mx_screen_kernel(ScreenArgs a, MxArgs x) {
  constexpr int PB = MxShape<V>::PB, RB = MX_RB, MX_T = MxShape<V>::T, NA = MX_TILE / 16 / MX_T;
  constexpr int NJC = 2 * 8 * BJ;  // j-side chunks per stage (two column blocks)
  __shared__ __attribute__((aligned(16))) uint8_t sA[2][MX_TILE];
  __shared__ __attribute__((aligned(16))) uint8_t sI[2][MX_BI * NB_REC];
  __shared__ __attribute__((aligned(16))) uint8_t sJ[2][2 * BJ * NB_REC];
  __shared__ __attribute__((aligned(16))) uint8_t eI[2][MX_BI * NB_E];
  __shared__ __attribute__((aligned(16))) uint8_t eJ[2][2 * BJ * NB_E];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int tl = a.tiles[MX_TE * blockIdx.x];
  if (tl < 0) return;  // padding of the XCD deal
  const int Jt[2] = {a.tiles[MX_TE * blockIdx.x + 1], a.tiles[MX_TE * blockIdx.x + 2]};
  const int *trow = a.tile_rows + (int64_t)tl * MX_BI;  // band rows of this tile (-1 = none)
  const int half = (PB * w) / (MX_BI / 2);             // this wave's column block
  const int64_t J0 = (int64_t)Jt[half] * BJ;
  const int nK = x.nK;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(x.tiles, x.tiles_bytes);
  const __amdgpu_buffer_rsrc_t rsI = make_rsrc(x.nib_i, x.nib_bytes);
  const __amdgpu_buffer_rsrc_t rsJ = make_rsrc(x.nib_j, x.nib_bytes);

  int64_t ti[PB];
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    const int r = trow[PB * w + t];
    ti[t] = (r >= 0) ? a.rows[r] : -1;
  }
  // staging roles (branch-free): NA 16-byte A chunks per thread (a straight copy of the tile
  // image); j-side chunks (column block jh, SNP js, physical slot jq <- logical slot jq ^ f(js)) and
  // one i-side chunk per thread, threads beyond the 512 / 128 chunks repeating them (identical
  // stores)
  const unsigned OOR = 0xFFFFFFF0u;  // out of range -> the buffer load returns zeros
  const int jc = tid % NJC, jh = jc >> 8, js = (jc >> 3) & 31, jq = jc & 7, jl = jq ^ ((js >> 1) & 7);
  const int is = (tid >> 3) & 15;
  unsigned voffJ = OOR, voffI = OOR;
  {
    const int64_t jj = (int64_t)Jt[jh] * BJ + js;
    if (Jt[jh] >= 0 && jj < a.m) voffJ = (unsigned)(jj * nK * NB_REC + jl * 16);
  }
  if (trow[is] >= 0) voffI = (unsigned)(a.rows[trow[is]] * nK * NB_REC + jq * 16);

  v4i ra[NA], rnj, rni;
  auto load = [&](int kb, int cs) __attribute__((always_inline)) {
    const int soffA = (kb * nK + cs) * MX_TILE;
#pragma unroll
    for (int u = 0; u < NA; ++u) ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rsA, (tid + u * MX_T) * 16, soffA, 0);
    rnj = __builtin_amdgcn_raw_buffer_load_b128(rsJ, voffJ, cs * NB_REC, 0);
    rni = __builtin_amdgcn_raw_buffer_load_b128(rsI, voffI, cs * NB_REC, 0);
  };
  auto store = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NA; ++u) *(v4i *)&sA[b][(tid + u * MX_T) * 16] = ra[u];
    *(v4i *)&sJ[b][(jh * BJ + js) * NB_REC + jq * 16] = rnj;
    *(v4i *)&sI[b][is * NB_REC + jq * 16] = rni;
  };
  // the genotype records of a K-block's diagonal stage (in buffer b) kept for its epilogue
  auto keep_diag = [&](int b, int q) __attribute__((always_inline)) {
    const v4i vj = *(const v4i *)&sJ[b][(jh * BJ + js) * NB_REC + jq * 16];
    const v4i vi = *(const v4i *)&sI[b][is * NB_REC + jq * 16];
    *(v4i *)&eJ[q][(jh * BJ + js) * NB_E + jl * 16] = vj;
    *(v4i *)&eI[q][is * NB_E + jq * 16] = vi;
  };

  v16f_ acc[RB][PB];
  const int sw16 = 16 * ((c >> 3) & 1);  // half swap of this lane's A rows
  const int jf = (c >> 1) & 7;           // j-side slot swizzle of this lane's SNP
  const int jrow = (half * BJ + c) * NB_REC, erow = (half * BJ + c) * NB_E;
  // one stage (128 individuals = two 64-deep k-steps) from LDS buffer b
  auto compute = [&](int b, bool diag) __attribute__((always_inline)) {
    const int bscale = diag ? 128 : 129;  // x2 (fp4 codes hold w/2), x4 beyond the diagonal block
    const v16f_ z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i j1 = *(const v4i *)&sJ[b][jrow + 16 * ((2 * kk + h) ^ jf)];
      const v4i j2 = j1 << 1;  // S2 = 2b = S1 << 1 (nibbles <= 4: no carry)
      v8i_ fb[PB];
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        const v4i i1 = *(const v4i *)&sI[b][(PB * w + t) * NB_REC + 32 * kk + 16 * h];
        const v4i i2 = *(const v4i *)&sI[b][(PB * w + t) * NB_REC + 64 + 32 * kk + 16 * h];
#pragma unroll
        for (int q = 0; q < 4; ++q) fb[t][q] = (i1[q] & j1[q]) | (i2[q] & j2[q]);
#pragma unroll
        for (int q = 4; q < 8; ++q) fb[t][q] = 0;
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const uint8_t *ar = &sA[b][(2 * kk + h) * 4096 + (32 * r + c) * 32];
        const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
        const v8i_ fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int t = 0; t < PB; ++t)
          acc[r][t] = mfma_mx(fa, fb[t], (diag && kk == 0) ? z : acc[r][t], hi[2], bscale);
      }
    }
  };

  double tot[PB];
  unsigned sw[PB];
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    tot[t] = 0.0;
    sw[t] = 0;
  }
  // epilogue of a K-block: sum_rows w[row] * acc[row]; acc register e of this lane <-> storage
  // slot 16h + e of each 32-row tile <-> nibble e of the 8 bytes at 16r + 8h of the planes
  auto epilogue = [&](int q) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      v2f_ s2 = {0.f, 0.f};
      unsigned sq = 0;
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const v2i_ m1 = *(const v2i_ *)&eI[q][(PB * w + t) * NB_E + 16 * r + 8 * h];
        const v2i_ m2 = *(const v2i_ *)&eI[q][(PB * w + t) * NB_E + 64 + 16 * r + 8 * h];
        const v2i_ b1 = *(const v2i_ *)&eJ[q][erow + 16 * r + 8 * h];
        const v2i_ b2 = *(const v2i_ *)&eJ[q][erow + 64 + 16 * r + 8 * h];
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const unsigned wd = (unsigned)((m1[d] & b1[d]) | (m2[d] & b2[d]));
          sq = __builtin_amdgcn_udot8(wd, wd, sq, false);  // codes are the integers w
#pragma unroll
          for (int bb = 0; bb < 4; ++bb) {
            const v2f_ wf = bb == 0 ? fp4_pair<0>(wd) : bb == 1 ? fp4_pair<1>(wd) : bb == 2 ? fp4_pair<2>(wd) : fp4_pair<3>(wd);
            const v2f_ av = {acc[r][t][8 * d + 2 * bb], acc[r][t][8 * d + 2 * bb + 1]};
            s2 = __builtin_elementwise_fma(wf, av, s2);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // consume the accumulators a tile at a time
      }
      tot[t] += (double)s2[0] + (double)s2[1];
      sw[t] += sq;
    }
  };

  // one stage from buffer b with the next stage (nkb, ncs) fetched meanwhile into buffer b^1
  auto iter = [&](int b, bool diag, int nkb, int ncs) __attribute__((always_inline)) {
    load(nkb, ncs);
    __builtin_amdgcn_sched_barrier(0);  // keep the next stage's fetch ahead of this stage's work
    compute(b, diag);
    store(b ^ 1);
    __syncthreads();
  };

  load(0, 0);
  store(0);
  __syncthreads();
  keep_diag(0, 0);
  int b = 0;
  for (int kb = 0; kb < nK; ++kb) {
    // stages (kb, kb) .. (kb, nK-1); the last one prefetches (kb+1, kb+1) (clamped at the end)
    const int nb = kb + 1 < nK ? kb + 1 : kb;
    if (kb + 1 < nK) iter(b, true, kb, kb + 1);
    else iter(b, true, nb, nb);
    b ^= 1;
#pragma unroll 1
    for (int cs = kb + 1; cs < nK; ++cs) {
      const bool lastc = cs + 1 == nK;
      iter(b, false, lastc ? nb : kb, lastc ? nb : cs + 1);
      b ^= 1;
    }
    if (kb + 1 < nK) keep_diag(b, (kb + 1) & 1);  // buffer b now holds stage (kb+1, kb+1)
    epilogue(kb & 1);
  }
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    const double other = __shfl_xor(tot[t], 32);
    const unsigned osw = __shfl_xor(sw[t], 32);
    if (h != 0 || ti[t] < 0) continue;
    cand_test(a, trow[PB * w + t], ti[t], J0 + c, tot[t] + other, (double)(sw[t] + osw));
  }
}

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

// Workgroup / wave layout, tile entries, staging and LDS images as mx_screen_kernel (MxShape<1>);
// per tile the loop is chunk ch (128 eigen-directions) -> stage (SK x 128 individuals, one barrier),
// every stage a full K-sweep step (no symmetry), with the chunk's epilogue after its last stage.
// Each workgroup works through several tile entries (b, b + grid, ...; the grid is a multiple of 8,
// so an entry keeps the XCD it was dealt to), and a tile's fixed costs run beside its stages:
//  * the first stage of the next chunk / tile is loaded during the last stage of this one and lands
//    during the epilogue and the test;
//  * the chunk's epilogue operands (G' rows of the 16 slots, H rows of the 64 columns) and, with the
//    first chunk, every test operand (E3 slices, code products, per-SNP records: a lane fetches those
//    of its own pair) are fetched by LDS-DMA as the youngest operations of the second-to-last stage,
//    whose wait (a counted vmcnt: VMEM operations retire in order) lets them land during the last
//    stage.  Every wait is one asm statement with the barrier (vm_wait_barrier): the compiler does
//    not know that the DMA asm writes LDS.
// NSL LDS stage slots (a ring): stage g + NSL - 1 is loaded while stage g multiplies.
template <int SK, int NSL>
__global__ __launch_bounds__(MxShape<1>::T, 1) void lr_screen_kernel(ScreenArgs a, LrArgs x) {
  constexpr int PB = MxShape<1>::PB, RB = MX_RB, MX_T = MxShape<1>::T, NA = MX_TILE / 16 / MX_T;
  // j side: only the S1 plane (first 64 bytes of a record: b as fp4 codes) is staged, S2 = S1 << 1
  constexpr int JB = NB_REC / 2, SI = MX_BI * NB_REC, SJ = 2 * BJ * JB;
  static_assert(PB == 2, "one slot per lane half");
  __shared__ __attribute__((aligned(16))) uint8_t sA[NSL][SK * MX_TILE];
  __shared__ __attribute__((aligned(16))) uint8_t sI[NSL][SK * SI];
  __shared__ __attribute__((aligned(16))) uint8_t sJ[NSL][SK * SJ];
  __shared__ __attribute__((aligned(16))) uint8_t sE[40 * 1024];    // chunk epilogue operands
  __shared__ __attribute__((aligned(16))) uint8_t sT[LR_ST_BYTES];  // test operands
  // per-lane DMA source offsets parked in LDS (registers are the loop's): [tile parity][thread] the
  // stage record offset (i side for waves 0, 1, j side for waves 4..7), [tile parity][lane] wave 0's
  // slot record offset
  __shared__ unsigned sO[2][MxShape<1>::T], sRo[2][64];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int half = (PB * w) / (MX_BI / 2);  // this wave's column block
  const int nK = x.nK, nC = x.nC, nS = nK / SK, G = (int)gridDim.x;
  const int64_t R = x.R;
  auto next_entry = [&](int e) __attribute__((always_inline)) {
    while (e < x.n_tiles && a.tiles[MX_TE * e] < 0) e += G;
    return e < x.n_tiles ? e : -1;
  };
  int e = next_entry((int)blockIdx.x);
  if (e < 0) return;

  // Stage operands by LDS-DMA (global_load_lds_dwordx4: lane i's 16 bytes land at M0 + 16 i): the A
  // tile image (NA wave-instructions per image), the j-side S1 planes (waves 4..7: 16 columns x 4
  // chunks each, physical chunk p of column js holding logical chunk p ^ ((js >> 2) & 3): the 16
  // lanes of a ds_read_b128 group hit 16 distinct 16-byte bank slots) and the i-side records (waves
  // 0 and 1: 16 slots x 8 chunks).  Lanes whose
  // column or slot is unused read SNP 0 (finite data in accumulators nobody tests).
  auto src_offsets = [&](int tl, int J0t, int J1t, unsigned &oI, unsigned &oJ) __attribute__((always_inline)) {
    oI = oJ = 0;
    if (w >= 4) {
      const int jc = tid - 256, jh = jc >> 7, js = (jc >> 2) & 31, jq = jc & 3;
      const int Jh = jh ? J1t : J0t;
      const int64_t jj = (int64_t)Jh * BJ + js;
      oJ = (unsigned)(((Jh >= 0 && jj < a.m) ? jj : 0) * nK * NB_REC + (jq ^ ((js >> 2) & 3)) * 16);
    }
    if (w < 2) {
      const int r = a.tile_rows[(int64_t)tl * MX_BI + (tid >> 3)];
      oI = (unsigned)((r >= 0 ? a.rows[r] : 0) * nK * NB_REC + (tid & 7) * 16);
    }
  };
  auto load = [&](int nb, int ch, int cs2, unsigned oI, unsigned oJ) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < SK; ++s) {
      const int cs = cs2 * SK + s;
      const uint8_t *src = x.tiles + (int64_t)(ch * nK + cs) * MX_TILE;
#pragma unroll
      for (int u = 0; u < NA; ++u)
        lds_dma16(src + (tid + u * MX_T) * 16, &sA[nb][s * MX_TILE + (w * 64 + u * MX_T) * 16]);
      if (w >= 4) lds_dma16(x.nib_j + oJ + cs * NB_REC, &sJ[nb][s * SJ + (w - 4) * 1024]);
      if (w < 2) lds_dma16(x.nib_i + oI + cs * NB_REC, &sI[nb][s * SI + w * 1024]);
    }
  };
  const int NL = SK * (NA + (w >= 4 ? 1 : 0) + (w < 2 ? 1 : 0));  // this wave's DMAs per stage load

  v16f_ acc[RB][PB];
  const int sw16 = 16 * ((c >> 3) & 1);
  const int jf = (c >> 2) & 3;
  const int jrow = (half * BJ + c) * JB;
  // A fragment r of (stage s, half kk): the 6 fp6 dwords + the scale dword of row 32 r + c
  auto afrag = [&](int b, int s, int kk, int r) __attribute__((always_inline)) {
    const uint8_t *ar = &sA[b][s * MX_TILE + (2 * kk + h) * 4096 + (32 * r + c) * 32];
    const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
    return v8i_{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  // Software-pipelined: the next A fragment is read from LDS while the current one's MFMAs run
  // (the compiler otherwise waits for every fragment right before its MFMAs).
  auto compute = [&](int b, bool first) __attribute__((always_inline)) {
    const v16f_ z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    v8i_ fa = afrag(b, 0, 0, 0);
#pragma unroll
    for (int s = 0; s < SK; ++s)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const v4i j1 = *(const v4i *)&sJ[b][s * SJ + jrow + 16 * ((2 * kk + h) ^ jf)];
        const v4i j2 = j1 << 1;
        v8i_ fb[PB];
#pragma unroll
        for (int t = 0; t < PB; ++t) {
          const v4i i1 = *(const v4i *)&sI[b][s * SI + (PB * w + t) * NB_REC + 32 * kk + 16 * h];
          const v4i i2 = *(const v4i *)&sI[b][s * SI + (PB * w + t) * NB_REC + 64 + 32 * kk + 16 * h];
#pragma unroll
          for (int q = 0; q < 4; ++q) fb[t][q] = (i1[q] & j1[q]) | (i2[q] & j2[q]);
#pragma unroll
          for (int q = 4; q < 8; ++q) fb[t][q] = 0;
        }
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          const bool last = s == SK - 1 && kk == 1 && r == RB - 1;
          const int ns = r < RB - 1 ? s : (kk == 1 ? s + 1 : s), nkk = r < RB - 1 ? kk : (kk ^ 1);
          const v8i_ fn = last ? fa : afrag(b, ns, nkk, (r + 1) % RB);
#pragma unroll
          for (int t = 0; t < PB; ++t)  // x2 (scale 128): the fp4 codes hold w/2
            acc[r][t] = mfma_mx(fa, fb[t], (first && s == 0 && kk == 0) ? z : acc[r][t], fa[6], 128);
          fa = fn;
        }
      }
  };
  // Chunk epilogue operands (1 KB per wave instruction q, written linearly at sE + q KB): q 0..7 =
  // G' rows of the 16 slots (512 B each), q 8..39 = H rows of the 64 columns (physical 16-byte chunk
  // p of column row holds logical chunk p ^ (row & 15): conflict-free reads).  Wave w issues q = w,
  // 8 + w, .., 32 + w.
  // The fetches' pointers and lane indices are laundered through empty asm at the point of use: the
  // compiler would otherwise hoist their address arithmetic out of the stage loop and keep it in
  // registers the accumulators need.
  auto fetch_epi = [&](int ch, int J0t, int J1t, int64_t i0, int64_t i1) __attribute__((always_inline)) {
    const float *Gp = x.G, *Hp = x.H;
    int ln = lane;
    asm volatile("" : "+s"(Gp), "+s"(Hp), "+v"(ln));
    const int hh = ln >> 5, cc = ln & 31;
    const int64_t ig = hh ? i1 : i0;
    lds_dma16(Gp + (ig < 0 ? 0 : ig) * R + ch * MXK + 4 * cc, &sE[w * 1024]);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int row = 2 * (w + 8 * u) + hh;
      const int Jh = (row >> 5) ? J1t : J0t;
      const int64_t jj = Jh < 0 ? 0 : min((int64_t)Jh * BJ + (row & 31), a.m - 1);
      lds_dma16(Hp + jj * R + ch * MXK + 4 * (cc ^ (row & 15)), &sE[(8 + w + 8 * u) * 1024]);
    }
  };
  // Test operands of the lane's own pair (slot 2w + h, column c of the wave's block): SIDE_T + 4
  // planes by global_load_lds_dword (lane i's 4 bytes at M0 + 4 i); wave 0 fetches the 16 slot
  // records (lane: slot lane / 4, quarter lane % 4), waves 1..4 the 64 column records (16 each).
  // Unused slots / columns read offset 0 (SNP 0, band row 0, column j_lo).
  auto fetch_test = [&](int J0t, int J1t, int ri, unsigned orec) __attribute__((always_inline)) {
    const int *c13 = a.c13, *pfc = a.pfc;
    const double *recL = x.recL, *recR = x.recR;
    int ln = lane;
    asm volatile("" : "+s"(c13), "+s"(pfc), "+s"(recL), "+s"(recR), "+v"(ln));
    const int Jh = half ? J1t : J0t;
    const int64_t j = (int64_t)Jh * BJ + (ln & 31);
    const bool ok = ri >= 0 && Jh >= 0 && j >= a.j_lo && j < a.m;
    const int64_t o1 = ok ? (int64_t)ri * a.ld_e + (j - a.j_lo) : 0;
    const int64_t o3 = ok ? o1 + (int64_t)a.n_rows * a.ld_e : 0;
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t)
      lds_dma4(c13 + (t < a.e3_t ? t * a.c13_stride + o3 : 0), sT + t * LR_PLANE + 2 * w * BJ * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k)
      lds_dma4(pfc + k * a.pfc_stride + o1, sT + (SIDE_T + k) * LR_PLANE + 2 * w * BJ * 4);
    if (w == 0) lds_dma16(recL + orec, sT + LR_OFF_RL);
    if (w >= 1 && w <= 4) {
      const int col = 16 * (w - 1) + (ln >> 2);
      const int Jc = (col >> 5) ? J1t : J0t;
      const int64_t jj = Jc < 0 ? 0 : min((int64_t)Jc * BJ + (col & 31), a.m - 1);
      lds_dma16(recR + jj * LR_REC + 2 * (ln & 3), sT + LR_OFF_RR + (w - 1) * 1024);
    }
  };
  // sum of c~_r^2 over the chunk's rows: c~ = acc - beta G' - alpha H, two rows per v_pk_fma_f32
  const int hrow = half * BJ + c;
  // (r, q) outer: one H chunk per (r, q) serves both slots; the reads of a row tile are issued
  // together (no scheduling barrier: the epilogue is latency-, not register-bound)
  auto epilogue = [&](double *lowrank) __attribute__((always_inline)) {
    const float be = (float)((const double *)(sT + LR_OFF_RR))[hrow * LR_REC];
    const v2f_ nbe = {-be, -be};
    v2f_ nal[PB], s2[PB];
#pragma unroll
    for (int t = 0; t < PB; ++t) {
      const float al = (float)((const double *)(sT + LR_OFF_RL))[(PB * w + t) * LR_REC];
      nal[t] = v2f_{-al, -al};
      s2[t] = v2f_{0.f, 0.f};
    }
#pragma unroll
    for (int r = 0; r < RB; ++r) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int k = 8 * r + 2 * q + h;  // logical 16-byte chunk of the chunk's 128 rows
        const float4 hh = *(const float4 *)&sE[8192 + hrow * 512 + 16 * (k ^ (hrow & 15))];
#pragma unroll
        for (int t = 0; t < PB; ++t) {
          const float4 g = *(const float4 *)&sE[(PB * w + t) * 512 + 16 * k];
#pragma unroll
          for (int u = 0; u < 4; u += 2) {
            const v2f_ av = {acc[r][t][4 * q + u], acc[r][t][4 * q + u + 1]};
            const v2f_ gv = {u ? g.z : g.x, u ? g.w : g.y}, hv = {u ? hh.z : hh.x, u ? hh.w : hh.y};
            v2f_ cr = __builtin_elementwise_fma(nbe, gv, av);
            cr = __builtin_elementwise_fma(nal[t], hv, cr);
            s2[t] = __builtin_elementwise_fma(cr, cr, s2[t]);
          }
        }
      }
    }
#pragma unroll
    for (int t = 0; t < PB; ++t) lowrank[t] += (double)s2[t][0] + (double)s2[t][1];
  };

  constexpr int LA = NSL - 1;  // stages in flight beyond the one being multiplied
  const int P = nC * nS;        // stages per tile
  int tl = a.tiles[MX_TE * e], J0t = a.tiles[MX_TE * e + 1], J1t = a.tiles[MX_TE * e + 2];
  {
    unsigned oI, oJ;
    src_offsets(tl, J0t, J1t, oI, oJ);
    sO[0][tid] = w < 2 ? oI : oJ;
  }
  // Vector-memory bookkeeping (wave-uniform): `issued` counts this wave's DMAs; at the start of stage
  // g, mk[k] (k < LA - 1) is its value right after the loads of stage g + 1 + k (the stages in flight,
  // oldest first); the stage appends stage g + LA's mark, and waiting for stage g + 1 is
  // vmcnt(issued - mk[0]) (VMEM operations retire in order).
  int issued = 0, mk[LA];
  int g = 0;  // this workgroup's stage counter: stage g lives in slot g % NSL
  // the stage q positions ahead of the tile start (chunk, stage of the tile, or of the next tile)
  auto issue = [&](int q, int slot, int pr, int en_) __attribute__((always_inline)) {
    if (q < P) {
      const unsigned o = sO[pr][tid];
      load(slot, q / nS, q % nS, o, o);
      issued += NL;
    } else if (en_ >= 0) {
      const unsigned o = sO[pr ^ 1][tid];
      load(slot, 0, q - P, o, o);
      issued += NL;
    }
  };
#pragma unroll
  for (int q = 0; q < LA; ++q) {
    issue(q, q, 0, -1);
    mk[q] = issued;
  }
  vm_wait_barrier(issued - mk[0]);  // stage 0 of the first tile
#pragma unroll
  for (int q = 0; q + 1 < LA; ++q) mk[q] = mk[q + 1];
  int par = 0;
  for (;;) {
    // this tile's slots (wave-uniform: slots 2w, 2w + 1) and the next entry's stage sources
    const int *trow = a.tile_rows + (int64_t)tl * MX_BI;
    const int r0 = trow[PB * w], r1 = trow[PB * w + 1];
    const int64_t i0 = r0 >= 0 ? a.rows[r0] : -1, i1 = r1 >= 0 ? a.rows[r1] : -1;
    const int en = next_entry(e + G);
    int tln = 0, J0n = -1, J1n = -1;
    if (en >= 0) {
      tln = a.tiles[MX_TE * en];
      J0n = a.tiles[MX_TE * en + 1];
      J1n = a.tiles[MX_TE * en + 2];
      unsigned oIn, oJn;
      src_offsets(tln, J0n, J1n, oIn, oJn);
      sO[par ^ 1][tid] = w < 2 ? oIn : oJn;
    }
    if (w == 0) {  // the slot record quarter this lane fetches
      const int r = trow[lane >> 2];
      sRo[par][lane] = (unsigned)((r >= 0 ? a.rows[r] : 0) * LR_REC + 2 * (lane & 3));
    }
    // (the tile's first stage was waited for by the previous stage or the prologue)
    double lowrank[PB] = {0.0, 0.0};
    for (int ch = 0; ch < nC; ++ch) {
      // one stage at tile position p: load the stage LA ahead (possibly of the next tile), the
      // epilogue (and with the first chunk the test) operands after it with the chunk's first stage,
      // multiply, then wait for the next stage (the younger DMAs stay in flight)
      auto stage = [&](int cs2, bool first) __attribute__((always_inline)) {
        const int p = ch * nS + cs2;
        issue(p + LA, (g + LA) % NSL, par, en);
        mk[LA - 1] = issued;
        if (first) {
          fetch_epi(ch, J0t, J1t, i0, i1);
          issued += 5;
          if (ch == 0) {
            fetch_test(J0t, J1t, h ? r1 : r0, w == 0 ? sRo[par][lane] : 0u);
            issued += SIDE_T + 4 + (w <= 4 ? 1 : 0);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        compute(g % NSL, first);
        const bool more = p + 1 < P || en >= 0;
        vm_wait_barrier(more ? issued - mk[0] : 0);
#pragma unroll
        for (int q = 0; q + 1 < LA; ++q) mk[q] = mk[q + 1];
        ++g;
      };
      stage(0, true);
#pragma unroll 1
      for (int cs2 = 1; cs2 < nS; ++cs2) stage(cs2, false);
      epilogue(lowrank);
      __syncthreads();  // every wave is past the epilogue's reads of sE before the next fetch
    }
    // lane half h tests slot PB w + h of column c (both halves hold the sums after the exchange)
    {
      const double tot = (h ? lowrank[1] : lowrank[0]) + __shfl_xor(h ? lowrank[0] : lowrank[1], 32);
      const int ri = h ? r1 : r0;
      const int64_t i = h ? i1 : i0;
      const int Jh = half ? J1t : J0t;
      const int64_t j = (int64_t)Jh * BJ + c;
      const bool ok = i >= 0 && ri >= 0 && Jh >= 0 && j >= a.j_lo && j < a.m && !(a.tri && j <= i);
      lr_test(a, x, sT, PB * w + h, c, half, ok, i, j, tot);
    }
    if (en < 0) break;
    __syncthreads();  // every wave is past the test's reads of sT before the next tile's fetch
    e = en;
    tl = tln;
    J0t = J0n;
    J1t = J1n;
    par ^= 1;
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
// j-side bytes per column and stage: the S1 plane at 2 bits (J2) or as the nibble plane
template <bool J2> constexpr int lrc_jb() { return J2 ? 32 : 64; }

// slot pair p's record (lc_fill: the prefilter's E3 slices and code products of the pair)
__device__ __forceinline__ void lrc_test(const ScreenArgs &a, const LrcArgs &x, int64_t p, int64_t i, int64_t j,
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
  if (!(vlo > 0.0) || eff_hi * eff_hi * (1.0 + 1e-9) >= a.chi_cut * vlo) {
    const unsigned long long k = atomicAdd(a.counter, 1ULL);
    if ((int64_t)k < a.cap) {
      a.cand_i[k] = i;
      a.cand_j[k] = j;
    }
  }
}

template <bool J2, int NSL>
__global__ __launch_bounds__(512, 1) void lrc_screen_kernel(ScreenArgs a, LrcArgs x) {
  constexpr int T = 512, RB = MX_RB, PB = 2, NA = MX_TILE / 16 / T, LA = NSL - 1;
  constexpr int LRC_JB = lrc_jb<J2>(), NJ = LRC_JB / 16;  // j-side bytes per column and stage; DMAs per wave
  __shared__ __attribute__((aligned(16))) uint8_t sA[NSL][MX_TILE];
  __shared__ __attribute__((aligned(16))) uint8_t sI[NSL][MX_BI * NB_REC];
  __shared__ __attribute__((aligned(16))) uint8_t sJ[NSL][MX_BI * 32 * LRC_JB];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nK = x.nK, nC = x.nC;
  const int64_t R = x.R;
  const int sbase = (int)blockIdx.x * MX_BI;  // the tile's first slot
  // this wave's two slots (wave-uniform)
  const int rr0 = x.slot_row[sbase + PB * w], rr1 = x.slot_row[sbase + PB * w + 1];
  if (__builtin_amdgcn_readfirstlane(x.slot_row[sbase]) < 0) return;  // empty tile (never queued)
  const int64_t i0 = rr0 >= 0 ? a.rows[rr0] : -1, i1 = rr1 >= 0 ? a.rows[rr1] : -1;
  // DMA sources.  j side (round 4: the S1 planes at 2 bits, 32 B per column and stage, half the bytes
  // of the nibble plane): instruction u of wave w moves its slots' (t, column, 16-byte chunk) = item
  // 64 u + lane (t = item / 64, column = item / 2 % 32, physical chunk = item % 2 holding logical chunk
  // (item % 2) ^ ((column >> 3) & 1): 2-way bank conflicts at most on the 8-byte reads).
  // (!J2: the nibble plane, 64 B, four chunks per column, physical chunk (item % 4) ^ ((column >> 2) & 3))
  unsigned oJ[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int item = 64 * u + lane;
    const int t = J2 ? item >> 6 : item >> 7, col = J2 ? (item >> 1) & 31 : (item >> 2) & 31;
    const int pc = J2 ? item & 1 : item & 3, sw = J2 ? (col >> 3) & 1 : (col >> 2) & 3;
    const int rr = t ? rr1 : rr0;
    const int jj = rr >= 0 ? x.slot_j[(sbase + PB * w + t) * 32 + col] : -1;
    oJ[u] = (unsigned)((jj >= 0 ? jj : 0) * nK * (J2 ? LRC_JB : NB_REC) + (pc ^ sw) * 16);
  }
  unsigned oI = 0;  // i side (waves 0, 1): slot tid / 8 of the tile, 16-byte chunk tid % 8 of its record
  if (w < 2) {
    const int r = x.slot_row[sbase + (tid >> 3)];
    oI = (unsigned)((r >= 0 ? a.rows[r] : 0) * nK * NB_REC + (tid & 7) * 16);
  }
  auto load = [&](int nb, int q) __attribute__((always_inline)) {  // stage q = (chunk q / nK, stage q % nK)
    const int ch = q / nK, kc = q % nK;
    const uint8_t *src = x.tiles + (int64_t)(ch * nK + kc) * MX_TILE;
#pragma unroll
    for (int u = 0; u < NA; ++u) lds_dma16(src + (tid + u * T) * 16, &sA[nb][(w * 64 + u * T) * 16]);
#pragma unroll
    for (int u = 0; u < NJ; ++u)
      lds_dma16((J2 ? x.s1c2 + kc * LRC_JB : x.nib_j + kc * NB_REC) + oJ[u], &sJ[nb][w * NJ * 1024 + u * 1024]);
    if (w < 2) lds_dma16(x.nib_i + oI + kc * NB_REC, &sI[nb][w * 1024]);
  };
  const int NL = NA + NJ + (w < 2 ? 1 : 0);  // this wave's DMAs per stage
  v16f_ acc[RB][PB];
  const int sw16 = 16 * ((c >> 3) & 1), jf = J2 ? (c >> 3) & 1 : (c >> 2) & 3;
  auto afrag = [&](int b, int kk, int r) __attribute__((always_inline)) {
    const uint8_t *ar = &sA[b][(2 * kk + h) * 4096 + (32 * r + c) * 32];
    const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
    return v8i_{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  auto compute = [&](int b, bool first) __attribute__((always_inline)) {
    const v16f_ z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    v8i_ fa = afrag(b, 0, 0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8i_ fb[PB];
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        // logical 8-byte piece 2 kk + h of the column: chunk kk (swizzled), half h; expanded to the
        // nibble plane's four dwords (piece = D0 | D1 << 2, D2 | D3 << 2)
        v4i j1;
        if (J2) {
          const v2i_ e2 = *(const v2i_ *)&sJ[b][(PB * w + t) * 32 * LRC_JB + c * LRC_JB + 16 * (kk ^ jf) + 8 * h];
          j1 = v4i{e2[0] & 0x33333333, (e2[0] >> 2) & 0x33333333, e2[1] & 0x33333333, (e2[1] >> 2) & 0x33333333};
        } else {
          j1 = *(const v4i *)&sJ[b][(PB * w + t) * 32 * LRC_JB + c * LRC_JB + 16 * ((2 * kk + h) ^ jf)];
        }
        const v4i j2 = j1 << 1;
        const v4i m1 = *(const v4i *)&sI[b][(PB * w + t) * NB_REC + 32 * kk + 16 * h];
        const v4i m2 = *(const v4i *)&sI[b][(PB * w + t) * NB_REC + 64 + 32 * kk + 16 * h];
#pragma unroll
        for (int q = 0; q < 4; ++q) fb[t][q] = (m1[q] & j1[q]) | (m2[q] & j2[q]);
#pragma unroll
        for (int q = 4; q < 8; ++q) fb[t][q] = 0;
      }
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        const bool last = kk == 1 && r == RB - 1;
        const v8i_ fn = last ? fa : afrag(b, r < RB - 1 ? kk : 1, (r + 1) % RB);
#pragma unroll
        for (int t = 0; t < PB; ++t)  // x2 (scale 128): the fp4 codes hold w/2
          acc[r][t] = mfma_mx(fa, fb[t], (first && kk == 0) ? z : acc[r][t], fa[6], 128);
        fa = fn;
      }
    }
  };
  // chunk epilogue: sum_r (c~_r)^2, c~ = acc - beta_j G'(i) - alpha_i H(j), G' / H read from memory
  // (accumulator element e of lane (c, h) in row tile r is row 32 r + 8 (e / 4) + 4 h + e % 4)
  int64_t jc[PB];
  float nbe[PB], nal[PB];
#pragma unroll
  for (int t = 0; t < PB; ++t) {
    const int rr = t ? rr1 : rr0;
    const int jj = rr >= 0 ? x.slot_j[(sbase + PB * w + t) * 32 + c] : -1;
    jc[t] = jj;
    nbe[t] = jj >= 0 ? -(float)x.recR[(int64_t)jj * LR_REC] : 0.f;
    const int64_t ii = t ? i1 : i0;
    nal[t] = ii >= 0 ? -(float)x.recL[ii * LR_REC] : 0.f;
  }
  double lowrank[PB] = {0.0, 0.0};
  auto epilogue = [&](int ch) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      float4 g[PB][4], hv[PB][4];
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        const int64_t ii = t ? i1 : i0;
        const float *gp = x.G + (ii >= 0 ? ii : 0) * R + ch * MXK + 32 * r + 4 * h;
        const float *hp = x.H + (jc[t] >= 0 ? jc[t] : 0) * R + ch * MXK + 32 * r + 4 * h;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          g[t][q] = *(const float4 *)(gp + 8 * q);
          hv[t][q] = *(const float4 *)(hp + 8 * q);
        }
      }
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        v2f_ s2 = {0.f, 0.f};
        const v2f_ nb2 = {nbe[t], nbe[t]}, na2 = {nal[t], nal[t]};
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int u = 0; u < 4; u += 2) {
            const v2f_ av = {acc[r][t][4 * q + u], acc[r][t][4 * q + u + 1]};
            const v2f_ gv = {u ? g[t][q].z : g[t][q].x, u ? g[t][q].w : g[t][q].y};
            const v2f_ hh = {u ? hv[t][q].z : hv[t][q].x, u ? hv[t][q].w : hv[t][q].y};
            v2f_ cr = __builtin_elementwise_fma(nb2, gv, av);
            cr = __builtin_elementwise_fma(na2, hh, cr);
            s2 = __builtin_elementwise_fma(cr, cr, s2);
          }
        lowrank[t] += (double)s2[0] + (double)s2[1];
      }
    }
  };
  // stage pipeline: LA stages in flight; slot of stage q is q % NSL; the wait before stage q + 1
  // leaves the younger stages' DMAs in flight (VMEM operations retire in order)
  const int P = nC * nK;
  for (int q = 0; q < LA && q < P; ++q) load(q % NSL, q);
  vm_wait_barrier(NL * (min(LA, P) - 1));
  for (int q = 0; q < P; ++q) {
    if (q + LA < P) load((q + LA) % NSL, q + LA);  // its slot was read in stage q - 1 (barrier passed)
    const int kc = q % nK;
    compute(q % NSL, kc == 0);
    if (kc == nK - 1) epilogue(q / nK);
    const int ahead = min(q + LA, P - 1) - (q + 1);  // stages issued beyond q + 1
    vm_wait_barrier(q + 1 < P ? NL * ahead : 0);
  }
  // lane half h tests slot PB w + h, column c (the other half-wave's rows of the same column added)
  const double tot = (h ? lowrank[1] : lowrank[0]) + __shfl_xor(h ? lowrank[0] : lowrank[1], 32);
  const int ri = h ? rr1 : rr0;
  const int64_t i = h ? i1 : i0, j = h ? jc[1] : jc[0];
  if (ri >= 0 && j >= 0) lrc_test(a, x, (int64_t)(sbase + PB * w + h) * 32 + c, i, j, tot);
}

// Left / right test records of a coding (lr_screen_kernel's per-SNP test operands in one 64-byte
// record each: one LDS-DMA chunk per quarter)
__global__ void lr_rec_kernel(int64_t m, const double *soff, const double *csum, const double *csq, const double *sL3,
                              const double *sa, const double *sb, const uint8_t *mono, double *recL, double *recR) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const double mo = mono[j] ? 1.0 : 0.0;
  const double l[LR_REC] = {soff[j], csum[j], csq[j], sL3[j], sa[j], mo, 0.0, 0.0};
  const double r[LR_REC] = {soff[j], csum[j], csq[j], sb[j], mo, 0.0, 0.0, 0.0};
#pragma unroll
  for (int k = 0; k < LR_REC; ++k) {
    recL[j * LR_REC + k] = l[k];
    recR[j * LR_REC + k] = r[k];
  }
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
__global__ __launch_bounds__(RT, 2) void refine_kernel(int64_t n_pad, const double *__restrict__ P,
                                                       const double *__restrict__ py, const int8_t *left,
                                                       const int8_t *right, const double *alpha, const double *beta,
                                                       const int64_t *pi, const int64_t *pj, int64_t np, double *eff,
                                                       double *var, double *eff_part, double *var_part) {
  __shared__ double As[RK][RM + 1];
  __shared__ double Bs[RK][RP + 1];
  __shared__ double red[4][RP];
  // 8 waves: rows 32 (w >> 1) .. +32 of the row block x pairs 64 (w & 1) .. +64
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wm = w >> 1, wn = w & 1;
  const int64_t p0 = (int64_t)blockIdx.x * RP;
  // staging roles: A row ar = tid / 4, 8 doubles from column ak; E column gcol, 8 k from gk
  const int ar = tid >> 2, ak = (tid & 3) * 8;
  const int gcol = tid & (RP - 1), gk = (tid >> 7) * 8;
  const int64_t gp = p0 + gcol;
  const bool gval = gp < np;
  const int8_t *gl = gval ? left + pi[gp] * n_pad : left;
  const int8_t *gr = gval ? right + pj[gp] * n_pad : right;
  const double gal = gval ? alpha[pi[gp]] : 0.0, gbe = gval ? beta[pj[gp]] : 0.0;
  double vpart[4] = {0, 0, 0, 0};  // per 16-pair subtile partial of var
  double effp = 0.0;
  v2d_ ra[4];
  v2i__ rl, rr;
  auto fetch = [&](int64_t rb, int64_t k0) __attribute__((always_inline)) {
    const v2d_ *src = (const v2d_ *)(P + (rb + ar) * n_pad + k0 + ak);
#pragma unroll
    for (int q = 0; q < 4; ++q) ra[q] = src[q];
    rl = *(const v2i__ *)(gl + k0 + gk);
    rr = *(const v2i__ *)(gr + k0 + gk);
  };
  // this segment's stages [tb, te) of the sequence (rb = 0, RM, ..; k0 = rb, rb + RK, .. < n_pad)
  int64_t T = 0;
  for (int64_t b = 0; b < n_pad; b += RM) T += (n_pad - b) / RK;
  const int seg = blockIdx.y, nseg = gridDim.y;
  const int64_t tb = T * seg / nseg, te = T * (seg + 1) / nseg;
  int64_t rb = 0, t = 0;
  while (t + (n_pad - rb) / RK <= tb) {
    t += (n_pad - rb) / RK;
    rb += RM;
  }
  int64_t k0 = rb + (tb - t) * RK, nleft = te - tb;
  if (nleft > 0) fetch(rb, k0);
  while (nleft > 0) {
    v4d acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = v4d{0, 0, 0, 0};
    // symmetric P: only column blocks k0 >= rb, the off-diagonal ones counted twice (x2 is
    // exact); the rb == 0 stages cover every k and also accumulate the eff partials
    for (; k0 < n_pad && nleft > 0; k0 += RK, --nleft) {
      const double f = k0 >= rb + RM ? 2.0 : 1.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        As[ak + 2 * q][ar] = f * ra[q][0];
        As[ak + 2 * q + 1][ar] = f * ra[q][1];
      }
      {
        const int8_t *lb = (const int8_t *)&rl, *rbb = (const int8_t *)&rr;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const double e = gval ? ((double)lb[q] - gal) * ((double)rbb[q] - gbe) : 0.0;
          Bs[gk + q][gcol] = e;
          if (rb == 0) effp += e * py[k0 + gk + q];
        }
      }
      __syncthreads();
      {  // next stage (this row block's next columns, or the next row block's first)
        int64_t nrb = rb, nk = k0 + RK;
        if (nk >= n_pad) {
          nrb = rb + RM;
          nk = nrb;
        }
        if (nleft > 1 && nrb < n_pad) fetch(nrb, nk);
      }
#pragma unroll
      for (int ks = 0; ks < RK / 4; ++ks) {
        const int kk = ks * 4 + (lane >> 4);
        const double a0 = As[kk][wm * 32 + (lane & 15)], a1 = As[kk][wm * 32 + 16 + (lane & 15)];
#pragma unroll
        for (int jt = 0; jt < 4; ++jt) {
          const double bj = Bs[kk][wn * 64 + jt * 16 + (lane & 15)];
          acc[0][jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, bj, acc[0][jt], 0, 0, 0);
          acc[1][jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, bj, acc[1][jt], 0, 0, 0);
        }
      }
      __syncthreads();
    }
    // fold: var[col] += sum_rows E[row][col] * C[row][col]
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const int col = wn * 64 + jt * 16 + (lane & 15);
      const int64_t p = p0 + col;
      if (p >= np) continue;
      const int8_t *l = left + pi[p] * n_pad, *r = right + pj[p] * n_pad;
      const double al = alpha[pi[p]], be = beta[pj[p]];
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t row = rb + wm * 32 + it * 16 + (lane >> 4) + 4 * e;
          vpart[jt] += ecode(l, r, al, be, row) * acc[it][jt][e];
        }
    }
    if (k0 >= n_pad) {
      rb += RM;
      k0 = rb;
    }
  }
  // reduce var partials: lanes with equal (lane & 15) in a wave, then the four wm waves
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    double v = vpart[jt];
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (lane < 16) red[wm][wn * 64 + jt * 16 + lane] = v;
  }
  // eff partials: 4 threads per column (tid >> 7), reduce via LDS after var
  __syncthreads();
  __shared__ double effr[4][RP];
  effr[tid >> 7][gcol] = effp;
  __syncthreads();
  if (tid < RP) {
    const int col = tid;
    const int64_t p = p0 + col;
    if (p < np) {
      const double v = (red[0][col] + red[1][col]) + (red[2][col] + red[3][col]);
      const double f = (effr[0][col] + effr[1][col]) + (effr[2][col] + effr[3][col]);
      if (nseg == 1) {
        var[p] = v;
        eff[p] = f;
      } else {
        var_part[seg * np + p] = v;
        eff_part[seg * np + p] = f;
      }
    }
  }
}

// var / eff = the segments' partials added in segment order (deterministic)
__global__ void refine_sum_kernel(int64_t np, int nseg, const double *eff_part, const double *var_part, double *eff,
                                  double *var) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  double v = 0.0, f = 0.0;
  for (int s = 0; s < nseg; ++s) {
    v += var_part[s * np + t];
    f += eff_part[s * np + t];
  }
  var[t] = v;
  eff[t] = f;
}

// p-values and hit compaction: chi = eff^2/var, p = chi2.sf(chi, 1) = erfc(sqrt(chi/2))
__global__ void pvalue_kernel(int64_t np, const double *eff, const double *var, double *chi, double *p) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= np) return;
  const double c = eff[t] * eff[t] / var[t];
  chi[t] = c;
  p[t] = (c < 0.0) ? 1.0 : erfc(sqrt(0.5 * c));
}

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
__host__ __device__ inline int64_t r8_toff(int64_t kb, int64_t NS) {  // tiles of the row blocks before kb
  const int64_t h = kb >> 1;
  return kb * NS - ((kb & 1) ? h * h : h * (h - 1));
}
// the 16-byte chunk swizzle of a tile row (row & 15): chunk k of row r sits at k ^ r8_swz(r), so that
// each 16-lane group of refine8_kernel's ds_read_b128 (rows c, chunks g) covers all 64 banks (k ^ (r & 3)
// alone left rows r and r + 4 on the same banks: 2-way conflicts, ~20 % of the kernel's cycles)
__host__ __device__ inline int r8_swz(int r) { return (r & 3) ^ ((r >> 1) & 2); }
__global__ void r8_image_kernel(int64_t n_pad, const double *__restrict__ Ps, double inv_unit, int8_t *__restrict__ tiles) {
  const int64_t NB = n_pad / 32, NS = n_pad / 64;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // (row, column) of a tile row
  const int64_t rs = idx / n_pad, cc = idx % n_pad;  // storage row, column
  if (rs >= n_pad) return;
  const int64_t kb = rs / 32, cs = cc / 64;
  if (cs < kb / 2) return;
  const int64_t bc = cc / 32;
  const double f = bc > kb ? 2.0 : (bc == kb ? 1.0 : 0.0);
  double r = (rs != cc) ? f * Ps[rs * n_pad + cc] * inv_unit : 0.0;
  const int rt = (int)((rs % 32) / 16), row = (int)(rs % 16), k = (int)(cc % 64);
  int8_t *t = tiles + (r8_toff(kb, NS) + cs - kb / 2) * R8_TILE + (rt * 16 + row) * 64 + 16 * ((k / 16) ^ r8_swz(row)) + k % 16;
  for (int s = 0; s < R8_S; ++s) {
    const double q = rint(r);
    t[s * R8_TB] = (int8_t)q;
    r = (r - q) * 128.0;
  }
  (void)NB;
}

__global__ __launch_bounds__(512, 1) void refine8_kernel(int64_t n_pad, const int8_t *__restrict__ tiles,
                                                         const int8_t *__restrict__ sl, const int8_t *__restrict__ sr,
                                                         const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                         int64_t np, double unit, double *__restrict__ varw,
                                                         double *__restrict__ tpart) {
  constexpr int NSL = 8, LA = 6;  // ring slots, tiles in flight (112 KB of LDS)
  __shared__ __attribute__((aligned(16))) int8_t sA[NSL][R8_TILE];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = (int)(n_pad / 32), NS = (int)(n_pad / 64);
  // segment blockIdx.y of gridDim.y: the row blocks [kb_lo, kb_hi) holding its share of the tiles (a
  // short pair list is spread over more workgroups); its per-slice integer sums go to tpart, added by
  // refine8_side_kernel (exact: the same bits for any number of segments)
  const int nseg = (int)gridDim.y, seg = (int)blockIdx.y;
  const int64_t N_all = r8_toff(NB, NS);
  int kb_lo = 0, kb_hi = 0;
  while (kb_lo < NB && r8_toff(kb_lo, NS) * nseg < N_all * seg) ++kb_lo;
  kb_hi = kb_lo;
  while (kb_hi < NB && r8_toff(kb_hi, NS) * nseg < N_all * (seg + 1)) ++kb_hi;
  const int N = (int)(r8_toff(kb_hi, NS) - r8_toff(kb_lo, NS));
  const int64_t p = (int64_t)blockIdx.x * R8_PP + 16 * w + c;
  const bool valid = p < np;
  // w = a o b (screen codes 0 / 1 / 2): chunk kc holds individuals 64 kc + 16 g .. + 15 of pair c
  v4i wf[R8_NC];
  {
    const int8_t *ra = sl + (valid ? pi[p] : 0) * n_pad, *rb = sr + (valid ? pj[p] : 0) * n_pad;
#pragma unroll
    for (int kc = 0; kc < R8_NC; ++kc) {
      v4i v = {0, 0, 0, 0};
      if (valid && kc < NS) {
        const v4i va = *(const v4i *)(ra + 64 * kc + 16 * g), vb = *(const v4i *)(rb + 64 * kc + 16 * g);
#pragma unroll
        for (int d = 0; d < 4; ++d)
          v[d] = (int)__builtin_amdgcn_perm(T_HI, T_LO, to_offset((unsigned)va[d]) + (unsigned)vb[d]);
      }
      wf[kc] = v;
    }
  }
  // tile ring: visit v reads slot v % NSL; tile v + LA goes out at visit v into the slot of visit v - 1.
  // Past the last tile the DMAs repeat tile 0 into slots no visit reads again, so that every visit
  // waits with the same vmcnt (one static wait: the unrolled loop stays small enough to unroll fully)
  const bool two = w + 8 < R8_TILE / 1024;  // this wave moves two 1-KB pieces per tile, else one
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&sA[0][0]) + w * 1024;
  int kb_p = kb_lo, cs_p = NS - 1, issued = 0;
  auto issue_next = [&]() __attribute__((always_inline)) {
    const int8_t *src = issued < N ? tiles + (r8_toff(kb_p, NS) + cs_p - kb_p / 2) * R8_TILE : tiles;
    const unsigned dst = ring_m0 + (unsigned)(issued % NSL) * R8_TILE;
    lds_dma16_m0(src + (w * 64 + lane) * 16, dst);
    if (two) lds_dma16_m0(src + ((w + 8) * 64 + lane) * 16, dst + 8 * 1024);
    if (issued < N && --cs_p < kb_p / 2) {
      ++kb_p;
      cs_p = NS - 1;
    }
    ++issued;
  };
  for (int q = 0; q < LA; ++q) issue_next();
  const v4i zv = {0, 0, 0, 0};
  v4i acc[R8_S][2];
  double T[R8_S];
#pragma unroll
  for (int s = 0; s < R8_S; ++s) T[s] = 0.0;
  const int swz = 16 * (g ^ r8_swz(c));
  int v = 0;
  for (int kb = kb_lo; kb < kb_hi; ++kb) {
    const int c0 = kb >> 1;
#pragma unroll
    for (int cs = R8_NC - 1; cs >= 0; --cs) {
      int cq = c0;  // opaque per unrolled copy (see pair_mxr_kernel)
      asm volatile("" : "+s"(cq));
      if (cs < NS && cs >= cq) {
        // tile v has landed (the LA - 1 younger tiles may be in flight)
        static_assert(LA == 6, "vmcnt values");
        if (two)
          asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        issue_next();
        const int8_t *tb = sA[v % NSL];
        const bool first = cs == NS - 1;
#pragma unroll
        for (int s = 0; s < R8_S; ++s)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const v4i fa = *(const v4i *)(tb + s * R8_TB + (rt * 16 + c) * 64 + swz);
            acc[s][rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, wf[cs], first ? zv : acc[s][rt], 0, 0, 0);
          }
        if (cs == cq) {  // rows of block kb done: fold with w at the lane's rows 4 g .. 4 g + 3 of each row tile
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const int sl_ = c + 16 * (2 * (kb & 1) + rt);  // the lanes holding the row tile's w
            const v4i src = wf[cs];
            const int d0 = __shfl(src[0], sl_), d1 = __shfl(src[1], sl_), d2 = __shfl(src[2], sl_),
                      d3 = __shfl(src[3], sl_);
            const unsigned wd = (unsigned)(g == 0 ? d0 : g == 1 ? d1 : g == 2 ? d2 : d3);
            const int w0 = (int)(wd & 0xff), w1 = (int)((wd >> 8) & 0xff), w2 = (int)((wd >> 16) & 0xff),
                      w3 = (int)(wd >> 24);
#pragma unroll
            for (int s = 0; s < R8_S; ++s)
              T[s] += (double)(w0 * acc[s][rt][0] + w1 * acc[s][rt][1] + w2 * acc[s][rt][2] + w3 * acc[s][rt][3]);
          }
        }
        ++v;
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs land before the workgroup ends
#pragma unroll
  for (int s = 0; s < R8_S; ++s) {
    T[s] += __shfl_xor(T[s], 16);
    T[s] += __shfl_xor(T[s], 32);
  }
  if (g || !valid) return;
  if (nseg > 1) {
#pragma unroll
    for (int s = 0; s < R8_S; ++s) tpart[((int64_t)seg * R8_S + s) * np + p] = T[s];
    return;
  }
  double sum = 0.0;
#pragma unroll
  for (int s = R8_S - 1; s >= 0; --s) sum = sum * (1.0 / 128.0) + T[s];
  varw[p] = unit * sum;
}
// refine8_kernel for n_pad > 64 R8_NC (configs[4]: 80 stages), where one wave cannot hold every chunk of
// its pairs' w: the (row block, column stage) tiles are cut into squares of R8_NC column stages by the
// 2 R8_NC row blocks beside them, one per segment (gridDim.y: square (qi, qj), qi <= qj, row-major), a
// wave holds w of its square's column stages only, and a row block's accumulators are folded at the end
// of its row of the square with w of the block's rows formed from the screen codes in memory.  The
// per-slice sums are integers, so the segments add up (refine8_side_kernel) to the unsegmented bits.
__global__ __launch_bounds__(512, 1) void refine8w_kernel(int64_t n_pad, const int8_t *__restrict__ tiles,
                                                          const int8_t *__restrict__ sl, const int8_t *__restrict__ sr,
                                                          const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                          int64_t np, double *__restrict__ tpart) {
  constexpr int NSL = 8, LA = 6;
  __shared__ __attribute__((aligned(16))) int8_t sA[NSL][R8_TILE];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 15, g = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int NB = (int)(n_pad / 32), NS = (int)(n_pad / 64), nQ = (NS + R8_NC - 1) / R8_NC;
  int sq = (int)blockIdx.y, qi = 0;
  while (sq >= nQ - qi) {
    sq -= nQ - qi;
    ++qi;
  }
  const int qj = qi + sq;
  const int K0 = 2 * R8_NC * qi, K1 = min(NB, K0 + 2 * R8_NC), C0 = R8_NC * qj, C1 = min(NS, C0 + R8_NC);
  int N = 0;
  for (int kb = K0; kb < K1; ++kb) N += max(0, C1 - max(C0, kb >> 1));
  const int64_t p = (int64_t)blockIdx.x * R8_PP + 16 * w + c;
  const bool valid = p < np;
  const int8_t *ra = sl + (valid ? pi[p] : 0) * n_pad, *rb = sr + (valid ? pj[p] : 0) * n_pad;
  v4i wf[R8_NC];  // chunk kc: individuals 64 (C0 + kc) + 16 g .. + 15 of pair c
#pragma unroll
  for (int kc = 0; kc < R8_NC; ++kc) {
    v4i v = {0, 0, 0, 0};
    if (valid && C0 + kc < C1) {
      const v4i va = *(const v4i *)(ra + 64 * (C0 + kc) + 16 * g), vb = *(const v4i *)(rb + 64 * (C0 + kc) + 16 * g);
#pragma unroll
      for (int d = 0; d < 4; ++d) v[d] = (int)__builtin_amdgcn_perm(T_HI, T_LO, to_offset((unsigned)va[d]) + (unsigned)vb[d]);
    }
    wf[kc] = v;
  }
  const bool two = w + 8 < R8_TILE / 1024;
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&sA[0][0]) + w * 1024;
  int kb_p = K0, cs_p = C1 - 1, issued = 0;
  while (kb_p < K1 && C1 - 1 < max(C0, kb_p >> 1)) ++kb_p;  // row blocks of the square without a tile
  auto issue_next = [&]() __attribute__((always_inline)) {
    const int8_t *src = issued < N ? tiles + (r8_toff(kb_p, NS) + cs_p - kb_p / 2) * R8_TILE : tiles;
    const unsigned dst = ring_m0 + (unsigned)(issued % NSL) * R8_TILE;
    lds_dma16_m0(src + (w * 64 + lane) * 16, dst);
    if (two) lds_dma16_m0(src + ((w + 8) * 64 + lane) * 16, dst + 8 * 1024);
    if (issued < N && --cs_p < max(C0, kb_p >> 1)) {
      ++kb_p;
      cs_p = C1 - 1;
    }
    ++issued;
  };
  for (int q = 0; q < LA; ++q) issue_next();
  const v4i zv = {0, 0, 0, 0};
  v4i acc[R8_S][2];
  double T[R8_S];
#pragma unroll
  for (int s2 = 0; s2 < R8_S; ++s2) T[s2] = 0.0;
  const int swz = 16 * (g ^ r8_swz(c));
  int v = 0;
  for (int kb = K0; kb < K1; ++kb) {
    int lo = max(C0, kb >> 1);
    asm volatile("" : "+s"(lo));  // opaque per unrolled copy (see pair_mxr_kernel)
    if (lo > C1 - 1) continue;
#pragma unroll
    for (int kc = R8_NC - 1; kc >= 0; --kc) {
      if (C0 + kc < C1 && C0 + kc >= lo) {
        static_assert(LA == 6, "vmcnt values");
        if (two)
          asm volatile("s_waitcnt vmcnt(10) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(5) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        issue_next();
        const int8_t *tb = sA[v % NSL];
        const bool first = C0 + kc == C1 - 1;
#pragma unroll
        for (int s2 = 0; s2 < R8_S; ++s2)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const v4i fa = *(const v4i *)(tb + s2 * R8_TB + (rt * 16 + c) * 64 + swz);
            acc[s2][rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, wf[kc], first ? zv : acc[s2][rt], 0, 0, 0);
          }
        ++v;
      }
    }
    // the row block's rows 4 g .. 4 g + 3 of each row tile: w from the screen codes
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      unsigned wd = 0u;
      if (valid) {
        const int64_t q0 = 32 * (int64_t)kb + 16 * rt + 4 * g;
        wd = __builtin_amdgcn_perm(T_HI, T_LO, to_offset(*(const unsigned *)(ra + q0)) + *(const unsigned *)(rb + q0));
      }
      const int w0 = (int)(wd & 0xff), w1 = (int)((wd >> 8) & 0xff), w2 = (int)((wd >> 16) & 0xff), w3 = (int)(wd >> 24);
#pragma unroll
      for (int s2 = 0; s2 < R8_S; ++s2)
        T[s2] += (double)(w0 * acc[s2][rt][0] + w1 * acc[s2][rt][1] + w2 * acc[s2][rt][2] + w3 * acc[s2][rt][3]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int s2 = 0; s2 < R8_S; ++s2) {
    T[s2] += __shfl_xor(T[s2], 16);
    T[s2] += __shfl_xor(T[s2], 32);
  }
  if (g || !valid) return;
#pragma unroll
  for (int s2 = 0; s2 < R8_S; ++s2) tpart[((int64_t)blockIdx.y * R8_S + s2) * np + p] = T[s2];
}
// the most row-block segments a short refine8 / pair_mxr list is split into (GMAT_SEG_MAX, default 8)
int seg_max() {
  const char *s = getenv("GMAT_SEG_MAX");
  return s ? std::max(1, std::min(16, atoi(s))) : 8;
}

// The O(n) terms of e'Pe in fp64 (refine8_kernel's expansion) and eff = e'Py from the reference
// codes; one wave per pair, lanes over individuals, lane partials added in a fixed tree.
__global__ __launch_bounds__(256) void refine8_side_kernel(int64_t n_pad, const int8_t *__restrict__ sl,
                                                           const int8_t *__restrict__ sr, const double *__restrict__ Ua,
                                                           const double *__restrict__ Ub, const double *__restrict__ z,
                                                           const double *__restrict__ dg, const double *__restrict__ py,
                                                           const int8_t *__restrict__ lp, const int8_t *__restrict__ rp,
                                                           const double *soff_l, const double *soff_r, const double *off_l,
                                                           const double *off_r, const double *qa, const double *ra,
                                                           const double *qb, const double *rb, double zz,
                                                           const uint8_t *mono_l, const uint8_t *mono_r,
                                                           const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                           int64_t np, const double *varw, int nseg, const double *tpart,
                                                           double unit, double *eff, double *var, double *chi,
                                                           double *pv) {
  const int lane = threadIdx.x & 63;
  const int64_t p = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= np) return;
  const int64_t i = pi[p], j = pj[p];
  const double al = soff_l[i], be = soff_r[j], ab = al * be, ral = off_l[i], rbe = off_r[j];
  const int8_t *a = sl + i * n_pad, *b = sr + j * n_pad, *la = lp + i * n_pad, *lb = rp + j * n_pad;
  const double *ua = Ua + i * n_pad, *ub = Ub + j * n_pad;
  double s1 = 0.0, s2 = 0.0, s3 = 0.0, ef = 0.0;
  for (int64_t q = lane; q < n_pad; q += 64) {
    const double av = (double)a[q], bv = (double)b[q], wv = av * bv;
    s1 += wv * ((ab * z[q] - be * ua[q]) - al * ub[q]);
    s2 += av * ub[q];
    s3 += dg[q] * (wv * wv);
    ef += (((double)la[q] - ral) * ((double)lb[q] - rbe)) * py[q];
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    s3 += __shfl_xor(s3, off);
    ef += __shfl_xor(ef, off);
  }
  if (lane) return;
  const double t3 = be * be * qa[i], t5 = al * al * qb[j], t7 = ab * ab * zz, t8 = 2.0 * ab * s2, t4 = -2.0 * ab * be * ra[i],
               t6 = -2.0 * ab * al * rb[j];
  // w'P_off w: refine8_kernel's value, or its segments' integer sums added exactly in fp64 (integers
  // < 2^53) and combined in the single-segment order: the same bits for any number of segments
  double vw;
  if (nseg > 1) {
    double sum = 0.0;
    for (int s = R8_S - 1; s >= 0; --s) {
      double t = 0.0;
      for (int k = 0; k < nseg; ++k) t += tpart[((int64_t)k * R8_S + s) * np + p];
      sum = sum * (1.0 / 128.0) + t;
    }
    vw = unit * sum;
  } else {
    vw = varw[p];
  }
  // x == 0 (monomorphic): e = 0 exactly, var = 0 as the reference computes it (its chi and p are NaN)
  const double v = (mono_l[i] || mono_r[j]) ? 0.0 : vw + s3 + 2.0 * s1 + t3 + t5 + t7 + t8 + t4 + t6;
  var[p] = v;
  eff[p] = ef;
  // chi and p as pvalue_kernel
  const double cc = ef * ef / v;
  chi[p] = cc;
  pv[p] = (cc < 0.0) ? 1.0 : erfc(sqrt(0.5 * cc));
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
// the screens), and eff = e'Py; pair_mx_kernel evaluates w'P_off w on the MX screen's fp6 tile
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
__global__ __launch_bounds__(256) void pair_side_kernel(PairArgs x) {
  extern __shared__ __attribute__((aligned(16))) float zdp[];  // [3][n_pad]: z, diag(P), Py
  const int64_t n_pad = x.n_pad;
  for (int64_t q = threadIdx.x; q < n_pad; q += blockDim.x) {
    zdp[q] = (float)x.z[q];
    zdp[n_pad + q] = (float)x.dg[q];
    zdp[2 * n_pad + q] = (float)x.py[q];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int k = 0; k < PS_PPW; ++k) {
    const int64_t p = ((int64_t)blockIdx.x * 4 + wv) * PS_PPW + k;
    if (p >= x.np) return;
    const int64_t i = x.ci[p], j = x.cj[p];
    const double dal = x.alpha[i], dbe = x.beta[j], dab = dal * dbe;
    const float al = (float)dal, be = (float)dbe, ab = (float)dab;
    const int8_t *pa = x.a + i * n_pad, *pb = x.b + j * n_pad;
    const _Float16 *ua = x.Ua + i * n_pad, *ub = x.Ub + j * n_pad;
    float s1 = 0, s1a = 0, s2 = 0, s2a = 0, s3 = 0, s3a = 0, ef = 0, efa = 0, sw = 0;
    // (the codes at 2 bits instead of int8, a quarter of the code bytes, measured the same: 18.3 ms per
    // configs[2] step either way; the gathers are latency-bound)
    for (int64_t q0 = 8 * lane; q0 < n_pad; q0 += 512) {
      const v2i_ va = *(const v2i_ *)(pa + q0), vb = *(const v2i_ *)(pb + q0);
      const int8_t *ca = (const int8_t *)&va, *cb = (const int8_t *)&vb;
      typedef _Float16 h8_ __attribute__((ext_vector_type(8)));
      const h8_ u8 = *(const h8_ *)(ua + q0), v8 = *(const h8_ *)(ub + q0);
      float uu[8], vv[8];
#pragma unroll
      for (int t = 0; t < 8; ++t) {
        uu[t] = (float)u8[t];
        vv[t] = (float)v8[t];
      }
      // z, diag(P), Py of the lane's 8 individuals as 16-byte LDS reads (a lane's 32 bytes: 8 scalar reads at
      // a 32-byte lane stride were 8-way bank conflicts).  Lanes with bit 3 set read their second half
      // first: each 16-lane group of a ds_read_b128 then covers all 64 banks (in one order the groups'
      // lanes l and l + 8 or l + 24 met on a bank, 2-way: ~40 % of the kernel's cycles by SQ_LDS_BANK_CONFLICT)
      float zz8[8], dd8[8], yy8[8];
      {
        const int o1 = (lane & 8) ? 4 : 0, o2 = 4 - o1;
        const bool sw = lane & 8;
        auto rd2 = [&](const float *base, float *dst) __attribute__((always_inline)) {
          const float4 f1 = *(const float4 *)&base[q0 + o1];
          const float4 f2 = *(const float4 *)&base[q0 + o2];
          *(float4 *)&dst[0] = sw ? f2 : f1;
          *(float4 *)&dst[4] = sw ? f1 : f2;
        };
        rd2(zdp, zz8);
        rd2(zdp + n_pad, dd8);
        rd2(zdp + 2 * n_pad, yy8);
      }
#pragma unroll
      for (int h = 0; h < 8; ++h) {
        const float av = (float)ca[h], bv = (float)cb[h], w = av * bv;  // exact small integers
        const float z = zz8[h], d = dd8[h], y = yy8[h];
        const float tu = be * uu[h], tv = al * vv[h], tz = ab * z;
        s1 += w * ((tz - tu) - tv);
        s1a += w * ((fabsf(tu) + fabsf(tv)) + fabsf(tz));
        s2 += av * vv[h];
        s2a += av * fabsf(vv[h]);
        s3 += d * (w * w);
        s3a += fabsf(d) * (w * w);
        const float ey = ((av - al) * (bv - be)) * y;
        ef += ey;
        efa += fabsf(ey);
        sw += w * w;
      }
    }
    double r[9] = {s1, s1a, s2, s2a, s3, s3a, ef, efa, sw};
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) r[t] += __shfl_xor(r[t], off);
    if (lane != 0) continue;
    const double t3 = dbe * dbe * x.qa[i], t5 = dal * dal * x.qb[j], t7 = dab * dab * x.zz, t8 = 2.0 * dab * r[2],
                 t4 = -2.0 * dab * dbe * x.ra[i], t6 = -2.0 * dab * dal * x.rb[j];
    x.side[p] = r[4] + 2.0 * r[0] + t3 + t5 + t7 + t8 + t4 + t6;
    // fp32 sums: a lane adds n_pad / 64 terms of at most 4 roundings each, so a sum is within
    // (n_pad / 64 + 4) 2^-24 of its absolute sum (the lane reduction is fp64); fsl doubles that.  U is
    // stored in fp16: a normal value is within 2^-11 of U, relative, so the U terms (su, their magnitudes
    // from the rounded values) are within 2^-10.9 su; a subnormal one within 2^-25 absolute, at most
    // 2^-25 (|alpha| + |beta|) 4 n_pad in total (an overflow gives inf / NaN: the pair is kept).  Plus
    // the fp64 rounding of U = P x codes and of the host terms (far inside 1e-10 of the magnitudes).
    // side[3 np + p] is the eff bound's slack.
    const double fsl = 2.0 * (double)(n_pad / 64 + 8) * 0x1p-24;
    const double su = 2.0 * r[1] + 2.0 * fabs(dab) * r[3];
    x.side[x.np + p] = fsl * (su + r[5]) + 0x1p-10 * su + 0x1p-23 * (fabs(dal) + fabs(dbe)) * 4.0 * (double)n_pad +
                       1e-10 * (r[5] + su + fabs(t3) + fabs(t5) + fabs(t7) + fabs(t4) + fabs(t6));
    x.side[2 * x.np + p] = r[6];
    x.side[3 * x.np + p] = (fsl + 1e-10) * r[7];
    x.side[4 * x.np + p] = r[8];
  }
}

// PP pairs per workgroup (PP / 32 column tiles x four 32-row tiles, one wave each); the pairs' w
// codes for all individuals stay in LDS (pitch nK * 64 + 16 bytes: conflict-free fragment reads),
// the tile images stream through a double buffer in the block-upper stage order of mx_screen.
template <int PP>
__global__ __launch_bounds__(PP * 8) void pair_mx_kernel(PairArgs x) {
  constexpr int T = PP * 8, NC16 = MX_TILE / 16, NA = (NC16 + T - 1) / T;  // 16-byte chunks per tile
  extern __shared__ __attribute__((aligned(16))) uint8_t dyn[];
  uint8_t *sA = dyn;                        // [2][MX_TILE]
  uint8_t *wpl = dyn + 2 * MX_TILE;         // [PP][pitch]
  const int nK = x.nK, pitch = nK * 64 + 16;
  double *red = (double *)(wpl + PP * pitch);  // [4][PP]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5, c = lane & 31;
  const int r = w & 3, t = w >> 2;
  const int64_t p0 = (int64_t)blockIdx.x * PP;
  // w planes: w = (M1 & S1) | (M2 & 2 S1) per 16-byte chunk (the MX screen's fp4 codes of w / 2)
  for (int k = tid; k < PP * nK * 4; k += T) {
    const int pl = k / (nK * 4), s = (k >> 2) % nK, q = k & 3;
    const int64_t gp = p0 + pl;
    v4i wv = {0, 0, 0, 0};
    if (gp < x.np) {
      const uint8_t *ri = x.nib_i + (x.ci[gp] * nK + s) * NB_REC + 16 * q;
      const v4i m1 = *(const v4i *)ri, m2 = *(const v4i *)(ri + 64);
      const v4i s1 = *(const v4i *)(x.nib_j + (x.cj[gp] * nK + s) * NB_REC + 16 * q);
      wv = (m1 & s1) | (m2 & (s1 << 1));
    }
    *(v4i *)&wpl[pl * pitch + s * 64 + 16 * q] = wv;
  }
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(x.tiles, x.tiles_bytes);
  v4i ra[NA];
  auto load = [&](int kb, int cs) __attribute__((always_inline)) {
    const int soffA = (kb * nK + cs) * MX_TILE;
#pragma unroll
    for (int u = 0; u < NA; ++u)
      if (NC16 % T == 0 || tid + u * T < NC16) ra[u] = __builtin_amdgcn_raw_buffer_load_b128(rsA, (tid + u * T) * 16, soffA, 0);
  };
  auto store = [&](int b) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < NA; ++u)
      if (NC16 % T == 0 || tid + u * T < NC16) *(v4i *)&sA[b * MX_TILE + (tid + u * T) * 16] = ra[u];
  };
  const uint8_t *wrow = wpl + (32 * t + c) * pitch;
  const int sw16 = 16 * ((c >> 3) & 1);
  v16f_ acc;
  auto compute = [&](int b, int cs, bool diag) __attribute__((always_inline)) {
    const int bscale = diag ? 128 : 129;
    const v16f_ zv = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i wb = *(const v4i *)(wrow + cs * 64 + 16 * (2 * kk + h));
      const v8i_ fb = {wb[0], wb[1], wb[2], wb[3], 0, 0, 0, 0};
      const uint8_t *ar = &sA[b * MX_TILE + (2 * kk + h) * 4096 + (32 * r + c) * 32];
      const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
      const v8i_ fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      acc = mfma_mx(fa, fb, (diag && kk == 0) ? zv : acc, hi[2], bscale);
    }
  };
  double tot = 0.0;
  load(0, 0);
  store(0);
  __syncthreads();
  int b = 0;
  for (int kb = 0; kb < nK; ++kb) {
#pragma unroll 1
    for (int cs = kb; cs < nK; ++cs) {
      const bool more = cs + 1 < nK || kb + 1 < nK;
      if (more) load(cs + 1 < nK ? kb : kb + 1, cs + 1 < nK ? cs + 1 : kb + 1);
      __builtin_amdgcn_sched_barrier(0);
      compute(b, cs, cs == kb);
      if (more) store(b ^ 1);
      __syncthreads();
      b ^= 1;
    }
    // sum_rows w[row] acc[row]: register e of this lane <-> storage slot 16h + e of row tile r
    const v2i_ m = *(const v2i_ *)(wrow + kb * 64 + 16 * r + 8 * h);
    v2f_ s2 = {0.f, 0.f};
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const unsigned wd = (unsigned)m[d];
#pragma unroll
      for (int bb = 0; bb < 4; ++bb) {
        const v2f_ wf = bb == 0 ? fp4_pair<0>(wd) : bb == 1 ? fp4_pair<1>(wd) : bb == 2 ? fp4_pair<2>(wd) : fp4_pair<3>(wd);
        const v2f_ av = {acc[8 * d + 2 * bb], acc[8 * d + 2 * bb + 1]};
        s2 = __builtin_elementwise_fma(wf, av, s2);
      }
    }
    tot += (double)s2[0] + (double)s2[1];
  }
  tot += __shfl_xor(tot, 32);
  if (h == 0) red[r * PP + 32 * t + c] = tot;
  __syncthreads();
  if (tid >= PP) return;
  const int64_t p = p0 + tid;
  if (p >= x.np) return;
  pair_test(x, p, (red[tid] + red[PP + tid]) + (red[2 * PP + tid] + red[3 * PP + tid]));
}

// The same quadratic form with each pair's w held in REGISTERS (n_pad <= 128 PXR_NK): a wave owns 32
// pairs, lane (c, h) holds pair c's fp4 w for 32 individuals of every 64-individual chunk (the MFMA
// B fragments, 4 registers per chunk), so 8 waves carry 256 pairs and the P tile images stream
// through LDS once per 256 pairs (pair_mx_kernel: once per 96, from its LDS-resident w planes) in an
// eight-slot LDS-DMA ring, six tiles in flight (the tiles compete for L2 with the pairs' record
// gathers).  Visit order: row block kb, then column stage cs from
// the last down to kb (the inner loop is unrolled so that every register index is static; its last
// visit, the diagonal tile, folds the row block's accumulators with w of block kb, fetched from the
// lane half that holds them).  Same operands, scales and test as pair_mx_kernel.
constexpr int PXR_NK = 16, PXR_NSL = 8;  // w chunks in registers (n_pad <= 2048); LDS ring slots
__global__ __launch_bounds__(512, 1) void pair_mxr_kernel(PairArgs x) {
  constexpr int NSL = PXR_NSL, LA = PXR_NSL - 2;
  __shared__ __attribute__((aligned(16))) uint8_t sA[NSL][MX_TILE];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nK = x.nK;
  // segment blockIdx.y of gridDim.y: the row blocks [kb_lo, kb_hi) holding its share of the tiles (a
  // short candidate list is spread over more workgroups); partial sums to x.mpart (pair_test_kernel)
  const int nseg = (int)gridDim.y, seg = (int)blockIdx.y, N_all = nK * (nK + 1) / 2;
  auto toff = [&](int kb) __attribute__((always_inline)) { return kb * nK - kb * (kb - 1) / 2; };
  int kb_lo = 0;
  while (kb_lo < nK && toff(kb_lo) * nseg < N_all * seg) ++kb_lo;
  int kb_hi = kb_lo;
  while (kb_hi < nK && toff(kb_hi) * nseg < N_all * (seg + 1)) ++kb_hi;
  const int N = toff(kb_hi) - toff(kb_lo);
  const int64_t p = (int64_t)blockIdx.x * 256 + 32 * w + c;
  const bool valid = p < x.np;
  v4i wf[2 * PXR_NK];
  {
    const uint8_t *ri = x.nib_i + (valid ? x.ci[p] : 0) * nK * NB_REC, *rj = x.nib_j + (valid ? x.cj[p] : 0) * nK * NB_REC;
#pragma unroll
    for (int g = 0; g < 2 * PXR_NK; ++g) {
      v4i v = {0, 0, 0, 0};
      if (valid && g < 2 * nK) {  // chunk g = stage g / 2, 16-byte piece 2 (g % 2) + h of its planes
        const int s = g >> 1, q = 2 * (g & 1) + h;
        const v4i m1 = *(const v4i *)(ri + s * NB_REC + 16 * q), m2 = *(const v4i *)(ri + s * NB_REC + 64 + 16 * q);
        const v4i s1 = *(const v4i *)(rj + s * NB_REC + 16 * q);
        v = (m1 & s1) | (m2 & (s1 << 1));
      }
      wf[g] = v;
    }
  }
  // tile ring: visit v reads slot v % NSL; the DMA of tile v + LA goes out at visit v into the slot
  // visit v - 1 read (every wave has passed visit v's barrier)
  int kb_p = kb_lo, cs_p = nK - 1, issued = 0;
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (issued < N) {
      const uint8_t *src = x.tiles + (int64_t)(kb_p * nK + cs_p) * MX_TILE;
      uint8_t *dst = sA[issued % NSL];
      lds_dma16(src + (w * 64 + lane) * 16, dst + w * 1024);
      lds_dma16(src + ((8 + w) * 64 + lane) * 16, dst + (8 + w) * 1024);
      if (--cs_p < kb_p) {
        ++kb_p;
        cs_p = nK - 1;
      }
    }
    ++issued;
  };
  for (int q = 0; q < LA; ++q) issue_next();
  const int sw16 = 16 * ((c >> 3) & 1);
  const v16f_ zv = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  v16f_ acc[MX_RB];
  double tot = 0.0;
  int v = 0;
  for (int kb = kb_lo; kb < kb_hi; ++kb) {
#pragma unroll
    for (int cs = PXR_NK - 1; cs >= 0; --cs) {
      // an opaque copy of kb per unrolled copy: with kb itself the compiler turns the copies' kb == cs
      // tests into one switch and merges the fold copies into one block that indexes wf dynamically
      // (through scratch)
      int kq = kb;
      asm volatile("" : "+s"(kq));
      if (cs < nK && cs >= kq) {
        vm_wait_barrier(2 * min(LA - 1, N - 1 - v));  // tile v has landed (younger DMAs may be in flight)
        issue_next();
        const uint8_t *tb = sA[v % NSL];
        const int bs = cs == kb ? 128 : 129;  // off-diagonal tiles count twice
        const bool first = cs == nK - 1;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const v4i wb = wf[2 * cs + kk];
          const v8i_ fb = {wb[0], wb[1], wb[2], wb[3], 0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < MX_RB; ++r) {
            const uint8_t *ar = tb + (2 * kk + h) * 4096 + (32 * r + c) * 32;
            const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
            const v8i_ fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            acc[r] = mfma_mx(fa, fb, (first && kk == 0) ? zv : acc[r], hi[2], bs);
          }
        }
        if (cs == kq) {  // row block kb complete: sum_rows w[row] acc[row] (register e <-> slot 16 h + e)
#pragma unroll
          for (int r = 0; r < MX_RB; ++r) {
            const v4i src = wf[2 * cs + (r >> 1)];  // row tile r: lanes of half r & 1 hold its 32 slots
            const int sl = c + 32 * (r & 1);
            const int a0 = __shfl(src[0], sl), a1 = __shfl(src[1], sl), a2 = __shfl(src[2], sl),
                      a3 = __shfl(src[3], sl);
            const unsigned m[2] = {(unsigned)(h ? a2 : a0), (unsigned)(h ? a3 : a1)};
            v2f_ s2 = {0.f, 0.f};
#pragma unroll
            for (int d = 0; d < 2; ++d) {
#pragma unroll
              for (int bb = 0; bb < 4; ++bb) {
                const v2f_ wv = bb == 0 ? fp4_pair<0>(m[d]) : bb == 1 ? fp4_pair<1>(m[d]) : bb == 2 ? fp4_pair<2>(m[d]) : fp4_pair<3>(m[d]);
                const v2f_ av = {acc[r][8 * d + 2 * bb], acc[r][8 * d + 2 * bb + 1]};
                s2 = __builtin_elementwise_fma(wv, av, s2);
              }
            }
            tot += (double)s2[0] + (double)s2[1];
          }
        }
        ++v;
      }
    }
  }
  tot += __shfl_xor(tot, 32);
  if (h || !valid) return;
  if (nseg > 1)
    x.mpart[(int64_t)seg * x.np + p] = tot;
  else
    pair_test(x, p, tot);
}
// pair_mxr_kernel for n_pad > 64 PXR_NK (configs[4]: 40 stages), where one wave cannot hold every
// stage of its pairs' w: the triangle of (row block, column stage) tiles is cut into squares of
// PXR_NK x PXR_NK stages, one per segment (gridDim.y: square (qi, qj), qi <= qj, row-major), so a wave
// holds the w of its square's PXR_NK column stages only; a row block's accumulators are folded at the
// end of its row of the square with w of that block read from the nibble records (L2).  Per (square,
// pair) partial sums go to mpart (pair_test_kernel adds them).  The LDS-resident pair_mx_kernel it
// replaces at these sizes holds 32 pairs per workgroup and streamed the whole tile set per 32 pairs.
__global__ __launch_bounds__(512, 1) void pair_mxw_kernel(PairArgs x) {
  constexpr int NSL = PXR_NSL, LA = PXR_NSL - 2;
  __shared__ __attribute__((aligned(16))) uint8_t sA[NSL][MX_TILE];
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nK = x.nK, nQ = (nK + PXR_NK - 1) / PXR_NK;
  int sq = (int)blockIdx.y, qi = 0;
  while (sq >= nQ - qi) {
    sq -= nQ - qi;
    ++qi;
  }
  const int qj = qi + sq;
  const int K0 = qi * PXR_NK, K1 = min(nK, K0 + PXR_NK), C0 = qj * PXR_NK, C1 = min(nK, C0 + PXR_NK);
  int N = 0;
  for (int kb = K0; kb < K1; ++kb) N += C1 - max(C0, kb);
  const int64_t p = (int64_t)blockIdx.x * 256 + 32 * w + c;
  const bool valid = p < x.np;
  const uint8_t *ri = x.nib_i + (valid ? x.ci[p] : 0) * nK * NB_REC, *rj = x.nib_j + (valid ? x.cj[p] : 0) * nK * NB_REC;
  v4i wf[2 * PXR_NK];  // chunk g: column stage C0 + g / 2, 16-byte piece 2 (g % 2) + h
#pragma unroll
  for (int g = 0; g < 2 * PXR_NK; ++g) {
    v4i v = {0, 0, 0, 0};
    if (valid && C0 + (g >> 1) < C1) {
      const int s = C0 + (g >> 1), q = 2 * (g & 1) + h;
      const v4i m1 = *(const v4i *)(ri + s * NB_REC + 16 * q), m2 = *(const v4i *)(ri + s * NB_REC + 64 + 16 * q);
      const v4i s1 = *(const v4i *)(rj + s * NB_REC + 16 * q);
      v = (m1 & s1) | (m2 & (s1 << 1));
    }
    wf[g] = v;
  }
  int kb_p = K0, cs_p = C1 - 1, issued = 0;
  auto issue_next = [&]() __attribute__((always_inline)) {
    if (issued < N) {
      const uint8_t *src = x.tiles + (int64_t)(kb_p * nK + cs_p) * MX_TILE;
      uint8_t *dst = sA[issued % NSL];
      lds_dma16(src + (w * 64 + lane) * 16, dst + w * 1024);
      lds_dma16(src + ((8 + w) * 64 + lane) * 16, dst + (8 + w) * 1024);
      if (--cs_p < max(C0, kb_p)) {
        ++kb_p;
        cs_p = C1 - 1;
      }
    }
    ++issued;
  };
  for (int q = 0; q < LA; ++q) issue_next();
  const int sw16 = 16 * ((c >> 3) & 1);
  const v16f_ zv = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  v16f_ acc[MX_RB];
  double tot = 0.0;
  int v = 0;
  for (int kb = K0; kb < K1; ++kb) {
    int lo = max(C0, kb);
    asm volatile("" : "+s"(lo));  // opaque per unrolled copy (see pair_mxr_kernel)
#pragma unroll
    for (int cl = PXR_NK - 1; cl >= 0; --cl) {
      if (C0 + cl < C1 && C0 + cl >= lo) {
        vm_wait_barrier(2 * min(LA - 1, N - 1 - v));  // tile v has landed (younger DMAs may be in flight)
        issue_next();
        const uint8_t *tb = sA[v % NSL];
        const int bs = C0 + cl == kb ? 128 : 129;  // off-diagonal tiles count twice
        const bool first = C0 + cl == C1 - 1;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const v4i wb = wf[2 * cl + kk];
          const v8i_ fb = {wb[0], wb[1], wb[2], wb[3], 0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < MX_RB; ++r) {
            const uint8_t *ar = tb + (2 * kk + h) * 4096 + (32 * r + c) * 32;
            const v4i lo4 = *(const v4i *)(ar + sw16), hi4 = *(const v4i *)(ar + (16 - sw16));
            const v8i_ fa = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            acc[r] = mfma_mx(fa, fb, (first && kk == 0) ? zv : acc[r], hi4[2], bs);
          }
        }
        ++v;
      }
    }
    // row block kb of the square done: sum_rows w[row] acc[row] with w of block kb (piece r = row tile
    // r; this lane half's slots 16 h .. 16 h + 15 are dwords 2 h, 2 h + 1 of the piece)
#pragma unroll
    for (int r = 0; r < MX_RB; ++r) {
      v4i wv = {0, 0, 0, 0};
      if (valid) {
        const v4i m1 = *(const v4i *)(ri + kb * NB_REC + 16 * r), m2 = *(const v4i *)(ri + kb * NB_REC + 64 + 16 * r);
        const v4i s1 = *(const v4i *)(rj + kb * NB_REC + 16 * r);
        wv = (m1 & s1) | (m2 & (s1 << 1));
      }
      const unsigned m[2] = {(unsigned)(h ? wv[2] : wv[0]), (unsigned)(h ? wv[3] : wv[1])};
      v2f_ s2 = {0.f, 0.f};
#pragma unroll
      for (int d = 0; d < 2; ++d) {
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) {
          const v2f_ wq = bb == 0 ? fp4_pair<0>(m[d]) : bb == 1 ? fp4_pair<1>(m[d]) : bb == 2 ? fp4_pair<2>(m[d]) : fp4_pair<3>(m[d]);
          const v2f_ av = {acc[r][8 * d + 2 * bb], acc[r][8 * d + 2 * bb + 1]};
          s2 = __builtin_elementwise_fma(wq, av, s2);
        }
      }
      tot += (double)s2[0] + (double)s2[1];
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs land before the workgroup ends
  tot += __shfl_xor(tot, 32);
  if (h || !valid) return;
  x.mpart[(int64_t)blockIdx.y * x.np + p] = tot;
}
__global__ void pair_test_kernel(PairArgs x, int nseg) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= x.np) return;
  double M = 0.0;
  for (int k = 0; k < nseg; ++k) M += x.mpart[(int64_t)k * x.np + p];
  pair_test(x, p, M);
}

// ------------------------------------------------------------------ setup kernels

// P_store[q][q'] = P[nat(q)][nat(q')], zero padded; z = P_store 1 computed later.
__global__ void permute_p_kernel(int64_t n, int64_t n_pad, const double *P, double *Ps) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t q = idx / n_pad, q2 = idx % n_pad;
  const int64_t r = (q & ~31LL) + perm_nat((int)(q & 31)), c = (q2 & ~31LL) + perm_nat((int)(q2 & 31));
  Ps[idx] = (r < n && c < n) ? P[r * n + c] : 0.0;
}
__global__ void permute_vec_kernel(int64_t n, int64_t n_pad, const double *v, double *vs) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n_pad) return;
  const int64_t r = (q & ~31LL) + perm_nat((int)(q & 31));
  vs[q] = (r < n) ? v[r] : 0.0;
}
// slices A_s[rho][t] (rho natural row, t storage column) of P_off*127/qmax (zero diagonal:
// the diagonal enters the screen exactly, as a side term)
__global__ void slice_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                             int8_t *slices) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t rho = idx / n_pad, t = idx % n_pad;
  const int64_t c = (t & ~31LL) + perm_nat((int)(t & 31));
  double r = (rho < n && c < n && rho != c) ? P[rho * n + c] * inv_unit : 0.0;
  for (int s = 0; s < n_slice; ++s) {
    const double q = rint(r);
    slices[(int64_t)s * n_pad * n_pad + idx] = (int8_t)q;
    r = (r - q) * 128.0;
  }
}

// residual of the slicing, R = P_off - P~ (natural order, zero padded and zero diagonal), scaled
__global__ void residual_kernel(int64_t n, int64_t n_pad, const double *P, double inv_unit, int n_slice,
                                double out_scale, double *R) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t r0 = idx / n_pad, c0 = idx % n_pad;
  double r = (r0 < n && c0 < n && r0 != c0) ? P[r0 * n + c0] * inv_unit : 0.0;
  for (int s = 0; s < n_slice; ++s) r = (r - rint(r)) * 128.0;
  R[idx] = r * out_scale;
}

// per-SNP side vectors for the left coding: L' = a o (u - alpha z), L3 = a o py,
// Ld = diag(P) o a o a, and scalars qa = a.u, ra = a.z, sa = a.py.  One workgroup per SNP.
__global__ __launch_bounds__(256) void left_side_kernel(int64_t n_pad, const int8_t *panel, const double *U,
                                                        const double *z, const double *py, const double *dg,
                                                        const double *alpha, double *Lp, double *L3, double *Ld,
                                                        double *qa, double *ra, double *sa) {
  const int64_t j = blockIdx.x;
  const double al = alpha[j];
  double s1 = 0, s2 = 0, s3 = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const double av = (double)panel[j * n_pad + q];
    const double u = U[j * n_pad + q];
    if (Lp) Lp[j * n_pad + q] = av * (u - al * z[q]);  // Lp, Ld: the block-granular screens only
    if (L3) L3[j * n_pad + q] = av * py[q];
    if (Ld) Ld[j * n_pad + q] = av * av * dg[q];
    s1 += av * u;
    s2 += av * z[q];
    s3 += av * py[q];
  }
  __shared__ double red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    s3 += __shfl_xor(s3, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
    red[2][threadIdx.x >> 6] = s3;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    qa[j] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    ra[j] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    sa[j] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
  }
}
// right coding: R' = (b - beta) o v, qb = b.v, rb = b.z, sb = b.py
__global__ __launch_bounds__(256) void right_side_kernel(int64_t n_pad, const int8_t *panel, const double *V,
                                                         const double *z, const double *py, const double *beta,
                                                         double *Rp, double *qb, double *rb, double *sb) {
  const int64_t j = blockIdx.x;
  const double be = beta[j];
  double s1 = 0, s2 = 0, s3 = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const double bv = (double)panel[j * n_pad + q];
    const double v = V[j * n_pad + q];
    if (Rp) Rp[j * n_pad + q] = (bv - be) * v;
    s1 += bv * v;
    s2 += bv * z[q];
    s3 += bv * py[q];
  }
  __shared__ double red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s1 += __shfl_xor(s1, off);
    s2 += __shfl_xor(s2, off);
    s3 += __shfl_xor(s3, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s1;
    red[1][threadIdx.x >> 6] = s2;
    red[2][threadIdx.x >> 6] = s3;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    qb[j] = ((red[0][0] + red[0][1]) + red[0][2]) + red[0][3];
    rb[j] = ((red[1][0] + red[1][1]) + red[1][2]) + red[1][3];
    sb[j] = ((red[2][0] + red[2][1]) + red[2][2]) + red[2][3];
  }
}

// Per-row int8 slices of an fp64 [rows][n_pad] matrix: v = s (sum_{t<T} 128^-t Q_t + r) with
// s = max|v|/127, |Q_0| <= 127, |Q_t| <= 64, |r| <= 0.5 * 128^-(T-1) (+ fp64 rounding).
__global__ __launch_bounds__(256) void quantize_rows_kernel(int64_t n_pad, int64_t slice_stride, const double *v,
                                                            int8_t *q, double *scale) {
  const int64_t j = blockIdx.x;
  const double *row = v + j * n_pad;
  double mx = 0.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) mx = fmax(mx, fabs(row[k]));
  for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
  const double s = mx / 127.0, inv = mx > 0.0 ? 127.0 / mx : 0.0;
  for (int64_t k = threadIdx.x; k < n_pad; k += 256) {
    double r = row[k] * inv;
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t) {
      const double qv = rint(r);
      q[t * slice_stride + j * n_pad + k] = (int8_t)qv;
      r = (r - qv) * 128.0;
    }
  }
  if (threadIdx.x == 0) scale[j] = s;
}

// gather band rows of the int8 side slices: BL[t][r] = Lq[t][rows[r]], BL[t][R+r] = L3q[t][rows[r]],
// BL[t][2R+r] = Ldq[t][rows[r]], BA[r] = panel[rows[r]], BA[R+r] = sqpanel[rows[r]] (squared codes)
__global__ void gather_band_kernel(int64_t n_pad, int R, int64_t slice_stride, const int64_t *rows, const int8_t *Lq,
                                   const int8_t *L3q, const int8_t *Ldq, const int8_t *panel, const int8_t *sqpanel,
                                   int8_t *BL, int8_t *BA) {
  const int r = blockIdx.x;
  const int64_t src = rows[r];
  for (int64_t q = threadIdx.x * 16; q < n_pad; q += blockDim.x * 16) {
#pragma unroll
    for (int t = 0; t < SIDE_T; ++t) {
      const int64_t o = (int64_t)t * SIDE_P * R + r, so = t * slice_stride + src * n_pad + q;
      *(v4i *)&BL[o * n_pad + q] = *(const v4i *)&Lq[so];
      *(v4i *)&BL[(o + R) * n_pad + q] = *(const v4i *)&L3q[so];
      *(v4i *)&BL[(o + 2 * R) * n_pad + q] = *(const v4i *)&Ldq[so];
    }
    *(v4i *)&BA[(int64_t)r * n_pad + q] = *(const v4i *)&panel[src * n_pad + q];
    *(v4i *)&BA[(int64_t)(R + r) * n_pad + q] = *(const v4i *)&sqpanel[src * n_pad + q];
  }
}

// C[z] (M x N int32, ldc) = A[z] (M x K int8, lda) . B[z]^T (N x K int8, ldb) for z = blockIdx.z;
// K a multiple of 64.  64 x 128 tile per workgroup, each wave 32 x 64 (two 32x32x32 i8 MFMAs
// per k-step), 64-deep LDS stages with the 80-byte pitch.  Exact int32 accumulation.
constexpr int GM = 64, GN = 128, GKK = 64, GPI = 80;
__global__ __launch_bounds__(256) void i8gemm_nt_kernel(int M, int N, int K, const int8_t *__restrict__ A, int64_t lda,
                                                        int64_t za, const int8_t *__restrict__ B, int64_t ldb,
                                                        int64_t zb, int *__restrict__ C, int64_t ldc, int64_t zc) {
  A += blockIdx.z * za;
  B += blockIdx.z * zb;
  C += blockIdx.z * zc;
  const int m0 = blockIdx.y * GM, n0 = blockIdx.x * GN;
  __shared__ __attribute__((aligned(16))) int8_t sa[GM * GPI];
  __shared__ __attribute__((aligned(16))) int8_t sb[GN * GPI];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, wr = w >> 1, wc = w & 1;
  v16i acc[2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[t][e] = 0;
  const int ar = tid >> 2, c16 = (tid & 3) * 16;
  const v4i zero = {0, 0, 0, 0};
  for (int k0 = 0; k0 < K; k0 += GKK) {
    *(v4i *)&sa[ar * GPI + c16] = (m0 + ar < M) ? *(const v4i *)&A[(int64_t)(m0 + ar) * lda + k0 + c16] : zero;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int br = ar + 64 * u;
      *(v4i *)&sb[br * GPI + c16] = (n0 + br < N) ? *(const v4i *)&B[(int64_t)(n0 + br) * ldb + k0 + c16] : zero;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i fa = *(const v4i *)&sa[(wr * 32 + (lane & 31)) * GPI + kk * 32 + (lane >> 5) * 16];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const v4i fb = *(const v4i *)&sb[(wc * 64 + t * 32 + (lane & 31)) * GPI + kk * 32 + (lane >> 5) * 16];
        acc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa, fb, acc[t], 0, 0, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int row = m0 + wr * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int col = n0 + wc * 64 + t * 32 + (lane & 31);
      if (row < M && col < N) C[(int64_t)row * ldc + col] = acc[t][e];
    }
}

int i8gemm_nt(hipStream_t st, int Z, int M, int N, int K, const int8_t *A, int64_t lda, int64_t za, const int8_t *B,
              int64_t ldb, int64_t zb, int *C, int64_t ldc, int64_t zc) {
  if (M <= 0 || N <= 0) return GMAT_OK;
  hipLaunchKernelGGL(i8gemm_nt_kernel, dim3((unsigned)cdiv(N, GN), (unsigned)cdiv(M, GM), (unsigned)Z), dim3(256), 0,
                     st, M, N, K, A, lda, za, B, ldb, zb, C, ldc, zc);
  GMAT_HIP(hipGetLastError());
  return GMAT_OK;
}

// screen panel of the additive coding: minor-allele dosage a~ = flip ? 2 - a : a (padding stays
// 0), and its square a~^2 in {0, 1, 4}
__global__ void flip_panel_kernel(int64_t n, int64_t n_pad, int64_t m, const int8_t *src, const uint8_t *flip,
                                  int8_t *dst, int8_t *sq) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * n_pad) return;
  const int64_t j = idx / n_pad, q = idx % n_pad;
  const int64_t nat = (q & ~31LL) + perm_nat((int)(q & 31));
  const int a = src[idx];
  const int v = (flip[j] && nat < n) ? 2 - a : a;
  dst[idx] = (int8_t)v;
  sq[idx] = (int8_t)(v * v);
}

__global__ void diag_kernel(int64_t n_pad, const double *Ps, double *dg) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n_pad) dg[q] = Ps[q * n_pad + q];
}

__global__ void zsum_kernel(int64_t n_pad, const double *Ps, double *z) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (q >= n_pad) return;
  double s = 0.0;
  for (int64_t k = lane; k < n_pad; k += 64) s += Ps[q * n_pad + k];
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) z[q] = s;
}

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
__global__ void mx_quant_kernel(int64_t n, int64_t n_pad, int nK, const double *P, uint32_t *tiles, double *Qn) {
  const int64_t nblk = n_pad / 32;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * nblk) return;
  const int64_t rho = idx / nblk, bI = idx % nblk;
  double v[32], dq[32];
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    v[j] = (rho < n && c < n && rho != c) ? P[rho * n + c] : 0.0;
  }
  uint32_t wds[8];
  fp6_block(v, wds, dq);
  for (int j = 0; j < 32; ++j) Qn[rho * n_pad + bI * 32 + perm_nat(j)] = dq[j];
  fp6_store(tiles, nK, rho, bI, wds);
}

// R = (P_off - E) * out_scale with E the symmetric matrix the MX screen actually evaluates
// (block-upper visit over 128-row K-blocks: off-diagonal blocks from the upper row's scales,
// diagonal blocks symmetrised), natural order; rowabs[k] = sum_l |E_kl|.  One workgroup per row.
__global__ __launch_bounds__(256) void mx_residual_kernel(int64_t n, int64_t n_pad, const double *P, const double *Qn,
                                                          double out_scale, double *R, double *rowabs) {
  const int64_t k = blockIdx.x, bk = k / MXK;
  double s = 0.0;
  for (int64_t l = threadIdx.x; l < n_pad; l += 256) {
    const int64_t bl = l / MXK;
    const double E = bl == bk ? 0.5 * (Qn[k * n_pad + l] + Qn[l * n_pad + k])
                              : (bl > bk ? Qn[k * n_pad + l] : Qn[l * n_pad + k]);
    const double po = (k < n && l < n && k != l) ? P[k * n + l] : 0.0;
    R[k * n_pad + l] = (po - E) * out_scale;
    s += fabs(E);
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) rowabs[k] = (red[0] + red[1]) + (red[2] + red[3]);
}

// nibble planes of a screen panel (storage order, codes 0..2): record (SNP, stage) = two 64-byte
// planes, individual q of the stage at nibble q & 1 of byte q >> 1.  i side: M1 = [a==1] 0xF,
// M2 = [a==2] 0xF; j side: S1 = b, S2 = 2b (fp4 codes of w/2 for w = 1*b, 2*b).
__global__ void nibble_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *nib_i,
                              uint32_t *nib_j) {
  const int64_t per = n_pad / 8;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * per) return;
  const int64_t j = idx / per, d = idx % per;
  const int64_t stage = d / 16, dd = d % 16;
  const int8_t *src = panel + j * n_pad + 8 * d;
  uint32_t m1 = 0, m2 = 0, s1 = 0, s2 = 0;
  for (int e = 0; e < 8; ++e) {
    const uint32_t a = (uint32_t)src[e];
    m1 |= (a == 1 ? 0xFu : 0u) << (4 * e);
    m2 |= (a == 2 ? 0xFu : 0u) << (4 * e);
    s1 |= a << (4 * e);
    s2 |= (2 * a) << (4 * e);
  }
  const int64_t rec = (j * nK + stage) * (NB_REC / 4);
  nib_i[rec + dd] = m1;
  nib_i[rec + 16 + dd] = m2;
  nib_j[rec + dd] = s1;
  nib_j[rec + 16 + dd] = s2;
}

// the j side's S1 planes (nibble_kernel: nibble e of dword dd = code of individual 8 dd + e) at 2 bits
// for the compacted low-rank screen: per (SNP, 128-individual stage) 32 bytes, 8-byte piece k packing
// the plane's dwords 4k .. 4k + 3 as D0 | D1 << 2, D2 | D3 << 2 (codes 0..2 fit two bits)
__global__ void s1_code2_kernel(int64_t m, int64_t n_pad, int nK, const int8_t *panel, uint32_t *out) {
  const int64_t per = n_pad / 16;  // one output dword per 16 individuals
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * per) return;
  const int64_t j = idx / per, g = idx % per;  // g: output dword (16 individuals: plane dwords 2g, 2g + 1)
  const int8_t *src = panel + j * n_pad + 16 * g;
  uint32_t d = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) d |= ((uint32_t)(src[e] & 3) | ((uint32_t)(src[8 + e] & 3) << 2)) << (4 * e);
  out[j * (n_pad / 16) + g] = d;
}

// per row i of P (n x n, natural order): max |P_ik| off the diagonal, |P_ii| and the sum (mod 2^64)
// of a 64-bit mix of every element's bits with its index (the plan's fingerprint of P, order-free)
__global__ __launch_bounds__(256) void p_scan_kernel(int64_t n, const double *P, double *out) {
  const int64_t i = blockIdx.x;
  const double *row = P + i * n;
  double q = 0.0;
  uint64_t h = 0;
  for (int64_t k = threadIdx.x; k < n; k += 256) {
    const double v = row[k];
    if (k != i) q = fmax(q, fabs(v));
    uint64_t z = (uint64_t)__double_as_longlong(v) ^ ((uint64_t)(i * n + k) * 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    h += z ^ (z >> 31);
  }
  __shared__ double sq[256];
  __shared__ uint64_t sh[256];
  sq[threadIdx.x] = q;
  sh[threadIdx.x] = h;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) {
      sq[threadIdx.x] = fmax(sq[threadIdx.x], sq[threadIdx.x + off]);
      sh[threadIdx.x] += sh[threadIdx.x + off];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    out[i] = sq[0];
    out[n + i] = fabs(row[i]);
    out[2 * n + i] = __longlong_as_double((long long)sh[0]);
  }
}

// A = P + (mu + tau) 11'/n - mu I (natural order, n x n) for the prefilter's Cholesky certificate
__global__ void pf_shift_kernel(int64_t n, const double *P, double mu, double tau, double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  const int64_t r = idx / n, c = idx % n;
  A[idx] = P[idx] + (mu + tau) / (double)n - (r == c ? mu : 0.0);
}

// fp4 e2m1 copy of a screen panel (codes 0, 1, 2 -> 0x0, 0x2, 0x4; the prefilter derives the
// squares' codes in registers, sq4); individual 2q at the low nibble of byte q (the MFMA's packing)
// A = P + (mu + tau) 11'/n + ku C - mu I  (C = U U', or none)
__global__ void pf_shift_u_kernel(int64_t n, const double *P, const double *C, double mu, double tau, double ku,
                                  double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  double v = P[idx] + (mu + tau) / (double)n;
  if (C) v += ku * C[idx];
  if (idx / n == idx % n) v -= mu;
  A[idx] = v;
}
// covariate direction dots of a coding: dot[j] = sum_t code[j][t] u[t] (fixed-order reduction)
__global__ __launch_bounds__(256) void cov_dot_kernel(int64_t n_pad, const int8_t *panel, const double *u, double *dot) {
  const int64_t j = blockIdx.x;
  const int8_t *pj = panel + j * n_pad;
  __shared__ double rsum[256];
  double sm = 0.0;
  for (int64_t t = threadIdx.x; t < n_pad; t += 256) sm += (double)pj[t] * u[t];
  rsum[threadIdx.x] = sm;
  __syncthreads();
  for (int off = 128; off > 0; off >>= 1) {
    if ((int)threadIdx.x < off) rsum[threadIdx.x] += rsum[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) dot[j] = rsum[0];
}
// stage-blocked copy of an SNP-major int8 panel (dst[(st m + snp) w + b] = src[snp W + st w + b] for
// stages st of w bytes, W bytes per SNP, 16 bytes per thread), each 8 bytes reordered to individuals
// 0 2 4 6 1 3 5 7 (the K slot order of i8x2_of_fp4_eo)
__global__ void block_panel_perm8_kernel(int64_t m, int64_t W, int64_t w, const uint8_t *__restrict__ src,
                                         uint8_t *__restrict__ dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, per = W / 16;
  if (t >= m * per) return;
  const int64_t snp = t / per, o = (t % per) * 16, st = o / w, b = o % w;
  v4i v = *(const v4i *)(src + snp * W + o);
#pragma unroll
  for (int h = 0; h < 2; ++h) {  // bytes 0..7 of dwords (2h, 2h + 1): even ones first, then odd
    const unsigned lo = (unsigned)v[2 * h], hi = (unsigned)v[2 * h + 1];
    v[2 * h] = (int)__builtin_amdgcn_perm(hi, lo, 0x06040200u);
    v[2 * h + 1] = (int)__builtin_amdgcn_perm(hi, lo, 0x07050301u);
  }
  *(v4i *)(dst + (st * m + snp) * w + b) = v;
}
// prefilter test records (prefilter_pass_kernel's epilogue, 32 bytes per SNP, fetched by LDS-DMA with
// the first stage): fp64 per-SNP sums rounded once to fp32, exactly the values the test used to derive
// itself.  Row role: [i (int bits; -1 = monomorphic), alpha, csum, R1 = csq - 2 alpha csum, sL3, sa,
// (2 + alpha)^2, 0]; column role: [beta, csum, C1n = csq - 2 beta csum + n beta^2, n beta - csum,
// beta spy - sb, sum_k (b + beta)^2, monomorphic, 0]
__global__ void pf_rec_kernel(int64_t m, double n, double spy, const double *__restrict__ soff,
                              const double *__restrict__ csum, const double *__restrict__ csq,
                              const double *__restrict__ sL3, const double *__restrict__ sa,
                              const double *__restrict__ sb, const uint8_t *__restrict__ mono, float *recL,
                              float *recR) {
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= m) return;
  const double al = soff[j], c = csum[j], c2 = csq[j];
  float *l = recL + j * PF_REC, *r = recR + j * PF_REC;
  l[0] = __int_as_float(mono[j] ? -1 : (int)j);
  l[1] = (float)al;
  l[2] = (float)c;
  l[3] = (float)(c2 - 2.0 * al * c);
  l[4] = (float)sL3[j];
  l[5] = (float)sa[j];
  l[6] = (float)((2.0 + al) * (2.0 + al));
  l[7] = 0.0f;
  r[0] = (float)al;
  r[1] = (float)c;
  r[2] = (float)(c2 - 2.0 * al * c + n * al * al);
  r[3] = (float)(n * al - c);
  r[4] = (float)(al * spy - sb[j]);
  r[5] = (float)(c2 + 2.0 * al * c + n * al * al);
  r[6] = mono[j] ? 1.0f : 0.0f;
  r[7] = 0.0f;
}
__global__ void fp4_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint8_t *p4) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= m * (n_pad / 2)) return;
  const int v0 = panel[2 * idx], v1 = panel[2 * idx + 1];
  auto code = [](int v) { return v == 0 ? 0 : v == 1 ? 2 : 4; };
  p4[idx] = (uint8_t)(code(v0) | (code(v1) << 4));
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
__global__ void u8_unit_kernel(int64_t n_pad, const double *__restrict__ Ps, double *__restrict__ unit) {
  const int64_t q = blockIdx.x;
  double mx = 0.0;
  for (int64_t r = threadIdx.x; r < n_pad; r += blockDim.x) mx = fmax(mx, fabs(Ps[q * n_pad + r]));
  for (int off = 32; off > 0; off >>= 1) mx = fmax(mx, __shfl_xor(mx, off));
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x == 0) {
    const double m4 = fmax(fmax(red[0], red[1]), fmax(red[2], red[3]));
    unit[q] = m4 > 0.0 ? m4 / 127.0 : 1.0;
  }
}
__global__ void u8_slice_kernel(int64_t n_pad, const double *__restrict__ Ps, const double *__restrict__ unit,
                                int8_t *__restrict__ out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n_pad * n_pad) return;
  const int64_t q = idx / n_pad, r = idx % n_pad;
  const int64_t st = r / 64;
  const int rr = (int)(r % 64), chunk = rr >> 4, pos = u8_pos(rr & 15);
  const int phys = chunk ^ u8_swz((int)(q & 31));
  double v = Ps[idx] / unit[q];
  int8_t *o = out + (st * U8_S * n_pad + q) * 64 + phys * 16 + pos;
  for (int sl = 0; sl < U8_S; ++sl) {
    const double t = rint(v);
    o[(int64_t)sl * n_pad * 64] = (int8_t)t;
    v = (v - t) * 128.0;
  }
}
// int8 values of the 16 genotype codes of one dword of the 2-bit panel (nibble k = c[k] | c[8 + k] << 2),
// in the order 0 2 4 6 | 1 3 5 7 | 8 10 12 14 | 9 11 13 15
__device__ __forceinline__ v4i i8_of_code2(unsigned d) {
  const unsigned lo = d & 0x33333333u, hi = (d >> 2) & 0x33333333u;
  return v4i{(int)(lo & 0x0f0f0f0fu), (int)((lo >> 4) & 0x0f0f0f0fu), (int)(hi & 0x0f0f0f0fu), (int)((hi >> 4) & 0x0f0f0f0fu)};
}
__global__ __launch_bounds__(512, 1) void u8_gemm_kernel(int64_t m, int64_t n_pad, const uint8_t *__restrict__ p2b,
                                                         const int8_t *__restrict__ slices, const double *__restrict__ unit,
                                                         double *__restrict__ U) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[U8_NS][U8_ST];
  const int tid = threadIdx.x, lane = tid & 63, c = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t j0 = (int64_t)blockIdx.x * U8_J, q0 = (int64_t)blockIdx.y * U8_Q;
  const int S = (int)(n_pad / SG_K);
  // DMAs per stage: wave w the two 1-KB pieces of slice w (q rows 0-15, 16-31); waves 0-3 also the
  // codes of SNPs j0 + 64 w .. + 63 (16 B each)
  const int nq = w < 4 ? 3 : 2;
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]);
  const int8_t *bsrc = slices + ((int64_t)w * n_pad + q0) * 64 + lane * 16;
  const uint8_t *asrc = p2b + std::min<int64_t>(j0 + 64 * w + lane, m - 1) * 16;
  auto issue = [&](int st, int slot) __attribute__((always_inline)) {
    const unsigned base = ring_m0 + slot * U8_ST;
    const int8_t *b = bsrc + (int64_t)st * U8_S * n_pad * 64;
    lds_dma16_m0(b, base + U8_AB + w * 2048);
    lds_dma16_m0(b + 1024, base + U8_AB + w * 2048 + 1024);
    if (w < 4) lds_dma16_m0(asrc + (int64_t)st * m * 16, base + w * 1024);
  };
  static_assert(U8_NS == 4, "wait_for's vmcnt values");
  auto wait_for = [&](int ahead) __attribute__((always_inline)) {
    if (nq == 3) {
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(6)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(3)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    } else {
      if (ahead >= 2)
        asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
      else if (ahead == 1)
        asm volatile("s_waitcnt vmcnt(2)\n\ts_barrier" ::: "memory");
      else
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
  };
  const int pre = min(S, U8_NS - 1);
  for (int st = 0; st < pre; ++st) issue(st, st);
  v16i acc[U8_S];
#pragma unroll
  for (int sl = 0; sl < U8_S; ++sl)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[sl][e] = 0;
  const int sw = u8_swz(c);
  for (int st = 0; st < S; ++st) {
    // stage st landed (the younger stages issued may be in flight), then every wave has left stage
    // st - 1, whose slot the stage issued next reuses
    wait_for(min(st + U8_NS - 2, S - 1) - st);
    if (st + U8_NS - 1 < S) issue(st + U8_NS - 1, (st + U8_NS - 1) % U8_NS);
    const uint8_t *bf = ring[st % U8_NS];
    const v4i ad = *(const v4i *)&bf[(32 * w + c) * 16];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const v4i a8 = i8_of_code2((unsigned)ad[2 * kk + h]);
#pragma unroll
      for (int sl = 0; sl < U8_S; ++sl) {
        const v4i b8 = *(const v4i *)&bf[U8_AB + sl * 2048 + c * 64 + 16 * ((2 * kk + h) ^ sw)];
        acc[sl] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a8, b8, acc[sl], 0, 0, 0);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int64_t q = q0 + c;
  const double uq = unit[q];
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int64_t j = j0 + 32 * w + (e & 3) + 8 * (e >> 2) + 4 * h;
    double sum = (double)acc[U8_S - 1][e];
#pragma unroll
    for (int sl = U8_S - 2; sl >= 0; --sl) sum = sum * (1.0 / 128.0) + (double)acc[sl][e];
    if (j < m) U[j * n_pad + q] = uq * sum;
  }
}

__global__ void code2_panel_kernel(int64_t m, int64_t n_pad, const int8_t *panel, uint32_t *dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x, per = n_pad / 16;
  if (idx >= m * per) return;
  const int64_t snp = idx / per, g = idx % per, st = g >> 2;
  const int8_t *p = panel + snp * n_pad + 16 * g;
  unsigned d = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) d |= (unsigned)((p[k] & 3) | ((p[8 + k] & 3) << 2)) << (4 * k);
  dst[(st * m + snp) * 4 + (g & 3)] = d;
}

// A = P + C + (lam + tau) 11'/n - lam I (natural order) for the low-rank screen's certificate
__global__ void lr_shift_kernel(int64_t n, const double *P, const double *C, double lam, double tau, double *A) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * n) return;
  const int64_t r = idx / n, c = idx % n;
  A[idx] = P[idx] + C[idx] + (lam + tau) / (double)n - (r == c ? lam : 0.0);
}
// G'[j][r] = G[j][r] - soff[j] q1[r] (fp64, rounded once to fp32)
__global__ void lr_adjust_kernel(int64_t m, int64_t R, const double *G, const double *soff, const double *q1, float *out) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < m * R) out[idx] = (float)(G[idx] - soff[idx / R] * q1[idx % R]);
}
__global__ void f64_to_f16_kernel(int64_t count, const double *src, _Float16 *dst) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < count) dst[t] = (_Float16)src[t];  // |U| << 65504 (P entries ~ 1 / sigma, codes <= 2)
}
__global__ void f64_to_f32_kernel(int64_t count, const double *src, float *dst) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < count) dst[idx] = (float)src[idx];
}

double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// ------------------------------------------------------------------ plan object

// ---- tile lists of the low-rank screen built on the device from the prefilter's flags (the host
// builder of build_mx, restated): per 32-column block J the flagged band rows in row order, packed
// into half-tiles of MX_BI/2 rows, consecutive half-tiles (J-major) paired into MX tiles, tile t
// dealt to entry 8 (t mod C) + t / C (C = ceil(tiles / 8): the 8 XCDs get contiguous chunks),
// padding entries -1.  Thread (jl, rg) of a 1024-thread workgroup: column block 64 b + jl, rows
// [TL_R rg, TL_R rg + TL_R) (16 row groups: short load chains, 16 waves per column group).
constexpr int TL_G = 16, TL_R = ROWS_PER_LAUNCH / TL_G;  // row groups, band rows per thread
__global__ __launch_bounds__(1024) void tl_count_kernel(const uint8_t *__restrict__ flags, int Rn, int nJ,
                                                        int *__restrict__ cnt4) {
  const int jl = threadIdx.x & 63, rg = threadIdx.x >> 6, J = blockIdx.x * 64 + jl;
  if (J >= nJ) return;
  int c = 0;
  const int r1 = min(Rn, TL_R * (rg + 1));
#pragma unroll 16
  for (int r = TL_R * rg; r < r1; ++r) c += flags[(size_t)r * nJ + J] != 0;
  cnt4[TL_G * J + rg] = c;
}
__device__ __forceinline__ int tl_total(const int *cnt, int J) {
  int c = 0;
#pragma unroll
  for (int g = 0; g < TL_G; ++g) c += cnt[TL_G * J + g];
  return c;
}
// one workgroup: exclusive scan of the half-tile counts over J; info = {halves, tiles, entries}
__global__ __launch_bounds__(1024) void tl_scan_kernel(const int *__restrict__ cnt4, int nJ, int *__restrict__ H,
                                                       int *__restrict__ info, int *__restrict__ mxt,
                                                       int *__restrict__ mxr) {
  __shared__ int part[1024];
  const int t = threadIdx.x, per = (nJ + 1023) / 1024, j0 = t * per, j1 = min(nJ, j0 + per);
  int sum = 0;
  for (int J = j0; J < j1; ++J) {
    const int c = tl_total(cnt4, J);
    sum += (c + MX_BI / 2 - 1) / (MX_BI / 2);
  }
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int J = j0; J < j1; ++J) {
    H[J] = run;
    const int c = tl_total(cnt4, J);
    run += (c + MX_BI / 2 - 1) / (MX_BI / 2);
  }
  if (t == 0) {
    const int halves = part[1023], tiles = (halves + 1) / 2, C = (tiles + 7) / 8;
    info[0] = halves;
    info[1] = tiles;
    info[2] = 8 * C;
    for (int q = tiles; q < 8 * C; ++q) {  // padding entries
      const int bb = 8 * (q % C) + q / C;
      for (int k = 0; k < MX_TE; ++k) mxt[MX_TE * bb + k] = -1;
    }
    if (halves % 2) {  // the last tile has one half
      const int tl = tiles - 1, bb = 8 * (tl % C) + tl / C;
      mxt[MX_TE * bb + 2] = -1;
      for (int q = 0; q < MX_BI / 2; ++q) mxr[tl * MX_BI + MX_BI / 2 + q] = -1;
    }
  }
}
__global__ __launch_bounds__(1024) void tl_fill_kernel(const uint8_t *__restrict__ flags, int Rn, int nJ,
                                                      const int *__restrict__ cnt4, const int *__restrict__ H,
                                                      const int *__restrict__ info, int *__restrict__ mxt,
                                                      int *__restrict__ mxr) {
  const int jl = threadIdx.x & 63, rg = threadIdx.x >> 6, J = blockIdx.x * 64 + jl;
  if (J >= nJ) return;
  const int C = info[2] / 8, h0 = H[J];
  int idx = 0;
  for (int g = 0; g < rg; ++g) idx += cnt4[TL_G * J + g];
  const int r1 = min(Rn, TL_R * (rg + 1));
#pragma unroll 16
  for (int r = TL_R * rg; r < r1; ++r)
    if (flags[(size_t)r * nJ + J]) {
      const int k = h0 + idx / (MX_BI / 2);
      mxr[(k / 2) * MX_BI + (k % 2) * (MX_BI / 2) + idx % (MX_BI / 2)] = r;
      ++idx;
    }
  if (rg == 0) {  // the tile entries of J's half-tiles and the empty slots of its last one
    const int c = tl_total(cnt4, J);
    const int nh = (c + MX_BI / 2 - 1) / (MX_BI / 2);
    for (int q = c; q < nh * (MX_BI / 2); ++q) {
      const int k = h0 + q / (MX_BI / 2);
      mxr[(k / 2) * MX_BI + (k % 2) * (MX_BI / 2) + q % (MX_BI / 2)] = -1;
    }
    for (int u = 0; u < nh; ++u) {
      const int k = h0 + u, tl = k / 2, bb = 8 * (tl % C) + tl / C;
      if (k % 2 == 0) {
        mxt[MX_TE * bb] = tl;
        mxt[MX_TE * bb + 1] = J;
      } else {
        mxt[MX_TE * bb + 2] = J;
      }
    }
  }
}

// ---- slot lists of the compacted low-rank screen (lrc_screen_kernel), built on the device from the
// prefilter's live-pair masks: band row r's live pairs, in ascending j, are cut into slots of 32
// (the last one padded with -1); slot s = (slot_row[s], slot_j[32 s .. 32 s + 31]).  Slots are
// numbered row by row and grouped 16 to a tile; the padding slots of the last tile have row -1.
// lc_count: live pairs per band row (one workgroup per row).
constexpr int LC_T = 256, LC_SLOTS = MX_BI;  // threads per row; slots per tile
__global__ __launch_bounds__(LC_T) void lc_count_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ,
                                                        int *__restrict__ cnt) {
  __shared__ int part[LC_T / 64];
  const int r = blockIdx.x, tid = threadIdx.x;
  int c = 0;
  for (int J = tid; J < nJ; J += LC_T) c += __popc(lm_mask(lmask[(int64_t)r * nJ + J], tag));
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if ((tid & 63) == 0) part[tid >> 6] = c;
  __syncthreads();
  if (tid == 0) cnt[r] = (part[0] + part[1]) + (part[2] + part[3]);
}
// one workgroup: exclusive scan of the rows' slot counts (soff), info = {slots, tiles}, the padding
// slots of the last tile
__global__ __launch_bounds__(1024) void lc_scan_kernel(const int *__restrict__ cnt, int Rn, int *__restrict__ soff,
                                                       int *__restrict__ info, int *__restrict__ slot_row,
                                                       int64_t slot_cap) {
  __shared__ int part[1024];
  const int t = threadIdx.x, per = (Rn + 1023) / 1024, r0 = t * per, r1 = min(Rn, r0 + per);
  int sum = 0;
  for (int r = r0; r < r1; ++r) sum += (cnt[r] + 31) / 32;
  part[t] = sum;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
    const int v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int r = r0; r < r1; ++r) {
    soff[r] = run;
    run += (cnt[r] + 31) / 32;
  }
  if (t == 0) {
    const int slots = part[1023], tiles = (slots + LC_SLOTS - 1) / LC_SLOTS;
    info[0] = slots;
    info[1] = tiles;
    for (int q = slots; q < tiles * LC_SLOTS && q < slot_cap; ++q) slot_row[q] = -1;
  }
}
// lc_fill: band row r's live second SNPs in ascending order into its slots (one workgroup per row;
// each thread takes a contiguous range of column blocks, a block-wide scan places its pairs), and
// each live pair's record (the prefilter's, at its block's first record + its rank in the block) copied to
// its slot position in slot_ops
__global__ __launch_bounds__(LC_T) void lc_fill_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ,
                                                       const int *__restrict__ cnt, const int *__restrict__ soff,
                                                       int *__restrict__ slot_row, int *__restrict__ slot_j,
                                                       const int *__restrict__ ops, int64_t ops_cap,
                                                       int *__restrict__ slot_ops, int64_t slot_cap) {
  __shared__ int part[LC_T];
  const int r = blockIdx.x, tid = threadIdx.x;
  const int per = (nJ + LC_T - 1) / LC_T, J0 = min(nJ, tid * per), J1 = min(nJ, J0 + per);
  const uint64_t *mk = lmask + (int64_t)r * nJ;
  int c = 0;
  for (int J = J0; J < J1; ++J) c += __popc(lm_mask(mk[J], tag));
  part[tid] = c;
  __syncthreads();
  for (int off = 1; off < LC_T; off <<= 1) {
    const int v = tid >= off ? part[tid - off] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  const int base = soff[r] * 32, n_live = cnt[r], n_slots = (n_live + 31) / 32;
  if ((int64_t)soff[r] + n_slots > slot_cap) return;  // records overflowed: the host reruns the launch
  int k = part[tid] - c;
  for (int J = J0; J < J1; ++J) {
    const uint64_t ent = mk[J];
    uint32_t w = lm_mask(ent, tag);
    if (!w) continue;
    uint32_t src = lm_base(ent);
    while (w) {
      const int b = __ffs(w) - 1;
      w &= w - 1;
      if ((int64_t)src < ops_cap) {  // else the records overflowed: the host reruns the launch
        const v4i *s4 = (const v4i *)(ops + (int64_t)src * OPS_REC);
        v4i *d4 = (v4i *)(slot_ops + (int64_t)(base + k) * OPS_REC);
        d4[0] = s4[0];
        d4[1] = s4[1];
      }
      ++src;
      slot_j[base + k++] = 32 * J + b;
    }
  }
  for (int q = n_live + tid; q < n_slots * 32; q += LC_T) slot_j[base + q] = -1;
  for (int q = tid; q < n_slots; q += LC_T) slot_row[soff[r] + q] = r;
}

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

struct gmat_epi {
  gmat_geno *g = nullptr;
  int64_t n = 0, n_pad = 0, m = 0;
  int n_slice = 3;
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
  DBuf cpack;                                 // refined candidates packed for the read-back
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
  struct LrcBuffers {  // three sets: the prefilters of launches L + 1 and L + 2 are queued while L screens
    DBuf drows[3], lmask[3], ops[3], opc[3], slot_ops[3], slot_row[3], slot_j[3], cnt[3], soff[3], info[3], tlist[3];
    int64_t rl = 0, ops_cap = 0, slot_cap = 0;  // the sets' rows per launch, record and slot capacities
                                                // (grown, never shrunk)
    unsigned ltag[3] = {0, 0, 0};               // the live-block entries' tag of each set's last launch
    void *lm_ptr[3] = {nullptr, nullptr, nullptr};  // the entry buffer that tag refers to
  } lrc;  // compacted low-rank scan buffers (scan_lowrank)
  ~gmat_epi() {
    for (auto ev : kev) (void)hipEventDestroy(ev);
    for (auto ev : sev) (void)hipEventDestroy(ev);
    stream_release(s1);
    stream_release(s2);
    stream_release(s3);
    stream_release(s4);
  }
};

namespace {

// screen panel of a coding (inside e->spanels) and its squared codes (B operand of the Ld term)
const int8_t *screen_panel(const gmat_epi *e, int which) { return e->spanels.as<int8_t>() + which * e->m * e->n_pad; }

// kernel timers: kt_begin records the start event of a launch on st, kt_end its end event
enum { KT_PAIR_SIDE = 0, KT_PAIR_MX = 1, KT_REFINE = 2, KT_REFINE_SIDE = 3, KT_N = 4 };
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
  GMAT_TRY(cd.L3q.alloc((size_t)SIDE_T * m * n_pad));
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
    const int64_t wgs = cdiv(np, R8_PP);
    const bool wide = e->n_pad > 64 * R8_NC;  // w by squares of stages (refine8w_kernel)
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
    size_t kt0;
    GMAT_TRY(kt_begin(e, st, &kt0));
    if (wide)
      hipLaunchKernelGGL(refine8w_kernel, dim3((unsigned)wgs, (unsigned)nseg), dim3(512), 0, st, e->n_pad,
                         e->r8_tiles.as<int8_t>(), sl, sr, pi, pj, np, tpart);
    else
      hipLaunchKernelGGL(refine8_kernel, dim3((unsigned)wgs, (unsigned)nseg), dim3(512), 0, st, e->n_pad,
                         e->r8_tiles.as<int8_t>(), sl, sr, pi, pj, np, e->r8_unit, e->r8_varw.as<double>(), tpart);
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(kt_end(e, st, KT_REFINE, kt0, (double)np));
    GMAT_TRY(kt_begin(e, st, &kt0));
    // the O(n) terms, the segments' combination and the p-values in one launch (as three launches they
    // were two more dependent steps at the end of every scan)
    hipLaunchKernelGGL(refine8_side_kernel, dim3((unsigned)cdiv(np, 4)), dim3(256), 0, st, e->n_pad, sl, sr,
                       L.U.as<double>(), R.U.as<double>(), e->z.as<double>(), e->dg.as<double>(), e->py.as<double>(), lp,
                       rp, L.soff.as<double>(), R.soff.as<double>(), L.off.as<double>(), R.off.as<double>(),
                       L.qa.as<double>(), L.ra.as<double>(), R.qb.as<double>(), R.rb.as<double>(), e->zz,
                       L.mono.as<uint8_t>(), R.mono.as<uint8_t>(), pi, pj, np, e->r8_varw.as<double>(), nseg, tpart,
                       e->r8_unit, eff, var, chi, p);
    GMAT_HIP(hipGetLastError());
    GMAT_TRY(kt_end(e, st, KT_REFINE_SIDE, kt0, (double)np));
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
                const int64_t *pi, const int64_t *pj, int64_t np, double chi_cut, int64_t *n_out, bool reset = true) {
  if (n_out) *n_out = 0;
  if (np <= 0 && !n_out) return GMAT_OK;
  if (np <= 0 && reset) return GMAT_OK;
  // pairs per workgroup: as many as the LDS holds (the P tiles streamed per workgroup are the cost;
  // GMAT_PS_PP caps it for A/B runs)
  const int nK = e->nK;
  auto lds_of = [&](int q) { return 2 * (size_t)MX_TILE + (size_t)q * (nK * 64 + 16) + 4 * (size_t)q * sizeof(double); };
  const int pp_cap = getenv("GMAT_PS_PP") ? atoi(getenv("GMAT_PS_PP")) : 96;
  const int pp = (pp_cap >= 96 && lds_of(96) <= 160 * 1024 - 256) ? 96 : (lds_of(64) <= 160 * 1024 - 256 && pp_cap >= 64) ? 64 : 32;
  GMAT_CHECK(nK <= 63, GMAT_E_ARG, "pair screen: %d stages exceed the LDS", nK);
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
  const size_t lds = lds_of(pp);
  static bool attr = false;
  if (!attr) {
    GMAT_HIP(hipFuncSetAttribute((const void *)pair_mx_kernel<96>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 256));
    GMAT_HIP(hipFuncSetAttribute((const void *)pair_mx_kernel<64>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 256));
    GMAT_HIP(hipFuncSetAttribute((const void *)pair_mx_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                 160 * 1024 - 256));
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
  if (nK <= PXR_NK && !getenv("GMAT_PS_OLD")) {  // w in registers: 256 pairs per workgroup
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
  } else if (nK <= 63 && !getenv("GMAT_PS_OLD")) {  // w in registers by squares of stages (pair_mxw_kernel)
    const int nQ = cdiv(nK, PXR_NK), nseg = nQ * (nQ + 1) / 2;
    if (e->ps_mpart.bytes < (size_t)nseg * np * sizeof(double)) {
      GMAT_HIP(hipStreamSynchronize(st));
      GMAT_TRY(e->ps_mpart.alloc((size_t)std::max(8, nseg) * std::max<int64_t>(np, 1 << 16) * sizeof(double)));
    }
    x.mpart = e->ps_mpart.as<double>();
    hipLaunchKernelGGL(pair_mxw_kernel, dim3((unsigned)cdiv(np, 256), (unsigned)nseg), dim3(512), 0, st, x);
    GMAT_HIP(hipGetLastError());
    hipLaunchKernelGGL(pair_test_kernel, dim3((unsigned)cdiv(np, 256)), dim3(256), 0, st, x, nseg);
  } else if (pp == 96)
    hipLaunchKernelGGL(pair_mx_kernel<96>, dim3((unsigned)cdiv(np, 96)), dim3(768), lds, st, x);
  else if (pp == 64)
    hipLaunchKernelGGL(pair_mx_kernel<64>, dim3((unsigned)cdiv(np, 64)), dim3(512), lds, st, x);
  else
    hipLaunchKernelGGL(pair_mx_kernel<32>, dim3((unsigned)cdiv(np, 32)), dim3(256), lds, st, x);
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

// Q(lam) on the device: block (r, bI) of sqrt(d_r) u_r quantised to fp6 (fp6_block), dequantised
// into Bn (natural [k][r]) and Bs (storage [q][r]), and the tile images when img is given.
__global__ void lr_quant_kernel(int64_t n, int64_t n_pad, int nK, int Rp, const double *__restrict__ Z,
                                const double *__restrict__ sd, double *__restrict__ Bn, double *__restrict__ Bs,
                                uint32_t *__restrict__ img) {
  const int64_t nblk = n_pad / 32;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)Rp * nblk) return;
  const int r = (int)(idx / nblk);
  const int64_t bI = idx % nblk;
  const double s = sd[r];
  double v[32], dq[32];
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    v[j] = (s > 0.0 && c < n) ? s * Z[(size_t)r * n + c] : 0.0;
  }
  uint32_t wds[8];
  fp6_block(v, wds, dq);
  if (img) fp6_store(img, nK, r, bI, wds);
  for (int j = 0; j < 32; ++j) {
    const int64_t c = bI * 32 + perm_nat(j);
    if (c < n) Bn[(size_t)c * Rp + r] = dq[j];
    Bs[(size_t)(bI * 32 + j) * Rp + r] = dq[j];
  }
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
}  // namespace

namespace {
constexpr uint64_t EPI_STATE_MAGIC = 0x31495045544d4147ULL;  // "GMATEPI1"
int import_state(gmat_epi *e, const uint8_t *st, int64_t bytes);
}  // namespace

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
static int ensure_rho(gmat_epi *e, int S) {
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

static int epi_create_impl(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                           const uint8_t *state, int64_t state_bytes) {
  GMAT_CHECK(out && g && pvp && py, GMAT_E_ARG, "gmat_epi_create: bad arguments");
  GMAT_CHECK(n_slice >= 1 && n_slice <= 4, GMAT_E_ARG, "gmat_epi_create: n_slice must be 1..4");
  GMAT_CHECK(g->total_missing == 0, GMAT_E_ARG, "gmat_epi_create: panel has missing genotypes (impute first)");
  GMAT_CHECK(g->n_pad <= 8192 && 2 * g->m * g->n_pad < (1LL << 32), GMAT_E_ARG,
             "gmat_epi_create: supports n_id <= 8192 and 2 * n_snp * n_pad < 2^32 (32-bit buffer offsets)");
  const double t_create = now();
  auto *e = new gmat_epi();
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
      (rc = e->slices.alloc((size_t)n_slice * n_pad * n_pad)) || (rc = e->spanels.alloc((size_t)2 * e->m * n_pad)))
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
  if ((rc = stream_acquire(&sx)) != GMAT_OK) return fail(rc);
  struct StreamGuard {
    hipStream_t s;
    ~StreamGuard() { stream_release(s); }
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
}

extern "C" int gmat_epi_create(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice) {
  return epi_create_impl(out, g, pvp, py, n_slice, nullptr, 0);
}

extern "C" int gmat_epi_create_with(gmat_epi **out, gmat_geno *g, const double *pvp, const double *py, int n_slice,
                                    const uint8_t *state, int64_t state_bytes) {
  GMAT_CHECK(state && state_bytes > 0, GMAT_E_ARG, "gmat_epi_create_with: no state");
  return epi_create_impl(out, g, pvp, py, n_slice, state, state_bytes);
}

namespace {
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
}  // namespace

// The plan's spectral state -- the prefilter and low-rank certificates (P's covariate directions,
// mu, lam, tau, eps and the certified Q's tile images and fp64 copy) -- serialised so that one
// rank computes it and every other rank imports it (gmat_epi_create_with): the eigendecomposition
// and the certificate searches run once per job.  *needed = the size; buf may be null.
extern "C" int gmat_epi_export(const gmat_epi *e, uint8_t *buf, int64_t cap, int64_t *needed) {
  GMAT_CHECK(e && needed, GMAT_E_ARG, "gmat_epi_export: bad arguments");
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
  for (int k = 0; k < 7; ++k) out8[k] = e->setup[k];
  out8[7] = e->pf_ncov;
  return GMAT_OK;
}

extern "C" int gmat_epi_info(const gmat_epi *e, double *out4) {
  GMAT_CHECK(e && out4, GMAT_E_ARG, "gmat_epi_info: bad arguments");
  out4[0] = e->lr_R;
  out4[1] = e->lr_lam;
  out4[2] = e->pf_mu;
  out4[3] = (double)e->n_pad;
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

// (i, j) of every pair of rows[r] (j > i for the triangular kinds, every j for AD), row r's pairs
// starting at offs[r]
__global__ void all_pairs_kernel(const int64_t *__restrict__ rows, const int64_t *__restrict__ offs, int64_t m, int tri,
                                 int64_t *__restrict__ pi, int64_t *__restrict__ pj) {
  const int r = blockIdx.y;
  const int64_t i = rows[r], j0 = tri ? i + 1 : 0, cnt = m - j0, base = offs[r];
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < cnt; t += (int64_t)gridDim.x * blockDim.x) {
    pi[base + t] = i;
    pj[base + t] = j0 + t;
  }
}

// pairs with p < p_cut appended at *count (one atomic per wave; order restored by the host's sort)
__global__ __launch_bounds__(256) void hit_compact_kernel(int64_t np, const int64_t *__restrict__ pi,
                                                          const int64_t *__restrict__ pj, const double *__restrict__ eff,
                                                          const double *__restrict__ var, const double *__restrict__ chi,
                                                          const double *__restrict__ p, double p_cut,
                                                          unsigned long long *count, int64_t *hi, int64_t *hj,
                                                          double *he, double *hv, double *hc, double *hp) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool hit = t < np && p[t] < p_cut;  // NaN never passes (res[res[4] < p_cut])
  const uint64_t mask = __ballot(hit);
  if (!mask) return;
  const int lane = threadIdx.x & 63;
  unsigned long long base = 0;
  if (lane == __ffsll((unsigned long long)mask) - 1) base = atomicAdd(count, (unsigned long long)__popcll(mask));
  base = __shfl(base, __ffsll((unsigned long long)mask) - 1);
  if (!hit) return;
  const int64_t o = (int64_t)base + __popcll(mask & ((1ull << lane) - 1));
  hi[o] = pi[t];
  hj[o] = pj[t];
  he[o] = eff[t];
  hv[o] = var[t];
  hc[o] = chi[t];
  hp[o] = p[t];
}

// ------------------------------------------------------------------ bound audit (diagnostic)
// The certified lower bounds of e'Pe the screens test with, evaluated exactly (fp64, no screen
// arithmetic) for listed pairs, e = (a - alpha)(b - beta) of the screen codes over the real
// individuals: the prefilter's mu |e|^2 - (mu + tau)(1'e)^2/n - ku |U'e|^2 - eps |e|^2 and the
// low-rank screen's lam |Pi e|^2 - tau (1'e)^2/n - eps |e|^2 - |Q'e|^2 (Q = the certified fp6 basis).
// The caller compares them with the exact e'Pe (gmat_epi_pairs): every ratio must be >= 1.
// One workgroup per pair; out[5 t + ..] = {lb_prefilter, lb_lowrank, |e|^2, 1'e, |Q'e|^2}.
constexpr int AUD_T = 256;
__global__ __launch_bounds__(AUD_T) void audit_kernel(int64_t n, int64_t n_pad, int R, int ncov, const int8_t *left,
                                                      const int8_t *right, const double *alpha, const double *beta,
                                                      const int64_t *pi, const int64_t *pj, const double *Q,
                                                      const double *U, double pf_mu, double pf_tau, double pf_eps,
                                                      double pf_ku, double lr_lam, double lr_tau, double lr_eps,
                                                      double *out) {
  __shared__ double es[AUD_T];
  __shared__ double red[AUD_T / 64][8];
  const int tid = threadIdx.x;
  const int64_t t = blockIdx.x, i = pi[t], j = pj[t];
  const int8_t *a = left + i * n_pad, *b = right + j * n_pad;
  const double al = alpha[i], be = beta[j];
  double ee = 0, se = 0, cr = 0, cu[4] = {0, 0, 0, 0};
  for (int64_t s0 = 0; s0 < n_pad; s0 += AUD_T) {
    const int64_t s = s0 + tid;
    const int64_t nat = (s & ~31LL) + perm_nat((int)(s & 31));
    const double e = (nat < n) ? ((double)a[s] - al) * ((double)b[s] - be) : 0.0;
    ee += e * e;
    se += e;
    for (int k = 0; k < ncov; ++k) cu[k] += U[k * n_pad + s] * e;
    es[tid] = e;
    __syncthreads();
    if (tid < R)
      for (int q = 0; q < AUD_T; ++q) cr += Q[(s0 + q) * R + tid] * es[q];
    __syncthreads();
  }
  double v[7] = {ee, se, tid < R ? cr * cr : 0.0, cu[0], cu[1], cu[2], cu[3]};
  for (int q = 0; q < 7; ++q)
    for (int o = 32; o > 0; o >>= 1) v[q] += __shfl_xor(v[q], o);
  if ((tid & 63) == 0)
    for (int q = 0; q < 7; ++q) red[tid >> 6][q] = v[q];
  __syncthreads();
  if (tid == 0) {
    double s7[7];
    for (int q = 0; q < 7; ++q) s7[q] = (red[0][q] + red[1][q]) + (red[2][q] + red[3][q]);
    const double EE = s7[0], SE = s7[1], QQ = s7[2], dn = (double)n;
    double uu = 0.0;
    for (int k = 0; k < ncov; ++k) uu += s7[3 + k] * s7[3 + k];
    out[5 * t + 0] = pf_mu > 0 ? (pf_mu - pf_eps) * EE - (pf_mu + pf_tau) * SE * SE / dn - pf_ku * uu : -INFINITY;
    out[5 * t + 1] = R > 0 ? lr_lam * (EE - SE * SE / dn) - lr_tau * SE * SE / dn - lr_eps * EE - QQ : -INFINITY;
    out[5 * t + 2] = EE;
    out[5 * t + 3] = SE;
    out[5 * t + 4] = QQ;
  }
}

extern "C" int gmat_epi_audit(gmat_epi *e, int kind, const int64_t *pairs, int64_t n_pairs, double *out5) {
  GMAT_CHECK(e && (n_pairs == 0 || (pairs && out5)), GMAT_E_ARG, "gmat_epi_audit: bad arguments");
  GMAT_CHECK(kind >= 0 && kind <= 2, GMAT_E_ARG, "gmat_epi_audit: bad kind");
  if (n_pairs == 0) return GMAT_OK;
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

namespace {

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
                                      int64_t rl = ROWS_PER_LAUNCH) {
  std::vector<ScanLaunch> plan;
  *pairs = 0;
  const int64_t half = rl / 2, nc = cdiv(n_rows, half);
  for (int64_t k = 0, l = nc - 1; k <= l; ++k, --l) {
    ScanLaunch ln;
    for (int64_t t = k * half; t < std::min(n_rows, (k + 1) * half); ++t) ln.rows.push_back(rows[t]);
    if (l != k)
      for (int64_t t = l * half; t < std::min(n_rows, (l + 1) * half); ++t) ln.rows.push_back(rows[t]);
    if (ln.rows.empty()) continue;
    ln.j_lo = tri ? ln.rows[0] + 1 : 0;
    if (tri && ln.j_lo >= m) continue;
    for (int64_t r : ln.rows) *pairs += tri ? (double)(m - 1 - r) : (double)m;
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

// The flush of a screened scan, on stream st, of candidates [lo, hi): the pair screen (use_ps) of
// [ps_done, hi) (those in [lo, ps_done) were pair-screened into cand2 beside the launches), the exact
// fp64 refine of the survivors, and the hits p < p_cut appended to the plan's lists.  Candidates
// below hi are free afterwards.
// [i | j | eff | var | chi | p] of n refined candidates in one buffer (one read-back copy)
__global__ void cand_pack_kernel(int64_t n, const int64_t *ci, const int64_t *cj, const double *eff, const double *var,
                                 const double *chi, const double *p, double *out) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (k >= n) return;
  ((int64_t *)out)[k] = ci[k];
  ((int64_t *)out)[n + k] = cj[k];
  out[2 * n + k] = eff[k];
  out[3 * n + k] = var[k];
  out[4 * n + k] = chi[k];
  out[5 * n + k] = p[k];
}

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
    GMAT_TRY(pin.reserve((size_t)nf * 48));
    int64_t *ci = pin.as<int64_t>(), *cj = ci + nf;
    double *ce = (double *)(cj + nf), *cv = ce + nf, *cc = cv + nf, *cq = cc + nf;
    // the six candidate arrays packed on the device and read back in one copy (six copies cost ~0.1 ms
    // of a step: each is a round trip)
    if (e->cpack.bytes < (size_t)nf * 48) {
      GMAT_HIP(hipStreamSynchronize(st));
      GMAT_TRY(e->cpack.alloc((size_t)std::max<int64_t>(nf, 1 << 16) * 48));
    }
    hipLaunchKernelGGL(cand_pack_kernel, dim3((unsigned)cdiv(nf, 256)), dim3(256), 0, st, nf, fi, fj, e->ceff.as<double>(),
                       e->cvar.as<double>(), e->cchi.as<double>(), e->cp.as<double>(), e->cpack.as<double>());
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpyAsync(ci, e->cpack.p, (size_t)nf * 48, hipMemcpyDeviceToHost, st));
    GMAT_HIP(hipEventRecord(end, st));
    GMAT_HIP(hipStreamSynchronize(st));
    // one bulk copy out of the pinned staging block (element-wise reads of it cost ~50 ns each)
    std::vector<double> hb((size_t)nf * 6);
    std::memcpy(hb.data(), ci, (size_t)nf * 48);
    const int64_t *hi_ = (const int64_t *)hb.data(), *hj_ = hi_ + nf;
    const double *he_ = hb.data() + 2 * nf, *hv_ = he_ + nf, *hc_ = hv_ + nf, *hq_ = hc_ + nf;
    (void)ce, (void)cv, (void)cc, (void)cq;
    for (int64_t k = 0; k < nf; ++k)
      if (hq_[k] < p_cut) {  // NaN never passes, as in the reference's res[res[4] < p_cut]
        e->hit_i.push_back(hi_[k]);
        e->hit_j.push_back(hj_[k]);
        e->hit_eff.push_back(he_[k]);
        e->hit_var.push_back(hv_[k]);
        e->hit_chi.push_back(hc_[k]);
        e->hit_p.push_back(hq_[k]);
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

// hits in (i, j) order, as the reference's row loop emits them
int64_t sort_hits(gmat_epi *e) {
  std::vector<int64_t> ord(e->hit_i.size());
  std::iota(ord.begin(), ord.end(), 0);
  std::sort(ord.begin(), ord.end(), [&](int64_t x, int64_t y) {
    return e->hit_i[x] != e->hit_i[y] ? e->hit_i[x] < e->hit_i[y] : e->hit_j[x] < e->hit_j[y];
  });
  auto apply = [&](auto &v) {
    auto c2 = v;
    for (size_t k = 0; k < ord.size(); ++k) v[k] = c2[ord[k]];
  };
  apply(e->hit_i);
  apply(e->hit_j);
  apply(e->hit_eff);
  apply(e->hit_var);
  apply(e->hit_chi);
  apply(e->hit_p);
  return (int64_t)e->hit_i.size();
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
  const int64_t cap = std::max<int64_t>(m, getenv("GMAT_EXH_CHUNK") ? atoll(getenv("GMAT_EXH_CHUNK")) : (1 << 24));
  if (!e->s3) GMAT_TRY(stream_acquire(&e->s3));
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
      const int64_t c = tri ? m - 1 - rows[r1] : m;
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
      const int64_t per_row = tri ? m - 1 - rows[r0] : m;  // the longest row of the chunk (rows increase)
      hipLaunchKernelGGL(all_pairs_kernel, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(cdiv(per_row, 256), 64)),
                                                (unsigned)nr),
                         dim3(256), 0, st, drows.as<int64_t>(), doffs.as<int64_t>(), m, tri, di.as<int64_t>(),
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
  // first SNPs per launch: LRC_ROWS_PER_LAUNCH, but at least GMAT_LRC_MIN_LAUNCHES (4) launches down to
  // 512 rows (a rank's part of a multi-GPU split keeps the prefilter-ahead pipeline filled), and no more
  // than the three sets' live masks and record bases (8 bytes per (row, 32-column block)) fit in an
  // eighth of the free HBM; GMAT_LRC_ROWS forces it for A/B runs (a multiple of 128, at most 4096)
  int64_t RL = 0;
  {
    const int64_t min_launches = getenv("GMAT_LRC_MIN_LAUNCHES") ? std::max(1, atoi(getenv("GMAT_LRC_MIN_LAUNCHES"))) : 4;
    RL = getenv("GMAT_LRC_ROWS")
             ? std::min<int64_t>(4096, std::max<int64_t>(128, atoll(getenv("GMAT_LRC_ROWS")) / 128 * 128))
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
  const std::vector<ScanLaunch> plan = fold_launches(rows, n_rows, m, tri, &pairs_tested, RL);
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
      GMAT_TRY(B.tlist[b].alloc((size_t)cdiv(rl, PC_TR) * (cdiv(m, PC_TC) + 1) * sizeof(int)));  // PC tiles: the most
      GMAT_TRY(e->pins.tl[b].reserve((size_t)cdiv(rl, PC_TR) * (cdiv(m, PC_TC) + 1) * sizeof(int)));
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
  // (A/B: 23.8 against 24.2 ms per configs[2] step for the column-tile-major list, GMAT_PF_COLORDER)
  const bool pf_blocked_order = !getenv("GMAT_PF_COLORDER");
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
  const int pf_wg = getenv("GMAT_PF_WG") ? std::max(8, atoi(getenv("GMAT_PF_WG"))) : std::max(8, e->n_cu * 7 / 8);
  if (getenv("GMAT_PF_STAMPS")) {
    GMAT_TRY(pf_st.alloc((size_t)PF_NSTAMP * 8 * 1 << 20));
    GMAT_HIP(hipMemset(pf_st.p, 0, (size_t)PF_NSTAMP * 8 * 1 << 20));
  }
  if (!e->s1) GMAT_TRY(stream_acquire(&e->s1));
  if (!e->s2) GMAT_TRY(stream_acquire(&e->s2));
  if (!e->s3) GMAT_TRY(stream_acquire(&e->s3));
  if (!e->s4) GMAT_TRY(stream_acquire(&e->s4));
  // the prefilter passes of even / odd launches on two streams: launch L + 1 (other buffer set) can
  // start on the CUs that the tail of launch L leaves idle (a launch's ~800 equal tiles fill its last
  // round of 256 CUs only partly; on one stream the next launch would wait for the whole tail)
  const hipStream_t sm = e->s1, S3 = e->s3;
  const hipStream_t S2b[2] = {e->s2, getenv("GMAT_PF_ONE_STREAM") ? e->s2 : e->s4};
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
      x.n_rt = (int)cdiv(Rn, PF_TR);
      // the tiles that run (a tile entirely left of the diagonal has no pair), in tile order
      // rt + n_rt ct; MFMA work per pair: 4 fp4 code products + 2 int8 E3 slices over n_pad
      // individuals = 16 n_pad fp4-equivalent ops
      int *tl = e->pins.tl[b].as<int>();
      int run = 0;
      const int64_t n_ct = cdiv(ncols, PF_TC);
      auto runs = [&](int rt, int64_t ct) {
        const int64_t c0 = (ln.j_lo / 32) * 32 + ct * PF_TC;
        return c0 < m && !(tri && c0 + PF_TC - 1 <= ln.rows[rt * PF_TR]);
      };
      if (pf_blocked_order) {
        // blocks of 4 row tiles x 8 column tiles (the 32 workgroups of an XCD run one block at a time:
        // 4 row and 8 column panels per stage instead of 32 + 1), blocks of a row group consecutive
        // (its rows stay in L2 while the columns stream), row groups dealt to the XCDs in eighths
        for (int rg = 0; rg < x.n_rt; rg += 4)
          for (int64_t cg = 0; cg < n_ct; cg += 8)
            for (int64_t ct = cg; ct < std::min(n_ct, cg + 8); ++ct)
              for (int rt = rg; rt < std::min(x.n_rt, rg + 4); ++rt)
                if (runs(rt, ct)) tl[run++] = rt + x.n_rt * (int)ct;
      } else {
        for (int64_t ct = 0; ct < n_ct; ++ct)
          for (int rt = 0; rt < x.n_rt; ++rt)
            if (runs(rt, ct)) tl[run++] = rt + x.n_rt * (int)ct;
      }
      pf_ops_of[li] = (double)run * PF_TR * PF_TC * 16.0 * (double)n_pad;
      GMAT_HIP(hipEventRecord(pf_beg[b], S2));
      if (pf_list) {
        // persistent grid over the list: one workgroup per CU (a multiple of 8).  (Same-box A/B: 27.6
        // against 27.7 ms per configs[2] step for as few workgroups as finish in the same number of
        // tile rounds, and 28.0 against 28.2 for one workgroup per tile, GMAT_PF_NOLIST.)
        GMAT_HIP(hipMemcpyAsync(B.tlist[b].p, tl, (size_t)run * sizeof(int), hipMemcpyHostToDevice, S2));
        x.tile_list = B.tlist[b].as<int>();
        x.n_list = run;
        const int g = 8 * (int)std::min<int64_t>(cdiv(pf_wg, 8), cdiv(run, 8));
        if (run > 0) hipLaunchKernelGGL((prefilter_pass_kernel<true, true>), dim3((unsigned)g), dim3(512), 0, S2, x);
      } else {
        if (li == stamp_launch) stamp_grid = x.n_rt * cdiv(ncols, PF_TC);
        hipLaunchKernelGGL((prefilter_pass_kernel<false, true>), dim3((unsigned)(x.n_rt * cdiv(ncols, PF_TC))), dim3(512),
                           0, S2, x);
      }
      GMAT_HIP(hipEventRecord(pf_end[b], S2));
    } else {
      for (int t = 0; t < E3_PF; ++t) x.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;  // stage-blocked operands
      x.rs2 = L.p2b.as<uint8_t>();
      x.cs2 = R.p2b.as<uint8_t>();
      x.n_rt = (int)cdiv(Rn, PC_TR);
      // the running 64 x 128 tiles in blocks of 4 row x 8 column tiles (as the intercept-only prefilter's
      // list), a persistent grid of one workgroup per CU over them (GMAT_PF_NOLIST: one per tile)
      int *tl = e->pins.tl[b].as<int>();
      int run = 0;
      const int64_t n_ct = cdiv(ncols, PC_TC);
      for (int rg = 0; rg < x.n_rt; rg += 4)
        for (int64_t cg = 0; cg < n_ct; cg += 8)
          for (int64_t ct = cg; ct < std::min(n_ct, cg + 8); ++ct)
            for (int rt = rg; rt < std::min(x.n_rt, rg + 4); ++rt) {
              const int64_t c0 = (ln.j_lo / 32) * 32 + ct * PC_TC;
              if (c0 < m && !(tri && c0 + PC_TC - 1 <= ln.rows[rt * PC_TR])) tl[run++] = rt + x.n_rt * (int)ct;
            }
      // MFMA work per pair: 4 fp4 code products + (2 + K0) int8 products over n_pad individuals
      pf_ops_of[li] = (double)run * PC_TR * PC_TC * (8.0 + 4.0 * (2 + e->pf_ncov)) * (double)n_pad;
      GMAT_HIP(hipEventRecord(pf_beg[b], S2));
      // persistent (one-box A/B, covariate configs[2] step: 35.8 against 41.9 ms for one workgroup per
      // tile, GMAT_PF_NOLIST; the persistent variant spills a few registers at three or four directions)
      if (run > 0 && pf_list) {
        GMAT_HIP(hipMemcpyAsync(B.tlist[b].p, tl, (size_t)run * sizeof(int), hipMemcpyHostToDevice, S2));
        x.tile_list = B.tlist[b].as<int>();
        x.n_list = run;
        const dim3 gp((unsigned)(8 * (int)std::min<int64_t>(cdiv(pf_wg, 8), cdiv(run, 8))));
        switch (e->pf_ncov) {
          case 1: hipLaunchKernelGGL((prefilter_cov_kernel<1, true>), gp, dim3(512), 0, S2, x); break;
          case 2: hipLaunchKernelGGL((prefilter_cov_kernel<2, true>), gp, dim3(512), 0, S2, x); break;
          case 3: hipLaunchKernelGGL((prefilter_cov_kernel<3, true>), gp, dim3(512), 0, S2, x); break;
          default: hipLaunchKernelGGL((prefilter_cov_kernel<4, true>), gp, dim3(512), 0, S2, x); break;
        }
      } else if (run > 0) {
        const dim3 gp((unsigned)(x.n_rt * n_ct));
        if (li == stamp_launch) stamp_grid = x.n_rt * n_ct;
        switch (e->pf_ncov) {
          case 1: hipLaunchKernelGGL((prefilter_cov_kernel<1, false>), gp, dim3(512), 0, S2, x); break;
          case 2: hipLaunchKernelGGL((prefilter_cov_kernel<2, false>), gp, dim3(512), 0, S2, x); break;
          case 3: hipLaunchKernelGGL((prefilter_cov_kernel<3, false>), gp, dim3(512), 0, S2, x); break;
          default: hipLaunchKernelGGL((prefilter_cov_kernel<4, false>), gp, dim3(512), 0, S2, x); break;
        }
      }
      GMAT_HIP(hipEventRecord(pf_end[b], S2));
    }
    GMAT_HIP(hipGetLastError());
    hipLaunchKernelGGL(lc_count_kernel, dim3(Rn), dim3(LC_T), 0, S2, B.lmask[b].as<uint64_t>(), tag, (int)nJ,
                       B.cnt[b].as<int>());
    hipLaunchKernelGGL(lc_scan_kernel, dim3(1), dim3(1024), 0, S2, B.cnt[b].as<int>(), Rn, B.soff[b].as<int>(),
                       B.info[b].as<int>(), B.slot_row[b].as<int>(), B.slot_cap);
    hipLaunchKernelGGL(lc_fill_kernel, dim3(Rn), dim3(LC_T), 0, S2, B.lmask[b].as<uint64_t>(), tag, (int)nJ,
                       B.cnt[b].as<int>(), B.soff[b].as<int>(), B.slot_row[b].as<int>(), B.slot_j[b].as<int>(),
                       B.ops[b].as<int>(), B.ops_cap, B.slot_ops[b].as<int>(), B.slot_cap);
    GMAT_HIP(hipGetLastError());
    GMAT_HIP(hipMemcpyAsync(e->pins.t2[b].p, B.info[b].p, 4 * sizeof(int), hipMemcpyDeviceToHost, S2));
    GMAT_HIP(hipMemcpyAsync(e->pins.t2[b].as<int>() + 4, B.opc[b].p, sizeof(int), hipMemcpyDeviceToHost, S2));
    GMAT_HIP(hipEventRecord(side_end[b], S2));
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
  const bool lrc_j4 = getenv("GMAT_LRC_J4") != nullptr;  // j side as the 4-bit nibble plane (A/B)
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
  const size_t ahead = getenv("GMAT_LRC_AHEAD") ? (size_t)std::max(1, std::min(NBUF - 1, atoi(getenv("GMAT_LRC_AHEAD")))) : 1;
  for (size_t li = 0; li < std::min<size_t>(ahead, plan.size()); ++li) GMAT_TRY(enqueue_side(li, (int)li));
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
      if (lrc_j4)
        hipLaunchKernelGGL((lrc_screen_kernel<false, 3>), dim3((unsigned)tiles), dim3(512), 0, sm, sa, lx);
      else
        hipLaunchKernelGGL((lrc_screen_kernel<true, 3>), dim3((unsigned)tiles), dim3(512), 0, sm, sa, lx);
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
  if (!plan.empty()) {
    const int lb = (int)((plan.size() - 1) % NBUF);
    float ms;
    GMAT_HIP(hipEventElapsedTime(&ms, scr_beg[lb], scr_end[lb]));
    t_screen += ms * 1e-3;
    GMAT_TRY(flush(read_count(lb)));
  }
  *n_hits = sort_hits(e);
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
    double d[PF_NSTAMP - 1] = {0, 0, 0, 0, 0, 0};
    unsigned long long t_min = ~0ull, t_max = 0;
    int64_t nw = 0;
    for (int64_t g = 0; g < stamp_grid; ++g) {
      const unsigned long long *q = &hs[PF_NSTAMP * g];
      if (!q[0] || !q[PF_NSTAMP - 1]) continue;  // tiles that exit at once
      ++nw;
      for (int k = 0; k + 1 < PF_NSTAMP; ++k) d[k] += (double)(q[k + 1] - q[k]) * 0.01;  // 100 MHz ticks -> us
      t_min = std::min(t_min, q[0]);
      t_max = std::max(t_max, q[PF_NSTAMP - 1]);
    }
    const double nn = (double)std::max<int64_t>(nw, 1);
    fprintf(stderr, "prefilter launch %zu: %lld tiles run, per tile: prologue %.2f us, main loop %.2f us, epilogue "
            "%.2f us (column records %.2f, tests %.2f, stores %.2f, masks %.2f); launch span %.1f us\n", stamp_launch,
            (long long)nw, d[0] / nn, d[1] / nn, (d[2] + d[3] + d[4] + d[5]) / nn, d[2] / nn, d[3] / nn, d[4] / nn,
            d[5] / nn, (double)(t_max - t_min) * 0.01);
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
  std::vector<ScanLaunch> plan = fold_launches(rows, n_rows, m, tri, &pairs_tested);

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
  if (!e->s1) GMAT_TRY(stream_acquire(&e->s1));
  if (!e->s2) GMAT_TRY(stream_acquire(&e->s2));
  if (!e->s3) GMAT_TRY(stream_acquire(&e->s3));
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
      const int64_t jb0 = tri ? (ln.rows[r0] + 1) / BJ : 0;
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
        hipLaunchKernelGGL((prefilter_pass_kernel<false, false>), dim3(gp), dim3(512), 0, S2, xp);
      } else {  // covariate designs: 64 x 128 tiles with the direction products
        SideArgs xp = x;
        xp.qimg = e->pf_q.as<uint8_t>();
        for (int t = 0; t < E3_PF; ++t) xp.rs[t] = (const int8_t *)L.L3b.as<uint8_t>() + t * ss;  // stage-blocked
        xp.rs2 = L.p2b.as<uint8_t>();
        xp.cs2 = R.p2b.as<uint8_t>();
        xp.n_rt = (int)cdiv(Rn, PC_TR);
        const unsigned gp = (unsigned)(xp.n_rt * cdiv(ncols, PC_TC));
        switch (e->pf_ncov) {
          case 1: hipLaunchKernelGGL((prefilter_cov_kernel<1, false>), dim3(gp), dim3(512), 0, S2, xp); break;
          case 2: hipLaunchKernelGGL((prefilter_cov_kernel<2, false>), dim3(gp), dim3(512), 0, S2, xp); break;
          case 3: hipLaunchKernelGGL((prefilter_cov_kernel<3, false>), dim3(gp), dim3(512), 0, S2, xp); break;
          default: hipLaunchKernelGGL((prefilter_cov_kernel<4, false>), dim3(gp), dim3(512), 0, S2, xp); break;
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

}  // namespace

extern "C" int gmat_epi_scan(gmat_epi *e, int kind, const int64_t *rows, int64_t n_rows, double p_cut, double chi_cut,
                             int n_slice, int64_t *n_hits) {
  GMAT_CHECK(e && rows && n_hits, GMAT_E_ARG, "gmat_epi_scan: bad arguments");
  GMAT_CHECK(kind >= 0 && kind <= 2, GMAT_E_ARG, "gmat_epi_scan: bad kind");
  const int64_t m = e->m, n_pad = e->n_pad;
  for (int64_t t = 0; t < n_rows; ++t) {
    GMAT_CHECK(rows[t] >= 0 && rows[t] < m, GMAT_E_ARG, "row %lld out of range", (long long)rows[t]);
    GMAT_CHECK(t == 0 || rows[t] > rows[t - 1], GMAT_E_ARG, "rows must be strictly increasing");
  }
  if (n_slice == GMAT_SCREEN_NONE) return scan_exhaustive(e, kind, rows, n_rows, p_cut, n_hits);
  // the compacted low-rank scan serves the low-rank level (automatic at p_cut <= 1e-4, or forced by
  // n_slice -2); GMAT_LR_BLOCKS=1 keeps the block-granular path below (A/B runs)
  const bool lr_level = e->lr_R > 0 && e->pf_mu > 0.0 && (n_slice == -2 || (n_slice == 0 && p_cut <= 1e-4));
  if (lr_level && pair_screen_fits(e) && !getenv("GMAT_LR_BLOCKS") && !getenv("GMAT_NO_PREFILTER"))
    return scan_lowrank(e, kind, rows, n_rows, p_cut, chi_cut, n_hits);
  return scan_blocks(e, kind, rows, n_rows, p_cut, chi_cut, n_slice, n_hits);
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

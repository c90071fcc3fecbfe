// PLINK .bed decoding into device panels, and the genomic relationship matrices.
//
// Decode semantics follow process_plink/_read_plink_bed.c:17-44 (2-bit code c of
// individual k at bits 2*(k%4) of byte k/4 of the SNP's ceil(n/4)-byte row; dosage
// (c^2+c)/6 with code 01 = missing).  The GRM replaces the fp64 GEMM np.dot(X, X.T) of
// gmatrix.py:63 (additive) / :127 (dominance) by an EXACT integer product of the
// uncentred 0/1/2 (or 0/1) codes on int8 MFMA, then applies the centring as fp64
// rank-one corrections:  (G - 1c')(G - 1c')' = GG' - r1' - 1r' + (c'c) 11',  r = Gc.
#include <algorithm>
#include <cstdlib>

#include "dla.h"
#include "geno.h"

using namespace gmat;

namespace {

// one workgroup per SNP: decode, permute into storage order, count
__global__ __launch_bounds__(256) void decode_kernel(const uint8_t *__restrict__ packed, int64_t nb, int64_t n,
                                                     int64_t n_pad, int8_t *__restrict__ dose,
                                                     int8_t *__restrict__ het, int64_t *__restrict__ cnt) {
  const int64_t snp = blockIdx.x;
  const uint8_t *row = packed + snp * nb;
  int s_dose = 0, s_het = 0, s_miss = 0;
  for (int64_t q = threadIdx.x; q < n_pad; q += 256) {
    const int64_t k = (q & ~31LL) + perm_nat((int)(q & 31));
    int d = 0, h = 0;
    if (k < n) {
      const int c = (row[k >> 2] >> (2 * (k & 3))) & 3;
      if (c == 1) {
        s_miss++;
      } else {
        d = (c == 0) ? 0 : c - 1;  // 00->0, 10->1, 11->2
        h = (c == 2);
      }
    }
    dose[snp * n_pad + q] = (int8_t)d;
    het[snp * n_pad + q] = (int8_t)h;
    s_dose += d;
    s_het += h;
  }
  __shared__ int red[3][4];
  for (int off = 32; off > 0; off >>= 1) {
    s_dose += __shfl_xor(s_dose, off);
    s_het += __shfl_xor(s_het, off);
    s_miss += __shfl_xor(s_miss, off);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s_dose;
    red[1][threadIdx.x >> 6] = s_het;
    red[2][threadIdx.x >> 6] = s_miss;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    int64_t t = 0;
    for (int w = 0; w < 4; ++w) t += red[threadIdx.x][w];
    cnt[snp * 3 + threadIdx.x] = t;
  }
}

// ---- GRM: SYRK of the 0/1/2 codes on the block-scaled fp4 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4).
//
// The codes are exact in fp4 e2m1 as halves (0, 0.5 = 0001, 1.0 = 0010: the 2-bit dosage itself in
// the nibble's low bits), so with an e8m0 scale of 2 on each operand every product is the integer
// g_a g_b and the fp32 accumulators hold exact integers (a sum is at most 4m <= 8e6 < 2^24).  fp4 runs
// the 32x32 MFMA at K = 64 in the cycles the int8 form needs for K = 32.
//
// Image (grm_image_kernel, once per call): the panel transposed into 2-bit fragment images, one
// 1 KB image per (32-individual row block rb, 128-SNP stage s) at ((rb S + s) 64 + L) 16: lane L
// holds individual 32 rb + (L & 31); its dword k (< 4) the 16 codes of SNPs 128 s + 64 (k >> 1) +
// 32 (L >> 5) + 16 (k & 1) + [0, 16), code t at bits 2t.  A wave expands dwords 2kk, 2kk + 1 into
// the fp4 fragment of chunk kk with two masks (x & 0x33.., (x >> 2) & 0x33..: the codes of even and
// odd t in the nibbles' low bits; the K order inside a fragment is the same for both operands).
// Individuals past n and SNPs past m are zeros.  The image has the packed panel's size, so the
// stages stream half the bytes fp4 images would (the LDS-DMA fabric, not the MFMA, bounds this loop).
//
// SYRK (grm_partial_kernel): the lower-triangular 256 x 256 tiles of GG', each a K loop over 128-SNP
// stages (two 64-SNP chunks); the (tile, stage) iterations are laid out tile-major and dealt to one
// workgroup (8 waves, each a 128 x 64 block) per CU in equal contiguous ranges (stream-K), so a
// 2,000-individual panel (36 tiles) still fills 256 CUs; every range writes its partial tile (exact
// integers) to a slot and grm_epilogue_kernel sums a tile's slots (exact: order-free).  A stage's
// 16 images (8 KB per operand) stream into a six-stage LDS ring by LDS-DMA (2 per wave), the waves
// read them with conflict-free ds_read_b128 (lane-contiguous images).
constexpr int GT = 256, GS = 128, GNS = 6;
constexpr int GSTAGE = 2 * (GT / 32) * 1024;  // bytes per ring stage: A and B tiles, 16 KB
constexpr int GNT = 512;                            // threads: 8 waves, 2 x 4 wave tiles of 128 x 64

// 2-bit codes of an imputed panel (no 01) to dosages 00 -> 0, 10 -> 1, 11 -> 2 (c - c/2, no borrow
// between fields) or to the heterozygote indicator (10 -> 1)
template <int KIND>
__device__ inline uint32_t grm_decode(uint32_t x) {
  if (KIND == GMAT_GRM_ADD) return x - ((x >> 1) & 0x55555555u);
  return (x >> 1) & ~x & 0x55555555u;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t grm_rsrc(const void *base, int64_t bytes) {
  const uint64_t b = (uint64_t)base;
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)b), hi = __builtin_amdgcn_readfirstlane((unsigned)(b >> 32));
  const unsigned nr = __builtin_amdgcn_readfirstlane((unsigned)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void *)(((uint64_t)hi << 32) | lo), (short)0, (int)nr, 0x00020000);
}

// r[a] = sum_j code[a][j] c[j] in two passes with fixed summation order: part[ch][a] over chunks of
// GR SNP rows (one thread per dword position = 16 individuals, loads unrolled), then one wave per
// individual sums the chunks.
constexpr int GR = 32;
template <int KIND, bool ALIGNED>
__global__ __launch_bounds__(64) void grm_rowdot_kernel(const uint8_t *__restrict__ packed, int64_t nb, int64_t m,
                                                        const double *__restrict__ c, int64_t nd,
                                                        double *__restrict__ part) {
  const int64_t dp = (int64_t)blockIdx.x * 64 + threadIdx.x, ch = blockIdx.y;
  if (dp >= nd) return;
  double acc[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) acc[q] = 0.0;
  const int64_t j0 = ch * GR, j1 = std::min<int64_t>(m, j0 + GR);
  // the chunk's rows through a buffer resource (rows past m read 0): the loads go out together
  const __amdgpu_buffer_rsrc_t rs = grm_rsrc(packed + j0 * nb, (j1 - j0) * nb);
  for (int64_t jb = j0; jb < j1; jb += 16) {
    uint32_t raw[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int so = (int)((jb + u - j0) * nb);
      if (ALIGNED) {
        raw[u] = __builtin_amdgcn_raw_buffer_load_b32(rs, (int)(4 * dp), so, 0);
      } else {
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, (int)(4 * dp) + k, so, 0) << (8 * k);
        raw[u] = v;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      if (jb + u >= j1) break;
      const uint32_t wd = grm_decode<KIND>(raw[u]);
      const double cj = c[jb + u];
#pragma unroll
      for (int q = 0; q < 16; ++q) acc[q] += (double)((wd >> (2 * q)) & 3u) * cj;
    }
  }
  double *dst = part + ch * 16 * nd + 16 * dp;
#pragma unroll
  for (int q = 0; q < 16; ++q) dst[q] = acc[q];
}

__global__ __launch_bounds__(256) void grm_rowdot_reduce_kernel(const double *__restrict__ part, int64_t nd, int64_t n,
                                                                int nch, double *__restrict__ r) {
  const int64_t a = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (a >= n) return;
  double s = 0.0;
  for (int ch = lane; ch < nch; ch += 64) s += part[(int64_t)ch * 16 * nd + a];
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if (lane == 0) r[a] = s;
}

// rows of the packed panel copied to a 4-byte-aligned stride (the SYRK reads dwords of rows)
__global__ __launch_bounds__(256) void pad_rows_kernel(const uint8_t *__restrict__ src, int64_t nb, int64_t m, int64_t nb4,
                                                       uint8_t *__restrict__ dst) {
  const int64_t j = blockIdx.y, b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < m && b < nb4) dst[j * nb4 + b] = b < nb ? src[j * nb + b] : 0;
}

// the images of one (dword position dp = 16 individuals, stage s, lane half h): 64 row dwords decoded,
// each individual's 4 dwords written as its lane's 16 bytes (16 consecutive lanes: 256 B contiguous)
template <int KIND>
__global__ __launch_bounds__(64) void grm_image_kernel(const uint8_t *__restrict__ packed, int64_t nbs, int64_t m,
                                                       int64_t nd, int64_t S, uint8_t *__restrict__ img) {
  const int64_t dp = (int64_t)blockIdx.x * 64 + threadIdx.x, s = blockIdx.y >> 1, h = blockIdx.y & 1;
  // threads past nd (when nd is not a multiple of 64) load zeros and store nothing (the LDS pass below
  // needs every thread of the block)
  // the stage's rows through a buffer resource: rows past m read 0 (range check), no branches
  const int64_t rows = std::min<int64_t>(128, m - 128 * s);
  const __amdgpu_buffer_rsrc_t rs = grm_rsrc(packed + 128 * s * nbs, rows * nbs);
  // dword positions past the row (individuals past n) read out of range too: zeros, no branches
  const int vo = (dp < nd && 4 * dp < nbs) ? (int)(4 * dp) : 0x40000000;
  uint32_t d[64];  // row (SNP) 128 s + 64 (k >> 1) + 32 h + 16 (k & 1) + t at d[16 k + t]
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int r = 64 * (k >> 1) + 32 * (int)h + 16 * (k & 1) + t;
      d[16 * k + t] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo, r * (int)nbs, 0);
    }
  // every load issued before the first decode (otherwise the scheduler can put each decode, and so a
  // vmcnt(0) wait, right behind its load: 64 serial round trips)
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int t = 0; t < 64; ++t) d[t] = grm_decode<KIND>(d[t]);  // zero codes decode to zero
  // each k block: the 16 x 16 matrix of 2-bit codes (row t = SNP, field x = individual) transposed in
  // place by delta swaps (blocks of 8, 4, 2, 1 fields): afterwards d[16 k + x] holds individual x's
  // 16 codes, SNP t at bits 2t
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    uint32_t *q = d + 16 * k;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = 8 >> jj;
      const uint32_t msk = jj == 0 ? 0x0000ffffu : jj == 1 ? 0x00ff00ffu : jj == 2 ? 0x0f0f0f0fu : 0x33333333u;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (r & j) continue;
        const uint32_t t = ((q[r] >> (2 * j)) ^ q[r + j]) & msk;
        q[r + j] ^= t;
        q[r] ^= t << (2 * j);
      }
    }
  }
  // through LDS, so that every store instruction writes two whole 512-byte lane-half runs: thread t's
  // individual x (block-local 16 t + x) at LDS slot 17 t + x (conflict-free 16-byte writes), then lane
  // l of pass p stores individual 32 (2 p + (l >> 5)) + (l & 31) of the block
  __shared__ v4i stg[64 * 17];
  const int tl = threadIdx.x;
#pragma unroll
  for (int x = 0; x < 16; ++x) stg[17 * tl + x] = v4i{(int)d[x], (int)d[16 + x], (int)d[32 + x], (int)d[48 + x]};
  __syncthreads();
  const int64_t nrb = nd / 2;  // row blocks of the image (32 individuals = 2 dword positions each)
#pragma unroll 4
  for (int p = 0; p < 16; ++p) {
    const int il = 32 * (2 * p + (tl >> 5)) + (tl & 31);
    const int64_t rb = ((int64_t)blockIdx.x * 1024 + il) >> 5;
    if (rb < nrb) *(v4i *)(img + ((rb * S + s) * 64 + (il & 31) + 32 * h) * 16) = stg[17 * (il >> 4) + (il & 15)];
  }
}

struct GrmWork {
  const int *seg0;   // [W + 1]: the segments of workgroup w are [seg0[w], seg0[w+1])
  const int *stile;  // per segment: tile, first and end stage (the segment's slot = its index)
  const int *sit0, *sit1;
  const int *ta, *tb;  // per tile: row / column tile
  const int *wrec;     // per workgroup, 8 ints: its segments [s0, s1) and its first segment's tile, first
                       // and end stage, row and column tile (one scalar load at the start, not a chain of 3)
};

typedef int v8i_g __attribute__((ext_vector_type(8)));
typedef float v16f_g __attribute__((ext_vector_type(16)));

// LDS-DMA of one 1 KB image per wave (lane i's 16 bytes land at m0 + 16 i), issued through inline asm
// so that the kernel, not the compiler, counts vmcnt (the builtin makes every ds_read wait for it)
__device__ __forceinline__ void grm_dma(unsigned voff, const void *sbase, unsigned m0) {
  asm volatile("s_nop 0\n\tglobal_load_lds_dwordx4 %0, %1" : : "v"(voff), "s"(sbase), "{m0}"(m0) : "memory");
}

// the fp4 fragment (dwords 2kk, 2kk + 1 of a lane's image bytes): codes of even / odd t per nibble
__device__ __forceinline__ v8i_g grm_expand(int x0, int x1) {
  const unsigned a = (unsigned)x0, b = (unsigned)x1;
  return v8i_g{(int)(a & 0x33333333u), (int)((a >> 2) & 0x33333333u), (int)(b & 0x33333333u),
               (int)((b >> 2) & 0x33333333u), 0, 0, 0, 0};
}

// SHORT: slots of 16-bit counts (a segment of at most 127 stages sums at most 4 x 128 x 127 < 2^16
// per entry): half the slot bytes written here and read by the epilogue
template <bool SHORT>
__global__ __launch_bounds__(GNT) void grm_partial_kernel(const uint8_t *__restrict__ img, int S, GrmWork wk,
                                                          int *__restrict__ partial) {
  __shared__ __attribute__((aligned(1024))) uint8_t ring[GNS * GSTAGE];  // 96 KB
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = w >> 2, wc = w & 3;  // wave block: rows 128 wr .. +128, columns 64 wc .. +64
  // DMA role: waves 0-3 the row tile's images, 4-7 the column tile's; wave w moves the images of
  // row blocks 2 (w & 3) + u (u < 2) of its operand
  const int op = w >> 2, q0 = 2 * (w & 3);
  const unsigned ring_b = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0]);
  // XCD-aware: workgroup b runs on XCD b mod 8, so the work ranges are dealt in 8 contiguous
  // groups -- the workgroups of one XCD stream neighbouring tiles (shared row panels) in its L2
  const int nx = gridDim.x % 8 == 0 ? 8 : 1, bl = (blockIdx.x % nx) * (gridDim.x / nx) + blockIdx.x / nx;
  // the workgroup's record in two 16-byte loads issued together (the table starts with the records)
  const v4i wa = ((const v4i *)wk.wrec)[2 * bl], wb = ((const v4i *)wk.wrec)[2 * bl + 1];
  const int s0 = __builtin_amdgcn_readfirstlane(wa[0]), s1 = __builtin_amdgcn_readfirstlane(wa[1]);
  const unsigned voff = 16u * lane;
  for (int sg = s0; sg < s1; ++sg) {
    int t, it0, it1, ta, tb;
    if (sg == s0) {
      t = wa[2];
      it0 = wa[3];
      it1 = wb[0];
      ta = wb[1];
      tb = wb[2];
    } else {
      t = wk.stile[sg];
      it0 = wk.sit0[sg];
      it1 = wk.sit1[sg];
      ta = wk.ta[t];
      tb = wk.tb[t];
    }
    t = __builtin_amdgcn_readfirstlane(t);
    it0 = __builtin_amdgcn_readfirstlane(it0);
    it1 = __builtin_amdgcn_readfirstlane(it1);
    const int64_t rb0 = (int64_t)__builtin_amdgcn_readfirstlane(op ? tb : ta) * (GT / 32);
    const uint8_t *src[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) src[u] = img + (rb0 + q0 + u) * S * 1024;
    // stage st of the ring (stages past the end re-read the last one: fixed DMA counts)
    auto issue = [&](int st) __attribute__((always_inline)) {
      const int sc = min(st, S - 1);
      const unsigned m0 = ring_b + (unsigned)(st % GNS) * GSTAGE + op * (GSTAGE / 2) + q0 * 1024;
#pragma unroll
      for (int u = 0; u < 2; ++u) grm_dma(voff, src[u] + (int64_t)sc * 1024, m0 + u * 1024);
    };
    v16f_g acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.0f;
#pragma unroll
    for (int u = 0; u < GNS - 1; ++u) issue(it0 + u);
    for (int st = it0; st < it1; ++st) {
      // stage st has landed for this wave (the later GNS - 2 stages may be in flight) and, after the
      // barrier, for every wave; every wave is past stage st - 1, so its slot takes stage st + GNS - 1
      static_assert(GNS == 6, "vmcnt: the later GNS - 2 stages' 2 DMAs per wave");
      asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
      issue(st + GNS - 1);
      const uint8_t *A = ring + (st % GNS) * GSTAGE, *B = A + GSTAGE / 2;
      v4i xa[4], xb[2];
#pragma unroll
      for (int tt = 0; tt < 4; ++tt) xa[tt] = *(const v4i *)&A[(wr * 4 + tt) * 1024 + 16 * lane];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) xb[tt] = *(const v4i *)&B[(wc * 2 + tt) * 1024 + 16 * lane];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        v8i_g fa[4], fb[2];
#pragma unroll
        for (int tt = 0; tt < 4; ++tt) fa[tt] = grm_expand(xa[tt][2 * kk], xa[tt][2 * kk + 1]);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt) fb[tt] = grm_expand(xb[tt][2 * kk], xb[tt][2 * kk + 1]);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa[i], fb[j], acc[i][j], 4, 4, 0, 128, 0, 128);
      }
    }
    // the ring's last (re-read) stages land before the next segment's prologue refills it
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    // slot layout [wave][i][j][e4][lane][4 counts]: every store instruction writes 1 KB (512 B
    // SHORT) contiguous
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          const int64_t at = (int64_t)sg * (GT * GT / 4) + (((w * 8 + i * 2 + j) * 4 + e4) * 64) + lane;
          const float a[4] = {acc[i][j][4 * e4], acc[i][j][4 * e4 + 1], acc[i][j][4 * e4 + 2], acc[i][j][4 * e4 + 3]};
          if (SHORT) {
            typedef int v2i_g __attribute__((ext_vector_type(2)));
            ((v2i_g *)partial)[at] = v2i_g{(int)a[0] | ((int)a[1] << 16), (int)a[2] | ((int)a[3] << 16)};
          } else {
            ((v4i *)partial)[at] = v4i{(int)a[0], (int)a[1], (int)a[2], (int)a[3]};
          }
        }
  }
}

// One workgroup per (tile, 128 x 64 wave block, 64-row half): sum the block's partial slots, centre
// and scale in fp64 (v = (g - r_a - r_b + c'c) / scale, diagonal times (1 + small_val)) and write it
// and its mirror with coalesced rows through an LDS copy.  Accumulator element (i, j, e, lane) of a
// wave is row 32 i + (e & 3) + 8 (e >> 2) + 4 (lane >> 5), column 32 j + (lane & 31) of its block.
template <bool SHORT>
__global__ __launch_bounds__(256) void grm_epilogue_kernel(const int *__restrict__ partial, const int *__restrict__ slot0,
                                                           const int *__restrict__ ta_, const int *__restrict__ tb_,
                                                           int64_t n, const double *__restrict__ r, double cc,
                                                           double scale, double small_val, double *__restrict__ kin) {
  __shared__ double sk[64][65];
  const int t = blockIdx.x, w = blockIdx.y, h = blockIdx.z, tid = threadIdx.x;
  const int wr = w >> 2, wc = w & 3;
  const int sbeg = slot0[t], send = slot0[t + 1];
  const int64_t a0 = (int64_t)ta_[t] * GT + wr * 128 + h * 64, b0 = (int64_t)tb_[t] * GT + wc * 64;
  // this half's v4 positions: ((i*2 + j)*4 + e4)*64 + lane with i in {2h, 2h + 1}
  v4i s[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) s[k] = v4i{0, 0, 0, 0};
  const size_t base = (size_t)w * 2048 + h * 1024 + tid;
  for (int sl = sbeg; sl < send; ++sl) {
    const size_t at = base + (size_t)sl * (GT * GT / 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (SHORT) {
        typedef unsigned v2u_g __attribute__((ext_vector_type(2)));
        const v2u_g x = ((const v2u_g *)partial)[at + k * 256];
        s[k] += v4i{(int)(x[0] & 0xffffu), (int)(x[0] >> 16), (int)(x[1] & 0xffffu), (int)(x[1] >> 16)};
      } else {
        s[k] += ((const v4i *)partial)[at + k * 256];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v4 = h * 1024 + tid + k * 256;
    const int lane = v4 & 63, e0 = ((v4 >> 6) & 3) * 4, ij = v4 >> 8;
    const int i = ij >> 1, j = ij & 1;
    const int bi = j * 32 + (lane & 31);
    const int64_t b = b0 + bi;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = e0 + q;
      const int ai = (i & 1) * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);  // i in {2h, 2h + 1}
      const int64_t a = a0 + ai;
      double v = 0.0;
      if (a < n && b < n) {
        v = ((double)s[k][q] - r[a] - r[b] + cc) / scale;
        if (a == b) v = v + v * small_val;
      }
      sk[ai][bi] = v;
    }
  }
  __syncthreads();
  for (int e = tid; e < 64 * 64; e += 256) {  // block rows
    const int ai = e >> 6, bi = e & 63;
    const int64_t a = a0 + ai, b = b0 + bi;
    if (a < n && b < n) kin[a * n + b] = sk[ai][bi];
  }
  if (ta_[t] != tb_[t])
    for (int e = tid; e < 64 * 64; e += 256) {  // mirror rows
      const int bi = e >> 6, ai = e & 63;
      const int64_t a = a0 + ai, b = b0 + bi;
      if (a < n && b < n) kin[b * n + a] = sk[ai][bi];
    }
}

}  // namespace

extern "C" int gmat_geno_create(gmat_geno **out, const uint8_t *bed_body, int64_t body_bytes, int64_t n_id,
                                int64_t n_snp) {
  GMAT_CHECK(out && bed_body && n_id > 0 && n_snp > 0, GMAT_E_ARG, "gmat_geno_create: bad arguments");
  const int64_t nb = (n_id + 3) / 4;
  GMAT_CHECK(body_bytes >= nb * n_snp, GMAT_E_ARG,
             "gmat_geno_create: .bed body has %lld bytes, %lld x %lld individuals/SNPs need %lld",
             (long long)body_bytes, (long long)n_snp, (long long)n_id, (long long)(nb * n_snp));
  auto *g = new gmat_geno();
  g->n = n_id;
  g->m = n_snp;
  g->nb = nb;
  g->n_pad = round_up(n_id, 256);
  int rc = g->packed.alloc(nb * n_snp + 256);  // tail: dword reads at the end of the last row stay in bounds
  if (rc == GMAT_OK) rc = g->panels.alloc(2 * g->n_pad * n_snp);
  DBuf cnt;
  if (rc == GMAT_OK) rc = cnt.alloc(3 * n_snp * sizeof(int64_t));
  if (rc != GMAT_OK) {
    delete g;
    return rc;
  }
  hipError_t e = hipMemset(g->packed.as<uint8_t>() + nb * n_snp, 0, 256);
  if (e == hipSuccess) e = hipMemcpy(g->packed.p, bed_body, nb * n_snp, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(decode_kernel, dim3((unsigned)n_snp), dim3(256), 0, 0, g->packed.as<uint8_t>(), nb, n_id,
                       g->n_pad, g->dose_ptr(), g->het_ptr(), cnt.as<int64_t>());
    e = hipGetLastError();
  }
  std::vector<int64_t> h(3 * n_snp);
  if (e == hipSuccess) e = hipMemcpy(h.data(), cnt.p, h.size() * sizeof(int64_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) {
    set_error("gmat_geno_create: %s", hipGetErrorString(e));
    delete g;
    return GMAT_E_HIP;
  }
  g->sum_dose.resize(n_snp);
  g->n_het.resize(n_snp);
  g->n_miss.resize(n_snp);
  for (int64_t j = 0; j < n_snp; ++j) {
    g->sum_dose[j] = h[3 * j];
    g->n_het[j] = h[3 * j + 1];
    g->n_miss[j] = h[3 * j + 2];
    g->total_missing += h[3 * j + 2];
  }
  *out = g;
  return GMAT_OK;
}

int geno_subset(const gmat_geno *g, const int64_t *lo, const int64_t *hi, int nr, gmat_geno **out) {
  GMAT_CHECK(g && out && nr >= 1, GMAT_E_ARG, "geno_subset: bad arguments");
  int64_t m = 0;
  for (int r = 0; r < nr; ++r) {
    GMAT_CHECK(lo[r] >= 0 && lo[r] < hi[r] && hi[r] <= g->m, GMAT_E_ARG, "geno_subset: range [%lld, %lld) of %lld SNPs",
               (long long)lo[r], (long long)hi[r], (long long)g->m);
    m += hi[r] - lo[r];
  }
  auto *s = new gmat_geno();
  s->n = g->n;
  s->m = m;
  s->nb = g->nb;
  s->n_pad = g->n_pad;
  if (int rc = s->panels.alloc((size_t)2 * s->n_pad * m)) {
    delete s;
    return rc;
  }
  int64_t at = 0;
  for (int r = 0; r < nr; ++r) {
    const size_t bytes = (size_t)(hi[r] - lo[r]) * g->n_pad;
    hipError_t e = hipMemcpy(s->dose_ptr() + at * s->n_pad, g->dose_ptr() + lo[r] * g->n_pad, bytes, hipMemcpyDeviceToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(s->het_ptr() + at * s->n_pad, g->het_ptr() + lo[r] * g->n_pad, bytes, hipMemcpyDeviceToDevice);
    if (e != hipSuccess) {
      set_error("geno_subset: %s", hipGetErrorString(e));
      delete s;
      return GMAT_E_HIP;
    }
    for (int64_t j = lo[r]; j < hi[r]; ++j) {
      s->sum_dose.push_back(g->sum_dose[j]);
      s->n_het.push_back(g->n_het[j]);
      s->n_miss.push_back(g->n_miss[j]);
      s->total_missing += g->n_miss[j];
    }
    at += hi[r] - lo[r];
  }
  *out = s;
  return GMAT_OK;
}

extern "C" int gmat_geno_counts(const gmat_geno *g, int64_t *sum_dose, int64_t *n_het, int64_t *n_miss) {
  GMAT_CHECK(g, GMAT_E_ARG, "gmat_geno_counts: null handle");
  if (sum_dose) memcpy(sum_dose, g->sum_dose.data(), g->m * sizeof(int64_t));
  if (n_het) memcpy(n_het, g->n_het.data(), g->m * sizeof(int64_t));
  if (n_miss) memcpy(n_miss, g->n_miss.data(), g->m * sizeof(int64_t));
  return GMAT_OK;
}

extern "C" int gmat_geno_destroy(gmat_geno *g) {
  delete g;
  return GMAT_OK;
}

static double g_grm_stats[4] = {0, 0, 0, 0};

extern "C" int gmat_grm_stats(double *out4) {
  GMAT_CHECK(out4, GMAT_E_ARG, "gmat_grm_stats: null");
  for (int k = 0; k < 4; ++k) out4[k] = g_grm_stats[k];
  return GMAT_OK;
}

extern "C" int gmat_grm(gmat_geno *g, int kind, double small_val, double *kin, double *scale_out) {
  GMAT_CHECK(g && kin, GMAT_E_ARG, "gmat_grm: bad arguments");
  GMAT_CHECK(kind == GMAT_GRM_ADD || kind == GMAT_GRM_DOM, GMAT_E_ARG, "gmat_grm: unknown kind %d", kind);
  GMAT_CHECK(g->total_missing == 0, GMAT_E_ARG, "gmat_grm: panel has %lld missing genotypes (impute first)",
             (long long)g->total_missing);
  const int64_t n = g->n, m = g->m, nb = g->nb;
  GMAT_CHECK(m <= 2000000, GMAT_E_ARG, "gmat_grm: at most 2,000,000 SNPs (exact fp32 / int32 accumulation)");
  // centring vector and scale exactly as gmatrix.py:53-57 (additive) / :116-120 (dominance)
  std::vector<double> c(m);
  double scale = 0.0, cc = 0.0;
  for (int64_t j = 0; j < m; ++j) {
    const double freq = (double)g->sum_dose[j] / (2.0 * (double)n);
    const double s = 2.0 * freq * (1.0 - freq);
    if (kind == GMAT_GRM_ADD) {
      c[j] = 2.0 * freq;
      scale += s;
    } else {
      c[j] = s;
      scale += s * (1.0 - s);
    }
    cc += c[j] * c[j];
  }
  if (scale_out) *scale_out = scale;
  // stream-K work list: tiles (ta >= tb) x stages, tile-major, dealt in equal ranges
  const int nt = (int)cdiv(n, GT), ntile = nt * (nt + 1) / 2;
  const int64_t S = cdiv(m, GS), L = (int64_t)ntile * S;  // image SNPs past m are zeros
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const int W = (int)std::max<int64_t>(1, std::min<int64_t>(L, cus));  // one workgroup per CU (128 KB ring)
  std::vector<int> ta(ntile), tb(ntile), seg0(W + 1), st, s0, s1, slot0(ntile + 1, 0);
  for (int a = 0, t = 0; a < nt; ++a)
    for (int b = 0; b <= a; ++b, ++t) {
      ta[t] = a;
      tb[t] = b;
    }
  for (int w = 0; w < W; ++w) {
    seg0[w] = (int)st.size();
    const int64_t i0 = L * w / W, i1 = L * (w + 1) / W;
    for (int64_t it = i0; it < i1;) {
      const int64_t t = it / S, e = std::min(i1, (t + 1) * S);
      st.push_back((int)t);
      s0.push_back((int)(it - t * S));
      s1.push_back((int)(e - t * S));
      it = e;
    }
  }
  seg0[W] = (int)st.size();
  const int nseg = (int)st.size();
  int longest = 0;
  for (int sg = 0; sg < nseg; ++sg) longest = std::max(longest, s1[sg] - s0[sg]);
  const bool shorts = longest * GS * 4 < 65536;  // 16-bit slots hold every segment's counts
  for (int sg = 0; sg < nseg; ++sg) slot0[st[sg] + 1] = sg + 1;  // segments are in tile order
  for (int t = 0; t < ntile; ++t) slot0[t + 1] = std::max(slot0[t + 1], slot0[t]);
  std::vector<int> tabl;
  std::vector<int> wrec(8 * (size_t)W, 0);
  for (int w = 0; w < W; ++w) {
    const int f = seg0[w];
    int *r8 = &wrec[8 * (size_t)w];
    r8[0] = seg0[w];
    r8[1] = seg0[w + 1];
    if (f < seg0[w + 1]) {
      r8[2] = st[f];
      r8[3] = s0[f];
      r8[4] = s1[f];
      r8[5] = ta[st[f]];
      r8[6] = tb[st[f]];
    }
  }
  for (auto *v : {&wrec, &seg0, &st, &s0, &s1, &ta, &tb, &slot0}) tabl.insert(tabl.end(), v->begin(), v->end());
  DBuf dc, dr, dpart, dk, dtab, dpar, dimg;
  const int64_t nd_img = (int64_t)nt * GT / 16;  // image dword positions: every tile row
  const int64_t nd = cdiv(nb, 4);
  const int nch = (int)cdiv(m, GR);
  GMAT_TRY(dc.alloc(m * sizeof(double)));
  GMAT_TRY(dr.alloc(n * sizeof(double)));
  GMAT_TRY(dpar.alloc((size_t)nch * 16 * nd * sizeof(double)));
  GMAT_TRY(dpart.alloc((size_t)nseg * GT * GT * sizeof(int)));
  GMAT_TRY(dk.alloc(n * n * sizeof(double)));
  GMAT_TRY(dimg.alloc((size_t)nt * (GT / 32) * S * 1024));
  GMAT_TRY(dtab.alloc(tabl.size() * sizeof(int)));
  GMAT_HIP(hipMemcpy(dc.p, c.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dtab.p, tabl.data(), tabl.size() * sizeof(int), hipMemcpyHostToDevice));
  const int *tp = dtab.as<int>();
  GrmWork wk;
  wk.wrec = tp;  // first: 32-byte records at the buffer's (aligned) start
  wk.seg0 = tp + 8 * (size_t)W;
  wk.stile = wk.seg0 + (W + 1);
  wk.sit0 = wk.stile + nseg;
  wk.sit1 = wk.sit0 + nseg;
  wk.ta = wk.sit1 + nseg;
  wk.tb = wk.ta + ntile;
  const int *dslot0 = wk.tb + ntile;
  hipEvent_t ev[4];
  for (auto &x : ev) GMAT_HIP(hipEventCreate(&x));
  GMAT_HIP(hipEventRecord(ev[0], 0));
  // rows at a 4-byte-aligned stride: dword buffer loads instead of four byte loads per dword
  const uint8_t *pk = g->packed.as<uint8_t>();
  int64_t nbs = nb;
  DBuf aligned;
  if (nb % 4) {
    nbs = round_up(nb, 4);
    GMAT_TRY(aligned.alloc((size_t)m * nbs + 256));
    GMAT_HIP(hipMemsetAsync(aligned.as<uint8_t>() + (size_t)m * nbs, 0, 256, 0));
    hipLaunchKernelGGL(pad_rows_kernel, dim3((unsigned)cdiv(nbs, 256), (unsigned)m), dim3(256), 0, 0, pk, nb, m, nbs,
                       aligned.as<uint8_t>());
    GMAT_HIP(hipGetLastError());
    pk = aligned.as<uint8_t>();
  }
  const bool al = nbs % 4 == 0;  // always: the rows were padded above
  const dim3 rg((unsigned)cdiv(nd, 64), (unsigned)nch);
  auto rk = kind == GMAT_GRM_ADD ? (al ? grm_rowdot_kernel<GMAT_GRM_ADD, true> : grm_rowdot_kernel<GMAT_GRM_ADD, false>)
                                 : (al ? grm_rowdot_kernel<GMAT_GRM_DOM, true> : grm_rowdot_kernel<GMAT_GRM_DOM, false>);
  hipLaunchKernelGGL(rk, rg, dim3(64), 0, 0, pk, nbs, m, dc.as<double>(), nd, dpar.as<double>());
  hipLaunchKernelGGL(grm_rowdot_reduce_kernel, dim3((unsigned)cdiv(n, 4)), dim3(256), 0, 0, dpar.as<double>(), nd, n,
                     nch, dr.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(ev[1], 0));
  hipLaunchKernelGGL(kind == GMAT_GRM_ADD ? grm_image_kernel<GMAT_GRM_ADD> : grm_image_kernel<GMAT_GRM_DOM>,
                     dim3((unsigned)cdiv(nd_img, 64), (unsigned)(2 * S)), dim3(64), 0, 0, pk, nbs, m, nd_img, S,
                     dimg.as<uint8_t>());
  GMAT_HIP(hipGetLastError());
  hipLaunchKernelGGL(shorts ? grm_partial_kernel<true> : grm_partial_kernel<false>, dim3((unsigned)W), dim3(GNT), 0, 0,
                     dimg.as<uint8_t>(), (int)S, wk, dpart.as<int>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(ev[2], 0));
  hipLaunchKernelGGL(shorts ? grm_epilogue_kernel<true> : grm_epilogue_kernel<false>, dim3((unsigned)ntile, 8, 2), dim3(256),
                     0, 0, dpart.as<int>(), dslot0, wk.ta, wk.tb, n,
                     dr.as<double>(), cc, scale, small_val, dk.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(ev[3], 0));
  GMAT_HIP(hipEventSynchronize(ev[3]));
  float ms_gemm = 0, ms_all = 0;
  GMAT_HIP(hipEventElapsedTime(&ms_gemm, ev[1], ev[2]));
  GMAT_HIP(hipEventElapsedTime(&ms_all, ev[0], ev[3]));
  for (auto &x : ev) (void)hipEventDestroy(x);
  g_grm_stats[0] = ms_gemm * 1e-3;                                   // image + the fp4 SYRK
  g_grm_stats[1] = (double)ntile * 2.0 * GT * GT * (double)(S * GS);  // fp4 MFMA ops of the lower tiles
  g_grm_stats[2] = 2.0 * (double)n * n * m;                           // dense-equivalent flop 2n^2m
  g_grm_stats[3] = ms_all * 1e-3;                                     // row sums + SYRK + epilogue
  GMAT_HIP(hipMemcpy(kin, dk.p, n * n * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

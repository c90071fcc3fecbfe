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

// ---- GRM: int8 MFMA SYRK straight from the packed .bed rows.
//
// Work: the lower-triangular 256 x 256 tiles of GG' (G: individuals x SNPs codes), each a K loop
// over 64-SNP stages.  The (tile, stage) iterations are laid out tile-major and dealt to a grid of
// one workgroup (8 waves, each a 128 x 64 block) per CU in equal contiguous ranges (stream-K), so
// a 2,000-individual panel (36 tiles) still fills 256 CUs; every range writes its int32 partial tile
// to a slot and
// grm_epilogue_kernel sums a tile's slots in a fixed order (exact integers: deterministic).
//
// Staging: each thread loads 4 SNP rows x 4 bytes (16 individuals x 4 SNPs, 2 bits each) of the
// packed rows, decodes the 2-bit codes in place (SWAR), gathers the 4 rows' bytes per byte position
// with v_perm and writes each individual's 4 SNP codes as one dword of the LDS tile [row][k]
// (pitch 80 B: conflict-free ds_read_b128 fragments, at most 2-way on the stores).  The code of individual 4p+f sits at bits
// 2f of byte p; fields 0-2 are masked in place (values scaled by 1, 4, 16) and field 3 shifted by 4
// (scale 4), so one AND (two for f = 3) yields int8 values <= 32; the product picks up the exact
// factor s(f_a) s(f_b) <= 256, divided out in the epilogue.  LDS row of tile individual i (i =
// 64h + 16d + x, x = 4b + f): 64h + 8(x >> 1) + 2d + (x & 1), so a wave's 64 x 64 quadrant of the
// tile holds 64 contiguous individuals on each side, and the 32 lanes of a store group (four dword
// positions d on rows 2 apart = 8 banks apart at the 80-byte pitch, eight SNP quads) hit 32
// distinct banks.
constexpr int GT = 256, GS = 64, GP = 80, GD = 4;  // GD: stages of packed rows in flight per thread
constexpr int GNT = 512;                            // threads: 8 waves, 2 x 4 wave tiles of 128 x 64

// i = 64h + 16d + x  ->  row = 64h + 8(x >> 1) + 2d + (x & 1)
__device__ __host__ inline int grm_row_of(int i) {
  const int x = i & 15, d = (i >> 4) & 3;
  return (i & ~63) + 8 * (x >> 1) + 2 * d + (x & 1);
}
__device__ __host__ inline int grm_ind_of(int row) {
  const int r = row & 63;
  return (row & ~63) + 16 * ((r >> 1) & 3) + 2 * (r >> 3) + (r & 1);
}
__device__ __host__ inline int grm_scale_of_row(int row) {
  const int f = ((row >> 2) & 2) | (row & 1);  // field of the individual = its index mod 4
  return f == 0 ? 1 : (f == 2 ? 16 : 4);
}

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
  for (int64_t jb = j0; jb < j1; jb += 16) {
    uint32_t raw[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int64_t j = jb + u;
      uint32_t v = 0;
      if (j < j1) {
        const uint8_t *src = packed + j * nb + 4 * dp;
        if (ALIGNED)
          v = *(const uint32_t *)src;
        else
          v = (uint32_t)src[0] | ((uint32_t)src[1] << 8) | ((uint32_t)src[2] << 16) | ((uint32_t)src[3] << 24);
      }
      raw[u] = v;
    }
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

struct GrmWork {
  const int *seg0;   // [W + 1]: the segments of workgroup w are [seg0[w], seg0[w+1])
  const int *stile;  // per segment: tile, first and end stage (the segment's slot = its index)
  const int *sit0, *sit1;
  const int *ta, *tb;  // per tile: row / column tile
};

template <int KIND, bool ALIGNED>
__global__ __launch_bounds__(GNT) void grm_partial_kernel(const uint8_t *__restrict__ packed, int64_t nb, int64_t m,
                                                          GrmWork wk, int *__restrict__ partial) {
  __shared__ __attribute__((aligned(16))) int8_t sm[2][2][GT * GP];  // [buffer][operand]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wr = w >> 2, wc = w & 3;  // wave block: rows 128 wr .. +128, columns 64 wc .. +64
  // loader (waves 0-3: row tile, 4-7: column tile): a store group of 32 lanes covers four dword
  // positions (rows 2 apart) x eight SNP quads; each lane loads its dword of four stage rows
  const int op = w >> 2, wv = w & 3;
  const int dpos = (lane & 3) + 4 * (lane >> 5) + 8 * (wv & 1), qd = (wv >> 1) * 8 + ((lane >> 2) & 7);
  // XCD-aware: workgroup b runs on XCD b mod 8, so the work ranges are dealt in 8 contiguous
  // groups -- the workgroups of one XCD stream neighbouring tiles (shared row panels) in its L2
  const int nx = gridDim.x % 8 == 0 ? 8 : 1, bl = (blockIdx.x % nx) * (gridDim.x / nx) + blockIdx.x / nx;
  const int s0 = wk.seg0[bl], s1 = wk.seg0[bl + 1];
  const __amdgpu_buffer_rsrc_t rs = grm_rsrc(packed, m * nb + 256);  // + the zeroed tail of the panel
  for (int sg = s0; sg < s1; ++sg) {
    const int t = wk.stile[sg], it0 = wk.sit0[sg], it1 = wk.sit1[sg];
    // byte offsets of this thread's dword in its four rows of a stage; the stage adds it * GS * nb
    // as the scalar offset, and rows past the panel read the zeroed tail or 0 (buffer range)
    const int boff = (op ? wk.tb[t] : wk.ta[t]) * (GT / 4) + 4 * dpos;
    int vo[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) vo[q] = (4 * qd + q) * (int)nb + boff;
    uint32_t raw[GD][4];  // register ring: stages in flight
    auto load = [&](int it, uint32_t (&rw)[4]) {  // unconditional (past the segment: ignored or zeros),
      const int so = it * GS * (int)nb;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (ALIGNED) {
          rw[q] = __builtin_amdgcn_raw_buffer_load_b32(rs, vo[q], so, 0);
        } else {
          uint32_t v = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) v |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rs, vo[q] + k, so, 0) << (8 * k);
          rw[q] = v;
        }
      }
    };
    auto unpack = [&](int buf, const uint32_t (&rw)[4]) {
      const uint32_t d0 = grm_decode<KIND>(rw[0]), d1 = grm_decode<KIND>(rw[1]), d2 = grm_decode<KIND>(rw[2]),
                     d3 = grm_decode<KIND>(rw[3]);
      // X_b = [d0.b, d1.b, d2.b, d3.b]: byte position b of the four SNP rows
      const uint32_t t01l = __builtin_amdgcn_perm(d1, d0, 0x05010400u), t23l = __builtin_amdgcn_perm(d3, d2, 0x05010400u);
      const uint32_t t01h = __builtin_amdgcn_perm(d1, d0, 0x07030602u), t23h = __builtin_amdgcn_perm(d3, d2, 0x07030602u);
      uint32_t X[4];
      X[0] = __builtin_amdgcn_perm(t23l, t01l, 0x05040100u);
      X[1] = __builtin_amdgcn_perm(t23l, t01l, 0x07060302u);
      X[2] = __builtin_amdgcn_perm(t23h, t01h, 0x05040100u);
      X[3] = __builtin_amdgcn_perm(t23h, t01h, 0x07060302u);
      int8_t *dst = sm[buf][op] + 4 * qd;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int i0 = 16 * dpos + 4 * b;  // individuals i0 .. i0+3 (fields 0..3)
        *(uint32_t *)(dst + grm_row_of(i0 + 0) * GP) = X[b] & 0x03030303u;
        *(uint32_t *)(dst + grm_row_of(i0 + 1) * GP) = X[b] & 0x0c0c0c0cu;
        *(uint32_t *)(dst + grm_row_of(i0 + 2) * GP) = X[b] & 0x30303030u;
        *(uint32_t *)(dst + grm_row_of(i0 + 3) * GP) = (X[b] >> 4) & 0x0c0c0c0cu;
      }
    };
    v16i acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[i][j][e] = 0;
    // ring slot u holds stage it0 + u (mod GD); stage it0 is unpacked before the loop
#pragma unroll
    for (int u = 0; u < GD; ++u) load(it0 + u, raw[u]);
    unpack(0, raw[0]);
    __syncthreads();
    for (int base = it0; base < it1; base += GD) {  // segments hold whole multiples of GD stages
#pragma unroll
      for (int u = 0; u < GD; ++u) {
        const int it = base + u;
        const int cur = (it - it0) & 1;
        load(it + GD, raw[u]);  // slot u's stage (it) is already in LDS
        const int8_t *A = sm[cur][0], *B = sm[cur][1];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          v4i fa[4], fb[2];
#pragma unroll
          for (int tt = 0; tt < 4; ++tt)
            fa[tt] = *(const v4i *)&A[(wr * 128 + tt * 32 + (lane & 31)) * GP + kk * 32 + (lane >> 5) * 16];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt)
            fb[tt] = *(const v4i *)&B[(wc * 64 + tt * 32 + (lane & 31)) * GP + kk * 32 + (lane >> 5) * 16];
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[i], fb[j], acc[i][j], 0, 0, 0);
        }
        if (it + 1 < it1) unpack(cur ^ 1, raw[(u + 1) % GD]);
        __syncthreads();
      }
    }
    int *dst = partial + (int64_t)sg * GT * GT;
    // slot layout [wave][i][j][e4][lane][4]: every store instruction writes 1 KB contiguous
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e4 = 0; e4 < 4; ++e4) {
          v4i v;
          v[0] = acc[i][j][4 * e4];
          v[1] = acc[i][j][4 * e4 + 1];
          v[2] = acc[i][j][4 * e4 + 2];
          v[3] = acc[i][j][4 * e4 + 3];
          ((v4i *)dst)[(((w * 8 + i * 2 + j) * 4 + e4) * 64) + lane] = v;
        }
  }
}

// One workgroup per (tile, 128 x 64 wave block, 64-row half): sum the block's partial slots (fixed
// order), undo the field scales, centre and scale in fp64 (v = (g - r_a - r_b + c'c) / scale,
// diagonal times (1 + small_val)) and write it and its mirror with coalesced rows through an LDS
// copy.
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
  const v4i *base = (const v4i *)partial + (size_t)w * 2048 + h * 1024 + tid;
  for (int sl = sbeg; sl < send; ++sl) {
    const v4i *src = base + (size_t)sl * (GT * GT / 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) s[k] += src[k * 256];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v4 = h * 1024 + tid + k * 256;
    const int lane = v4 & 63, e0 = ((v4 >> 6) & 3) * 4, ij = v4 >> 8;
    const int i = ij >> 1, j = ij & 1;
    const int col = wc * 64 + j * 32 + (lane & 31);
    const int bi = grm_ind_of(col) - wc * 64, sb = grm_scale_of_row(col);
    const int64_t b = b0 + bi;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = e0 + q;
      const int row = wr * 128 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5);
      const int ai = grm_ind_of(row) - wr * 128 - h * 64, sa = grm_scale_of_row(row);
      const int64_t a = a0 + ai;
      double v = 0.0;
      if (a < n && b < n) {
        const int g = s[k][q] / (sa * sb);  // exact: every product carries the factor sa * sb
        v = ((double)g - r[a] - r[b] + cc) / scale;
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
  GMAT_CHECK(m <= 2000000 && (m + 2 * GS * GD) * round_up(nb, 4) + 256 < (1LL << 31), GMAT_E_ARG,
             "gmat_grm: at most 2,000,000 SNPs and 2 GB of packed codes (int32 accumulation, 32-bit offsets)");
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
  const int64_t S = round_up(cdiv(m, GS), GD), L = (int64_t)ntile * S;  // stages past m read zeros
  int cus = 256;
  {
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  }
  const char *wenv = getenv("GMAT_GRM_WG_PER_CU");
  const int W = (int)std::max<int64_t>(1, std::min<int64_t>(L / GD, (int64_t)cus * (wenv ? std::max(1, atoi(wenv)) : 1)));
  std::vector<int> ta(ntile), tb(ntile), seg0(W + 1), st, s0, s1, slot0(ntile + 1, 0);
  for (int a = 0, t = 0; a < nt; ++a)
    for (int b = 0; b <= a; ++b, ++t) {
      ta[t] = a;
      tb[t] = b;
    }
  for (int w = 0; w < W; ++w) {
    seg0[w] = (int)st.size();
    const int64_t i0 = L / GD * w / W * GD, i1 = L / GD * (w + 1) / W * GD;
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
  for (int sg = 0; sg < nseg; ++sg) slot0[st[sg] + 1] = sg + 1;  // segments are in tile order
  for (int t = 0; t < ntile; ++t) slot0[t + 1] = std::max(slot0[t + 1], slot0[t]);
  std::vector<int> tabl;
  for (auto *v : {&seg0, &st, &s0, &s1, &ta, &tb, &slot0}) tabl.insert(tabl.end(), v->begin(), v->end());
  DBuf dc, dr, dpart, dk, dtab, dpar;
  const int64_t nd = cdiv(nb, 4);
  const int nch = (int)cdiv(m, GR);
  GMAT_TRY(dc.alloc(m * sizeof(double)));
  GMAT_TRY(dr.alloc(n * sizeof(double)));
  GMAT_TRY(dpar.alloc((size_t)nch * 16 * nd * sizeof(double)));
  GMAT_TRY(dpart.alloc((size_t)nseg * GT * GT * sizeof(int)));
  GMAT_TRY(dk.alloc(n * n * sizeof(double)));
  GMAT_TRY(dtab.alloc(tabl.size() * sizeof(int)));
  GMAT_HIP(hipMemcpy(dc.p, c.data(), m * sizeof(double), hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(dtab.p, tabl.data(), tabl.size() * sizeof(int), hipMemcpyHostToDevice));
  const int *tp = dtab.as<int>();
  GrmWork wk;
  wk.seg0 = tp;
  wk.stile = tp + (W + 1);
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
  auto kern = kind == GMAT_GRM_ADD ? (al ? grm_partial_kernel<GMAT_GRM_ADD, true> : grm_partial_kernel<GMAT_GRM_ADD, false>)
                                   : (al ? grm_partial_kernel<GMAT_GRM_DOM, true> : grm_partial_kernel<GMAT_GRM_DOM, false>);
  hipLaunchKernelGGL(kern, dim3((unsigned)W), dim3(GNT), 0, 0, pk, nbs, m, wk, dpart.as<int>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(ev[2], 0));
  hipLaunchKernelGGL(grm_epilogue_kernel, dim3((unsigned)ntile, 8, 2), dim3(256), 0, 0, dpart.as<int>(), dslot0, wk.ta, wk.tb, n,
                     dr.as<double>(), cc, scale, small_val, dk.as<double>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipEventRecord(ev[3], 0));
  GMAT_HIP(hipEventSynchronize(ev[3]));
  float ms_gemm = 0, ms_all = 0;
  GMAT_HIP(hipEventElapsedTime(&ms_gemm, ev[1], ev[2]));
  GMAT_HIP(hipEventElapsedTime(&ms_all, ev[0], ev[3]));
  for (auto &x : ev) (void)hipEventDestroy(x);
  g_grm_stats[0] = ms_gemm * 1e-3;                                   // grm_partial_kernel (the int8 SYRK)
  g_grm_stats[1] = (double)ntile * 2.0 * GT * GT * (double)(cdiv(m, GS) * GS);  // int8 ops of the lower tiles
  g_grm_stats[2] = 2.0 * (double)n * n * m;                           // dense-equivalent flop 2n^2m
  g_grm_stats[3] = ms_all * 1e-3;                                     // row sums + SYRK + epilogue
  GMAT_HIP(hipMemcpy(kin, dk.p, n * n * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// Exact refine of candidate pairs, the pair screen in front of it, hit compaction (see epi.h for the stage files).
#include "epi.h"

namespace gmat {
namespace epi {

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

// w = a o b of 16 individuals (4 dwords of int8 values 0 / 1 / 2 / 4) as 16 2-bit codes {0, 1, 2, 3}
__device__ __forceinline__ unsigned r8_pack_w(v4i v) {
  unsigned d = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const unsigned x = (unsigned)v[k], c = x - ((x >> 2) & 0x01010101u);  // 4 -> 3
    d |= ((c | (c >> 6) | (c >> 12) | (c >> 18)) & 0xffu) << (8 * k);
  }
  return d;
}
// the 4 int8 w of codes 4 k .. 4 k + 3 of a packed dword (byte j: code j of byte k of d, through {0, 1, 2, 4})
__device__ __forceinline__ int r8_w4(unsigned d, int k) {
  const unsigned x = (d >> (8 * k)) & 0xffu;
  const unsigned y = (x << 6) | x;
  const unsigned sel = ((y << 12) | y) & 0x03030303u;
  return (int)__builtin_amdgcn_perm(0u, 0x04020100u, sel);
}
__device__ __forceinline__ v4i r8_unpack_w(unsigned d) { return v4i{r8_w4(d, 0), r8_w4(d, 1), r8_w4(d, 2), r8_w4(d, 3)}; }

// 256 pairs per workgroup (R8_PP2): a wave holds w of two 16-pair groups as 2-bit codes (one dword per
// 64-individual chunk and lane instead of four int8 dwords), expanded into the MFMA's B fragments per tile
// (five VALU per dword), so every slice tile streamed into LDS serves twice the pairs of the int8-register
// layout: the kernel is bound by that L2 -> LDS stream (14.7 MB per workgroup at n_pad 2,048).
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
  // pair group u of the wave: pairs 32 w + 16 u + c; chunk kc of w (screen codes 0 / 1 / 2 multiplied)
  // holds individuals 64 kc + 16 g .. + 15 as 2-bit codes
  int64_t p[2];
  bool valid[2];
  unsigned wf[2][R8_NC];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    p[u] = (int64_t)blockIdx.x * R8_PP2 + 32 * w + 16 * u + c;
    valid[u] = p[u] < np;
    const int8_t *ra = sl + (valid[u] ? pi[p[u]] : 0) * n_pad, *rb = sr + (valid[u] ? pj[p[u]] : 0) * n_pad;
#pragma unroll
    for (int kc = 0; kc < R8_NC; ++kc) {
      v4i v = {0, 0, 0, 0};
      if (valid[u] && kc < NS) {
        const v4i va = *(const v4i *)(ra + 64 * kc + 16 * g), vb = *(const v4i *)(rb + 64 * kc + 16 * g);
#pragma unroll
        for (int d = 0; d < 4; ++d)
          v[d] = (int)__builtin_amdgcn_perm(T_HI, T_LO, to_offset((unsigned)va[d]) + (unsigned)vb[d]);
      }
      wf[u][kc] = r8_pack_w(v);
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
  v4i acc[2][R8_S][2];
  // per-lane slice sums in int32: |acc| <= 127 * 4 * n_pad = 2^20 (n_pad <= 2,048), a fold of four rows
  // <= 2^24, at most 64 row blocks per lane <= 2^30; the lanes' sums are added in fp64
  int T[2][R8_S];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < R8_S; ++s) T[u][s] = 0;
  const int swz = 16 * (g ^ r8_swz(c));
  int v = 0;
  unsigned wlast[2] = {0u, 0u};
  for (int kb = kb_lo; kb < kb_hi; ++kb) {
    const int c0 = kb >> 1;
    // the row block's sums start at zero (its first tile is cs = NS - 1; a zero C operand selected per
    // tile compiled to a v_cndmask per accumulator register in every tile)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int s = 0; s < R8_S; ++s) acc[u][s][0] = acc[u][s][1] = zv;
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
        unsigned wc[2] = {wf[0][cs], wf[1][cs]};
        // opaque per visit: else the expansion of every chunk is hoisted out of the row-block loop (256
        // registers of B fragments, spilled)
        asm volatile("" : "+v"(wc[0]), "+v"(wc[1]));
        const v4i wb0 = r8_unpack_w(wc[0]), wb1 = r8_unpack_w(wc[1]);
#pragma unroll
        for (int s = 0; s < R8_S; ++s)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const v4i fa = *(const v4i *)(tb + s * R8_TB + (rt * 16 + c) * 64 + swz);
            acc[0][s][rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, wb0, acc[0][s][rt], 0, 0, 0);
            acc[1][s][rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, wb1, acc[1][s][rt], 0, 0, 0);
          }
        if (cs == cq) {  // the row block's last tile: its w is the fold's
          wlast[0] = wc[0];
          wlast[1] = wc[1];
        }
        ++v;
      }
    }
    // rows of block kb done: fold with w at the lane's rows 4 g .. 4 g + 3 of each row tile (after the
    // unrolled visits, which stay small enough to unroll fully: a fold inside each copy put wf in scratch)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        // row tile rt of block kb is individuals 64 cs + 16 (2 (kb & 1) + rt) + .. of chunk cs = kb / 2: group
        // 2 (kb & 1) + rt, held by lane c + 16 (2 (kb & 1) + rt); this lane's rows 4 g .. + 3 are its byte g
        const unsigned wd = (unsigned)__shfl((int)wlast[u], c + 16 * (2 * (kb & 1) + rt));
        const unsigned w4 = (unsigned)r8_w4(wd, g);
        const int w0 = (int)(w4 & 0xff), w1 = (int)((w4 >> 8) & 0xff), w2 = (int)((w4 >> 16) & 0xff), w3 = (int)(w4 >> 24);
#pragma unroll
        for (int s = 0; s < R8_S; ++s)  // |acc| < 2^21: 24-bit multiplies are exact
          T[u][s] += __mul24(w0, acc[u][s][rt][0]) + __mul24(w1, acc[u][s][rt][1]) + __mul24(w2, acc[u][s][rt][2]) +
                     __mul24(w3, acc[u][s][rt][3]);
      }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing DMAs land before the workgroup ends
  double Td[2][R8_S];
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int s = 0; s < R8_S; ++s) {
      Td[u][s] = (double)T[u][s];
      Td[u][s] += __shfl_xor(Td[u][s], 16);
      Td[u][s] += __shfl_xor(Td[u][s], 32);
    }
  if (g) return;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!valid[u]) continue;
    if (nseg > 1) {
#pragma unroll
      for (int s = 0; s < R8_S; ++s) tpart[((int64_t)seg * R8_S + s) * np + p[u]] = Td[u][s];
      continue;
    }
    double sum = 0.0;
#pragma unroll
    for (int s = R8_S - 1; s >= 0; --s) sum = sum * (1.0 / 128.0) + Td[u][s];
    varw[p[u]] = unit * sum;
  }
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
    for (int s2 = 0; s2 < R8_S; ++s2) acc[s2][0] = acc[s2][1] = zv;  // (as refine8_kernel)
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
#pragma unroll
        for (int s2 = 0; s2 < R8_S; ++s2)
#pragma unroll
          for (int rt = 0; rt < 2; ++rt) {
            const v4i fa = *(const v4i *)(tb + s2 * R8_TB + (rt * 16 + c) * 64 + swz);
            acc[s2][rt] = __builtin_amdgcn_mfma_i32_16x16x64_i8(fa, wf[kc], acc[s2][rt], 0, 0, 0);
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

// The O(n) terms of e'Pe in fp64 (refine8_kernel's expansion) and eff = e'Py from the reference
// codes; one wave per pair, lanes over individuals, lane partials added in a fixed tree.  Round 5: it
// runs on a second stream beside refine8_kernel (whose 2 waves per SIMD leave room for a third) and
// stores its terms; refine8_fin_kernel adds them to w'P_off w in the order one kernel used (same bits).
__global__ __launch_bounds__(256) void refine8_side_kernel(int64_t n_pad, const int8_t *__restrict__ sl,
                                                           const int8_t *__restrict__ sr, const double *__restrict__ Ua,
                                                           const double *__restrict__ Ub, const double *__restrict__ z,
                                                           const double *__restrict__ dg, const double *__restrict__ py,
                                                           const int8_t *__restrict__ lp, const int8_t *__restrict__ rp,
                                                           const double *soff_l, const double *soff_r, const double *off_l,
                                                           const double *off_r, const double *qa, const double *ra,
                                                           const double *qb, const double *rb, double zz,
                                                           const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                           int64_t np, double *__restrict__ terms) {
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
  const double tv[R8_NT] = {s1, s2, s3, ef};
#pragma unroll
  for (int k = 0; k < R8_NT; ++k) terms[(int64_t)k * np + p] = tv[k];
}

// var = w'P_off w + the O(n) terms (refine8_side_kernel's, added in its former order), chi, p
__global__ __launch_bounds__(256) void refine8_fin_kernel(int64_t np, const double *__restrict__ terms,
                                                          const double *soff_l, const double *soff_r, const double *qa,
                                                          const double *ra, const double *qb, const double *rb, double zz,
                                                          const uint8_t *mono_l, const uint8_t *mono_r,
                                                          const int64_t *__restrict__ pi, const int64_t *__restrict__ pj,
                                                          const double *varw, int nseg, const double *tpart, double unit,
                                                          double *eff, double *var, double *chi, double *pv) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= np) return;
  const int64_t i = pi[p], j = pj[p];
  const double al = soff_l[i], be = soff_r[j], ab = al * be;
  const double s1 = terms[p], s2 = terms[np + p], s3 = terms[2 * np + p], ef = terms[3 * np + p];
  // (the expressions of the single kernel, so that the compiler forms the same products and sums)
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
    for (int r = 0; r < MX_RB; ++r) acc[r] = zv;  // the row block's first tile is cs = nK - 1 (as refine8_kernel)
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
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const v4i wb = wf[2 * cs + kk];
          const v8i_ fb = {wb[0], wb[1], wb[2], wb[3], 0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < MX_RB; ++r) {
            const uint8_t *ar = tb + (2 * kk + h) * 4096 + (32 * r + c) * 32;
            const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
            const v8i_ fa = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            acc[r] = mfma_mx(fa, fb, acc[r], hi[2], bs);
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
// pair) partial sums go to mpart (pair_test_kernel adds them).  The LDS-resident pair_mx_kernel (removed in round 5) it
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
    for (int r = 0; r < MX_RB; ++r) acc[r] = zv;  // (as pair_mxr_kernel)
#pragma unroll
    for (int cl = PXR_NK - 1; cl >= 0; --cl) {
      if (C0 + cl < C1 && C0 + cl >= lo) {
        vm_wait_barrier(2 * min(LA - 1, N - 1 - v));  // tile v has landed (younger DMAs may be in flight)
        issue_next();
        const uint8_t *tb = sA[v % NSL];
        const int bs = C0 + cl == kb ? 128 : 129;  // off-diagonal tiles count twice
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const v4i wb = wf[2 * cl + kk];
          const v8i_ fb = {wb[0], wb[1], wb[2], wb[3], 0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < MX_RB; ++r) {
            const uint8_t *ar = tb + (2 * kk + h) * 4096 + (32 * r + c) * 32;
            const v4i lo4 = *(const v4i *)(ar + sw16), hi4 = *(const v4i *)(ar + (16 - sw16));
            const v8i_ fa = {lo4[0], lo4[1], lo4[2], lo4[3], hi4[0], hi4[1], hi4[2], hi4[3]};
            acc[r] = mfma_mx(fa, fb, acc[r], hi4[2], bs);
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

// (i, j) of every pair of rows[r] (j > i for the triangular kinds, every j for AD; j >= col_lo), row r's
// pairs starting at offs[r]
__global__ void all_pairs_kernel(const int64_t *__restrict__ rows, const int64_t *__restrict__ offs, int64_t m, int tri,
                                 int64_t col_lo, int64_t *__restrict__ pi, int64_t *__restrict__ pj) {
  const int r = blockIdx.y;
  const int64_t i = rows[r], j0 = tri ? max(i + 1, col_lo) : col_lo, cnt = m - j0, base = offs[r];
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

// The flush of a screened scan, on stream st, of candidates [lo, hi): the pair screen (use_ps) of
// [ps_done, hi) (those in [lo, ps_done) were pair-screened into cand2 beside the launches), the exact
// fp64 refine of the survivors, and the hits p < p_cut appended to the plan's lists.  Candidates
// below hi are free afterwards.
// [i | j | eff | var | chi | p] of n refined candidates in one buffer (one read-back copy)
// the refined candidates with p < p_cut (NaN never passes, as in the reference's res[res[4] < p_cut]) as
// 48-byte records (i, j, eff, var, chi, p) in any order (the caller sorts by (i, j)); one atomic per wave
__global__ void hit_pack_kernel(int64_t n, const int64_t *ci, const int64_t *cj, const double *eff, const double *var,
                                const double *chi, const double *p, double p_cut, double *out,
                                unsigned long long *count) {
  const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool hit = k < n && p[k] < p_cut;
  const unsigned long long bal = __ballot(hit);
  if (!bal) return;
  unsigned long long base = 0;
  if ((threadIdx.x & 63) == __builtin_ctzll(bal)) base = atomicAdd(count, (unsigned long long)__popcll(bal));
  base = __shfl(base, __builtin_ctzll(bal));
  if (!hit) return;
  const unsigned long long r = base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
  double *o = out + r * 6;
  ((int64_t *)o)[0] = ci[k];
  ((int64_t *)o)[1] = cj[k];
  o[2] = eff[k];
  o[3] = var[k];
  o[4] = chi[k];
  o[5] = p[k];
}



}  // namespace epi
}  // namespace gmat

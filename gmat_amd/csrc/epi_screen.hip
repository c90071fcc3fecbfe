// Screens of the scans: int8 slices, fp6 x fp4 quadratic form, low-rank spectral screens, tile / slot lists (see epi.h for the stage files).
#include "epi.h"

namespace gmat {
namespace epi {

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

template <int NSL>
__global__ __launch_bounds__(512, 1) void lrc_screen_kernel(ScreenArgs a, LrcArgs x) {
  constexpr int T = 512, RB = MX_RB, PB = 2, NA = MX_TILE / 16 / T, LA = NSL - 1;
  constexpr int LRC_JB = LRC_J2B, NJ = LRC_JB / 16;  // j-side bytes per column and stage; DMAs per wave
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
  unsigned oJ[NJ];
#pragma unroll
  for (int u = 0; u < NJ; ++u) {
    const int item = 64 * u + lane;
    const int t = item >> 6, col = (item >> 1) & 31;
    const int pc = item & 1, sw = (col >> 3) & 1;
    const int rr = t ? rr1 : rr0;
    const int jj = rr >= 0 ? x.slot_j[(sbase + PB * w + t) * 32 + col] : -1;
    oJ[u] = (unsigned)((jj >= 0 ? jj : 0) * nK * LRC_JB + (pc ^ sw) * 16);
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
      lds_dma16(x.s1c2 + kc * LRC_JB + oJ[u], &sJ[nb][w * NJ * 1024 + u * 1024]);
    if (w < 2) lds_dma16(x.nib_i + oI + kc * NB_REC, &sI[nb][w * 1024]);
  };
  const int NL = NA + NJ + (w < 2 ? 1 : 0);  // this wave's DMAs per stage
  v16f_ acc[RB][PB];
  const int sw16 = 16 * ((c >> 3) & 1), jf = (c >> 3) & 1;
  auto afrag = [&](int b, int kk, int r) __attribute__((always_inline)) {
    const uint8_t *ar = &sA[b][(2 * kk + h) * 4096 + (32 * r + c) * 32];
    const v4i lo = *(const v4i *)(ar + sw16), hi = *(const v4i *)(ar + (16 - sw16));
    return v8i_{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  };
  // the accumulators are zeroed at each chunk's start (a branch taken once per nK stages: selecting a zero
  // C operand for a chunk's first stage compiled to 128 v_cndmask in EVERY stage)
  auto zero_acc = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int t = 0; t < PB; ++t)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[r][t][e] = 0.f;
  };
  auto compute = [&](int b) __attribute__((always_inline)) {
    v8i_ fa = afrag(b, 0, 0);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      v8i_ fb[PB];
#pragma unroll
      for (int t = 0; t < PB; ++t) {
        // logical 8-byte piece 2 kk + h of the column: chunk kk (swizzled), half h; expanded to the
        // nibble plane's four dwords (piece = D0 | D1 << 2, D2 | D3 << 2)
        const v2i_ e2 = *(const v2i_ *)&sJ[b][(PB * w + t) * 32 * LRC_JB + c * LRC_JB + 16 * (kk ^ jf) + 8 * h];
        const v4i j1 = {e2[0] & 0x33333333, (e2[0] >> 2) & 0x33333333, e2[1] & 0x33333333, (e2[1] >> 2) & 0x33333333};
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
          acc[r][t] = mfma_mx(fa, fb[t], acc[r][t], fa[6], 128);
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
  zero_acc();
  vm_wait_barrier(NL * (min(LA, P) - 1));
  for (int q = 0; q < P; ++q) {
    if (q + LA < P) load((q + LA) % NSL, q + LA);  // its slot was read in stage q - 1 (barrier passed)
    const int kc = q % nK;
    compute(q % NSL);
    if (kc == nK - 1) {
      epilogue(q / nK);
      zero_acc();
    }
    const int ahead = min(q + LA, P - 1) - (q + 1);  // stages issued beyond q + 1
    vm_wait_barrier(q + 1 < P ? NL * ahead : 0);
  }
  // lane half h tests slot PB w + h, column c (the other half-wave's rows of the same column added)
  const double tot = (h ? lowrank[1] : lowrank[0]) + __shfl_xor(h ? lowrank[0] : lowrank[1], 32);
  const int ri = h ? rr1 : rr0;
  const int64_t i = h ? i1 : i0, j = h ? jc[1] : jc[0];
  const bool cand = ri >= 0 && j >= 0 && lrc_cand(a, x, (int64_t)(sbase + PB * w + h) * 32 + c, i, j, tot);
  // the wave's candidates with one atomic, slot 0's then slot 1's in column order (a slot's candidates
  // -- one first SNP -- stay adjacent for the pair screen)
  const unsigned long long bal = __ballot(cand);
  if (bal) {
    unsigned long long base = 0;
    if (lane == 0) base = atomicAdd(a.counter, (unsigned long long)__popcll(bal));
    base = ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((int)(base >> 32)) << 32) |
           (unsigned)__builtin_amdgcn_readfirstlane((int)base);
    if (cand) {
      const unsigned long long k =
          base + __builtin_amdgcn_mbcnt_hi((unsigned)(bal >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bal, 0u));
      if ((int64_t)k < a.cap) {
        a.cand_i[k] = i;
        a.cand_j[k] = j;
      }
    }
  }
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

// The slot lists of a launch (the compacted low-rank screen's input) from the prefilter's tagged live-block
// entries: lc_count (live pairs per band row), lc_scan (slots per row -> the rows' first slots), lc_fill
// (each row's live second SNPs in ascending order into its slots, with their records).  One wave per row,
// LC_T / 64 rows per workgroup: the row's entries are read 64 at a time (coalesced) and placed with a
// wave shuffle scan (round 5: a workgroup per row, contiguous per-thread ranges and a 16-barrier LDS scan).
__global__ __launch_bounds__(LC_T) void lc_count_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ, int Rn,
                                                        int *__restrict__ cnt) {
  const int r = (int)blockIdx.x * (LC_T / 64) + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= Rn) return;
  const uint64_t *mk = lmask + (int64_t)r * nJ;
  int c = 0;
  for (int J = lane; J < nJ; J += 64) c += __popc(lm_mask(mk[J], tag));
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) cnt[r] = c;
}

// wave-inclusive prefix sum of v over the 64 lanes
__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o);
    if (lane >= o) v += y;
  }
  return v;
}

// one workgroup: exclusive scan of the rows' slot counts (soff), info = {slots, tiles}, the padding
// slots of the last tile; 1,024 rows per pass (coalesced), wave shuffle scans and one LDS step
__global__ __launch_bounds__(1024) void lc_scan_kernel(const int *__restrict__ cnt, int Rn, int *__restrict__ soff,
                                                       int *__restrict__ info, int *__restrict__ slot_row,
                                                       int64_t slot_cap) {
  __shared__ int wsum[2][16];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  int run = 0, par = 0;  // slots of the passes before (uniform)
  for (int base = 0; base < Rn; base += 1024, par ^= 1) {
    const int r = base + t;
    const int sl = r < Rn ? (cnt[r] + 31) / 32 : 0;
    const int inc = wave_incl_scan(sl, lane);
    if (lane == 63) wsum[par][wv] = inc;
    __syncthreads();  // (the two buffers: a pass's totals are not overwritten while the previous one reads)
    int wpre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int v = wsum[par][k];
      wpre += k < wv ? v : 0;
      tot += v;
    }
    if (r < Rn) soff[r] = run + wpre + inc - sl;
    run += tot;
  }
  const int slots = run, tiles = (slots + LC_SLOTS - 1) / LC_SLOTS;
  if (t == 0) {
    info[0] = slots;
    info[1] = tiles;
  }
  const int q = slots + t;
  if (q < tiles * LC_SLOTS && q < slot_cap) slot_row[q] = -1;
}

// lc_fill: band row r's live second SNPs in ascending order into its slots, and each live pair's record
// (the prefilter's, at its block's first record + its rank in the block) copied to its slot position in
// slot_ops.  One wave per row: 64 entries per step, the next step's entries loaded ahead.
__global__ __launch_bounds__(LC_T) void lc_fill_kernel(const uint64_t *__restrict__ lmask, unsigned tag, int nJ, int Rn,
                                                       const int *__restrict__ cnt, const int *__restrict__ soff,
                                                       int *__restrict__ slot_row, int *__restrict__ slot_j,
                                                       const int *__restrict__ ops, int64_t ops_cap,
                                                       int *__restrict__ slot_ops, int64_t slot_cap) {
  const int r = (int)blockIdx.x * (LC_T / 64) + (int)(threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (r >= Rn) return;
  const uint64_t *mk = lmask + (int64_t)r * nJ;
  const int base = soff[r] * 32, n_live = cnt[r], n_slots = (n_live + 31) / 32;
  if ((int64_t)soff[r] + n_slots > slot_cap) return;  // records overflowed: the host reruns the launch
  int k0 = 0;  // pairs placed by the earlier steps
  uint64_t nxt = lane < nJ ? mk[lane] : 0ull;
  for (int J0 = 0; J0 < nJ; J0 += 64) {
    const uint64_t ent = nxt;
    nxt = J0 + 64 + lane < nJ ? mk[J0 + 64 + lane] : 0ull;
    uint32_t w = lm_mask(ent, tag);
    const int c = __popc(w);
    const int inc = wave_incl_scan(c, lane);
    int k = k0 + inc - c;
    uint32_t src = lm_base(ent);
    const int J = J0 + lane;
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
    k0 += __shfl(inc, 63);
  }
  for (int q = n_live + lane; q < n_slots * 32; q += 64) slot_j[base + q] = -1;
  for (int q = lane; q < n_slots; q += 64) slot_row[soff[r] + q] = r;
}

// the instantiations the host code launches
template __global__ void screen_kernel<SCREEN_SHAPE>(ScreenArgs);
template __global__ void mx_screen_kernel<1>(ScreenArgs, MxArgs);
template __global__ void lr_screen_kernel<1, 2>(ScreenArgs, LrArgs);
template __global__ void lr_screen_kernel<2, 2>(ScreenArgs, LrArgs);
template __global__ void lrc_screen_kernel<3>(ScreenArgs, LrcArgs);

}  // namespace epi
}  // namespace gmat

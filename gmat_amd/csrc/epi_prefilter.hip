// Spectral prefilter of the screened scans (see epi.h for the stage files).
#include "epi.h"

namespace gmat {
namespace epi {

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

// COMPACT: the compacted low-rank path's output (live masks + one record per live pair at a.ops); else
// the block-granular path's (flags + E3 and code products of every pair of a live block, dense)
// TR = 64: 64 x 256 tiles, 8 waves (2 row x 4 column waves), one workgroup per CU; TR = 32: 32 x 256
// tiles, 4 waves (1 x 4), two workgroups per CU (each SIMD then holds one wave of each of two
// independent workgroups, whose stage barriers and epilogues fall at different times)
template <bool LIST, bool COMPACT, bool STAMP, int TR, int NS>
__global__ __launch_bounds__(TR * 8, TR == 64 ? 1 : 2) void prefilter_pass_kernel(SideArgs x) {
  static_assert(NS == 5 || NS == 6, "prefilter ring depth");
  static_assert(TR == 64 || TR == 32, "prefilter tile rows");
  constexpr int NW = TR / 8;  // waves
  // stage image: int8 L3 slices 0, 1 (TR rows x 64 B each), the rows' 2-bit codes (TR x 16 B, in a
  // whole 1 KB DMA), the columns' 2-bit codes (256 x 16 B)
  constexpr int O_R8 = 0, O_R8S = TR * 64, O_R4 = 2 * TR * 64, O_C4 = O_R4 + 1024, ST = O_C4 + PF_TC * 16;
  static_assert(TR != 64 || (ST == PF_ST && O_C4 == 9216), "prefilter stage image");
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
    const int tr0 = (t % x.n_rt) * TR;
    const int64_t tc0 = (a.j_lo / 32) * 32 + (int64_t)(t / x.n_rt) * PF_TC;
    if (tr0 >= a.n_rows || tc0 >= a.m) return -1;
    if (a.tri && tc0 + PF_TC - 1 <= a.rows[tr0]) return -1;  // rows ascend within a launch
    return t;
  };
  int it = 0, tile = tile_at(0);
  if (tile < 0) return;
  int r0 = (tile % x.n_rt) * TR;
  int64_t c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * PF_TC;
  auto pstamp = [&](int k) __attribute__((always_inline)) {  // the workgroup's first tile only
    if (STAMP && a.pf_stamp && threadIdx.x == 0) {
      a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + k] = __builtin_amdgcn_s_memrealtime();
      if (k == 0 || k == PF_NPHASE - 1)
        a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + PF_NPHASE + (k ? 1 : 0)] = __builtin_amdgcn_s_memtime();
    }
  };
  pstamp(0);
  // wave w = rows 32 (w >> 2) .. +32 x columns 64 (w & 3) .. +64 (two 32-column blocks)
  const int tid = threadIdx.x, lane = tid & 63, h = lane >> 5, c = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6), wr = w >> 2, wc = w & 3;  // wave-uniform (SGPR)
  // stage DMAs of this wave: TR = 64: q = w, w + 8 (waves 0-4 two, 5-7 one; q 8 the rows' codes);
  // TR = 32: the L3 piece w, the columns 64 w .., and wave 0 the rows' codes
  const int nq = TR == 64 ? (w + 8 < PF_NQ ? 2 : 1) : (w == 0 ? 3 : 2);
  __shared__ __attribute__((aligned(16))) uint8_t ring[NS][ST];
  // stage-blocked panels: a stage's 64-byte / 16-byte pieces of consecutive SNPs are contiguous, so
  // an instruction's 1 KB comes from 8 whole 128-byte lines (int8 pieces in the even / odd
  // individual order of i8x2_of_fp4_eo).  Sources: a wave-uniform base per instruction (the panel's
  // stage st, SGPRs) + a 32-bit lane offset
  constexpr int64_t rstride = SG_K, cstride = SG_K / 4;
  constexpr int RQ = TR / 16;                                      // L3 DMAs per slice
  const uint8_t *sbase0 = (const uint8_t *)x.rs[w / RQ];           // q = w: L3 slice w / RQ
  const uint8_t *sbase1 = (TR == 64 && w == 0) ? x.rs2 : x.cs2;    // TR = 64, q = w + 8: codes
  const int64_t sstep0 = a.m * SG_K, sstep1 = a.m * cstride;
  unsigned voff[3];
  auto set_src = [&](int r0, int64_t c0) __attribute__((always_inline)) {
    {  // int8 L3 slices: 16 rows x 4 chunks per instruction
      const int row = (w % RQ) * 16 + (lane >> 2), lg = (lane & 3) ^ ((row >> 2) & 3);
      voff[0] = (unsigned)(a.rows[min(r0 + row, a.n_rows - 1)] * rstride + 16 * lg);
    }
    if (TR == 64) {
      if (w == 0)  // q 8: 2-bit codes of the 64 rows, one per lane
        voff[1] = (unsigned)(a.rows[min(r0 + lane, a.n_rows - 1)] * cstride);
      else  // q 9..12: 2-bit codes of 64 columns per instruction
        voff[1] = (unsigned)(min(c0 + 64 * (w - 1) + lane, a.m - 1) * cstride);
    } else {
      voff[1] = (unsigned)(min(c0 + 64 * w + lane, a.m - 1) * cstride);
      if (w == 0)  // the 32 rows' codes, twice (lanes 32-63 fill the unused half of the 1 KB)
        voff[2] = (unsigned)(a.rows[min(r0 + (lane & 31), a.n_rows - 1)] * cstride);
    }
  };
  set_src(r0, c0);
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_b = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]);
  const unsigned ring_m0 = ring_b + w * 1024;
  // stage st into ring slot `slot` (= st % NS, kept by the caller)
  auto issue = [&](int st, int slot) __attribute__((always_inline)) {
    lds_dma16_sv(voff[0], sbase0 + st * sstep0, ring_m0 + slot * ST);
    if (TR == 64) {
      if (nq == 2) lds_dma16_sv(voff[1], sbase1 + st * sstep1, ring_m0 + slot * ST + 8 * 1024);
    } else {
      lds_dma16_sv(voff[1], x.cs2 + st * sstep1, ring_b + slot * ST + O_C4 + w * 1024);
      if (w == 0) lds_dma16_sv(voff[2], x.rs2 + st * sstep1, ring_b + slot * ST + O_R4);
    }
  };
  // wait until stage `st` has landed given the stages issued up to `last` (nq DMAs per stage), then
  // the workgroup barrier, in ONE asm statement: the compiler does not know that the DMA asm writes
  // LDS, and the barrier builtin is no memory fence, so a separate builtin would let it hoist the next
  // stage's ds_reads above the barrier.  The counted vmcnt assumes that VMEM operations retire in order
  // (they do on gfx9 for loads).  (The record DMAs are older than any stage.)
  // The steady state (NS - 2 stages younger than st in flight) tests one wave-uniform condition; the
  // generic chain of cases (a dozen scalar compares and branches per stage) only runs at a tile's end.
  static_assert(NS == 5, "wait_for's steady-state vmcnt values");
  auto wait_for = [&](int st, int last) __attribute__((always_inline)) {
    const int ahead = min(last - st, NS - 2);
    if (ahead == NS - 2) {
      if (nq == (TR == 64 ? 2 : 3)) {
        if (TR == 64)
          asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else {
        if (TR == 64)
          asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else
          asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      return;
    }
    switch (nq * ahead) {
      case 9: asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      case 6: asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory"); break;
    }
  };
  v16i acc[2][E3_PF];
  v16f_ acc4[2][4];  // per column block: a.b, a^2.b, a.b^2, a^2.b^2
  const int S = (int)(x.n_pad / SG_K);
  const int pre = min(S, NS - 1);
  // the epilogue's test records (32 B per row / column) by LDS-DMA ahead of the stages: wave w the
  // 32 columns 32 w .., waves 0 and 1 also the 32 rows 32 w ..; lane l half l & 1 of record l / 2.
  // They retire before stage 0 (in-order vmcnt), so the stage waits cover them.
  // Two record buffers: the next tile's land while the current tile's epilogue reads its own.
  __shared__ __attribute__((aligned(16))) float rec[2][TR + PF_TC][PF_REC];
  // COMPACT: per wave, lane (b, h)'s live-column mask and first record (the epilogue's store table)
  __shared__ uint2 ptab[COMPACT ? NW : 1][64];
  auto issue_rec = [&](int r0, int64_t c0, int rb) __attribute__((always_inline)) {
    const int k = 32 * w + (lane >> 1);
    if (w < TR / 32)
      lds_dma16(x.recL + a.rows[min(r0 + k, a.n_rows - 1)] * PF_REC + 4 * (lane & 1), &rec[rb][32 * w][0]);
#pragma unroll
    for (int u = 0; u < PF_TC / 32 / NW; ++u) {  // wave w: the columns 32 (w + NW u) ..
      const int kc = 32 * (w + NW * u) + (lane >> 1);
      lds_dma16(x.recR + min(c0 + kc, a.m - 1) * PF_REC + 4 * (lane & 1), &rec[rb][TR + 32 * (w + NW * u)][0]);
    }
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
    // the main loop at issue priority 1, the epilogue at 0: on a SIMD, one workgroup's MFMA stages take the
    // issue slots before the other workgroup's epilogue VALU work (round 6: 1,347 -> 1,322 us per launch
    // serialised, 1.446 -> 1.385 ms in the configs[2] step, step time unchanged)
    if (TR == 32) __builtin_amdgcn_s_setprio(1);
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
    int slot = 0, slot_ahead = NS - 1;  // ring slots of stage st and of stage st + NS - 1
    for (int st = 0; st < S; ++st) {
      const uint8_t *bf = ring[slot];
      // slot (st + 4) % 5 was read in stage st - 1, which every wave has left (barrier)
      if (st + NS - 1 < S) issue(st + NS - 1, slot_ahead);
      slot = slot == NS - 1 ? 0 : slot + 1;
      slot_ahead = slot_ahead == NS - 1 ? 0 : slot_ahead + 1;
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
      wait_for(st + 1, min(st + NS - 1, S - 1));
    }
    pstamp(2);
    if (TR == 32) __builtin_amdgcn_s_setprio(0);
    // every wave has passed the last stage's barrier (its vmcnt(0) wait): the ring is free, so the
    // next tile's records and first stages go out now and land while this tile's epilogue runs
    const int nxt = tile_at(it + 1);
    if (nxt >= 0) {
      const int nr0 = (nxt % x.n_rt) * TR;
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
      const float4 cv0 = rv[2 * (TR + cl)], cv1 = rv[2 * (TR + cl) + 1];
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
        if (COMPACT) {  // this lane's pair is live (the masks come from one bit transpose below)
          st_bits |= (lv ? 1u : 0u) << (2 * e + q);
        } else {
          const unsigned long long bal = __ballot(lv);
          n_live += (unsigned)__popcll(bal);
          const unsigned w0 = (unsigned)bal, w1 = (unsigned)(bal >> 32);
          mine[q] = te == e ? (th ? w1 : w0) : mine[q];
          // a live block (its row r < n_rows: some lane of the half passed rok) whose column this lane holds
          st_bits |= ((((h ? w1 : w0) != 0u) & cok[q]) ? 1u : 0u) << (2 * e + q);
        }
      }
    }
    pstamp(4);
    if (COMPACT) {
      // One record per live pair.  Lane (c, h) holds bit b = 2 e + q of st_bits for column c of element
      // (e, q); a 32 x 32 bit transpose inside each half-wave (five xor-shuffle rounds) gives lane (b, h)
      // the live-column mask W of element b's row in half h -- the (row, 32-column block) entry -- in ~25
      // VALU, where a ballot per element cost ~50 instructions per element (round 4's store phase took
      // ~5 us of a tile's ~11 us epilogue).  The entries' records are numbered in lane order by a prefix
      // sum of popc(W) (a block's pairs consecutive, ascending j, as lc_fill reads them), the wave
      // reserves them with one atomic per PF_CHUNK or more, each lane writes its entry, and each live pair
      // its record at entry base + rank of its column in W (base and W of the lane's elements read back
      // from a per-wave LDS table; elements without a live pair in the wave are skipped by a scalar test).
      unsigned wv = st_bits;
      constexpr unsigned TMASK[5] = {0x0000FFFFu, 0x00FF00FFu, 0x0F0F0F0Fu, 0x33333333u, 0x55555555u};
#pragma unroll
      for (int rd = 0; rd < 5; ++rd) {
        const int s2 = 16 >> rd;
        const unsigned ml = TMASK[rd];
        const unsigned y = (unsigned)__shfl_xor((int)wv, s2);
        wv = (c & s2) ? ((wv & ~ml) | ((y >> s2) & ml)) : ((wv & ml) | ((y & ml) << s2));
      }
      // lane (b, h): element b = 2 e + q, row 32 wr + kr(e) + 4 h, 32-column block J
      const int eb = c >> 1, qb = c & 1;
      const int trr = r0 + 32 * wr + (eb & 3) + 8 * (eb >> 2) + 4 * h;
      const int Jb = (int)((c0 + 64 * wc + 32 * qb) / 32);
      const unsigned cnt = (unsigned)__popc(wv);
      unsigned incl = cnt;  // inclusive prefix sum over the 64 lanes
#pragma unroll
      for (int rd = 0; rd < 6; ++rd) {
        const int s2 = 1 << rd;
        const unsigned y = (unsigned)__shfl_up((int)incl, s2);
        incl += lane >= s2 ? y : 0u;
      }
      n_live = (unsigned)__builtin_amdgcn_readlane((int)incl, 63);
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
      const unsigned ebase = base + incl - cnt;  // the first record of lane (b, h)'s entry
      if (wv && trr < a.n_rows && Jb < a.nJ) a.lmask[(int64_t)trr * a.nJ + Jb] = lm_entry(wv, ebase, a.ltag);
      const bool fits = (int64_t)base + n_live <= a.ops_cap;
      // elements with a live pair anywhere in the wave (bit b: either half)
      const unsigned long long anyb = __ballot(wv != 0u);
      const unsigned elem_any = (unsigned)anyb | (unsigned)(anyb >> 32);
      if (n_live) {
        ptab[w][lane] = make_uint2(wv, ebase);
        __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's table writes are visible to its reads
        __builtin_amdgcn_wave_barrier();
      }
      int *const ops = a.ops;
      const unsigned below = (1u << c) - 1u;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int b = 2 * e + q;
          if ((elem_any >> b) & 1u) {  // wave-uniform
            if (((st_bits >> b) & 1u) && fits) {
              const uint2 t = ptab[w][32 * h + b];
              const unsigned k = t.y + (unsigned)__popc(t.x & below);
              v4i r0v = {acc[q][0][e] >> 1, acc[q][1][e] >> 1, (int)acc4[q][0][e], (int)acc4[q][1][e]};  // exact
              v4i r1v = {(int)acc4[q][2][e], (int)acc4[q][3][e], jq[q], 0};
              *(v4i *)(ops + (int64_t)k * OPS_REC) = r0v;
              *(v4i *)(ops + (int64_t)k * OPS_REC + 4) = r1v;
            }
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
    if (STAMP && a.pf_stamp) __syncthreads();  // the phase stamps time the slowest wave
    pstamp(6);
    if (nxt < 0) break;
    r0 = (nxt % x.n_rt) * TR;
    c0 = (a.j_lo / 32) * 32 + (int64_t)(nxt / x.n_rt) * PF_TC;
    set_src(r0, c0);  // again: the source addresses stay out of the epilogue's registers
  }
}

// LIST: a persistent grid over the launch's tile list (as prefilter_pass_kernel<true>: XCD x takes the
// list's x-th eighth, its workgroups stride through it, and the next tile's first stages stream into
// the ring while this tile's epilogue runs); else one workgroup per tile of the XCD-aware remap.
template <int NC, bool LIST, int TC>
__global__ __launch_bounds__(TC * 2, TC == PC_TC ? 1 : 2) void prefilter_cov_kernel(SideArgs x) {
  static_assert(TC == 256 || TC == 128, "covariate prefilter tile columns");
  using SH = PcShape<NC, TC>;
  constexpr int NW = TC / 32, NS = SH::NS, NCQ = 5 + TC / 64;  // waves, ring slots, first q-slice DMA
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
    const int64_t c0_ = (a.j_lo / 32) * 32 + (int64_t)(t / x.n_rt) * TC;
    if (r0_ >= a.n_rows || c0_ >= a.m) return -1;
    if (a.tri && c0_ + TC - 1 <= a.rows[r0_]) return -1;  // rows ascend within a launch
    return t;
  };
  auto pstamp = [&](int st_) __attribute__((always_inline)) {  // GMAT_PF_STAMPS (one tile per workgroup)
    if (!LIST && a.pf_stamp && threadIdx.x == 0) {
      a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + st_] = __builtin_amdgcn_s_memrealtime();
      if (st_ == 0 || st_ == PF_NPHASE - 1)
        a.pf_stamp[PF_NSTAMP * (int64_t)blockIdx.x + PF_NPHASE + (st_ ? 1 : 0)] = __builtin_amdgcn_s_memtime();
    }
  };
  pstamp(0);
  int tile = tile_at(0);
  if (tile < 0) return;
  // NW waves (two per SIMD: one workgroup of 8 or two of 4): wave w = the tile's 32 rows x columns 32 w .. +32
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), h = lane >> 5,
            c = lane & 31;
  __shared__ __attribute__((aligned(16))) uint8_t ring[NS][SH::ST];
  __shared__ __attribute__((aligned(16))) uint8_t img[2][NC][2048];  // direction images, stages s % 2
  // DMA instruction q = w + NW u (u < 2): a wave-uniform base per instruction (the panel at stage st,
  // SGPRs) + a 32-bit lane offset
  const int nq = (w + NW < SH::QT) ? 2 : 1;  // DMA instructions this wave issues per stage
  auto base_of = [&](int q) __attribute__((always_inline)) -> const uint8_t * {
    return q < 4 ? (const uint8_t *)x.rs[q >> 1] : q == 4 ? x.rs2 : q < NCQ ? x.cs2 : x.qimg;
  };
  auto step_of = [&](int q) __attribute__((always_inline)) -> int64_t {
    return q < 4 ? (int64_t)SG_K * a.m : q < NCQ ? (int64_t)(SG_K / 4) * a.m : (int64_t)SG_K;
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
      } else if (q < NCQ) {  // 2-bit codes of 64 columns per instruction
        voff[u] = (unsigned)(min(c0 + 64 * (q - 5) + lane, a.m - 1) * (SG_K / 4));
      } else {  // the q slices: lane l = direction min(l / 4, NC - 1), chunk l % 4
        voff[u] = (unsigned)(min(lane >> 2, NC - 1) * x.n_pad + 16 * (lane & 3));
      }
    }
  };
  typedef __attribute__((address_space(3))) const void *lds_ct;
  const unsigned ring_m0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_ct)&ring[0][0]) + w * 1024;
  auto issue = [&](int st) __attribute__((always_inline)) {
    const unsigned m0 = ring_m0 + (st % NS) * SH::ST;
    lds_dma16_sv(voff[0], sbase0 + st * sstep0, m0);
    if (nq == 2) lds_dma16_sv(voff[1], sbase1 + st * sstep1, m0 + NW * 1024);
  };
  // the direction images of stage st (its codes and q slices have landed): thread t < 128 NC forms
  // direction t / 128, row (t / 4) % 32, 16-individual chunk t % 4
  auto image = [&](int st) __attribute__((always_inline)) {
#pragma unroll
    for (int t = tid; t < 128 * NC; t += 64 * NW) {
      uint8_t *sl = ring[st % NS];
      const int k = t >> 7, row = (t >> 2) & 31, ch = t & 3;
      const unsigned cw = *(const unsigned *)(sl + SH::O_A2 + row * 16 + 4 * ch);  // 16 individuals, 2 bits each
      const v4i qv = *(const v4i *)(sl + SH::O_Q + 64 * k + 16 * ch);
      *(v4i *)(&img[st & 1][k][row * 64 + 16 * (ch ^ ((row >> 2) & 3))]) =
          aq_of_fp4_eo((cw << 1) & 0x66666666u, (cw >> 1) & 0x66666666u, qv);
    }
  };
  const int S = (int)(x.n_pad / SG_K);
  const int pre = min(S, NS - 1);
  int r0 = (tile % x.n_rt) * PC_TR;
  int64_t c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * TC;
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
    const uint8_t *bf = ring[st % NS];
    if (st + NS - 1 < S) issue(st + NS - 1);
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
    vm_wait_barrier(nq * max(0, min(st + NS - 1, S - 1) - (st + 2)));
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
    set_src((nxt % x.n_rt) * PC_TR, (a.j_lo / 32) * 32 + (int64_t)(nxt / x.n_rt) * TC);
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
  c0 = (a.j_lo / 32) * 32 + (int64_t)(tile / x.n_rt) * TC;
  }  // tile loop
}

// the instantiations the host code launches
template __global__ void side_gemm_kernel<2>(SideArgs);
template __global__ void side_gemm_kernel<3>(SideArgs);
template __global__ void side_gemm_kernel<4>(SideArgs);
template __global__ void prefilter_pass_kernel<false, false, false, 64, PF_NS>(SideArgs);
template __global__ void prefilter_pass_kernel<true, true, false, 32, 5>(SideArgs);
template __global__ void prefilter_pass_kernel<true, true, true, 32, 5>(SideArgs);
template __global__ void prefilter_cov_kernel<1, false, 256>(SideArgs);
template __global__ void prefilter_cov_kernel<2, false, 256>(SideArgs);
template __global__ void prefilter_cov_kernel<3, false, 256>(SideArgs);
template __global__ void prefilter_cov_kernel<4, false, 256>(SideArgs);
template __global__ void prefilter_cov_kernel<1, true, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<1, false, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<2, true, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<2, false, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<3, true, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<3, false, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<4, true, 128>(SideArgs);
template __global__ void prefilter_cov_kernel<4, false, 128>(SideArgs);

}  // namespace epi
}  // namespace gmat

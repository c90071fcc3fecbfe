// Stage timings of chol_step_kernel's D task (the per-step critical path): tile loads, the two 64^3
// products, the 64 x 64 factor + inverse.  One workgroup; wall_clock64 (100 MHz) between stages.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/chol_micro.hip -Lgmat_amd -lgmat_hip -o /tmp/chol_micro
__device__ long long g_stamp[8];
#define CHOL_STAMP(i) \
  if (threadIdx.x == 0) g_stamp[i] += wall_clock64();
// per-task (start, end) wall clock of chol_step_kernel: g_task[((k + 1) * MAXT + task) * 2]
__device__ long long *g_task;
constexpr int MAXT = 4096;
#define CHOL_TASK_BEGIN const long long t_begin_ = wall_clock64();
#define CHOL_TASK_END(task)                                                        \
  if (threadIdx.x == 0 && g_task && (task) < MAXT) {                               \
    g_task[((int64_t)(x.k + 1) * MAXT + (task)) * 2] = t_begin_;                   \
    g_task[((int64_t)(x.k + 1) * MAXT + (task)) * 2 + 1] = wall_clock64();         \
  }
#include "../gmat_amd/csrc/chol.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>

namespace gmat {
namespace {
__global__ __launch_bounds__(256) void micro_kernel(const double *a, const double *dinv, long long *t, int reps) {
  __shared__ double Ls[NB][NB + 1];
  __shared__ double Xs[NB][NB + 1];
  __shared__ double piv[NB];
  long long c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  v4d acc[2][2];
  double sink = 0.0;
  for (int r = 0; r < reps; ++r) {
    __syncthreads();
    long long t0 = wall_clock64();
    {
      TileRegs r0, r1;
      tile_load(r1, dinv, NB, 0, 0, NB, NB, false);
      tile_load(r0, a, NB, 0, 0, NB, NB, false);
      tile_to_lds(Xs, r1, false);
      tile_to_lds(Ls, r0, false);
    }
    __syncthreads();
    long long t1 = wall_clock64();
    acc_zero(acc);
    mm_abt(Ls, Xs, acc);
    __syncthreads();
    acc_to_lds(Ls, acc, false);
    __syncthreads();
    long long t2 = wall_clock64();
    acc_zero(acc);
    mm_abt(Ls, Ls, acc);
    __syncthreads();
    sink += acc[0][0][0];
    long long t3 = wall_clock64();
    {
      TileRegs r0;
      tile_load(r0, a, NB, 0, 0, NB, NB, true);
      tile_to_lds(Ls, r0, false);
    }
    for (int e = threadIdx.x; e < NB * NB; e += 256) Xs[e / NB][e % NB] = 0.0;
    __syncthreads();
    long long t4 = wall_clock64();
    if (threadIdx.x == 0) g_stamp[0] += t4;
    const bool bad = factor_invert_block(Ls, Xs, piv, NB);
    long long t5 = wall_clock64();
    sink += bad ? 1.0 : Xs[threadIdx.x & 63][0];
    c[0] += t1 - t0;
    c[1] += t2 - t1;
    c[2] += t3 - t2;
    c[3] += t4 - t3;
    c[4] += t5 - t4;
  }
  if (threadIdx.x == 0) {
    for (int i = 0; i < 5; ++i) t[i] = c[i];
    t[7] = (long long)sink;
  }
}
}  // namespace
}  // namespace gmat

// cholesky_steps at n (L^-1 and V^-1) with per-task timestamps: per launch the task count, the D task's
// duration, the other tasks' mean / max, the launch's span and the gap after the previous launch
static void steps_trace(int64_t n) {
  using namespace gmat;
  const int K = (int)((n + NB - 1) / NB);
  std::vector<double> h(n * n);
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j <= i; ++j) {
      const double v = (i == j) ? 4.0 + (double)(i % 7) : 1.0 / (double)(1 + ((i * 31 + j * 17) % 97));
      h[i * n + j] = h[j * n + i] = v;
    }
  double *a, *a0, *dinv, *linv, *vinv, *sm;
  hipMalloc(&a, n * n * 8);
  hipMalloc(&a0, n * n * 8);
  hipMalloc(&dinv, n * NB * 8);
  hipMalloc(&linv, n * n * 8);
  hipMalloc(&vinv, n * n * 8);
  hipMalloc(&sm, 16);
  long long *tr;
  const size_t trn = (size_t)(K + 3) * MAXT * 2;
  hipMalloc(&tr, trn * 8);
  hipMemcpy(a0, h.data(), n * n * 8, hipMemcpyHostToDevice);
  long long *null_ptr = nullptr;
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpyToSymbol(HIP_SYMBOL(g_task), rep == 2 ? &tr : &null_ptr, sizeof(tr));
    hipMemset(tr, 0, trn * 8);
    hipMemcpy(a, a0, n * n * 8, hipMemcpyDeviceToDevice);
    hipDeviceSynchronize();
    cholesky_steps(0, n, a, n, dinv, sm, (int *)(sm + 1), linv, false, vinv);
    hipDeviceSynchronize();
  }
  std::vector<long long> ht(trn);
  hipMemcpy(ht.data(), tr, trn * 8, hipMemcpyDeviceToHost);
  long long prev_end = 0, t_first = 0, t_last = 0;
  printf("n = %lld: launch  tasks  D_us  T_mean_us  T_max_us  span_us  gap_us\n", (long long)n);
  for (int L = 0; L < K + 3; ++L) {
    long long lo = 0, hi = 0, dsum = 0, dmax = 0, d0 = 0;
    int cnt = 0;
    for (int t = 0; t < MAXT; ++t) {
      const long long b = ht[((size_t)L * MAXT + t) * 2], e = ht[((size_t)L * MAXT + t) * 2 + 1];
      if (!b) continue;
      if (!cnt || b < lo) lo = b;
      if (!cnt || e > hi) hi = e;
      if (t == 0) d0 = e - b;
      else {
        dsum += e - b;
        dmax = std::max(dmax, e - b);
      }
      ++cnt;
    }
    if (!cnt) continue;
    if (!t_first) t_first = lo;
    t_last = hi;
    printf("  %3d %6d %7.2f %9.2f %9.2f %8.2f %7.2f\n", L - 1, cnt, d0 / 100.0, cnt > 1 ? dsum / 100.0 / (cnt - 1) : 0.0,
           dmax / 100.0, (hi - lo) / 100.0, prev_end ? (lo - prev_end) / 100.0 : 0.0);
    prev_end = hi;
  }
  printf("total %.1f us\n", (t_last - t_first) / 100.0);
}

int main(int argc, char **argv) {
  using namespace gmat;
  if (argc > 1) {
    steps_trace(atoll(argv[1]));
    return 0;
  }
  const int reps = 50;
  std::vector<double> h(NB * NB), hd(NB * NB, 0.0);
  for (int i = 0; i < NB; ++i)
    for (int j = 0; j < NB; ++j) h[i * NB + j] = (i == j ? NB : 0.0) + 1.0 / (1.0 + i + j);
  for (int i = 0; i < NB; ++i) hd[i * NB + i] = 0.5;
  double *a, *d;
  long long *t;
  hipMalloc(&a, NB * NB * 8);
  hipMalloc(&d, NB * NB * 8);
  hipMalloc(&t, 8 * 8);
  hipMemcpy(a, h.data(), NB * NB * 8, hipMemcpyHostToDevice);
  hipMemcpy(d, hd.data(), NB * NB * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(micro_kernel, dim3(1), dim3(256), 0, 0, a, d, t, 2);
  long long zero[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st[8];
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamp), zero, sizeof(zero));
  hipLaunchKernelGGL(micro_kernel, dim3(1), dim3(256), 0, 0, a, d, t, reps);
  long long ht[8];
  hipMemcpy(ht, t, 64, hipMemcpyDeviceToHost);
  hipMemcpyFromSymbol(st, HIP_SYMBOL(g_stamp), sizeof(st));
  const char *sn[5] = {"panel 0", "panel 1 (+X row 0)", "panel 2 (+X row 1)", "panel 3 (+X row 2)", "X row 3"};
  for (int i = 1; i < 6; ++i) printf("  %-22s %8.2f us\n", sn[i - 1], (st[i] - st[i - 1]) / (double)reps / 100.0);
  const char *names[5] = {"load 2 tiles", "product 1 + LDS store", "product 2", "load (factor input)", "factor+inverse"};
  for (int i = 0; i < 5; ++i) printf("%-24s %8.2f us\n", names[i], ht[i] / (double)reps / 100.0);
  return 0;
}

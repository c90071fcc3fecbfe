// MFMA probe for gfx950: verifies operand/accumulator lane maps of the
// int8 and fp64 MFMA forms used by the scan / GRM / REML kernels, and
// measures their sustained issue rate with every CU busy.
// Build: hipcc --offload-arch=gfx950 -O3 -o probe_mfma probe_mfma.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef double v4d __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

// ---- layout probes: A,B given row-major int8 [32][32]; hypothesis h picks
// the k of byte j in lane l.
__device__ int kmap32(int h, int l, int j) {
  if (h == 0) return 16 * (l >> 5) + j;                         // contiguous 16 per half
  return (j < 8) ? 8 * (l >> 5) + j : 16 + 8 * (l >> 5) + (j - 8);  // two 8-runs
}
__global__ void i8_32x32x32_probe(const int8_t *A, const int8_t *B, int *D, int h) {
  int l = threadIdx.x;
  union { v4i v; int8_t b[16]; } a, b;
  for (int j = 0; j < 16; ++j) {
    int k = kmap32(h, l, j);
    a.b[j] = A[(l & 31) * 32 + k];
    b.b[j] = B[k * 32 + (l & 31)];
  }
  v16i c = {0};
  c = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, b.v, c, 0, 0, 0);
  for (int r = 0; r < 16; ++r) {
    int row = (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
    D[row * 32 + (l & 31)] = c[r];
  }
}
__device__ int kmap16(int h, int l, int j) {
  if (h == 0) return 16 * (l >> 4) + j;
  return (j < 8) ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8);
}
__global__ void i8_16x16x64_probe(const int8_t *A, const int8_t *B, int *D, int h) {
  int l = threadIdx.x;
  union { v4i v; int8_t b[16]; } a, b;
  for (int j = 0; j < 16; ++j) {
    int k = kmap16(h, l, j);
    a.b[j] = A[(l & 15) * 64 + k];
    b.b[j] = B[k * 16 + (l & 15)];
  }
  v4i c = {0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, b.v, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) * 4 + r;
    D[row * 16 + (l & 15)] = c[r];
  }
}
__global__ void f64_16x16x4_probe(const double *A, const double *B, double *D) {
  int l = threadIdx.x;
  double a = A[(l & 15) * 4 + (l >> 4)];
  double b = B[(l >> 4) * 16 + (l & 15)];
  v4d c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) {
    int row = (l >> 4) + 4 * r;
    D[row * 16 + (l & 15)] = c[r];
  }
}

// ---- rate kernels: 4 independent accumulators, ITER back-to-back MFMAs.
template <int ITER>
__global__ void __launch_bounds__(256) rate_i8_32(int *out, int seed) {
  v4i a = {seed, seed + 1, seed + 2, seed + 3}, b = {seed ^ 5, seed ^ 7, seed ^ 9, seed ^ 11};
  v16i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < ITER; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_32x32x32_i8(b, b, c3, 0, 0, 0);
  }
  int s = 0;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 0x12345) out[0] = s;
}
template <int ITER>
__global__ void __launch_bounds__(256) rate_i8_16(int *out, int seed) {
  v4i a = {seed, seed + 1, seed + 2, seed + 3}, b = {seed ^ 5, seed ^ 7, seed ^ 9, seed ^ 11};
  v4i c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < ITER; ++i) {
    c0 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(b, b, c3, 0, 0, 0);
  }
  int s = 0;
  for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 0x12345) out[0] = s;
}
template <int ITER>
__global__ void __launch_bounds__(256) rate_f64(double *out, double seed) {
  double a = seed, b = seed * 0.5;
  v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  for (int i = 0; i < ITER; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
  }
  double s = 0;
  for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 12345.0) out[0] = s;
}
template <int ITER>
__global__ void __launch_bounds__(256) rate_fma64(double *out, double seed) {
  double x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3, x4 = seed + 4, x5 = seed + 5, x6 = seed + 6, x7 = seed + 7;
  double m = 0.999999, q = 1e-9;
  for (int i = 0; i < ITER; ++i) {
    x0 = fma(x0, m, q); x1 = fma(x1, m, q); x2 = fma(x2, m, q); x3 = fma(x3, m, q);
    x4 = fma(x4, m, q); x5 = fma(x5, m, q); x6 = fma(x6, m, q); x7 = fma(x7, m, q);
  }
  double s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  if (s == 12345.0) out[0] = s;
}

template <typename K>
double time_kernel(K k, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k(blocks);  // warm
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k(blocks);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  srand(1);
  // i8 32x32x32
  {
    std::vector<int8_t> A(32 * 32), B(32 * 32);
    for (auto &x : A) x = (rand() % 255) - 127;
    for (auto &x : B) x = (rand() % 255) - 127;
    std::vector<int> ref(32 * 32, 0), D(32 * 32);
    for (int r = 0; r < 32; ++r) for (int c = 0; c < 32; ++c) {
      int s = 0; for (int k = 0; k < 32; ++k) s += A[r * 32 + k] * B[k * 32 + c]; ref[r * 32 + c] = s; }
    int8_t *dA, *dB; int *dD;
    CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dD, 4096));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    for (int h = 0; h < 2; ++h) {
      hipLaunchKernelGGL(i8_32x32x32_probe, 1, 64, 0, 0, dA, dB, dD, h);
      CK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
      int bad = 0; for (int i = 0; i < 1024; ++i) bad += D[i] != ref[i];
      printf("i8_32x32x32 hypothesis %d: mismatches %d/1024\n", h, bad);
    }
  }
  // i8 16x16x64
  {
    std::vector<int8_t> A(16 * 64), B(64 * 16);
    for (auto &x : A) x = (rand() % 255) - 127;
    for (auto &x : B) x = (rand() % 255) - 127;
    std::vector<int> ref(256, 0), D(256);
    for (int r = 0; r < 16; ++r) for (int c = 0; c < 16; ++c) {
      int s = 0; for (int k = 0; k < 64; ++k) s += A[r * 64 + k] * B[k * 16 + c]; ref[r * 16 + c] = s; }
    int8_t *dA, *dB; int *dD;
    CK(hipMalloc(&dA, 1024)); CK(hipMalloc(&dB, 1024)); CK(hipMalloc(&dD, 1024));
    CK(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    for (int h = 0; h < 2; ++h) {
      hipLaunchKernelGGL(i8_16x16x64_probe, 1, 64, 0, 0, dA, dB, dD, h);
      CK(hipMemcpy(D.data(), dD, 1024, hipMemcpyDeviceToHost));
      int bad = 0; for (int i = 0; i < 256; ++i) bad += D[i] != ref[i];
      printf("i8_16x16x64 hypothesis %d: mismatches %d/256\n", h, bad);
    }
  }
  // f64 16x16x4
  {
    std::vector<double> A(64), B(64), ref(256, 0), D(256);
    for (auto &x : A) x = (rand() % 1000) / 7.0;
    for (auto &x : B) x = (rand() % 1000) / 3.0;
    for (int r = 0; r < 16; ++r) for (int c = 0; c < 16; ++c) {
      double s = 0; for (int k = 0; k < 4; ++k) s += A[r * 4 + k] * B[k * 16 + c]; ref[r * 16 + c] = s; }
    double *dA, *dB, *dD;
    CK(hipMalloc(&dA, 512)); CK(hipMalloc(&dB, 512)); CK(hipMalloc(&dD, 2048));
    CK(hipMemcpy(dA, A.data(), 512, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), 512, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(f64_16x16x4_probe, 1, 64, 0, 0, dA, dB, dD);
    CK(hipMemcpy(D.data(), dD, 2048, hipMemcpyDeviceToHost));
    int bad = 0; double maxrel = 0;
    for (int i = 0; i < 256; ++i) { double rel = fabs(D[i] - ref[i]) / (fabs(ref[i]) + 1e-30); if (rel > 1e-12) bad++; if (rel > maxrel) maxrel = rel; }
    printf("f64_16x16x4: mismatches %d/256 maxrel %.3g\n", bad, maxrel);
  }
  // rates
  {
    int *dout; CK(hipMalloc(&dout, 64));
    double *ddo; CK(hipMalloc(&ddo, 64));
    const int IT = 4096;
    for (int bpc : {1, 2}) {
      int blocks = 256 * bpc;  // 4 waves per block -> 1 wave/SIMD per block
      double ms = time_kernel([&](int b) { hipLaunchKernelGGL(rate_i8_32<IT>, b, 256, 0, 0, dout, 3); }, blocks, 5);
      double ops = (double)blocks * 4 * IT * 4 * (32.0 * 32 * 32 * 2);
      printf("i8 32x32x32 %d blk/CU: %.3f ms  %.1f TOPS\n", bpc, ms, ops / ms / 1e9);
      ms = time_kernel([&](int b) { hipLaunchKernelGGL(rate_i8_16<IT>, b, 256, 0, 0, dout, 3); }, blocks, 5);
      ops = (double)blocks * 4 * IT * 4 * (16.0 * 16 * 64 * 2);
      printf("i8 16x16x64 %d blk/CU: %.3f ms  %.1f TOPS\n", bpc, ms, ops / ms / 1e9);
      ms = time_kernel([&](int b) { hipLaunchKernelGGL(rate_f64<IT>, b, 256, 0, 0, ddo, 1.0001); }, blocks, 5);
      ops = (double)blocks * 4 * IT * 4 * (16.0 * 16 * 4 * 2);
      printf("f64 16x16x4 %d blk/CU: %.3f ms  %.2f TFLOPS\n", bpc, ms, ops / ms / 1e9);
      ms = time_kernel([&](int b) { hipLaunchKernelGGL(rate_fma64<IT>, b, 256, 0, 0, ddo, 1.0001); }, blocks, 5);
      ops = (double)blocks * 256 * IT * 8 * 2;
      printf("f64 VALU fma %d blk/CU: %.3f ms  %.2f TFLOPS\n", bpc, ms, ops / ms / 1e9);
    }
  }
  hipDeviceProp_t p; CK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs %d clock %d kHz L2 %d\n", p.gcnArchName, p.multiProcessorCount, p.clockRate, p.l2CacheSize);
  return 0;
}

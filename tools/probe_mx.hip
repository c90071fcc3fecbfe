// Block-scaled MFMA probe for gfx950 (v_mfma_scale_f32_32x32x64_f8f6f4):
//  * A in fp6 e2m3 (cbsz 2), B in fp4 e2m1 (blgp 4): which k each packed element of a lane
//    holds, how 32 fp6 / fp4 codes pack into the lane's dwords, and the e8m0 scale semantics
//    (one scale per lane = per (row|column, 32-deep k block)), checked with exact values;
//  * the sustained rate of that form next to fp8 x fp8, fp6 x fp6 and the int8 32x32x32.
// Build: hipcc --offload-arch=gfx950 -O3 -o probe_mx probe_mx.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v8i __attribute__((ext_vector_type(8)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef float v16f __attribute__((ext_vector_type(16)));

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { \
  printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); exit(1);} } while (0)

static double fp6_val(int c) {  // e2m3, bias 1
  const int s = (c >> 5) & 1, e = (c >> 3) & 3, m = c & 7;
  const double v = e ? std::ldexp(1.0 + m / 8.0, e - 1) : m / 8.0;
  return s ? -v : v;
}
static double fp4_val(int c) {  // e2m1, bias 1
  const int s = (c >> 3) & 1, e = (c >> 1) & 3, m = c & 1;
  const double v = e ? std::ldexp(1.0 + m / 2.0, e - 1) : m / 2.0;
  return s ? -v : v;
}

// k held by element j of lane l under hypothesis h
__host__ __device__ int kmap(int h, int l, int j) {
  const int hh = l >> 5;
  if (h == 0) return 32 * hh + j;
  if (h == 1) return (j < 16) ? 16 * hh + j : 32 + 16 * hh + (j - 16);
  return (j >> 3) * 16 + 8 * hh + (j & 7);
}

// codes: A6[32 rows][64 k] fp6 codes, B4[64 k][32 cols] fp4 codes, per-lane scales sa, sb.
__global__ void probe(const uint8_t *A6, const uint8_t *B4, const int *sa, const int *sb, float *D, int h) {
  const int l = threadIdx.x, r = l & 31;
  uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < 32; ++j) {
    const int k = kmap(h, l, j);
    const uint32_t ca = A6[r * 64 + k], cb = B4[k * 32 + r];
    const int bit = 6 * j;  // fp6: element j at bits 6j .. 6j+5 of the lane's 192 bits
    a[bit >> 5] |= ca << (bit & 31);
    if ((bit & 31) > 26) a[(bit >> 5) + 1] |= ca >> (32 - (bit & 31));
    b[j >> 3] |= cb << (4 * (j & 7));  // fp4: element j at bits 4j .. 4j+3
  }
  v8i av, bv;
  for (int q = 0; q < 8; ++q) { av[q] = (int)a[q]; bv[q] = (int)b[q]; }
  v16f c = {0};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 2, 4, 0, sa[l], 0, sb[l]);
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
    D[row * 32 + r] = c[q];
  }
}

// opsel: the scale byte taken from byte 1 (A) / byte 2 (B) of the scale registers
__global__ void probe_opsel(const uint8_t *A6, const uint8_t *B4, const int *sa, const int *sb, float *D) {
  const int l = threadIdx.x, r = l & 31;
  uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0}, b[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = 0; j < 32; ++j) {
    const int k = kmap(0, l, j);
    const uint32_t ca = A6[r * 64 + k], cb = B4[k * 32 + r];
    const int bit = 6 * j;
    a[bit >> 5] |= ca << (bit & 31);
    if ((bit & 31) > 26) a[(bit >> 5) + 1] |= ca >> (32 - (bit & 31));
    b[j >> 3] |= cb << (4 * (j & 7));
  }
  v8i av, bv;
  for (int q = 0; q < 8; ++q) { av[q] = (int)a[q]; bv[q] = (int)b[q]; }
  v16f c = {0};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 2, 4, 1, (sa[l] << 8) | 0x11, 2, (sb[l] << 16) | 0x2222);
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
    D[row * 32 + r] = c[q];
  }
}
typedef float v2f __attribute__((ext_vector_type(2)));
__global__ void probe_cvt(const unsigned *x, float *out) {
  const int l = threadIdx.x;
  v2f r0 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x[l], 2.0f, 0);
  v2f r1 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x[l], 2.0f, 1);
  v2f r2 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x[l], 2.0f, 2);
  v2f r3 = __builtin_amdgcn_cvt_scalef32_pk_f32_fp4(x[l], 2.0f, 3);
  out[8 * l + 0] = r0.x; out[8 * l + 1] = r0.y; out[8 * l + 2] = r1.x; out[8 * l + 3] = r1.y;
  out[8 * l + 4] = r2.x; out[8 * l + 5] = r2.y; out[8 * l + 6] = r3.x; out[8 * l + 7] = r3.y;
}

template <int ITER, int FA, int FB>
__global__ void __launch_bounds__(256) rate_mx(float *out, int seed) {
  v8i a, b;
  for (int q = 0; q < 8; ++q) { a[q] = seed * 0x01010101 + q; b[q] = (seed ^ 0x5a5a5a5a) + 3 * q; }
  v16f c0 = {0}, c1 = {0}, c2 = {0}, c3 = {0};
  for (int i = 0; i < ITER; ++i) {
    c0 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c0, FA, FB, 0, 127, 0, 127);
    c1 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, a, c1, FA, FB, 0, 127, 0, 127);
    c2 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, a, c2, FA, FB, 0, 127, 0, 127);
    c3 = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(b, b, c3, FA, FB, 0, 127, 0, 127);
  }
  float s = 0;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  if (s == 12345.f) out[0] = s;
}
template <int ITER>
__global__ void __launch_bounds__(256) rate_i8(float *out, int seed) {
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
  if (s == 0x12345) out[0] = (float)s;
}

template <typename K>
double time_kernel(K k, int blocks, int reps) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  k(blocks);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k(blocks);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms; CK(hipEventElapsedTime(&ms, e0, e1));
  return ms / reps;
}

int main() {
  srand(7);
  std::vector<uint8_t> A(32 * 64), B(64 * 32);
  std::vector<int> sa(64), sb(64);
  for (auto &x : A) x = rand() % 64;
  for (auto &x : B) x = rand() % 16;
  for (auto &x : sa) x = 120 + rand() % 15;
  for (auto &x : sb) x = 120 + rand() % 15;
  uint8_t *dA, *dB; int *dsa, *dsb; float *dD;
  CK(hipMalloc(&dA, 2048)); CK(hipMalloc(&dB, 2048)); CK(hipMalloc(&dsa, 256)); CK(hipMalloc(&dsb, 256));
  CK(hipMalloc(&dD, 4096));
  CK(hipMemcpy(dA, A.data(), 2048, hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), 2048, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, sa.data(), 256, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb.data(), 256, hipMemcpyHostToDevice));
  std::vector<float> D(1024);
  for (int h = 0; h < 3; ++h) {
    // reference under hypothesis h: scale of lane l applies to its own 32 elements
    std::vector<double> ref(1024, 0.0), mag(1024, 0.0);
    for (int row = 0; row < 32; ++row)
      for (int col = 0; col < 32; ++col)
        for (int hh = 0; hh < 2; ++hh)
          for (int j = 0; j < 32; ++j) {
            const int la = row + 32 * hh, lb = col + 32 * hh;
            const int k = kmap(h, la, j);
            if (kmap(h, lb, j) != k) printf("asymmetric map\n");
            const double t = fp6_val(A[row * 64 + k]) * std::ldexp(1.0, sa[la] - 127) * fp4_val(B[k * 32 + col]) *
                             std::ldexp(1.0, sb[lb] - 127);
            ref[row * 32 + col] += t;
            mag[row * 32 + col] += fabs(t);
          }
    hipLaunchKernelGGL(probe, 1, 64, 0, 0, dA, dB, dsa, dsb, dD, h);
    CK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    double worst = 0;
    for (int i = 0; i < 1024; ++i) {
      const double e = fabs(D[i] - ref[i]) / (mag[i] + 1e-300);
      if (e > 1e-6) ++bad;
      if (e > worst) worst = e;
    }
    printf("fp6 x fp4 32x32x64 hypothesis %d: mismatches %d/1024, worst |err|/sum|t| %.3g\n", h, bad, worst);
  }
  {  // opsel (reference = hypothesis 0 with the same scales)
    std::vector<double> ref(1024, 0.0), mag(1024, 0.0);
    for (int row = 0; row < 32; ++row)
      for (int col = 0; col < 32; ++col)
        for (int hh = 0; hh < 2; ++hh)
          for (int j = 0; j < 32; ++j) {
            const int la = row + 32 * hh, lb = col + 32 * hh, k = kmap(0, la, j);
            const double t = fp6_val(A[row * 64 + k]) * std::ldexp(1.0, sa[la] - 127) * fp4_val(B[k * 32 + col]) *
                             std::ldexp(1.0, sb[lb] - 127);
            ref[row * 32 + col] += t;
            mag[row * 32 + col] += fabs(t);
          }
    hipLaunchKernelGGL(probe_opsel, 1, 64, 0, 0, dA, dB, dsa, dsb, dD);
    CK(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 1024; ++i) bad += fabs(D[i] - ref[i]) / (mag[i] + 1e-300) > 1e-6;
    printf("opsel_a=1 / opsel_b=2 byte select: mismatches %d/1024\n", bad);
  }
  {  // cvt_scalef32_pk_f32_fp4: which nibble lands in .x / .y of each byte select
    std::vector<unsigned> x(64);
    for (int l = 0; l < 64; ++l) x[l] = 0x76543210u + (unsigned)l * 0x11111111u;
    unsigned *dx; float *dout2;
    CK(hipMalloc(&dx, 256)); CK(hipMalloc(&dout2, 64 * 8 * 4));
    CK(hipMemcpy(dx, x.data(), 256, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(probe_cvt, 1, 64, 0, 0, dx, dout2);
    std::vector<float> o(512);
    CK(hipMemcpy(o.data(), dout2, 2048, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 8; ++e) bad += o[8 * l + e] != (float)(2.0 * fp4_val((x[l] >> (4 * e)) & 15));
    printf("cvt_scalef32_pk_f32_fp4 (nibble e -> element e, x2): mismatches %d/512; lane0 %g %g %g %g %g %g %g %g\n", bad,
           o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]);
  }
  // rates: 4 waves per block, 1 or 2 blocks per CU
  float *dout; CK(hipMalloc(&dout, 64));
  const int IT = 4096;
  for (int bpc : {1, 2}) {
    const int blocks = 256 * bpc;
    const double mac = (double)blocks * 4 * IT * 4;
    double ms = time_kernel([&](int b) { hipLaunchKernelGGL((rate_mx<IT, 2, 4>), b, 256, 0, 0, dout, 3); }, blocks, 5);
    printf("mx fp6 x fp4 %d blk/CU: %.3f ms  %.1f TFLOPS\n", bpc, ms, mac * 32 * 32 * 64 * 2 / ms / 1e9);
    ms = time_kernel([&](int b) { hipLaunchKernelGGL((rate_mx<IT, 2, 2>), b, 256, 0, 0, dout, 3); }, blocks, 5);
    printf("mx fp6 x fp6 %d blk/CU: %.3f ms  %.1f TFLOPS\n", bpc, ms, mac * 32 * 32 * 64 * 2 / ms / 1e9);
    ms = time_kernel([&](int b) { hipLaunchKernelGGL((rate_mx<IT, 4, 4>), b, 256, 0, 0, dout, 3); }, blocks, 5);
    printf("mx fp4 x fp4 %d blk/CU: %.3f ms  %.1f TFLOPS\n", bpc, ms, mac * 32 * 32 * 64 * 2 / ms / 1e9);
    ms = time_kernel([&](int b) { hipLaunchKernelGGL((rate_mx<IT, 0, 4>), b, 256, 0, 0, dout, 3); }, blocks, 5);
    printf("mx fp8 x fp4 %d blk/CU: %.3f ms  %.1f TFLOPS\n", bpc, ms, mac * 32 * 32 * 64 * 2 / ms / 1e9);
    ms = time_kernel([&](int b) { hipLaunchKernelGGL((rate_i8<IT>), b, 256, 0, 0, dout, 3); }, blocks, 5);
    printf("i8 32x32x32 %d blk/CU: %.3f ms  %.1f TOPS\n", bpc, ms, mac * 32 * 32 * 32 * 2 / ms / 1e9);
  }
  return 0;
}

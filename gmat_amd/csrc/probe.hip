// Diagnostics entry points that exercise single instructions the screens rely on, so that
// tests can check the rigorous error bounds the screens assume against the hardware itself.
//
// gmat_probe_mx_accum: the low-rank screen's accumulation (lr_screen_kernel, epi.hip) -- a chain of
// v_mfma_scale_f32_32x32x64_f8f6f4 (A fp6 e2m3 with one e8m0 scale per lane = per (row, 32 k),
// B fp4 e2m1) accumulated in fp32 over n_steps k-blocks of 64, exactly the instruction, operand
// formats, B scale (128: the fp4 codes hold w/2) and accumulation order of the screen.  B is the
// screen's worst case everywhere (w = 4, fp4 code 0x4 = 2.0), so every column of the result equals
// 4 sum_k A[r][k] and the exact value needs no knowledge of the lane -> k map.
#include "common.h"

namespace {
typedef int v8i_ __attribute__((ext_vector_type(8)));
typedef float v16f_ __attribute__((ext_vector_type(16)));

// codes: [n_steps][32 rows][2 halves][32] fp6 codes (0..63); scales: [n_steps][32][2] e8m0
__global__ __launch_bounds__(64) void mx_accum_probe_kernel(int n_steps, const uint8_t *codes, const uint8_t *scales,
                                                             float *out) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  v16f_ acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  v8i_ fb;
  for (int q = 0; q < 8; ++q) fb[q] = q < 4 ? 0x44444444 : 0;
  for (int s = 0; s < n_steps; ++s) {
    const uint8_t *cs = codes + (((int64_t)s * 32 + r) * 2 + h) * 32;
    uint32_t a[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < 32; ++j) {
      const uint32_t c = cs[j] & 63u;
      const int bit = 6 * j;
      a[bit >> 5] |= c << (bit & 31);
      if ((bit & 31) > 26) a[(bit >> 5) + 1] |= c >> (32 - (bit & 31));
    }
    v8i_ fa;
    for (int q = 0; q < 8; ++q) fa[q] = (int)a[q];
    const int sa = scales[((int64_t)s * 32 + r) * 2 + h];
    acc = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fa, fb, acc, 2, 4, 0, sa, 0, 128);
  }
  for (int q = 0; q < 16; ++q) {
    const int row = (q & 3) + 8 * (q >> 2) + 4 * h;
    out[row * 32 + r] = acc[q];
  }
}
}  // namespace

extern "C" int gmat_probe_mx_accum(int n_steps, const uint8_t *codes, const uint8_t *scales, float *out) {
  using namespace gmat;
  GMAT_CHECK(n_steps > 0 && n_steps <= 1024 && codes && scales && out, GMAT_E_ARG, "gmat_probe_mx_accum: bad arguments");
  DBuf dc, ds, dout;
  GMAT_TRY(dc.alloc((size_t)n_steps * 32 * 2 * 32));
  GMAT_TRY(ds.alloc((size_t)n_steps * 32 * 2));
  GMAT_TRY(dout.alloc(32 * 32 * sizeof(float)));
  GMAT_HIP(hipMemcpy(dc.p, codes, (size_t)n_steps * 32 * 2 * 32, hipMemcpyHostToDevice));
  GMAT_HIP(hipMemcpy(ds.p, scales, (size_t)n_steps * 32 * 2, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(mx_accum_probe_kernel, dim3(1), dim3(64), 0, 0, n_steps, dc.as<uint8_t>(), ds.as<uint8_t>(),
                     dout.as<float>());
  GMAT_HIP(hipGetLastError());
  GMAT_HIP(hipMemcpy(out, dout.p, 32 * 32 * sizeof(float), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// gmat_probe_eig_bottom: the plan's partial symmetric eigensolver (eig.hip: Chebyshev-filtered
// subspace iteration with a device Rayleigh-Ritz) on a host matrix, so tests can compare it with a
// dense reference decomposition.  res_out (ne residual norms) and iters_out may be null.
#include "dla.h"
extern "C" int gmat_probe_eig_bottom(int64_t n, const double *a_host, int ne, double tol, int maxit, double *w_out,
                                     double *z_out, double *res_out, int *iters_out) {
  using namespace gmat;
  GMAT_CHECK(n >= 2 && a_host && w_out && z_out && ne >= 1 && ne <= n && maxit >= 1, GMAT_E_ARG,
             "gmat_probe_eig_bottom: bad arguments");
  DBuf a, z;
  GMAT_TRY(a.alloc((size_t)n * n * sizeof(double)));
  GMAT_TRY(z.alloc((size_t)n * ne * sizeof(double)));
  GMAT_HIP(hipMemcpy(a.p, a_host, (size_t)n * n * sizeof(double), hipMemcpyHostToDevice));
  GMAT_TRY(sym_eig_bottom(n, a.as<double>(), ne, tol, maxit, w_out, z.as<double>(), res_out, iters_out));
  GMAT_HIP(hipMemcpy(z_out, z.p, (size_t)n * ne * sizeof(double), hipMemcpyDeviceToHost));
  return GMAT_OK;
}

// ViT residual + LayerScale + LayerNorm as one row pass (DINOv2 blocks under SajayR/TRIAD
// model.py:207-266: x = x + ls(attn(norm1(x))); x = x + ls(mlp(norm2(x))), bf16 autocast).
//
// Under autocast the unfused chain makes five HBM passes per residual step over the fp32
// residual stream (LayerScale multiply, add, LayerNorm, cast to bf16 for the next GEMM) and
// twice that in the backward. Here:
//   forward : xn = x + g * y (fp32, the residual stream), ln = LN(xn) * w + b (bf16, or fp32
//             for the final norm), per-row mean / rstd saved;
//   backward: dxn = dres + rstd * (w dln - mean(w dln) - xhat mean(w dln xhat)), dy = bf16(g dxn)
//             (the frozen backbone's LayerNorm / LayerScale parameters get no gradient).
// One wave per row, D = 256 k (4 consecutive elements per lane per 256-column block), two-pass
// mean / variance in registers (fp32), same formulas as ATen's layer_norm kernels.
#include "common.h"

namespace {

template <int NB>  // NB = D / 256
__device__ __forceinline__ void row_stats(const float (&v)[NB][4], int D, float eps, float& mean, float& rstd) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) s += v[i][c];
  mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float d = v[i][c] - mean;
      q = fmaf(d, d, q);
    }
  rstd = rsqrtf(wave_sum(q) / D + eps);
}

template <int NB, bool HAS_Y, bool OUT_F32>
__global__ __launch_bounds__(256) void addln_fwd_kernel(const float* __restrict__ x, const bf16* __restrict__ y,
                                                        const float* __restrict__ g, const float* __restrict__ w,
                                                        const float* __restrict__ b, float eps, int M,
                                                        float* __restrict__ xn, void* __restrict__ ln,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int D = NB * 256;
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NB][4];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    const f32x4 xv = *(const f32x4*)(x + row * D + c0);
    if (HAS_Y) {
      const bf16x4 yv = *(const bf16x4*)(y + row * D + c0);
      const f32x4 gv = *(const f32x4*)(g + c0);
#pragma unroll
      for (int c = 0; c < 4; ++c) v[i][c] = __fadd_rn(xv[c], __fmul_rn(gv[c], (float)yv[c]));  // x + (g * y), unfused
      *(f32x4*)(xn + row * D + c0) = (f32x4){v[i][0], v[i][1], v[i][2], v[i][3]};
    } else {
#pragma unroll
      for (int c = 0; c < 4; ++c) v[i][c] = xv[c];
    }
  }
  float mean, rstd;
  row_stats<NB>(v, D, eps, mean, rstd);
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    const f32x4 wv = *(const f32x4*)(w + c0);
    const f32x4 bv = *(const f32x4*)(b + c0);
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) o[c] = (v[i][c] - mean) * rstd * wv[c] + bv[c];
    if (OUT_F32) {
      *(f32x4*)((float*)ln + row * D + c0) = (f32x4){o[0], o[1], o[2], o[3]};
    } else {
      bf16x4 ob;
#pragma unroll
      for (int c = 0; c < 4; ++c) ob[c] = (bf16)o[c];
      *(bf16x4*)((bf16*)ln + row * D + c0) = ob;
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

template <int NB, bool DLN_F32, bool HAS_RES>
__global__ __launch_bounds__(256) void addln_bwd_kernel(const void* __restrict__ dln, const float* __restrict__ dres,
                                                        const float* __restrict__ xn, const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in, const float* __restrict__ w,
                                                        const float* __restrict__ g, int M, float* __restrict__ dx,
                                                        bf16* __restrict__ dy) {
  constexpr int D = NB * 256;
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float mean = mean_in[row], rstd = rstd_in[row];
  float xh[NB][4], wd[NB][4];
  float s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    const f32x4 xv = *(const f32x4*)(xn + row * D + c0);
    const f32x4 wv = *(const f32x4*)(w + c0);
    float dv[4];
    if (DLN_F32) {
      const f32x4 t = *(const f32x4*)((const float*)dln + row * D + c0);
#pragma unroll
      for (int c = 0; c < 4; ++c) dv[c] = t[c];
    } else {
      const bf16x4 t = *(const bf16x4*)((const bf16*)dln + row * D + c0);
#pragma unroll
      for (int c = 0; c < 4; ++c) dv[c] = (float)t[c];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      xh[i][c] = (xv[c] - mean) * rstd;
      wd[i][c] = wv[c] * dv[c];
      s1 += wd[i][c];
      s2 = fmaf(wd[i][c], xh[i][c], s2);
    }
  }
  const float c1 = wave_sum(s1) / D, c2 = wave_sum(s2) / D;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    f32x4 r = HAS_RES ? *(const f32x4*)(dres + row * D + c0) : (f32x4){0.f, 0.f, 0.f, 0.f};
    const f32x4 gv = *(const f32x4*)(g + c0);
    bf16x4 yb;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      r[c] += rstd * (wd[i][c] - c1 - xh[i][c] * c2);
      yb[c] = (bf16)__fmul_rn(gv[c], r[c]);
    }
    *(f32x4*)(dx + row * D + c0) = r;
    *(bf16x4*)(dy + row * D + c0) = yb;
  }
}

}  // namespace

extern "C" {

// xn = x + g * y (y may be NULL: xn not written, LN of x), ln = LN(xn) * w + b as bf16
// (out_f32 = 0) or fp32; mean / rstd per row. D % 256 == 0, D <= 1536.
int triad_addln_fwd(const float* x, const void* y, const float* g, const float* w, const float* b, float eps, int M,
                    int D, float* xn, void* ln, int out_f32, float* mean, float* rstd, hipStream_t stream) {
  if (M <= 0 || D % 256 || D > 1536) return TRIAD_EINVAL;
  const dim3 grid((M + 3) / 4);
#define ADDLN_F(NB)                                                                                             \
  if (D == NB * 256) {                                                                                          \
    if (y && out_f32)                                                                                           \
      hipLaunchKernelGGL((addln_fwd_kernel<NB, true, true>), grid, dim3(256), 0, stream, x, (const bf16*)y, g, w, b, \
                         eps, M, xn, ln, mean, rstd);                                                           \
    else if (y)                                                                                                 \
      hipLaunchKernelGGL((addln_fwd_kernel<NB, true, false>), grid, dim3(256), 0, stream, x, (const bf16*)y, g, w, b, \
                         eps, M, xn, ln, mean, rstd);                                                           \
    else if (out_f32)                                                                                           \
      hipLaunchKernelGGL((addln_fwd_kernel<NB, false, true>), grid, dim3(256), 0, stream, x, (const bf16*)y, g, w, b, \
                         eps, M, xn, ln, mean, rstd);                                                           \
    else                                                                                                        \
      hipLaunchKernelGGL((addln_fwd_kernel<NB, false, false>), grid, dim3(256), 0, stream, x, (const bf16*)y, g, w, \
                         b, eps, M, xn, ln, mean, rstd);                                                        \
    TRIAD_CHECK_LAUNCH();                                                                                       \
    return TRIAD_OK;                                                                                            \
  }
  ADDLN_F(1) ADDLN_F(2) ADDLN_F(3) ADDLN_F(4) ADDLN_F(5) ADDLN_F(6)
#undef ADDLN_F
  return TRIAD_EINVAL;
}

// dx = dres (may be NULL) + LN backward of dln (bf16, or fp32 if dln_f32) at xn; dy = bf16(g * dx).
int triad_addln_bwd(const void* dln, int dln_f32, const float* dres, const float* xn, const float* mean,
                    const float* rstd, const float* w, const float* g, int M, int D, float* dx, void* dy,
                    hipStream_t stream) {
  if (M <= 0 || D % 256 || D > 1536) return TRIAD_EINVAL;
  const dim3 grid((M + 3) / 4);
#define ADDLN_B(NB, DF, HR)                                                                                      \
  hipLaunchKernelGGL((addln_bwd_kernel<NB, DF, HR>), grid, dim3(256), 0, stream, dln, dres, xn, mean, rstd, w, g, M, \
                     dx, (bf16*)dy)
#define ADDLN_BD(NB)                                                                                             \
  if (D == NB * 256) {                                                                                           \
    if (dln_f32 && dres) ADDLN_B(NB, true, true);                                                                \
    else if (dln_f32) ADDLN_B(NB, true, false);                                                                  \
    else if (dres) ADDLN_B(NB, false, true);                                                                     \
    else ADDLN_B(NB, false, false);                                                                              \
    TRIAD_CHECK_LAUNCH();                                                                                        \
    return TRIAD_OK;                                                                                             \
  }
  ADDLN_BD(1) ADDLN_BD(2) ADDLN_BD(3) ADDLN_BD(4) ADDLN_BD(5) ADDLN_BD(6)
#undef ADDLN_BD
#undef ADDLN_B
  return TRIAD_EINVAL;
}

}  // extern "C"

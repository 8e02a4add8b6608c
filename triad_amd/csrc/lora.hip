// Skinny GEMMs of the ViT's LoRA adapters (SajayR/TRIAD model.py:223-266: peft LoRA r=8 on the
// DINOv2 attn.qkv / attn.proj Linears, y = W x + b + (alpha/r) B A x).
//
// With M = B*N tokens (66 816 at c3) and rank r = 8 these products are HBM-bound streams over
// one (M, K) activation, which the library GEMMs run at a fraction of bandwidth:
//   triad_rows_nt: out[m][j] = sum_k X[m][k] W[j][k]      (t = x A^T, dt = dy (sB))   MFMA 16x16x32,
//                  rows of X straight from HBM, W fragments from L2, j < J <= 16;
//   triad_rows_tn: out[o][j] = alpha sum_m Y[m][o] T[m][j] (dB = s dy^T t, dA^T = x^T dt)  fp32 VALU,
//                  one pass over Y split into row slabs, partials reduced by a second kernel.
#include "common.h"

namespace {

typedef float f32x4_t __attribute__((ext_vector_type(4)));

// 4 waves x 16 rows; lane (row l & 15, k-group l >> 4) loads X[row][32 s + 8 kg .. +7]
__global__ __launch_bounds__(256) void rows_nt_kernel(const bf16* __restrict__ X, long long ldx, int M, int K,
                                                      const bf16* __restrict__ W, int J, bf16* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, kg = lane >> 4;
  const long long row0 = ((long long)blockIdx.x * 4 + wave) * 16;
  if (row0 >= M) return;
  const long long rr = min(row0 + r, (long long)M - 1);  // clamp: rows past M computed, not stored
  const bf16* xp = X + rr * ldx + 8 * kg;
  const bool wok = r < J;
  const bf16* wp = W + (long long)(wok ? r : 0) * K + 8 * kg;
  const int ns = K / 32;
  constexpr int PF = 4;
  bf16x8 xa[PF];
#pragma unroll
  for (int i = 0; i < PF; ++i) xa[i] = i < ns ? *(const bf16x8*)(xp + 32 * i) : (bf16x8){};
  f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int s = 0; s < ns; s += PF) {
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      if (s + i < ns) {
        const bf16x8 a = xa[i];
        if (s + i + PF < ns) xa[i] = *(const bf16x8*)(xp + 32 * (s + i + PF));
        const bf16x8 w = wok ? *(const bf16x8*)(wp + 32 * (s + i)) : (bf16x8){};
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, w, acc, 0, 0, 0);
      }
    }
  }
  // C: col = lane & 15 (j), rows 4 kg + i
  if (r < J) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const long long row = row0 + 4 * kg + i;
      if (row < M) out[row * J + r] = (bf16)acc[i];
    }
  }
}

// thread = 8 consecutive columns o of Y; grid.y = row slabs. slab[s][o][j] (fp32).
constexpr int TJ = 8;
__global__ __launch_bounds__(256) void rows_tn_kernel(const bf16* __restrict__ Y, long long ldy, int M, int O,
                                                      const bf16* __restrict__ T, int rows_per_slab,
                                                      float* __restrict__ slab) {
  const int c8 = blockIdx.x * blockDim.x + threadIdx.x;
  if (8 * c8 >= O) return;
  const int m0 = blockIdx.y * rows_per_slab, m1 = min(M, m0 + rows_per_slab);
  float acc[8][TJ];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int j = 0; j < TJ; ++j) acc[c][j] = 0.f;
  const bf16* yp = Y + 8 * c8;
#pragma unroll 4
  for (int m = m0; m < m1; ++m) {
    const bf16x8 y = *(const bf16x8*)(yp + (long long)m * ldy);
    const bf16x8 t = *(const bf16x8*)(T + (long long)m * TJ);
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int j = 0; j < TJ; ++j) acc[c][j] = fmaf((float)y[c], (float)t[j], acc[c][j]);
  }
  float* sp = slab + ((long long)blockIdx.y * O + 8 * c8) * TJ;
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int j = 0; j < TJ; j += 4)
      *(f32x4_t*)(sp + c * TJ + j) = (f32x4_t){acc[c][j], acc[c][j + 1], acc[c][j + 2], acc[c][j + 3]};
}

__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ slab, int S, long long n, float alpha,
                                                       float* __restrict__ out) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  float s = 0.f;
  for (int i = 0; i < S; ++i) s += slab[i * n + e];
  out[e] = alpha * s;
}

}  // namespace

extern "C" {

int triad_rows_nt(const void* X, long long ldx, int M, int K, const void* W, int J, void* out, hipStream_t stream) {
  if (M <= 0 || K <= 0 || K % 32 || J <= 0 || J > 16 || ldx < K || ldx % 8) return TRIAD_EINVAL;
  const int blocks = (M + 63) / 64;
  hipLaunchKernelGGL(rows_nt_kernel, dim3(blocks), dim3(256), 0, stream, (const bf16*)X, ldx, M, K, (const bf16*)W, J,
                     (bf16*)out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_rows_tn_slabs(int M) { return M >= 32768 ? 256 : (M + 127) / 128; }

int triad_rows_tn(const void* Y, long long ldy, int M, int O, const void* T, int J, float alpha, float* slabs,
                  float* out, hipStream_t stream) {
  if (M <= 0 || O <= 0 || O % 8 || J != TJ || ldy < O || ldy % 8) return TRIAD_EINVAL;
  const int S = triad_rows_tn_slabs(M);
  const int rows = (M + S - 1) / S;
  const int threads = O / 8 >= 256 ? 256 : ((O / 8 + 63) / 64) * 64;
  const dim3 grid((O / 8 + threads - 1) / threads, S);
  hipLaunchKernelGGL(rows_tn_kernel, grid, dim3(threads), 0, stream, (const bf16*)Y, ldy, M, O, (const bf16*)T, rows,
                     slabs);
  const long long n = (long long)O * TJ;
  hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, slabs, S, n, alpha,
                     out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

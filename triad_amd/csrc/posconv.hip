// HuBERT positional convolution (SajayR/TRIAD model.py:29-30,66 -> transformers
// HubertPositionalConvEmbedding: Conv1d(C, C, kernel 128, padding 64, groups 16), weight-
// normalised, its last output dropped by HubertSamePadLayer) as an implicit GEMM over
// channels-last activations, for the forward and the input gradient.
//
//   y[b, t, g*CG + n] = bias[g*CG + n] + sum_{j < KT} sum_{c < CG} x[b, t + j - pad, g*CG + c] * W[g*CG + n, c, j]
//
// for t < T (x zero outside [0, T)). Per (sample, group) this is a GEMM whose A operand is a
// Hankel matrix: with the group's window of x stored compactly in LDS (row w = time
// t0 - pad + w, CG channels, zero-filled), row t of A over k = j*CG + c is the CONTIGUOUS
// slice xwin[(t - t0)*CG + k ...] -- so A fragments are plain ds_read_b128 at k-step offsets
// and no im2col tensor exists. The input gradient is the same GEMM with W flipped along j and
// transposed per group, and pad' = KT - 1 - pad.
//
// Workgroup = (group, sample, 208-row time block); 4 waves; wave w owns the 16-row time tiles
// w, w+4, w+8, w+12 and all CG/16 channel tiles (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
// B fragments (Wt[g][n][k], k contiguous) come straight from L2, prefetched one k-step ahead:
// blockIdx.x = group, so consecutive workgroups (dealt round-robin to the 8 XCDs) put only
// G/8 groups' weights into each XCD's L2.
#include "common.h"

namespace {

constexpr int KT = 128;       // taps
constexpr int MT = 13;        // 16-row time tiles per workgroup (208 rows >= T = 199 at 4 s)
constexpr int ROWS = MT * 16;
constexpr int NWAVE = 4;
constexpr int MT_PER_WAVE = (MT + NWAVE - 1) / NWAVE;  // 4

typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int CG>
__global__ __launch_bounds__(256) void posconv_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wt,
                                                      const float* __restrict__ bias, bf16* __restrict__ y, int T,
                                                      int C, int pad) {
  constexpr int NT = CG / 16;            // channel tiles
  constexpr int KTOT = KT * CG;          // GEMM depth
  constexpr int NKS = KTOT / 32;         // k-steps
  constexpr int WIN = ROWS + KT - 1;     // window rows
  __shared__ __attribute__((aligned(16))) bf16 xwin[WIN * CG];

  const int g = blockIdx.x, b = blockIdx.y, t0 = blockIdx.z * ROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  // window: rows w <-> time t0 - pad + w, 16-byte pieces, zero outside [0, T)
  constexpr int PIECES = CG / 8;
  for (int e = threadIdx.x; e < WIN * PIECES; e += 256) {
    const int w = e / PIECES, p = e - w * PIECES;
    const int t = t0 - pad + w;
    bf16x8 v = {};
    if (t >= 0 && t < T) v = *(const bf16x8*)(x + ((size_t)b * T + t) * C + g * CG + p * 8);
    *(bf16x8*)(xwin + w * CG + p * 8) = v;
  }
  __syncthreads();

  const int r = lane & 15, q = lane >> 4;
  // A fragment of time tile m at k-step s: xwin[(16 m + r) * CG + 32 s + 8 q .. +7]
  const bf16* abase = xwin + r * CG + 8 * q;
  // B fragment of channel tile n at k-step s: wt[g][16 n + r][32 s + 8 q .. +7]
  const bf16* bbase = wt + ((size_t)g * CG + r) * KTOT + 8 * q;

  f32x4_t acc[MT_PER_WAVE][NT];
#pragma unroll
  for (int i = 0; i < MT_PER_WAVE; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  bf16x8 bcur[NT], bnext[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) bcur[n] = *(const bf16x8*)(bbase + (size_t)n * 16 * KTOT);
  for (int s = 0; s < NKS; ++s) {
    if (s + 1 < NKS) {
#pragma unroll
      for (int n = 0; n < NT; ++n) bnext[n] = *(const bf16x8*)(bbase + (size_t)n * 16 * KTOT + (s + 1) * 32);
    }
#pragma unroll
    for (int i = 0; i < MT_PER_WAVE; ++i) {
      const int m = wave + NWAVE * i;
      if (m < MT) {
        const bf16x8 a = *(const bf16x8*)(abase + m * 16 * CG + s * 32);
#pragma unroll
        for (int n = 0; n < NT; ++n) acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bcur[n], acc[i][n], 0, 0, 0);
      }
    }
#pragma unroll
    for (int n = 0; n < NT; ++n) bcur[n] = bnext[n];
  }

  // C/D layout: col = lane & 15, row = 4 * (lane >> 4) + v
#pragma unroll
  for (int i = 0; i < MT_PER_WAVE; ++i) {
    const int m = wave + NWAVE * i;
    if (m >= MT) continue;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int ch = g * CG + n * 16 + r;
      const float bv = bias ? bias[ch] : 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int t = t0 + m * 16 + 4 * q + v;
        if (t < T) y[((size_t)b * T + t) * C + ch] = (bf16)(acc[i][n][v] + bv);
      }
    }
  }
}

}  // namespace

extern "C" {

int triad_posconv(const void* x, const void* wt, const float* bias, void* y, int B, int T, int C, int groups,
                  int pad, hipStream_t stream) {
  if (B <= 0 || T <= 0 || groups <= 0 || C % groups || pad < 0 || pad >= KT) return TRIAD_EINVAL;
  const int cg = C / groups;
  const dim3 grid(groups, B, (T + ROWS - 1) / ROWS);
  if (cg == 48)
    hipLaunchKernelGGL(posconv_kernel<48>, grid, dim3(256), 0, stream, (const bf16*)x, (const bf16*)wt, bias,
                       (bf16*)y, T, C, pad);
  else if (cg == 64)
    hipLaunchKernelGGL(posconv_kernel<64>, grid, dim3(256), 0, stream, (const bf16*)x, (const bf16*)wt, bias,
                       (bf16*)y, T, C, pad);
  else
    return TRIAD_EINVAL;
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

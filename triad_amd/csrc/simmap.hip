// Inference similarity maps (SajayR/TRIAD model.py:355-368 compute_similarity_matrix, called by
// forward() at model.py:630-636 and viz.py:182): sim[b] = temp * normalize(f1[b]) . normalize(f2[b])^T,
// (B, N1, N2) fp32, ONE launch over all B samples with the L2 normalisation in the prologue and
// the temperature in the epilogue (round 4 ran an l2norm pass per operand and then a host loop of
// padded copies + one GEMM launch per sample).
//
// Workgroup = 4 waves, a 64 x 64 output tile of one sample: wave w owns rows 16 w .. 16 w + 15 of
// the tile against its 64 columns (4 blocks of 16 x 16 on v_mfma_f32_16x16x32_bf16). Fragments
// come straight from global memory (16 contiguous bytes of one row per lane; the tiles are small
// and L2-resident, no LDS staging). Two passes over the rows' D features: the first accumulates
// each row's sum of squares on the lanes that will feed it to the MFMA (four k-chunk lanes per row,
// combined by two lane swaps), the second scales every element by 1 / max(||row||, eps), rounds it
// to bf16 -- F.normalize's bf16 output -- and multiplies. Rows past N1 / N2 re-read the last row
// (in bounds) and are not stored.
#include "common.h"

namespace {

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float sumsq8(bf16x8 v) {
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s += (float)v[i] * (float)v[i];
  return s;
}

__device__ __forceinline__ bf16x8 scale8(bf16x8 v, float inv) {
  bf16x8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = (bf16)((float)v[i] * inv);
  return o;
}

__global__ __launch_bounds__(256) void simmap_kernel(const bf16* __restrict__ f1, const bf16* __restrict__ f2, int N1,
                                                     int N2, int D, const float* __restrict__ temp, float eps,
                                                     float* __restrict__ out) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const long long b = blockIdx.z;
  const int m = blockIdx.y * 64 + 16 * wave + l16;   // this lane's f1 row (A fragment)
  const int n0 = blockIdx.x * 64;
  const bf16* ar = f1 + (b * N1 + (m < N1 ? m : N1 - 1)) * (long long)D + 8 * q;
  const bf16* br[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int n = n0 + 16 * cb + l16;
    br[cb] = f2 + (b * N2 + (n < N2 ? n : N2 - 1)) * (long long)D + 8 * q;
  }
  // pass 1: row norms (each row's D features are spread over its four q lanes)
  float sa = 0.f, sb[4] = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < D; k += 32) {
    sa += sumsq8(*(const bf16x8*)(ar + k));
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) sb[cb] += sumsq8(*(const bf16x8*)(br[cb] + k));
  }
  sa += __shfl_xor(sa, 16);
  sa += __shfl_xor(sa, 32);
  const float ia = 1.f / fmaxf(sqrtf(sa), eps);
  float ib[4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    sb[cb] += __shfl_xor(sb[cb], 16);
    sb[cb] += __shfl_xor(sb[cb], 32);
    ib[cb] = 1.f / fmaxf(sqrtf(sb[cb]), eps);
  }
  // pass 2: normalised bf16 operands into the MFMA (the f2 fragment first: each lane's four
  // accumulators are then four consecutive output columns of one row)
  f32x4 acc[4] = {};
  for (int k = 0; k < D; k += 32) {
    const bf16x8 af = scale8(*(const bf16x8*)(ar + k), ia);
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[cb] = mfma16(scale8(*(const bf16x8*)(br[cb] + k), ib[cb]), af, acc[cb]);
  }
  if (m >= N1) return;
  const float t = *temp;
  float* orow = out + (b * N1 + m) * (long long)N2;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int n = n0 + 16 * cb + 4 * q;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (n + i < N2) orow[n + i] = acc[cb][i] * t;
  }
}

}  // namespace

extern "C" {

// sim[b][i][j] = temp * <f1[b][i] / max(||f1[b][i]||, eps), f2[b][j] / max(||f2[b][j]||, eps)>,
// f1 (B, N1, D), f2 (B, N2, D) contiguous bf16 (D % 32 == 0), temp a device scalar, sim fp32.
int triad_similarity_maps(const void* f1, const void* f2, int B, int N1, int N2, int D, const float* temp, float eps,
                          float* sim, hipStream_t stream) {
  if (!f1 || !f2 || !temp || !sim || B <= 0 || N1 <= 0 || N2 <= 0 || D <= 0 || D % 32 || B > 65535 ||
      (N1 + 63) / 64 > 65535 || ((uintptr_t)f1 & 15) || ((uintptr_t)f2 & 15))
    return TRIAD_EINVAL;
  hipLaunchKernelGGL(simmap_kernel, dim3((N2 + 63) / 64, (N1 + 63) / 64, B), dim3(256), 0, stream, (const bf16*)f1,
                     (const bf16*)f2, N1, N2, D, temp, eps, sim);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

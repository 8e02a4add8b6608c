// Inference similarity maps (SajayR/TRIAD model.py:355-368 compute_similarity_matrix, called by
// forward() at model.py:630-636 and viz.py:182): sim[b] = temp * normalize(f1[b]) . normalize(f2[b])^T,
// (B, N1, N2) fp32, ONE launch over all B samples with the L2 normalisation in the prologue and
// the temperature in the epilogue (round 4 ran an l2norm pass per operand and then a host loop of
// padded copies + one GEMM launch per sample).
//
// Workgroup = 4 waves = one sample b x 64 rows of f1 x ALL N2 columns (64-column blocks in a loop):
//   * the f1 rows are L2-normalised once per workgroup into LDS (bf16, F.normalize's output type);
//   * per 64-column block the f2 rows are normalised the same way into a second LDS tile, shared
//     by the four waves (round 5's first form re-read every f2 row from global memory in every wave
//     and every row tile, twice: ~8x the loads, 0.32 ms for a 256 x 199 x 256 map);
//   * wave w owns rows 16 w .. 16 w + 15 against the block's 64 columns: 4 blocks of 16 x 16 on
//     v_mfma_f32_16x16x32_bf16, the f2 fragment first, so each lane's four accumulators are four
//     consecutive output columns of one row -> one 16-byte store.
// Normalising a tile: thread t owns row t >> 2 and every fourth 16-byte chunk of it; the row's sum
// of squares is combined over its 4 lanes, then the chunks are re-read, scaled by
// 1 / max(||row||, eps), rounded to bf16 and stored at chunk c ^ (row & swz_mask) (the MFMA fragment
// reads, 16 rows x one chunk per lane group, are then conflict-free at 1 KB rows). Rows past
// N1 / N2 re-read the last row (in bounds) and are not stored.
#include "common.h"

namespace {

constexpr int SM_ROWS = 64;

// XOR mask of the chunk swizzle: (row & 15) when a row has a multiple of 16 chunks (D % 128 == 0,
// conflict-free at D = 512), else the largest power-of-two group of chunks D / 8 is a multiple of
// (>= 4 since D % 32 == 0), so a swizzled chunk never leaves its row
__device__ __forceinline__ int swz_mask(int D) {
  const int nc = D / 8, low = nc & -nc;
  return (low < 16 ? low : 16) - 1;
}

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

__device__ __forceinline__ void norm_tile(const bf16* __restrict__ src, int nrows, int r0, int D, float eps,
                                          bf16* __restrict__ tile) {
  const int t = threadIdx.x, row = t >> 2, t4 = t & 3;
  const int r = r0 + row < nrows ? r0 + row : nrows - 1;
  const bf16* p = src + (long long)r * D;
  const int nc = D / 8, g = swz_mask(D);
  float ss = 0.f;
  for (int c = t4; c < nc; c += 4) ss += sumsq8(*(const bf16x8*)(p + 8 * c));
  ss += __shfl_xor(ss, 1);
  ss += __shfl_xor(ss, 2);
  const float inv = 1.f / fmaxf(sqrtf(ss), eps);
  for (int c = t4; c < nc; c += 4)
    *(bf16x8*)(tile + row * D + 8 * (c ^ (row & g))) = scale8(*(const bf16x8*)(p + 8 * c), inv);
}

__global__ __launch_bounds__(256) void simmap_kernel(const bf16* __restrict__ f1, const bf16* __restrict__ f2, int N1,
                                                     int N2, int D, const float* __restrict__ temp, float eps,
                                                     float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) bf16 sm[];
  bf16* ta = sm;                      // [64][D] normalised f1 rows
  bf16* tb = sm + SM_ROWS * D;        // [64][D] normalised f2 rows of the current column block
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const long long b = blockIdx.y;
  const int m0 = blockIdx.x * SM_ROWS;
  const int m = m0 + 16 * wave + l16;
  const float t = *temp;
  norm_tile(f1 + b * N1 * (long long)D, N1, m0, D, eps, ta);
  const bf16* arow = ta + (16 * wave + l16) * D;
  const int sw = l16 & swz_mask(D);   // fragment rows 16 j + l16: row & mask == l16 & mask
  float* orow = out + (b * N1 + (m < N1 ? m : 0)) * (long long)N2;
  for (int n0 = 0; n0 < N2; n0 += SM_ROWS) {
    __syncthreads();   // the previous block's fragment reads are done before tb is rewritten
    norm_tile(f2 + b * N2 * (long long)D, N2, n0, D, eps, tb);
    __syncthreads();
    f32x4 acc[4] = {};
    for (int k = 0; k < D; k += 32) {
      const int c = k / 8 + q;
      const bf16x8 af = *(const bf16x8*)(arow + 8 * (c ^ sw));
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[cb] = mfma16(*(const bf16x8*)(tb + (16 * cb + l16) * D + 8 * (c ^ sw)), af, acc[cb]);
    }
    if (m < N1) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const int n = n0 + 16 * cb + 4 * q;
        const f32x4 v = acc[cb] * t;
        if (n + 3 < N2 && (N2 & 3) == 0) {
          *(f32x4*)(orow + n) = v;
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (n + i < N2) orow[n + i] = v[i];
        }
      }
    }
  }
}

}  // namespace

extern "C" {

// sim[b][i][j] = temp * <f1[b][i] / max(||f1[b][i]||, eps), f2[b][j] / max(||f2[b][j]||, eps)>,
// f1 (B, N1, D), f2 (B, N2, D) contiguous bf16 (D % 32 == 0, D <= 512), temp a device scalar, sim fp32.
int triad_similarity_maps(const void* f1, const void* f2, int B, int N1, int N2, int D, const float* temp, float eps,
                          float* sim, hipStream_t stream) {
  // two [64][D] bf16 tiles in LDS: D <= 512 (128 KB); the fp32 output pointer 16-byte aligned
  if (!f1 || !f2 || !temp || !sim || B <= 0 || N1 <= 0 || N2 <= 0 || D <= 0 || D % 32 || D > 512 || B > 65535 ||
      ((uintptr_t)f1 & 15) || ((uintptr_t)f2 & 15) || ((uintptr_t)sim & 15))
    return TRIAD_EINVAL;
  const size_t lds = 2 * (size_t)SM_ROWS * D * sizeof(bf16);
  // more than 64 KB of dynamic LDS: allow it once (an error here is cleared, the launch reports its own)
  static const bool attr = [] {
    if (hipFuncSetAttribute((const void*)simmap_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            2 * SM_ROWS * 512 * (int)sizeof(bf16)) != hipSuccess)
      (void)hipGetLastError();
    return true;
  }();
  (void)attr;
  hipLaunchKernelGGL(simmap_kernel, dim3((N1 + SM_ROWS - 1) / SM_ROWS, B), dim3(256), lds, stream, (const bf16*)f1,
                     (const bf16*)f2, N1, N2, D, temp, eps, sim);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

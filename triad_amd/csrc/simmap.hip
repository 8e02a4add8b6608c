// Inference similarity maps (SajayR/TRIAD model.py:355-368 compute_similarity_matrix, called by
// forward() at model.py:630-636 and viz.py:182): sim[b] = temp * normalize(f1[b]) . normalize(f2[b])^T,
// (B, N1, N2) fp32, ONE launch over all B samples with the L2 normalisation in the prologue and
// the temperature in the epilogue (round 4 ran an l2norm pass per operand and then a host loop of
// padded copies + one GEMM launch per sample).
//
// Workgroup = 4 waves = one sample b x 64 rows of f1 x ALL N2 columns (64-column blocks in a loop):
//   * wave w loads its 16 f1 rows once as MFMA A fragments (lane: one row, chunks 4 s + q, all 16
//     k steps in flight), L2-normalises them in registers (the row's sum of squares over its four
//     q lanes) and keeps them as bf16 -- F.normalize's output type;
//   * per 64-column block the f2 rows are normalised the same way into ONE 64 KB LDS tile shared by
//     the four waves (two workgroups per CU), every thread's 16 chunk loads in flight at once (round
//     5's first form re-read every f2 row from global memory in every wave and row tile, twice,
//     with one load in flight: 0.32 ms for a 256 x 199 x 256 map, 0.19 with a shared tile);
//   * 4 blocks of 16 x 16 on v_mfma_f32_16x16x32_bf16 per wave, the f2 fragment first, so each
//     lane's four accumulators are four consecutive output columns of one row -> one 16-byte store.
// The LDS tile's rows are padded by 16 bytes (D + 8 elements): a fragment read (16 rows x one
// 16-byte chunk per lane group) then covers 16 different bank quads at D = 512, and every address
// stays linear in the k step (immediate offsets; an XOR swizzle cost one address VGPR per fragment).
// Rows past N1 / N2 re-read the last row (in bounds) and are not stored. D <= 512.
#include "common.h"

namespace {

constexpr int SM_ROWS = 64;

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

constexpr int SM_KMAX = 16;   // 32-deep k steps for D <= 512

// f2 rows [r0, r0 + 64) of one sample, normalised, into the LDS tile: thread t owns row t >> 2 and
// chunks t4, t4 + 4, ... (up to 16, all loads issued before the first use)
__device__ __forceinline__ void norm_tile(const bf16* __restrict__ src, int nrows, int r0, int D, float eps,
                                          bf16* __restrict__ tile) {
  const int t = threadIdx.x, row = t >> 2, t4 = t & 3;
  const int r = r0 + row < nrows ? r0 + row : nrows - 1;
  const bf16* p = src + (long long)r * D;
  const int nc = D / 8, ld = D + 8;
  bf16x8 v[SM_KMAX];
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < SM_KMAX; ++j) {
    const int c = t4 + 4 * j;
    v[j] = c < nc ? *(const bf16x8*)(p + 8 * c) : bf16x8{};
  }
#pragma unroll
  for (int j = 0; j < SM_KMAX; ++j) {
    ss += sumsq8(v[j]);
    asm volatile("" : "+v"(v[j]));   // keep the packed bf16 live, not 8 fp32 copies (re-unpacked below)
  }
  ss += __shfl_xor(ss, 1);
  ss += __shfl_xor(ss, 2);
  const float inv = 1.f / fmaxf(sqrtf(ss), eps);
#pragma unroll
  for (int j = 0; j < SM_KMAX; ++j) {
    const int c = t4 + 4 * j;
    if (c < nc) *(bf16x8*)(tile + row * ld + 8 * c) = scale8(v[j], inv);
    if (j % 4 == 3) __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ __launch_bounds__(256, 2) void simmap_kernel(const bf16* __restrict__ f1, const bf16* __restrict__ f2,
                                                        int N1, int N2, int D, const float* __restrict__ temp,
                                                        float eps, float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) bf16 tb[];   // [64][D + 8] normalised f2 rows of a block
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const long long b = blockIdx.y;
  const int m = blockIdx.x * SM_ROWS + 16 * wave + l16;
  const int ks = D / 32;
  // this lane's A fragments: row m, chunk 4 s + q of every k step s, normalised in registers
  bf16x8 af[SM_KMAX];
  {
    const bf16* ar = f1 + (b * N1 + (m < N1 ? m : N1 - 1)) * (long long)D + 8 * q;
    float ss = 0.f;
#pragma unroll
    for (int s = 0; s < SM_KMAX; ++s) af[s] = s < ks ? *(const bf16x8*)(ar + 32 * s) : bf16x8{};
#pragma unroll
    for (int s = 0; s < SM_KMAX; ++s) {
      ss += sumsq8(af[s]);
      asm volatile("" : "+v"(af[s]));
    }
    ss += __shfl_xor(ss, 16);
    ss += __shfl_xor(ss, 32);
    const float inv = 1.f / fmaxf(sqrtf(ss), eps);
#pragma unroll
    for (int s = 0; s < SM_KMAX; ++s) {
      af[s] = scale8(af[s], inv);
      if (s % 4 == 3) __builtin_amdgcn_sched_barrier(0);
    }
  }
  const bf16* bfr = tb + l16 * (D + 8) + 8 * q;   // + (16 cb) rows + 32 s: B fragment of (cb, s)
  const float t = *temp;
  float* orow = out + (b * N1 + (m < N1 ? m : 0)) * (long long)N2;
  for (int n0 = 0; n0 < N2; n0 += SM_ROWS) {
    __syncthreads();   // the previous block's fragment reads are done before tb is rewritten
    norm_tile(f2 + b * N2 * (long long)D, N2, n0, D, eps, tb);
    __syncthreads();
    f32x4 acc[4] = {};
#pragma unroll
    for (int s = 0; s < SM_KMAX; ++s) {
      if (s < ks) {
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[cb] = mfma16(*(const bf16x8*)(bfr + 16 * cb * (D + 8) + 32 * s), af[s], acc[cb]);
      }
      if (s % 4 == 3) __builtin_amdgcn_sched_barrier(0);   // at most 16 B fragments in flight
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
  // one [64][D + 8] bf16 tile in LDS (65 KB at D = 512), the A fragments in registers: D <= 512; the
  // fp32 output pointer 16-byte aligned
  if (!f1 || !f2 || !temp || !sim || B <= 0 || N1 <= 0 || N2 <= 0 || D <= 0 || D % 32 || D > 512 || B > 65535 ||
      ((uintptr_t)f1 & 15) || ((uintptr_t)f2 & 15) || ((uintptr_t)sim & 15))
    return TRIAD_EINVAL;
  const size_t lds = (size_t)SM_ROWS * (D + 8) * sizeof(bf16);
  // more than 64 KB of dynamic LDS: allow it once (an error here is cleared, the launch reports its own)
  static const bool attr = [] {
    if (hipFuncSetAttribute((const void*)simmap_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            SM_ROWS * (512 + 8) * (int)sizeof(bf16)) != hipSuccess)
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

// Fused per-token projection head proj2(LN(proj1(h))) (SajayR/TRIAD src/model.py:32-34,68 /
// 81-83,116 / 253-255,326) under bf16 autocast semantics (model.py:483,603):
//   y1  = bf16(h . W1^T + b1)                  Linear(H -> 512), bf16 out
//   ln  = LayerNorm(y1) in fp32 (eps 1e-5), affine, then bf16 for the next Linear
//   y   = bf16(ln . W2^T + b2)                 Linear(512 -> 512), bf16 out
// One workgroup owns 64 token rows x all 512 features, so the LayerNorm row
// statistics never leave the chip and `ln` feeds the second GEMM from LDS.
// Also: LayerNorm backward, column sums (bias / affine grads) and the split-K
// reduce used by the head's backward GEMMs.
#include "common.h"

namespace {

constexpr int PM = 64;        // rows per workgroup
constexpr int PN = 512;       // projection width
constexpr int PK = 32;        // k per stage
constexpr int PWAVES = 8;     // wave w owns columns [64w, 64w+64)
constexpr int A_STAGE = PM * PK;           // 2048 elems (4 KB)
constexpr int B_STAGE = PN * PK;           // 16384 elems (32 KB)
constexpr int STAGE = A_STAGE + B_STAGE;
constexpr int LN_ELEMS = PM * PN;          // 64 KB bf16 LN output (GEMM2 A operand)

// [rows][32 k] images with 64-B rows: 16-B chunk c (0..3) of row m at c ^ ((m >> 2) & 3)
__device__ __forceinline__ int k32_off(int m, int c) { return m * PK + ((c ^ ((m >> 2) & 3)) << 3); }
// [64 rows][512 k] LN image, 1 KB rows: chunk c (0..63) at c ^ (m & 15)
__device__ __forceinline__ int ln_off(int m, int c) { return m * PN + ((c ^ (m & 15)) << 3); }

// Stage rows [r0, r0+nrows) x k [k0, k0+32) of a k-contiguous bf16 matrix into a k32 image.
// One wave-instruction covers 16 rows x 64 B. Rows >= limit read row limit-1 (masked later).
__device__ __forceinline__ void stage_k32(const bf16* __restrict__ X, long long ld, int r0, int nrows, int limit,
                                          int k0, bf16* dst, int wave, int lane) {
  const int ninst = nrows / 16;
  for (int inst = wave; inst < ninst; inst += PWAVES) {
    const int m = inst * 16 + (lane >> 2), cp = lane & 3;
    const int c = cp ^ ((m >> 2) & 3);
    int r = r0 + m;
    r = r < limit ? r : limit - 1;
    glds16(X + (size_t)r * ld + k0 + c * 8, dst + inst * 512);
  }
}

__global__ __launch_bounds__(512, 1) void projhead_fwd_kernel(
    const bf16* __restrict__ h, int M, int H, const bf16* __restrict__ W1, const float* __restrict__ b1,
    const float* __restrict__ gamma, const float* __restrict__ beta, float eps, const bf16* __restrict__ W2,
    const float* __restrict__ b2, bf16* __restrict__ y, long long ldy, bf16* __restrict__ y1_out,
    bf16* __restrict__ ln_out, float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * STAGE + LN_ELEMS + 2 * PWAVES * PM * 2];
  bf16* lnimg = lds + 2 * STAGE;
  float* red = (float*)(lnimg + LN_ELEMS);  // [PWAVES][PM]
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), h2 = lane >> 5,
            l32 = lane & 31;
  const int r0 = blockIdx.x * PM;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){};

  // ---------------- GEMM1: y1 = h . W1^T ----------------
  const int nk1 = H / PK;
  stage_k32(h, H, r0, PM, M, 0, lds, wave, lane);
  stage_k32(W1, H, 0, PN, PN, 0, lds + A_STAGE, wave, lane);
  for (int kt = 0; kt < nk1; ++kt) {
    lds_dma_barrier();
    if (kt + 1 < nk1) {
      bf16* nb = lds + ((kt + 1) & 1) * STAGE;
      stage_k32(h, H, r0, PM, M, (kt + 1) * PK, nb, wave, lane);
      stage_k32(W1, H, 0, PN, PN, (kt + 1) * PK, nb + A_STAGE, wave, lane);
    }
    const bf16* ai = lds + (kt & 1) * STAGE;
    const bf16* bi = ai + A_STAGE;
#pragma unroll
    for (int s = 0; s < PK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = *(const bf16x8*)(ai + k32_off(t * 32 + l32, 2 * s + h2));
        bfr[t] = *(const bf16x8*)(bi + k32_off(wave * 64 + t * 32 + l32, 2 * s + h2));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
    }
  }

  // ---------------- bias, bf16 rounding, LayerNorm ----------------
  // lane holds column n = wave*64 + b*32 + l32 for rows m = a*32 + (v&3) + 8(v>>2) + 4*h2.
  float colb1[2], colg[2], colbt[2];
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int n = wave * 64 + b * 32 + l32;
    colb1[b] = b1[n];
    colg[b] = gamma[n];
    colbt[b] = beta[n];
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int v = 0; v < 16; ++v) acc[a][b][v] = (float)(bf16)(acc[a][b][v] + colb1[b]);
  // row sums: over the 2 column tiles, the 32 lanes of a half, then the 8 waves (LDS)
  float mean[2][16], rstd[2][16];
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        float s;
        if (pass == 0) s = acc[a][0][v] + acc[a][1][v];
        else {
          const float d0 = acc[a][0][v] - mean[a][v], d1 = acc[a][1][v] - mean[a][v];
          s = d0 * d0 + d1 * d1;
        }
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o);  // within the 32-lane half
        const int m = a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h2;
        if (l32 == 0) red[wave * PM + m] = s;
      }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h2;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < PWAVES; ++w) t += red[w * PM + m];
        if (pass == 0) mean[a][v] = t * (1.f / PN);
        else rstd[a][v] = rsqrtf(t * (1.f / PN) + eps);
      }
    __syncthreads();
  }
  // normalise, affine, round to bf16; save y1 / ln / stats; LN image in LDS for GEMM2
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = wave * 64 + b * 32 + l32;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h2;
        const float x = acc[a][b][v];
        const bf16 lnv = (bf16)((x - mean[a][v]) * rstd[a][v] * colg[b] + colbt[b]);
        lnimg[ln_off(m, n >> 3) + (n & 7)] = lnv;
        if (r0 + m < M) {
          y1_out[(size_t)(r0 + m) * PN + n] = (bf16)x;
          ln_out[(size_t)(r0 + m) * PN + n] = lnv;
        }
      }
    }
  if (wave == 0) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h2;
        if (l32 == 0 && r0 + m < M) {
          mean_out[r0 + m] = mean[a][v];
          rstd_out[r0 + m] = rstd[a][v];
        }
      }
  }

  // ---------------- GEMM2: y = ln . W2^T + b2 ----------------
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){};
  const int nk2 = PN / PK;
  __syncthreads();  // LN image complete; staging buffers free
  stage_k32(W2, PN, 0, PN, PN, 0, lds + A_STAGE, wave, lane);
  for (int kt = 0; kt < nk2; ++kt) {
    lds_dma_barrier();
    if (kt + 1 < nk2) stage_k32(W2, PN, 0, PN, PN, (kt + 1) * PK, lds + ((kt + 1) & 1) * STAGE + A_STAGE, wave, lane);
    const bf16* bi = lds + (kt & 1) * STAGE + A_STAGE;
#pragma unroll
    for (int s = 0; s < PK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        af[t] = *(const bf16x8*)(lnimg + ln_off(t * 32 + l32, kt * 4 + 2 * s + h2));
        bfr[t] = *(const bf16x8*)(bi + k32_off(wave * 64 + t * 32 + l32, 2 * s + h2));
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
    }
  }
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int n = wave * 64 + b * 32 + l32;
    const float bias = b2[n];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h2;
        if (r0 + m < M) y[(size_t)(r0 + m) * ldy + n] = (bf16)(acc[a][b][v] + bias);
      }
  }
}

// LayerNorm backward, one wave per row (512 features, 8 per lane):
//   xh = (y1 - mean) * rstd;  g = dln * gamma
//   dy1 = rstd * (g - mean(g) - xh * mean(g * xh))     (bf16 out)
// plus per-workgroup column partials of dgamma = sum dln*xh and dbeta = sum dln.
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dln, const bf16* __restrict__ y1,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, int M, bf16* __restrict__ dy1,
                                                     float* __restrict__ dgb_part /* [grid][2][512] */) {
  __shared__ float sg[4][PN], sb[4][PN];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float pg[8], pb[8], gm[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { pg[k] = 0.f; pb[k] = 0.f; gm[k] = gamma[lane * 8 + k]; }
  for (int r = blockIdx.x * 4 + wave; r < M; r += gridDim.x * 4) {
    const float mu = mean[r], rs = rstd[r];
    const float* d = dln + (size_t)r * PN + lane * 8;
    const bf16x8 yv = *(const bf16x8*)(y1 + (size_t)r * PN + lane * 8);
    float xh[8], g[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xh[k] = ((float)yv[k] - mu) * rs;
      const float dv = d[k];
      g[k] = dv * gm[k];
      s1 += g[k];
      s2 += g[k] * xh[k];
      pg[k] += dv * xh[k];
      pb[k] += dv;
    }
    s1 = wave_sum(s1) * (1.f / PN);
    s2 = wave_sum(s2) * (1.f / PN);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)(rs * (g[k] - s1 - xh[k] * s2));
    *(bf16x8*)(dy1 + (size_t)r * PN + lane * 8) = o;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) { sg[wave][lane * 8 + k] = pg[k]; sb[wave][lane * 8 + k] = pb[k]; }
  __syncthreads();
  for (int n = threadIdx.x; n < PN; n += blockDim.x) {
    dgb_part[(size_t)blockIdx.x * 2 * PN + n] = sg[0][n] + sg[1][n] + sg[2][n] + sg[3][n];
    dgb_part[(size_t)blockIdx.x * 2 * PN + PN + n] = sb[0][n] + sb[1][n] + sb[2][n] + sb[3][n];
  }
}

// Column sums, HBM-rate form (bias gradients over 8-65 K token rows): thread = 8 consecutive
// columns (one 16-byte load per row) x a strided set of rows of the block's row slice; the row
// lanes meet in LDS; part[slice][cols] fp32. Then colsum_reduce_kernel: 64 columns x 16 slice
// lanes per block, LDS tree, out = alpha * sum (fp32 or bf16).
__global__ __launch_bounds__(256) void colsum8_kernel(const bf16* __restrict__ X, long long rows, int cols, long long ld,
                                                      int cg, float* __restrict__ part) {
  __shared__ float red[256 * 8];
  const int t = threadIdx.x, g = t % cg, rl = t / cg, nrl = 256 / cg;
  const int c8 = blockIdx.x * cg + g;
  const long long per = (rows + gridDim.y - 1) / gridDim.y;
  const long long a = blockIdx.y * per, b = min(rows, a + per);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c8 * 8 < cols && rl < nrl) {
    for (long long r = a + rl; r < b; r += nrl) {
      const bf16x8 v = *(const bf16x8*)(X + r * ld + c8 * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += (float)v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[t * 8 + i] = s[i];
  __syncthreads();
  if (rl == 0 && c8 * 8 < cols) {
    for (int l = 1; l < nrl; ++l)
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += red[(l * cg + g) * 8 + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) part[(size_t)blockIdx.y * cols + c8 * 8 + i] = s[i];
  }
}

__global__ __launch_bounds__(1024) void colsum_reduce_kernel(const float* __restrict__ part, int S, long long cols,
                                                             const float* __restrict__ alpha_p, float alpha,
                                                             int out_bf16, void* __restrict__ out) {
  __shared__ float red[16][64];
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long long c = (long long)blockIdx.x * 64 + el;
  // four independent partial sums: the loads of a thread's slices are in flight together
  // (one dependent chain of S / 16 loads made this a latency-bound 16 us launch)
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (c < cols) {
    int i = sl;
    for (; i + 48 < S; i += 64) {
      a0 += part[(size_t)i * cols + c];
      a1 += part[(size_t)(i + 16) * cols + c];
      a2 += part[(size_t)(i + 32) * cols + c];
      a3 += part[(size_t)(i + 48) * cols + c];
    }
    for (; i < S; i += 16) a0 += part[(size_t)i * cols + c];
  }
  red[sl][el] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][el];
    t *= alpha_p ? *alpha_p : alpha;
    if (out_bf16) ((bf16*)out)[c] = (bf16)t;
    else ((float*)out)[c] = t;
  }
}

__global__ __launch_bounds__(256) void sum_slabs_kernel(const float* __restrict__ slabs, int nslab, long long n,
                                                        const float* __restrict__ alpha_p, int out_bf16,
                                                        void* __restrict__ out) {
  const float alpha = alpha_p ? *alpha_p : 1.f;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;  // independent chains: loads in flight together
    int i = 0;
    for (; i + 3 < nslab; i += 4) {
      s0 += slabs[(size_t)i * n + e];
      s1 += slabs[(size_t)(i + 1) * n + e];
      s2 += slabs[(size_t)(i + 2) * n + e];
      s3 += slabs[(size_t)(i + 3) * n + e];
    }
    for (; i < nslab; ++i) s0 += slabs[(size_t)i * n + e];
    float s = ((s0 + s1) + (s2 + s3)) * alpha;
    if (out_bf16) ((bf16*)out)[e] = (bf16)s;
    else ((float*)out)[e] = s;
  }
}

}  // namespace

extern "C" {

int triad_projhead_fwd(const void* h, int M, int H, const void* W1, const float* b1, const float* gamma,
                       const float* beta, float eps, const void* W2, const float* b2, void* y, long long ldy,
                       void* y1, void* ln, float* mean, float* rstd, hipStream_t stream) {
  if (M <= 0 || H % PK || H < PK) return TRIAD_EINVAL;
  const int grid = (M + PM - 1) / PM;
  hipLaunchKernelGGL(projhead_fwd_kernel, dim3(grid), dim3(512), 0, stream, (const bf16*)h, M, H, (const bf16*)W1,
                     b1, gamma, beta, eps, (const bf16*)W2, b2, (bf16*)y, ldy, (bf16*)y1, (bf16*)ln, mean, rstd);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_ln_bwd(const float* dln, const void* y1, const float* mean, const float* rstd, const float* gamma, int M,
                 void* dy1, float* dgb_part, int nblocks, hipStream_t stream) {
  if (M <= 0 || nblocks <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(nblocks), dim3(256), 0, stream, dln, (const bf16*)y1, mean, rstd, gamma, M,
                     (bf16*)dy1, dgb_part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_sum_slabs(const float* slabs, int nslab, long long n, const float* alpha, int out_bf16, void* out,
                    hipStream_t stream) {
  if (nslab <= 0 || n <= 0) return TRIAD_EINVAL;
  if (nslab >= 16 && n <= (1 << 20)) {  // many slabs of a short vector: 16 slab lanes per element
    hipLaunchKernelGGL(colsum_reduce_kernel, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, stream, slabs, nslab, n,
                       alpha, 1.f, out_bf16, out);
    TRIAD_CHECK_LAUNCH();
    return TRIAD_OK;
  }
  long long blocks = (n + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(sum_slabs_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, slabs, nslab, n, alpha, out_bf16,
                     out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// out[c] = alpha * sum_{r < rows} X[r][c], X bf16 [rows][ld] (cols % 8 == 0, ld % 8 == 0); part:
// triad_colsum_splits(rows, cols) * cols floats of scratch; out fp32 or bf16.
int triad_colsum_splits(long long rows, int cols) {
  const int cg = cols / 8 < 256 ? cols / 8 : 256;
  const int gx = (cols / 8 + cg - 1) / cg;
  long long s = 1024 / gx;
  if (s > rows / 16) s = rows / 16;
  return (int)(s < 1 ? 1 : s);
}

int triad_colsum(const void* X, long long rows, int cols, long long ld, float* part, float alpha, int out_bf16,
                 void* out, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 8 || ld % 8 || ld < cols) return TRIAD_EINVAL;
  const int cg = cols / 8 < 256 ? cols / 8 : 256;
  const int S = triad_colsum_splits(rows, cols);
  const dim3 grid((cols / 8 + cg - 1) / cg, S);
  hipLaunchKernelGGL(colsum8_kernel, grid, dim3(256), 0, stream, (const bf16*)X, rows, cols, ld, cg, part);
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3((cols + 63) / 64), dim3(1024), 0, stream, part, S, (long long)cols,
                     (const float*)nullptr, alpha, out_bf16, out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

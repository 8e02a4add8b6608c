// Projection-head helpers: the LayerNorm forward / backward row passes of the "passes" head form
// (the "rows" form runs them in its GEMM epilogues, csrc/rowgemm.hip), column sums (bias
// gradients, also of the backbones) and the split-K slab reduce.
#include "common.h"

namespace {

constexpr int PN = 512;       // projection width

// LayerNorm(512) forward of the library-GEMM projection head, one wave per row (8 features per
// lane): mean / biased variance in fp32 over the bf16 y1 row (F.layer_norm under autocast runs in
// fp32, model.py:68/116/326), ln = bf16((y1 - mean) * rstd * gamma + beta) -- the operand autocast
// feeds projection2 -- and mean / rstd kept for the backward.
__global__ __launch_bounds__(256) void ln_fwd_kernel(const bf16* __restrict__ y1, int M, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps, bf16* __restrict__ ln,
                                                     float* __restrict__ mean, float* __restrict__ rstd) {
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float gm[8], bt[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { gm[k] = gamma[lane * 8 + k]; bt[k] = beta[lane * 8 + k]; }
  for (int r = blockIdx.x * 4 + wave; r < M; r += gridDim.x * 4) {
    const bf16x8 yv = *(const bf16x8*)(y1 + (size_t)r * PN + lane * 8);
    float x[8], s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) { x[k] = (float)yv[k]; s += x[k]; }
    const float mu = wave_sum(s) * (1.f / PN);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) { const float d = x[k] - mu; q += d * d; }
    const float rs = rsqrtf(wave_sum(q) * (1.f / PN) + eps);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)((x[k] - mu) * rs * gm[k] + bt[k]);
    *(bf16x8*)(ln + (size_t)r * PN + lane * 8) = o;
    if (lane == 0) { mean[r] = mu; rstd[r] = rs; }
  }
}

// LayerNorm backward of the library-GEMM head: dln bf16 (autocast's projection2 input gradient),
// dy1 = bf16(rstd (g - mean(g) - xh mean(g xh))), g = dln gamma, and per-workgroup column
// partials [grid][3][512] of dgamma = sum dln xh, dbeta = sum dln, db1 = sum dy1 (the layout of
// triad_projhead_bwd's colpart, reduced by triad_sum_slabs).
__global__ __launch_bounds__(256) void ln_bwd3_kernel(const bf16* __restrict__ dln, const bf16* __restrict__ y1,
                                                      const float* __restrict__ mean, const float* __restrict__ rstd,
                                                      const float* __restrict__ gamma, int M, bf16* __restrict__ dy1,
                                                      float* __restrict__ part) {
  __shared__ float sp[3][4][PN];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float pg[8], pb[8], p1[8], gm[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { pg[k] = 0.f; pb[k] = 0.f; p1[k] = 0.f; gm[k] = gamma[lane * 8 + k]; }
  for (int r = blockIdx.x * 4 + wave; r < M; r += gridDim.x * 4) {
    const float mu = mean[r], rs = rstd[r];
    const bf16x8 dv8 = *(const bf16x8*)(dln + (size_t)r * PN + lane * 8);
    const bf16x8 yv = *(const bf16x8*)(y1 + (size_t)r * PN + lane * 8);
    float xh[8], g[8], s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xh[k] = ((float)yv[k] - mu) * rs;
      const float dv = (float)dv8[k];
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
    for (int k = 0; k < 8; ++k) {
      o[k] = (bf16)(rs * (g[k] - s1 - xh[k] * s2));
      p1[k] += (float)o[k];
    }
    *(bf16x8*)(dy1 + (size_t)r * PN + lane * 8) = o;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    sp[0][wave][lane * 8 + k] = pg[k];
    sp[1][wave][lane * 8 + k] = pb[k];
    sp[2][wave][lane * 8 + k] = p1[k];
  }
  __syncthreads();
  for (int n = threadIdx.x; n < 3 * PN; n += blockDim.x) {
    const int c = n / PN, f = n - c * PN;
    part[(size_t)blockIdx.x * 3 * PN + n] = sp[c][0][f] + sp[c][1][f] + sp[c][2][f] + sp[c][3][f];
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
    // four rows' loads in flight per thread (one dependent load per iteration left the
    // 3,072-column bias gradients at ~3 TB/s, profiles/r03_bench_kernel_stats_r03e.csv)
    long long r = a + rl;
    for (; r + 3 * nrl < b; r += 4 * nrl) {
      const bf16x8 v0 = *(const bf16x8*)(X + r * ld + c8 * 8);
      const bf16x8 v1 = *(const bf16x8*)(X + (r + nrl) * ld + c8 * 8);
      const bf16x8 v2 = *(const bf16x8*)(X + (r + 2 * nrl) * ld + c8 * 8);
      const bf16x8 v3 = *(const bf16x8*)(X + (r + 3 * nrl) * ld + c8 * 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += ((float)v0[i] + (float)v1[i]) + ((float)v2[i] + (float)v3[i]);
    }
    for (; r < b; r += nrl) {
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

// ---- column sums through LDS-DMA (the step's bias gradients) -----------------
// Rows stream into LDS by 16-byte LDS-DMA (global_load_lds, as the GEMMs load their operands),
// chunks of 16 rows x 512 bytes of one column tile in a CD_SLOTS ring (CD_SLOTS - 1 chunks in
// flight while one is summed: 8 KB per chunk is too little to cover HBM latency on its own);
// the sums are VALU over LDS.
// Pass 1: bf16 X, 256-column tiles x row splits -> fp32 partials [splits][cols]; pass 2: the
// partials (fp32, 128-column tiles, one split) -> out. A thread owns 4 bytes of a row (two bf16
// columns / one fp32 column) and every other row of a chunk; the two row halves meet in LDS.
constexpr int CD_ROWS = 16;    // rows per chunk (16 x 512 B = 8 KB = 8 one-KB LDS-DMA pieces)
#ifndef TRIAD_CD_SLOTS
#define TRIAD_CD_SLOTS 4
#endif
#ifndef TRIAD_CD_WG
#define TRIAD_CD_WG 512
#endif
constexpr int CD_SLOTS = TRIAD_CD_SLOTS;   // LDS ring depth (2..4: two workgroups per CU)
constexpr int CD_WG = TRIAD_CD_WG;         // first-pass workgroup target (2 per CU)
// (Sweep, profiles/r04_colsum_dma_ring_variants.log: at 256 workgroups a 4-slot ring is no faster
// than 2 slots; 512 workgroups take 50,944 x 2,304 from 84 to 49 us; 1,024 are slower again.)
// (Measured and not kept: a 12-slot ring for the second pass, all its chunks in flight at once --
// 26.5 -> 26.2 us at 50,944 x 768, 15.6 -> 17.1 at 8,192 x 768, profiles/r04_colsum_dma_pass2.log.)
static_assert(CD_SLOTS >= 2 && CD_SLOTS <= 4, "ring depth");

// s_waitcnt with an immediate for `later` (0..L) outstanding chunks of 2 pieces per wave
template <int L>
__device__ __forceinline__ void cd_wait(int later) {
  if constexpr (L == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    if (later >= L) TRIAD_VMCNT(2 * L);
    else cd_wait<L - 1>(later);
  }
}

// Any column count that is a multiple of 8 (16 bytes of bf16): the last column tile is masked --
// its lanes past `cols` re-read the tile's last valid 16 bytes (in bounds, never summed into an
// output) and only columns < cols are written.
template <bool F32, int SLOTS>
__global__ __launch_bounds__(256) void colsum_dma_kernel(const void* __restrict__ Xv, long long rows, long long ld,
                                                         long long cols, long long per, float alpha, int out_mode,
                                                         void* __restrict__ out, long long out_ld) {
  __shared__ __attribute__((aligned(16))) char buf[SLOTS][CD_ROWS * 512];
  __shared__ float fin[2][128][2];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr int TILE = F32 ? 128 : 256;                 // columns per 512-byte row slice
  const long long c0 = (long long)blockIdx.x * TILE;
  const long long r0 = (long long)blockIdx.y * per, r1 = r0 + per < rows ? r0 + per : rows;
  const char* X = (const char*)Xv;
  const int esz = F32 ? 4 : 2;
  const int nchunk = r1 > r0 ? (int)((r1 - r0 + CD_ROWS - 1) / CD_ROWS) : 0;
  // wave w issues pieces 2w, 2w + 1 of a chunk: piece p = rows 2p, 2p + 1, lane L -> row 2p + (L >> 5),
  // 16 bytes at column offset (L & 31) * 16 B; rows past the range re-read the last row (not summed)
  constexpr int PER16 = F32 ? 4 : 8;                    // columns per 16-byte piece
  const long long last16 = cols - c0 - PER16;           // the tile's last valid piece (cols % PER16 == 0)
  const long long off16 = (lane & 31) * PER16 <= last16 ? (lane & 31) * PER16 : last16;
  auto issue = [&](int c, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int p = 2 * wave + u;
      long long r = r0 + (long long)c * CD_ROWS + 2 * p + (lane >> 5);
      r = r < r1 ? r : r1 - 1;
      glds16(X + (r * ld + c0 + off16) * esz, buf[slot] + p * 1024);
    }
  };
  const int cp = t & 127, rh = t >> 7;                  // 4-byte column slot, row parity
  float a0 = 0.f, a1 = 0.f;
  constexpr int AHEAD = SLOTS - 1;
#pragma unroll
  for (int c = 0; c < AHEAD; ++c)
    if (c < nchunk) issue(c, c);
  for (int c = 0; c < nchunk; ++c) {
    // chunk c + AHEAD refills the slot chunk c - 1 left (free since the last barrier); then wait for
    // chunk c's 2 pieces per wave while the chunks issued after it stay in flight
    if (c + AHEAD < nchunk) issue(c + AHEAD, (c + AHEAD) % SLOTS);
    cd_wait<AHEAD>(nchunk - 1 - c < AHEAD ? nchunk - 1 - c : AHEAD);
    __syncthreads();
    const char* b = buf[c % SLOTS];
    const int nr = (int)((r1 - r0 - (long long)c * CD_ROWS) < CD_ROWS ? (r1 - r0 - (long long)c * CD_ROWS) : CD_ROWS);
#pragma unroll
    for (int k = 0; k < CD_ROWS / 2; ++k) {
      const int rr = 2 * k + rh;
      if (rr < nr) {
        const unsigned v = *(const unsigned*)(b + rr * 512 + cp * 4);
        if (F32) {
          a0 += __builtin_bit_cast(float, v);
        } else {
          a0 += __builtin_bit_cast(float, v << 16);
          a1 += __builtin_bit_cast(float, v & 0xffff0000u);
        }
      }
    }
    __syncthreads();                                    // slot c % SLOTS is refilled next iteration
  }
  fin[rh][cp][0] = a0;
  fin[rh][cp][1] = a1;
  __syncthreads();
  if (rh == 0 && c0 + (F32 ? 1 : 2) * cp < cols) {
    const float s0 = fin[0][cp][0] + fin[1][cp][0], s1 = fin[0][cp][1] + fin[1][cp][1];
    if (F32) {
      const long long col = c0 + cp;
      const float v = alpha * s0;
      if (out_mode == 2) ((bf16*)out)[col] = (bf16)v;
      else ((float*)out)[(long long)blockIdx.y * out_ld + col] = v;
    } else {
      const long long col = c0 + 2 * cp;
      float* o = (float*)out + (long long)blockIdx.y * out_ld + col;   // fp32 partials of this split
      o[0] = s0;
      o[1] = s1;
    }
  }
}

}  // namespace

extern "C" {

int triad_ln_fwd(const void* y1, int M, const float* gamma, const float* beta, float eps, void* ln, float* mean,
                 float* rstd, hipStream_t stream) {
  if (M <= 0) return TRIAD_EINVAL;
  const int nb = (M + 3) / 4 < 4096 ? (M + 3) / 4 : 4096;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(nb), dim3(256), 0, stream, (const bf16*)y1, M, gamma, beta, eps, (bf16*)ln,
                     mean, rstd);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_ln_bwd3(const void* dln, const void* y1, const float* mean, const float* rstd, const float* gamma, int M,
                  void* dy1, float* part, int nblocks, hipStream_t stream) {
  if (M <= 0 || nblocks <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(ln_bwd3_kernel, dim3(nblocks), dim3(256), 0, stream, (const bf16*)dln, (const bf16*)y1, mean,
                     rstd, gamma, M, (bf16*)dy1, part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_sum_slabs(const float* slabs, int nslab, long long n, const float* alpha, int out_bf16, void* out,
                    hipStream_t stream) {
  if (nslab <= 0 || n <= 0) return TRIAD_EINVAL;
  // many slabs of a short vector (bias / LayerNorm column partials: <= 3 x 512 columns over up to
  // 1,024 slabs): 16 slab lanes per element. Long vectors (the split-K weight-gradient slabs,
  // 262,144-393,216 elements x 32 slabs) stream with one element per thread instead: the 64-column
  // blocks of colsum_reduce read them at ~2 TB/s (41 us for a visual head's two dW, r04 profile)
  if (nslab >= 16 && n <= 16384) {
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
  // 256 column-slab blocks fill the chip for the first pass; more slabs only lengthen the
  // reduce's load chains (1,024 slabs: a 24 us reduce at 512 columns, profiles/r03_projhead_kernels.log)
  long long s = 256 / gx;
  if (s > rows / 16) s = rows / 16;
  return (int)(s < 1 ? 1 : s);
}

// Column sums through LDS-DMA: part = triad_colsum_dma_splits(rows, cols) * cols floats of scratch.
// Any cols % 8 == 0 (a 256-column tile count rounded up, the last tile masked); X 16-byte aligned.
int triad_colsum_dma_splits(long long rows, int cols) {
  if (cols <= 0 || cols % 8) return 0;
  const long long tiles = (cols + 255) / 256;
  long long s = (CD_WG + tiles - 1) / tiles;            // one round of >= CD_WG workgroups
  const long long cap = rows / (4 * CD_ROWS);           // >= 4 chunks per split
  if (s > cap) s = cap;
  return (int)(s < 1 ? 1 : s);
}

int triad_colsum_dma(const void* X, long long rows, int cols, long long ld, float* part, float alpha, int out_bf16,
                     void* out, hipStream_t stream) {
  if (rows <= 0 || cols <= 0 || cols % 8 || ld % 8 || ld < cols || !part || !X || !out ||
      ((uintptr_t)X & 15))
    return TRIAD_EINVAL;
  const int S = triad_colsum_dma_splits(rows, cols);
  long long per = (rows + S - 1) / S;
  hipLaunchKernelGGL((colsum_dma_kernel<false, CD_SLOTS>), dim3((cols + 255) / 256, S), dim3(256), 0, stream, X, rows,
                     ld, (long long)cols, per, 1.f, 0, (void*)part, (long long)cols);
  TRIAD_CHECK_LAUNCH();
  hipLaunchKernelGGL((colsum_dma_kernel<true, CD_SLOTS>), dim3((cols + 127) / 128, 1), dim3(256), 0, stream,
                     (const void*)part, (long long)S, (long long)cols, (long long)cols, (long long)S, alpha,
                     out_bf16 ? 2 : 1, out, 0LL);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
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

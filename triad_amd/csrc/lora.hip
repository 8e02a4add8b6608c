// Skinny GEMMs of the ViT's LoRA adapters (SajayR/TRIAD model.py:223-266: peft LoRA r=8 on the
// DINOv2 attn.qkv / attn.proj Linears, y = W x + b + (alpha/r) B A x).
//
// With M = B*N tokens (66 816 at c3) and rank r = 8 these products are HBM-bound streams over
// one (M, K) activation, which the library GEMMs run at a fraction of bandwidth:
//   triad_rows_nt: out[m][j] = sum_k X[m][k] W[j][k]  (t = x A^T)  MFMA 16x16x32, rows of X
//                  straight from HBM, W fragments from L2, j < J <= 16;
//   triad_lora_tn: out[o][j] = alpha sum_m Y[m][o] T[m][j]  (dB = s dy^T t, dA^T = x^T dt)  MFMA,
//                  Y tiles transposed by ds_read_b64_tr_b16 out of LDS, fused with dt[m][j] = sum_o Y[m][o] Wt[j][o] over the same tiles: ONE pass over
//                  dy gives both dB and dt; a second pass over x gives dA;
//   triad_lora_update: Y[m][o] += sum_j T[m][j] Bs[o][j] in place (the rank-8 update of the base
//                  GEMM's output / of dX), one read + one write of Y.
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

constexpr int TJ = 8;  // LoRA rank

// out[e] = alpha * sum_s slab[s][e]: block = 64 consecutive elements x 16 slab lanes (coalesced
// 256-B rows per slab, 16 independent load chains per element), LDS tree over the lanes
__global__ __launch_bounds__(1024) void slab_sum_kernel(const float* __restrict__ slab, int S, long long n, float alpha,
                                                        float* __restrict__ out) {
  __shared__ float part[16][64];
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const long long e = (long long)blockIdx.x * 64 + el;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;  // independent chains: loads in flight together
  if (e < n) {
    int i = sl;
    for (; i + 48 < S; i += 64) {
      a0 += slab[i * n + e];
      a1 += slab[(i + 16) * n + e];
      a2 += slab[(i + 32) * n + e];
      a3 += slab[(i + 48) * n + e];
    }
    for (; i < S; i += 16) a0 += slab[i * n + e];
  }
  part[sl][el] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (sl == 0 && e < n) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][el];
    out[e] = alpha * t;
  }
}

// ---- rank-8 update -------------------------------------------------------------------------
// thread = 8 consecutive columns (its Bs rows held in registers as fp32) x a strided set of rows
__global__ __launch_bounds__(256) void lora_update_kernel(bf16* __restrict__ Y, long long ldy, int M, int O,
                                                          const bf16* __restrict__ T, const bf16* __restrict__ Bs) {
  const int C8 = O / 8;
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nthreads = (long long)gridDim.x * blockDim.x;
  const int rstride = (int)(nthreads / C8);
  if (g >= (long long)rstride * C8) return;
  const int c8 = (int)(g % C8);
  const int r0 = (int)(g / C8);
  float b[8][TJ];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const bf16x8 w = *(const bf16x8*)(Bs + (long long)(8 * c8 + c) * TJ);
#pragma unroll
    for (int j = 0; j < TJ; ++j) b[c][j] = (float)w[j];
  }
  for (int m = r0; m < M; m += rstride) {
    bf16* yp = Y + (long long)m * ldy + 8 * c8;
    const bf16x8 y = *(const bf16x8*)yp;
    const bf16x8 t = *(const bf16x8*)(T + (long long)m * TJ);
    float tf[TJ];
#pragma unroll
    for (int j = 0; j < TJ; ++j) tf[j] = (float)t[j];
    bf16x8 o;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      float a = (float)y[c];
#pragma unroll
      for (int j = 0; j < TJ; ++j) a = fmaf(tf[j], b[c][j], a);
      o[c] = (bf16)a;
    }
    *(bf16x8*)yp = o;
  }
}

// ---- fused dB / dt (or dA) ----------------------------------------------------------------
// Block = 8 waves over a slab of rows, in 32-row tiles; Y tiles [32][256] bf16 staged through
// LDS (register prefetch of the next chunk). Wave w owns o-tiles 2w, 2w+1 (16 columns each) of
// every 256-column chunk: out^T accumulates by v_mfma_f32_16x16x32_bf16 with A = Y^T (two
// transposed LDS reads) and B = T (rank padded to 16); dt accumulates with A = Y rows
// (ds_read_b128) and B = Wt (global, [16][O] zero-padded), reduced over the 8 waves per tile.
constexpr int TN_O = 256;                 // columns per chunk
constexpr int TN_MAXC = 12;               // O <= 3072 (O / 256 in {1, 2, 3, 4, 6, 8, 9, 12})
// 16-B chunk swizzle of a 512-B LDS row: conflict-free for 16-row b128 reads at one chunk and
// for 4-row transposed reads of two adjacent chunks
__device__ __forceinline__ int tn_swz(int r) { return ((r & 3) << 1) | ((r >> 2) & 1) | (r & 8); }
__device__ __forceinline__ int tn_off(int r, int col) {  // element offset of (row, col) in [32][256]
  return r * TN_O + ((((col >> 3) ^ tn_swz(r & 15))) << 3) + (col & 7);
}

template <bool DO_DT, int NCH>
__global__ __launch_bounds__(512, 2) void lora_tn_kernel(const bf16* __restrict__ Y, long long ldy, int M, int O,
                                                         const bf16* __restrict__ T, const bf16* __restrict__ Wt,
                                                         bf16* __restrict__ dt, int tiles_per_block,
                                                         float* __restrict__ slab) {
  __shared__ __attribute__((aligned(16))) bf16 ybuf[32 * TN_O];
  __shared__ __attribute__((aligned(16))) bf16 tbuf[32 * 16];
  __shared__ float red[DO_DT ? 8 * 32 * 16 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, g = lane >> 4;
  constexpr int nch = NCH;  // O / TN_O: the accumulators stay in registers (fully unrolled)
  f32x4 acc[NCH][2];
#pragma unroll
  for (int c = 0; c < NCH; ++c) acc[c][0] = acc[c][1] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int tile0 = blockIdx.x * tiles_per_block;
  const int ntiles = (M + 31) / 32;
  for (int tt = tile0; tt < min(ntiles, tile0 + tiles_per_block); ++tt) {
    const int m0 = tt * 32;
    // T tile [32][16] (rank padded with zeros)
    if (tid < 64) {
      const int r = tid >> 1, half = tid & 1;
      bf16x8 v = {};
      if (half == 0 && m0 + r < M) v = *(const bf16x8*)(T + (long long)(m0 + r) * TJ);
      *(bf16x8*)(tbuf + r * 16 + half * 8) = v;
    }
    // this thread's two 16-B pieces of a chunk: rows (tid >> 5) and +16, 16-B column (tid & 31)
    const int pr = tid >> 5, pc = tid & 31;
    auto ld = [&](int c, int rr) __attribute__((always_inline)) -> bf16x8 {
      const int m = m0 + rr;
      return m < M ? *(const bf16x8*)(Y + (long long)m * ldy + c * TN_O + pc * 8) : (bf16x8){};
    };
    bf16x8 nx0 = ld(0, pr), nx1 = ld(0, pr + 16);
    f32x4 dacc[2] = {(f32x4){0.f, 0.f, 0.f, 0.f}, (f32x4){0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      __syncthreads();  // previous chunk's LDS reads done (and tbuf written, for c == 0)
      *(bf16x8*)(ybuf + tn_off(pr, pc * 8)) = nx0;
      *(bf16x8*)(ybuf + tn_off(pr + 16, pc * 8)) = nx1;
      if (c + 1 < nch) { nx0 = ld(c + 1, pr); nx1 = ld(c + 1, pr + 16); }
      __syncthreads();
      // B operand of out^T: T rows 8g .. 8g+7, rank column li (transposed reads of tbuf)
      bf16x8 tb;
      {
        s16x4* rp = (s16x4*)&tb;
        const int q = li >> 2, p = li & 3;
        rp[0] = lds_tr16(tbuf + (8 * g + q) * 16 + 4 * p);
        rp[1] = lds_tr16(tbuf + (8 * g + 4 + q) * 16 + 4 * p);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int o0 = (2 * wave + u) * 16;  // column base inside the chunk
        // A = Y^T: row o0 + li, k = rows 8g .. 8g+7 -> two 4-row transposed reads
        bf16x8 ya;
        s16x4* rp = (s16x4*)&ya;
        const int q = li >> 2, p = li & 3;
        rp[0] = lds_tr16(ybuf + tn_off(8 * g + q, o0 + 4 * p));
        rp[1] = lds_tr16(ybuf + tn_off(8 * g + 4 + q, o0 + 4 * p));
        acc[c][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ya, tb, acc[c][u], 0, 0, 0);
      }
      if constexpr (DO_DT) {
        // k = this wave's 32 columns of the chunk; B = Wt[li][col .. col+7]
        const int col = c * TN_O + wave * 32 + 8 * g;
        const bf16x8 wb = *(const bf16x8*)(Wt + (long long)li * O + col);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x8 ya = *(const bf16x8*)(ybuf + tn_off(16 * h + li, wave * 32 + 8 * g));
          dacc[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ya, wb, dacc[h], 0, 0, 0);
        }
      }
    }
    if constexpr (DO_DT) {
      // dacc[h]: rank column li, rows 16h + 4g + i; sum the 8 waves' partials
#pragma unroll
      for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int i = 0; i < 4; ++i) red[(wave * 32 + 16 * h + 4 * g + i) * 16 + li] = dacc[h][i];
      __syncthreads();
      if (tid < 32 * TJ) {
        const int r = tid >> 3, j = tid & 7;
        float sum = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) sum += red[(w * 32 + r) * 16 + j];
        if (m0 + r < M) dt[(long long)(m0 + r) * TJ + j] = (bf16)sum;
      }
    }
  }
  // out^T partials: lane holds rank li (< 8 valid), columns o = 4g + i of each o-tile
  if (li < TJ) {
    float* sp = slab + (long long)blockIdx.x * O * TJ;
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int o = c * TN_O + (2 * wave + u) * 16 + 4 * g + i;
          sp[(long long)o * TJ + li] = acc[c][u][i];
        }
    }
  }
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

int triad_lora_update(void* Y, long long ldy, int M, int O, const void* T, const void* Bs, hipStream_t stream) {
  if (M <= 0 || O <= 0 || O % 8 || ldy < O || ldy % 8) return TRIAD_EINVAL;
  const int C8 = O / 8;
  long long want = (long long)C8 * 1024;  // ~1024 row groups in flight per column group
  const long long rows = (long long)M * C8;
  if (want > rows) want = rows;
  const int blocks = (int)((want + 255) / 256);
  hipLaunchKernelGGL(lora_update_kernel, dim3(blocks), dim3(256), 0, stream, (bf16*)Y, ldy, M, O, (const bf16*)T,
                     (const bf16*)Bs);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_lora_tn_blocks(int M) {
  const int tiles = (M + 31) / 32;
  return tiles < 512 ? tiles : 512;
}

int triad_lora_tn(const void* Y, long long ldy, int M, int O, const void* T, const void* Wt, void* dt, float alpha,
                  float* slabs, float* out, hipStream_t stream) {
  if (M <= 0 || O <= 0 || O % TN_O || O > TN_O * TN_MAXC || ldy < O || ldy % 8 || (Wt && !dt)) return TRIAD_EINVAL;
  const int G = triad_lora_tn_blocks(M);
  const int tiles = (M + 31) / 32;
  const int per = (tiles + G - 1) / G;
#define TN_CASE(NC)                                                                                          \
  case NC:                                                                                                   \
    if (Wt)                                                                                                  \
      hipLaunchKernelGGL((lora_tn_kernel<true, NC>), dim3(G), dim3(512), 0, stream, (const bf16*)Y, ldy, M, O,  \
                         (const bf16*)T, (const bf16*)Wt, (bf16*)dt, per, slabs);                            \
    else                                                                                                     \
      hipLaunchKernelGGL((lora_tn_kernel<false, NC>), dim3(G), dim3(512), 0, stream, (const bf16*)Y, ldy, M, O, \
                         (const bf16*)T, (const bf16*)nullptr, (bf16*)nullptr, per, slabs);                  \
    break;
  switch (O / TN_O) {
    TN_CASE(1) TN_CASE(2) TN_CASE(3) TN_CASE(4) TN_CASE(6) TN_CASE(8) TN_CASE(9) TN_CASE(12)
    default: return TRIAD_EINVAL;
  }
#undef TN_CASE
  const long long n = (long long)O * TJ;
  hipLaunchKernelGGL(slab_sum_kernel, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, stream, slabs, G, n, alpha,
                     out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

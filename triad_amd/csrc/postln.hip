// HuBERT post-LN encoder layer passes (SajayR/TRIAD model.py:29-30, 79-80: HubertModel trained
// end to end after unfreeze, bf16 autocast; transformers HubertEncoderLayer / HubertFeedForward):
//   h1 = LN1(res + dropout(attn(res)));  h2 = LN2(h1 + dropout(fc2(dropout(gelu(fc1(h1))))))
//
// Under autocast each residual step is four to six HBM passes (dropout with its stored mask, add,
// LayerNorm, casts of the fp32 result for the q / k / v / fc1 GEMMs) and twice that backward.
// Here each is one row pass:
//   dropaddln_fwd: z = res + bf16(y * keep / (1 - p)); h = LN(z) (fp32 residual) and hb = bf16(h)
//                  (the next GEMMs' operand), per-row mean / rstd;
//   dropaddln_bwd: dl = dh + dhb; dz = LN'(dl) at z (z recomputed from res, y and the mask);
//                  dres = dz, dy = bf16(bf16(dz) * keep / (1 - p)); per-block dgamma / dbeta partials;
//   geludrop_fwd / _bwd: v = bf16(bf16(gelu(u)) * keep / (1 - p)) and its gradient, no mask tensor.
// Dropout keep bits come from a counter-based hash of (seed, element pair): 16-bit uniform per
// element, keep iff >= round(p * 65536); forward and backward regenerate the same bits
// (triad_dropout_keep exposes them for tests). The roundings follow the autocast chain
// (bf16 dropout output, fp32 add / LayerNorm, bf16 GELU output).
#include "common.h"

namespace {

// hash32 / keep_pair: common.h

__device__ __forceinline__ float drop(float v, bool keep, float scale) { return keep ? (float)(bf16)(v * scale) : 0.f; }

template <int NB>
__device__ __forceinline__ void stats(const float (&v)[NB][4], float eps, float& mean, float& rstd) {
  constexpr int D = NB * 256;
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

// z for one lane's 4 x NB elements (row-major index e = row * D + c0 + c, pairs q = e / 2)
template <int NB>
__device__ __forceinline__ void load_z(const float* __restrict__ res, const bf16* __restrict__ y, long long row,
                                       int lane, unsigned seed, unsigned thr, float scale, float (&v)[NB][4]) {
  constexpr int D = NB * 256;
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    const long long e = row * D + c0;
    const f32x4 r = *(const f32x4*)(res + e);
    const bf16x4 yv = *(const bf16x4*)(y + e);
    const unsigned k = keep_pair((unsigned long long)e >> 1, seed, thr) | (keep_pair(((unsigned long long)e >> 1) + 1, seed, thr) << 2);
#pragma unroll
    for (int c = 0; c < 4; ++c) v[i][c] = r[c] + drop((float)yv[c], (k >> c) & 1u, scale);
  }
}

template <int NB>
__global__ __launch_bounds__(256) void dropaddln_fwd_kernel(const float* __restrict__ res, const bf16* __restrict__ y,
                                                            const float* __restrict__ w, const float* __restrict__ b,
                                                            float eps, int M, unsigned seed, unsigned thr, float scale,
                                                            float* __restrict__ h, bf16* __restrict__ hb,
                                                            float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int D = NB * 256;
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  float v[NB][4];
  load_z<NB>(res, y, row, lane, seed, thr, scale, v);
  float mean, rstd;
  stats<NB>(v, eps, mean, rstd);
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int c0 = i * 256 + lane * 4;
    const f32x4 wv = *(const f32x4*)(w + c0);
    const f32x4 bv = *(const f32x4*)(b + c0);
    f32x4 o;
    bf16x4 ob;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      o[c] = (v[i][c] - mean) * rstd * wv[c] + bv[c];
      ob[c] = (bf16)o[c];
    }
    *(f32x4*)(h + row * D + c0) = o;
    *(bf16x4*)(hb + row * D + c0) = ob;
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// grid-stride over rows (wave = row); dgamma / dbeta partials per block: part[blk][0 / 1][D]
template <int NB>
__global__ __launch_bounds__(256) void dropaddln_bwd_kernel(const float* __restrict__ dh, const bf16* __restrict__ dhb,
                                                            const float* __restrict__ res, const bf16* __restrict__ y,
                                                            const float* __restrict__ mean_in,
                                                            const float* __restrict__ rstd_in, const float* __restrict__ w,
                                                            int M, unsigned seed, unsigned thr, float scale,
                                                            float* __restrict__ dres, bf16* __restrict__ dy,
                                                            float* __restrict__ part) {
  constexpr int D = NB * 256;
  __shared__ float red[4][2][D];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float gw[NB][4] = {}, gb[NB][4] = {};
  for (long long row = (long long)blockIdx.x * 4 + wave; row < M; row += (long long)gridDim.x * 4) {
    float z[NB][4];
    load_z<NB>(res, y, row, lane, seed, thr, scale, z);
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NB][4], wd[NB][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c0 = i * 256 + lane * 4;
      const long long e = row * D + c0;
      f32x4 d = dh ? *(const f32x4*)(dh + e) : (f32x4){0.f, 0.f, 0.f, 0.f};
      if (dhb) {
        const bf16x4 t = *(const bf16x4*)(dhb + e);
#pragma unroll
        for (int c = 0; c < 4; ++c) d[c] += (float)t[c];
      }
      const f32x4 wv = *(const f32x4*)(w + c0);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        xh[i][c] = (z[i][c] - mean) * rstd;
        gw[i][c] = fmaf(d[c], xh[i][c], gw[i][c]);
        gb[i][c] += d[c];
        wd[i][c] = wv[c] * d[c];
        s1 += wd[i][c];
        s2 = fmaf(wd[i][c], xh[i][c], s2);
      }
    }
    const float c1 = wave_sum(s1) / D, c2 = wave_sum(s2) / D;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int c0 = i * 256 + lane * 4;
      const long long e = row * D + c0;
      const unsigned k = keep_pair((unsigned long long)e >> 1, seed, thr) | (keep_pair(((unsigned long long)e >> 1) + 1, seed, thr) << 2);
      f32x4 dz;
      bf16x4 yb;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        dz[c] = rstd * (wd[i][c] - c1 - xh[i][c] * c2);
        yb[c] = (bf16)drop((float)(bf16)dz[c], (k >> c) & 1u, scale);
      }
      *(f32x4*)(dres + e) = dz;
      *(bf16x4*)(dy + e) = yb;
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      red[wave][0][i * 256 + lane * 4 + c] = gw[i][c];
      red[wave][1][i * 256 + lane * 4 + c] = gb[i][c];
    }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * D; t += 256) {
    const int which = t / D, col = t % D;
    part[((long long)blockIdx.x * 2 + which) * D + col] =
        red[0][which][col] + red[1][which][col] + red[2][which][col] + red[3][which][col];
  }
}

constexpr float kAlpha = 0.70710678118654752440f;                 // M_SQRT1_2
constexpr float kBeta = 1.12837916709551257390f * 0.70710678118654752440f * 0.5f;  // M_2_SQRTPI * M_SQRT1_2 / 2

__device__ __forceinline__ float gelu_val(float x) { return 0.5f * x * (1.0f + erff(x * kAlpha)); }
__device__ __forceinline__ float gelu_slope(float x) {  // aten gelu_backward's factor: cdf + x * pdf
  const float cdf = 0.5f * (1.0f + erff(x * kAlpha));
  const float pdf = expf(-0.5f * x * x) * kBeta;
  return cdf + x * pdf;
}

// GELU of a bf16 input has only 65536 possible arguments, so the erf / exp work (~28 VALU
// instructions per element, which made the pass VALU-bound at ~60 % of HBM rate) is done once
// into a table: entry i covers the bf16 pattern with exponent field GL_E0 + i / 256, sign
// (i >> 7) & 1, mantissa i & 127, i.e. every finite |x| in [2^-40, 2^6); other patterns (zero,
// tiny, huge, inf / NaN) take the direct formula. Values are computed by the same device code,
// so table and formula agree bit for bit. Layout: GL_N fp32 slopes, then GL_N bf16 values.
constexpr int GL_E0 = 127 - 40, GL_NE = 46, GL_N = GL_NE * 256;
constexpr int GL_BYTES = GL_N * 4 + GL_N * 2;

__device__ __forceinline__ int gl_index(unsigned bits) {
  const int idx = (int)((bits >> 7) & 255u) - GL_E0;
  return (unsigned)idx < (unsigned)GL_NE ? (idx << 8) | (int)(bits >> 8 & 128u) | (int)(bits & 127u) : -1;
}

__global__ __launch_bounds__(256) void gelu_table_kernel(float* __restrict__ slope, bf16* __restrict__ val) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= GL_N) return;
  const unsigned bits = ((unsigned)(i >> 7 & 1) << 15) | ((unsigned)(GL_E0 + (i >> 8)) << 7) | (unsigned)(i & 127);
  const float x = __uint_as_float(bits << 16);
  slope[i] = gelu_slope(x);
  val[i] = (bf16)gelu_val(x);
}

__device__ __forceinline__ unsigned bf16_bits(bf16 v) { return (unsigned)__builtin_bit_cast(unsigned short, v); }

// Persistent passes (grid ~ a few blocks per CU, table staged in LDS once per block), thread =
// 8 consecutive elements (4 pairs) per iteration; DROP = false: p = 0 (plain GELU, no hash).
// TABLE = false: the direct formula (no table buffer given).
constexpr int GL_NT = 512;
constexpr int GL_BPC = 2;  // persistent blocks per CU

template <bool DROP, bool TABLE>
__global__ __launch_bounds__(GL_NT) void geludrop_fwd_kernel(const bf16* __restrict__ u, long long n, unsigned seed,
                                                             unsigned thr, float scale, const bf16* __restrict__ tval,
                                                             bf16* __restrict__ v) {
  __shared__ bf16 tab[TABLE ? GL_N : 1];
  if constexpr (TABLE) {
    for (int i = threadIdx.x * 8; i < GL_N; i += GL_NT * 8) *(bf16x8*)(tab + i) = *(const bf16x8*)(tval + i);
    __syncthreads();
  }
  for (long long e0 = ((long long)blockIdx.x * GL_NT + threadIdx.x) * 8; e0 < n; e0 += (long long)gridDim.x * GL_NT * 8) {
    const bf16x8 x = *(const bf16x8*)(u + e0);
    bf16x8 o;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const unsigned k = DROP ? keep_pair((unsigned long long)(e0 >> 1) + p, seed, thr) : 3u;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16 xb = x[2 * p + c];
        bf16 g;
        const int idx = TABLE ? gl_index(bf16_bits(xb)) : -1;
        if (idx >= 0) g = tab[idx];
        else g = (bf16)gelu_val((float)xb);
        o[2 * p + c] = DROP ? (bf16)drop((float)g, (k >> c) & 1u, scale) : g;
      }
    }
    *(bf16x8*)(v + e0) = o;
  }
}

template <bool DROP, bool TABLE>
__global__ __launch_bounds__(GL_NT) void geludrop_bwd_kernel(const bf16* __restrict__ u, const bf16* __restrict__ dv,
                                                             long long n, unsigned seed, unsigned thr, float scale,
                                                             const float* __restrict__ tslope, bf16* __restrict__ du) {
  __shared__ float tab[TABLE ? GL_N : 1];
  if constexpr (TABLE) {
    for (int i = threadIdx.x * 4; i < GL_N; i += GL_NT * 4) *(f32x4*)(tab + i) = *(const f32x4*)(tslope + i);
    __syncthreads();
  }
  for (long long e0 = ((long long)blockIdx.x * GL_NT + threadIdx.x) * 8; e0 < n; e0 += (long long)gridDim.x * GL_NT * 8) {
    const bf16x8 x = *(const bf16x8*)(u + e0);
    const bf16x8 d = *(const bf16x8*)(dv + e0);
    bf16x8 o;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const unsigned k = DROP ? keep_pair((unsigned long long)(e0 >> 1) + p, seed, thr) : 3u;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const bf16 xb = x[2 * p + c];
        const float dg = DROP ? drop((float)d[2 * p + c], (k >> c) & 1u, scale) : (float)d[2 * p + c];  // dropout bwd
        const int idx = TABLE ? gl_index(bf16_bits(xb)) : -1;
        const float sl = idx >= 0 ? tab[idx] : gelu_slope((float)xb);
        o[2 * p + c] = (bf16)(dg * sl);
      }
    }
    *(bf16x8*)(du + e0) = o;
  }
}

int gl_blocks(long long n) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  const long long need = (n / 8 + GL_NT - 1) / GL_NT;
  return (int)(need < (long long)GL_BPC * cus ? need : (long long)GL_BPC * cus);
}

__global__ __launch_bounds__(256) void dropout_keep_kernel(long long n, unsigned seed, unsigned thr,
                                                           unsigned char* __restrict__ out) {
  const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  out[e] = (keep_pair((unsigned long long)e >> 1, seed, thr) >> (e & 1)) & 1u;
}

unsigned drop_thr(float p) { return triad_drop_thr(p); }

}  // namespace

extern "C" {

// h = LN(res + dropout(y)) fp32 and hb = bf16(h); res fp32 [M][D], y bf16 [M][D]; D % 256 == 0.
int triad_dropaddln_fwd(const float* res, const void* y, const float* w, const float* b, float eps, int M, int D,
                        float p, unsigned seed, float* h, void* hb, float* mean, float* rstd, hipStream_t stream) {
  if (M <= 0 || D % 256 || D > 1024 || p < 0.f || p >= 1.f) return TRIAD_EINVAL;
  const float scale = 1.f / (1.f - p);
  const dim3 grid((M + 3) / 4);
#define DAL_F(NB)                                                                                                  \
  if (D == NB * 256) {                                                                                             \
    hipLaunchKernelGGL(dropaddln_fwd_kernel<NB>, grid, dim3(256), 0, stream, res, (const bf16*)y, w, b, eps, M, seed, \
                       drop_thr(p), scale, h, (bf16*)hb, mean, rstd);                                              \
    TRIAD_CHECK_LAUNCH();                                                                                          \
    return TRIAD_OK;                                                                                               \
  }
  DAL_F(1) DAL_F(2) DAL_F(3) DAL_F(4)
#undef DAL_F
  return TRIAD_EINVAL;
}

int triad_dropaddln_bwd_blocks(int M) { return M < 4 * 1024 ? (M + 3) / 4 : 1024; }

// dres = LN'(dh + dhb) (either may be NULL), dy = dropout'(bf16(dres)); part: blocks x 2 x D
// fp32 dgamma / dbeta partials (triad_dropaddln_bwd_blocks(M) blocks).
int triad_dropaddln_bwd(const float* dh, const void* dhb, const float* res, const void* y, const float* mean,
                        const float* rstd, const float* w, int M, int D, float p, unsigned seed, float* dres, void* dy,
                        float* part, hipStream_t stream) {
  if (M <= 0 || D % 256 || D > 1024 || p < 0.f || p >= 1.f) return TRIAD_EINVAL;
  const float scale = 1.f / (1.f - p);
  const dim3 grid(triad_dropaddln_bwd_blocks(M));
#define DAL_B(NB)                                                                                                  \
  if (D == NB * 256) {                                                                                             \
    hipLaunchKernelGGL(dropaddln_bwd_kernel<NB>, grid, dim3(256), 0, stream, dh, (const bf16*)dhb, res,             \
                       (const bf16*)y, mean, rstd, w, M, seed, drop_thr(p), scale, dres, (bf16*)dy, part);         \
    TRIAD_CHECK_LAUNCH();                                                                                          \
    return TRIAD_OK;                                                                                               \
  }
  DAL_B(1) DAL_B(2) DAL_B(3) DAL_B(4)
#undef DAL_B
  return TRIAD_EINVAL;
}

// Table for the GELU passes below (caller-owned device buffer of triad_gelu_table_bytes() bytes,
// built once per device by triad_gelu_table; a NULL table makes the passes use the formula).
long long triad_gelu_table_bytes(void) { return GL_BYTES; }

int triad_gelu_table(void* table, hipStream_t stream) {
  if (!table) return TRIAD_EINVAL;
  hipLaunchKernelGGL(gelu_table_kernel, dim3((GL_N + 255) / 256), dim3(256), 0, stream, (float*)table,
                     (bf16*)((char*)table + GL_N * 4));
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// v = dropout(gelu(u)) over n bf16 elements (n % 8 == 0); p = 0: plain exact-erf GELU (aten's roundings)
int triad_geludrop_fwd(const void* u, long long n, float p, unsigned seed, const void* table, void* v,
                       hipStream_t stream) {
  if (n <= 0 || n % 8 || p < 0.f || p >= 1.f) return TRIAD_EINVAL;
  const bf16* tv = table ? (const bf16*)((const char*)table + GL_N * 4) : nullptr;
  auto kern = p > 0.f ? (table ? geludrop_fwd_kernel<true, true> : geludrop_fwd_kernel<true, false>)
                      : (table ? geludrop_fwd_kernel<false, true> : geludrop_fwd_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(gl_blocks(n)), dim3(GL_NT), 0, stream, (const bf16*)u, n, seed, drop_thr(p),
                     1.f / (1.f - p), tv, (bf16*)v);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_geludrop_bwd(const void* u, const void* dv, long long n, float p, unsigned seed, const void* table, void* du,
                       hipStream_t stream) {
  if (n <= 0 || n % 8 || p < 0.f || p >= 1.f) return TRIAD_EINVAL;
  auto kern = p > 0.f ? (table ? geludrop_bwd_kernel<true, true> : geludrop_bwd_kernel<true, false>)
                      : (table ? geludrop_bwd_kernel<false, true> : geludrop_bwd_kernel<false, false>);
  hipLaunchKernelGGL(kern, dim3(gl_blocks(n)), dim3(GL_NT), 0, stream, (const bf16*)u, (const bf16*)dv, n, seed,
                     drop_thr(p), 1.f / (1.f - p), (const float*)table, (bf16*)du);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// keep bit of each of n elements (u8 0 / 1) for the given seed and p (test / debug view of the masks)
int triad_dropout_keep(long long n, float p, unsigned seed, void* out, hipStream_t stream) {
  if (n <= 0 || p < 0.f || p >= 1.f) return TRIAD_EINVAL;
  hipLaunchKernelGGL(dropout_keep_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, seed,
                     drop_thr(p), (unsigned char*)out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

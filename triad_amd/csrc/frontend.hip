// HuBERT conv feature encoder, layer 0 (SajayR/TRIAD model.py:29-30,66 -> transformers
// HubertGroupNormConvLayer): GroupNorm(num_groups = C) + exact GELU over the conv output,
// fused, in channels-last (B, T, C) bf16 layout.
//
// GroupNorm with one channel per group normalises every (sample, channel) over time. Under the
// reference's bf16 autocast the norm runs in fp32 and GELU on its fp32 output; the next conv
// casts to bf16. Here the statistics and the whole elementwise chain are fp32 in registers
// and only the bf16 result is stored: bf16(gelu(gn(x))) -- the value the next conv reads.
//
// Layout: x[b][t][c], C % 8 == 0 and C / 8 a divisor of 256 (HuBERT: C = 512). One thread owns
// 8 channels (one 16-byte vector) of a time row; a 256-thread block covers 256 / (C/8) rows per
// sweep over a chunk of CHUNK time steps. HBM-bound: fwd reads x twice and writes y once; bwd
// reads x, dy twice and writes dx once.
#include "common.h"

namespace {

constexpr int CHUNK = 128;
constexpr int NT = 256;

struct V8 {
  float v[8];
};

__device__ __forceinline__ V8 load8(const bf16* p) {
  const bf16x8 r = *(const bf16x8*)p;
  V8 o;
#pragma unroll
  for (int i = 0; i < 8; ++i) o.v[i] = (float)r[i];
  return o;
}

__device__ __forceinline__ void store8(bf16* p, const V8& x) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (bf16)x.v[i];
  *(bf16x8*)p = r;
}

__device__ __forceinline__ float gelu(float z) { return 0.5f * z * (1.f + erff(z * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float z) {
  return 0.5f * (1.f + erff(z * 0.70710678118654752f)) + z * 0.39894228040143268f * __expf(-0.5f * z * z);
}

// partial[b][chunk][c] = (sum, sumsq) over the chunk's rows (fp32; < CHUNK terms each)
// MODE 0: x itself (forward statistics)
// MODE 1: (dz, dz * xhat) with dz = dy * gelu'(xhat * gamma + beta) (backward sums)
template <int MODE>
__global__ __launch_bounds__(NT) void chgn_sums_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                       int T, int Tp, int C, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd,
                                                       const float* __restrict__ gamma,
                                                       const float* __restrict__ beta, float2* __restrict__ part) {
  __shared__ float2 red[NT * 8];
  const int b = blockIdx.y, chunk = blockIdx.x, nchunk = gridDim.x;
  const int tpr = C / 8;                // threads per row
  const int rows = NT / tpr;            // rows per sweep
  const int cg = threadIdx.x % tpr, r0 = threadIdx.x / tpr;
  const int c0 = cg * 8;
  float s[8], q[8], mu[8], rs[8], g[8], be[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s[i] = 0.f;
    q[i] = 0.f;
    if (MODE == 1) {
      mu[i] = mean[(size_t)b * C + c0 + i];
      rs[i] = rstd[(size_t)b * C + c0 + i];
      g[i] = gamma[c0 + i];
      be[i] = beta[c0 + i];
    }
  }
  const int t1 = min(T, (chunk + 1) * CHUNK);
  for (int t = chunk * CHUNK + r0; t < t1; t += rows) {
    const size_t off = ((size_t)b * Tp + t) * C + c0;
    const V8 xv = load8(x + off);
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += xv.v[i];
        q[i] = fmaf(xv.v[i], xv.v[i], q[i]);
      }
    } else {
      const V8 dv = load8(dy + off);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (xv.v[i] - mu[i]) * rs[i];
        const float dz = dv.v[i] * gelu_grad(fmaf(xh, g[i], be[i]));
        s[i] += dz;
        q[i] = fmaf(dz, xh, q[i]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[threadIdx.x * 8 + i] = make_float2(s[i], q[i]);
  __syncthreads();
  // one thread per channel: sum the `rows` row-groups
  for (int c = threadIdx.x; c < C; c += NT) {
    const int g8 = c / 8, i = c % 8;
    float2 acc = make_float2(0.f, 0.f);
    for (int r = 0; r < rows; ++r) {
      const float2 v = red[(r * tpr + g8) * 8 + i];
      acc.x += v.x;
      acc.y += v.y;
    }
    part[((size_t)b * nchunk + chunk) * C + c] = acc;
  }
}

// Forward finalize: mean / rstd per (b, c) from the chunk partials (double accumulation).
__global__ void chgn_stats_kernel(const float2* __restrict__ part, int nchunk, int T, int C, float eps,
                                  float* __restrict__ mean, float* __restrict__ rstd) {
  const int b = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const float2 v = part[((size_t)b * nchunk + k) * C + c];
    s += v.x;
    q += v.y;
  }
  const double m = s / T;
  double var = q / T - m * m;
  if (var < 0.0) var = 0.0;
  mean[(size_t)b * C + c] = (float)m;
  rstd[(size_t)b * C + c] = (float)(1.0 / sqrt(var + (double)eps));
}

// Backward finalize, per (b, c): cA = gamma * sum(dz) / T, cB = gamma * sum(dz * xhat) / T into
// coef[b][c] (float2); per-(b, c) totals into tot[b][c] for dgamma / dbeta.
__global__ void chgn_bwd_coef_kernel(const float2* __restrict__ part, int nchunk, int T, int C,
                                     const float* __restrict__ gamma, float2* __restrict__ coef,
                                     double2* __restrict__ tot) {
  const int b = blockIdx.y, c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int k = 0; k < nchunk; ++k) {
    const float2 v = part[((size_t)b * nchunk + k) * C + c];
    s += v.x;
    q += v.y;
  }
  const double gm = gamma[c];
  coef[(size_t)b * C + c] = make_float2((float)(gm * s / T), (float)(gm * q / T));
  tot[(size_t)b * C + c] = make_double2(s, q);
}

// dgamma[c] = sum_b sum(dz * xhat), dbeta[c] = sum_b sum(dz)
__global__ void chgn_param_grad_kernel(const double2* __restrict__ tot, int B, int C, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < B; ++b) {
    const double2 v = tot[(size_t)b * C + c];
    s += v.x;
    q += v.y;
  }
  dgamma[c] = (float)q;
  dbeta[c] = (float)s;
}

// MODE 0: y = gelu(xhat * gamma + beta)
// MODE 1: dx = rstd * (dz * gamma - cA - xhat * cB)
template <int MODE>
__global__ __launch_bounds__(NT) void chgn_apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        int T, int Tp, int C, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd,
                                                        const float* __restrict__ gamma,
                                                        const float* __restrict__ beta,
                                                        const float2* __restrict__ coef, bf16* __restrict__ out) {
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int tpr = C / 8;
  const int rows = NT / tpr;
  const int cg = threadIdx.x % tpr, r0 = threadIdx.x / tpr;
  const int c0 = cg * 8;
  float mu[8], rs[8], g[8], be[8], ca[8], cb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    mu[i] = mean[(size_t)b * C + c0 + i];
    rs[i] = rstd[(size_t)b * C + c0 + i];
    g[i] = gamma[c0 + i];
    be[i] = beta[c0 + i];
    if (MODE == 1) {
      const float2 k = coef[(size_t)b * C + c0 + i];
      ca[i] = k.x;
      cb[i] = k.y;
    }
  }
  const int t1 = min(T, (chunk + 1) * CHUNK);
  if (chunk == gridDim.x - 1) {  // padding frames T .. Tp-1 of the sample: zeros (finite, no gradient)
    V8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z.v[i] = 0.f;
    for (int t = T + r0; t < Tp; t += rows) store8(out + ((size_t)b * Tp + t) * C + c0, z);
  }
  for (int t = chunk * CHUNK + r0; t < t1; t += rows) {
    const size_t off = ((size_t)b * Tp + t) * C + c0;
    const V8 xv = load8(x + off);
    V8 o;
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) o.v[i] = gelu(fmaf((xv.v[i] - mu[i]) * rs[i], g[i], be[i]));
    } else {
      const V8 dv = load8(dy + off);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float xh = (xv.v[i] - mu[i]) * rs[i];
        const float dz = dv.v[i] * gelu_grad(fmaf(xh, g[i], be[i]));
        o.v[i] = rs[i] * (dz * g[i] - ca[i] - xh * cb[i]);
      }
    }
    store8(out + off, o);
  }
}

// ---- conv0 + GroupNorm + GELU forward with conv0 recomputed from the waveform ---------------
// HuBERT's conv layer 0 (1 -> C channels, kernel 10, stride 5, no bias) has 10 taps per output:
// recomputing y0[b][t][c] = bf16(sum_j w[c][j] s[b][5t + j]) from the (bf16) waveform costs 10
// FMAs per element where reading y0 costs 2 bytes. The forward therefore never reads y0: MODE 0
// = GroupNorm statistics (chunk partials, finalised by chgn_stats_kernel), MODE 1 = output
// h = bf16(gelu(gn(y0))) plus y0 itself for the backward (chgn_*<1> over y0 and dy, which is
// HBM-bound there; recomputing y0 and its GELU' twice made the backward VALU-bound -- measured).
// The block stages its rows' waveform span in LDS (fp32).
constexpr int C0_K = 10, C0_S = 5;

template <int MODE>
__global__ __launch_bounds__(NT) void c0gn_kernel(const bf16* __restrict__ wave, long long Lp,
                                                  const bf16* __restrict__ w0, int T, int Tp, int C,
                                                  const float* __restrict__ mean, const float* __restrict__ rstd,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  bf16* __restrict__ out, bf16* __restrict__ y0out,
                                                  float2* __restrict__ part) {
  __shared__ float smp[C0_S * CHUNK + C0_K];
  __shared__ float2 red[MODE == 0 ? NT * 8 : 1];
  const int b = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int tpr = C / 8, rows = NT / tpr;
  const int cg = threadIdx.x % tpr, r0 = threadIdx.x / tpr;
  const int c0 = cg * 8;
  const int t0 = blk * CHUNK, t1 = min(T, t0 + CHUNK);
  const int nsmp = (t1 > t0) ? C0_S * (t1 - t0 - 1) + C0_K : 0;
  for (int i = threadIdx.x; i < nsmp; i += NT) smp[i] = (float)wave[(long long)b * Lp + (long long)C0_S * t0 + i];
  // the thread's 8 channels x 10 taps = 160 contiguous bytes at a 32-byte-aligned offset
  // (c0 % 8 == 0), loaded as ten ALIGNED 16-byte vectors (element-wise loads let hipcc merge them
  // into dwordx3 / dwordx4 loads at 2-byte alignment). Round 3 changed this load form together with
  // the build-wide removal of packed-FP32 ops when this kernel returned wrong values in lanes 48-63
  // beside a co-resident 128 x 128 GEMM; round 4's isolated probes of both instruction classes were
  // clean, so neither is the established cause (the product runs one stream)
  float w[8][C0_K];
  {
    bf16x8 wv[C0_K];
#pragma unroll
    for (int q = 0; q < C0_K; ++q) wv[q] = *(const bf16x8*)(w0 + c0 * C0_K + 8 * q);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < C0_K; ++j) w[i][j] = (float)wv[(i * C0_K + j) >> 3][(i * C0_K + j) & 7];
  }
  float mu[8], rs[8], g[8], be[8], s[8], q[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    s[i] = 0.f;
    q[i] = 0.f;
    if (MODE == 1) {
      mu[i] = mean[(size_t)b * C + c0 + i];
      rs[i] = rstd[(size_t)b * C + c0 + i];
      g[i] = gamma[c0 + i];
      be[i] = beta[c0 + i];
    }
  }
  __syncthreads();
  if (MODE == 1 && blk == nblk - 1) {  // padding frames T .. Tp-1: zeros
    bf16x8 z;
#pragma unroll
    for (int i = 0; i < 8; ++i) z[i] = (bf16)0.f;
    for (int t = T + r0; t < Tp; t += rows) {
      *(bf16x8*)(out + ((size_t)b * Tp + t) * C + c0) = z;
      *(bf16x8*)(y0out + ((size_t)b * Tp + t) * C + c0) = z;
    }
  }
  for (int t = t0 + r0; t < t1; t += rows) {
    const float* sp = smp + C0_S * (t - t0);
    float sv[C0_K];
#pragma unroll
    for (int j = 0; j < C0_K; ++j) sv[j] = sp[j];
    float y[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float a = 0.f;
#pragma unroll
      for (int j = 0; j < C0_K; ++j) a = fmaf(w[i][j], sv[j], a);
      y[i] = (float)(bf16)a;  // the bf16 conv output autocast's conv would store
    }
    if (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        s[i] += y[i];
        q[i] = fmaf(y[i], y[i], q[i]);
      }
    } else {
      const size_t off = ((size_t)b * Tp + t) * C + c0;
      bf16x8 o, yb;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        o[i] = (bf16)gelu(fmaf((y[i] - mu[i]) * rs[i], g[i], be[i]));
        yb[i] = (bf16)y[i];
      }
      *(bf16x8*)(out + off) = o;
      *(bf16x8*)(y0out + off) = yb;
    }
  }
  if (MODE == 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) red[threadIdx.x * 8 + i] = make_float2(s[i], q[i]);
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
      const int g8 = c / 8, i = c % 8;
      float2 acc = make_float2(0.f, 0.f);
      for (int r = 0; r < rows; ++r) {
        const float2 v = red[(r * tpr + g8) * 8 + i];
        acc.x += v.x;
        acc.y += v.y;
      }
      part[((size_t)b * nblk + blk) * C + c] = acc;
    }
  }
}

// dW0[c][j] = sum_{b, t < T} dy0[b][t][c] * s[b][5t + j]: conv0's weight gradient straight from the
// waveform windows (a K = 3.3 M-row, 10-column contraction the library GEMM runs at < 1/3 of HBM
// rate). Block = 1024 rows of one sample, waveform span in LDS, 8 channels x 10 taps per thread;
// row lanes summed through LDS into per-block partials dwpart[b * nblk + blk][c * 10 + j].
constexpr int C0_DW_ROWS = 1024;

__global__ __launch_bounds__(NT) void c0dw_kernel(const bf16* __restrict__ wave, long long Lp, const bf16* __restrict__ dy,
                                                  int T, int Tp, int C, float* __restrict__ dwpart) {
  __shared__ float smp[C0_S * C0_DW_ROWS + C0_K];
  __shared__ float red[NT * 8 * 2];
  const int b = blockIdx.y, blk = blockIdx.x, nblk = gridDim.x;
  const int tpr = C / 8, rows = NT / tpr;
  const int cg = threadIdx.x % tpr, r0 = threadIdx.x / tpr;
  const int c0 = cg * 8;
  const int t0 = blk * C0_DW_ROWS, t1 = min(T, t0 + C0_DW_ROWS);
  const int nsmp = (t1 > t0) ? C0_S * (t1 - t0 - 1) + C0_K : 0;
  for (int i = threadIdx.x; i < nsmp; i += NT) smp[i] = (float)wave[(long long)b * Lp + (long long)C0_S * t0 + i];
  __syncthreads();
  float dw[8][C0_K];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < C0_K; ++j) dw[i][j] = 0.f;
  for (int t = t0 + r0; t < t1; t += rows) {
    const V8 dv = load8(dy + ((size_t)b * Tp + t) * C + c0);
    const float* sp = smp + C0_S * (t - t0);
#pragma unroll
    for (int j = 0; j < C0_K; ++j) {
      const float sj = sp[j];
#pragma unroll
      for (int i = 0; i < 8; ++i) dw[i][j] = fmaf(dv.v[i], sj, dw[i][j]);
    }
  }
  float* dst = dwpart + ((size_t)b * nblk + blk) * C * C0_K;
#pragma unroll
  for (int j0 = 0; j0 < C0_K; j0 += 2) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      red[(threadIdx.x * 8 + i) * 2] = dw[i][j0];
      red[(threadIdx.x * 8 + i) * 2 + 1] = dw[i][j0 + 1];
    }
    __syncthreads();
    for (int c = threadIdx.x; c < C; c += NT) {
      const int g8 = c / 8, i = c % 8;
      float a0 = 0.f, a1 = 0.f;
      for (int r = 0; r < rows; ++r) {
        a0 += red[((r * tpr + g8) * 8 + i) * 2];
        a1 += red[((r * tpr + g8) * 8 + i) * 2 + 1];
      }
      dst[c * C0_K + j0] = a0;
      dst[c * C0_K + j0 + 1] = a1;
    }
  }
}

bool shape_ok(int B, int T, int C) {
  return B > 0 && T > 0 && C > 0 && C % 8 == 0 && NT % (C / 8) == 0;
}

}  // namespace

extern "C" {

long long triad_chgn_workspace_bytes(int B, int T, int C) {
  const long long nchunk = (T + CHUNK - 1) / CHUNK;
  // chunk partials (float2) + backward coefficients (float2) + per-(b, c) totals (double2)
  return (long long)B * nchunk * C * 8 + (long long)B * C * 8 + (long long)B * C * 16;
}

int triad_chgn_gelu_fwd(const void* x, int B, int T, int Tp, int C, const float* gamma, const float* beta,
                        float eps, float* mean, float* rstd, void* ws, void* y, hipStream_t stream) {
  if (!shape_ok(B, T, C) || Tp < T) return TRIAD_EINVAL;
  const int nchunk = (T + CHUNK - 1) / CHUNK;
  float2* part = (float2*)ws;
  hipLaunchKernelGGL(chgn_sums_kernel<0>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)x, nullptr, T, Tp, C,
                     nullptr, nullptr, nullptr, nullptr, part);
  hipLaunchKernelGGL(chgn_stats_kernel, dim3((C + 255) / 256, B), dim3(256), 0, stream, part, nchunk, T, C, eps,
                     mean, rstd);
  hipLaunchKernelGGL(chgn_apply_kernel<0>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)x, nullptr, T, Tp, C,
                     mean, rstd, gamma, beta, nullptr, (bf16*)y);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_chgn_gelu_bwd(const void* x, const void* dy, int B, int T, int Tp, int C, const float* gamma,
                        const float* beta, const float* mean, const float* rstd, void* ws, void* dx, float* dgamma,
                        float* dbeta, hipStream_t stream) {
  if (!shape_ok(B, T, C) || Tp < T) return TRIAD_EINVAL;
  const int nchunk = (T + CHUNK - 1) / CHUNK;
  float2* part = (float2*)ws;
  float2* coef = part + (size_t)B * nchunk * C;
  double2* tot = (double2*)(coef + (size_t)B * C);
  hipLaunchKernelGGL(chgn_sums_kernel<1>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)x, (const bf16*)dy,
                     T, Tp, C, mean, rstd, gamma, beta, part);
  hipLaunchKernelGGL(chgn_bwd_coef_kernel, dim3((C + 255) / 256, B), dim3(256), 0, stream, part, nchunk, T, C, gamma,
                     coef, tot);
  hipLaunchKernelGGL(chgn_param_grad_kernel, dim3((C + 255) / 256), dim3(256), 0, stream, tot, B, C, dgamma, dbeta);
  hipLaunchKernelGGL(chgn_apply_kernel<1>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)x, (const bf16*)dy, T,
                     Tp, C, mean, rstd, gamma, beta, coef, (bf16*)dx);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// conv0 (1 -> C, kernel 10, stride 5, no bias) + GroupNorm(C groups) + GELU forward, conv0 recomputed
// from the bf16 waveform wave[b][Lp] (Lp >= 5 (Tp - 1) + 10); writes the padded frame buffers
// out = bf16(gelu(gn(y0))) and y0out = y0 ([b*Tp + t][c], frames T .. Tp-1 zero); mean / rstd for the
// backward (triad_chgn_gelu_bwd over y0out). ws: triad_chgn_workspace_bytes(B, T, C) bytes.
int triad_c0gn_fwd(const void* wave, long long Lp, const void* w0, int B, int T, int Tp, int C, const float* gamma,
                   const float* beta, float eps, float* mean, float* rstd, void* ws, void* out, void* y0out,
                   hipStream_t stream) {
  if (!shape_ok(B, T, C) || Tp < T || Lp < (long long)C0_S * (Tp - 1) + C0_K) return TRIAD_EINVAL;
  const int nchunk = (T + CHUNK - 1) / CHUNK;
  float2* part = (float2*)ws;
  hipLaunchKernelGGL(c0gn_kernel<0>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)wave, Lp, (const bf16*)w0, T,
                     Tp, C, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, part);
  hipLaunchKernelGGL(chgn_stats_kernel, dim3((C + 255) / 256, B), dim3(256), 0, stream, part, nchunk, T, C, eps,
                     mean, rstd);
  hipLaunchKernelGGL(c0gn_kernel<1>, dim3(nchunk, B), dim3(NT), 0, stream, (const bf16*)wave, Lp, (const bf16*)w0, T,
                     Tp, C, mean, rstd, gamma, beta, (bf16*)out, (bf16*)y0out, nullptr);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// dw0[c][j] (fp32) = sum_{b, t < T} dy0[b*Tp + t][c] * wave[b][5t + j]; ws: triad_conv0_dw_workspace_bytes.
long long triad_conv0_dw_workspace_bytes(int B, int T, int C) {
  return (long long)B * ((T + C0_DW_ROWS - 1) / C0_DW_ROWS) * C * C0_K * 4;
}

int triad_conv0_dw(const void* wave, long long Lp, const void* dy0, int B, int T, int Tp, int C, void* ws, float* dw0,
                   hipStream_t stream) {
  if (!shape_ok(B, T, C) || Tp < T || Lp < (long long)C0_S * (T - 1) + C0_K) return TRIAD_EINVAL;
  const int nblk = (T + C0_DW_ROWS - 1) / C0_DW_ROWS;
  hipLaunchKernelGGL(c0dw_kernel, dim3(nblk, B), dim3(NT), 0, stream, (const bf16*)wave, Lp, (const bf16*)dy0, T, Tp,
                     C, (float*)ws);
  TRIAD_CHECK_LAUNCH();
  return triad_sum_slabs((const float*)ws, B * nblk, (long long)C * C0_K, nullptr, 0, dw0, stream);
}
}  // extern "C"

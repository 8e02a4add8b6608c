// Materialising debug path of the loss head (the reference's
// compute_all_similarities_{av,tv} / compute_contrastive_loss_{av,tv} /
// compute_regularization_losses_{av,tv} / compute_temporal_smoothness_loss keep their
// signatures and return the (B, B, Nq, Nk) token similarities for small B). The training
// path never calls these: it uses the fused kernels of pairsim_fwd.hip / pairsim.hip.
//
// Token similarities S are fp32, laid out (Bq, Bk, Nq, Nk) as the reference returns them
// (model.py:384-387 / 502-505). All kernels here are HBM-bound elementwise / row passes.
#include "common.h"

namespace {

// rowmax[j][i*Nq+q] = max_k S[i][j][q][k], argmax = first index of the max (torch.max ties,
// measured on CPU). One wave per (i, j, q) row.
__global__ __launch_bounds__(256) void dense_rowmax_kernel(const float* __restrict__ S, int Bq, int Bk, int Nq,
                                                           int Nk, int R_pad, float* __restrict__ rowmax,
                                                           int* __restrict__ argmax) {
  const int lane = threadIdx.x & 63;
  const long long row = (long long)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const long long rows = (long long)Bq * Bk * Nq;
  if (row >= rows) return;
  const int q = (int)(row % Nq);
  const long long ij = row / Nq;
  const int j = (int)(ij % Bk), i = (int)(ij / Bk);
  const float* s = S + row * Nk;
  float mx = -INFINITY;
  int ix = 0x7fffffff;
  for (int k = lane; k < Nk; k += 64) {
    const float v = s[k];
    if (v > mx || (v != v && mx == mx)) { mx = v; ix = k; }  // NaN propagates like torch.max
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(mx, o);
    const int oi = __shfl_xor(ix, o);
    if (ov > mx || (ov == mx && oi < ix) || (ov != ov && mx == mx)) { mx = ov; ix = oi; }
  }
  if (lane == 0) {
    rowmax[(size_t)j * R_pad + (size_t)i * Nq + q] = mx;
    argmax[(size_t)j * R_pad + (size_t)i * Nq + q] = ix;
  }
}

// part[block] = sum clamp(S, lo, 0)^2 over a grid-stride slice (model.py:417-418 / 524-525).
__global__ __launch_bounds__(256) void nonneg_fwd_kernel(const float* __restrict__ S, long long n, float lo,
                                                         double* __restrict__ part) {
  __shared__ double red[4];
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float c = fminf(fmaxf(S[e], lo), 0.f);
    acc += (double)(c * c);
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// dS = coef[0] * scale * 2 clamp(S, lo, 0) * [lo <= S <= 0]  (clamp backward is inclusive at
// both bounds).
__global__ __launch_bounds__(256) void nonneg_bwd_kernel(const float* __restrict__ S, long long n, float lo,
                                                         float scale, const float* __restrict__ coef,
                                                         float* __restrict__ dS) {
  const float c0 = coef ? coef[0] * scale : scale;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const float s = S[e];
    dS[e] = (s >= lo && s <= 0.f) ? c0 * 2.f * s : 0.f;
  }
}

// Backward of (clip, token_sims) = all_similarities(q, k): the total gradient of S,
//   G[i][j][q][k] = dtok[i][j][q][k] + [k == argmax_ijq] * dclip[i][j] * qw[i*Nq+q],
// written as the bf16 GEMM operand A[(i*Nq+q)][j*Nk+k] (row stride lda), and per-block partial
// sums of G * S / temp (d/dtemp, since S = temp * <q, k>).
__global__ __launch_bounds__(256) void sims_bwd_pack_kernel(const float* __restrict__ S,
                                                            const float* __restrict__ dtok,
                                                            const float* __restrict__ dclip,
                                                            const float* __restrict__ qw,
                                                            const int* __restrict__ argmax, int Bq, int Bk, int Nq,
                                                            int Nk, int R_pad, const float* __restrict__ temp,
                                                            bf16* __restrict__ A, long long lda,
                                                            double* __restrict__ part) {
  __shared__ double red[4];
  const long long n = (long long)Bq * Bk * Nq * Nk;
  const float inv_t = 1.f / temp[0];
  double acc = 0.0;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n; e += (long long)gridDim.x * blockDim.x) {
    const int k = (int)(e % Nk);
    const long long row = e / Nk;
    const int q = (int)(row % Nq);
    const long long ij = row / Nq;
    const int j = (int)(ij % Bk), i = (int)(ij / Bk);
    const int r = i * Nq + q;
    float g = dtok ? dtok[e] : 0.f;
    if (dclip && argmax[(size_t)j * R_pad + r] == k) g += dclip[(size_t)i * Bk + j] * qw[r];
    A[(size_t)r * lda + (size_t)j * Nk + k] = (bf16)g;
    acc += (double)g * (double)(S[e] * inv_t);
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// out[0] = sum part (as float) -- finishes the two-level reductions above on the device.
__global__ void sum_parts_kernel(const double* __restrict__ part, int n, double scale, float* __restrict__ out) {
  __shared__ double red[4];
  double s = 0.0;
  for (int e = threadIdx.x; e < n; e += blockDim.x) s += part[e];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) out[0] = (float)(s * scale);
}

inline int blocks_for(long long n, int cap) {
  long long b = (n + 255) / 256;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" {

int triad_dense_nparts(long long n) { return blocks_for(n, 2048); }

int triad_dense_rowmax(const float* S, int Bq, int Bk, int Nq, int Nk, int R_pad, float* rowmax, int* argmax,
                       hipStream_t stream) {
  if (Bq <= 0 || Bk <= 0 || Nq <= 0 || Nk <= 0 || R_pad < Bq * Nq) return TRIAD_EINVAL;
  const long long rows = (long long)Bq * Bk * Nq;
  hipLaunchKernelGGL(dense_rowmax_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, S, Bq, Bk, Nq, Nk,
                     R_pad, rowmax, argmax);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_nonneg_fwd(const float* S, long long n, float lo, double* part, hipStream_t stream) {
  if (n <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(nonneg_fwd_kernel, dim3(blocks_for(n, 2048)), dim3(256), 0, stream, S, n, lo, part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_nonneg_bwd(const float* S, long long n, float lo, float scale, const float* coef, float* dS,
                     hipStream_t stream) {
  if (n <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(nonneg_bwd_kernel, dim3(blocks_for(n, 8192)), dim3(256), 0, stream, S, n, lo, scale, coef, dS);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_sims_bwd_pack(const float* S, const float* dtok, const float* dclip, const float* qw, const int* argmax,
                        int Bq, int Bk, int Nq, int Nk, int R_pad, const float* temp, void* A, long long lda,
                        double* part, hipStream_t stream) {
  if (Bq <= 0 || Bk <= 0 || Nq <= 0 || Nk <= 0 || lda < (long long)Bk * Nk || R_pad < Bq * Nq ||
      (dclip && (!qw || !argmax)))
    return TRIAD_EINVAL;
  const long long n = (long long)Bq * Bk * Nq * Nk;
  hipLaunchKernelGGL(sims_bwd_pack_kernel, dim3(blocks_for(n, 2048)), dim3(256), 0, stream, S, dtok, dclip, qw,
                     argmax, Bq, Bk, Nq, Nk, R_pad, temp, (bf16*)A, lda, part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_sum_parts(const double* part, int n, double scale, float* out, hipStream_t stream) {
  if (n <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(sum_parts_kernel, dim3(1), dim3(256), 0, stream, part, n, scale, out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

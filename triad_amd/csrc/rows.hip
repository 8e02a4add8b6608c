// Row movement kernels around the similarity head:
//   * patch-dropout compaction (model.py:268-308): out[b][t] = x[b][idx[b][t]] or 0,
//     where idx lists each sample's kept tokens in original order and -1 pads;
//   * its backward (scatter == gather with the inverse index);
//   * per-token L2 normalisation for the inference similarity maps (model.py:363-364).
#include "common.h"

namespace {

// One thread moves 16 bytes; rows are row_bytes long (multiple of 16).
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint4* __restrict__ src, long long src_rows,
                                                          const int* __restrict__ idx, int M, int chunks,
                                                          long long total, uint4* __restrict__ dst) {
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < total;
       e += (long long)gridDim.x * blockDim.x) {
    const long long rowo = e / chunks;
    const int c = (int)(e - rowo * chunks);
    const int b = (int)(rowo / M);
    const int s = idx[rowo];
    uint4 v = make_uint4(0, 0, 0, 0);
    if (s >= 0) v = src[((long long)b * src_rows + s) * chunks + c];
    dst[e] = v;
  }
}

// y[r] = x[r] / max(||x[r]||_2, eps), bf16 in/out, fp32 math; one wave per row.
__global__ __launch_bounds__(256) void l2norm_rows_kernel(const bf16* __restrict__ x, int rows, int D, float eps,
                                                          bf16* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const bf16* xr = x + (size_t)r * D;
  float ss = 0.f;
  for (int d = lane * 8; d < D; d += 512) {
    const bf16x8 v = *(const bf16x8*)(xr + d);
#pragma unroll
    for (int k = 0; k < 8; ++k) ss += (float)v[k] * (float)v[k];
  }
  ss = wave_sum(ss);
  const float inv = 1.f / fmaxf(sqrtf(ss), eps);
  bf16* yr = y + (size_t)r * D;
  for (int d = lane * 8; d < D; d += 512) {
    const bf16x8 v = *(const bf16x8*)(xr + d);
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)((float)v[k] * inv);
    *(bf16x8*)(yr + d) = o;
  }
}

}  // namespace

extern "C" {

// dst[b][t][:] = idx[b][t] >= 0 ? src[b][idx[b][t]][:] : 0, for b < B, t < M.
int triad_gather_rows(const void* src, long long src_rows, const int* idx, int B, int M, int row_bytes,
                      void* dst, hipStream_t stream) {
  if (row_bytes % 16 || B <= 0 || M <= 0) return TRIAD_EINVAL;
  const int chunks = row_bytes / 16;
  const long long total = (long long)B * M * chunks;
  long long blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(gather_rows_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const uint4*)src,
                     src_rows, idx, M, chunks, total, (uint4*)dst);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_l2norm_rows(const void* x, int rows, int D, float eps, void* y, hipStream_t stream) {
  if (D % 8 || rows <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(l2norm_rows_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, (const bf16*)x, rows, D, eps,
                     (bf16*)y);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

namespace {

// pass 1: per-block partial (sum, sum of squares) in double; 16-byte loads, two in flight per
// thread (4-byte loads with one dependent fp64 chain made the c3 audio batch a 0.2 ms pass)
template <bool VEC>
__global__ __launch_bounds__(256) void znorm_stats_kernel(const float* __restrict__ x, long long n,
                                                          double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0, q = 0.0, s2 = 0.0, q2 = 0.0;
  const long long n4 = VEC ? n / 4 : 0, stride = (long long)gridDim.x * blockDim.x;
  const float4* x4 = (const float4*)x;
  long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x;
  for (; e + stride < n4; e += 2 * stride) {
    const float4 a = x4[e], b = x4[e + stride];
    s += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
    q += ((double)a.x * a.x + (double)a.y * a.y) + ((double)a.z * a.z + (double)a.w * a.w);
    s2 += ((double)b.x + (double)b.y) + ((double)b.z + (double)b.w);
    q2 += ((double)b.x * b.x + (double)b.y * b.y) + ((double)b.z * b.z + (double)b.w * b.w);
  }
  for (; e < n4; e += stride) {
    const float4 a = x4[e];
    s += ((double)a.x + (double)a.y) + ((double)a.z + (double)a.w);
    q += ((double)a.x * a.x + (double)a.y * a.y) + ((double)a.z * a.z + (double)a.w * a.w);
  }
  // the tail (VEC) or everything (a buffer not 16-byte aligned), element-wise
  const long long t0 = 4 * n4, tst = VEC ? blockDim.x : stride;
  for (long long t = t0 + (VEC ? (blockIdx.x == 0 ? threadIdx.x : n) : blockIdx.x * (long long)blockDim.x + threadIdx.x);
       t < n; t += tst) {
    const double v = x[t];
    s += v;
    q += v * v;
  }
  s = block_sum_d(s + s2, red);
  q = block_sum_d(q + q2, red);
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = s;
    part[2 * blockIdx.x + 1] = q;
  }
}

// pass 2: every block re-reduces the partials, then normalises its slice (16-byte accesses)
template <bool VEC>
__global__ __launch_bounds__(256) void znorm_apply_kernel(const float* __restrict__ x, long long n, float eps,
                                                          const double* __restrict__ part, int nparts,
                                                          float* __restrict__ y) {
  __shared__ double red[4];
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    s += part[2 * i];
    q += part[2 * i + 1];
  }
  s = block_sum_d(s, red);
  q = block_sum_d(q, red);
  const double mean = s / (double)n;
  const double var = q / (double)n - mean * mean;
  const float m = (float)mean;
  const float inv = (float)(1.0 / sqrt((var > 0.0 ? var : 0.0) + (double)eps));
  const long long n4 = VEC ? n / 4 : 0, stride = (long long)gridDim.x * blockDim.x;
  const float4* x4 = (const float4*)x;
  float4* y4 = (float4*)y;
  for (long long e = blockIdx.x * (long long)blockDim.x + threadIdx.x; e < n4; e += stride) {
    const float4 a = x4[e];
    y4[e] = make_float4((a.x - m) * inv, (a.y - m) * inv, (a.z - m) * inv, (a.w - m) * inv);
  }
  const long long t0 = 4 * n4, tst = VEC ? blockDim.x : stride;
  for (long long t = t0 + (VEC ? (blockIdx.x == 0 ? threadIdx.x : n) : blockIdx.x * (long long)blockDim.x + threadIdx.x);
       t < n; t += tst)
    y[t] = (x[t] - m) * inv;
}

}  // namespace

extern "C" int triad_global_znorm(const float* x, long long n, float eps, float* y, double* part, int nblocks,
                                  hipStream_t stream) {
  if (n <= 0 || nblocks <= 0) return TRIAD_EINVAL;
  if ((((size_t)x) | ((size_t)y)) % 16 == 0) {
    hipLaunchKernelGGL(znorm_stats_kernel<true>, dim3(nblocks), dim3(256), 0, stream, x, n, part);
    hipLaunchKernelGGL(znorm_apply_kernel<true>, dim3(nblocks), dim3(256), 0, stream, x, n, eps, part, nblocks, y);
  } else {
    hipLaunchKernelGGL(znorm_stats_kernel<false>, dim3(nblocks), dim3(256), 0, stream, x, n, part);
    hipLaunchKernelGGL(znorm_apply_kernel<false>, dim3(nblocks), dim3(256), 0, stream, x, n, eps, part, nblocks, y);
  }
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

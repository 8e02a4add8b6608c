// Fused optimizer step over flat parameter / gradient buffers (SajayR/TRIAD src/train.py:990-1041):
//   per-parameter gradient sum-of-squares (grad-norm logging train.py:992-1002 and
//   clip_grad_norm_ train.py:1004-1006), then ONE AdamW pass for every stepped
//   optimizer (train.py:272-287: torch.optim.AdamW defaults, betas (0.9, 0.999),
//   eps 1e-8, weight_decay 1e-2) with the clip factor applied on the fly.
// Parameters, gradients and both moments live in single contiguous fp32 buffers
// (the Python side re-points each nn.Parameter's .data/.grad at views), so the
// whole step is two launches and the data-parallel all-reduce is one buffer.
// Mixed precision (bf16 autocast backbones, model.py:483,603): the Linear / Conv weights that
// autocast would cast to bf16 on every forward can instead BE bf16 model parameters backed by
// the fp32 master in the flat buffer: the AdamW pass writes their bf16 copy (what autocast's
// cast would produce), and their bf16 gradients (what autocast's backward produces before
// the cast to fp32) are gathered into the flat fp32 gradient buffer by one multi-tensor launch
// instead of one cast + one accumulate launch per parameter.
#include "common.h"

namespace {

struct Chunk {  // a slice of one parameter: elements [off, off + n) of the flat buffers
  long long off;
  int n;
  int param;
};

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, const Chunk* __restrict__ chunks,
                                                    double* __restrict__ out /* per chunk */) {
  __shared__ double red[4];
  const Chunk c = chunks[blockIdx.x];
  double s = 0.0;
  const float* p = g + c.off;
  for (int i = threadIdx.x * 4; i < c.n; i += blockDim.x * 4) {
    if (i + 3 < c.n) {
      const float4 v = *(const float4*)(p + i);
      s += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
    } else {
      for (int k = i; k < c.n; ++k) s += (double)p[k] * p[k];
    }
  }
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

// pp: per parameter {step_size = lr/bc1, 1/bc2_sqrt, wd_factor = 1 - lr*wd}; scale: clip factor per parameter
__global__ __launch_bounds__(256) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v,
                                                    const Chunk* __restrict__ chunks, const float* __restrict__ pp,
                                                    const float* __restrict__ scale, float beta1, float beta2,
                                                    float omb1, float omb2, float eps,
                                                    const unsigned long long* __restrict__ shadow) {
  const Chunk c = chunks[blockIdx.x];
  // shadow[param]: address of the bf16 model weight minus 2 * (its flat offset), 0 = none
  bf16* const sh = shadow && shadow[c.param] ? (bf16*)(shadow[c.param]) : nullptr;
  const float step_size = pp[3 * c.param], inv_bc2 = pp[3 * c.param + 1], wdf = pp[3 * c.param + 2];
  const float sc = scale ? scale[c.param] : 1.f;
  for (int i = threadIdx.x; i < c.n; i += blockDim.x) {
    const long long e = c.off + i;
    const float gr = g[e] * sc;
    float pv = p[e] * wdf;
    float mv = m[e];
    mv = mv + omb1 * (gr - mv);              // exp_avg.lerp_(grad, 1 - beta1)
    float vv = v[e] * beta2 + omb2 * gr * gr;  // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
    const float denom = sqrtf(vv) * inv_bc2 + eps;
    pv = pv - step_size * (mv / denom);
    p[e] = pv;
    m[e] = mv;
    v[e] = vv;
    if (sh) sh[e] = (bf16)pv;
  }
}

struct GradPiece {  // bf16 (f32 == 0) or fp32 (f32 == 1) gradient slice -> flat fp32 gradient [dst, dst + n)
  const void* src;
  long long dst;
  int n;
  int f32;
};

__global__ __launch_bounds__(256) void gather_grads_kernel(const GradPiece* __restrict__ pieces,
                                                           float* __restrict__ g, int accumulate) {
  const GradPiece c = pieces[blockIdx.x];
  float* out = g + c.dst;
  for (int i = threadIdx.x; i < c.n; i += blockDim.x) {
    const float x = c.f32 ? ((const float*)c.src)[i] : (float)((const bf16*)c.src)[i];
    out[i] = accumulate ? out[i] + x : x;
  }
}

}  // namespace

extern "C" {

// out[c] = sum of squares of g over chunk c (chunks: device array of {off, n, param}).
int triad_grad_sumsq(const float* g, const void* chunks, int nchunks, double* out, hipStream_t stream) {
  if (nchunks <= 0) return TRIAD_OK;
  hipLaunchKernelGGL(sumsq_kernel, dim3(nchunks), dim3(256), 0, stream, g, (const Chunk*)chunks, out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_adamw_step(float* p, const float* g, float* m, float* v, const void* chunks, int nchunks,
                     const float* pp, const float* scale, float beta1, float beta2, float omb1, float omb2,
                     float eps, const unsigned long long* shadow, hipStream_t stream) {
  if (nchunks <= 0) return TRIAD_OK;
  hipLaunchKernelGGL(adamw_kernel, dim3(nchunks), dim3(256), 0, stream, p, g, m, v, (const Chunk*)chunks, pp, scale,
                     beta1, beta2, omb1, omb2, eps, shadow);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_gather_grads(const void* pieces, int npieces, float* g, int accumulate, hipStream_t stream) {
  if (npieces <= 0) return TRIAD_OK;
  hipLaunchKernelGGL(gather_grads_kernel, dim3(npieces), dim3(256), 0, stream, (const GradPiece*)pieces, g,
                     accumulate);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

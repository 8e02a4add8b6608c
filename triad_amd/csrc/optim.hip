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

// Chunk offsets are multiples of 4 elements (FlatParamSpace: parameter slots of ALIGN = 64
// elements, chunks of CHUNK = 16384), so every chunk starts 16-byte aligned: the streaming
// kernels below move float4 (and bf16x4 / bf16x8) per lane, U groups in flight per thread, with a
// scalar tail for a chunk length that is not a multiple of 4. Same per-element arithmetic as the
// scalar forms (bit-identical outputs); round 5: the scalar forms ran the optimizer phase at
// 4.4-4.8 TB/s (adamw 1.03 ms, gather 0.26, sumsq 0.14 per bench step).
constexpr int U = 4;

__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, const Chunk* __restrict__ chunks,
                                                    double* __restrict__ out /* per chunk */) {
  __shared__ double red[4];
  const Chunk c = chunks[blockIdx.x];
  double s = 0.0;
  const float* p = g + c.off;
  const int nv = c.n >> 2;
  const float4* p4 = (const float4*)p;
  for (int i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
    float4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = i0 + 256 * u < nv ? p4[i0 + 256 * u] : float4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < U; ++u)
      s += (double)x[u].x * x[u].x + (double)x[u].y * x[u].y + (double)x[u].z * x[u].z + (double)x[u].w * x[u].w;
  }
  for (int k = 4 * nv + threadIdx.x; k < c.n; k += 256) s += (double)p[k] * p[k];
  s = block_sum_d(s, red);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

struct AdamConsts {
  float step_size, inv_bc2, wdf, sc, beta2, omb1, omb2, eps;
};

// torch.optim.AdamW's update of one element (single-tensor form, torch/optim/adamw.py)
__device__ __forceinline__ void adamw_elem(const AdamConsts& k, float& pv, float gr, float& mv, float& vv) {
  gr = gr * k.sc;
  pv = pv * k.wdf;
  mv = mv + k.omb1 * (gr - mv);              // exp_avg.lerp_(grad, 1 - beta1)
  vv = vv * k.beta2 + k.omb2 * gr * gr;      // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float denom = sqrtf(vv) * k.inv_bc2 + k.eps;
  pv = pv - k.step_size * (mv / denom);
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
  bf16* const sh = shadow && shadow[c.param] ? (bf16*)(shadow[c.param]) + c.off : nullptr;
  const AdamConsts k = {pp[3 * c.param], pp[3 * c.param + 1], pp[3 * c.param + 2], scale ? scale[c.param] : 1.f,
                        beta2, omb1, omb2, eps};
  float4* const p4 = (float4*)(p + c.off);
  const float4* const g4 = (const float4*)(g + c.off);
  float4* const m4 = (float4*)(m + c.off);
  float4* const v4 = (float4*)(v + c.off);
  const int nv = c.n >> 2;
  for (int i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
    float4 pa[U], ga[U], ma[U], va[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 256 * u;
      if (i < nv) { pa[u] = p4[i]; ga[u] = g4[i]; ma[u] = m4[i]; va[u] = v4[i]; }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + 256 * u;
      if (i < nv) {
        adamw_elem(k, pa[u].x, ga[u].x, ma[u].x, va[u].x);
        adamw_elem(k, pa[u].y, ga[u].y, ma[u].y, va[u].y);
        adamw_elem(k, pa[u].z, ga[u].z, ma[u].z, va[u].z);
        adamw_elem(k, pa[u].w, ga[u].w, ma[u].w, va[u].w);
        p4[i] = pa[u];
        m4[i] = ma[u];
        v4[i] = va[u];
        if (sh) *(bf16x4*)(sh + 4 * i) = bf16x4{(bf16)pa[u].x, (bf16)pa[u].y, (bf16)pa[u].z, (bf16)pa[u].w};
      }
    }
  }
  for (int i = 4 * nv + threadIdx.x; i < c.n; i += 256) {
    const long long e = c.off + i;
    float pv = p[e], mv = m[e], vv = v[e];
    adamw_elem(k, pv, g[e], mv, vv);
    p[e] = pv;
    m[e] = mv;
    v[e] = vv;
    if (sh) sh[i] = (bf16)pv;
  }
}

struct GradPiece {  // bf16 (f32 == 0) or fp32 (f32 == 1) gradient slice -> flat fp32 gradient [dst, dst + n)
  const void* src;
  long long dst;
  int n;
  int f32;
};

// dst is 16-byte aligned (as the chunks above); a source that is not (a .grad view at an odd
// offset) takes the scalar loop
__global__ __launch_bounds__(256) void gather_grads_kernel(const GradPiece* __restrict__ pieces,
                                                           float* __restrict__ g, int accumulate) {
  const GradPiece c = pieces[blockIdx.x];
  float* out = g + c.dst;
  int done = 0;
  if (!((uintptr_t)c.src & 15)) {
    float4* const o4 = (float4*)out;
    if (c.f32) {
      const float4* const s4 = (const float4*)c.src;
      const int nv = c.n >> 2;
      for (int i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
        float4 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + 256 * u;
          if (i < nv) {
            x[u] = s4[i];
            if (accumulate) y[u] = o4[i];
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + 256 * u;
          if (i < nv) {
            if (accumulate) x[u] = float4{y[u].x + x[u].x, y[u].y + x[u].y, y[u].z + x[u].z, y[u].w + x[u].w};
            o4[i] = x[u];
          }
        }
      }
      done = 4 * nv;
    } else {
      const bf16x8* const s8 = (const bf16x8*)c.src;
      const int nv = c.n >> 3;
      for (int i0 = threadIdx.x; i0 < nv; i0 += 256 * U) {
        bf16x8 x[U];
        float4 y[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + 256 * u;
          if (i < nv) {
            x[u] = s8[i];
            if (accumulate) { y[u][0] = o4[2 * i]; y[u][1] = o4[2 * i + 1]; }
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = i0 + 256 * u;
          if (i < nv) {
            float4 a = {(float)x[u][0], (float)x[u][1], (float)x[u][2], (float)x[u][3]};
            float4 b = {(float)x[u][4], (float)x[u][5], (float)x[u][6], (float)x[u][7]};
            if (accumulate) {
              a = float4{y[u][0].x + a.x, y[u][0].y + a.y, y[u][0].z + a.z, y[u][0].w + a.w};
              b = float4{y[u][1].x + b.x, y[u][1].y + b.y, y[u][1].z + b.z, y[u][1].w + b.w};
            }
            o4[2 * i] = a;
            o4[2 * i + 1] = b;
          }
        }
      }
      done = 8 * nv;
    }
  }
  for (int i = done + threadIdx.x; i < c.n; i += blockDim.x) {
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

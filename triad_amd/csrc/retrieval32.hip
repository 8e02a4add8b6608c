// Reference-precision mode of the 1000-way retrieval drop-in: the reference
// scores every (query, item) pair in fp32 -- retrieval.py:106-114, aggregator_av_a2v / _v2a:
//   token_sims = matmul(q, k^T) / temperature;  max over the item's tokens;  mean over the query's
// -- with a Python double loop over the N^2 pairs. triad_retrieval_maxmean_f32 does all pairs in
// ONE launch, in fp32 end to end, for callers that embed in fp32 (model.use_amp == False, as the
// reference's retrieval.py embeds): the product path (bf16 features, triad_pairsim_fwd's MFMA
// chain) stays the default. gfx950 has no fp32-input MFMA at the bf16 rate, and packed fp32 VALU
// is kept out of the library, so this is a plain fp32 FMA tile kernel:
//   * workgroup = one (query sample i, item sample j) pair, 256 threads as 16 x 16; the pair's
//     query x item token matrix in 64 x 64 tiles, 32-deep feature slices of both through LDS
//     (transposed so each thread reads its 4 queries / 4 items as one 16-byte ds_read);
//   * per tile: s = dot / temperature (the reference's division), padded items masked, the row
//     max reduced over the 16 threads of a query row (lane shuffles within the wave) into a running
//     max per query; per query tile the valid queries' maxima summed in fp64; sim = sum / n_q.
#include "common.h"

namespace {

constexpr int RT = 64;   // query / item tokens per tile
constexpr int RD = 32;   // feature slice per LDS stage
constexpr int RS = RT + 4;  // LDS row stride (floats): 16-byte aligned rows

__global__ __launch_bounds__(256) void maxmean_f32_kernel(const float* __restrict__ Q, const int* __restrict__ qlen,
                                                          int nq_pad, const float* __restrict__ K,
                                                          const int* __restrict__ klen, int nk_pad, int D, float temp,
                                                          float* __restrict__ sim, int Bk) {
  __shared__ __attribute__((aligned(16))) float qs[RD][RS];
  __shared__ __attribute__((aligned(16))) float ks[RD][RS];
  __shared__ double red[4];
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const int j = blockIdx.x, i = blockIdx.y;
  const int nq = min(qlen[i], nq_pad), nk = min(klen[j], nk_pad);
  const float* Qi = Q + (size_t)i * nq_pad * D;
  const float* Kj = K + (size_t)j * nk_pad * D;
  const int lr = t >> 2, lc = (t & 3) * 8;   // loader: token row lr, features lc .. lc + 7 of the slice
  double sum = 0.0;
  for (int q0 = 0; q0 < nq; q0 += RT) {
    float rmax[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
    for (int k0 = 0; k0 < nk; k0 += RT) {
      float acc[4][4] = {};
      for (int d0 = 0; d0 < D; d0 += RD) {
        // rows < nq_pad / nk_pad (multiples of 64): inside the allocations
        const float* qp = Qi + (size_t)(q0 + lr) * D + d0 + lc;
        const float* kp = Kj + (size_t)(k0 + lr) * D + d0 + lc;
        const float4 qa = *(const float4*)qp, qb = *(const float4*)(qp + 4);
        const float4 ka = *(const float4*)kp, kb = *(const float4*)(kp + 4);
        __syncthreads();   // the previous slice's reads are done
        qs[lc + 0][lr] = qa.x; qs[lc + 1][lr] = qa.y; qs[lc + 2][lr] = qa.z; qs[lc + 3][lr] = qa.w;
        qs[lc + 4][lr] = qb.x; qs[lc + 5][lr] = qb.y; qs[lc + 6][lr] = qb.z; qs[lc + 7][lr] = qb.w;
        ks[lc + 0][lr] = ka.x; ks[lc + 1][lr] = ka.y; ks[lc + 2][lr] = ka.z; ks[lc + 3][lr] = ka.w;
        ks[lc + 4][lr] = kb.x; ks[lc + 5][lr] = kb.y; ks[lc + 6][lr] = kb.z; ks[lc + 7][lr] = kb.w;
        __syncthreads();
#pragma unroll 8
        for (int d = 0; d < RD; ++d) {
          const float4 a = *(const float4*)&qs[d][4 * ty];
          const float4 b = *(const float4*)&ks[d][4 * tx];
          const float av[4] = {a.x, a.y, a.z, a.w}, bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int v = 0; v < 4; ++v) acc[u][v] = fmaf(av[u], bv[v], acc[u][v]);
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        float m = -INFINITY;
#pragma unroll
        for (int v = 0; v < 4; ++v)
          if (k0 + 4 * tx + v < nk) m = fmaxf(m, acc[u][v] / temp);
#pragma unroll
        for (int x = 1; x < 16; x *= 2) m = fmaxf(m, __shfl_xor(m, x));   // the 16 threads of this row
        rmax[u] = fmaxf(rmax[u], m);
      }
    }
    if (tx == 0) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (q0 + 4 * ty + u < nq) sum += (double)rmax[u];
    }
  }
  sum = block_sum_d(sum, red);
  if (t == 0) sim[(size_t)i * Bk + j] = (float)(sum / (double)nq);
}

// y = x / max(||x||_2, eps) per row, fp32 (F.normalize's division); one wave per row.
__global__ __launch_bounds__(256) void l2norm_rows_f32_kernel(const float* __restrict__ x, int rows, int D, float eps,
                                                              float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  const float* xr = x + (size_t)r * D;
  float ss = 0.f;
  for (int d = lane * 4; d < D; d += 256) {
    const float4 v = *(const float4*)(xr + d);
    ss += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  ss = wave_sum(ss);
  const float den = fmaxf(sqrtf(ss), eps);
  float* yr = y + (size_t)r * D;
  for (int d = lane * 4; d < D; d += 256) {
    const float4 v = *(const float4*)(xr + d);
    *(float4*)(yr + d) = float4{v.x / den, v.y / den, v.z / den, v.w / den};
  }
}

}  // namespace

extern "C" {

int triad_retrieval_maxmean_f32(const float* Q, const int* qlen, int Bq, int nq_pad, const float* K, const int* klen,
                                int Bk, int nk_pad, int D, float temp, float* sim, hipStream_t stream) {
  if (!Q || !qlen || !K || !klen || !sim || Bq <= 0 || Bk <= 0 || Bq > 65535 || nq_pad <= 0 || nq_pad % RT ||
      nk_pad <= 0 || nk_pad % RT || D <= 0 || D % RD || ((uintptr_t)Q & 15) || ((uintptr_t)K & 15))
    return TRIAD_EINVAL;
  hipLaunchKernelGGL(maxmean_f32_kernel, dim3(Bk, Bq), dim3(256), 0, stream, Q, qlen, nq_pad, K, klen, nk_pad, D,
                     temp, sim, Bk);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_l2norm_rows_f32(const float* x, int rows, int D, float eps, float* y, hipStream_t stream) {
  if (!x || !y || D % 4 || D <= 0 || rows <= 0 || ((uintptr_t)x & 15) || ((uintptr_t)y & 15)) return TRIAD_EINVAL;
  hipLaunchKernelGGL(l2norm_rows_f32_kernel, dim3((rows + 3) / 4), dim3(256), 0, stream, x, rows, D, eps, y);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

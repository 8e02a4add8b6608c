// Fused pairwise token-similarity kernels for TRIAD's dense contrastive head.
//
// Reference semantics (SajayR/TRIAD src/model.py):
//   S[i,j,q,k] = temp * <Q[i,q], K[j,k]>           model.py:384-387 / 502-505
//   clip[i,j]  = mean_q max_k S   (TV: mask-weighted) model.py:389-391 / 507-512
//   l_nonneg   = mean clamp(S, lo, 0)^2            model.py:417-418 / 524-525
// The (Bq,Bk,Nq,Nk) tensor is never materialised: one kernel streams key tiles
// through LDS against query fragments held in VGPRs and reduces in registers.
//
// Layouts (HBM):
//   Q      [R_pad][512] bf16  query tokens flattened (row r = i*Nq + q), rows >= R are 0
//   K      [Bk][Nk_pad][512] bf16 key tokens, per-sample zero padded to Nk_pad (multiple of 32);
//          columns k < Nk_eff take part in max / l_nonneg (patch-dropout zero rows included,
//          model.py:296-307), columns k >= Nk_eff are excluded.
//   rowmax [Bk][R_pad] f32, argmax [Bk][R_pad] i32   max_k S and its first index
//   dS     [R_pad][C_alloc] bf16, C_alloc >= Bk*Nk_pad  dL/dS for the two backward GEMMs
//
// Wave tiling (CDNA4, wave64): each wave owns 32 query rows; its Q fragments
// (32 rows x 512 d = 128 VGPRs) stay in registers for the whole launch. A key
// tile is 32 keys x 512 d (32 KB) in LDS. One 32-step chain of
// v_mfma_f32_32x32x16_bf16 computes S^T = K_tile . Q_rows^T with the QUERY on
// the lane and the 32 keys in the 16 accumulator registers (x 2 lane halves), so
// the row max/argmax is lane-local plus one half-wave exchange.
#include "common.h"

int triad_pairsim_fwd2_launch(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                              int Nk_eff, const float* temp, float clamp_lo, int diag, int diag_off, float* rowmax,
                              int* argmax, double* nn_part, float* diagS, void* dS, long long CT, double* st_part,
                              const int* k_len, int xb, int ys, int jpw, hipStream_t stream);
int triad_pairsim_fwd_multi_launch(const triad_pairsim_problem* pr, const int* xb, const int* ys, const int* jpw,
                                   int n, hipStream_t stream);
int triad_pairsim_diag_launch(const triad_pairsim_problem* pr, int n, hipStream_t stream);

namespace {

constexpr int D = 512;
constexpr int NS = D / 16;          // MFMA k-steps per key tile
constexpr int WAVES = 8;            // 512-thread workgroup, 2 waves per SIMD
constexpr int ROWS_PER_WG = 32 * WAVES;
constexpr int KT_ELEMS = 32 * D;    // one key tile in LDS (bf16 elements)

struct PairArgs {
  const bf16* Q;
  const bf16* K;
  int R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff, j_per_wg;
  int diag, diag_off;  // diag: query sample i pairs with key sample i + diag_off
  const float* temp;
  float clamp_lo;
  // forward outputs
  float* rowmax;
  int* argmax;
  double* part;        // per-workgroup partial (l_nonneg sum in fwd, dtemp in bwd)
  float* diagS;        // [Bq][Nq][Nk_pad] S on the diagonal pairs (fwd, may be null)
  // backward inputs
  const float* dclip;  // [Bq][Bk] dCE/dclip (unit upstream gradient)
  const float* qw;     // [R] d clip / d rowmax per row (1/Nq or mask/len)
  const float* dSdiag; // [Bq][Nq][Nk_pad] unit grad of the diagonal regulariser (may be null)
  const float* coef;   // [4] c_ce, c_nn (=0.15*2*c_reg/N_el), c_diag, c_cal
  bf16* dS;            // tiled dS (see bwd_gemm.hip): [R_pad/32][CT][1024]
  long long CT;        // key tiles per row panel of dS (>= Bk*Nk_pad/32)
  double* part2;       // fwd with dS output: per-workgroup sum of S*S_raw over lo<=S<=0
  const int* klen;     // optional per-key-sample valid length (forward only; retrieval)
};

// Store this wave's 32x32 tile of dS (accumulator order, chunks in ds_chunk order: two 1 KB runs).
__device__ __forceinline__ void store_tile(bf16* dS, long long CT, int rt, long long ct, int lane,
                                           const bf16 (&v)[16]) {
  bf16* dst = dS + ((long long)rt * CT + ct) * 1024 + lane * 8;  // chunks 2 lane, 2 lane + 1 (ds_chunk)
  bf16x8 a, b;
#pragma unroll
  for (int k = 0; k < 8; ++k) { a[k] = v[k]; b[k] = v[8 + k]; }
  *(bf16x8*)dst = a;
  *(bf16x8*)(dst + 512) = b;
}

// Stage key tile (j, kb) into LDS buffer `dst`. Row t of the tile is one
// wave-instruction (64 lanes x 16 B = one 1 KB key row); LDS chunk c of row t
// holds global chunk c ^ (t & 15), which makes the later ds_read_b128 of 32
// different rows at one chunk conflict-free.
__device__ __forceinline__ void stage_key_tile(const PairArgs& a, bf16* dst, int j, int kb,
                                               int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 32 / WAVES; ++u) {
    const int t = wave * (32 / WAVES) + u;
    const bf16* src = a.K + ((size_t)j * a.Nk_pad + kb * 32 + t) * D + ((lane ^ (t & 15)) * 8);
    glds16(src, dst + t * D);
  }
}

// Recompute form of dL/dS (any mix of upstream gradients): S per tile, then the full dS
// (clamp + max + diagonal terms) into the tiled layout and the per-workgroup dL/dtemp partial.
__global__ __launch_bounds__(512, 2) void pairsim_dS_kernel(PairArgs a) {
  // All LDS in ONE array (a second __shared__ object can make hipcc drain the
  // in-flight LDS-DMA before every ds_read).
  __shared__ __attribute__((aligned(16))) bf16 kbuf[2 * KT_ELEMS + 8 * WAVES];
  double* red = (double*)(kbuf + 2 * KT_ELEMS);

  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const int row = blockIdx.x * ROWS_PER_WG + wave * 32 + ql;
  const bool row_ok = row < a.R;
  const int qi = row_ok ? row / a.Nq : -1;
  const int qq = row_ok ? row - qi * a.Nq : 0;

  int koff[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) koff[k] = ((2 * k + h) ^ (ql & 15)) * 8;

  const int j0 = blockIdx.y * a.j_per_wg;
  const int j1 = min(a.Bk, j0 + a.j_per_wg);
  const int nkb = a.Nk_pad / 32;
  const int nblocks = (j1 - j0) * nkb;
  if (nblocks <= 0) {  // uniform across the workgroup
    if (threadIdx.x == 0) {
      a.part[blockIdx.y * gridDim.x + blockIdx.x] = 0.0;
    }
    return;
  }

  stage_key_tile(a, kbuf, j0, 0, wave, lane);

  // Query fragments: lane holds Q[row][16 s + 8 h .. +8] for s = 0..31 (the B operand).
  bf16x8 qf[NS];
  {
    const bf16* qp = a.Q + (size_t)row * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *(const bf16x8*)(qp + 16 * s);
  }
  const float temp = *a.temp;
  const float lo = a.clamp_lo;

  const float c_ce = a.coef[0], c_nn = a.coef[1], c_dg = a.coef[2];
  const float wrow = row_ok ? a.qw[row] : 0.f;

  float gmax = 0.f;
  int amax = -1;
  double accd = 0.0;
  const int rt = blockIdx.x * WAVES + wave;  // this wave's row tile of dS

  for (int b = 0; b < nblocks; ++b) {
    const int j = j0 + b / nkb, kb = b - (b / nkb) * nkb;
    lds_dma_barrier();  // tile b has landed; all waves are done with buffer (b+1)&1
    if (b + 1 < nblocks) {
      const int b1 = b + 1;
      stage_key_tile(a, kbuf + ((b1 & 1) ? KT_ELEMS : 0), j0 + b1 / nkb, b1 - (b1 / nkb) * nkb,
                     wave, lane);
    }
    const bf16* kt = kbuf + ((b & 1) ? KT_ELEMS : 0) + ql * D;
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      // chunk (2s+h) ^ (key & 15): the swizzle only touches the low 4 bits, so 8 per-lane
      // offsets + an immediate of 256 B * (s >> 3) address all 32 fragments
      const bf16x8 af = *(const bf16x8*)(kt + koff[s & 7] + (s >> 3) * 128);
      acc = mfma32(af, qf[s], acc);
    }

    const bool diag_pair = a.diag && row_ok && (j == qi + a.diag_off);
    const int key0 = kb * 32 + 4 * h;

    if (kb == 0) {
      gmax = row_ok ? c_ce * a.dclip[(size_t)qi * a.Bk + j] * wrow : 0.f;
      amax = row_ok ? a.argmax[(size_t)j * a.R_pad + row] : -1;
    }
    const float* dg = (diag_pair && a.dSdiag) ? a.dSdiag + ((size_t)qi * a.Nq + qq) * a.Nk_pad : nullptr;
    float dt = 0.f;
    bf16 out[16];
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int key = key0 + (v & 3) + 8 * (v >> 2);
      const float sraw = acc[v];
      const float s = sraw * temp;
      float g = (s >= lo && s <= 0.f) ? c_nn * s : 0.f;  // clamp grad, inclusive bounds
      if (key == amax) g += gmax;
      if (dg && key < a.Nk_eff) g += c_dg * dg[key];
      g = (row_ok && key < a.Nk_eff) ? g : 0.f;
      dt += g * sraw;
      out[v] = (bf16)g;
    }
    accd += (double)dt;
    store_tile(a.dS, a.CT, rt, (long long)j * nkb + kb, lane, out);
  }

  // Workgroup partial of dL/dtemp, in double.
  const double v = wave_sum_d(accd);
  if (lane == 0) red[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < WAVES; ++w) t += red[w];
    a.part[blockIdx.y * gridDim.x + blockIdx.x] = t;
  }
}

// clip[i][j] = sum_q w_q rowmax[j][i*Nq+q] / norm_i  (model.py:389-391, 507-512);
// also writes qw[r] = d clip / d rowmax for the backward.
__global__ __launch_bounds__(256) void clip_reduce_kernel(const float* __restrict__ rowmax, int R_pad,
                                                          int Nq, int Bq, int Bk,
                                                          const float* __restrict__ qmask,
                                                          float* __restrict__ clip, float* __restrict__ qw) {
  // one wave per (i, j): every row's loads in flight at once (a wave looping over 64 rows
  // made this a latency-bound 0.14 ms launch at B = 256)
  const int j = blockIdx.x;
  const int lane = threadIdx.x & 63, i = blockIdx.y * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (i >= Bq) return;
  float s = 0.f, cnt = 0.f;
  const float* rm = rowmax + (size_t)j * R_pad + (size_t)i * Nq;
  for (int q = lane; q < Nq; q += 64) {
    const float w = qmask ? qmask[(size_t)i * Nq + q] : 1.f;
    s += rm[q] * w;
    cnt += w;
  }
  s = wave_sum(s);
  cnt = wave_sum(cnt);
  const float norm = qmask ? fmaxf(cnt, 1e-7f) : (float)Nq;
  if (lane == 0) clip[(size_t)i * Bk + j] = s / norm;
  if (j == 0 && qw) {
    for (int q = lane; q < Nq; q += 64) {
      const float w = qmask ? qmask[(size_t)i * Nq + q] : 1.f;
      qw[(size_t)i * Nq + q] = w / norm;
    }
  }
}

// AV temporal smoothness on the diagonal pairs (model.py:394-408):
//   l_smooth = sum_{i,q>=1,k} (S_ii[q,k] - S_ii[q-1,k])^2 / cnt
// Writes part[i] = the sample's sum, g[i][q][k] = d l_smooth / d S_ii[q,k] and
// dt_part[i] = sum g * S (for d/dtemp; S = temp * S_raw).
__global__ __launch_bounds__(1024) void diag_smooth_kernel(const float* __restrict__ dS_in, int Nq, int Nk_pad,
                                                           int Nk_eff, double inv_cnt,
                                                           double* __restrict__ part, float* __restrict__ g,
                                                           double* __restrict__ dt_part) {
  __shared__ double red[16];
  const int i = blockIdx.x;
  const float* S = dS_in + (size_t)i * Nq * Nk_pad;
  float* G = g + (size_t)i * Nq * Nk_pad;
  double acc = 0.0, dacc = 0.0;
  const float two_inv = (float)(2.0 * inv_cnt);
  const int n = Nq * Nk_eff;
  // four elements per thread per pass, their loads issued together (one element per pass made
  // this a latency-bound 0.16 ms launch at c3)
  for (int e0 = threadIdx.x; e0 < n; e0 += 4 * blockDim.x) {
    float s[4], sp[4], sn[4];
    int q[4], k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * (int)blockDim.x, n - 1);
      q[u] = e / Nk_eff;
      k[u] = e - q[u] * Nk_eff;
      s[u] = S[(size_t)q[u] * Nk_pad + k[u]];
      sp[u] = q[u] >= 1 ? S[(size_t)(q[u] - 1) * Nk_pad + k[u]] : 0.f;
      sn[u] = q[u] + 1 < Nq ? S[(size_t)(q[u] + 1) * Nk_pad + k[u]] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + u * (int)blockDim.x >= n) break;
      float grad = 0.f;
      if (q[u] >= 1) {
        const float d = s[u] - sp[u];
        acc += (double)(d * d);
        grad += two_inv * d;
      }
      if (q[u] + 1 < Nq) grad -= two_inv * (sn[u] - s[u]);
      G[(size_t)q[u] * Nk_pad + k[u]] = grad;
      dacc += (double)grad * (double)s[u];
    }
  }
  const double t = block_sum_d(acc, red);
  const double dt = block_sum_d(dacc, red);
  if (threadIdx.x == 0) { part[i] = t; dt_part[i] = dt; }
}

// TV patch-usage sparsity on the diagonal pairs (model.py:527-540):
//   P = softmax_k S_ii[t,:];  frac[k] = sum_t P[t,k] / Nt;  loss = sum relu(frac-thr)^2 / cnt
// Writes part[i], g[i][t][k] = d loss / d S_ii[t,k] and dt_part[i] = sum g * S.
constexpr int SP_MAXT = 1024;
__global__ __launch_bounds__(256) void diag_sparsity_kernel(const float* __restrict__ S_g, int Nt, int Nk_pad,
                                                            int Nk_eff, float thr, double inv_cnt,
                                                            double* __restrict__ part, float* __restrict__ G_g,
                                                            double* __restrict__ dt_part) {
  extern __shared__ float sh[];  // per-column gradient wrt P [Nk_eff]
  __shared__ float rmx[SP_MAXT], rinv[SP_MAXT];
  __shared__ double red[4];
  const int i = blockIdx.x;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const float* S = S_g + (size_t)i * Nt * Nk_pad;
  float* G = G_g + (size_t)i * Nt * Nk_pad;
  // 1) row softmax statistics
  for (int t = wave; t < Nt; t += nw) {
    const float* r = S + (size_t)t * Nk_pad;
    float mx = -INFINITY;
    for (int k = lane; k < Nk_eff; k += 64) mx = fmaxf(mx, r[k]);
    mx = wave_max(mx);
    float sum = 0.f;
    for (int k = lane; k < Nk_eff; k += 64) sum += __expf(r[k] - mx);
    sum = wave_sum(sum);
    if (lane == 0) { rmx[t] = mx; rinv[t] = 1.f / sum; }
  }
  __syncthreads();
  // 2) frac, excess, loss partial, per-column gradient wrt P (incl. the 1/Nt of frac)
  double acc = 0.0;
  const float scale = (float)(2.0 * inv_cnt) / (float)Nt;
  for (int k = threadIdx.x; k < Nk_eff; k += blockDim.x) {
    float f = 0.f;
    for (int t = 0; t < Nt; ++t) f += __expf(S[(size_t)t * Nk_pad + k] - rmx[t]) * rinv[t];
    f /= (float)Nt;
    const float ex = f - thr;
    const float r = ex > 0.f ? ex : 0.f;   // relu'(0) = 0 as in torch
    acc += (double)r * (double)r;
    sh[k] = scale * r;
  }
  const double tot = block_sum_d(acc, red);  // includes a barrier
  // 3) softmax backward per row
  double dacc = 0.0;
  for (int t = wave; t < Nt; t += nw) {
    const float* r = S + (size_t)t * Nk_pad;
    float* gr = G + (size_t)t * Nk_pad;
    float dot = 0.f;
    for (int k = lane; k < Nk_eff; k += 64) dot += __expf(r[k] - rmx[t]) * rinv[t] * sh[k];
    dot = wave_sum(dot);
    for (int k = lane; k < Nk_eff; k += 64) {
      const float pk = __expf(r[k] - rmx[t]) * rinv[t];
      const float gv = pk * (sh[k] - dot);
      gr[k] = gv;
      dacc += (double)gv * (double)r[k];
    }
  }
  const double dt = block_sum_d(dacc, red);
  if (threadIdx.x == 0) { part[i] = tot; dt_part[i] = dt; }
}

// The forward stores the unit l_nonneg gradient divided by su = |temp| (1 when temp == 0; the
// per-element multiply moved here and into the tile GEMMs' alpha): the terms below are added
// divided by su too, so the tiled dS holds dS_unit / su and alpha carries su.
__device__ __forceinline__ float unit_scale(const float* temp) {
  const float t = *temp;
  return 1.f / (t != 0.f ? fabsf(t) : 1.f);
}

// Sparse (max) term of dS, added in place to the tiled unit l_nonneg gradient written by the
// forward: dS[r][j*Nk_pad + argmax[j][r]] += ratio / su * dclip[i][j] * qw[r]  (the backward of
// max over keys, model.py:389/507, feeding mean/masked-mean and the CE).
// part[block] = sum dclip * qw * rowmax (-> d/dtemp of this term).
// Column of key `key` of key sample j in the tiled dS: j Nk_pad + key, or with compact key tiles
// (kt = the stored-tile prefix sum, triad_pairsim_problem.k_tiles) 32 kt[j] + key, -1 when the key
// lies in the sample's unstored all-zero last tile.
__device__ __forceinline__ long long ds_col(const int* __restrict__ kt, int Nk_pad, int j, int key) {
  if (!kt) return (long long)j * Nk_pad + key;
  const int t0 = kt[j];
  return key < 32 * (kt[j + 1] - t0) ? (long long)t0 * 32 + key : -1;
}

__device__ __forceinline__ long long tile_elem(long long CT, int r, long long c) {
  const int kl = (int)(c & 31);
  const int lane = (r & 31) + 32 * ((kl >> 2) & 1);
  const int v = (kl & 3) + 4 * (kl >> 3);
  return ((long long)(r >> 5) * CT + (c >> 5)) * 1024 + ds_chunk(2 * lane + (v >> 3)) * 8 + (v & 7);
}

#ifndef PATCH_U
#define PATCH_U 4   // elements per thread per pass (A/B knob; round 6, tools/gpu_ab_patch.sh,
#endif              // profiles/r06_patch_ilp_ab.log: 8 / 16 and 2048 / 4096 workgroups 2-20 % slower)
// Four elements per thread per pass with all their loads issued together, 32-bit index math:
// one element per pass (a dependent argmax -> dS round trip each, 64-bit divisions) made the AV
// patch a latency-bound 0.3 ms launch at c3.
__global__ __launch_bounds__(256) void dS_patch_max_kernel(bf16* __restrict__ dS, long long CT, int R, int R_pad,
                                                           int Nq, int Bk, int Nk_pad,
                                                           const int* __restrict__ argmax,
                                                           const float* __restrict__ rowmax,
                                                           const float* __restrict__ dclip,
                                                           const float* __restrict__ qw, float ratio,
                                                           double* __restrict__ part, const int* __restrict__ kt,
                                                           const float* __restrict__ temp) {
  __shared__ double red[4];
  double acc = 0.0;
  const float rs = ratio * unit_scale(temp);
  const int total = Bk * R;   // < 2^31 (host check)
  const int stride = gridDim.x * blockDim.x;
  for (int e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += PATCH_U * stride) {
    float w[PATCH_U], rm[PATCH_U], old[PATCH_U];
    bf16* p[PATCH_U];
#pragma unroll
    for (int u = 0; u < PATCH_U; ++u) {
      const int e = min(e0 + u * stride, total - 1);
      const int j = e / R, r = e - j * R;
      const int i = r / Nq;
      w[u] = dclip[(size_t)i * Bk + j] * qw[r];
      rm[u] = rowmax[(size_t)j * R_pad + r];
      const int key = argmax[(size_t)j * R_pad + r];
      const long long c = ds_col(kt, Nk_pad, j, key);
      p[u] = c < 0 ? nullptr : dS + tile_elem(CT, r, c);   // unstored zero tile: K there is zero
    }
#pragma unroll
    for (int u = 0; u < PATCH_U; ++u) old[u] = p[u] ? (float)*p[u] : 0.f;
#pragma unroll
    for (int u = 0; u < PATCH_U; ++u) {
      if (e0 + u * stride >= total) break;
      if (p[u]) *p[u] = (bf16)(old[u] + rs * w[u]);
      acc += (double)w[u] * (double)rm[u];
    }
  }
  const double t = block_sum_d(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

// Diagonal regulariser term: dS[i*Nq+q][(i+off)*Nk_pad + k] += ratio / su * g[i][q][k] (four
// elements per thread per pass, as above).
__global__ __launch_bounds__(256) void dS_patch_diag_kernel(bf16* __restrict__ dS, long long CT, int Bq, int Nq,
                                                            int Nk_pad, int Nk_eff, int diag_off,
                                                            const float* __restrict__ g, float ratio,
                                                            const int* __restrict__ kt,
                                                            const float* __restrict__ temp) {
  const int total = Bq * Nq * Nk_eff;   // < 2^31 (host check)
  const float rs = ratio * unit_scale(temp);
  const int stride = gridDim.x * blockDim.x;
  for (int e0 = blockIdx.x * blockDim.x + threadIdx.x; e0 < total; e0 += 4 * stride) {
    float gv[4], old[4];
    bf16* p[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * stride, total - 1);
      const int k = e % Nk_eff, iq = e / Nk_eff;
      const int i = iq / Nq;
      gv[u] = g[(size_t)iq * Nk_pad + k];
      const long long c = ds_col(kt, Nk_pad, i + diag_off, k);
      p[u] = c < 0 ? nullptr : dS + tile_elem(CT, iq, c);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) old[u] = p[u] ? (float)*p[u] : 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + u * stride >= total) break;
      if (p[u]) *p[u] = (bf16)(old[u] + rs * gv[u]);
    }
  }
}

// Loss head over the B x B clip matrix (model.py:430-472 / 544-593), one workgroup.
// out: [0] total [1] ce [2] reg [3] 0.01*smooth (AV) / sparsity (TV)
//      [4..9] pos_mean pos_std neg_mean neg_std separation hardest_negative
//      [10] l_nonneg [11] l_cal [12] diag regulariser (l_smooth / sparsity)
// dclip: d ce / d clip (unit upstream gradient).
// Row (r < B) / column (r >= B) log-sum-exp of the clip matrix, one wave per line, all lines in
// parallel (inside the one-workgroup loss head this phase was a latency-bound 0.1+ ms loop).
__global__ __launch_bounds__(256) void clip_lse_kernel(const float* __restrict__ clip, int B,
                                                       float* __restrict__ lse) {
  const int lane = threadIdx.x & 63, r = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (r >= 2 * B) return;
  const bool col = r >= B;
  const int x = col ? r - B : r;
  float mx = -INFINITY;
  for (int y = lane; y < B; y += 64) mx = fmaxf(mx, col ? clip[(size_t)y * B + x] : clip[(size_t)x * B + y]);
  mx = wave_max(mx);
  float s = 0.f;
  for (int y = lane; y < B; y += 64) s += expf((col ? clip[(size_t)y * B + x] : clip[(size_t)x * B + y]) - mx);
  s = wave_sum(s);
  if (lane == 0) lse[r] = mx + logf(s);
}

__global__ __launch_bounds__(1024) void losshead_kernel(const float* __restrict__ clip, int B, int kind,
                                                        const float* __restrict__ temp_p,
                                                        const double* __restrict__ nn_part, int n_nn,
                                                        double inv_nel,
                                                        const double* __restrict__ dg_part, int n_dg,
                                                        double inv_dg, float w_sparse,
                                                        float* __restrict__ out, float* __restrict__ dclip,
                                                        const float* __restrict__ lse /* [2B], clip_lse_kernel */) {
  __shared__ double redd[16];
  __shared__ float redf[16];
  double ce = 0.0, pos = 0.0, neg = 0.0;
  float hard = -INFINITY;
  for (int i = threadIdx.x; i < B; i += blockDim.x) {
    const float c = clip[(size_t)i * B + i];
    ce += (double)(lse[i] - c) + (double)(lse[B + i] - c);
    pos += c;
  }
  const float inv2b = 0.5f / (float)B;
  const int BB = B * B;
  const int bd = blockDim.x;
  // four elements per thread per pass, loads issued together (latency-bound otherwise)
  for (int e0 = threadIdx.x; e0 < BB; e0 += 4 * bd) {
    float c[4], li[4], lj[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = min(e0 + u * bd, BB - 1);
      const int i = e / B, j = e - i * B;
      c[u] = clip[e];
      li[u] = lse[i];
      lj[u] = lse[B + j];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * bd;
      if (e >= BB) break;
      const int i = e / B, j = e - i * B;
      float g = expf(c[u] - li[u]) + expf(c[u] - lj[u]);
      if (i == j) g -= 2.f;
      else { neg += c[u]; hard = fmaxf(hard, c[u]); }
      dclip[e] = g * inv2b;
    }
  }
  ce = block_sum_d(ce, redd);
  pos = block_sum_d(pos, redd);
  neg = block_sum_d(neg, redd);
  hard = block_max(hard, redf);
  const double nneg = (double)B * B - B;
  const double pm = pos / B, nm = neg / nneg;
  double pv = 0.0, nv = 0.0;
  for (int e0 = threadIdx.x; e0 < BB; e0 += 4 * bd) {
    float c[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) c[u] = clip[min(e0 + u * bd, BB - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * bd;
      if (e >= BB) break;
      const int i = e / B, j = e - i * B;
      const double d = (double)c[u] - (i == j ? pm : nm);
      if (i == j) pv += d * d; else nv += d * d;
    }
  }
  pv = block_sum_d(pv, redd);
  nv = block_sum_d(nv, redd);
  double nn = 0.0;
  for (int e = threadIdx.x; e < n_nn; e += blockDim.x) nn += nn_part[e];
  nn = block_sum_d(nn, redd);
  double dg = 0.0;
  for (int e = threadIdx.x; e < n_dg; e += blockDim.x) dg += dg_part[e];
  dg = block_sum_d(dg, redd);
  if (threadIdx.x == 0) {
    const double cev = ce / (2.0 * B);
    const double l_nn = nn * inv_nel;
    const double l_dg = dg * inv_dg;  // 0 * inf -> NaN when the diagonal set is empty (reference: mean of empty)
    double l_cal = 0.0, reg, sm;
    if (kind == 0) {
      const double lt = -log((double)*temp_p);
      l_cal = lt > 0.0 ? lt * lt : 0.0;
      reg = 20.0 * l_cal + 0.15 * l_nn + 0.01 * l_dg;
      sm = 0.01 * l_dg;
    } else {
      reg = 0.15 * l_nn + (double)w_sparse * l_dg;
      sm = l_dg;
    }
    out[0] = (float)(cev + reg);
    out[1] = (float)cev;
    out[2] = (float)reg;
    out[3] = (float)sm;
    out[4] = (float)pm;
    out[5] = (float)sqrt(pv / (B - 1));
    out[6] = (float)nm;
    out[7] = (float)sqrt(nv / (nneg - 1));
    out[8] = (float)(pm - nm);
    out[9] = hard;
    out[10] = (float)l_nn;
    out[11] = (float)l_cal;
    out[12] = (float)l_dg;
  }
}

// dL/dtemp = sum_k w[k] * sum(part_k) + w[3] * d l_cal / d temp   (AV only has l_cal, model.py:420-424)
// fast path: parts = {sum S*S_raw (nonneg), sum dclip*qw*rowmax, sum g*S (diag)},
//            w = {c_nn, c_ce / temp, c_diag / temp, c_cal}
// recompute path: parts = {sum dS*S_raw}, w = {1, -, -, c_cal}
__global__ void dtemp_finalize_kernel(const double* __restrict__ p0, int n0, const double* __restrict__ p1, int n1,
                                      const double* __restrict__ p2, int n2, const float* __restrict__ temp_p,
                                      const float* __restrict__ w, int has_cal, float* __restrict__ out) {
  __shared__ double red[4];
  double s0 = 0.0, s1 = 0.0, s2 = 0.0;
  for (int e = threadIdx.x; e < n0; e += blockDim.x) s0 += p0[e];
  for (int e = threadIdx.x; e < n1; e += blockDim.x) s1 += p1[e];
  for (int e = threadIdx.x; e < n2; e += blockDim.x) s2 += p2[e];
  s0 = block_sum_d(s0, red);
  s1 = block_sum_d(s1, red);
  s2 = block_sum_d(s2, red);
  if (threadIdx.x == 0) {
    double s = (double)w[0] * s0 + (n1 ? (double)w[1] * s1 : 0.0) + (n2 ? (double)w[2] * s2 : 0.0);
    if (has_cal) {
      const double t = (double)*temp_p;
      const double x = -log(t);
      if (x >= 0.0) s += (double)w[3] * 2.0 * x * (-1.0 / t);
    }
    out[0] = (float)s;
  }
}

// Key-sample split of the (256-row block, key samples) grid: the count minimising
// (dispatch rounds of one workgroup per CU over 256 CUs) x (key samples per workgroup + the
// query-fragment load, ~0.3 sample). Whole rounds keep the last wave of workgroups from leaving
// CUs idle; fewer, longer workgroups amortise the query load (TV: 32 row blocks -> 8 splits of
// 32 samples, one round; AV: 199 row blocks -> 9 splits of 29, 7 rounds). Measured against the former fixed
// 2048-workgroup target: AV train forward 3.00 -> 2.96 ms, TV 0.567 -> 0.532 ms
// (profiles/r02_fwd_grid_ab.log).
int grid_for(int R_pad, int Bk, int* jpw, int* ysplit) {
  const int xb = R_pad / ROWS_PER_WG;
  double best = 1e30;
  int ys = 1;
  for (int y = 1; y <= Bk; ++y) {
    const int j = (Bk + y - 1) / y, ya = (Bk + j - 1) / j;
    const double c = (double)((xb * ya + 255) / 256) * (j + 0.3);
    if (c < best - 1e-9) { best = c; ys = ya; }
  }
  *jpw = (Bk + ys - 1) / ys;
  *ysplit = (Bk + *jpw - 1) / *jpw;
  return xb;
}

int check_shape(int R, int R_pad, int Nq, int Bk, int Nk_pad, int Nk_eff, int D_) {
  if (D_ != D || R_pad % ROWS_PER_WG || R > R_pad || Nq <= 0 || Bk <= 0 || Nk_pad % 32 ||
      Nk_eff <= 0 || Nk_eff > Nk_pad)
    return TRIAD_EINVAL;
  return TRIAD_OK;
}

}  // namespace

extern "C" {

int triad_pairsim_nparts(int R_pad, int Bk) {
  int jpw, ys;
  const int xb = grid_for(R_pad, Bk, &jpw, &ys);
  return xb * ys;
}

int triad_pairsim_fwd(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                      int Nk_eff, int D_, const float* temp, float clamp_lo, int diag, int diag_off,
                      float* rowmax, int* argmax, double* nn_part, float* diagS, void* dS, long long CT,
                      double* st_part, const int* k_len, hipStream_t stream) {
  if (int e = check_shape(R, R_pad, Nq, Bk, Nk_pad, Nk_eff, D_)) return e;
  if (dS && (CT < (long long)Bk * (Nk_pad / 32) || !st_part)) return TRIAD_EINVAL;
  if (k_len && (dS || diagS)) return TRIAD_EINVAL;  // per-sample key lengths: forward-only use
  if (diag && diagS && (diag_off < 0 || diag_off + Bq > Bk)) return TRIAD_EINVAL;
  PairArgs a = {};
  a.Q = (const bf16*)Q; a.K = (const bf16*)K;
  a.R = R; a.R_pad = R_pad; a.Nq = Nq; a.Bq = Bq; a.Bk = Bk; a.Nk_pad = Nk_pad; a.Nk_eff = Nk_eff;
  a.diag = diag; a.diag_off = diag_off; a.temp = temp; a.clamp_lo = clamp_lo;
  a.rowmax = rowmax; a.argmax = argmax; a.part = nn_part; a.diagS = diagS;
  a.dS = (bf16*)dS; a.CT = CT; a.part2 = st_part; a.klen = k_len;
  int ys;
  const int xb = grid_for(R_pad, Bk, &a.j_per_wg, &ys);
  return triad_pairsim_fwd2_launch(Q, K, R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff, temp, clamp_lo, diag, diag_off,
                                   rowmax, argmax, nn_part, diagS, dS, CT, st_part, k_len, xb, ys, a.j_per_wg,
                                   stream);
}

int triad_pairsim_fwd_multi(const triad_pairsim_problem* problems, int n, hipStream_t stream) {
  if (!problems || n < 1 || n > 2) return TRIAD_EINVAL;
  int xb[2], ys[2], jpw[2];
  for (int i = 0; i < n; ++i) {
    const triad_pairsim_problem& p = problems[i];
    if (int e = check_shape(p.R, p.R_pad, p.Nq, p.Bk, p.Nk_pad, p.Nk_eff, D)) return e;
    // (compact key tiles: CT >= k_tiles[Bk] is the caller's, the prefix sum lives on the device)
    if (p.dS && (p.CT < (p.k_tiles ? 1LL : (long long)p.Bk * (p.Nk_pad / 32)) || !p.st_part)) return TRIAD_EINVAL;
    if (!p.Q || !p.K || !p.temp || !p.rowmax || !p.argmax || !p.nn_part) return TRIAD_EINVAL;
    if (p.diag && p.diagS && (p.diag_off < 0 || p.diag_off + p.Bq > p.Bk)) return TRIAD_EINVAL;
    xb[i] = grid_for(p.R_pad, p.Bk, &jpw[i], &ys[i]);  // same decomposition as triad_pairsim_nparts
  }
  return triad_pairsim_fwd_multi_launch(problems, xb, ys, jpw, n, stream);
}

int triad_pairsim_diag(const triad_pairsim_problem* problems, int n, hipStream_t stream) {
  if (!problems || n < 1 || n > 2) return TRIAD_EINVAL;
  for (int i = 0; i < n; ++i) {
    const triad_pairsim_problem& p = problems[i];
    if (int e = check_shape(p.R, p.R_pad, p.Nq, p.Bk, p.Nk_pad, p.Nk_eff, D)) return e;
    if (p.diag && p.diagS && (!p.Q || !p.K || !p.temp || p.diag_off < 0 || p.diag_off + p.Bq > p.Bk))
      return TRIAD_EINVAL;
    // diag_sim addresses K in the padded layout (sample j at rows j * Nk_pad); a compact key set
    // (k_tiles) has fewer rows and would be read past its end
    if (p.diag && p.diagS && p.k_tiles) return TRIAD_EINVAL;
  }
  return triad_pairsim_diag_launch(problems, n, stream);
}

int triad_clip_reduce(const float* rowmax, int R_pad, int Nq, int Bq, int Bk, const float* qmask,
                      float* clip, float* qw, hipStream_t stream) {
  if (Bq <= 0 || Bk <= 0 || Nq <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(clip_reduce_kernel, dim3(Bk, (Bq + 3) / 4), dim3(256), 0, stream, rowmax, R_pad, Nq, Bq, Bk,
                     qmask, clip, qw);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_diag_smooth(const float* diagS, int Bq, int Nq, int Nk_pad, int Nk_eff, double cnt, double* part,
                      float* g, double* dt_part, hipStream_t stream) {
  if (Bq <= 0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(diag_smooth_kernel, dim3(Bq), dim3(1024), 0, stream, diagS, Nq, Nk_pad, Nk_eff,
                     cnt > 0.0 ? 1.0 / cnt : 0.0, part, g, dt_part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_diag_sparsity(const float* diagS, int Bq, int Nt, int Nk_pad, int Nk_eff, float thr, double cnt,
                        double* part, float* g, double* dt_part, hipStream_t stream) {
  if (Bq <= 0 || Nk_eff > 16384 || Nt > SP_MAXT || cnt <= 0.0) return TRIAD_EINVAL;
  hipLaunchKernelGGL(diag_sparsity_kernel, dim3(Bq), dim3(256), Nk_eff * sizeof(float), stream, diagS, Nt,
                     Nk_pad, Nk_eff, thr, 1.0 / cnt, part, g, dt_part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_losshead(const float* clip, int B, int kind, const float* temp, const double* nn_part, int n_nn,
                   double n_el, const double* dg_part, int n_dg, double dg_cnt, float w_sparse, float* out,
                   float* dclip, float* lse_scratch, hipStream_t stream) {
  if (B < 2 || B > 46340 || (kind != 0 && kind != 1)) return TRIAD_EINVAL;  // B * B fits an int
  const double inv_dg = dg_cnt > 0.0 ? 1.0 / dg_cnt : NAN;
  hipLaunchKernelGGL(clip_lse_kernel, dim3((2 * B + 3) / 4), dim3(256), 0, stream, clip, B, lse_scratch);
  hipLaunchKernelGGL(losshead_kernel, dim3(1), dim3(1024), 0, stream, clip, B, kind, temp, nn_part, n_nn,
                     1.0 / n_el, dg_part, n_dg, inv_dg, w_sparse, out, dclip, (const float*)lse_scratch);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_pairsim_dS(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                     int Nk_eff, int D_, const float* temp, float clamp_lo, int diag, int diag_off,
                     const int* argmax, const float* dclip, const float* qw, const float* dSdiag,
                     const float* coef, void* dS, long long CT, double* dt_part, hipStream_t stream) {
  if (int e = check_shape(R, R_pad, Nq, Bk, Nk_pad, Nk_eff, D_)) return e;
  if (CT < (long long)Bk * (Nk_pad / 32)) return TRIAD_EINVAL;
  PairArgs a = {};
  a.Q = (const bf16*)Q; a.K = (const bf16*)K;
  a.R = R; a.R_pad = R_pad; a.Nq = Nq; a.Bq = Bq; a.Bk = Bk; a.Nk_pad = Nk_pad; a.Nk_eff = Nk_eff;
  a.diag = diag; a.diag_off = diag_off; a.temp = temp; a.clamp_lo = clamp_lo;
  a.argmax = (int*)argmax; a.dclip = dclip; a.qw = qw; a.dSdiag = dSdiag; a.coef = coef;
  a.dS = (bf16*)dS; a.CT = CT; a.part = dt_part;
  int ys;
  const int xb = grid_for(R_pad, Bk, &a.j_per_wg, &ys);
  hipLaunchKernelGGL(pairsim_dS_kernel, dim3(xb, ys), dim3(512), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_dS_patch_tiles(void* dS, long long CT, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad, int Nk_eff,
                         int diag_off, const int* argmax, const float* rowmax, const float* dclip, const float* qw,
                         float ratio_max, const float* gdiag, float ratio_diag, double* max_part, int n_max_part,
                         const float* temp, const int* k_tiles, hipStream_t stream) {
  if (R <= 0 || Bk <= 0 || n_max_part <= 0 || Nk_pad % 32 || CT <= 0 || !temp) return TRIAD_EINVAL;
  if (!k_tiles && CT < (long long)Bk * (Nk_pad / 32)) return TRIAD_EINVAL;
  if ((long long)Bk * R >= (1LL << 31) || (long long)Bq * Nq * Nk_eff >= (1LL << 31)) return TRIAD_EINVAL;
  hipLaunchKernelGGL(dS_patch_max_kernel, dim3(n_max_part), dim3(256), 0, stream, (bf16*)dS, CT, R, R_pad, Nq, Bk,
                     Nk_pad, argmax, rowmax, dclip, qw, ratio_max, max_part, k_tiles, temp);
  if (gdiag) {
    const long long total = (long long)Bq * Nq * Nk_eff;
    long long blocks = (total + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(dS_patch_diag_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (bf16*)dS, CT, Bq, Nq,
                       Nk_pad, Nk_eff, diag_off, gdiag, ratio_diag, k_tiles, temp);
  }
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_dS_patch(void* dS, long long CT, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad, int Nk_eff,
                   int diag_off, const int* argmax, const float* rowmax, const float* dclip, const float* qw,
                   float ratio_max, const float* gdiag, float ratio_diag, double* max_part, int n_max_part,
                   const float* temp, hipStream_t stream) {
  return triad_dS_patch_tiles(dS, CT, R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff, diag_off, argmax, rowmax, dclip, qw,
                              ratio_max, gdiag, ratio_diag, max_part, n_max_part, temp, nullptr, stream);
}

int triad_dtemp_finalize(const double* p0, int n0, const double* p1, int n1, const double* p2, int n2,
                         const float* temp, const float* w, int has_cal, float* out, hipStream_t stream) {
  hipLaunchKernelGGL(dtemp_finalize_kernel, dim3(1), dim3(256), 0, stream, p0, n0, p1, n1, p2, n2, temp, w, has_cal,
                     out);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

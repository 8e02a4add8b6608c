// Forward of the fused similarity head, one wave per SIMD ("64 query rows per wave").
//
// Same contract as pairsim_kernel<0> (pairsim.hip; SajayR/TRIAD model.py:370-392 / 490-514 /
// 417-418 / 524-525): rowmax / argmax per (key sample, query row), l_nonneg partial sums,
// diagonal S, and (training) the unit l_nonneg gradient written in the tiled dS layout.
//
// Structure (gfx950, 256-thread workgroup = 4 waves = one per SIMD, 512 VGPRs each):
//  * each wave keeps the bf16 fragments of 64 query rows x 512 features in VGPRs
//    (2 x 128 registers) for the whole launch: every key fragment read from LDS feeds two
//    v_mfma_f32_32x32x16_bf16 (halving LDS traffic per MFMA vs 32 rows per wave);
//  * key tiles (32 keys x 512 x bf16 = 32 KB) stream through a 3-slot LDS ring by 16-byte
//    LDS-DMA issued two tiles ahead; one counted `s_waitcnt vmcnt(8)` + raw s_barrier per tile
//    (the DMA of the next tile stays in flight across it);
//  * the epilogue of tile b-1 (scale, max/argmax, clamp^2, unit dS, stores) is software-
//    pipelined against the MFMA chain of tile b in one basic block, so its VALU work issues
//    in the MFMA shadows instead of after them.
#include "common.h"

namespace {

constexpr int D = 512;
constexpr int NS = D / 16;
constexpr int WAVES = 4;
constexpr int ROWS_PER_WG = 64 * WAVES;  // 256, as pairsim_kernel
constexpr int KT_ELEMS = 32 * D;
constexpr int NBUF = 3;
constexpr int GLDS_PER_TILE = 32 / WAVES;  // wave-instructions per wave per key tile (8)

struct FwdArgs {
  const bf16* Q;
  const bf16* K;
  int R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff, j_per_wg;
  int diag, diag_off;
  const float* temp;
  float clamp_lo;
  float* rowmax;
  int* argmax;
  double* part;
  float* diagS;
  bf16* dS;
  long long CT;
  double* part2;
  const int* klen;
};

__device__ __forceinline__ void stage_tile(const FwdArgs& a, bf16* dst, int j, int kb, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < GLDS_PER_TILE; ++u) {
    const int t = wave * GLDS_PER_TILE + u;
    const bf16* src = a.K + ((size_t)j * a.Nk_pad + kb * 32 + t) * D + ((lane ^ (t & 15)) * 8);
    glds16(src, dst + t * D);
  }
}

struct RowState {
  int row, qi, qq;
  bool ok;
  float m;
  int am;
};

// one 32x32 tile epilogue (branch-free math): running max/argmax, l_nonneg sum, sum of S*S_raw,
// and (training) the unit dS tile, packed to bf16 pairs and stored at once (short live range)
__device__ __forceinline__ void tile_epi(const f32x16& acc, RowState& rs, int nvalid, int key0, int h, float temp,
                                         float lo, float& nn, float& st, bf16* dst) {
  unsigned pk[8];
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const bool ok = 4 * h + (v & 3) + 8 * (v >> 2) < nvalid;
    const float s = acc[v] * temp;
    const bool better = ok && s > rs.m;  // keys ascend with v: strict > keeps the first index
    rs.m = better ? s : rs.m;
    rs.am = better ? key0 + (v & 3) + 8 * (v >> 2) : rs.am;
    const float c = ok ? fminf(fmaxf(s, lo), 0.f) : 0.f;
    nn += c * c;
    const float d = (ok && c == s) ? s : 0.f;  // S on [lo, 0]: unit grad of the l_nonneg term
    st += d * acc[v];
    const bf16 db = (bf16)d;
    const unsigned u = (unsigned)__builtin_bit_cast(unsigned short, db);
    pk[v >> 1] = (v & 1) ? (pk[v >> 1] | (u << 16)) : u;
  }
  if (dst) {
    *(uint4*)dst = make_uint4(pk[0], pk[1], pk[2], pk[3]);
    *(uint4*)(dst + 8) = make_uint4(pk[4], pk[5], pk[6], pk[7]);
  }
}

__global__ __launch_bounds__(256, 1) void pairsim_fwd2_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 kbuf[NBUF * KT_ELEMS + 16 * WAVES];
  double* red = (double*)(kbuf + NBUF * KT_ELEMS);

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, ql = lane & 31;
  RowState rs[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    rs[x].row = blockIdx.x * ROWS_PER_WG + wave * 64 + x * 32 + ql;
    rs[x].ok = rs[x].row < a.R;
    rs[x].qi = rs[x].ok ? rs[x].row / a.Nq : -1;
    rs[x].qq = rs[x].ok ? rs[x].row - rs[x].qi * a.Nq : 0;
    rs[x].m = -INFINITY;
    rs[x].am = 0;
  }
  const int rt0 = (blockIdx.x * ROWS_PER_WG + wave * 64) / 32;

  const int j0 = blockIdx.y * a.j_per_wg;
  const int j1 = min(a.Bk, j0 + a.j_per_wg);
  const int nkb = a.Nk_pad / 32;
  const int nblocks = (j1 - j0) * nkb;
  if (nblocks <= 0) {
    if (threadIdx.x == 0) {
      a.part[blockIdx.y * gridDim.x + blockIdx.x] = 0.0;
      if (a.part2) a.part2[blockIdx.y * gridDim.x + blockIdx.x] = 0.0;
    }
    return;
  }

  // prologue: two tiles in flight
  stage_tile(a, kbuf, j0, 0, wave, lane);
  if (nblocks > 1) stage_tile(a, kbuf + KT_ELEMS, j0 + 1 / nkb, 1 % nkb, wave, lane);

  // query fragments live in AGPRs (the MFMA reads srcB from the AccVGPR file), leaving the
  // 256 architectural VGPRs to accumulators, key fragments and the epilogue
  bf16x8 qf0[NS], qf1[NS];
  {
    const bf16* q0 = a.Q + (size_t)rs[0].row * D + 8 * h;
    const bf16* q1 = a.Q + (size_t)rs[1].row * D + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 t0 = *(const bf16x8*)(q0 + 16 * s);
      const bf16x8 t1 = *(const bf16x8*)(q1 + 16 * s);
      asm volatile("; q0 -> agpr" : "=a"(qf0[s]) : "0"(t0));
      asm volatile("; q1 -> agpr" : "=a"(qf1[s]) : "0"(t1));
    }
  }
  int koff[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) koff[k] = ((2 * k + h) ^ (ql & 15)) * 8;
  const float temp = *a.temp;
  const float lo = a.clamp_lo;
  double accd = 0.0, accd2 = 0.0;
  int nk = a.Nk_eff;  // valid keys of the sample whose tile is being finished

  f32x16 cA0, cA1, cB0, cB1;

  // MFMA chain of tile b into (c0, c1) from ring slot b % NBUF
  auto chain = [&](int b, f32x16& c0, f32x16& c1) {
    const bf16* kt = kbuf + (b % NBUF) * KT_ELEMS + ql * D;
    c0 = (f32x16){};
    c1 = (f32x16){};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 af = *(const bf16x8*)(kt + koff[s & 7] + (s >> 3) * 128);
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c0) : "v"(af), "a"(qf0[s]));
      asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(c1) : "v"(af), "a"(qf1[s]));
    }
    // the compiler's hazard recognizer does not see through inline asm: cover the
    // MFMA-result -> VALU-read wait states before anyone reads (c0, c1)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 4" : "+v"(c0), "+v"(c1));
  };

  // epilogue of tile b from (p0, p1)
  auto finish = [&](int b, const f32x16& p0, const f32x16& p1) {
    const int j = j0 + b / nkb, kb = b - (b / nkb) * nkb;
    if (kb == 0 && a.klen) nk = min(a.klen[j], a.Nk_eff);
    const int key0 = kb * 32 + 4 * h;
    float nn = 0.f, st = 0.f;
    const int nv0 = rs[0].ok ? min(32, nk - kb * 32) : 0;
    const int nv1 = rs[1].ok ? min(32, nk - kb * 32) : 0;
    const long long ct = (long long)j * nkb + kb;
    bf16* d0 = a.dS ? a.dS + ((long long)rt0 * a.CT + ct) * 1024 + lane * 16 : nullptr;
    bf16* d1 = a.dS ? d0 + a.CT * 1024 : nullptr;
    tile_epi(p0, rs[0], nv0, key0, h, temp, lo, nn, st, d0);
    tile_epi(p1, rs[1], nv1, key0, h, temp, lo, nn, st, d1);
    accd += (double)nn;
    accd2 += (double)st;
    if (a.diagS) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const bool dp = a.diag && rs[x].ok && (j == rs[x].qi + a.diag_off);
        if (__any(dp)) {
          if (dp) {
            const f32x16& p = x ? p1 : p0;
            float* drow = a.diagS + ((size_t)rs[x].qi * a.Nq + rs[x].qq) * a.Nk_pad;
#pragma unroll
            for (int v = 0; v < 16; ++v) {
              const int key = key0 + (v & 3) + 8 * (v >> 2);
              if (key < nk) drow[key] = p[v] * temp;
            }
          }
        }
      }
    }
    if (kb == nkb - 1) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        float m = rs[x].m;
        int am = rs[x].am;
        const float m2 = __shfl_xor(m, 32);
        const int am2 = __shfl_xor(am, 32);
        if (m2 > m || (m2 == m && am2 < am)) { m = m2; am = am2; }
        if (h == 0) {
          a.rowmax[(size_t)j * a.R_pad + rs[x].row] = m;
          a.argmax[(size_t)j * a.R_pad + rs[x].row] = am;
        }
        rs[x].m = -INFINITY;
        rs[x].am = 0;
      }
    }
  };

  auto sync_tile = [&](int b) {
    // tile b was issued two iterations ago; only tile b+1's 8 DMAs may still be outstanding
    if (b + 1 < nblocks) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  };
  auto prefetch = [&](int b) {  // tile b + 2 into the slot read by tile b - 1 (all waves are past it)
    const int b2 = b + 2;
    if (b2 < nblocks) stage_tile(a, kbuf + (b2 % NBUF) * KT_ELEMS, j0 + b2 / nkb, b2 % nkb, wave, lane);
  };

  // b = 0: chain only
  sync_tile(0);
  chain(0, cA0, cA1);
  prefetch(0);
  int b = 1;
  for (; b + 1 < nblocks; b += 2) {
    sync_tile(b);
    chain(b, cB0, cB1);
    finish(b - 1, cA0, cA1);
    prefetch(b);
    sync_tile(b + 1);
    chain(b + 1, cA0, cA1);
    finish(b, cB0, cB1);
    prefetch(b + 1);
  }
  if (b < nblocks) {  // odd count: one more chain, then its predecessor's epilogue
    sync_tile(b);
    chain(b, cB0, cB1);
    finish(b - 1, cA0, cA1);
    prefetch(b);
    finish(b, cB0, cB1);
  } else {
    finish(b - 1, cA0, cA1);
  }

  double v = wave_sum_d(accd);
  double v2 = wave_sum_d(accd2);
  __syncthreads();
  if (lane == 0) { red[wave] = v; red[WAVES + wave] = v2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, t2 = 0.0;
    for (int w = 0; w < WAVES; ++w) { t += red[w]; t2 += red[WAVES + w]; }
    a.part[blockIdx.y * gridDim.x + blockIdx.x] = t;
    if (a.part2) a.part2[blockIdx.y * gridDim.x + blockIdx.x] = t2;
  }
}

}  // namespace

// Same grid decomposition as pairsim_kernel (triad_pairsim_nparts), so partial arrays match.
int triad_pairsim_fwd2_launch(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                              int Nk_eff, const float* temp, float clamp_lo, int diag, int diag_off, float* rowmax,
                              int* argmax, double* nn_part, float* diagS, void* dS, long long CT, double* st_part,
                              const int* k_len, int xb, int ys, int jpw, hipStream_t stream) {
  FwdArgs a = {};
  a.Q = (const bf16*)Q; a.K = (const bf16*)K;
  a.R = R; a.R_pad = R_pad; a.Nq = Nq; a.Bq = Bq; a.Bk = Bk; a.Nk_pad = Nk_pad; a.Nk_eff = Nk_eff;
  a.j_per_wg = jpw; a.diag = diag; a.diag_off = diag_off; a.temp = temp; a.clamp_lo = clamp_lo;
  a.rowmax = rowmax; a.argmax = argmax; a.part = nn_part; a.diagS = diagS;
  a.dS = (bf16*)dS; a.CT = CT; a.part2 = st_part; a.klen = k_len;
  hipLaunchKernelGGL(pairsim_fwd2_kernel, dim3(xb, ys), dim3(256), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

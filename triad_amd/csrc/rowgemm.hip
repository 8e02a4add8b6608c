// Projection head (SajayR/TRIAD model.py:32-34,68 / 81-83,116 / 253-255,326: Linear(H->512) ->
// LayerNorm(512) -> Linear(512->512) under bf16 autocast) on ROW-PANEL GEMMs: a workgroup owns 128
// token rows x ALL 512 output columns, so the LayerNorm -- a reduction over those 512 columns --
// and its backward run in the GEMM's epilogue instead of separate passes over HBM:
//   triad_projhead_fwd     the whole forward in one kernel: y1 = bf16(h W1^T + b1); mean / rstd of
//                          y1's rows; ln = bf16(LN(y1)), kept in LDS as the A operand of
//                          y = bf16(ln W2^T + b2) (y1 / ln / mean / rstd also stored for the backward)
//   triad_projhead_ln_fwd  its first half alone (y1, mean / rstd, ln)
//   triad_rowgemm_bias     C = bf16(A W^T + b) (its second half alone, from ln in HBM)
//   triad_projhead_ln_bwd  dln = bf16(dy W2); dy1 = bf16(LN backward(dln)) + the dgamma / dbeta /
//                          db1 column partials of the panel
// (dh = dy1 W1 and the weight gradients stay on the tiled / split-K GEMMs: no row reduction there.)
//
// The GEMM is the similarity head's direct-B structure (bwd_gemm.hip) with a row-major A:
//   * 8 waves, wave w owns output columns [64 w, 64 w + 64): 8 x 4 blocks of 16 x 16 on
//     v_mfma_f32_16x16x32_bf16 (128 fp32 accumulators per lane);
//   * A (the token rows, 128 x 32 bf16 = 8 KB per 32-deep k tile) through a 4-slot LDS ring by
//     16-byte LDS-DMA, one 1 KB piece per wave per tile, chunks XOR-swizzled by row (rp_swz) so the
//     fragment reads are conflict-free;
//   * B (the weight, shared by every workgroup and L2-resident) pre-arranged once per call in
//     MFMA-fragment order and streamed by each wave straight into registers with four ordinary
//     16-byte loads per tile (counted by hipcc; see bwd_gemm.hip for why not inline asm), three
//     tiles ahead;
//   * the MFMA takes the weight fragment as its FIRST operand, so each lane's accumulators hold
//     four CONSECUTIVE columns of one row: the epilogue's row reductions are in-lane plus two
//     lane swaps plus one LDS exchange between the 8 waves, and every store / load of a row
//     segment is 8 bytes.
// Row addressing of A is two-level (row r at A + (r / n_per) * bstride + (r % n_per) * lda), so a
// strided view of the backbone's tokens -- the ViT's patch tokens behind its CLS / register
// tokens -- is read in place, without a packing copy. Rows >= M of the last panel re-read row
// M - 1 (in bounds) and their outputs are written as zeros.
#include <type_traits>

#include "common.h"

namespace {

constexpr int RP_M = 128, RP_N = 512, RP_K = 32;   // panel rows, columns, k tile
constexpr int RP_DD = 3, RP_NB = RP_DD + 1;        // stages in flight ahead, ring slots
constexpr int RP_SLOT = RP_M * RP_K;              // elements per A ring slot (8 KB)
// EPI 2 (LayerNorm backward) brings the panel's 128 y1 rows (128 KB) into LDS by LDS-DMA after the
// k loop, behind the 16 KB the epilogue's row exchange / column vectors use
constexpr int RP_Y1_OFF = 8192;                    // elements
// EPI 3 (the fused forward) keeps the LN'd panel (128 x 512 bf16 = 128 KB) in LDS after the ring
constexpr int RP_PAN_OFF = RP_NB * RP_SLOT;        // elements

struct RPArgs {
  const bf16* A;            // token rows (two-level addressing below)
  long long lda, n_per, bstride;
  long long M;              // valid rows
  int K;                    // contraction (multiple of 32)
  const bf16* Bp;           // packed weight fragments (triad_wpack / triad_bfrag_pack16 dk = 1)
  const bf16* bias;         // [512] bf16 (autocast's F.linear bias; EPI 0: b, EPI 1 / 3: b1)
  const float* gamma;       // LayerNorm weight / bias [512] fp32
  const float* beta;
  float eps;
  bf16* out0;               // y (EPI 0) / y1 (EPI 1) / dy1 (EPI 2): [M_pad][512] bf16, ld 512
  bf16* out1;               // ln (EPI 1)
  float* mean;              // [M_pad] (EPI 1 writes, EPI 2 reads)
  float* rstd;
  const bf16* y1;           // EPI 2: the forward's y1
  float* part;              // EPI 2: [panels][3][512] column partials (dgamma, dbeta, db1)
  const bf16* Bp2;          // EPI 3: packed W2 fragments (triad_wpack(W2, 512))
  const bf16* bias2;        // EPI 3: b2 [512] bf16
  bf16* out2;               // EPI 3: y [M_pad][512] bf16
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// two bf16 in one 32-bit register (the epilogues keep exact-bf16 row values packed: 64 VGPRs per
// 128 x 64 panel slice instead of 128) and their fp32 values
__device__ __forceinline__ unsigned pack_bf2(float a, float b) {
  return (unsigned)__builtin_bit_cast(unsigned short, (bf16)a) |
         ((unsigned)__builtin_bit_cast(unsigned short, (bf16)b) << 16);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __builtin_bit_cast(float, u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __builtin_bit_cast(float, u & 0xffff0000u); }
__device__ __forceinline__ float bf_at(const unsigned (&p)[2], int i) { return i & 1 ? bf_hi(p[i >> 1]) : bf_lo(p[i >> 1]); }
// make packed values opaque between epilogue phases: hipcc would otherwise keep their unpacked fp32
// copies from one phase to the next (128 registers instead of 64)
template <int A, int B>
__device__ __forceinline__ void opaque(unsigned (&p)[A][B][2]) {
#pragma unroll
  for (int x = 0; x < A; ++x)
#pragma unroll
    for (int y = 0; y < B; ++y) asm volatile("" : "+v"(p[x][y][0]), "+v"(p[x][y][1]));
}

template <int U, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (U < N) {
    f(std::integral_constant<int, U>{});
    static_for<U + 1, N>(f);
  }
}

// Weight packing: fragment (k tile kt, wave w, column block cb, lane l) = Bt[32 kt + 8 (l >> 4) + i]
// [64 w + 16 cb + (l & 15)], i = 0..7, at ((kt * 8 + w) * 4 + cb) * 512 + l * 8 -- the B-fragment
// order of bfrag_pack16 (dk = 1). Here Bt[k][n] = W[n][k] for a Linear weight W [512][K]: each
// fragment is 16 contiguous bytes of one weight row.
__global__ __launch_bounds__(256) void wpack_t_kernel(const bf16* __restrict__ W, int K, bf16* __restrict__ Bp) {
  const long long f = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // fragment index
  const long long nfrag = (long long)(K / RP_K) * 8 * 4 * 64;
  if (f >= nfrag) return;
  const int l = (int)(f & 63), cb = (int)((f >> 6) & 3), w = (int)((f >> 8) & 7);
  const long long kt = f >> 11;
  const int n = 64 * w + 16 * cb + (l & 15);
  const long long k = kt * RP_K + 8 * (l >> 4);
  *(bf16x8*)(Bp + f * 8) = *(const bf16x8*)(W + (long long)n * K + k);
}

// A ring slot = [128 rows][32 k] bf16, 64 B per row: 16-byte chunk c of row r sits at chunk
// c ^ rp_swz(r). ds_read_b128 serves a wave in four lane groups of 16 ({0-3, 12-15, 20-27}, ...,
// MI355X_MICROARCH.md LDS table), bank = (byte / 4) mod 64; a fragment read has lane l at row
// 16 rb + (l & 15), chunk l >> 4. Row r & 3 picks the 16-dword bank block, so each group needs its
// four (chunk ^ swz) values distinct: swz = (-(r >> 2)) & 3 does that for all four groups (the plain
// (r >> 2) & 3 left 2-way conflicts in every group: SQ_LDS_BANK_CONFLICT 41-44 % of the LDS cycles,
// profiles/r05_projhead_pmc.txt).
__device__ __forceinline__ int rp_swz(int r) { return (-(r >> 2)) & 3; }

// both weights of a head in one launch (grid.y = 2)
__global__ __launch_bounds__(256) void wpack2_kernel(const bf16* __restrict__ W1, int K1, bf16* __restrict__ Bp1,
                                                     const bf16* __restrict__ W2, int K2, bf16* __restrict__ Bp2) {
  const bf16* W = blockIdx.y ? W2 : W1;
  const int K = blockIdx.y ? K2 : K1;
  bf16* Bp = blockIdx.y ? Bp2 : Bp1;
  const long long f = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (f >= (long long)(K / RP_K) * 2048) return;
  const int l = (int)(f & 63), cb = (int)((f >> 6) & 3), w = (int)((f >> 8) & 7);
  const long long kt = f >> 11;
  const int n = 64 * w + 16 * cb + (l & 15);
  const long long k = kt * RP_K + 8 * (l >> 4);
  *(bf16x8*)(Bp + f * 8) = *(const bf16x8*)(W + (long long)n * K + k);
}

template <int EPI>
__global__ __launch_bounds__(512, 1) void rowpanel_kernel(RPArgs a) {
  // the A ring during the k loop; the epilogue reuses it (row exchange, per-column vectors; EPI 2:
  // + the y1 panel)
  __shared__ __attribute__((aligned(16))) bf16 lds[EPI == 2 ? RP_Y1_OFF + RP_M * RP_N
                                                  : EPI == 3 ? RP_PAN_OFF + RP_M * RP_N : RP_NB * RP_SLOT];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, q = lane >> 4;
  const long long m0 = (long long)blockIdx.x * RP_M;
  const int nkt = a.K / RP_K;

  // this lane's LDS-DMA source row (fixed over the k loop): panel row 16 wave + (lane >> 2),
  // 16-byte chunk (lane & 3) ^ rp_swz(row) of each 64-byte k-tile row
  const int pr = 16 * wave + (lane >> 2);
  const long long srow = m0 + pr < a.M ? m0 + pr : a.M - 1;
  const bf16* asrc = a.A + (srow / a.n_per) * a.bstride + (srow % a.n_per) * a.lda +
                     8 * ((lane & 3) ^ rp_swz(pr));
  // this lane's fragment reads: row 16 rb + l16, chunk q
  const int aoff = l16 * RP_K + 8 * (q ^ rp_swz(l16));   // + rb * 16 * RP_K (rb * 16 keeps rp_swz)
  const bf16* bsrc = a.Bp + (long long)wave * 2048 + lane * 8;

  f32x4 acc[8][4];
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = (f32x4){};

  bf16x8 bq[RP_NB][4];
  auto load_stage = [&](int kt, int slot) __attribute__((always_inline)) {   // kt clamped: a stage past the end re-loads the last tile
    const int k = kt < nkt ? kt : nkt - 1;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) bq[slot][cb] = *(const bf16x8*)(bsrc + (long long)k * 16384 + cb * 512);
    glds16(asrc + k * RP_K, lds + slot * RP_SLOT + wave * 512);
  };
  // TAIL: a trailing stage (nkt % RP_NB): its prefetch's B loads are dead code hipcc removes, so
  // fewer younger VMEM ops are in flight than the counted wait assumes -- drain instead (as the
  // direct-B tile GEMM, bwd_gemm.hip)
  auto stage = [&](auto U, int kt, auto TAIL) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    if constexpr (decltype(TAIL)::value) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else TRIAD_VMCNT(5 * (RP_DD - 1));   // this stage's A piece landed; the DD - 1 younger stages in flight
    __syncthreads();
    const bf16* As = lds + u * RP_SLOT;
    bf16x8 af[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) af[rb] = *(const bf16x8*)(As + rb * 16 * RP_K + aoff);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = mfma16(bq[u][cb], af[rb], acc[rb][cb]);
      if (rb == 1) {
        __builtin_amdgcn_sched_barrier(0);
        load_stage(kt + RP_DD, (u + RP_DD) % RP_NB);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
  static_for<0, RP_DD>([&](auto P) __attribute__((always_inline)) { load_stage(decltype(P)::value, decltype(P)::value); });
  const int ngroups = nkt / RP_NB;
  for (int g = 0; g < ngroups; ++g)
    static_for<0, RP_NB>([&](auto U) __attribute__((always_inline)) {
      stage(U, g * RP_NB + decltype(U)::value, std::false_type{});
    });
  const int rem = nkt - ngroups * RP_NB, base = ngroups * RP_NB;
  static_for<0, RP_NB - 1>([&](auto U) __attribute__((always_inline)) {
    if (decltype(U)::value < rem) stage(U, base + decltype(U)::value, std::true_type{});
  });
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();   // every wave is done with the ring: the epilogue may reuse it
  if constexpr (EPI == 2) {
    // the panel's y1 rows, one 1 KB row per LDS-DMA piece (wave w: rows 16 w ..), 16-byte chunk c
    // of row r at chunk c ^ (r & 15): the epilogue's 8-byte reads (16 rows x one chunk per half
    // wave) are then conflict-free. One wait for all of it, instead of 16 dependent global loads
    // per lane (SQ_WAIT_ANY 0.53 of this kernel's wave time with those, profiles/r05_projhead_pmc.txt)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int r = 16 * wave + i;
      glds16(a.y1 + (m0 + r) * RP_N + 8 * (lane ^ (r & 15)), lds + RP_Y1_OFF + r * RP_N);
    }
  }

  // lane holds, per (rb, cb): row m0 + 16 rb + l16, columns n0 + i, n0 = 64 wave + 16 cb + 4 q
  float* red = (float*)lds;   // row exchange (<= 2304 floats); per-column vectors at + 2304
  // row sums over the 512 columns: in-lane over (cb, i), lanes q = 0..3 (xor 16, 32), then waves
  // v[r] (rows 16 (rb0 + r) + l16 of the panel) summed over the 512 columns and returned to every
  // lane holding the row
  auto row_reduce = [&](auto& v, int rb0) __attribute__((always_inline)) {
    constexpr int R = sizeof(v) / sizeof(float);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      v[r] += __shfl_xor(v[r], 16);
      v[r] += __shfl_xor(v[r], 32);
    }
    if (q == 0)
#pragma unroll
      for (int r = 0; r < R; ++r) red[wave * RP_M + 16 * (rb0 + r) + l16] = v[r];
    __syncthreads();
    if (threadIdx.x < RP_M) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) t += red[w * RP_M + threadIdx.x];
      red[8 * RP_M + threadIdx.x] = t;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = red[8 * RP_M + 16 * (rb0 + r) + l16];
    __syncthreads();   // red is rewritten by the next reduction
  };

  // per-column vectors (bias, gamma, beta) staged in LDS: each (cb) read is one broadcast ds_read_b128
  float* vec = red + 2304;
  const int cw = 64 * wave + 4 * q;   // + 16 cb: this lane's first column of a column block
  auto col4 = [&](int which, int cb) __attribute__((always_inline)) { return *(const f32x4*)(vec + which * RP_N + cw + 16 * cb); };
  if (threadIdx.x < RP_N) {
    const int n = threadIdx.x;
    if (EPI != 2) vec[n] = (float)a.bias[n];
    if (EPI != 0) vec[RP_N + n] = a.gamma[n];
    if (EPI == 1 || EPI == 3) vec[2 * RP_N + n] = a.beta[n];
    if (EPI == 3) vec[3 * RP_N + n] = (float)a.bias2[n];
  }
  __syncthreads();

  if constexpr (EPI == 0) {
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const long long m = m0 + 16 * rb + l16;
      const bool ok = m < a.M;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const f32x4 b = col4(0, cb);
        const uint2 o = ok ? make_uint2(pack_bf2(acc[rb][cb][0] + b[0], acc[rb][cb][1] + b[1]),
                                        pack_bf2(acc[rb][cb][2] + b[2], acc[rb][cb][3] + b[3]))
                           : make_uint2(0u, 0u);
        *(uint2*)(a.out0 + m * RP_N + cw + 16 * cb) = o;
      }
    }
  } else if constexpr (EPI == 1 || EPI == 3) {
    // y1 = bf16(acc + b1) (autocast's F.linear output), stored at once and kept packed (exact bf16
    // values: 64 VGPRs instead of 128); LayerNorm in fp32 over the bf16 y1 row (F.layer_norm under
    // autocast): two-pass mean / biased variance, ln = bf16(xh gamma + beta)
    unsigned y[8][4][2];
    float s[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const long long m = m0 + 16 * rb + l16;
      const bool ok = m < a.M;
      s[rb] = 0.f;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const f32x4 b = col4(0, cb);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          y[rb][cb][j] = pack_bf2(ok ? acc[rb][cb][2 * j] + b[2 * j] : 0.f, ok ? acc[rb][cb][2 * j + 1] + b[2 * j + 1] : 0.f);
#pragma unroll
        for (int i = 0; i < 4; ++i) s[rb] += bf_at(y[rb][cb], i);
        *(uint2*)(a.out0 + m * RP_N + cw + 16 * cb) = make_uint2(y[rb][cb][0], y[rb][cb][1]);
      }
    }
    row_reduce(s, 0);
    opaque(y);
    float v[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      s[rb] *= (1.f / RP_N);   // the row mean
      v[rb] = 0.f;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float d = bf_at(y[rb][cb], i) - s[rb];
          v[rb] += d * d;
        }
    }
    row_reduce(v, 0);
    opaque(y);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const long long m = m0 + 16 * rb + l16;
      const bool ok = m < a.M;
      const float mu = s[rb], rs = rsqrtf(v[rb] * (1.f / RP_N) + a.eps);
      if (wave == 0 && q == 0) {
        a.mean[m] = ok ? mu : 0.f;
        a.rstd[m] = ok ? rs : 0.f;
      }
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const f32x4 gm = col4(1, cb), bt = col4(2, cb);
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = ok ? (bf_at(y[rb][cb], i) - mu) * rs * gm[i] + bt[i] : 0.f;
        const uint2 lnv = make_uint2(pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3]));
        *(uint2*)(a.out1 + m * RP_N + cw + 16 * cb) = lnv;
        if constexpr (EPI == 3) {
          // the LN'd row into the LDS panel, 16-byte chunk c of row r at chunk c ^ (r & 15): the
          // GEMM2 fragment reads (row 16 rb + l16, chunk 4 kt + q) are then conflict-free
          const int c = 8 * wave + 2 * cb + (q >> 1);
          *(uint2*)(lds + RP_PAN_OFF + (16 * rb + l16) * RP_N + 8 * (c ^ l16) + 4 * (q & 1)) = lnv;
        }
      }
    }
    if constexpr (EPI == 3) {
      // projection2 over the panel: A = the LN'd rows from LDS (no HBM read, no ring, no barrier
      // per k tile), B = W2's fragments streamed into registers three tiles ahead as in the k loop
      __syncthreads();
      const bf16* bsrc2 = a.Bp2 + (long long)wave * 2048 + lane * 8;
      const bf16* pan = lds + RP_PAN_OFF + l16 * RP_N;
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = (f32x4){};
      constexpr int NK2 = RP_N / RP_K;
      auto load_b2 = [&](int kt, int slot) __attribute__((always_inline)) {
        const int k = kt < NK2 ? kt : NK2 - 1;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) bq[slot][cb] = *(const bf16x8*)(bsrc2 + (long long)k * 16384 + cb * 512);
      };
      static_for<0, RP_DD>([&](auto P) __attribute__((always_inline)) { load_b2(decltype(P)::value, decltype(P)::value); });
      static_for<0, NK2>([&](auto T) __attribute__((always_inline)) {
        constexpr int kt = decltype(T)::value, u = kt % RP_NB;
        bf16x8 af[8];
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) af[rb] = *(const bf16x8*)(pan + rb * 16 * RP_N + 8 * ((4 * kt + q) ^ l16));
#pragma unroll
        for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = mfma16(bq[u][cb], af[rb], acc[rb][cb]);
          if (rb == 1) {
            __builtin_amdgcn_sched_barrier(0);
            load_b2(kt + RP_DD, (kt + RP_DD) % RP_NB);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      });
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the clamped tail loads
#pragma unroll
      for (int rb = 0; rb < 8; ++rb) {
        const long long m = m0 + 16 * rb + l16;
        const bool ok = m < a.M;
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          const f32x4 b = col4(3, cb);
          const uint2 o = ok ? make_uint2(pack_bf2(acc[rb][cb][0] + b[0], acc[rb][cb][1] + b[1]),
                                          pack_bf2(acc[rb][cb][2] + b[2], acc[rb][cb][3] + b[3]))
                             : make_uint2(0u, 0u);
          *(uint2*)(a.out2 + m * RP_N + cw + 16 * cb) = o;
        }
      }
    }
  } else {
    // dln = bf16(dy W2) (autocast's projection2 input gradient, packed: the accumulators die here);
    // LayerNorm backward in fp32: xh = (y1 - mean) rstd, g = dln gamma,
    // dy1 = bf16(rstd (g - mean(g) - xh mean(g xh))); column partials over the panel's rows:
    // dgamma = sum dln xh, dbeta = sum dln, db1 = sum dy1. y1 / mean / rstd have the panel-padded
    // row count and the forward wrote zeros in the pad rows (xh = 0, rstd = 0 there: dy1 and every
    // partial get nothing from them) -- read unmasked (y1 from the LDS panel loaded after the k
    // loop). The scheduling fences keep hipcc from hoisting every row's reads at once (the live
    // state -- packed dln, row statistics, the 48 column partials -- then fits the register file
    // without spills).
    unsigned dl[8][4][2];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const bool ok = m0 + 16 * rb + l16 < a.M;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          dl[rb][cb][j] = pack_bf2(ok ? acc[rb][cb][2 * j] : 0.f, ok ? acc[rb][cb][2 * j + 1] : 0.f);
    }
    opaque(dl);   // packed here, once: the accumulators die (hipcc would sink each row's packing to its use)
    bf16* op = a.out0 + (m0 + l16) * RP_N + cw;
    // y1[row 16 rb + l16][cw + 16 cb .. + 3] from the LDS panel (swizzle above)
    auto y1_at = [&](int rb, int cb) __attribute__((always_inline)) {
      const int c = 8 * wave + 2 * cb + (q >> 1);
      return *(const uint2*)(lds + RP_Y1_OFF + (16 * rb + l16) * RP_N + 8 * (c ^ l16) + 4 * (q & 1));
    };
    float mu[8], rs[8], s1[8], s2[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      mu[rb] = a.mean[m0 + 16 * rb + l16];
      rs[rb] = a.rstd[m0 + 16 * rb + l16];
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the y1 panel (and mean / rstd) landed
    __syncthreads();
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      s1[rb] = 0.f;
      s2[rb] = 0.f;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const uint2 t = y1_at(rb, cb);
        const unsigned yv[2] = {t.x, t.y};
        const f32x4 gm = col4(1, cb);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float xh = (bf_at(yv, i) - mu[rb]) * rs[rb];
          const float g = bf_at(dl[rb][cb], i) * gm[i];
          s1[rb] += g;
          s2[rb] += g * xh;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    {
      // both row sums in one exchange
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        s1[r] += __shfl_xor(s1[r], 16);
        s1[r] += __shfl_xor(s1[r], 32);
        s2[r] += __shfl_xor(s2[r], 16);
        s2[r] += __shfl_xor(s2[r], 32);
      }
      if (q == 0)
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          red[wave * RP_M + 16 * r + l16] = s1[r];
          red[1024 + wave * RP_M + 16 * r + l16] = s2[r];
        }
      __syncthreads();
      if (threadIdx.x < 2 * RP_M) {
        const int which = threadIdx.x >> 7, row = threadIdx.x & 127;
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 8; ++w) t += red[which * 1024 + w * RP_M + row];
        red[2048 + threadIdx.x] = t;
      }
      __syncthreads();
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        s1[r] = red[2048 + 16 * r + l16];
        s2[r] = red[2048 + RP_M + 16 * r + l16];
      }
    }
    opaque(dl);
    float pg[4][4] = {}, pb[4][4] = {}, p1[4][4] = {};
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const float m1 = s1[rb] * (1.f / RP_N), m2 = s2[rb] * (1.f / RP_N);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        const uint2 t = y1_at(rb, cb);
        const unsigned yv[2] = {t.x, t.y};
        const f32x4 gm = col4(1, cb);
        float o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float dv = bf_at(dl[rb][cb], i);
          const float xh = (bf_at(yv, i) - mu[rb]) * rs[rb];
          o[i] = rs[rb] * (dv * gm[i] - m1 - xh * m2);   // 0 in a pad row (rstd 0)
          pg[cb][i] += dv * xh;
          pb[cb][i] += dv;
        }
        const unsigned ob[2] = {pack_bf2(o[0], o[1]), pack_bf2(o[2], o[3])};
#pragma unroll
        for (int i = 0; i < 4; ++i) p1[cb][i] += bf_at(ob, i);
        *(uint2*)(op + rb * 16 * RP_N + 16 * cb) = make_uint2(ob[0], ob[1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // column partials: sum over the 16 lanes of a lane group (rows), then lane l16 == 0 writes
#pragma unroll
    for (int cb = 0; cb < 4; ++cb)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          pg[cb][i] += __shfl_xor(pg[cb][i], o);
          pb[cb][i] += __shfl_xor(pb[cb][i], o);
          p1[cb][i] += __shfl_xor(p1[cb][i], o);
        }
    if (l16 == 0) {
      float* pp = a.part + (long long)blockIdx.x * 3 * RP_N + cw;
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        *(f32x4*)(pp + 16 * cb) = (f32x4){pg[cb][0], pg[cb][1], pg[cb][2], pg[cb][3]};
        *(f32x4*)(pp + RP_N + 16 * cb) = (f32x4){pb[cb][0], pb[cb][1], pb[cb][2], pb[cb][3]};
        *(f32x4*)(pp + 2 * RP_N + 16 * cb) = (f32x4){p1[cb][0], p1[cb][1], p1[cb][2], p1[cb][3]};
      }
    }
  }
}

int rp_check(const void* A, long long M, int K, long long lda, long long n_per, long long bstride, const void* Bp,
             const void* out0) {
  if (!A || !Bp || !out0 || M <= 0 || K <= 0 || K % RP_K || lda < K || lda % 8 || n_per <= 0 || bstride % 8 ||
      ((uintptr_t)A & 15))
    return TRIAD_EINVAL;
  return TRIAD_OK;
}

}  // namespace

extern "C" {

// Bt fragments of a Linear weight W [512][K] bf16 (Bt[k][n] = W[n][k]) -> Bp, K * 512 bf16.
int triad_wpack(const void* W, int K, void* Bp, hipStream_t stream) {
  if (!W || !Bp || K <= 0 || K % RP_K) return TRIAD_EINVAL;
  const long long nfrag = (long long)(K / RP_K) * 2048;
  hipLaunchKernelGGL(wpack_t_kernel, dim3((unsigned)((nfrag + 255) / 256)), dim3(256), 0, stream, (const bf16*)W, K,
                     (bf16*)Bp);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// triad_wpack of both weights of a head in one launch.
int triad_wpack2(const void* W1, int K1, void* Bp1, const void* W2, int K2, void* Bp2, hipStream_t stream) {
  if (!W1 || !Bp1 || !W2 || !Bp2 || K1 <= 0 || K1 % RP_K || K2 <= 0 || K2 % RP_K) return TRIAD_EINVAL;
  const long long nfrag = (long long)((K1 > K2 ? K1 : K2) / RP_K) * 2048;
  hipLaunchKernelGGL(wpack2_kernel, dim3((unsigned)((nfrag + 255) / 256), 2), dim3(256), 0, stream, (const bf16*)W1, K1,
                     (bf16*)Bp1, (const bf16*)W2, K2, (bf16*)Bp2);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_rowpanel_count(long long M) { return M > 0 ? (int)((M + RP_M - 1) / RP_M) : 0; }

// y1 = bf16(h W1^T + b1), mean / rstd of y1's rows, ln = bf16(LN(y1)) (model.py:32-33 + LN,
// autocast numerics). h rows: h + (r / n_per) * bstride + (r % n_per) * lda, r < M; W1p:
// triad_wpack(W1, H); y1 / ln [panels * 128][512] bf16, mean / rstd [panels * 128] fp32 (rows >= M
// written as zeros).
int triad_projhead_ln_fwd(const void* h, long long M, int H, long long lda, long long n_per, long long bstride,
                          const void* W1p, const void* b1, const float* gamma, const float* beta, float eps, void* y1,
                          void* ln, float* mean, float* rstd, hipStream_t stream) {
  if (rp_check(h, M, H, lda, n_per, bstride, W1p, y1) || !b1 || !gamma || !beta || !ln || !mean || !rstd)
    return TRIAD_EINVAL;
  RPArgs a{(const bf16*)h, lda, n_per, bstride, M, H, (const bf16*)W1p, (const bf16*)b1, gamma, beta, eps,
           (bf16*)y1, (bf16*)ln, mean, rstd, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(rowpanel_kernel<1>, dim3(triad_rowpanel_count(M)), dim3(512), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// The projection head's forward in one kernel (model.py:32-34 / 68, autocast numerics): y1, mean /
// rstd, ln as triad_projhead_ln_fwd, then y = bf16(ln W2^T + b2) from the LN'd panel kept in LDS
// (bit-identical to triad_projhead_ln_fwd + triad_rowgemm_bias). W1p / W2p: triad_wpack(2); b1, b2
// bf16 [512]; y [panels * 128][512] bf16 (rows >= M zero).
int triad_projhead_fwd(const void* h, long long M, int H, long long lda, long long n_per, long long bstride,
                       const void* W1p, const void* b1, const float* gamma, const float* beta, float eps,
                       const void* W2p, const void* b2, void* y1, void* ln, float* mean, float* rstd, void* y,
                       hipStream_t stream) {
  if (rp_check(h, M, H, lda, n_per, bstride, W1p, y1) || !b1 || !gamma || !beta || !ln || !mean || !rstd || !W2p ||
      !b2 || !y)
    return TRIAD_EINVAL;
  RPArgs a{(const bf16*)h, lda, n_per, bstride, M, H, (const bf16*)W1p, (const bf16*)b1, gamma, beta, eps,
           (bf16*)y1, (bf16*)ln, mean, rstd, nullptr, nullptr, (const bf16*)W2p, (const bf16*)b2, (bf16*)y};
  hipLaunchKernelGGL(rowpanel_kernel<3>, dim3(triad_rowpanel_count(M)), dim3(512), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// C = bf16(A Bt + bias), A [M][K] rows at lda, C [panels * 128][512] (ld 512; rows >= M zero);
// Bp: triad_wpack(W, K) for C = A W^T (model.py:34, projection2).
int triad_rowgemm_bias(const void* A, long long M, int K, long long lda, const void* Bp, const void* bias, void* C,
                       hipStream_t stream) {
  if (rp_check(A, M, K, lda, M, 0, Bp, C) || !bias) return TRIAD_EINVAL;
  RPArgs a{(const bf16*)A, lda, M, 0, M, K, (const bf16*)Bp, (const bf16*)bias, nullptr, nullptr, 0.f,
           (bf16*)C, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(rowpanel_kernel<0>, dim3(triad_rowpanel_count(M)), dim3(512), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// Backward through projection2 and the LayerNorm: dln = bf16(dy W2), dy1 = bf16(LN backward) (the
// gradient autocast hands projection1), part [panels][3][512] = per-panel column sums of dln xh
// (dgamma), dln (dbeta), dy1 (db1) -- reduce with triad_sum_slabs. dy [M][512] bf16 (ld 512); W2p:
// triad_bfrag_pack16(W2, 16, 1, .) (Bt = W2 itself); y1 / mean / rstd from triad_projhead_ln_fwd.
int triad_projhead_ln_bwd(const void* dy, long long M, const void* W2p, const void* y1, const float* mean,
                          const float* rstd, const float* gamma, void* dy1, float* part, hipStream_t stream) {
  if (rp_check(dy, M, RP_N, RP_N, M, 0, W2p, dy1) || !y1 || !mean || !rstd || !gamma || !part) return TRIAD_EINVAL;
  RPArgs a{(const bf16*)dy, RP_N, M, 0, M, RP_N, (const bf16*)W2p, nullptr, gamma, nullptr, 0.f,
           (bf16*)dy1, nullptr, const_cast<float*>(mean), const_cast<float*>(rstd), (const bf16*)y1, part,
           nullptr, nullptr, nullptr};
  hipLaunchKernelGGL(rowpanel_kernel<2>, dim3(triad_rowpanel_count(M)), dim3(512), 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

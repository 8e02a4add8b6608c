// bf16 MFMA GEMMs for the backward of the fused similarity head:
//   dQ[r][d] = temp * sum_c dS[r][c] * K[c][d]      (A = dS,   k-contiguous)
//   dK[c][d] = temp * sum_r dS[r][c] * Q[r][d]      (A = dS^T, read transposed from dS)
// i.e. the gradients of S = temp * Q K^T (model.py:387 / 505) w.r.t. both operands.
// B (= K or Q, [k][n] row-major, n-contiguous) is always read with the gfx950
// transposing LDS read ds_read_b64_tr_b16, so neither dS nor the features are
// ever copied into a transposed layout in HBM.
//
// Tile 128x128x64, 4 waves (2x2), each wave 64x64 = 2x2 tiles of
// v_mfma_f32_32x32x16_bf16. Operands are staged global->LDS with 16-byte LDS-DMA
// (global_load_lds_dwordx4) into two buffers; swizzles are applied on the
// global SOURCE address so the lane-linear DMA image is bank-conflict-free for
// the reads (ds_read_b128 for k-contiguous, ds_read_b64_tr_b16 for the others).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int A_ELEMS = BM * BK, B_ELEMS = BK * BN;

// k-contiguous image [m][64 k] (128-B rows): 16-B chunk c of row m lives at chunk c ^ ((m >> 1) & 7)
__device__ __forceinline__ int kc_off(int m, int chunk) { return m * BK + ((chunk ^ ((m >> 1) & 7)) << 3); }
// n-contiguous image [k][128 n] (256-B rows): chunk c of row k lives at chunk c ^ ((k & 3) << 2)
__device__ __forceinline__ int nc_off(int k, int col) {
  return k * BN + ((((col >> 3) ^ ((k & 3) << 2))) << 3) + (col & 7);
}

// piece u (0..3) of this wave's share of an A stage (one 16-byte LDS-DMA wave-instruction)
template <bool A_KCONTIG>
__device__ __forceinline__ void stage_a_piece(const bf16* __restrict__ A, long long lda, int m0, int k0, bf16* dst,
                                              int wave, int lane, int u) {
  const int inst = wave * 4 + u;
  if (A_KCONTIG) {  // 16 wave-instructions of 8 rows x 128 B
    const int m = inst * 8 + (lane >> 3), cp = lane & 7;
    const int c = cp ^ ((m >> 1) & 7);
    glds16(A + (size_t)(m0 + m) * lda + k0 + c * 8, dst + inst * 512);
  } else {  // A stored [k][m]: 16 wave-instructions of 4 k-rows x 256 B
    const int k = inst * 4 + (lane >> 4), cp = lane & 15;
    const int c = cp ^ ((k & 3) << 2);
    glds16(A + (size_t)(k0 + k) * lda + m0 + c * 8, dst + inst * 512);
  }
}

template <bool A_KCONTIG>
__device__ __forceinline__ void stage_a(const bf16* __restrict__ A, long long lda, int m0, int k0, bf16* dst,
                                        int wave, int lane) {
#pragma unroll
  for (int u = 0; u < 4; ++u) stage_a_piece<A_KCONTIG>(A, lda, m0, k0, dst, wave, lane, u);
}

// (Measured and not kept: staging through VGPRs + ds_write instead of LDS-DMA, and the next
// stage's DMA pieces spread between the MFMAs -- DESIGN.md §4b.)

// B is [k][n] (B_KCONTIG=0, n-contiguous) or [n][k] (B_KCONTIG=1) -- the same two
// images as A with the roles of m and n swapped.
template <bool B_KCONTIG>
__device__ __forceinline__ void stage_b(const bf16* __restrict__ B, long long ldb, int n0, int k0, bf16* dst,
                                        int wave, int lane) {
  stage_a<B_KCONTIG>(B, ldb, n0, k0, dst, wave, lane);
}

// Fragment of a [k][n]-image operand for MFMA 32x32x16: lane l needs
// X[k = 16 s + 8 h + j][n = n0 + (l & 31)], j = 0..7, via two 4-row transposed reads.
__device__ __forceinline__ bf16x8 frag_tr(const bf16* img, int n0, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, hh = g >> 1;
  const int col = n0 + 16 * (g & 1) + 4 * p;
  const int k0 = 16 * s + 8 * hh + q;
  const s16x4 lo = lds_tr16(img + nc_off(k0, col));
  const s16x4 hi = lds_tr16(img + nc_off(k0 + 4, col));
  bf16x8 r;
  s16x4* rp = (s16x4*)&r;
  rp[0] = lo;
  rp[1] = hi;
  return r;
}

// F.linear's bias for output column n, added before the one rounding: fp32, or bf16 as the
// autocast model holds it (read as is, no fp32 copy of the vector per call)
__device__ __forceinline__ float bias_at(const void* bias, int bias_bf16, int n) {
  if (!bias) return 0.f;
  return bias_bf16 ? (float)((const bf16*)bias)[n] : ((const float*)bias)[n];
}

// Workgroup -> (output tile, k split). Default: XCD-aware bijective remap of blockIdx.x -- blocks
// sharing an XCD (bid % 8 under round-robin placement) get consecutive tiles, so the column tiles
// of one row panel of A share that XCD's L2; blockIdx.y is the split. xsplit (split-K weight
// gradients, gridDim.y % 8 == 0): every tile of one split on ONE XCD instead, so that split's
// token slab of both operands is fetched from HBM once, into that XCD's L2, and read from there
// by all its tiles (the default mapping puts each split's tiles on all eight XCDs: each operand
// slab is fetched up to 8 times). Placement is a speed matter only; results do not depend on it.
__device__ __forceinline__ void tile_split(int xsplit, int& tile, int& split) {
  const int T = gridDim.x;
  if (xsplit) {
    const int L = blockIdx.y * T + blockIdx.x, c = L % 8, i = L / 8;
    tile = i % T;
    split = c + 8 * (i / T);
    return;
  }
  const int bid = blockIdx.x, q8 = T / 8, r8 = T % 8, x = bid % 8;
  tile = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  split = blockIdx.y;
}

template <bool A_KCONTIG, bool B_KCONTIG, typename OutT>
__global__ __launch_bounds__(256, 2) void gemm_kernel(const bf16* __restrict__ A, long long lda,
                                                      const bf16* __restrict__ B, long long ldb,
                                                      int M, int N, int Kd, const float* __restrict__ alpha_p,
                                                      OutT* __restrict__ C, long long ldc, int k_per_split,
                                                      long long slab_stride, const void* __restrict__ bias, int bias_bf16, int xsplit) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * (A_ELEMS + B_ELEMS)];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5;

  int swz, split;
  tile_split(xsplit, swz, split);
  const int ntn = N / BN;
  const int m0 = (swz / ntn) * BM, n0 = (swz % ntn) * BN;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){};

  // split-K: split owns k in [kbeg, kbeg + k_per_split) and writes its own slab of C
  const int kbeg = split * k_per_split;
  const int nk = min(k_per_split, Kd - kbeg) / BK;
  C += (size_t)split * slab_stride;
  if (nk > 0) {
    stage_a<A_KCONTIG>(A, lda, m0, kbeg, lds, wave, lane);
    stage_b<B_KCONTIG>(B, ldb, n0, kbeg, lds + A_ELEMS, wave, lane);
  }
  for (int kt = 0; kt < nk; ++kt) {
    lds_dma_barrier();
    bf16* const nb = lds + ((kt + 1) & 1) * (A_ELEMS + B_ELEMS);
    const bool pf = kt + 1 < nk;
    if (pf) {
      stage_a<A_KCONTIG>(A, lda, m0, kbeg + (kt + 1) * BK, nb, wave, lane);
      stage_b<B_KCONTIG>(B, ldb, n0, kbeg + (kt + 1) * BK, nb + A_ELEMS, wave, lane);
    }
    const bf16* ai = lds + (kt & 1) * (A_ELEMS + B_ELEMS);
    const bf16* bi = ai + A_ELEMS;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mrow = wm * 64 + t * 32;
        if (A_KCONTIG) {
          af[t] = *(const bf16x8*)(ai + kc_off(mrow + (lane & 31), 2 * s + h));
        } else {
          // A image is [k][m] (256-B rows, same layout as B's)
          af[t] = frag_tr(ai, mrow, s, lane);
        }
        const int ncol = wn * 64 + t * 32;
        if (B_KCONTIG) {
          bfr[t] = *(const bf16x8*)(bi + kc_off(ncol + (lane & 31), 2 * s + h));
        } else {
          bfr[t] = frag_tr(bi, ncol, s, lane);
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
        }
    }
  }

  const float alpha = alpha_p ? *alpha_p : 1.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + (lane & 31);
      const float bn = bias_at(bias, bias_bf16, n);   // F.linear's bias, added before the one rounding
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * 64 + a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        C[(size_t)m * ldc + n] = (OutT)(alpha * acc[a][b][v] + bn);
      }
    }
}

// ---- 256 x 128 ring form ----------------------------------------------------------------------
// Workgroup = 8 waves (4 x 2, each 64 x 64 as above), tile 256 (M) x 128 (N) x 64 (K) per stage,
// a 3-slot LDS ring (3 x 48 KB) with the next-but-one stage's LDS-DMA issued while the current
// one computes; each wave issues exactly 6 pieces per stage, so the wait for stage kt is a
// counted `s_waitcnt vmcnt(6)` (stage kt+1 stays in flight) + the barrier. Twice the B reuse
// of the 128 x 128 form. The A image is [256][64] (k-contiguous A) or two [64][128] halves.
constexpr int GB_M = 256, GB_NB = 3;
constexpr int GB_A = GB_M * BK, GB_ST = GB_A + B_ELEMS;  // elements per stage (48 KB)
constexpr int GB_PIECES = 6;

// the 6 DMA pieces of a stage issued between its 16 MFMAs (one per 2), not in a burst (measured)

template <bool A_KCONTIG, bool B_KCONTIG>
__device__ __forceinline__ void gb_piece(const bf16* __restrict__ A, long long lda, const bf16* __restrict__ B,
                                         long long ldb, int m0, int n0, int k0, bf16* dst, int wave, int lane,
                                         int u) {
  if (u < 4) {  // A: 32 pieces, 4 per wave
    const int inst = wave * 4 + u;
    if (A_KCONTIG) {  // 8 rows x 128 B
      const int m = inst * 8 + (lane >> 3), cp = lane & 7;
      const int c = cp ^ ((m >> 1) & 7);
      glds16(A + (size_t)(m0 + m) * lda + k0 + c * 8, dst + inst * 512);
    } else {  // half inst >> 4, 4 k-rows x 256 B
      const int half = inst >> 4, ii = inst & 15;
      const int k = ii * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ ((k & 3) << 2);
      glds16(A + (size_t)(k0 + k) * lda + m0 + half * 128 + c * 8, dst + half * (BK * 128) + ii * 512);
    }
  } else {  // B: 16 pieces, 2 per wave
    const int inst = wave * 2 + (u - 4);
    bf16* bd = dst + GB_A;
    if (B_KCONTIG) {
      const int n = inst * 8 + (lane >> 3), cp = lane & 7;
      const int c = cp ^ ((n >> 1) & 7);
      glds16(B + (size_t)(n0 + n) * ldb + k0 + c * 8, bd + inst * 512);
    } else {
      const int k = inst * 4 + (lane >> 4), cp = lane & 15;
      const int c = cp ^ ((k & 3) << 2);
      glds16(B + (size_t)(k0 + k) * ldb + n0 + c * 8, bd + inst * 512);
    }
  }
}

template <bool A_KCONTIG, bool B_KCONTIG, typename OutT>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(const bf16* __restrict__ A, long long lda,
                                                          const bf16* __restrict__ B, long long ldb, int M, int N,
                                                          int Kd, const float* __restrict__ alpha_p,
                                                          OutT* __restrict__ C, long long ldc, int k_per_split,
                                                          long long slab_stride, const void* __restrict__ bias, int bias_bf16, int xsplit) {
  __shared__ __attribute__((aligned(16))) bf16 lds[GB_NB * GB_ST];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int h = lane >> 5;
  int swz, split;
  tile_split(xsplit, swz, split);
  const int ntn = N / BN;
  const int m0 = (swz / ntn) * GB_M, n0 = (swz % ntn) * BN;

  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){};

  const int kbeg = split * k_per_split;
  const int nk = __builtin_amdgcn_readfirstlane(max(0, min(k_per_split, Kd - kbeg)) / BK);
  C += (size_t)split * slab_stride;
#pragma unroll
  for (int p = 0; p < GB_NB - 1; ++p)
    if (p < nk)
#pragma unroll
      for (int u = 0; u < GB_PIECES; ++u)
        gb_piece<A_KCONTIG, B_KCONTIG>(A, lda, B, ldb, m0, n0, kbeg + p * BK, lds + p * GB_ST, wave, lane, u);
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) TRIAD_VMCNT(GB_PIECES);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool pf = kt + GB_NB - 1 < nk;
    bf16* const nb = lds + ((kt + GB_NB - 1) % GB_NB) * GB_ST;
    const int kn = kbeg + (kt + GB_NB - 1) * BK;
    const bf16* ai = lds + (kt % GB_NB) * GB_ST;
    const bf16* bi = ai + GB_A;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int mrow = wm * 64 + t * 32;
        if (A_KCONTIG) af[t] = *(const bf16x8*)(ai + kc_off(mrow + (lane & 31), 2 * s + h));
        else af[t] = frag_tr(ai + (mrow >> 7) * (BK * 128), mrow & 127, s, lane);
        const int ncol = wn * 64 + t * 32;
        if (B_KCONTIG) bfr[t] = *(const bf16x8*)(bi + kc_off(ncol + (lane & 31), 2 * s + h));
        else bfr[t] = frag_tr(bi, ncol, s, lane);
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          acc[a][b] = mfma32(af[a], bfr[b], acc[a][b]);
          const int mi = s * 4 + a * 2 + b;
          if ((mi & 1) && mi / 2 < GB_PIECES) {
            __builtin_amdgcn_sched_barrier(0);
            if (pf) gb_piece<A_KCONTIG, B_KCONTIG>(A, lda, B, ldb, m0, n0, kn, nb, wave, lane, mi / 2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    }
  }

  const float alpha = alpha_p ? *alpha_p : 1.f;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + (lane & 31);
      const float bn = bias_at(bias, bias_bf16, n);   // F.linear's bias, added before the one rounding
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * 64 + a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        C[(size_t)m * ldc + n] = (OutT)(alpha * acc[a][b][v] + bn);
      }
    }
}

// ---- 256 x 256 tile: LDS images and staging (the eight-wave form below) -------------------------
// Tile 256 x 256 x 64 per stage, two 64 KB LDS slots, the next stage's DMA pieces issued in the
// first half of the current one, vmcnt(0) + barrier at the top of the next. (Round 1 ran this tile
// on four waves, 128 x 128 each; measured bounds, profiles/r01_gemm_w4_bounds.log: without the
// fragment reads 3 % faster, without the DMA 25 % faster -- the LDS-DMA fill rate (~64 KB per CU per
// stage) holds it under the MFMA rate. The eight-wave form replaced it in round 2, 3-13 % faster;
// the four-wave kernel was deleted in round 5.)
constexpr int GW_M = 256, GW_N = 256;
constexpr int GW_A = GW_M * BK, GW_ST = GW_A + GW_N * BK;  // elements per stage (64 KB)

template <bool KCONTIG>
__device__ __forceinline__ void gw_piece_one(const bf16* __restrict__ X, long long ld, int r0, int k0, bf16* img,
                                             int inst, int lane) {
  if (KCONTIG) {  // image [256][64]: 8 rows x 128 B per wave-instruction
    const int m = inst * 8 + (lane >> 3), cp = lane & 7;
    const int c = cp ^ ((m >> 1) & 7);
    glds16(X + (size_t)(r0 + m) * ld + k0 + c * 8, img + inst * 512);
  } else {  // X stored [k][rows]: two [64][128] halves, 4 k-rows x 256 B per wave-instruction
    const int half = inst >> 4, ii = inst & 15;
    const int k = ii * 4 + (lane >> 4), cp = lane & 15;
    const int c = cp ^ ((k & 3) << 2);
    glds16(X + (size_t)(k0 + k) * ld + r0 + half * 128 + c * 8, img + half * (BK * 128) + ii * 512);
  }
}

template <bool KCONTIG>
__device__ __forceinline__ bf16x8 gw_frag(const bf16* img, int row, int s, int lane) {
  if (KCONTIG) return *(const bf16x8*)(img + kc_off(row + (lane & 31), 2 * s + (lane >> 5)));
  return frag_tr(img + (row >> 7) * (BK * 128), row & 127, s, lane);
}

// ---- 256 x 256 eight-wave form -----------------------------------------------------------------
// The 256 x 256 tile, LDS images and staging with 8 waves (two per SIMD: one wave's DMA
// issue and barrier waits overlap the other's MFMAs): wave (wm, wn) of 2 x 4 owns 128 x 64 (4 x 2
// tiles of 32 x 32, 128 accumulators per lane), reads 6 fragments per 8 MFMAs per 16-deep step, and
// issues 8 of the next stage's 64 DMA pieces (one after every 2nd of its first 16 MFMAs).
constexpr int GE_PIECES = 8;
// Measured and not kept (tools/build_variants.py + variant_ab.py, profiles/r02_gemm_w8_variants_ab.log,
// 16 c3 shapes): s_setprio(1) around each step's MFMA cluster -0.4 %, a static priority for the
// younger four waves 0.0 %, the next stage's 8 DMA pieces in a burst after the barrier +3.9 %;
// transposed accumulators (B fragment first) with 8-byte row-run epilogue stores +10 %
// (profiles/r02_gemm_w8_tepi_ab.log); the bf16 tile staged through LDS and stored as 128-B row runs
// of 16-B stores: equal (profiles/r02_gemm_w8_ldsepi_ab.log). A diagnostic build without the
// epilogue stores ran 10 % faster (18 % on the wide K = 768 shapes, profiles/
// r02_gemm_w8_nostore_diag.log): the cost is the output write itself, ~128 KB per workgroup
// issued by every CU of a dispatch round at once and not overlapped with any MFMA work.

template <bool A_KCONTIG, bool B_KCONTIG>
__device__ __forceinline__ void ge_piece(const bf16* __restrict__ A, long long lda, const bf16* __restrict__ B,
                                         long long ldb, int m0, int n0, int k0, bf16* dst, int wave, int lane,
                                         int u) {
  if (u < 4) gw_piece_one<A_KCONTIG>(A, lda, m0, k0, dst, wave * 4 + u, lane);
  else gw_piece_one<B_KCONTIG>(B, ldb, n0, k0, dst + GW_A, wave * 4 + (u - 4), lane);
}

template <bool A_KCONTIG, bool B_KCONTIG, typename OutT>
__global__ __launch_bounds__(512, 1) void gemm_w8_kernel(const bf16* __restrict__ A, long long lda,
                                                         const bf16* __restrict__ B, long long ldb, int M, int N,
                                                         int Kd, const float* __restrict__ alpha_p,
                                                         OutT* __restrict__ C, long long ldc, int k_per_split,
                                                         long long slab_stride, const void* __restrict__ bias, int bias_bf16, int xsplit) {
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * GW_ST];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int h = lane >> 5;
  int swz, split;
  tile_split(xsplit, swz, split);
  const int ntn = N / GW_N;
  const int m0 = (swz / ntn) * GW_M, n0 = (swz % ntn) * GW_N;

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = (f32x16){};

  const int kbeg = split * k_per_split;
  const int nk = __builtin_amdgcn_readfirstlane(max(0, min(k_per_split, Kd - kbeg)) / BK);
  C += (size_t)split * slab_stride;
  if (nk > 0)
#pragma unroll
    for (int u = 0; u < GE_PIECES; ++u)
      ge_piece<A_KCONTIG, B_KCONTIG>(A, lda, B, ldb, m0, n0, kbeg, lds, wave, lane, u);
  for (int kt = 0; kt < nk; ++kt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool pf = kt + 1 < nk;
    bf16* const nb = lds + ((kt + 1) & 1) * GW_ST;
    const int kn = kbeg + (kt + 1) * BK;
    const bf16* ai = lds + (kt & 1) * GW_ST;
    const bf16* bi = ai + GW_A;
    bf16x8 af[2][4], bfr[2][2];
#pragma unroll
    for (int t = 0; t < 4; ++t) af[0][t] = gw_frag<A_KCONTIG>(ai, wm * 128 + t * 32, 0, lane);
#pragma unroll
    for (int t = 0; t < 2; ++t) bfr[0][t] = gw_frag<B_KCONTIG>(bi, wn * 64 + t * 32, 0, lane);
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      const int cur = s & 1;
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          acc[a][b] = mfma32(af[cur][a], bfr[cur][b], acc[a][b]);
          const int j = a * 2 + b, mi = s * 8 + j;
          if (s + 1 < BK / 16 && j < 6) {  // step s + 1's 6 fragments between step s's MFMAs
            __builtin_amdgcn_sched_barrier(0);
            if (j < 4) af[cur ^ 1][j] = gw_frag<A_KCONTIG>(ai, wm * 128 + j * 32, s + 1, lane);
            else bfr[cur ^ 1][j - 4] = gw_frag<B_KCONTIG>(bi, wn * 64 + (j - 4) * 32, s + 1, lane);
            __builtin_amdgcn_sched_barrier(0);
          }
          if (mi % 2 == 1 && mi / 2 < GE_PIECES) {
            __builtin_amdgcn_sched_barrier(0);
            if (pf) ge_piece<A_KCONTIG, B_KCONTIG>(A, lda, B, ldb, m0, n0, kn, nb, wave, lane, mi / 2);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    }
  }

  const float alpha = alpha_p ? *alpha_p : 1.f;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int n = n0 + wn * 64 + b * 32 + (lane & 31);
      const float bn = bias_at(bias, bias_bf16, n);
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + wm * 128 + a * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        C[(size_t)m * ldc + n] = (OutT)(alpha * acc[a][b][v] + bn);
      }
    }
}

// (Measured and not kept, round 4: the eight-wave tile on v_mfma_f32_16x16x32_bf16 -- bit-identical,
// but 2-30 % slower on every c3 projection-head / backbone shape, profiles/r04_gemm_m16_ab.log; the
// 16 x 16 x 32 shape pays off in the similarity head's direct-B tile GEMMs, not here.)

// The 256 x 256 form the size policy picks for tall outputs: the eight-wave form (4), 3-13 % faster
// than the four-wave form (3) on every c3 backbone / projection-head shape with M >= 50,944
// (profiles/r02_gemm_w8_probe.log). (Measured and not kept: the eight-wave tile on a 4-slot ring of
// 32-deep chunks with the DMA three chunks ahead, 5-8 % slower than this two-slot 64-deep form on
// every M >= 50,944 shape, profiles/r02_gemm_w8_ring_probe.log.) Tile forms are per-call arguments
// (triad_gemm_bf16_form, triad_gemm_bf16_splitk_form): there is no process-wide GEMM state.
constexpr int kBigForm = 4;
// form flag of the split-K entry points: the workgroups of one split all on one XCD (tile_split)
constexpr int kXcdSplit = 8;


template <bool AK, bool BK_, typename OutT>
int launch(const void* A, long long lda, const void* B, long long ldb, int M, int N, int Kd, const float* alpha,
           void* C, long long ldc, hipStream_t st, int splits = 1, long long slab_stride = 0,
           const void* bias = nullptr, int form = 0, int bias_bf16 = 0) {
  const int xsplit = (form & kXcdSplit) ? 1 : 0;
  form &= ~kXcdSplit;
  if (M % BM || N % BN || Kd % BK || lda % 8 || ldb % 8 || splits < 1) return TRIAD_EINVAL;
  if (xsplit && splits % 8) return TRIAD_EINVAL;
  const int kps = ((Kd / BK + splits - 1) / splits) * BK;
  // the 256-row ring pays off on long k loops or many row tiles (conv / projection GEMMs);
  // the short split-K weight-gradient loops keep the 128 x 128 form (measured, profiles/r01_dw_gemm_*.log)
  const bool w4_ok = M % GW_M == 0 && N % GW_N == 0;
  // the four-wave form measured faster on the long conv-stack GEMMs (tools/gemm_forms.py:
  // 2.94 -> 2.67 ms at M = 1.6 M, N = 512, K = 1536); the split-K weight gradients and the
  // shorter forward shapes keep the smaller tiles
  const bool w4_auto = AK && BK_ && splits == 1 && M >= 65536 && Kd >= 1024;
  if (form == 0 && w4_ok && w4_auto) form = kBigForm;
  if (w4_ok && (form == 4 || form == 3)) {   // (form 3, the four-wave 256 x 256 tile, was retired in round 5)
    const int nwg = (M / GW_M) * (N / GW_N);
    hipLaunchKernelGGL((gemm_w8_kernel<AK, BK_, OutT>), dim3(nwg, splits), dim3(512), 0, st, (const bf16*)A, lda,
                       (const bf16*)B, ldb, M, N, Kd, alpha, (OutT*)C, ldc, kps, slab_stride, bias, bias_bf16, xsplit);
    TRIAD_CHECK_LAUNCH();
    return TRIAD_OK;
  }
  if (form != 1 && M % GB_M == 0 &&
      (form == 2 || M >= 8192 || Kd / splits >= 32768)) {
    const int nwg = (M / GB_M) * (N / BN);
    hipLaunchKernelGGL((gemm_big_kernel<AK, BK_, OutT>), dim3(nwg, splits), dim3(512), 0, st, (const bf16*)A, lda,
                       (const bf16*)B, ldb, M, N, Kd, alpha, (OutT*)C, ldc, kps, slab_stride, bias, bias_bf16, xsplit);
    TRIAD_CHECK_LAUNCH();
    return TRIAD_OK;
  }
  const int nwg = (M / BM) * (N / BN);
  hipLaunchKernelGGL((gemm_kernel<AK, BK_, OutT>), dim3(nwg, splits), dim3(256), 0, st, (const bf16*)A, lda,
                     (const bf16*)B, ldb, M, N, Kd, alpha, (OutT*)C, ldc, kps, slab_stride, bias, bias_bf16, xsplit);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // namespace

extern "C" {

// C[M][N] = alpha * op(A) . op(B). a_kcontig=1: A stored [M][Kd] (lda), 0: [Kd][M].
// b_kcontig=1: B stored [N][Kd] (ldb), 0: [Kd][N]. out_bf16 selects a bf16 or fp32 C.
// form: 0 = the size policy of launch(), 1 = 128 x 128, 2 = 256 x 128 ring, 3 = (retired four-wave, runs as 4),
// 4 = 256 x 256 eight-wave (3 / 4 when M, N are multiples of 256; otherwise the policy's fallback).
int triad_gemm_bf16_form(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                         int M, int N, int Kd, const float* alpha, void* C, long long ldc, int out_bf16, int form,
                         hipStream_t stream) {
  if (form < 0 || form > 4) return TRIAD_EINVAL;
#define TRIAD_GEMM_CASE(AK, BKC)                                                                  \
  if (!!a_kcontig == AK && !!b_kcontig == BKC)                                                   \
    return out_bf16 ? launch<AK, BKC, bf16>(A, lda, B, ldb, M, N, Kd, alpha, C, ldc, stream, 1, 0, nullptr, form) \
                    : launch<AK, BKC, float>(A, lda, B, ldb, M, N, Kd, alpha, C, ldc, stream, 1, 0, nullptr, form);
  TRIAD_GEMM_CASE(true, true)
  TRIAD_GEMM_CASE(true, false)
  TRIAD_GEMM_CASE(false, true)
  TRIAD_GEMM_CASE(false, false)
#undef TRIAD_GEMM_CASE
  return TRIAD_EINVAL;
}

int triad_gemm_bf16(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                    int M, int N, int Kd, const float* alpha, void* C, long long ldc, int out_bf16,
                    hipStream_t stream) {
  return triad_gemm_bf16_form(A, lda, a_kcontig, B, ldb, b_kcontig, M, N, Kd, alpha, C, ldc, out_bf16, 0, stream);
}

// The backbone projections (torch's F.linear / matmul under autocast, routed here by
// triad_amd/gemm.py): C = op(A) op(B) (+ bias[n] before the one bf16 rounding), bf16 out. Tile
// form by shape, measured on the c3 shapes (tools/gemm_backend_probe.py,
// profiles/r02_gemm_backend_probe.log, r02_gemm_w8_probe.log): the 256 x 256 eight-wave form when
// the output is tall (M >= 32768, M and N multiples of 256), the 256 x 128 ring for other tall
// outputs, 128 x 128 below 8192 rows. 790-940 TFLOP/s; rocBLAS's own kernels run the same shapes
// at 300-790.
static int gemm_bias_launch(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig, int M,
                     int N, int Kd, const void* bias, int bias_bf16, void* C, long long ldc, hipStream_t stream) {
  // eight-wave 256 x 256 for every tall output it tiles; the 256 x 128 ring only when its tiles
  // fill the 256 CUs once (the 8,192-row text projection head at N = 512 has 128 such tiles, half
  // the chip, and runs on 256 128 x 128 tiles instead)
  int form = 1;
  if (M >= 32768 && M % GW_M == 0 && N % GW_N == 0) form = kBigForm;
  else if (M >= 8192 && M % GB_M == 0 && (long long)(M / GB_M) * (N / BN) >= 256) form = 2;
#define TRIAD_GEMM_B(AK, BKC)                                                                     \
  if (!!a_kcontig == AK && !!b_kcontig == BKC)                                                    \
    return launch<AK, BKC, bf16>(A, lda, B, ldb, M, N, Kd, nullptr, C, ldc, stream, 1, 0, bias, form, bias_bf16);
  TRIAD_GEMM_B(true, true)
  TRIAD_GEMM_B(true, false)
  TRIAD_GEMM_B(false, true)
  TRIAD_GEMM_B(false, false)
#undef TRIAD_GEMM_B
  return TRIAD_EINVAL;
}

int triad_gemm_bf16_bias(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                         int M, int N, int Kd, const float* bias, void* C, long long ldc, hipStream_t stream) {
  return gemm_bias_launch(A, lda, a_kcontig, B, ldb, b_kcontig, M, N, Kd, bias, 0, C, ldc, stream);
}

// The same with the bias as the bf16 vector the autocast model holds (F.linear under autocast
// casts the bias to bf16 and adds it in fp32 before the one rounding): no fp32 copy per call.
int triad_gemm_bf16_bias_bf16(const void* A, long long lda, int a_kcontig, const void* B, long long ldb,
                              int b_kcontig, int M, int N, int Kd, const void* bias, void* C, long long ldc,
                              hipStream_t stream) {
  return gemm_bias_launch(A, lda, a_kcontig, B, ldb, b_kcontig, M, N, Kd, bias, 1, C, ldc, stream);
}

// Split-K form for short-and-wide outputs (weight gradients: M, N = 512 / H, Kd = tokens):
// `splits` partial fp32 slabs in `slabs` ([splits][M][N], caller-owned), then
// C = alpha * sum(slabs) as fp32 or bf16 (ldc == N).
// form: as triad_gemm_bf16_form, + 8 (kXcdSplit) = the workgroups of one split all on one XCD
// (needs splits % 8 == 0).
int triad_gemm_bf16_splitk_form(const void* A, long long lda, int a_kcontig, const void* B, long long ldb,
                                int b_kcontig, int M, int N, int Kd, int splits, const float* alpha, float* slabs,
                                void* C, int out_bf16, int form, hipStream_t stream) {
  if ((form & ~kXcdSplit) < 0 || (form & ~kXcdSplit) > 4) return TRIAD_EINVAL;
  const long long slab = (long long)M * N;
  int rc = TRIAD_EINVAL;
#define TRIAD_GEMM_SK(AK, BKC)                                                                  \
  if (!!a_kcontig == AK && !!b_kcontig == BKC)                                                 \
    rc = launch<AK, BKC, float>(A, lda, B, ldb, M, N, Kd, nullptr, slabs, N, stream, splits, slab, nullptr, form);
  TRIAD_GEMM_SK(true, true)
  TRIAD_GEMM_SK(true, false)
  TRIAD_GEMM_SK(false, true)
  TRIAD_GEMM_SK(false, false)
#undef TRIAD_GEMM_SK
  if (rc) return rc;
  return triad_sum_slabs(slabs, splits, slab, alpha, out_bf16, C, stream);
}

int triad_gemm_bf16_splitk(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                           int M, int N, int Kd, int splits, const float* alpha, float* slabs, void* C,
                           int out_bf16, hipStream_t stream) {
  return triad_gemm_bf16_splitk_form(A, lda, a_kcontig, B, ldb, b_kcontig, M, N, Kd, splits, alpha, slabs, C,
                                     out_bf16, 0, stream);
}

}  // extern "C"

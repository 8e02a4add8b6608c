// Backward GEMMs of the fused similarity head over the TILED dS layout.
//
//   dQ[r][d] = alpha * sum_c dS[r][c] K[c][d]     (gradient of S = temp Q K^T w.r.t. Q)
//   dK[c][d] = alpha * sum_r dS[r][c] Q[r][d]     (w.r.t. K)        model.py:384-387 / 502-505
//
// dS layout (written by pairsim_kernel straight from its MFMA accumulators): 32 x 32
// tiles of 2 KB, tile (rt, ct) at ((rt * CT) + ct) * 1024 elements; inside a tile lane L
// (query q = L & 31, hh = L >> 5) holds 16 bf16 at L*16 + v for keys
// (v & 3) + 8 (v >> 2) + 4 hh -- the v_mfma_f32_32x32x16 accumulator order, its 16-byte chunks
// stored in ds_chunk order (common.h: two 1 KB runs, one per store instruction of the writing
// wave). The loaders below place chunk c of that canonical order at LDS chunk c (swizzled).
//
// dQ reads a tile row-wise: lane L's 8 values v = 8s'..8s'+7 ARE the A fragment of
// k-step s' (keys in the permuted order 16s' + 8(j>>2) + 4hh + (j&3)), so the B operand
// K is read with the same permutation by ds_read_b64_tr_b16 (rows 16s'+4h+q and +8).
// dK reads the same tile transposed with ds_read_b64_tr_b16 (queries on the k axis,
// keys on the lane), no second copy of dS in HBM.
//
// Workgroup: 8 waves, 128 output rows x all 512 columns (A is streamed from HBM exactly
// once); wave w owns columns [64w, 64w+64): 4 x 2 tiles of 32 x 32 accumulators; A and B
// through a 4-slot LDS ring by 16-byte LDS-DMA with source-side swizzles (conflict-free reads).
// Optional split-K over grid.y with fp32 slabs.
#include <type_traits>

#include "common.h"

namespace {

constexpr int TBM = 128, TBN = 512, TBK = 32;

// 16-byte chunk swizzles inside a 2 KB tile (involutions; glds writes lane-linear, the
// source chunk is permuted instead).
__device__ __forceinline__ int swz_q(int c) { return c ^ ((c >> 4) & 1); }          // dQ row reads
__device__ __forceinline__ int swz_k(int c) { return c ^ (((c >> 6) & 1) << 3); }   // dK transposed reads
// dK reads of the 16 x 16 x 32 form (a 32-lane half of a ds_read_b64_tr_b16 spans rows 8g + 0..7 and
// 32 + 8g + 0..7, g = 0, 1): bit 0 also flipped by row bit 3, so the two 16-lane groups of a half land
// on different banks (swz_k leaves them 2-way conflicting)
__device__ __forceinline__ int swz_k16(int c) { return c ^ (((c >> 6) & 1) << 3) ^ ((c >> 4) & 1); }
// B image [32][512], 1 KB rows: chunk c of row k at c ^ ((k & 3) << 2)
__device__ __forceinline__ int b_off(int k, int col) { return k * TBN + ((((col >> 3) ^ ((k & 3) << 2))) << 3) + (col & 7); }

// B fragment (rows = k, columns = n0 + lane&31): two 4-row transposed reads at rows r0, r0 + dr.
__device__ __forceinline__ bf16x8 bfrag(const bf16* img, int r0, int dr, int n0, int lane) {
  const int g = lane >> 4, i = lane & 15, p = i & 3;
  const int col = n0 + 16 * (g & 1) + 4 * p;
  bf16x8 r;
  s16x4* rp = (s16x4*)&r;
  rp[0] = lds_tr16(img + b_off(r0, col));
  rp[1] = lds_tr16(img + b_off(r0 + dr, col));
  return r;
}

// Ring form of the same GEMM: stage = ONE 32-deep k tile (A 4 tiles = 8 KB, B 32 rows x 512 =
// 32 KB), a 4-slot LDS ring (the full 160 KB) with the DMA issued three tiles ahead. Each wave
// issues exactly RING_PIECES LDS-DMA pieces per tile, so the wait for tile `it` is a counted
// `s_waitcnt vmcnt(RING_PIECES * younger)` (tiles it+1, it+2 stay in flight across it) followed by
// the workgroup barrier; the slot refilled after the barrier is the one every wave finished
// reading before it.
constexpr int RING_NB = 4;
constexpr int RING_ST = 4 * 1024 + TBK * TBN;  // 40 KB
constexpr int RING_PIECES = 1 + TBK / 8;       // per wave per tile: 1 A piece + 4 B rows

// one of a wave's RING_PIECES pieces of k tile kt: piece 0 = its A piece, 1..4 = its B rows
template <bool DK>
__device__ __forceinline__ void ring_piece(const bf16* __restrict__ Dt, long long CT, const bf16* __restrict__ B,
                                           int mt0, int kt, bf16* dst, int wave, int lane, int piece) {
  if (piece == 0) {
    const int t = wave >> 1, half = wave & 1;
    const int pos = half * 64 + lane;
    const int c = DK ? swz_k(pos) : swz_q(pos);
    const long long tile = DK ? ((long long)kt * CT + (mt0 + t)) : ((long long)(mt0 + t) * CT + kt);
    glds16(Dt + tile * 1024 + ds_chunk(c) * 8, dst + t * 1024 + half * 512);
  } else {
    const int k = wave * 4 + piece - 1;
    const int c = lane ^ ((k & 3) << 2);
    glds16(B + ((long long)kt * TBK + k) * TBN + c * 8, dst + 4096 + k * TBN);
  }
}

template <bool DK>
__device__ __forceinline__ void stage_ring(const bf16* __restrict__ Dt, long long CT, const bf16* __restrict__ B,
                                           int mt0, int kt, bf16* dst, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < RING_PIECES; ++u) ring_piece<DK>(Dt, CT, B, mt0, kt, dst, wave, lane, u);
}

template <bool DK, bool SLAB>
__global__ __launch_bounds__(512, 1) void tile_gemm_ring_kernel(const bf16* __restrict__ Dt, long long CT,
                                                                const bf16* __restrict__ B, int M, int nkt_total,
                                                                int kt_per_split, const float* __restrict__ alpha_p,
                                                                void* __restrict__ Cout) {
  __shared__ __attribute__((aligned(16))) bf16 lds[RING_NB * RING_ST];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, l32 = lane & 31;
  const int g = lane >> 4, i16 = lane & 15, q4 = i16 >> 2, p4 = i16 & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
  const int swz = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  const int m0 = swz * TBM, mt0 = m0 / 32;
  const int kt0 = blockIdx.y * kt_per_split;
  const int nkt = __builtin_amdgcn_readfirstlane(min(kt_per_split, nkt_total - kt0));

  f32x16 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < 2; ++n) acc[t][n] = (f32x16){};

#pragma unroll
  for (int p = 0; p < RING_NB - 1; ++p)
    if (p < nkt) stage_ring<DK>(Dt, CT, B, mt0, kt0 + p, lds + p * RING_ST, wave, lane);
  for (int it = 0; it < nkt; ++it) {
    const int younger = min(RING_NB - 2, nkt - 1 - it);  // uniform
    if (younger >= 2) TRIAD_VMCNT(2 * RING_PIECES);
    else if (younger == 1) TRIAD_VMCNT(RING_PIECES);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const bool pf = it + RING_NB - 1 < nkt;
    bf16* const pdst = lds + ((it + RING_NB - 1) % RING_NB) * RING_ST;
    const bf16* As = lds + (it % RING_NB) * RING_ST;
    const bf16* Bs = As + 4096;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 af[4], bf[2];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const bf16* tile = As + t * 1024;
        if (!DK) {
          af[t] = *(const bf16x8*)(tile + swz_q(2 * l32 + 64 * h + s) * 8);
        } else {
          const int a = 2 * (g & 1) + (p4 >> 1), hh = p4 & 1;
          s16x4* rp = (s16x4*)&af[t];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            const int qry = 16 * s + 8 * h + 4 * tt + q4;
            const int c = (qry + 32 * hh) * 2 + (a >> 1);
            rp[tt] = lds_tr16(tile + swz_k(c) * 8 + 4 * (a & 1));
          }
        }
      }
#pragma unroll
      for (int n = 0; n < 2; ++n) {
        const int n0 = wave * 64 + n * 32;
        bf[n] = DK ? bfrag(Bs, 16 * s + 8 * h + q4, 4, n0, lane) : bfrag(Bs, 16 * s + 4 * h + q4, 8, n0, lane);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int n = 0; n < 2; ++n) {
          acc[t][n] = mfma32(af[t], bf[n], acc[t][n]);
          const int m = s * 8 + t * 2 + n;
          // the next-but-two tile's DMA pieces between the MFMAs, one per 3 (measured 3-4 %
          // faster than a burst after the barrier)
          if (m % 3 == 0 && m / 3 < RING_PIECES) {
            __builtin_amdgcn_sched_barrier(0);
            if (pf) ring_piece<DK>(Dt, CT, B, mt0, kt0 + it + RING_NB - 1, pdst, wave, lane, m / 3);
            __builtin_amdgcn_sched_barrier(0);
          }
        }
    }
  }

  const float alpha = SLAB ? 1.f : *alpha_p;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const int col = wave * 64 + n * 32 + l32;
#pragma unroll
      for (int v = 0; v < 16; ++v) {
        const int m = m0 + t * 32 + (v & 3) + 8 * (v >> 2) + 4 * h;
        const float val = alpha * acc[t][n][v];
        if (SLAB) ((float*)Cout)[((size_t)blockIdx.y * M + m) * TBN + col] = val;
        else ((bf16*)Cout)[(size_t)m * TBN + col] = (bf16)val;
      }
    }
}

// ---- direct-B form on v_mfma_f32_16x16x32_bf16 (the product backward GEMM) ----------------------
// Wave w only ever multiplies columns [64w, 64w + 64) of B, so B needs no LDS: its fragments are
// pre-arranged once per backward (bfrag_pack16_kernel) and each wave streams its own 4 KB per k
// tile straight into registers with four coalesced 16-byte loads, stages ahead. Only A (dS, 8 KB
// per tile, shared by all eight waves) goes through LDS: one LDS-DMA piece per wave per tile.
// Each wave's 128 x 64 output is 8 x 4 blocks of 16 x 16 computed by v_mfma_f32_16x16x32_bf16 (32
// per 32-deep k tile): the shape the microarchitecture guide measures at ~1.12-1.15x the FLOP/s of
// 32x32x16 at the clock the chip holds under load (MI355X_MICROARCH.md, 'DVFS give-back' item 7).
//   A fragment (row block rb, lane l): query row r = 16 (rb & 1) + (l & 15) of tile rb >> 1, k
//   chunk kc = l >> 4 = 16-byte chunk (hh = kc & 1, j = kc >> 1) of the stored dS row, i.e. keys
//   16 j + 8 (i >> 2) + 4 hh + (i & 3), i = 0..7 -- the forward's accumulator order, read as is;
//   B fragment (column block cb): the same 8 keys of column 64 w + 16 cb + (l & 15), packed once
//   by bfrag_pack16_kernel at ((kt * 8 + w) * 4 + cb) * 512 + l * 8.
// dK (DK = true): A = dS^T, rows = keys, k = queries. Row block rb = 16 keys: tile rb >> 1, key
// half kb = rb & 1; lane l takes keys 16 kb + (l & 15) and the queries 8 (l >> 4) .. + 7 of the
// k tile by two ds_read_b64_tr_b16 (4 query rows each) -- natural query order, so the packed Q
// fragment of lane l is Q[8 (l >> 4) + i][col], i = 0..7.
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

template <bool DK>
__global__ __launch_bounds__(512) void bfrag_pack16_kernel(const bf16* __restrict__ B, bf16* __restrict__ Bp) {
  __shared__ __attribute__((aligned(16))) bf16 img[TBK * TBN];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const long long kt = blockIdx.x;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int k = wave * 4 + r;
    glds16(B + (kt * TBK + k) * TBN + (lane ^ ((k & 3) << 2)) * 8, img + k * TBN);
  }
  lds_dma_barrier();
  const int kc = lane >> 4, hh = kc & 1, j = kc >> 1;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int col = wave * 64 + cb * 16 + (lane & 15);
    bf16x8 f;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      f[i] = img[b_off(DK ? 8 * kc + i : 16 * j + 8 * (i >> 2) + 4 * hh + (i & 3), col)];
    *(bf16x8*)(Bp + ((kt * 8 + wave) * 4 + cb) * 512 + lane * 8) = f;
  }
}

// B fragment load: an ORDINARY 16-byte load that hipcc counts (round 5). Rounds 3-4
// hid it in an inline-asm global_load_dwordx4 with a "=v" output so hipcc would not drain the
// prefetches at the first use; hipcc then took the destination as written at ;;#ASMEND, and a
// build with more register pressure (the TRIAD_LDS_CHECK printf build) spilled ring registers
// right after their loads and reused them while the loads were in flight: the aperture violation
// of gpurun_out/r04d_py5.log (tile_gemm_db_kernel<true,true,2,2>, private_seg_size 120; its
// -save-temps output shows `global_load_dwordx4 v[134:137]` followed by a spill of v[134:137] and
// three more loads into the same range). A counted load is correct under ANY register allocation:
// hipcc waits for it before any copy, spill or reuse. What made hipcc drain the ring before was
// control flow, not the load: a conditional prologue / prefetch and a `break` out of the unrolled
// stage loop let the loop header merge paths with different loads in flight. So: every stage
// issues the same loads (a stage past the end re-loads the last tile, clamped in-bounds, into a
// slot nobody reads again), the main loop runs whole groups of NB stages with no exit inside, and
// the last nst % NB stages follow it in straight-line code. The packed B pointer is not
// __restrict__: with it, hipcc sank each prefetch down to the stage that consumes it (the
// LDS-DMA asm in between no longer ordered it). tests/test_isa_cpu.py checks the emitted waits.
__device__ __forceinline__ bf16x8 bload16(const bf16* p) { return *(const bf16x8*)p; }

// Cache policy of the dS loads (read once per GEMM): TRIAD_DS_LOAD_POL 0 plain, 1 nt (default),
// 2 sc1, 3 sc0 sc1. VERDICT r4 #3 asked to keep the 5.8 GB dS stream from evicting the packed K / Q
// fragments every workgroup re-reads from L2. Measured (tools/gpu_ab_dsload.sh, two alternated
// rounds, profiles/r05_bwd_ds_load_policy_ab.log): nt AV dQ 2.586 -> 2.575 ms, AV dK 2.496 -> 2.480,
// TV dQ 0.404 -> 0.390, TV dK equal; sc1 / sc0 sc1 within noise of plain.
#ifndef TRIAD_DS_LOAD_POL
#define TRIAD_DS_LOAD_POL 1
#endif
#if TRIAD_DS_LOAD_POL == 1
#define TRIAD_DS_LOAD_POLICY " nt"
#elif TRIAD_DS_LOAD_POL == 2
#define TRIAD_DS_LOAD_POLICY " sc1"
#elif TRIAD_DS_LOAD_POL == 3
#define TRIAD_DS_LOAD_POLICY " sc0 sc1"
#else
#define TRIAD_DS_LOAD_POLICY ""
#endif
__device__ __forceinline__ void glds16_ds(const void* gsrc, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(void, lds_base));
  TRIAD_LDS_DMA_CHECK(lds, 0);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off" TRIAD_DS_LOAD_POLICY "\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

// one stage = one 32-deep k tile kt (clamped to kt_last): 4 B loads + 1 A LDS-DMA piece per wave
template <bool DK>
__device__ __forceinline__ void db_stage(const bf16* __restrict__ Dt, long long CT, const bf16* Bp, int mt0, int kt,
                                         int kt_last, bf16* adst, bf16x8 (&bq)[4], int wave, int lane) {
  const int ktk = min(kt, kt_last);
  const bf16* src = Bp + ((long long)ktk * 8 + wave) * 2048 + lane * 8;
#pragma unroll
  for (int u = 0; u < 4; ++u) bq[u] = bload16(src + u * 512);
  const int t = wave >> 1, half = wave & 1;
  const int pos = half * 64 + lane;
  const int c = DK ? swz_k16(pos) : swz_q(pos);
  const long long tile = DK ? ((long long)ktk * CT + (mt0 + t)) : ((long long)(mt0 + t) * CT + ktk);
  glds16_ds(Dt + tile * 1024 + ds_chunk(c) * 8, adst + t * 1024 + half * 512);
}

template <int U, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (U < N) {
    f(std::integral_constant<int, U>{});
    static_for<U + 1, N>(f);
  }
}

#ifndef TRIAD_DB_PF_RB
#define TRIAD_DB_PF_RB 3   // row block after which a stage's prefetch is issued (A/B knob; round 6:
#endif                     // 3 vs 1: -0.6 to -0.8 % on all four c3 GEMMs, profiles/r06_bwd_pf_rb_ab.log)
// DD stages in flight ahead of the one being multiplied (A ring slots = B register ring depth =
// NB = DD + 1); one workgroup barrier per stage. DD = 3 for dQ and dK (dK with two k tiles per
// stage, as its 32x32x16 form had, would spill).
template <bool DK, bool SLAB, int DD>
__global__ __launch_bounds__(512, 1) void tile_gemm_db16_kernel(const bf16* __restrict__ Dt, long long CT,
                                                                 const bf16* Bp, int M, int nkt_total,
                                                                 int kt_per_split, const float* __restrict__ alpha_p,
                                                                 void* __restrict__ Cout) {
  static_assert(DD >= 1 && DD <= 4 && 5 * (DD - 1) <= 63, "stage shape");
  constexpr int NB = DD + 1;
  __shared__ __attribute__((aligned(16))) bf16 lds[NB * 4096];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l16 = lane & 15, kc = lane >> 4, q4 = l16 >> 2, p4 = l16 & 3;
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int q8 = nwg / 8, r8 = nwg % 8, x = bid % 8;
  const int swz = (x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8) + bid / 8;
  const int m0 = swz * TBM, mt0 = m0 / 32;
  const int kt0 = blockIdx.y * kt_per_split;
  const int nst = __builtin_amdgcn_readfirstlane(min(kt_per_split, nkt_total - kt0));   // k tiles = stages
  const int kt_last = kt0 + nst - 1;
  // this lane's A reads inside a 32-row tile, per row half (dQ: one chunk; dK: two transposed
  // 4-row reads) -- offsets in elements
  int aoff[2][2];
#pragma unroll
  for (int rh = 0; rh < 2; ++rh) {
    if (!DK) {
      aoff[rh][0] = swz_q(2 * (16 * rh + l16 + 32 * (kc & 1)) + (kc >> 1)) * 8;
      aoff[rh][1] = 0;
    } else {
      const int a = 2 * rh + (p4 >> 1), hh = p4 & 1;
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int qry = 8 * kc + 4 * tt + q4;
        aoff[rh][tt] = swz_k16((qry + 32 * hh) * 2 + (a >> 1)) * 8 + 4 * (a & 1);
      }
    }
  }

  f32x4 acc[8][4];
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = (f32x4){};

  bf16x8 bq[NB][4];
  // stage st in ring slot u = st % NB: wait for its A piece (the counted vmcnt: the DD - 1 younger
  // stages, 5 ops each, stay in flight; hipcc waits for its B loads itself), barrier, 32 MFMAs with
  // the prefetch of stage st + DD (into slot (u + DD) % NB, read for the last time by stage st - 1,
  // before this barrier) issued after row block TRIAD_DB_PF_RB
  // TAIL: one of the trailing nst % NB stages. Their own prefetches feed no later stage, so hipcc
  // drops those B loads as dead: a tail stage has fewer than 5 (DD - 1) younger VMEM ops in flight
  // and the counted wait would let it pass before its A piece landed (round 5: AV dK with 3 splits of
  // 534 stages gave a different result in 3 of 7 repeats, tools/pair_head_repeat.py; 4 splits of 400
  // -- no tail -- and 1 split were bit-stable). Tail stages drain vmcnt instead (<= 3 per launch).
  auto stage = [&](auto U, int st, auto TAIL) __attribute__((always_inline)) {
    constexpr int u = decltype(U)::value;
    if constexpr (decltype(TAIL)::value) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else TRIAD_VMCNT(5 * (DD - 1));
    __syncthreads();
    const bf16* As = lds + u * 4096;
    bf16x8 af[8];
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const bf16* tile = As + (rb >> 1) * 1024;
      if (!DK) {
        af[rb] = *(const bf16x8*)(tile + aoff[rb & 1][0]);
      } else {
        s16x4* rp = (s16x4*)&af[rb];
        rp[0] = lds_tr16(tile + aoff[rb & 1][0]);
        rp[1] = lds_tr16(tile + aoff[rb & 1][1]);
      }
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[rb][cb] = mfma16(af[rb], bq[u][cb], acc[rb][cb]);
      if (rb == TRIAD_DB_PF_RB) {
        __builtin_amdgcn_sched_barrier(0);
        db_stage<DK>(Dt, CT, Bp, mt0, kt0 + st + DD, kt_last, lds + ((u + DD) % NB) * 4096, bq[(u + DD) % NB],
                     wave, lane);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  if (nst > 0) {   // (an empty split leaves its slab zero)
    static_for<0, DD>([&](auto P) __attribute__((always_inline)) {
      constexpr int p = decltype(P)::value;
      db_stage<DK>(Dt, CT, Bp, mt0, kt0 + p, kt_last, lds + p * 4096, bq[p], wave, lane);
    });
    const int ngroups = nst / NB;
    for (int g = 0; g < ngroups; ++g)
      static_for<0, NB>([&](auto U) __attribute__((always_inline)) {
        stage(U, g * NB + decltype(U)::value, std::false_type{});
      });
    const int rem = nst - ngroups * NB, base = ngroups * NB;
    static_for<0, NB - 1>([&](auto U) __attribute__((always_inline)) {
      if (decltype(U)::value < rem) stage(U, base + decltype(U)::value, std::true_type{});
    });
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the past-the-end stages' LDS-DMA lands before exit
  }

  const float alpha = SLAB ? 1.f : *alpha_p;
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int col = wave * 64 + cb * 16 + l16;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + rb * 16 + kc * 4 + i;
        const float val = alpha * acc[rb][cb][i];
        if (SLAB) ((float*)Cout)[((size_t)blockIdx.y * M + m) * TBN + col] = val;
        else ((bf16*)Cout)[(size_t)m * TBN + col] = (bf16)val;
      }
    }
}

}  // namespace

extern "C" {

// dQ (dk = 0): M = query rows (R_pad), nkt = key tiles (C_pad / 32), B = K [C_pad][512].
// dK (dk = 1): M = key rows (CT * 32), nkt = query tiles (R_pad / 32), B = Q [R_pad][512].
// splits > 1: fp32 slabs [splits][M][512] in `slabs`, then C = alpha * sum (bf16).
int triad_tile_gemm(const void* Dt, long long CT, int dk, const void* B, int M, int nkt, const float* alpha,
                    int splits, float* slabs, void* C, hipStream_t stream) {
  if (M % TBM || nkt <= 0 || splits < 1 || (splits > 1 && !slabs)) return TRIAD_EINVAL;
  const int kps = (nkt + splits - 1) / splits;
  dim3 grid(M / TBM, splits);
  const bf16* d = (const bf16*)Dt;
  const bf16* b = (const bf16*)B;
  if (splits == 1) {
    if (dk) hipLaunchKernelGGL((tile_gemm_ring_kernel<true, false>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, alpha, C);
    else hipLaunchKernelGGL((tile_gemm_ring_kernel<false, false>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, alpha, C);
    TRIAD_CHECK_LAUNCH();
    return TRIAD_OK;
  }
  if (dk) hipLaunchKernelGGL((tile_gemm_ring_kernel<true, true>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, alpha, (void*)slabs);
  else hipLaunchKernelGGL((tile_gemm_ring_kernel<false, true>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, alpha, (void*)slabs);
  TRIAD_CHECK_LAUNCH();
  return triad_sum_slabs(slabs, splits, (long long)M * TBN, alpha, 1, C, stream);
}

// Unscaled fp32 slabs only: slabs[s][M][512] = partial (split s of nkt) of dS K (dk = 0) or
// dS^T Q (dk = 1); the caller reduces (triad_sum_slabs), possibly over several launches' slabs
// (the memory-bounded backward sums the dQ partials of its key-sample chunks this way).
int triad_tile_gemm_slabs(const void* Dt, long long CT, int dk, const void* B, int M, int nkt, int splits,
                          float* slabs, hipStream_t stream) {
  if (M % TBM || nkt <= 0 || splits < 1 || !slabs) return TRIAD_EINVAL;
  const int kps = (nkt + splits - 1) / splits;
  dim3 grid(M / TBM, splits);
  const bf16* d = (const bf16*)Dt;
  const bf16* b = (const bf16*)B;
  if (dk) hipLaunchKernelGGL((tile_gemm_ring_kernel<true, true>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, nullptr, (void*)slabs);
  else hipLaunchKernelGGL((tile_gemm_ring_kernel<false, true>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, nullptr, (void*)slabs);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// v_mfma_f32_16x16x32_bf16 forms: B's fragments in that MFMA's operand order (per dk).
int triad_bfrag_pack16(const void* B, int nkt, int dk, void* Bp, hipStream_t stream) {
  if (nkt <= 0 || !B || !Bp) return TRIAD_EINVAL;
  if (dk) hipLaunchKernelGGL(bfrag_pack16_kernel<true>, dim3(nkt), dim3(512), 0, stream, (const bf16*)B, (bf16*)Bp);
  else hipLaunchKernelGGL(bfrag_pack16_kernel<false>, dim3(nkt), dim3(512), 0, stream, (const bf16*)B, (bf16*)Bp);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

int triad_tile_gemm_packed16(const void* Dt, long long CT, int dk, const void* Bp, int M, int nkt, const float* alpha,
                             int splits, float* slabs, void* C, hipStream_t stream) {
  if (M % TBM || nkt <= 0 || splits < 1 || (splits > 1 && !slabs)) return TRIAD_EINVAL;
  const int kps = (nkt + splits - 1) / splits;
  dim3 grid(M / TBM, splits);
  const bf16* d = (const bf16*)Dt;
  const bf16* b = (const bf16*)Bp;
  void* out = splits > 1 ? (void*)slabs : C;
  const float* al = splits > 1 ? nullptr : alpha;
  if (dk) {
    if (splits == 1) hipLaunchKernelGGL((tile_gemm_db16_kernel<true, false, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, al, out);
    else hipLaunchKernelGGL((tile_gemm_db16_kernel<true, true, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, al, out);
  } else {
    if (splits == 1) hipLaunchKernelGGL((tile_gemm_db16_kernel<false, false, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, al, out);
    else hipLaunchKernelGGL((tile_gemm_db16_kernel<false, true, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, al, out);
  }
  TRIAD_CHECK_LAUNCH();
  if (splits == 1) return TRIAD_OK;
  return triad_sum_slabs(slabs, splits, (long long)M * TBN, alpha, 1, C, stream);
}

// Unscaled fp32 slabs over packed16 B (the memory-bounded backward's chunked dQ partials).
int triad_tile_gemm_packed16_slabs(const void* Dt, long long CT, int dk, const void* Bp, int M, int nkt, int splits,
                                   float* slabs, hipStream_t stream) {
  if (M % TBM || nkt <= 0 || splits < 1 || !slabs) return TRIAD_EINVAL;
  const int kps = (nkt + splits - 1) / splits;
  dim3 grid(M / TBM, splits);
  const bf16* d = (const bf16*)Dt;
  const bf16* b = (const bf16*)Bp;
  if (dk) hipLaunchKernelGGL((tile_gemm_db16_kernel<true, true, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, nullptr, (void*)slabs);
  else hipLaunchKernelGGL((tile_gemm_db16_kernel<false, true, 3>), grid, dim3(512), 0, stream, d, CT, b, M, nkt, kps, nullptr, (void*)slabs);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

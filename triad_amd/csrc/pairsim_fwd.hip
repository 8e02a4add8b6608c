// Forward of the fused similarity head with the epilogue software-pipelined into the MFMA chain.
//
// SajayR/TRIAD model.py:370-392 / 490-514 / 417-418 / 524-525: rowmax / argmax per (key sample, query row), l_nonneg partial sums,
// diagonal S (diag_sim_kernel below), and (training) the unit l_nonneg gradient written in the
// tiled dS layout.
//
// Structure (gfx950): 512-thread workgroup = 8 waves x 32 query rows (two waves per SIMD);
// each wave keeps its rows' bf16 fragments (32 x 512 = 128 VGPRs) for the whole launch.
//  * key tiles (32 keys x 512 x bf16 = 32 KB) stream through a 3-slot LDS ring by 16-byte
//    buffer LDS-DMA issued two tiles ahead; one counted `s_waitcnt vmcnt(N)` + s_barrier per
//    tile (the next tile's DMA stays in flight across it) -- per pair of tiles, 4 slots, in the
//    eval form's 16 x 16 x 32 body;
//  * the epilogue of tile b-1 (scale, max/argmax, clamp^2, unit dS, bf16 pack) is carried by
//    tile b's 32-step MFMA chain, one element per two k-steps, so its VALU issues in the MFMA
//    shadows.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace {

constexpr int D = 512;
constexpr int NS = D / 16;  // 32 k-steps
// Measured choices (DESIGN.md §4 tuning record): 8 waves (two per SIMD, one workgroup per CU),
// a 3-slot key ring (prefetch distance 2), key fragments read 2 k-steps ahead of their MFMA,
// scheduling regions of 2 k-steps, plain (temporal) dS stores, scalar f32 epilogue VALU.
constexpr int WAVES = 8;
constexpr int ROWS_PER_WG = 32 * WAVES;  // 256 query rows per workgroup
constexpr int KT_ELEMS = 32 * D;
#ifndef TRIAD_FWD_PF_AT
#define TRIAD_FWD_PF_AT 9   // k-step after which the next tile's DMA is issued; -1: before the chain
#endif                     // (round 6: 9 vs -1 AV -2.2 %, TV -2.5 %; 1-27 swept, profiles/r06_fwd_pf_at_ab.log)
#ifndef TRIAD_FWD_KPAD
#define TRIAD_FWD_KPAD 1   // training ring: padded unswizzled rows, immediate ds_read offsets (A/B knob;
#endif                   // AV -0.3 %, TV -0.6 %: profiles/r06_fwd_kpad_ab.log)
#ifndef TRIAD_FWD_PINGPONG
#define TRIAD_FWD_PINGPONG 1   // two tiles per loop trip, accumulator sets alternating (A/B knob)
#endif
#ifndef TRIAD_FWD_SYNC_FAST
#define TRIAD_FWD_SYNC_FAST 1   // sync_tile: steady-state wait tested first (A/B knob)
#endif
#ifndef TRIAD_FWD_TREEMAX
#define TRIAD_FWD_TREEMAX 0   // FULL tiles: max3 tree + reverse first-index scan (A/B knob; -8 VALU
#endif                      // per tile, timing equal: profiles/r06_fwd_treemax_ab.log)
#ifndef TRIAD_FWD_PAIRMAX
// training epilogue: max / argmax per pair of elements (5 VALU per pair instead of 6). Measured
// slower: AV training 2.925 / 2.928 ms element by element against 2.952 / 2.953 per pair
// (profiles/r06_fwd_variants_ab.log, alternated on one box); kept as an A/B knob, off
#define TRIAD_FWD_PAIRMAX 0
#endif
#ifndef TRIAD_FWD_NBUF
#define TRIAD_FWD_NBUF 3
#endif
constexpr int NBUF = TRIAD_FWD_NBUF;     // key-tile LDS ring slots (training body)
#ifndef TRIAD_FWD_LDSPF
#define TRIAD_FWD_LDSPF 2
#endif
#ifndef TRIAD_FWD_REGION
#define TRIAD_FWD_REGION 2
#endif
constexpr int LDSPF = TRIAD_FWD_LDSPF;   // key fragments read from LDS ahead of their MFMA
constexpr int REGION = TRIAD_FWD_REGION; // k-steps per scheduling region (sched_barrier spacing)
constexpr int GLDS_PER_TILE = 32 / WAVES;  // 1-KB LDS-DMA pieces per wave per key tile (4)

struct FwdArgs {
  const bf16* Q;
  const bf16* K;
  int R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff, j_per_wg;
  const float* temp;
  float clamp_lo;
  float* rowmax;
  int* argmax;
  double* part;
  bf16* dS;
  long long CT;
  double* part2;
  const int* klen;
  const int* ktiles;  // training: stored key tiles per sample as an exclusive prefix sum (compact K / dS), or null
  int exact;          // training: exact epilogue (fwd_body<true, true>), see exact_epilogue()
};

// Which training epilogue a head runs. The fast form stores d = clamp(u, lo, 0) and redoes
// the whole tile (89 VALU per wave, after the MFMA chain) when any u < lo; the exact form selects
// per element inside the chain (+3 VALU per element). Measured on the c3 shapes
// (profiles/r06_fwd_exact_ab.log, alternated three times, features N(0, 0.58^2)): TV (clamp -20,
// most tiles hold some S < -20) 0.543-0.570 -> 0.493-0.497 ms with the exact form; AV (clamp -60,
// few tiles reach it) 3.04 -> 3.14 ms. So: exact for windows whose lower clamp is at most 30 below 0.
// TRIAD_FWD_EXACT=0 / 1 forces one form for every head (parity tests of both bodies on both windows).
inline int exact_epilogue(float clamp_lo) {
  const char* v = getenv("TRIAD_FWD_EXACT");   // read per launch (host side, negligible)
  if (v && (v[0] == '0' || v[0] == '1') && v[1] == 0) return v[0] - '0';
  return clamp_lo >= -30.f ? 1 : 0;
}

typedef int i32x4 __attribute__((ext_vector_type(4)));

// 16-byte-per-lane buffer LDS-DMA (buffer_load_dwordx4 ... lds), written as inline asm so the
// compiler does not see an LDS write: it would otherwise drain vmcnt(0) -- including the DMA
// of the tile two ahead -- before every ds_read of the ring (it cannot tell the slots apart).
// Completion is counted by sync_tile's s_waitcnt vmcnt(N) + barrier. M0 = LDS destination
// (uniform), written and restored inside the statement.
__device__ __forceinline__ void dma16(i32x4 rsrc, unsigned lds_addr, unsigned voff, unsigned soff) {
  TRIAD_LDS_DMA_CHECK(lds_addr, 1);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_addr), "v"(voff), "s"(rsrc), "s"(soff)
      : "memory");
}

// One key tile (32 rows x 1 KB) into an LDS slot: 1-KB pieces, the row offset in soffset
// (uniform), the source-side swizzle chunk ^ (row & 15) in voffset. Piece u of this wave's
// GLDS_PER_TILE.
__device__ __forceinline__ void stage_piece(i32x4 kr, bf16* dst, int trow, int wave, int lane, int u) {
  const unsigned row0 = (unsigned)(trow + wave * GLDS_PER_TILE);
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) bf16*)dst;
  asm volatile("" : "+v"(lane));  // recompute the lane offsets here, do not keep them live
  const int t = wave * GLDS_PER_TILE + u;
  dma16(kr, __builtin_amdgcn_readfirstlane(lds0 + t * D * 2), (unsigned)((lane ^ (t & 15)) * 16),
        __builtin_amdgcn_readfirstlane((row0 + u) * (D * 2)));
}

// trow: the tile's first key row, relative to the buffer descriptor's base
__device__ __forceinline__ void stage_tile(i32x4 kr, bf16* dst, int trow, int wave, int lane) {
#pragma unroll
  for (int u = 0; u < GLDS_PER_TILE; ++u) stage_piece(kr, dst, trow, wave, lane, u);
}

// Training body's ring (TRIAD_FWD_KPAD): rows unswizzled at a 1040-byte stride (one 16-byte pad
// per row), so the 32 rows' reads of one chunk start 4 banks apart (conflict-free per 8 lanes of
// a 16-byte read) and a k-step's LDS offset is lane part + 32 s -- an immediate on every ds_read
// instead of a per-read address OR (the XOR swizzle's chunk depends on the lane).
constexpr int KROW_PAD_BYTES = D * 2 + 16;
constexpr int KT_SLOT_BYTES = 32 * KROW_PAD_BYTES;
__device__ __forceinline__ void stage_tile_pad(i32x4 kr, bf16* dst, int trow, int wave, int lane) {
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) bf16*)dst;
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int u = 0; u < GLDS_PER_TILE; ++u) {
    const int t = wave * GLDS_PER_TILE + u;
    dma16(kr, __builtin_amdgcn_readfirstlane(lds0 + t * KROW_PAD_BYTES), (unsigned)(lane * 16),
          __builtin_amdgcn_readfirstlane((unsigned)(trow + t) * (D * 2)));
  }
}

// 16-byte store hidden from hipcc's waitcnt bookkeeping (it would otherwise drain vmcnt(0) --
// the in-flight key DMA included -- before reusing the data registers); the trailing
// s_nop 1 covers the store-data read (cdna_hip_programming.md §5.7). Counted in sync_tile.
// Cache policy of the unit-dS stores: plain. Round 5 built sc1 / nt / sc0 sc1 /
// sc1 nt variants: training forward AV 3.04 ms plain vs 4.58-4.62 (sc1, sc0 sc1), 3.16 (nt),
// 5.71 (sc1 nt); TV 0.54 vs 0.76 / 0.55 / 0.94 (profiles/r05_fwd_ds_store_policy_ab.log) --
// letting L2 merge the 2 KB tiles before write-back is worth more than keeping them out of it.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16(void* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off\n\ts_nop 1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ unsigned pack_bf16x2(float lo, float hi) {  // one v_cvt_pk_bf16_f32
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){lo, hi}, bf16x2_t));
}

// The epilogue works on u = sgn(temp) * <q, k> (the sign folded into the query fragments
// once per launch) so that S = su * u with su = |temp| > 0 (su = 1, u = 0 when temp == 0):
// max / argmax of S are those of u (rounding is monotone: rowmax = su * max u exactly), and
// clamp(S, lo, 0) = su * clamp(u, lo / su, 0). Per element that leaves compare + 2 selects
// (max / argmax), one med3, one FMA and (training) half a convert -- no temperature
// multiply, no per-element SGPR-to-VGPR key moves (argmax within a tile is an inline
// constant, merged once per tile).
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct Epi {  // per-lane epilogue state (one 32-row block)
  float m;    // running max of u over the current key sample
  float m0;   // m when the current tile's epilogue started
  int am;     // argmax within the sample, without the 4h lane part (added at the sample's end)
  int at;     // vkey of the tile's best element (valid when m > m0)
  int lim;    // masked tiles: valid keys of the tile minus 4h
  f32x2 nn2;  // sum of c^2 over the tile, c = clamp(u, lo/su, 0) (pairs of elements)
  float mn;   // min u over the tile: any u < lo/su sends the tile through epi_fixup
  float prev;  // previous element's c (pairs into one packed op)
  unsigned pk[8];
  float prevd;  // EXACT: previous element's d
  f32x2 st2;    // EXACT: sum of d^2 over the tile (pairs of elements)
};

// key offset of accumulator element v inside a 32-key tile, without the 4h lane part
__device__ __forceinline__ constexpr int vkey(int v) { return (v & 3) + 8 * (v >> 2); }

// One element of a tile's epilogue. FULL: every key of the tile is valid (no mask; padded
// query rows are zero vectors, u = 0, and add nothing). The stored unit l_nonneg gradient is
// d = clamp(S, lo, 0) [S >= lo] / su -- in the window that is c itself, so no per-element
// multiply (su enters the backward once: the tile GEMMs' alpha and the dS patch terms; round 6,
// -1.5 % AV / -1.2 % TV training forward, profiles/r06_fwd_nosu_ab.log). Fast form: d = c,
// exact unless some u < lo/su (then c = lo/su but d = 0) -- the tile minimum tracked here
// detects that and epi_fixup redoes d for such (rare) tiles.
// Plain VALU ops as asm: the compiler canonicalises NaNs around fminf/fmaxf/med3-with-inf
// (extra v_max x, x per operand) and splits the packed f32 ops into scalar ones.
__device__ __forceinline__ float min3f(float a, float b, float c) {
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float maxf(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
// scalar forms: beside MFMAs a packed f32 op costs ~22 issue cycles more than two scalar ones
// (MI355X_MICROARCH.md, 'price of one filler beside MFMAs')
__device__ __forceinline__ float fma_sq(float c, float acc) {  // acc + c * c
  asm("v_fmac_f32 %0, %1, %1" : "+v"(acc) : "v"(c));
  return acc;
}
// u >= lo ? c : 0 -- plain C so hipcc's hazard recognizer sees the VALU-written lane mask the
// select reads (v_cmp + v_cndmask)
__device__ __forceinline__ float selge(float u, float lo, float c) { return u >= lo ? c : 0.f; }

// Empty volatile asm that "modifies" v: the value is computed before this point and stays in
// place (keeps the epilogue interleaved with the MFMA chain instead of sunk past it).
#define PIN(v) asm volatile("" : "+v"(v))

template <bool TRAIN, bool FULL, bool EXACT>
__device__ __forceinline__ void epi_elem(Epi& e, const f32x16& p, int v, float lo) {
  const float u = p[v];
  if constexpr (FULL) {
    // per PAIR of elements (keys ascend with v): the pair's max against the running max in one
    // v_max3, the pair's argmax (u1 > u0 strict, so a tie keeps the first key) taken only if the
    // running max rose (strict, so an earlier key keeps ties) -- 5 VALU per pair instead of 6,
    // the same max / argmax as element by element
#if TRIAD_FWD_TREEMAX
    // the tile's max (with the running max folded in) by a v_max3 tree at the first element, then
    // the first key holding it by a reverse scan, one compare + select per element: 40 VALU per
    // tile instead of 48. e.at is read only when the tile raised the running max (epi_end), and
    // then the first key equal to the new max is the one the element-by-element strict walk keeps.
    if (v == 0) {
      const float t0 = max3f(p[0], p[1], p[2]), t1 = max3f(p[3], p[4], p[5]), t2 = max3f(p[6], p[7], p[8]);
      const float t3 = max3f(p[9], p[10], p[11]), t4 = max3f(p[12], p[13], p[14]);
      const float t5 = max3f(t0, t1, t2), t6 = max3f(t3, t4, p[15]);
      e.m = max3f(t5, t6, e.m);
    }
    e.at = p[15 - v] == e.m ? vkey(15 - v) : e.at;
#elif TRIAD_FWD_PAIRMAX
    if (v & 1) {
      const float u0 = p[v - 1];
      const float mn = max3f(e.m, u0, u);
      const int kp = u > u0 ? vkey(v) : vkey(v - 1);
      e.at = mn > e.m ? kp : e.at;
      e.m = mn;
    }
#else
    e.at = u > e.m ? vkey(v) : e.at;
    e.m = maxf(u, e.m);
#endif
  } else {
    PIN(e.lim);  // keep the 16 masks from being hoisted
    const bool better = vkey(v) < e.lim && u > e.m;
    e.m = better ? u : e.m;
    e.at = better ? vkey(v) : e.at;
  }
  // padded keys are zero vectors (u = 0): they add nothing below without a mask
  const float c = __builtin_amdgcn_fmed3f(u, lo, 0.f);
  // EXACT: the unit gradient per element, d = c inside the window [lo, 0] and 0 below it (the
  // clamp's gradient), and the window's sum of d^2 beside the sum of c^2 -- no per-tile slow form
  float dd = 0.f;
  if constexpr (TRAIN && EXACT) {
    dd = selge(u, lo, c);
    if (v & 1) {
      e.st2.x = fma_sq(e.prevd, e.st2.x);
      e.st2.y = fma_sq(dd, e.st2.y);
      PIN(e.st2);
    }
  }
  if (v & 1) {
    const f32x2 cc = {e.prev, c};
    e.nn2.x = fma_sq(cc.x, e.nn2.x);
    e.nn2.y = fma_sq(cc.y, e.nn2.y);
    PIN(e.nn2);
    if constexpr (TRAIN) {
      f32x2 d = cc;
      if constexpr (EXACT) {
        d = (f32x2){e.prevd, dd};
      } else {
        e.mn = min3f(e.mn, p[v - 1], u);
        PIN(e.mn);
      }
      e.pk[v >> 1] = pack_bf16x2(d.x, d.y);
      PIN(e.pk[v >> 1]);
    }
  } else {
    e.prev = c;
    PIN(e.prev);
    if constexpr (TRAIN && EXACT) {
      e.prevd = dd;
      PIN(e.prevd);
    }
  }
  PIN(e.m);
  PIN(e.at);
}

// Slow form for a tile with some u < lo/su: d = u on [lo/su, 0], else 0; returns the tile's
// sum of d^2 (the fast form's sum of c^2 over-counts the clamped elements).
__device__ __forceinline__ float epi_fixup(Epi& e, const f32x16& p, float lo) {
  float st = 0.f, dp = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const float u = p[v];
    const float d = (u >= lo && u <= 0.f) ? u : 0.f;
    st = fmaf(d, d, st);
    if (v & 1) e.pk[v >> 1] = pack_bf16x2(dp, d);
    else dp = d;
  }
  return st;
}

// A wave-uniform int read through the scalar cache (s_load: lgkmcnt): a per-tile read of the key
// lengths (retrieval) as a vector load made hipcc drain vmcnt(0) right after it in the tile loop --
// the prefetched key tiles and the dS stores included. The lengths are written before the launch.
__device__ __forceinline__ int load_uniform(const int* p, int i) {
  return *((const __attribute__((address_space(4))) int*)p + i);
}

struct Cursor {  // wave-uniform position (sample j, key block kb) of a tile in the walk
  int j, kb;
  int t = 0;  // tiles walked so far (fwd_body: the tile's index among the workgroup's stored tiles)
  __device__ __forceinline__ void next(int nkb) {  // readfirstlane: provably uniform (SGPRs)
    const int k1 = kb + 1 == nkb ? 0 : kb + 1;
    j = __builtin_amdgcn_readfirstlane(k1 == 0 ? j + 1 : j);
    kb = __builtin_amdgcn_readfirstlane(k1);
  }
  // the same walk over samples of tiles(j) = nkb - skip bit (j - j0) tiles each
  __device__ __forceinline__ void next(int nkb, unsigned long long skip, int j0) {
    const int k1 = kb + 1 == tiles(nkb, skip, j0) ? 0 : kb + 1;
    j = __builtin_amdgcn_readfirstlane(k1 == 0 ? j + 1 : j);
    kb = __builtin_amdgcn_readfirstlane(k1);
    t = __builtin_amdgcn_readfirstlane(t + 1);
  }
  __device__ __forceinline__ int tiles(int nkb, unsigned long long skip, int j0) const {
    const int d = j - j0;
    return nkb - (d < 64 ? (int)((skip >> d) & 1ull) : 0);
  }
};

// SHORTQ tags the launches over short query lists (text captions, Nq <= 32) with their own
// symbol, so profiler summaries report the AV (long-query) launches' durations on their own; the
// code is identical.
// The 16 x 16 x 32 body (eval form) meets at the ring barrier once per TWO key tiles: 4 slots,
// pairs of tiles DMA'd together two tiles ahead (round 5, TRIAD_FWD_SYNC2 A/B, alternated x3 on
// one box, profiles/r05_fwd_sync2_ab.log: eval AV 2.36 -> 2.30-2.32 ms, TV 0.408 -> 0.392-0.399;
// the same pairing in the training body was 3 % slower, AV 3.00 -> 3.10, and the training form on
// this paired 16 x 16 x 32 body 4 % slower, AV 3.15 -> 3.27-3.30, profiles/r05_fwd_train16_ab.log).
constexpr int NBUF16 = 4;
template <bool TRAIN>
constexpr int kbuf_elems = (TRAIN ? NBUF * (TRIAD_FWD_KPAD ? KT_SLOT_BYTES / 2 : KT_ELEMS) : NBUF16 * KT_ELEMS) + 16 * WAVES;
constexpr int KSLOT_ELEMS = TRIAD_FWD_KPAD ? KT_SLOT_BYTES / 2 : KT_ELEMS;   // training ring slot

// One workgroup of the forward: 256-row block bx, key-sample split by (of gx row blocks) of
// problem a. kbuf = the workgroup's LDS (key ring + reduction scratch). EXACT (training): the
// unit gradient exact per element inside the MFMA chain instead of the fast form plus a slow
// per-tile redo when some u < lo (FwdArgs::exact, chosen per head by the host).
template <bool TRAIN, bool EXACT = false>
__device__ __forceinline__ void fwd_body(const FwdArgs& a, bf16* kbuf, const int bx, const int by, const int gx) {
  double* red = (double*)(kbuf + NBUF * KSLOT_ELEMS);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int h = lane >> 5, ql = lane & 31;
  const int row = bx * ROWS_PER_WG + wave * 32 + ql;
  const bool rok = row < a.R;
  const int rt = (bx * ROWS_PER_WG + wave * 32) / 32;

  const int j0 = by * a.j_per_wg;
  const int j1 = min(a.Bk, j0 + a.j_per_wg);
  const int nkb = a.Nk_pad / 32;
  // Compact key tiles (training, ktiles given): a key sample whose kept keys all lie before its
  // last 32-key tile holds only zero vectors there (patch dropout's padding), so S == 0 exactly on
  // that tile; the caller's K and the tiled dS then store only the other tiles -- sample j's at
  // tile rows ktiles[j] .. ktiles[j+1] - 1 -- and the tile is not multiplied: its epilogue is
  // applied in closed form at the sample's end (the max against 0 at the tile's first key, nothing
  // added to the sums). Bit j - j0 of `skip` (nkb - 1 stored tiles), for the workgroup's first
  // 64 samples; the host stores every tile of any later one.
  unsigned long long skip = 0;
  int tile0 = j0 * nkb, ntile_wg = (j1 - j0) * nkb;   // the workgroup's first stored tile, count
  if (TRAIN && a.ktiles && j1 > j0) {
    const int jj = j0 + lane;
    skip = __builtin_amdgcn_ballot_w64(jj < j1 && a.ktiles[jj + 1] - a.ktiles[jj] < nkb);
    tile0 = __builtin_amdgcn_readfirstlane(a.ktiles[j0]);
    ntile_wg = __builtin_amdgcn_readfirstlane(a.ktiles[j1]) - tile0;
  }
  const int nblocks = ntile_wg;
  if (nblocks <= 0) {
    if (threadIdx.x == 0) {
      a.part[by * gx + bx] = 0.0;
      if (a.part2) a.part2[by * gx + bx] = 0.0;
    }
    return;
  }

  // K through a buffer descriptor based at this workgroup's first key sample j0: 32-bit
  // offsets cover its j_per_wg samples (the host checks j_per_wg * Nk_pad * 1 KB < 2 GB), so the
  // whole key set may exceed 4 GB (global negatives). Descriptor words: base, stride 0,
  // num_records, gfx950 raw-buffer flags.
  const unsigned long long kaddr = (unsigned long long)(a.K + (size_t)tile0 * 32 * D);
  const i32x4 kr = {__builtin_amdgcn_readfirstlane((int)(unsigned)kaddr),
                    __builtin_amdgcn_readfirstlane((int)((unsigned)(kaddr >> 32) & 0xffffu)),
                    __builtin_amdgcn_readfirstlane((int)((unsigned)ntile_wg * 32 * (D * 2))), 0x00020000};
  // walk cursors: prefetch (tile b+2), chain (tile b), epilogue (tile b-1); ring slots
  Cursor fc{j0, 0}, cc{j0, 0}, ec{j0, 0};
  int fslot = 0, cslot = 0;
  auto prefetch = [&](int b2) __attribute__((always_inline)) {
#if TRIAD_FWD_KPAD
    if (b2 < nblocks) stage_tile_pad(kr, kbuf + fslot * KSLOT_ELEMS, b2 * 32, wave, lane);   // stored tiles in walk order
#else
    if (b2 < nblocks) stage_tile(kr, kbuf + fslot * KT_ELEMS, b2 * 32, wave, lane);   // stored tiles in walk order
#endif
    fc.next(nkb, skip, j0);
    fslot = __builtin_amdgcn_readfirstlane(fslot == NBUF - 1 ? 0 : fslot + 1);
  };
  // prologue: NBUF - 1 tiles in flight
#pragma unroll
  for (int i = 0; i < NBUF - 1; ++i) prefetch(i);

  bf16x8 qf[NS];
  {
    const bf16* q0 = a.Q + (size_t)row * D + 8 * h;  // rows < R_pad: zero tail, in the allocation
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *(const bf16x8*)(q0 + 16 * s);
  }
  // uniform (SGPR) temperature: the load completes here, not at a wait inside the loop
  const float temp = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, *a.temp)));
  // u = sgn(temp) <q, k>: fold the sign into the query fragments (exact bf16 sign flips; zeros
  // for temp == 0, where S == 0 everywhere and su = 1)
  const float su = temp != 0.f ? fabsf(temp) : 1.f;
  if (!(temp > 0.f)) {
    const unsigned flip = temp < 0.f ? 0x80008000u : 0u, keep = temp == 0.f ? 0u : 0xffffffffu;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      u32x4 w = __builtin_bit_cast(u32x4, qf[s]);
      w = (w & keep) ^ flip;
      qf[s] = __builtin_bit_cast(bf16x8, w);
    }
  }
  const float lo = a.clamp_lo / su;  // clamp window of u
  double accd = 0.0, accd2 = 0.0;
  // lane part of the LDS fragment offsets (bytes), k-step s reads chunk 2s+h of row ql
#if TRIAD_FWD_KPAD
  const int xo0 = ql * KROW_PAD_BYTES + h * 16;
  auto koff = [&](int s) __attribute__((always_inline)) { return xo0 + 32 * s; };
#else
  int xo[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) xo[k] = ql * (D * 2) + (((2 * k + h) ^ (ql & 15)) * 16);
  auto koff = [&](int s) __attribute__((always_inline)) { return xo[s & 7] + (s >> 3) * 256; };
#endif
  // this wave's dS row block (TRAIN): tile (rt, ct) at (rt*CT + ct)*1024 elements
  bf16* const dS_w = TRAIN ? a.dS + (long long)rt * a.CT * 1024 : nullptr;

  Epi e;
  e.m = -INFINITY;
  e.am = 0;
  e.at = 0;

  f32x16 cA, cB;

  auto sync_tile = [&](int b) __attribute__((always_inline)) {
    // VMEM ops younger than tile b's DMA, at least: tile b+1's 4 pieces (if any) and, in
    // training, one epilogue's 2 dS stores (b >= 2); vmcnt counts both, in issue order
    // (3-slot ring; a 2-slot ring has no younger tile in flight)
    // (general ring: the DMAs of tiles b+1 .. b+NBUF-2 below nblocks and the stores of the
    // epilogues of tiles b-NBUF+1 .. b-2; the oldest younger epilogue's stores are waited for)
    // (only the cases the ring can reach are compiled, so each counted wait in the ISA decodes to
    // one (nd, ns): tests/test_isa_cpu.py checks every one against the VMEM ops hipcc emitted)
    const int nd = min(NBUF - 2, nblocks - 1 - b);
    const int ns = TRAIN ? max(0, min(NBUF - 2, b - 1)) : 0;
#if TRIAD_FWD_SYNC_FAST
    // the steady state (nd = ns = 1: every tile but the first two and the last) tested first, so
    // the per-tile path to the barrier is one compare and branch instead of the switch's tree
    if (NBUF == 3 && TRAIN && __builtin_expect(b >= 2 && b <= nblocks - 2, 1)) {
      TRIAD_VMCNT(GLDS_PER_TILE + 2);
    } else
#endif
    if constexpr (NBUF == 3) {
      switch (nd * 2 + ns * 16) {
        case 2: TRIAD_VMCNT(GLDS_PER_TILE); break;
        case 16: TRIAD_VMCNT(2); break;
        case 18: TRIAD_VMCNT(GLDS_PER_TILE + 2); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    } else {
      static_assert(NBUF == 4, "sync_tile's counted waits cover 3- and 4-slot rings");
      switch (nd * 2 + ns * 16) {
        case 2: TRIAD_VMCNT(GLDS_PER_TILE); break;
        case 4: TRIAD_VMCNT(2 * GLDS_PER_TILE); break;
        case 16: TRIAD_VMCNT(2); break;
        case 18: TRIAD_VMCNT(GLDS_PER_TILE + 2); break;
        case 20: TRIAD_VMCNT(2 * GLDS_PER_TILE + 2); break;
        case 32: TRIAD_VMCNT(4); break;
        case 34: TRIAD_VMCNT(GLDS_PER_TILE + 4); break;
        case 36: TRIAD_VMCNT(2 * GLDS_PER_TILE + 4); break;
        default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      }
    }
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };

  auto epi_end = [&](const f32x16& p) __attribute__((always_inline)) {
    if (e.m > e.m0) e.am = ec.kb * 32 + e.at;  // the tile raised the running max
    const float nn = e.nn2.x + e.nn2.y;
    accd += (double)nn;
    if (TRAIN) {
      float st;
      if constexpr (EXACT) st = e.st2.x + e.st2.y;
      // some u below the window in this wave's tile: redo d (wave-uniform branch)
      else st = __builtin_amdgcn_ballot_w64(e.mn < lo) ? epi_fixup(e, p, lo) : nn;
      accd2 += (double)st;
      // canonical chunks 2 lane, 2 lane + 1 at ds_chunk(): two 1 KB contiguous stores per wave
      bf16* d = dS_w + ((long long)tile0 + ec.t) * 1024 + lane * 8;
      store16(d, (u32x4){e.pk[0], e.pk[1], e.pk[2], e.pk[3]});
      store16(d + 512, (u32x4){e.pk[4], e.pk[5], e.pk[6], e.pk[7]});
    }
    const int etiles = ec.tiles(nkb, skip, j0);
    if (ec.kb == etiles - 1) {  // end of a key sample: combine the half-waves' max / argmax
      if (etiles < nkb && 0.f > e.m) {  // its zero last tile (see `skip`): u = 0 from key 32 (nkb - 1) on
        e.m = 0.f;
        e.am = 32 * (nkb - 1) - 4 * h;
      }
      float m = e.m;
      int am = e.am + 4 * h;
      const float m2 = __shfl_xor(m, 32);
      const int am2 = __shfl_xor(am, 32);
      if (m2 > m || (m2 == m && am2 < am)) { m = m2; am = am2; }
      if (h == 0 && rok) {
        a.rowmax[(size_t)ec.j * a.R_pad + row] = su * m;  // max S = su * max u (monotone rounding)
        a.argmax[(size_t)ec.j * a.R_pad + row] = am;
      }
      e.m = -INFINITY;
      e.am = 0;
    }
    ec.next(nkb, skip, j0);
  };

  // one tile iteration: chain of tile b into c (CH) with the epilogue of tile b-1 from p (EP,
  // FULL or masked), one element per two k-steps
  auto iter = [&](auto CH, auto EP, auto FULLT, int b, f32x16& c, const f32x16& p) __attribute__((always_inline)) {
    constexpr bool ch = decltype(CH)::value, ep = decltype(EP)::value, full = decltype(FULLT)::value;
    if constexpr (ch) {
      sync_tile(b);
      if (TRIAD_FWD_PF_AT < 0) prefetch(b + NBUF - 1);
      const char* kt = (const char*)kbuf + cslot * (KSLOT_ELEMS * 2);
      cslot = __builtin_amdgcn_readfirstlane(cslot == NBUF - 1 ? 0 : cslot + 1);
      constexpr int P = LDSPF;
      bf16x8 af[P + 1];
#pragma unroll
      for (int s = 0; s < P; ++s) af[s] = *(const bf16x8*)(kt + koff(s));
      c = (f32x16){};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        if (s + P < NS) af[(s + P) % (P + 1)] = *(const bf16x8*)(kt + koff(s + P));
        c = mfma32(af[s % (P + 1)], qf[s], c);
        if constexpr (ep) {
          if (s & 1) epi_elem<TRAIN, full, EXACT>(e, p, s >> 1, lo);
        }
        // scheduling regions of 4 k-steps: two epilogue elements interleave and fill each
        // other's VALU->SGPR-mask wait states
        if (s % REGION == REGION - 1) __builtin_amdgcn_sched_barrier(0);
        // TRIAD_FWD_PF_AT >= 0: the next DMA issued inside the chain (its slot was last read
        // before this tile's barrier), off the barrier -> first MFMA path
        if (s == TRIAD_FWD_PF_AT) {
          __builtin_amdgcn_sched_barrier(0);
          prefetch(b + NBUF - 1);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if constexpr (ep) {
#pragma unroll
      for (int v = 0; v < 16; ++v) epi_elem<TRAIN, full, EXACT>(e, p, v, lo);
    }
    if constexpr (ep) epi_end(p);
  };
  using T = std::true_type;
  using F = std::false_type;
  // epilogue variant of tile ec: FULL unless its sample's valid keys end inside it
  auto tile_full = [&]() __attribute__((always_inline)) {
    const int nk = a.klen ? min(load_uniform(a.klen, ec.j), a.Nk_eff) : a.Nk_eff;
    const int nv = __builtin_amdgcn_readfirstlane(nk - ec.kb * 32);
    e.nn2 = (f32x2){0.f, 0.f};
    e.mn = INFINITY;
    if constexpr (EXACT) e.st2 = (f32x2){0.f, 0.f};
    e.m0 = e.m;
    e.lim = (rok ? min(32, nv) : 0) - 4 * h;
    return nv >= 32;
  };

  // chain(b) accumulates into one register set while the epilogue of b-1 reads the other
#if TRIAD_FWD_PINGPONG
  // two tiles per trip with the sets' roles swapped (no 16-register copy per tile; a copy once
  // per launch when the tile count is even)
  auto step = [&](int b, f32x16& c, const f32x16& p) __attribute__((always_inline)) {
    if (tile_full()) iter(T{}, T{}, T{}, b, c, p);
    else iter(T{}, T{}, F{}, b, c, p);
  };
  iter(T{}, F{}, T{}, 0, cB, cA);
  int b = 1;
  for (; b + 1 < nblocks; b += 2) {
    step(b, cA, cB);
    step(b + 1, cB, cA);
  }
  if (b < nblocks) {
    step(b, cA, cB);
    cB = cA;
  }
#else
  iter(T{}, F{}, T{}, 0, cA, cB);
  cB = cA;
  for (int b = 1; b < nblocks; ++b) {
    if (tile_full()) iter(T{}, T{}, T{}, b, cA, cB);
    else iter(T{}, T{}, F{}, b, cA, cB);
    cB = cA;
  }
#endif
  if (tile_full()) iter(F{}, T{}, T{}, nblocks, cA, cB);
  else iter(F{}, T{}, F{}, nblocks, cA, cB);

  double v = wave_sum_d(accd);
  double v2 = wave_sum_d(accd2);
  __syncthreads();
  if (lane == 0) { red[wave] = v; red[WAVES + wave] = v2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, t2 = 0.0;
    for (int w = 0; w < WAVES; ++w) { t += red[w]; t2 += red[WAVES + w]; }
    // sum clamp(S, lo, 0)^2 = su^2 sum c^2; sum S^2/temp over [lo, 0] = temp sum u^2 there
    a.part[by * gx + bx] = t * (double)su * (double)su;
    if (a.part2) a.part2[by * gx + bx] = t2 * (double)temp;
  }
}

// ---- the same workgroup on v_mfma_f32_16x16x32_bf16 (the eval form's body, fwd_any) ----------
// Per wave and key tile: 32 keys x 32 queries as 2 x 2 tiles of 16 x 16 (key half kb2, query half
// qb), sixteen 32-deep k-steps of 4 MFMAs, one epilogue element of the previous tile per k-step.
// Lane l (i = l & 15, g = l >> 4) holds queries 16 qb + i and keys 16 kb2 + 4 g + (0..3): two running
// max / argmax per lane (one per query half), combined over the four lane groups at each sample's
// end. The unit dS keeps the 32 x 32 tile layout the backward reads (element (q, k) at
// (q + 32 ((k >> 2) & 1)) * 16 + (k & 3) + 4 (k >> 3)): per query half and key half a lane's four
// keys are one 8-byte piece of a 16-element run whose other pieces lane l ^ 32 holds.
constexpr int NS16 = D / 32;  // 16 k-steps
// Eval body: two tiles per loop trip with the accumulator sets alternating (no per-tile copy), which
// fits the register file only with LDS fragments one k-step ahead instead of two (249 VGPRs, no
// spill; with two ahead it spills 24): AV -2.9 %, TV -2.5 % (round 6, profiles/r06_fwd_eval_pingpong_ab.log)
#ifndef TRIAD_FWD16_PF_AT
#define TRIAD_FWD16_PF_AT 8   // eval body: k-step after which a tile pair's DMA is issued (A/B knob;
#endif                      // 8 vs -1: AV -2.3 %, TV -1.3 %, 3 / 5 / 8 swept, profiles/r06_fwd_eval_pf_at_ab.log)
#ifndef TRIAD_FWD16_LDSPF
#define TRIAD_FWD16_LDSPF 1
#endif
#ifndef TRIAD_FWD16_PINGPONG
#define TRIAD_FWD16_PINGPONG 1   // (A/B knob)
#endif
constexpr int LDSPF16 = TRIAD_FWD16_LDSPF;

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}


struct Epi16 {
  float m[2], m0[2];  // running max of u per query half, and at the tile's start
  int am[2], at[2];   // argmax within the sample (without 4g) / best key of the tile (valid when m > m0)
  int lim[2];         // masked tiles: valid keys of the tile minus 4g (0 - 4g for a padded query row)
  f32x2 nn2;
  float mn, prev;
  unsigned pk[8];     // unit dS, bf16 pairs: pk[4 kb2 + 2 qb + 0..1]
};

// element v = 8 kb2 + 4 qb + ii: key 16 kb2 + ii (+ 4g) of query half qb; accumulator p[v >> 2][v & 3]
__device__ __forceinline__ constexpr int vkey16(int v) { return 16 * (v >> 3) + (v & 3); }

template <bool TRAIN, bool FULL>
__device__ __forceinline__ void epi_elem16(Epi16& e, const f32x4 (&p)[4], int v, float lo) {
  const int qb = (v >> 2) & 1;
  const float u = p[v >> 2][v & 3];
  if constexpr (FULL) {
    e.at[qb] = u > e.m[qb] ? vkey16(v) : e.at[qb];  // keys ascend with v within a query half
    e.m[qb] = maxf(u, e.m[qb]);
  } else {
    PIN(e.lim[qb]);
    const bool better = vkey16(v) < e.lim[qb] && u > e.m[qb];
    e.m[qb] = better ? u : e.m[qb];
    e.at[qb] = better ? vkey16(v) : e.at[qb];
  }
  const float c = __builtin_amdgcn_fmed3f(u, lo, 0.f);
  if (v & 1) {
    e.nn2.x = fma_sq(e.prev, e.nn2.x);
    e.nn2.y = fma_sq(c, e.nn2.y);
    PIN(e.nn2);
    if constexpr (TRAIN) {
      e.mn = min3f(e.mn, p[v >> 2][(v & 3) - 1], u);
      e.pk[v >> 1] = pack_bf16x2(e.prev, c);
      PIN(e.mn);
      PIN(e.pk[v >> 1]);
    }
  } else {
    e.prev = c;
    PIN(e.prev);
  }
  PIN(e.m[qb]);
  PIN(e.at[qb]);
}

__device__ __forceinline__ float epi_fixup16(Epi16& e, const f32x4 (&p)[4], float lo) {
  float st = 0.f, dp = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const float u = p[v >> 2][v & 3];
    const float d = (u >= lo && u <= 0.f) ? u : 0.f;
    st = fmaf(d, d, st);
    if (v & 1) e.pk[v >> 1] = pack_bf16x2(dp, d);
    else dp = d;
  }
  return st;
}

template <bool TRAIN>
__device__ __forceinline__ void fwd_body16(const FwdArgs& a, bf16* kbuf, const int bx, const int by, const int gx) {
  double* red = (double*)(kbuf + NBUF16 * KT_ELEMS);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i16 = lane & 15, g = lane >> 4;
  const int row0 = bx * ROWS_PER_WG + wave * 32;
  const int rowq[2] = {row0 + i16, row0 + 16 + i16};
  const bool rok[2] = {rowq[0] < a.R, rowq[1] < a.R};
  const int rt = row0 / 32;

  const int j0 = by * a.j_per_wg;
  const int j1 = min(a.Bk, j0 + a.j_per_wg);
  const int nkb = a.Nk_pad / 32;
  const int nblocks = (j1 - j0) * nkb;
  if (nblocks <= 0) {
    if (threadIdx.x == 0) {
      a.part[by * gx + bx] = 0.0;
      if (a.part2) a.part2[by * gx + bx] = 0.0;
    }
    return;
  }
  const unsigned long long kaddr = (unsigned long long)(a.K + (size_t)j0 * a.Nk_pad * D);
  const i32x4 kr = {__builtin_amdgcn_readfirstlane((int)(unsigned)kaddr),
                    __builtin_amdgcn_readfirstlane((int)((unsigned)(kaddr >> 32) & 0xffffu)),
                    __builtin_amdgcn_readfirstlane((int)((unsigned)(j1 - j0) * a.Nk_pad * (D * 2))), 0x00020000};
  Cursor fc{j0, 0}, cc{j0, 0}, ec{j0, 0};
  int fslot = 0, cslot = 0;
  auto prefetch = [&](int b2) __attribute__((always_inline)) {
    if (b2 < nblocks) stage_tile(kr, kbuf + fslot * KT_ELEMS, (fc.j - j0) * a.Nk_pad + fc.kb * 32, wave, lane);
    fc.next(nkb);
    fslot = __builtin_amdgcn_readfirstlane(fslot == NBUF16 - 1 ? 0 : fslot + 1);
  };
  prefetch(0);
  prefetch(1);

  bf16x8 qf[2][NS16];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const bf16* q0 = a.Q + (size_t)rowq[qb] * D + 8 * g;  // rows < R_pad: zero tail, in the allocation
#pragma unroll
    for (int s = 0; s < NS16; ++s) qf[qb][s] = *(const bf16x8*)(q0 + 32 * s);
  }
  const float temp = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, *a.temp)));
  const float su = temp != 0.f ? fabsf(temp) : 1.f;
  if (!(temp > 0.f)) {
    const unsigned flip = temp < 0.f ? 0x80008000u : 0u, keep = temp == 0.f ? 0u : 0xffffffffu;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int s = 0; s < NS16; ++s) {
        u32x4 w = __builtin_bit_cast(u32x4, qf[qb][s]);
        w = (w & keep) ^ flip;
        qf[qb][s] = __builtin_bit_cast(bf16x8, w);
      }
  }
  const float lo = a.clamp_lo / su;
  double accd = 0.0, accd2 = 0.0;
  // swizzled LDS key-fragment offsets (bytes): key row 16 kb2 + i, chunk 4 s + g
  int xo[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) xo[k] = i16 * (D * 2) + (((4 * k + g) ^ i16) * 16);
  bf16* const dS_w = TRAIN ? a.dS + (long long)rt * a.CT * 1024 : nullptr;
  // this lane's 16-byte dS run inside a 32 x 32 tile, per query half: row 16 qb + i + 32 (g & 1), half h5
  const int h5 = g >> 1;
  const int dso[2] = {ds_chunk((i16 + 32 * (g & 1)) * 2 + h5) * 8, ds_chunk((16 + i16 + 32 * (g & 1)) * 2 + h5) * 8};

  Epi16 e;
  e.m[0] = e.m[1] = -INFINITY;
  e.am[0] = e.am[1] = 0;
  e.at[0] = e.at[1] = 0;
  f32x4 cA[4], cB[4];

  auto sync_tile = [&](int b) __attribute__((always_inline)) {
    // one barrier per PAIR of key tiles (even b), both DMA'd together two tiles ahead; younger
    // than them: the dS stores of iterations b-2 and b-1 (2 each, from iteration 1 on)
    if (b & 1) return;
    if (TRAIN && b >= 4) TRIAD_VMCNT(4);
    else if (TRAIN && b >= 2) TRIAD_VMCNT(2);
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto refill = [&](int b) __attribute__((always_inline)) {
    if (!(b & 1)) { prefetch(b + 2); prefetch(b + 3); }
  };

  auto epi_end = [&](const f32x4 (&p)[4]) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
      if (e.m[qb] > e.m0[qb]) e.am[qb] = ec.kb * 32 + e.at[qb];
    const float nn = e.nn2.x + e.nn2.y;
    accd += (double)nn;
    if (TRAIN) {
      const float st = __builtin_amdgcn_ballot_w64(e.mn < lo) ? epi_fixup16(e, p, lo) : nn;
      accd2 += (double)st;
      // lanes l and l ^ 32 hold the two halves of the same 16-element runs: swap one 8-byte
      // piece so each lane stores one 16-byte run (h5 = 0: elements 0..7, h5 = 1: 8..15)
      bf16* d = dS_w + ((long long)ec.j * nkb + ec.kb) * 1024;
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const unsigned s0 = h5 ? e.pk[2 * qb] : e.pk[4 + 2 * qb];
        const unsigned s1 = h5 ? e.pk[2 * qb + 1] : e.pk[4 + 2 * qb + 1];
        const unsigned r0 = __shfl_xor(s0, 32), r1 = __shfl_xor(s1, 32);
        const u32x4 v = h5 ? (u32x4){r0, r1, e.pk[4 + 2 * qb], e.pk[4 + 2 * qb + 1]}
                           : (u32x4){e.pk[2 * qb], e.pk[2 * qb + 1], r0, r1};
        store16(d + dso[qb], v);
      }
    }
    if (ec.kb == nkb - 1) {  // end of a key sample: combine the four lane groups per query half
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float m = e.m[qb];
        int am = e.am[qb] + 4 * g;
#pragma unroll
        for (int x = 16; x <= 32; x *= 2) {
          const float m2 = __shfl_xor(m, x);
          const int am2 = __shfl_xor(am, x);
          if (m2 > m || (m2 == m && am2 < am)) { m = m2; am = am2; }
        }
        if (g == qb && rok[qb]) {
          a.rowmax[(size_t)ec.j * a.R_pad + rowq[qb]] = su * m;
          a.argmax[(size_t)ec.j * a.R_pad + rowq[qb]] = am;
        }
        e.m[qb] = -INFINITY;
        e.am[qb] = 0;
      }
    }
    ec.next(nkb);
  };

  auto iter = [&](auto CH, auto EP, auto FULLT, int b, f32x4 (&c)[4], const f32x4 (&p)[4]) {
    constexpr bool ch = decltype(CH)::value, ep = decltype(EP)::value, full = decltype(FULLT)::value;
    if constexpr (ch) {
      sync_tile(b);
      if (TRIAD_FWD16_PF_AT < 0) refill(b);
      const char* kt = (const char*)kbuf + cslot * (KT_ELEMS * 2);
      cslot = __builtin_amdgcn_readfirstlane(cslot == NBUF16 - 1 ? 0 : cslot + 1);
      constexpr int P = LDSPF16;
      bf16x8 af[P + 1][2];
#pragma unroll
      for (int s = 0; s < P; ++s)
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
          af[s][kb2] = *(const bf16x8*)(kt + kb2 * 16 * (D * 2) + xo[s & 3] + (s >> 2) * 256);
#pragma unroll
      for (int t = 0; t < 4; ++t) c[t] = (f32x4){};
#pragma unroll
      for (int s = 0; s < NS16; ++s) {
        if (s + P < NS16)
#pragma unroll
          for (int kb2 = 0; kb2 < 2; ++kb2)
            af[(s + P) % (P + 1)][kb2] =
                *(const bf16x8*)(kt + kb2 * 16 * (D * 2) + xo[(s + P) & 3] + ((s + P) >> 2) * 256);
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2)
#pragma unroll
          for (int qb = 0; qb < 2; ++qb)
            c[2 * kb2 + qb] = mfma16(af[s % (P + 1)][kb2], qf[qb][s], c[2 * kb2 + qb]);
        if constexpr (ep) epi_elem16<TRAIN, full>(e, p, s, lo);
        __builtin_amdgcn_sched_barrier(0);
        if (s == TRIAD_FWD16_PF_AT) {   // the pair's DMA inside the chain (as fwd_body's TRIAD_FWD_PF_AT)
          refill(b);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
    } else if constexpr (ep) {
#pragma unroll
      for (int v = 0; v < 16; ++v) epi_elem16<TRAIN, full>(e, p, v, lo);
    }
    if constexpr (ep) epi_end(p);
  };
  using T = std::true_type;
  using F = std::false_type;
  auto tile_full = [&]() __attribute__((always_inline)) {
    const int nk = a.klen ? min(load_uniform(a.klen, ec.j), a.Nk_eff) : a.Nk_eff;
    const int nv = __builtin_amdgcn_readfirstlane(nk - ec.kb * 32);
    e.nn2 = (f32x2){0.f, 0.f};
    e.mn = INFINITY;
    e.m0[0] = e.m[0];
    e.m0[1] = e.m[1];
    e.lim[0] = (rok[0] ? min(32, nv) : 0) - 4 * g;
    e.lim[1] = (rok[1] ? min(32, nv) : 0) - 4 * g;
    return nv >= 32;
  };
  auto copy = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < 4; ++t) cB[t] = cA[t];
  };

#if TRIAD_FWD16_PINGPONG
  auto step = [&](int b, f32x4 (&c)[4], const f32x4 (&p)[4]) __attribute__((always_inline)) {
    if (tile_full()) iter(T{}, T{}, T{}, b, c, p);
    else iter(T{}, T{}, F{}, b, c, p);
  };
  iter(T{}, F{}, T{}, 0, cB, cA);
  int b = 1;
  for (; b + 1 < nblocks; b += 2) {
    step(b, cA, cB);
    step(b + 1, cB, cA);
  }
  if (b < nblocks) {
    step(b, cA, cB);
    copy();
  }
#else
  iter(T{}, F{}, T{}, 0, cA, cB);
  copy();
  for (int b = 1; b < nblocks; ++b) {
    if (tile_full()) iter(T{}, T{}, T{}, b, cA, cB);
    else iter(T{}, T{}, F{}, b, cA, cB);
    copy();
  }
#endif
  if (tile_full()) iter(F{}, T{}, T{}, nblocks, cA, cB);
  else iter(F{}, T{}, F{}, nblocks, cA, cB);

  double v = wave_sum_d(accd);
  double v2 = wave_sum_d(accd2);
  __syncthreads();
  if (lane == 0) { red[wave] = v; red[WAVES + wave] = v2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, t2 = 0.0;
    for (int w = 0; w < WAVES; ++w) { t += red[w]; t2 += red[WAVES + w]; }
    a.part[by * gx + bx] = t * (double)su * (double)su;
    if (a.part2) a.part2[by * gx + bx] = t2 * (double)temp;
  }
}

// Which body: measured on one box, alternated (profiles/r04_fwd_m16_ab.log, c3 shapes): the eval
// form (no dS stream) runs 4.7 % faster on 16 x 16 x 32 MFMAs (AV 2.47 -> 2.36 ms); the training
// form does not gain (AV 3.07 -> 3.06 ms with 8-byte dS stores, 3.10 with the runs assembled to
// 16-byte stores by a lane swap) -- its time is the dS stream and the epilogue, not the MFMA clock.
// Both bodies pass the same head tests (tests/test_head_gpu.py, 67 / 67 with either).
template <bool TRAIN>
__device__ __forceinline__ void fwd_any(const FwdArgs& a, bf16* kbuf, const int bx, const int by, const int gx) {
  if constexpr (TRAIN) {
    if (a.exact) fwd_body<true, true>(a, kbuf, bx, by, gx);   // uniform per problem
    else fwd_body<true, false>(a, kbuf, bx, by, gx);
  }
  else fwd_body16<false>(a, kbuf, bx, by, gx);
}

template <bool TRAIN, bool SHORTQ>
__global__ __launch_bounds__(64 * WAVES, 1) void pairsim_fwd2_kernel(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) bf16 kbuf[kbuf_elems<TRAIN>];
  fwd_any<TRAIN>(a, kbuf, blockIdx.x, blockIdx.y, gridDim.x);
}

// Several heads' forwards in ONE launch (the tri-modal step's AV and TV heads, model.py:470-472 /
// 593, over their own key sets): a 1-D grid, problem p owning workgroups [first[p], first[p+1]),
// each problem keeping its own (row block, key split) decomposition and partial arrays. The host
// orders the problems by workgroup length, longest first, so the dispatcher back-fills the CUs
// with the shorter workgroups and the launch ends in one tail instead of one per head.
constexpr int MAX_PROBLEMS = 2;
struct MultiArgs {
  FwdArgs p[MAX_PROBLEMS];
  int first[MAX_PROBLEMS + 1];
  int gx[MAX_PROBLEMS];
  int n;
};

template <bool TRAIN>
__global__ __launch_bounds__(64 * WAVES, 1) void pairsim_fwd_multi_kernel(MultiArgs m) {
  __shared__ __attribute__((aligned(16))) bf16 kbuf[kbuf_elems<TRAIN>];
  const int b = blockIdx.x;
  const int q = (m.n > 1 && b >= m.first[1]) ? 1 : 0;  // uniform
  const int local = b - m.first[q];
  const int gx = m.gx[q];
  fwd_any<TRAIN>(m.p[q], kbuf, local % gx, local / gx, gx);
}

// Diagonal blocks of S for the regularisers (model.py:417-418 / 524-525):
// diagS[i][q][k] = temp * <Q[i*Nq + q], K[(i + diag_off)*Nk_pad + k]>, k < Nk_eff.
// 1/B of the forward's FLOPs, kept out of the streaming kernel: grid (query blocks of 32,
// samples), DIAG_WAVES waves striding over 32-key tiles; query fragments in registers, key fragments
// straight from global (L2-resident), query-on-row orientation so each accumulator
// register stores 32 consecutive keys (128 B) per row.
constexpr int DIAG_PF = 8;   // key fragments in flight per wave (diag_sim_kernel)
#ifndef TRIAD_DIAG_WAVES
#define TRIAD_DIAG_WAVES 1
#endif
// waves per diag_sim workgroup, striding over the sample's key tiles. One: each wave loads its 32
// query rows' fragments (32 KB) once for all of the sample's key tiles (four waves each loaded
// them for two tiles); 1,792 one-wave workgroups fit the chip in one round at two waves per SIMD.
constexpr int DIAG_WAVES = TRIAD_DIAG_WAVES;
__global__ __launch_bounds__(256) void diag_sim_kernel(const bf16* __restrict__ Q, const bf16* __restrict__ K, int Nq,
                                                       int Nk_pad, int Nk_eff, int diag_off,
                                                       const float* __restrict__ temp_p, float* __restrict__ diagS) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 5, l32 = lane & 31;
  const int i = blockIdx.y, q0 = blockIdx.x * 32;
  const int qa = min(q0 + l32, Nq - 1);  // clamp: rows past Nq are computed, never stored
  const bf16* qrow = Q + ((size_t)i * Nq + qa) * D + 8 * h;
  bf16x8 qf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) qf[s] = *(const bf16x8*)(qrow + 16 * s);
  const float temp = *temp_p;
  const int ntiles = (Nk_eff + 31) / 32;
  const size_t kbase = (size_t)(i + diag_off) * Nk_pad;
  for (int kt = wave; kt < ntiles; kt += DIAG_WAVES) {
    const bf16* krow = K + (kbase + kt * 32 + l32) * D + 8 * h;  // rows < Nk_pad: in the allocation
    // key fragments DIAG_PF steps ahead (hipcc counts the waits): one L2 round trip per PF
    // k-steps instead of one per k-step (the fragment-at-use form waited vmcnt(0) before each
    // MFMA: 0.17 ms per step for the two heads; same MFMA order, bit-identical)
    constexpr int PF = DIAG_PF;
    bf16x8 kf[PF];
#pragma unroll
    for (int s = 0; s < PF; ++s) kf[s] = *(const bf16x8*)(krow + 16 * s);
    __builtin_amdgcn_sched_barrier(0);   // keep the loads here (the scheduler sinks them to their use)
    f32x16 acc = {};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const bf16x8 cur = kf[s % PF];
      if (s + PF < NS) kf[s % PF] = *(const bf16x8*)(krow + 16 * (s + PF));
      acc = mfma32(qf[s], cur, acc);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int key = kt * 32 + l32;
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int q = q0 + (v & 3) + 8 * (v >> 2) + 4 * h;
      if (q < Nq && key < Nk_eff) diagS[((size_t)i * Nq + q) * Nk_pad + key] = acc[v] * temp;
    }
  }
}

}  // namespace

int triad_pairsim_diag_launch(const triad_pairsim_problem* pr, int n, hipStream_t stream);

// Grid: triad_pairsim_nparts' decomposition (pairsim.hip grid_for), so partial arrays match.
// The diagonal S (diagS != null) comes from diag_sim_kernel, launched after on the same stream.
int triad_pairsim_fwd2_launch(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                              int Nk_eff, const float* temp, float clamp_lo, int diag, int diag_off, float* rowmax,
                              int* argmax, double* nn_part, float* diagS, void* dS, long long CT, double* st_part,
                              const int* k_len, int xb, int ys, int jpw, hipStream_t stream) {
  if ((unsigned long long)jpw * Nk_pad * D * 2 >= (1ull << 31)) return TRIAD_EINVAL;  // 32-bit buffer offsets
  FwdArgs a = {};
  a.Q = (const bf16*)Q; a.K = (const bf16*)K;
  a.R = R; a.R_pad = R_pad; a.Nq = Nq; a.Bq = Bq; a.Bk = Bk; a.Nk_pad = Nk_pad; a.Nk_eff = Nk_eff;
  a.j_per_wg = jpw; a.temp = temp; a.clamp_lo = clamp_lo;
  a.rowmax = rowmax; a.argmax = argmax; a.part = nn_part;
  a.dS = (bf16*)dS; a.CT = CT; a.part2 = st_part; a.klen = k_len;
  a.exact = exact_epilogue(clamp_lo);
  const int xw = xb * (256 / ROWS_PER_WG);  // xb counts 256-row blocks
  const bool sq = Nq <= 32;
  const dim3 grid(xw, ys), block(64 * WAVES);
  if (dS && sq) hipLaunchKernelGGL((pairsim_fwd2_kernel<true, true>), grid, block, 0, stream, a);
  else if (dS) hipLaunchKernelGGL((pairsim_fwd2_kernel<true, false>), grid, block, 0, stream, a);
  else if (sq) hipLaunchKernelGGL((pairsim_fwd2_kernel<false, true>), grid, block, 0, stream, a);
  else hipLaunchKernelGGL((pairsim_fwd2_kernel<false, false>), grid, block, 0, stream, a);
  TRIAD_CHECK_LAUNCH();
  if (diagS && diag) {
    hipLaunchKernelGGL(diag_sim_kernel, dim3((Nq + 31) / 32, Bq), dim3(64 * DIAG_WAVES), 0, stream, (const bf16*)Q,
                       (const bf16*)K, Nq, Nk_pad, Nk_eff, diag_off, temp, diagS);
    TRIAD_CHECK_LAUNCH();
  }
  return TRIAD_OK;
}

// triad_pairsim_fwd_multi's launch: per problem (validated and with its grid decomposition by the
// caller) xb row blocks x ys key splits of jpw samples; problems with longer workgroups first.
int triad_pairsim_fwd_multi_launch(const triad_pairsim_problem* pr, const int* xb, const int* ys, const int* jpw,
                                   int n, hipStream_t stream) {
  if (n < 1 || n > MAX_PROBLEMS) return TRIAD_EINVAL;
  const bool train = pr[0].dS != nullptr;
  int order[MAX_PROBLEMS] = {0, 1};
  if (n == 2 && (long long)jpw[1] * pr[1].Nk_pad > (long long)jpw[0] * pr[0].Nk_pad) { order[0] = 1; order[1] = 0; }
  MultiArgs m = {};
  m.n = n;
  m.first[0] = 0;
  for (int i = 0; i < n; ++i) {
    const triad_pairsim_problem& p = pr[order[i]];
    if ((p.dS != nullptr) != train) return TRIAD_EINVAL;
    if ((unsigned long long)jpw[order[i]] * p.Nk_pad * D * 2 >= (1ull << 31)) return TRIAD_EINVAL;
    FwdArgs& a = m.p[i];
    a.Q = (const bf16*)p.Q; a.K = (const bf16*)p.K;
    a.R = p.R; a.R_pad = p.R_pad; a.Nq = p.Nq; a.Bq = p.Bq; a.Bk = p.Bk; a.Nk_pad = p.Nk_pad;
    a.Nk_eff = p.Nk_eff; a.j_per_wg = jpw[order[i]]; a.temp = p.temp; a.clamp_lo = p.clamp_lo;
    a.rowmax = p.rowmax; a.argmax = p.argmax; a.part = p.nn_part;
    a.dS = (bf16*)p.dS; a.CT = p.CT; a.part2 = p.st_part; a.klen = nullptr;
    a.ktiles = p.dS ? p.k_tiles : nullptr;
    a.exact = exact_epilogue(p.clamp_lo);
    m.gx[i] = xb[order[i]] * (256 / ROWS_PER_WG);
    m.first[i + 1] = m.first[i] + m.gx[i] * ys[order[i]];
  }
  const dim3 grid(m.first[n]), block(64 * WAVES);
  if (train) hipLaunchKernelGGL((pairsim_fwd_multi_kernel<true>), grid, block, 0, stream, m);
  else hipLaunchKernelGGL((pairsim_fwd_multi_kernel<false>), grid, block, 0, stream, m);
  TRIAD_CHECK_LAUNCH();
  // the caller passes diag = 0 and launches triad_pairsim_diag over the PADDED keys (the forward's K
  // may be the compact one, which diag_sim cannot address; triad_pairsim_diag refuses it)
  return triad_pairsim_diag_launch(pr, n, stream);
}

// diag_sim of every problem with a diagonal output (shapes validated by the caller)
int triad_pairsim_diag_launch(const triad_pairsim_problem* pr, int n, hipStream_t stream) {
  for (int i = 0; i < n; ++i) {
    const triad_pairsim_problem& p = pr[i];
    if (p.diagS && p.diag) {
      hipLaunchKernelGGL(diag_sim_kernel, dim3((p.Nq + 31) / 32, p.Bq), dim3(64 * DIAG_WAVES), 0, stream, (const bf16*)p.Q,
                         (const bf16*)p.K, p.Nq, p.Nk_pad, p.Nk_eff, p.diag_off, p.temp, p.diagS);
      TRIAD_CHECK_LAUNCH();
    }
  }
  return TRIAD_OK;
}

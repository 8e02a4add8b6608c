// Projection head proj2(LN(proj1(h))) (SajayR/TRIAD src/model.py:32-34,68 / 81-83,116 /
// 253-255,326) under bf16 autocast (model.py:483,603), forward and backward, as persistent
// row-panel kernels in which each wave owns 32 token rows x ALL 512 features:
//
//   forward   y1 = bf16(h W1^T + b1)      phase A: MFMA over H, weights streamed through LDS
//             ln = bf16(LN(y1))           in registers: a token's 512 features live in 2 lanes
//             y  = bf16(ln W2^T + b2)     phase B: ln is the MFMA B operand straight from registers
//   backward  dln = bf16(dy W2)           phase A (W2^T streamed)
//             dy1 = bf16(LN'(dln))        in registers; dgamma / dbeta / db1 column sums by an
//                                          in-register transpose-reduce over the wave's tokens
//             dh  = bf16(dy1 W1)          phase B (W1^T streamed), dy1 from registers
//
// Layout trick: phase-A weight rows are staged in the permuted order sigma, so the accumulator
// register v of lane half h2 in output tile t holds feature 32t + 16(v>>3) + 8h2 + (v&7): each
// lane owns runs of 8 consecutive features. A run is (a) one 16-byte store, (b) exactly the
// 8 k-values the lane supplies as the B operand of a 32x32x16 MFMA in phase B (k-step
// = 16-feature group, half h2 = 8-feature half), so no LDS round trip between the GEMMs.
// Phase-B weight rows use the same permutation, so its outputs are 16-byte runs as well.
//
// Pipeline: one continuous stage sequence per workgroup (all its token groups, both phases);
// stage = 256 weight rows x 32 k (16 KB, + the 32 k of the group's tokens in phase A) through a
// 4-slot LDS ring by 16-byte LDS-DMA issued three stages ahead, counted `s_waitcnt vmcnt` +
// one barrier per stage. WAVES waves (one per SIMD) share each staged weight slab.
#include "common.h"

namespace {

constexpr int PH_F = 512;                 // projection width
constexpr int PH_K = 64;                  // k per stage (4 MFMA k-steps)
constexpr int PH_WA = 256;                // phase-A weight rows per stage (one half: 8 tiles)
constexpr int PH_WB = 256;                // phase-B weight rows per stage (one pass: 8 tiles)
constexpr int PH_NB = 3;                  // ring slots (DMA two stages ahead)

// slab row i (MFMA A-row order) of a 32-row tile -> weight row inside the tile
__device__ __forceinline__ int ph_sigma(int i) {
  const int v = (i & 3) + 4 * (i >> 3), h2 = (i >> 2) & 1;
  return 16 * (v >> 3) + 8 * h2 + (v & 7);
}
// [rows][64 k] image, 128-byte rows, 16-byte chunk c of row m at c ^ ((m >> 1) & 7): the 16 rows of
// any ds_read_b128 lane group hit 16 distinct 4-bank groups
__device__ __forceinline__ int ph_swz(int m) { return (m >> 1) & 7; }
__device__ __forceinline__ int ph_off(int m, int c) { return m * PH_K + ((c ^ ph_swz(m)) << 3); }

template <int WAVES>
struct PHCfg {
  static constexpr int TOK = 32 * WAVES;              // tokens per group
  static constexpr int SLOT = PH_WA * PH_K + TOK * PH_K;   // ring slot elements (phase-A size)
  static constexpr int WPA = (PH_WA / 8) / WAVES;     // weight DMA pieces per wave, phase-A stage
  static constexpr int WPB = (PH_WB / 8) / WAVES;     // phase-B stage
  static constexpr int PA = WPA + 4;                  // + the wave's 32 token rows
  static constexpr int PB = WPB;
};

struct PHArgs {
  const bf16* tok; long long ld_tok;   // phase-A token operand: h [M][H] (fwd) / dy [M][512] (bwd)
  int M, KA;                           // tokens, phase-A depth (H fwd / 512 bwd)
  const bf16* WA; long long ld_wa;     // phase-A weights [512][KA]: W1 (fwd) / W2^T (bwd)
  const bf16* WB; int NBp;             // phase-B weights [NBp*256][512]: W2 (fwd) / W1^T (bwd)
  const float* b1; const float* gamma; const float* beta; const float* b2; float eps;
  bf16* out; long long ld_out;         // y [M][512] (fwd) / dh [M][H] (bwd)
  bf16* y1; bf16* ln; float* mean; float* rstd;   // fwd: written; bwd: y1 / mean / rstd read
  bf16* dy1; float* colpart;           // bwd: dy1 [M][512]; colpart [grid][3][512] (dgamma, dbeta, db1)
  int ngroups;
};

typedef int i32x4 __attribute__((ext_vector_type(4)));

// Raw buffer descriptor (base, stride 0, num_records bytes, gfx950 raw-buffer flags): loads past
// num_records return zeros, which pads the last token group without a clamp.
__device__ __forceinline__ i32x4 ph_rsrc(const void* base, unsigned bytes) {
  const unsigned long long a = (unsigned long long)base;
  return (i32x4){__builtin_amdgcn_readfirstlane((int)(unsigned)a),
                 __builtin_amdgcn_readfirstlane((int)((unsigned)(a >> 32) & 0xffffu)),
                 __builtin_amdgcn_readfirstlane((int)bytes), 0x00020000};
}

// 16-byte-per-lane buffer LDS-DMA (buffer_load_dwordx4 ... lds) as inline asm (the compiler would
// otherwise see an LDS write and drain vmcnt(0) before every ds_read of the ring); M0 = the
// uniform LDS destination, written and restored inside the statement. Per lane only a 32-bit
// offset: the base and the stage offset are scalars.
__device__ __forceinline__ void ph_dma(i32x4 rsrc, unsigned lds_addr, unsigned voff, unsigned soff) {
  TRIAD_LDS_DMA_CHECK(lds_addr, 2);
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

// 16-byte / 4-byte buffer stores (compiler builtins: the compiler must see them as stores to
// insert the VMEM-store-data hazard wait states); offsets past num_records are dropped by the
// hardware, so invalid rows store nothing.
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ph_srsrc(void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void ph_st16(__amdgpu_buffer_rsrc_t r, unsigned voff, bf16x8 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, (int)voff, 0, 0);
}
__device__ __forceinline__ void ph_st4(__amdgpu_buffer_rsrc_t r, unsigned voff, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, (int)voff, 0, 0);
}
constexpr unsigned PH_DROP = 0xfffffff0u;   // an offset no descriptor here reaches

// s_waitcnt vmcnt(n) for a run-time n (clamped to the 6-bit field: waiting for fewer is safe)
template <int K>
__device__ __forceinline__ void ph_vmcnt() { TRIAD_VMCNT(K); }
__device__ __forceinline__ void ph_vmcnt_dyn(int n) {
  switch (n < 63 ? n : 63) {
#define PH_C(k) case k: ph_vmcnt<k>(); break;
#define PH_C8(k) PH_C(k) PH_C(k + 1) PH_C(k + 2) PH_C(k + 3) PH_C(k + 4) PH_C(k + 5) PH_C(k + 6) PH_C(k + 7)
    PH_C8(0) PH_C8(8) PH_C8(16) PH_C8(24) PH_C8(32) PH_C8(40) PH_C8(48) PH_C8(56)
#undef PH_C8
#undef PH_C
    default: ph_vmcnt<0>(); break;
  }
}

// Per-lane byte offsets of a weight slab's wave-instructions (8 rows x 8 chunks each; rows
// tile-permuted by sigma; instruction inst = wave + u * WAVES). Instruction u + 32/(8 WAVES) moves
// the same rows of the next 32-row tile: same swizzle, offset + 32 ldw bytes -- so only the first
// 32/(8 WAVES) offsets are per-lane registers, the tile step rides in the scalar soffset.
template <int WAVES>
struct PHW {
  static constexpr int PER = 4 / WAVES;   // distinct per-lane offsets (instructions per 32-row tile)
};
template <int WAVES>
__device__ __forceinline__ void ph_woff(long long ldw, int wave, int lane, unsigned (&off)[PHW<WAVES>::PER]) {
#pragma unroll
  for (int u = 0; u < PHW<WAVES>::PER; ++u) {
    const int inst = wave + u * WAVES;
    const int m = inst * 8 + (lane >> 3), cp = lane & 7;
    const int c = cp ^ ph_swz(m);
    off[u] = (unsigned)((((m & ~31) + ph_sigma(m & 31)) * ldw + c * 8) * 2);
  }
}
// Token slab: the wave's own 32 rows (4 instructions), relative to the wave's first row; the
// offsets of instructions 0 and 1 (instructions 2, 3 = the same + 16 rows).
__device__ __forceinline__ void ph_toff(long long ld, int lane, unsigned (&off)[2]) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int m = u * 8 + (lane >> 3), cp = lane & 7;   // ph_swz(32 w + m) == ph_swz(m)
    const int c = cp ^ ph_swz(m);
    off[u] = (unsigned)((m * ld + c * 8) * 2);
  }
}
__device__ __forceinline__ unsigned ph_lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(void, p));
}

// Move a bf16x8 into the AGPR file (the value keeps an AGPR register class: phase B's MFMAs read
// it as their B operand from there, leaving the VGPRs to fragment prefetch).
__device__ __forceinline__ bf16x8 ph_agpr(bf16x8 v) {
  bf16x8 r;
  asm volatile("; ph_agpr %0" : "=a"(r) : "0"(v));
  return r;
}

// One stage's MFMAs: acc[t] += W[tile t] . B over the stage's 4 k-steps (64 k). The 8 A fragments
// of k-step ks+1 are read from LDS while the 8 MFMAs of ks issue (double-buffered registers, a
// sched_barrier per k-step): with one wave per SIMD nothing else hides the LDS latency. bop(ks): the B fragment of k-step ks (a register or an LDS read).
__device__ __forceinline__ void ph_stage_mfma(const bf16* Ws, int l32, int h2, f32x16 (&acc)[8], bf16x8 b0,
                                              bf16x8 b1, bf16x8 b2, bf16x8 b3) {
  bf16x8 af[2][8];
#pragma unroll
  for (int t = 0; t < 8; ++t) af[0][t] = *(const bf16x8*)(Ws + ph_off(t * 32 + l32, h2));
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const bf16x8 b = ks == 0 ? b0 : (ks == 1 ? b1 : (ks == 2 ? b2 : b3));
    if (ks + 1 < 4) {
#pragma unroll
      for (int t = 0; t < 8; ++t) af[(ks + 1) & 1][t] = *(const bf16x8*)(Ws + ph_off(t * 32 + l32, 2 * (ks + 1) + h2));
    }
    // fences: the k-step ks+1 reads issue BEFORE ks's MFMAs (the scheduler would otherwise sink
    // each read to just before its own MFMA and expose the LDS latency)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int t = 0; t < 8; ++t) acc[t] = mfma32(af[ks & 1][t], b, acc[t]);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Sum over the 32 lanes of one half (same h2) of v[0..31]: lane l32 returns the total of v[l32]
// (a butterfly that halves the vector each step: 16 + 8 + 4 + 2 + 1 exchanges).
__device__ __forceinline__ float ph_xreduce32(const float (&v)[32], int l32) {
  float a[16];
  const bool b4 = l32 & 16, b3 = l32 & 8, b2 = l32 & 4, b1 = l32 & 2, b0 = l32 & 1;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const float keep = b4 ? v[16 + i] : v[i], send = b4 ? v[i] : v[16 + i];
    a[i] = keep + __shfl_xor(send, 16);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float keep = b3 ? a[8 + i] : a[i], send = b3 ? a[i] : a[8 + i];
    a[i] = keep + __shfl_xor(send, 8);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float keep = b2 ? a[4 + i] : a[i], send = b2 ? a[i] : a[4 + i];
    a[i] = keep + __shfl_xor(send, 4);
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const float keep = b1 ? a[2 + i] : a[i], send = b1 ? a[i] : a[2 + i];
    a[i] = keep + __shfl_xor(send, 2);
  }
  const float keep = b0 ? a[1] : a[0], send = b0 ? a[0] : a[1];
  return keep + __shfl_xor(send, 1);
}

// Issue stage st's LDS-DMA (weights + the group's tokens in phase A, weights in phase B) into ring
// slot st % PH_NB. Everything by value: a lambda capturing these by reference turned the captures
// into pointers to scratch in this large kernel.
struct PHRing {
  i32x4 rA, rB, rT;
  unsigned lds0, oA0, oA1, oB0, oB1, oT0, oT1, tileA, tileB, tileT;
  int S, SA, KTA, TOK;
  long long ld_wa, ld_tok;
};

template <int WAVES>
__device__ __forceinline__ void ph_issue(const PHRing r, int st, int wave) {
  constexpr int PER = PHW<WAVES>::PER;
  using C = PHCfg<WAVES>;
  const int grp = blockIdx.x + (st / r.S) * gridDim.x, loc = st % r.S;
  const unsigned dst = r.lds0 + (unsigned)((st % PH_NB) * C::SLOT * 2);
  if (loc < r.SA) {
    const int half = loc >= r.KTA, kt = loc - half * r.KTA;
    const unsigned sA = (unsigned)((half * PH_WA * r.ld_wa + kt * PH_K) * 2);
#pragma unroll
    for (int u = 0; u < C::WPA; ++u)
      ph_dma(r.rA, dst + (wave + u * WAVES) * 1024, (u % PER) ? r.oA1 : r.oA0, sA + (u / PER) * r.tileA);
    const unsigned sT = (unsigned)(((long long)grp * r.TOK + wave * 32) * r.ld_tok * 2 + kt * PH_K * 2);
    // instruction u moves rows 8u..8u+7; u and u+2 share the swizzle (rows 16 apart)
#pragma unroll
    for (int u = 0; u < 4; ++u)
      ph_dma(r.rT, dst + PH_WA * PH_K * 2 + (wave * 4 + u) * 1024, (u & 1) ? r.oT1 : r.oT0,
             sT + (u >> 1) * r.tileT);
  } else {
    const int lb = loc - r.SA, pass = lb >> 3, kt = lb & 7;
    const unsigned sB = (unsigned)((pass * PH_WB * PH_F + kt * PH_K) * 2);
#pragma unroll
    for (int u = 0; u < C::WPB; ++u)
      ph_dma(r.rB, dst + (wave + u * WAVES) * 1024, (u % PER) ? r.oB1 : r.oB0, sB + (u / PER) * r.tileB);
  }
}

template <int WAVES, bool BWD>
__global__ __launch_bounds__(64 * WAVES, 1) void projhead_rows_kernel(PHArgs p) {
  using C = PHCfg<WAVES>;
  __shared__ __attribute__((aligned(16))) bf16 lds[PH_NB * C::SLOT];
  __shared__ float sprm[4][PH_F];  // fwd: b1, gamma, beta, b2; bwd: gamma
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int l32 = lane & 31, h2 = lane >> 5;

  for (int i = threadIdx.x; i < PH_F; i += 64 * WAVES) {
    sprm[1][i] = p.gamma[i];
    if (!BWD) {
      sprm[0][i] = p.b1[i];
      sprm[2][i] = p.beta[i];
      sprm[3][i] = p.b2[i];
    }
  }
  // (the first stage's barrier orders these writes before any read)

  const int KTA = p.KA / PH_K;                // phase-A stages per half
  const int SA = 2 * KTA;                     // phase-A stages per group (two 256-row halves)
  const int SB = 8 * p.NBp;                   // phase-B stages per group
  const int S = SA + SB;
  const int my_groups = (p.ngroups - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const int total = my_groups * S;

  // per-lane DMA offsets as named scalars (arrays captured by the lambdas below would be forced
  // into scratch memory): weight slabs need PER = 4 / WAVES bases, the token slab 4
  constexpr int PER = PHW<WAVES>::PER;
  static_assert(PER <= 2, "WAVES must be 2 or 4");
  unsigned tmpo[PER], tmpt[2];
  ph_woff<WAVES>(p.ld_wa, wave, lane, tmpo);
  const unsigned oA0 = tmpo[0], oA1 = tmpo[PER - 1];
  ph_woff<WAVES>(PH_F, wave, lane, tmpo);
  const unsigned oB0 = tmpo[0], oB1 = tmpo[PER - 1];
  ph_toff(p.ld_tok, lane, tmpt);
  const unsigned oT0 = tmpt[0], oT1 = tmpt[1];
  const unsigned tileA = (unsigned)(32 * p.ld_wa * 2), tileB = 32u * PH_F * 2;   // bytes per 32 weight rows
  const i32x4 rA = ph_rsrc(p.WA, (unsigned)(PH_F * p.ld_wa * 2));
  const i32x4 rB = ph_rsrc(p.WB, (unsigned)(p.NBp * PH_WB * PH_F * 2));
  const i32x4 rT = ph_rsrc(p.tok, (unsigned)((long long)p.M * p.ld_tok * 2));
  const unsigned lds0 = ph_lds_addr(lds);
  PHRing ring;
  ring.rA = rA; ring.rB = rB; ring.rT = rT; ring.lds0 = lds0;
  ring.oA0 = oA0; ring.oA1 = oA1; ring.oB0 = oB0; ring.oB1 = oB1;
  ring.oT0 = oT0; ring.oT1 = oT1; ring.tileT = (unsigned)(16 * p.ld_tok * 2);
  ring.tileA = tileA; ring.tileB = tileB; ring.S = S; ring.SA = SA; ring.KTA = KTA; ring.TOK = C::TOK;
  ring.ld_wa = p.ld_wa; ring.ld_tok = p.ld_tok;
  const auto rOut = ph_srsrc(p.out, (unsigned)((long long)p.M * p.ld_out * 2));
  const auto rRow = ph_srsrc(BWD ? (void*)p.dy1 : (void*)p.y1, (unsigned)(p.M * PH_F * 2));   // y1 (fwd) / dy1 (bwd)
  const auto rLn = ph_srsrc(BWD ? nullptr : p.ln, BWD ? 0u : (unsigned)(p.M * PH_F * 2));
  const auto rMean = ph_srsrc(BWD ? nullptr : p.mean, BWD ? 0u : (unsigned)(p.M * 4));
  const auto rRstd = ph_srsrc(BWD ? nullptr : p.rstd, BWD ? 0u : (unsigned)(p.M * 4));
  f32x16 acc[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) acc[t] = (f32x16){};
  // reg[t][a]: the lane's run of 8 features 32t + 16a + 8h2 + (0..7) of its token:
  // y1 -> ln (fwd) / dln -> dy1 (bwd); phase B's MFMA B operand
  bf16x8 reg[16][2];
  float colacc[3][8];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int c = 0; c < 8; ++c) colacc[q][c] = 0.f;

#pragma unroll
  for (int st = 0; st < PH_NB - 1; ++st)
    if (st < total) ph_issue<WAVES>(ring, st, wave);
  // Counted waits: LDS-DMA loads complete in issue order, so waiting until no more than stage s+1's
  // pieces are outstanding means stage s has landed. Output stores issued since then are not
  // counted as "younger" (stores are not ordered against loads): at worst the wait also covers them.
  int s = 0;   // running stage index (ring slot s % PH_NB)
#define PH_STORES(n) ((void)0)
  // wait for stage s (stage s+1's DMA stays in flight), barrier, refill the slot that stage s-1
  // freed; Ws = stage s's slot
#define PH_BEGIN(Ws)                                                                                  \
  do {                                                                                                \
    const int nx_ = s + 1 < total ? (((s + 1) % S) < SA ? C::PA : C::PB) : 0;                         \
    ph_vmcnt_dyn(nx_);                                                                                \
    __syncthreads();                                                                                  \
    if (s + PH_NB - 1 < total) ph_issue<WAVES>(ring, s + PH_NB - 1, wave);                           \
    Ws = lds + (s % PH_NB) * C::SLOT;                                                                 \
  } while (0)

  for (int gi = 0; gi < my_groups; ++gi) {
    const int grp = blockIdx.x + gi * gridDim.x;
    const int tokrow = grp * C::TOK + wave * 32 + l32;
    const bool valid = tokrow < p.M;
    // ---------------- phase A: acc[t] (+)= W_A[rows of tile t] . tokens^T, two 256-row halves ----------------
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      for (int kt = 0; kt < KTA; ++kt, ++s) {
        const bf16* Ws;
        PH_BEGIN(Ws);
        const bf16* Ts = Ws + PH_WA * PH_K;
        const int tr = wave * 32 + l32;
        ph_stage_mfma(Ws, l32, h2, acc, *(const bf16x8*)(Ts + ph_off(tr, h2)), *(const bf16x8*)(Ts + ph_off(tr, 2 + h2)),
                      *(const bf16x8*)(Ts + ph_off(tr, 4 + h2)), *(const bf16x8*)(Ts + ph_off(tr, 6 + h2)));
      }
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          bf16x8 r;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float x = acc[t][8 * a + j];
            if (!BWD) x += sprm[0][half * 256 + t * 32 + 16 * a + 8 * h2 + j];   // + b1, then bf16
            r[j] = (bf16)x;
          }
          reg[half * 8 + t][a] = ph_agpr(r);
        }
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = (f32x16){};
    }

    if (!BWD) {
      // ---------------- LayerNorm over the token's 512 features (2 lanes) ----------------
      // (sched_barrier every 4 tiles: the AGPR -> VGPR reads of reg stay a few tiles at a time)
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int j = 0; j < 8; ++j) sum += (float)reg[t][a][j];
        if (t % 4 == 3) __builtin_amdgcn_sched_barrier(0);
      }
      sum += __shfl_xor(sum, 32);
      const float mu = sum * (1.f / PH_F);
      float sq = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = (float)reg[t][a][j] - mu;
            sq += d * d;
          }
        if (t % 4 == 3) __builtin_amdgcn_sched_barrier(0);
      }
      sq += __shfl_xor(sq, 32);
      const float rs = rsqrtf(sq * (1.f / PH_F) + p.eps);
#pragma unroll
      for (int t = 0; t < 16; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int f0 = t * 32 + 16 * a + 8 * h2;
          const unsigned off = valid ? (unsigned)((tokrow * PH_F + f0) * 2) : PH_DROP;
          ph_st16(rRow, off, reg[t][a]);
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            o[j] = (bf16)(((float)reg[t][a][j] - mu) * rs * sprm[1][f0 + j] + sprm[2][f0 + j]);
          reg[t][a] = ph_agpr(o);
          ph_st16(rLn, off, o);
          __builtin_amdgcn_sched_barrier(0);
        }
      const unsigned moff = (valid && h2 == 0) ? (unsigned)(tokrow * 4) : PH_DROP;
      ph_st4(rMean, moff, mu);
      ph_st4(rRstd, moff, rs);
      PH_STORES(2 * 32 + 2);
    } else {
      // ---------------- LayerNorm backward (fp32) ----------------
      // xhat = (y1 - mean) rstd, g = dln gamma, dy1 = rstd (g - mean(g) - xhat mean(g xhat))
      const float mu = valid ? p.mean[tokrow] : 0.f, rs = valid ? p.rstd[tokrow] : 0.f;
      const bf16* yrow = p.y1 + (size_t)(valid ? tokrow : 0) * PH_F;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int t = 0; t < 16; ++t) {
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int f0 = t * 32 + 16 * a + 8 * h2;
          const bf16x8 yv = *(const bf16x8*)(yrow + f0);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float g = valid ? (float)reg[t][a][j] * sprm[1][f0 + j] : 0.f;
            s1 += g;
            s2 += g * (((float)yv[j] - mu) * rs);
          }
        }
        asm volatile("" ::: "memory");   // bound the y1 loads in flight (registers)
      }
      // memory clobber: the chunk loop below re-reads y1 from L1 instead of keeping the first
      // pass's 128 registers of loads alive (load CSE across the two passes)
      asm volatile("" ::: "memory");
      s1 += __shfl_xor(s1, 32);
      s2 += __shfl_xor(s2, 32);
      s1 *= (1.f / PH_F);
      s2 *= (1.f / PH_F);
      // per 32-feature chunk c (tiles 2c, 2c+1): dy1 (stored, and kept as phase B's operand) and
      // the column partials of dbeta (dln), dgamma (dln xhat), db1 (dy1); idx = 16 tt + 8 a + j
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        bf16x8 xv[2][2], dl[2][2];
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            xv[tt][a] = *(const bf16x8*)(yrow + (2 * c + tt) * 32 + 16 * a + 8 * h2);
            dl[tt][a] = valid ? reg[2 * c + tt][a] : (bf16x8){};
          }
        float v[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] = (float)dl[i >> 4][(i >> 3) & 1][i & 7];
        colacc[1][c] += ph_xreduce32(v, l32);
#pragma unroll
        for (int i = 0; i < 32; ++i) v[i] *= ((float)xv[i >> 4][(i >> 3) & 1][i & 7] - mu) * rs;
        colacc[0][c] += ph_xreduce32(v, l32);
#pragma unroll
        for (int tt = 0; tt < 2; ++tt)
#pragma unroll
          for (int a = 0; a < 2; ++a) {
            const int t = 2 * c + tt;
            const int f0 = t * 32 + 16 * a + 8 * h2;
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float xh = ((float)xv[tt][a][j] - mu) * rs;
              o[j] = (bf16)(rs * ((float)dl[tt][a][j] * sprm[1][f0 + j] - s1 - xh * s2));
              v[tt * 16 + a * 8 + j] = (float)o[j];
            }
            reg[t][a] = ph_agpr(o);
            ph_st16(rRow, valid ? (unsigned)((tokrow * PH_F + f0) * 2) : PH_DROP, o);
          }
        colacc[2][c] += ph_xreduce32(v, l32);
        asm volatile("" ::: "memory");   // one chunk's values live at a time
      }
      PH_STORES(32);
    }

    // ---------------- phase B: NBp passes of 256 rows of W_B . reg^T ----------------
    for (int pass = 0; pass < p.NBp; ++pass) {
#pragma unroll
      for (int kt = 0; kt < 8; ++kt, ++s) {
        const bf16* Ws;
        PH_BEGIN(Ws);
        // k-step ks: features 64 kt + 16 ks .. +15
        ph_stage_mfma(Ws, l32, h2, acc, reg[2 * kt][0], reg[2 * kt][1], reg[2 * kt + 1][0], reg[2 * kt + 1][1]);
      }
      // pass done: (+ b2) bf16 runs of 8 output columns
#pragma unroll
      for (int t = 0; t < 8; ++t)
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          const int col = pass * PH_WB + t * 32 + 16 * a + 8 * h2;
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float x = acc[t][8 * a + j];
            if (!BWD) x += sprm[3][col + j];
            o[j] = (bf16)x;
          }
          ph_st16(rOut, valid ? (unsigned)((tokrow * p.ld_out + col) * 2) : PH_DROP, o);
        }
      PH_STORES(16);
#pragma unroll
      for (int t = 0; t < 8; ++t) acc[t] = (f32x16){};
    }
  }
  if (BWD) {
    // column partials of this workgroup's waves: lane l32 of half h2 holds, for chunk c, feature
    // 64 c + 32 (l32 >> 4) + 16 ((l32 >> 3) & 1) + 8 h2 + (l32 & 7)
    __syncthreads();
    float* red = (float*)lds;   // [WAVES][3][512], the ring is idle now
#pragma unroll
    for (int qq = 0; qq < 3; ++qq)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const int f = 64 * c + 32 * (l32 >> 4) + 16 * ((l32 >> 3) & 1) + 8 * h2 + (l32 & 7);
        red[(wave * 3 + qq) * PH_F + f] = colacc[qq][c];
      }
    __syncthreads();
    for (int e = threadIdx.x; e < 3 * PH_F; e += 64 * WAVES) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < WAVES; ++w) t += red[w * 3 * PH_F + e];
      p.colpart[(size_t)blockIdx.x * 3 * PH_F + e] = t;
    }
  }
}

#undef PH_BEGIN
#undef PH_STORES

int ph_waves(int M) { return M >= 32768 ? 4 : 2; }

int ph_grid(int M, int waves) {
  const int groups = (M + 32 * waves - 1) / (32 * waves);
  const int slots = 256;   // one workgroup per CU (LDS: the 3-slot ring of 32 KB weight stages)
  return groups < slots ? groups : slots;
}

template <bool BWD>
int ph_launch(PHArgs& a, hipStream_t st) {
  const int w = ph_waves(a.M);
  a.ngroups = (a.M + 32 * w - 1) / (32 * w);
  const int grid = ph_grid(a.M, w);
  if (w == 4) hipLaunchKernelGGL((projhead_rows_kernel<4, BWD>), dim3(grid), dim3(256), 0, st, a);
  else hipLaunchKernelGGL((projhead_rows_kernel<2, BWD>), dim3(grid), dim3(128), 0, st, a);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // namespace

extern "C" {

int triad_projhead_fwd(const void* h, int M, int H, const void* W1, const float* b1, const float* gamma,
                       const float* beta, float eps, const void* W2, const float* b2, void* y, long long ldy,
                       void* y1, void* ln, float* mean, float* rstd, hipStream_t stream) {
  if (M <= 0 || H < PH_K || H % PH_K || ldy < PH_F || ldy % 8) return TRIAD_EINVAL;   // H % 32
  if ((long long)M * H * 2 >= (1ll << 31)) return TRIAD_EINVAL;   // 32-bit buffer offsets
  PHArgs a = {};
  a.tok = (const bf16*)h; a.ld_tok = H; a.M = M; a.KA = H;
  a.WA = (const bf16*)W1; a.ld_wa = H; a.WB = (const bf16*)W2; a.NBp = PH_F / PH_WB;
  a.b1 = b1; a.gamma = gamma; a.beta = beta; a.b2 = b2; a.eps = eps;
  a.out = (bf16*)y; a.ld_out = ldy; a.y1 = (bf16*)y1; a.ln = (bf16*)ln; a.mean = mean; a.rstd = rstd;
  return ph_launch<false>(a, stream);
}

int triad_projhead_bwd_slabs(int M) {
  if (M <= 0) return 0;
  return ph_grid(M, ph_waves(M));
}

int triad_projhead_bwd(const void* dy, int M, int H, const void* W2t, const void* W1t, const void* y1,
                       const float* mean, const float* rstd, const float* gamma, void* dy1, void* dh, long long ldh,
                       float* colpart, hipStream_t stream) {
  if (M <= 0 || H % PH_WB || H <= 0 || ldh < H || ldh % 8) return TRIAD_EINVAL;   // H % 256
  if ((long long)M * PH_F * 2 >= (1ll << 31)) return TRIAD_EINVAL;   // 32-bit buffer offsets
  PHArgs a = {};
  a.tok = (const bf16*)dy; a.ld_tok = PH_F; a.M = M; a.KA = PH_F;
  a.WA = (const bf16*)W2t; a.ld_wa = PH_F; a.WB = (const bf16*)W1t; a.NBp = H / PH_WB;
  a.gamma = gamma; a.out = (bf16*)dh; a.ld_out = ldh;
  a.y1 = (bf16*)y1; a.mean = (float*)mean; a.rstd = (float*)rstd; a.dy1 = (bf16*)dy1; a.colpart = colpart;
  return ph_launch<true>(a, stream);
}

}  // extern "C"

// Shared device helpers for the TRIAD MI355X (gfx950 / CDNA4) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "triad_hip.h"

#define TRIAD_OK 0

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// Dropout keep bits shared by every dropout kernel (postln.hip, attention.hip): a counter hash of
// (seed, element pair q = e / 2) gives one 16-bit uniform per element; keep iff >= thr
// (thr = round(p * 65536)). Bit 0 / bit 1 of keep_pair = elements 2q / 2q + 1.
__device__ __forceinline__ unsigned hash32(unsigned x) {  // lowbias32
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ unsigned keep_pair(unsigned long long q, unsigned seed, unsigned thr) {
  const unsigned h = hash32((unsigned)q * 0x9E3779B9u + seed + hash32((unsigned)(q >> 32) ^ 0x85ebca6bu));
  return ((h & 0xffffu) >= thr ? 1u : 0u) | ((h >> 16) >= thr ? 2u : 0u);
}
inline unsigned triad_drop_thr(float p) { return (unsigned)(p * 65536.f + 0.5f); }

// Debug builds (tools/build_variants.py; never the product library):
//  * TRIAD_LDS_CHECK: every LDS-DMA wave-instruction checks that its 1 KB destination (64 lanes x
//    16 B from the wave-uniform address) lies inside the kernel's static LDS allocation, and
//    prints the kernel's site and address if not -- a DMA beyond the allocation would land in a
//    co-resident workgroup's LDS;
//  * TRIAD_VMCNT0: every counted `s_waitcnt vmcnt(N)` becomes vmcnt(0). Outputs bit-identical
//    to the product build's show that the counted waits retire everything the code reads.
#ifdef TRIAD_LDS_CHECK
#include <cstdio>
__device__ __forceinline__ void lds_dma_check(unsigned lds_byte_addr, int site) {
  const unsigned size = __builtin_amdgcn_groupstaticsize();
  if (lds_byte_addr + 1024u > size && (threadIdx.x & 63) == 0)
    printf("TRIAD_LDS_CHECK OOB site %d block %d,%d wave %d lds %u + 1024 > %u\n", site, (int)blockIdx.x,
           (int)blockIdx.y, (int)(threadIdx.x >> 6), lds_byte_addr, size);
}
#define TRIAD_LDS_DMA_CHECK(addr, site) lds_dma_check((addr), (site))
#else
#define TRIAD_LDS_DMA_CHECK(addr, site) ((void)0)
#endif
#ifdef TRIAD_VMCNT0
#define TRIAD_VMCNT(n) asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
#else
#define TRIAD_VMCNT(n) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(n) : "memory")
#endif

// Storage order of the 16-byte chunks of a 2 KB tile of the tiled dS (pairsim_fwd.hip, bwd_gemm.hip):
// canonical chunk c -- lane L's values 8s..8s+7 (s = 0, 1) of the v_mfma_f32_32x32x16 accumulator
// order are chunk 2L + s -- is stored at (c >> 1) + 64 (c & 1), so each of the forward's two 16-byte
// stores per lane writes 1 KB contiguous (16 whole 64-byte lines) instead of 16 bytes of every 32.
// Round 5: training forward AV 3.03 -> 2.92 ms, TV 0.535 -> 0.516 (profiles/r05_fwd_ds_contig_ab.log).
// Readers map the canonical chunk through it (the LDS images they build are unchanged).
__device__ __forceinline__ int ds_chunk(int c) { return (c >> 1) | ((c & 1) << 6); }

// One 16-byte global->LDS DMA per lane (global_load_lds_dwordx4). The LDS
// destination is the wave-uniform `lds_base` + lane*16; the global source is
// per lane (CDNA4 LDS-DMA semantics).
// Inline asm on purpose: hipcc models the builtin as an LDS write it cannot tell apart from
// the ring slot being read, and drains vmcnt(0) -- the prefetch just issued included --
// before the next ds_read, serialising every double-buffered loop. Completion is the
// caller's: lds_dma_barrier() (vmcnt + barrier) before the data is read. M0 is written and
// restored inside the statement (cdna_hip_programming.md §5.7).
__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDS_PTR(void, lds_base));
  TRIAD_LDS_DMA_CHECK(lds, 0);
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds)
      : "memory");
}

// Make this wave's LDS-DMA writes complete, then barrier: the only ordering
// that makes global_load_lds data visible to other waves' ds_reads. (hipcc for
// gfx950 does NOT add the vmcnt wait to __syncthreads() by itself.)
__device__ __forceinline__ void lds_dma_barrier() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// 32x32x16 bf16 MFMA, fp32 accumulate.
__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Transposed LDS read (ds_read_b64_tr_b16): lane 4q+p of each 16-lane group
// supplies the address of row q, columns 4p..4p+3 of a 4x16 block; lane i of
// the group receives column i of the 4 rows.
__device__ __forceinline__ s16x4 lds_tr16(const void* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, p));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// Block-wide double sum; every thread gets the result. `red` needs
// blockDim.x/64 doubles of LDS.
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_d(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

#define TRIAD_CHECK_LAUNCH()                                   \
  do {                                                         \
    hipError_t _e = hipGetLastError();                         \
    if (_e != hipSuccess) return (int)_e;                      \
  } while (0)

// Co-residency hazard probe (diagnostic only, not part of the product library).
//
// Round 3 / 4 evidence: kernels whose fp32 arithmetic is packed (v_pk_*_f32) -- PyTorch's bf16
// sum reduction, an SLP-vectorised conv kernel -- return wrong values in some launches while one
// of the library's MFMA GEMMs runs on another stream, and never beside rocBLAS GEMMs or alone
// (tools/reduce_race.py). Here the aggressor is cut into its ingredients and the victims are
// minimal kernels with a fixed instruction choice (inline asm), each checked bit for bit against
// its solo result (tools/hazard_probe.py):
//   aggressors: mfma_loop (v_mfma_f32_32x32x16_bf16 chains, operands in registers), dma_loop
//               (global_load_lds_dwordx4 into an LDS ring + vmcnt / barrier, no MFMA), mix_loop
//               (both), valu_loop (scalar fp32 FMAs: control);
//   victims:    pk_victim (v_pk_fma_f32 chains), fma_victim (the same arithmetic as scalar
//               v_fma_f32), pk_add_victim (v_pk_add_f32 accumulation, a reduction's inner loop).
#include <hip/hip_runtime.h>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#define LDSP(p) ((__attribute__((address_space(3))) void*)(p))

__device__ __forceinline__ void glds16(const void* gsrc, void* lds_base) {
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(size_t)LDSP(lds_base));
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

extern "C" __global__ __launch_bounds__(256) void mfma_loop(float* out, int iters) {
  const int t = threadIdx.x;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * ((t * 7 + i) % 13) - 0.006f);
    b[i] = (__bf16)(0.001f * ((t * 5 + i) % 11) - 0.005f);
  }
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c3, 0, 0, 0);
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * 256 + t] = s;
}

extern "C" __global__ __launch_bounds__(256) void dma_loop(const float* src, long long n4, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float ring[4 * 4 * 256];   // 4 slots x 4 waves x 1 KB
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float s = 0.f;
  for (int it = 0; it < iters; ++it) {
    const int slot = it & 3;
    const long long row = ((long long)(blockIdx.x * 131 + it * 17 + wave) * 64 + lane) % n4;
    glds16(src + row * 4, ring + (slot * 4 + wave) * 256);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    s += ring[(slot * 4 + (wave ^ 1)) * 256 + lane * 4];
    __syncthreads();
  }
  out[blockIdx.x * 256 + t] = s;
}

extern "C" __global__ __launch_bounds__(256) void mix_loop(const float* src, long long n4, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float ring[4 * 4 * 256];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * ((t * 7 + i) % 13) - 0.006f);
    b[i] = (__bf16)(0.001f * ((t * 5 + i) % 11) - 0.005f);
  }
  f32x16 c0 = {}, c1 = {};
  float s = 0.f;
  for (int it = 0; it < iters; ++it) {
    const int slot = it & 3;
    const long long row = ((long long)(blockIdx.x * 131 + it * 17 + wave) * 64 + lane) % n4;
    glds16(src + row * 4, ring + (slot * 4 + wave) * 256);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, a, c1, 0, 0, 0);
    c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, a, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b, b, c1, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    s += ring[(slot * 4 + (wave ^ 1)) * 256 + lane * 4];
    __syncthreads();
  }
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i];
  out[blockIdx.x * 256 + t] = s;
}

extern "C" __global__ __launch_bounds__(256) void valu_loop(float* out, int iters) {
  float x = threadIdx.x * 1e-3f, y = 1.0001f;
  for (int it = 0; it < iters; ++it) {
    x = fmaf(x, y, 1e-6f);
    y = fmaf(y, 0.99999f, 1e-7f);
  }
  out[blockIdx.x * 256 + threadIdx.x] = x + y;
}

// victims: 64 dependent steps per element, element = (x, y) pair
extern "C" __global__ __launch_bounds__(256) void pk_victim(const f32x2* in, f32x2* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  f32x2 x = in[i];
  const f32x2 a = {0.9990234375f, 1.0009765625f}, b = {1e-3f, -1e-3f};
#pragma unroll 8
  for (int k = 0; k < 64; ++k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b));
  out[i] = x;
}

extern "C" __global__ __launch_bounds__(256) void fma_victim(const f32x2* in, f32x2* out, int n) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float x0 = in[i].x, x1 = in[i].y;
#pragma unroll 8
  for (int k = 0; k < 64; ++k) {
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x0) : "v"(0.9990234375f), "v"(1e-3f));
    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x1) : "v"(1.0009765625f), "v"(-1e-3f));
  }
  out[i] = (f32x2){x0, x1};
}

extern "C" __global__ __launch_bounds__(256) void pk_add_victim(const f32x2* in, f32x2* out, int n, int rows) {
  // column sums of a [rows][n] f32x2 matrix, accumulated with v_pk_add_f32
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  f32x2 acc = {0.f, 0.f};
  for (int r = 0; r < rows; ++r) {
    const f32x2 v = in[(long long)r * n + i];
    asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc) : "v"(v));
  }
  out[i] = acc;
}

// Second probe: the victim that IS disturbed (PyTorch's bf16 column sum, not its fp32 one) loads
// 16-bit values; these victims do the same column sums with three load forms.
template <int FORM>
__global__ __launch_bounds__(256) void ld16_victim(const unsigned short* in, float* out, int npairs, int rows) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= npairs) return;
  float a0 = 0.f, a1 = 0.f;
  for (int r = 0; r < rows; ++r) {
    const unsigned short* p = in + ((long long)r * npairs + i) * 2;
    unsigned v = 0x7fc07fc0u;   // the untouched half would show up as NaN
    if (FORM == 0) {            // d16: each load writes one half of the VGPR, the other half kept
      asm volatile("global_load_short_d16 %0, %1, off\n\tglobal_load_short_d16_hi %0, %2, off\n\ts_waitcnt vmcnt(0)"
                   : "+v"(v) : "v"(p), "v"(p + 1) : "memory");
    } else if (FORM == 1) {     // two zero-extending 16-bit loads into separate VGPRs
      unsigned lo, hi;
      asm volatile("global_load_ushort %0, %2, off\n\tglobal_load_ushort %1, %3, off\n\ts_waitcnt vmcnt(0)"
                   : "=&v"(lo), "=&v"(hi) : "v"(p), "v"(p + 1) : "memory");
      v = lo | (hi << 16);
    } else {                    // one 32-bit load of the pair
      asm volatile("global_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    }
    a0 += __builtin_bit_cast(float, v << 16);
    a1 += __builtin_bit_cast(float, v & 0xffff0000u);
  }
  out[2 * i] = a0;
  out[2 * i + 1] = a1;
}

// aggressor variants: LDS-DMA beside scalar VALU instead of MFMA; buffer-form LDS-DMA beside MFMA
extern "C" __global__ __launch_bounds__(256) void dma_valu_loop(const float* src, long long n4, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float ring[4 * 4 * 256];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  float s = 0.f, x = t * 1e-3f, y = 1.0001f;
  for (int it = 0; it < iters; ++it) {
    const int slot = it & 3;
    const long long row = ((long long)(blockIdx.x * 131 + it * 17 + wave) * 64 + lane) % n4;
    glds16(src + row * 4, ring + (slot * 4 + wave) * 256);
    for (int k = 0; k < 32; ++k) { x = fmaf(x, y, 1e-6f); y = fmaf(y, 0.99999f, 1e-7f); }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    s += ring[(slot * 4 + (wave ^ 1)) * 256 + lane * 4];
    __syncthreads();
  }
  out[blockIdx.x * 256 + t] = s + x + y;
}

// host launchers (ctypes): grids sized so aggressor workgroups leave room on every CU for a victim
extern "C" int hz_aggressor(int kind, const float* src, long long n4, float* out, int blocks, int iters,
                            hipStream_t s) {
  switch (kind) {
    case 0: hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, s, out, iters); break;
    case 1: hipLaunchKernelGGL(dma_loop, dim3(blocks), dim3(256), 0, s, src, n4, out, iters); break;
    case 2: hipLaunchKernelGGL(mix_loop, dim3(blocks), dim3(256), 0, s, src, n4, out, iters); break;
    case 3: hipLaunchKernelGGL(valu_loop, dim3(blocks), dim3(256), 0, s, out, iters); break;
    case 4: hipLaunchKernelGGL(dma_valu_loop, dim3(blocks), dim3(256), 0, s, src, n4, out, iters); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}

extern "C" int hz_victim(int kind, const void* in, void* out, int n, int rows, hipStream_t s) {
  const dim3 g((n + 255) / 256), b(256);
  switch (kind) {
    case 0: hipLaunchKernelGGL(pk_victim, g, b, 0, s, (const f32x2*)in, (f32x2*)out, n); break;
    case 1: hipLaunchKernelGGL(fma_victim, g, b, 0, s, (const f32x2*)in, (f32x2*)out, n); break;
    case 2: hipLaunchKernelGGL(pk_add_victim, g, b, 0, s, (const f32x2*)in, (f32x2*)out, n, rows); break;
    case 3: hipLaunchKernelGGL(ld16_victim<0>, g, b, 0, s, (const unsigned short*)in, (float*)out, n, rows); break;
    case 4: hipLaunchKernelGGL(ld16_victim<1>, g, b, 0, s, (const unsigned short*)in, (float*)out, n, rows); break;
    case 5: hipLaunchKernelGGL(ld16_victim<2>, g, b, 0, s, (const unsigned short*)in, (float*)out, n, rows); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}

// Third probe: every disturbed victim so far (PyTorch's reduce_kernel with its semaphore memset,
// rocprim's look-back partition) hands data between workgroups of ONE launch; every clean one
// (our colsum: two launches, the ld16 / pk victims) does not. Column sums of a bf16 [rows][ncols]
// matrix in three forms:
//   lds_colsum  (kind 6): one workgroup per 32 columns, 8 row-threads per column combined through
//               LDS -- an LDS hand-off inside a workgroup, no cross-workgroup traffic;
//   xblk_colsum (kind 7): grid.y row splits, partials to a staging buffer, __threadfence +
//               atomicAdd on a per-column-group semaphore, the last workgroup sums the partials
//               with plain loads (PyTorch's global_reduce / mark_block_finished pattern);
//   kind 8: the same with an agent-scope acquire fence after the semaphore;
//   kind 9: the same with the partials read by agent-scope relaxed atomic loads.
__global__ __launch_bounds__(256) void lds_colsum(const unsigned short* in, float* out, int ncols, int rows) {
  __shared__ float part[8][33];
  const int cx = threadIdx.x & 31, ry = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cx;
  float acc = 0.f;
  if (col < ncols)
    for (int r = ry; r < rows; r += 8) acc += __builtin_bit_cast(float, (unsigned)in[(long long)r * ncols + col] << 16);
  part[ry][cx] = acc;
  __syncthreads();
  if (ry == 0 && col < ncols) {
    float s = 0.f;
    for (int k = 0; k < 8; ++k) s += part[k][cx];
    out[col] = s;
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void xblk_colsum(const unsigned short* in, float* staging, int* sem, float* out,
                                                   int ncols, int rows, int nsplit) {
  const int col = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  const int r0 = (int)((long long)y * rows / nsplit), r1 = (int)((long long)(y + 1) * rows / nsplit);
  float acc = 0.f;
  if (col < ncols)
    for (int r = r0; r < r1; ++r) acc += __builtin_bit_cast(float, (unsigned)in[(long long)r * ncols + col] << 16);
  if (col < ncols) staging[(long long)y * ncols + col] = acc;
  __threadfence();
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(&sem[blockIdx.x], 1) == nsplit - 1;
  __syncthreads();
  if (!last || col >= ncols) return;
  if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  float s = 0.f;
  for (int k = 0; k < nsplit; ++k) {
    float* p = staging + (long long)k * ncols + col;
    s += MODE == 2 ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
  }
  out[col] = s;
}

// PyTorch's own form of that hand-off, as its ROCm reduce_kernel compiles for gfx950 (read from
// the disassembly of libtorch_hip.so's gfx950 code object, at::native::reduce_kernel<128, 4,
// ReduceOp<BFloat16 | float, sum ...>>): partials stored `sc1` (global_store_dwordx2 ... sc1),
// s_waitcnt vmcnt(0), barrier, one lane's returning atomic add on the semaphore, and the last
// workgroup reads the partials with PLAIN global_load_dwordx4 -- no agent-scope acquire between
// the semaphore and those loads (MI355X_MICROARCH.md, inter-workgroup visibility: "no acquire ->
// 24-50 % stale"). kind 10: that form; kind 11: + acquire fence after the semaphore; kind 12: the
// partials read by sc1 loads (agent-scope relaxed atomic loads).
template <int MODE>
__global__ __launch_bounds__(256) void torchform_colsum(const unsigned short* in, float* staging, int* sem, float* out,
                                                        int ncols, int rows, int nsplit) {
  const int col = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
  const int r0 = (int)((long long)y * rows / nsplit), r1 = (int)((long long)(y + 1) * rows / nsplit);
  float acc = 0.f;
  if (col < ncols)
    for (int r = r0; r < r1; ++r) acc += __builtin_bit_cast(float, (unsigned)in[(long long)r * ncols + col] << 16);
  if (col < ncols)
    __hip_atomic_store(staging + (long long)y * ncols + col, acc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(&sem[blockIdx.x], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsplit - 1;
  __syncthreads();
  if (!last || col >= ncols) return;
  if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  float s = 0.f;
  for (int k = 0; k < nsplit; ++k) {
    float* p = staging + (long long)k * ncols + col;
    s += MODE == 2 ? __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *p;
  }
  out[col] = s;
}

extern "C" int hz_victim2(int kind, const void* in, float* staging, int* sem, float* out, int ncols, int rows,
                          int nsplit, hipStream_t s) {
  const dim3 gx((ncols + 255) / 256, nsplit), b(256);
  switch (kind) {
    case 6: hipLaunchKernelGGL(lds_colsum, dim3((ncols + 31) / 32), b, 0, s, (const unsigned short*)in, out, ncols,
                               rows); break;
    case 7: hipLaunchKernelGGL(xblk_colsum<0>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols, rows,
                               nsplit); break;
    case 8: hipLaunchKernelGGL(xblk_colsum<1>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols, rows,
                               nsplit); break;
    case 9: hipLaunchKernelGGL(xblk_colsum<2>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols, rows,
                               nsplit); break;
    case 10: hipLaunchKernelGGL(torchform_colsum<0>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols,
                                rows, nsplit); break;
    case 11: hipLaunchKernelGGL(torchform_colsum<1>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols,
                                rows, nsplit); break;
    case 12: hipLaunchKernelGGL(torchform_colsum<2>, gx, b, 0, s, (const unsigned short*)in, staging, sem, out, ncols,
                                rows, nsplit); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}

// Fourth probe: where does a workgroup run? (CU-masked streams, tools/cu_mask_probe.py) -- the XCC
// id and the HW_ID register (CU / SH / SE fields) of each workgroup, read by s_getreg (a register
// read; nothing is written through the scalar cache).
extern "C" __global__ __launch_bounds__(64) void where_kernel(unsigned* out) {
  unsigned xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hw;
  }
}

extern "C" int hz_where(unsigned* out, int blocks, hipStream_t s) {
  hipLaunchKernelGGL(where_kernel, dim3(blocks), dim3(64), 0, s, out);
  return (int)hipGetLastError();
}

// Fifth probe: the library's own column sum (colsum8: four 16-byte loads in flight per thread) is
// disturbed in the tri-modal step and clean when run alone (tools/stream_repeat.py, TRIAD_ISOLATE).
// Copy victims that only load and store: out = in, 16-byte loads, DEPTH loads in flight per thread
// (kind 13: 1, kind 14: 4, kind 15: 4 with sc1 loads that bypass the CU's L1).
template <int DEPTH, bool SC1>
__global__ __launch_bounds__(256) void copy_victim(const uint4* __restrict__ in, uint4* __restrict__ out, long long n,
                                                   int rows_per_block) {
  const long long stride = (long long)gridDim.x * 256;
  for (long long base = (long long)blockIdx.x * 256 + threadIdx.x; base < n; base += stride * DEPTH) {
    uint4 v[DEPTH];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const long long e = base + d * stride;
      if (e < n) {
        if (SC1) {
          v[d].x = __hip_atomic_load(&in[e].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[d].y = __hip_atomic_load(&in[e].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[d].z = __hip_atomic_load(&in[e].z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          v[d].w = __hip_atomic_load(&in[e].w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
          v[d] = in[e];
        }
      }
    }
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      const long long e = base + d * stride;
      if (e < n) out[e] = v[d];
    }
  }
}

extern "C" int hz_copy(int kind, const void* in, void* out, long long n16, int blocks, hipStream_t s) {
  switch (kind) {
    case 13: hipLaunchKernelGGL((copy_victim<1, false>), dim3(blocks), dim3(256), 0, s, (const uint4*)in, (uint4*)out, n16, 0); break;
    case 14: hipLaunchKernelGGL((copy_victim<4, false>), dim3(blocks), dim3(256), 0, s, (const uint4*)in, (uint4*)out, n16, 0); break;
    case 15: hipLaunchKernelGGL((copy_victim<4, true>), dim3(blocks), dim3(256), 0, s, (const uint4*)in, (uint4*)out, n16, 0); break;
    default: return 1;
  }
  return (int)hipGetLastError();
}

// HuBERT positional convolution (SajayR/TRIAD model.py:29-30,66 -> transformers
// HubertPositionalConvEmbedding: Conv1d(C, C, kernel 128, padding 64, groups 16), weight-
// normalised, its last output dropped by HubertSamePadLayer) as an implicit GEMM over
// channels-last activations, for the forward and the input gradient.
//
//   y[b, t, g*CG + n] = bias[g*CG + n] + sum_{j < KT} sum_{c < CG} x[b, t + j - pad, g*CG + c] * W[g*CG + n, c, j]
//
// for t < T (x zero outside [0, T)). Per (sample, group) this is a GEMM whose A operand is a
// Hankel matrix: with the group's window of x stored compactly in LDS (row w = time
// t0 - pad + w, CG channels, zero-filled), row t of A over k = j*CG + c is the CONTIGUOUS
// slice xwin[(t - t0)*CG + k ...] -- so A fragments are plain ds_read_b128 at k-step offsets
// and no im2col tensor exists. The input gradient is the same GEMM with W flipped along j and
// transposed per group, and pad' = KT - 1 - pad.
//
// Workgroup = (group, sample, 208-row time block); 4 waves; wave w owns the 16-row time tiles
// w, w+4, w+8, w+12 and all CG/16 channel tiles (v_mfma_f32_16x16x32_bf16, fp32 accumulate).
// B fragments (Wt[g][n][k], k contiguous) come from 256-deep chunks of the group's weights staged
// in LDS (two slots, LDS-DMA): blockIdx.x = group, so consecutive workgroups (dealt round-robin
// to the 8 XCDs) put only G/8 groups' weights into each XCD's L2.
#include "common.h"

namespace {

constexpr int KT = 128;       // taps
constexpr int MT = 13;        // 16-row time tiles per workgroup (208 rows >= T = 199 at 4 s)
constexpr int ROWS = MT * 16;
constexpr int NWAVE = 4;
constexpr int MT_PER_WAVE = (MT + NWAVE - 1) / NWAVE;  // 4
constexpr int PC_KC = 256;  // W chunk depth (8 k-steps)

typedef float f32x4_t __attribute__((ext_vector_type(4)));

template <int CG>
__global__ __launch_bounds__(256) void posconv_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wt,
                                                      const float* __restrict__ bias, bf16* __restrict__ y, int T,
                                                      int C, int pad) {
  constexpr int NT = CG / 16;            // channel tiles
  constexpr int KTOT = KT * CG;          // GEMM depth
  constexpr int NKS = KTOT / 32;         // k-steps
  constexpr int WIN = ROWS + KT - 1;     // window rows
  __shared__ __attribute__((aligned(16))) bf16 xwin[WIN * CG];
  __shared__ __attribute__((aligned(16))) bf16 wl[2 * CG * PC_KC];

  const int g = blockIdx.x, b = blockIdx.y, t0 = blockIdx.z * ROWS;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;

  // window: rows w <-> time t0 - pad + w, 16-byte pieces, zero outside [0, T)
  constexpr int PIECES = CG / 8;
  for (int e = threadIdx.x; e < WIN * PIECES; e += 256) {
    const int w = e / PIECES, p = e - w * PIECES;
    const int t = t0 - pad + w;
    bf16x8 v = {};
    if (t >= 0 && t < T) v = *(const bf16x8*)(x + ((size_t)b * T + t) * C + g * CG + p * 8);
    *(bf16x8*)(xwin + w * CG + p * 8) = v;
  }
  __syncthreads();

  const int r = lane & 15, q = lane >> 4;
  // A fragment of time tile m at k-step s: xwin[(16 m + r) * CG + 32 s + 8 q .. +7]
  const bf16* abase = xwin + r * CG + 8 * q;

  f32x4_t acc[MT_PER_WAVE][NT];
#pragma unroll
  for (int i = 0; i < MT_PER_WAVE; ++i)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[i][n] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // W chunks (CG rows x PC_KC k, 512-B rows, 16-B chunk c stored at c ^ (row & 15): each
  // 16-lane group of a ds_read_b128 hits 16 distinct bank slots) stream through two LDS slots
  // by LDS-DMA, one chunk ahead, shared by the four waves (each wave fetching its own B
  // fragments from L2 moved 4x the bytes and ran at ~1/5 of the MFMA rate).
  constexpr int NCH = KTOT / PC_KC, CH_PIECES = CG * PC_KC * 2 / 1024 / NWAVE;  // per wave
  const bf16* wg = wt + (size_t)g * CG * KTOT;
  auto stage = [&](int ch, bf16* dst) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < CH_PIECES; ++u) {
      const int piece = wave * CH_PIECES + u, row = piece * 2 + (lane >> 5), pc = lane & 31;
      glds16(wg + (size_t)row * KTOT + ch * PC_KC + ((pc ^ (row & 15)) << 3), dst + piece * 512);
    }
  };
  stage(0, wl);
  for (int ch = 0; ch < NCH; ++ch) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (ch + 1 < NCH) stage(ch + 1, wl + ((ch + 1) & 1) * CG * PC_KC);
    const bf16* wc = wl + (ch & 1) * CG * PC_KC;
#pragma unroll 2
    for (int ss = 0; ss < PC_KC / 32; ++ss) {
      const int s = ch * (PC_KC / 32) + ss;
      bf16x8 bc[NT];
#pragma unroll
      for (int n = 0; n < NT; ++n) {
        const int row = 16 * n + r, c = 4 * ss + q;
        bc[n] = *(const bf16x8*)(wc + row * PC_KC + ((c ^ (row & 15)) << 3));
      }
#pragma unroll
      for (int i = 0; i < MT_PER_WAVE; ++i) {
        const int m = wave + NWAVE * i;
        if (m < MT) {
          const bf16x8 a = *(const bf16x8*)(abase + m * 16 * CG + s * 32);
#pragma unroll
          for (int n = 0; n < NT; ++n) acc[i][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bc[n], acc[i][n], 0, 0, 0);
        }
      }
    }
  }

  // C/D layout: col = lane & 15, row = 4 * (lane >> 4) + v
#pragma unroll
  for (int i = 0; i < MT_PER_WAVE; ++i) {
    const int m = wave + NWAVE * i;
    if (m >= MT) continue;
#pragma unroll
    for (int n = 0; n < NT; ++n) {
      const int ch = g * CG + n * 16 + r;
      const float bv = bias ? bias[ch] : 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int t = t0 + m * 16 + 4 * q + v;
        if (t < T) y[((size_t)b * T + t) * C + ch] = (bf16)(acc[i][n][v] + bv);
      }
    }
  }
}

// ---- weight gradient ----------------------------------------------------------------------------
// dW[g*CG + n][c][j] = sum_{b, t < T} dy[b, t, g*CG + n] * x[b, t + j - pad, g*CG + c]: per (group,
// tap) a CG x CG GEMM contracted over every (sample, time) row. Workgroup = (group, 16 taps,
// sample range); wave w owns taps j0 + 4w .. + 3 (4 x (CG/16)^2 accumulator tiles of
// v_mfma_f32_16x16x32_bf16). Per (sample, 224-row time block) dy and the x window (224 + 15
// rows, the 16 taps' shifts of each other) are staged in LDS; both operands are k(=time)-major,
// so their fragments are transposed LDS reads (ds_read_b64_tr_b16) and a tap's B fragment is the
// window read one row further down. Partials per sample range: part[s][g][j][n][c] (fp32).
constexpr int DW_TP = 224;   // time rows per block step
constexpr int DW_TAPS = 16;  // taps per workgroup (4 per wave)

template <int CG>
__device__ __forceinline__ bf16x8 dw_frag(const bf16* img, int row0, int col0, int lane) {
  // 8 consecutive rows (row0 + 8 (lane >> 4) ..) of column col0 + (lane & 15)
  const int g = lane & 15, q = lane >> 4;
  const bf16* p = img + (row0 + 8 * q + (g >> 2)) * CG + col0 + 4 * (g & 3);
  const s16x4 lo = lds_tr16(p);
  const s16x4 hi = lds_tr16(p + 4 * CG);
  bf16x8 r;
  s16x4* rp = (s16x4*)&r;
  rp[0] = lo;
  rp[1] = hi;
  return r;
}

template <int CG>
__global__ __launch_bounds__(256, 2) void posconv_dw_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                            int B, int T, int C, int pad, int spb,
                                                            float* __restrict__ part) {
  constexpr int NTL = CG / 16;
  constexpr int XW = DW_TP + DW_TAPS - 1;
  __shared__ __attribute__((aligned(16))) bf16 dyl[DW_TP * CG];
  __shared__ __attribute__((aligned(16))) bf16 xl[XW * CG];
  const int g = blockIdx.x, j0 = blockIdx.y * DW_TAPS, sidx = blockIdx.z;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int G = gridDim.x;

  f32x4_t acc[4][NTL][NTL];
#pragma unroll
  for (int tt = 0; tt < 4; ++tt)
#pragma unroll
    for (int a = 0; a < NTL; ++a)
#pragma unroll
      for (int b = 0; b < NTL; ++b) acc[tt][a][b] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  constexpr int PIECES = CG / 8;
  const int b_lo = sidx * spb, b_hi = min(B, b_lo + spb);
  for (int b = b_lo; b < b_hi; ++b)
    for (int tb = 0; tb < T; tb += DW_TP) {
      __syncthreads();  // previous step's reads done
      for (int e = threadIdx.x; e < DW_TP * PIECES; e += 256) {
        const int w = e / PIECES, p = e - w * PIECES, t = tb + w;
        bf16x8 v = {};
        if (t < T) v = *(const bf16x8*)(dy + ((size_t)b * T + t) * C + g * CG + p * 8);
        *(bf16x8*)(dyl + w * CG + p * 8) = v;
      }
      for (int e = threadIdx.x; e < XW * PIECES; e += 256) {
        const int w = e / PIECES, p = e - w * PIECES, t = tb + w + j0 - pad;
        bf16x8 v = {};
        if (t >= 0 && t < T) v = *(const bf16x8*)(x + ((size_t)b * T + t) * C + g * CG + p * 8);
        *(bf16x8*)(xl + w * CG + p * 8) = v;
      }
      __syncthreads();
      const int nks = (min(DW_TP, T - tb) + 31) / 32;
      for (int ks = 0; ks < nks; ++ks) {
        bf16x8 af[NTL];
#pragma unroll
        for (int a = 0; a < NTL; ++a) af[a] = dw_frag<CG>(dyl, ks * 32, a * 16, lane);
#pragma unroll
        for (int tt = 0; tt < 4; ++tt)
#pragma unroll
          for (int b2 = 0; b2 < NTL; ++b2) {
            const bf16x8 bf = dw_frag<CG>(xl, ks * 32 + wave * 4 + tt, b2 * 16, lane);
#pragma unroll
            for (int a = 0; a < NTL; ++a)
              acc[tt][a][b2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[a], bf, acc[tt][a][b2], 0, 0, 0);
          }
      }
    }

  // C/D layout: col = lane & 15, row = 4 * (lane >> 4) + v
  const int r = lane & 15, q = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) {
    const int j = j0 + wave * 4 + tt;
    float* dst = part + (((size_t)sidx * G + g) * KT + j) * CG * CG;
#pragma unroll
    for (int a = 0; a < NTL; ++a)
#pragma unroll
      for (int b2 = 0; b2 < NTL; ++b2)
#pragma unroll
        for (int v = 0; v < 4; ++v) dst[(a * 16 + 4 * q + v) * CG + b2 * 16 + r] = acc[tt][a][b2][v];
  }
}

}  // namespace

extern "C" {

int triad_posconv(const void* x, const void* wt, const float* bias, void* y, int B, int T, int C, int groups,
                  int pad, hipStream_t stream) {
  if (B <= 0 || T <= 0 || groups <= 0 || C % groups || pad < 0 || pad >= KT) return TRIAD_EINVAL;
  const int cg = C / groups;
  const dim3 grid(groups, B, (T + ROWS - 1) / ROWS);
  if (cg == 48)
    hipLaunchKernelGGL(posconv_kernel<48>, grid, dim3(256), 0, stream, (const bf16*)x, (const bf16*)wt, bias,
                       (bf16*)y, T, C, pad);
  else if (cg == 64)
    hipLaunchKernelGGL(posconv_kernel<64>, grid, dim3(256), 0, stream, (const bf16*)x, (const bf16*)wt, bias,
                       (bf16*)y, T, C, pad);
  else
    return TRIAD_EINVAL;
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

// Weight-gradient partials of the positional conv (C / groups == 48, HuBERT-base):
// part[s][g][j][n][c] (fp32, s < splits) with
// dW[g*CG + n][c][j] = sum_s part[s][g][j][n][c]; samples split into `splits` contiguous ranges.
long long triad_posconv_dw_part_bytes(int C, int groups, int splits) {
  return groups > 0 && C % groups == 0 ? (long long)splits * groups * KT * (C / groups) * (C / groups) * 4 : -1;
}

int triad_posconv_dw(const void* x, const void* dy, int B, int T, int C, int groups, int pad, int splits, float* part,
                     hipStream_t stream) {
  if (B <= 0 || T <= 0 || groups <= 0 || C % groups || pad < 0 || pad >= KT || splits <= 0 || splits > 65535)
    return TRIAD_EINVAL;
  const int cg = C / groups, spb = (B + splits - 1) / splits;
  const dim3 grid(groups, KT / DW_TAPS, splits);
  if (cg != 48) return TRIAD_EINVAL;  // 4 taps x 9 tiles per wave fit the registers at CG = 48 only
  hipLaunchKernelGGL(posconv_dw_kernel<48>, grid, dim3(256), 0, stream, (const bf16*)x, (const bf16*)dy, B, T, C, pad,
                     spb, part);
  TRIAD_CHECK_LAUNCH();
  return TRIAD_OK;
}

}  // extern "C"

/* libtriad_hip.so -- C ABI of the MI355X-native dense tri-modal contrastive hot path.
 *
 * The reference (SajayR/TRIAD @ 2025-06-14) has no FFI: its boundary is the Python
 * method API of src/model.py. Each entry point below replaces one step of that API;
 * the reference file:line it replaces is cited on each declaration. The Python
 * mirror of the reference API (triad_amd/model.py, triad_amd/ops.py) binds these
 * with ctypes; INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *   - every pointer is a device pointer to caller-owned memory (the PyTorch
 *     caching allocator in the Python mirror); no entry point allocates, frees or
 *     synchronises, so all of them are hipGraph-capturable;
 *   - work is enqueued on `stream` (the caller's current HIP stream);
 *   - return 0 on success, TRIAD_EINVAL (1001) on a bad shape/argument, or the
 *     hipError_t of a failed launch;
 *   - bf16 buffers are raw 16-bit bfloat16; "rows" are row-major with 512 features.
 *   - thread-safe when each thread uses its own stream and buffers.
 *
 * Layouts
 *   Q   [R_pad][512] bf16: query tokens of Bq samples flattened, row r = i*Nq + q,
 *       R = Bq*Nq valid rows, R_pad a multiple of 256 (rows >= R zero).
 *   K   [C_alloc][512] bf16: key tokens of Bk samples, sample j at rows
 *       [j*Nk_pad, (j+1)*Nk_pad), Nk_pad a multiple of 32; keys k < Nk_eff are real
 *       (zero rows from patch dropout included), keys >= Nk_eff are padding.
 *       C_alloc >= Bk*Nk_pad, a multiple of 128, rows beyond Bk*Nk_pad zero.
 */
#ifndef TRIAD_HIP_H
#define TRIAD_HIP_H

#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TRIAD_EINVAL 1001

/* Number of per-workgroup partials written by triad_pairsim_fwd / _dS. */
int triad_pairsim_nparts(int R_pad, int Bk);

/* Fused S = temp * Q K^T per (query row, key sample), never materialised:
 * rowmax[j][r] = max_k S, argmax[j][r] = first argmax, nn_part[wg] = partial
 * sum of clamp(S, clamp_lo, 0)^2 (double), diagS[i][q][k] = S on the diagonal
 * pairs (j == i + diag_off) when diag != 0 and diagS != NULL.
 * If dS != NULL it also writes the unit l_nonneg gradient S*[clamp_lo <= S <= 0] divided by
 * su = |temp| (su = 1 when temp == 0) in the tiled dS layout ([R_pad/32][CT][1024] bf16, see
 * triad_tile_gemm) and st_part[wg] = sum S*S/temp over those entries, so the backward needs no
 * recompute (the backward's GEMM alpha carries the factor su).
 * k_len (optional, forward-only: dS and diagS must be NULL): per-key-sample valid length,
 * keys >= k_len[j] are excluded (retrieval over trimmed token lists, retrieval.py:243-244).
 * Replaces model.py:370-392 (AV) / 490-514 (TV) token_sims + max, the
 * l_nonneg reduction of model.py:417-418 / 524-525, and retrieval.py:106-115 / 190-198. */
int triad_pairsim_fwd(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                      int Nk_eff, int D, const float* temp, float clamp_lo, int diag, int diag_off,
                      float* rowmax, int* argmax, double* nn_part, float* diagS, void* dS, long long CT,
                      double* st_part, const int* k_len, hipStream_t stream);

/* One head's forward for triad_pairsim_fwd_multi: the arguments of triad_pairsim_fwd (D = 512,
 * no k_len) as a plain C struct, plus k_tiles (training only; NULL = every tile stored): compact
 * key tiles. A key sample whose last 32-key tile holds only zero vectors (patch dropout's zero
 * padding, model.py:301-302) may leave that tile out: K and the tiled dS then hold sample j's
 * stored tiles at tile rows / columns k_tiles[j] .. k_tiles[j+1] - 1 (k_tiles: Bk + 1 entries, an
 * exclusive prefix sum of nkb or nkb - 1 tiles per sample, nkb = Nk_pad / 32; a sample at index
 * >= 64 within a forward workgroup's key split stores all nkb), CT >= k_tiles[Bk]. The left-out
 * tile's S == 0 enters the row max in closed form. diagS (triad_pairsim_diag) needs the full
 * padded K: give it the problems with the padded K and k_tiles NULL. */
typedef struct triad_pairsim_problem {
  const void* Q;
  const void* K;
  int R, R_pad, Nq, Bq, Bk, Nk_pad, Nk_eff;
  const float* temp;
  float clamp_lo;
  int diag, diag_off;
  float* rowmax;
  int* argmax;
  double* nn_part;
  float* diagS;
  void* dS;
  long long CT;
  double* st_part;
  const int* k_tiles;
} triad_pairsim_problem;

/* The forwards of n (1 or 2) heads as ONE kernel launch over their union of workgroups, each
 * problem with exactly triad_pairsim_fwd's outputs (partial arrays of triad_pairsim_nparts
 * entries each); either every problem writes dS (training) or none does. The tri-modal step's
 * AV and TV heads (model.py:470-472 and 593, one launch for both pair losses: the reference has
 * no audio-text loss, model.py:635-636 is inference only). */
int triad_pairsim_fwd_multi(const triad_pairsim_problem* problems, int n, hipStream_t stream);

/* The diagonal-S part alone (diag_sim over every problem with diag != 0 and diagS != NULL; the
 * regularisers' S blocks, model.py:417-418 / 524-525): triad_pairsim_fwd_multi over problems
 * with diag = 0 followed by this equals triad_pairsim_fwd_multi over the problems as given, bit
 * for bit -- the product path issues the two separately so the forward launch is timed alone. */
int triad_pairsim_diag(const triad_pairsim_problem* problems, int n, hipStream_t stream);

/* clip[i][j] = sum_q m_iq rowmax[j][i*Nq+q] / norm_i (AV: qmask NULL, norm = Nq;
 * TV: norm = max(sum_q m_iq, 1e-7)); qw[r] = d clip / d rowmax (may be NULL).
 * Replaces model.py:389-391 (mean over Na) / 509-512 (masked mean over Nt). */
int triad_clip_reduce(const float* rowmax, int R_pad, int Nq, int Bq, int Bk, const float* qmask, float* clip,
                      float* qw, hipStream_t stream);

/* AV temporal smoothness on the diagonal pairs: part[i] = sum_{q>=1,k} (S[q,k]-S[q-1,k])^2,
 * g = d(sum/cnt)/dS, dt_part[i] = sum g*S. cnt = B_global*(Nq-1)*Nk_eff. Replaces model.py:394-408. */
int triad_diag_smooth(const float* diagS, int Bq, int Nq, int Nk_pad, int Nk_eff, double cnt, double* part,
                      float* g, double* dt_part, hipStream_t stream);

/* TV patch-usage sparsity on the diagonal pairs: part[i], g = d(sum/cnt)/dS, dt_part[i] = sum g*S;
 * cnt = B_global*Nk_eff, Nt <= 1024. Replaces model.py:527-540. */
int triad_diag_sparsity(const float* diagS, int Bq, int Nt, int Nk_pad, int Nk_eff, float thr, double cnt,
                        double* part, float* g, double* dt_part, hipStream_t stream);

/* B x B loss head: symmetric InfoNCE, regulariser combination and similarity
 * statistics (kind 0 = AV, 1 = TV) into out[13]; dclip = d CE / d clip.
 * out: total, ce, reg, 0.01*smooth|sparsity, pos_mean, pos_std, neg_mean, neg_std,
 *      separation, hardest_negative, l_nonneg, l_cal, diag_loss.
 * Replaces model.py:430-472 (AV) / 544-593 (TV) and 410-428 / 516-542's combination. */
int triad_losshead(const float* clip, int B, int kind, const float* temp, const double* nn_part, int n_nn,
                   double n_el, const double* dg_part, int n_dg, double dg_cnt, float w_sparse, float* out,
                   float* dclip, float* lse_scratch, hipStream_t stream);

/* General backward of the fused head (any mix of upstream loss gradients): recompute S, form
 * dS = c_ce*dclip[i][j]*qw[r]*[k==argmax] + c_nn*S*[lo<=S<=0] + c_diag*dSdiag (diag pairs),
 * write it tiled (as triad_pairsim_fwd) and per-workgroup partials of sum(dS * S/temp).
 * coef = {c_ce, c_nn, c_diag, c_cal} (device). Autograd of model.py:384-428 / 502-542. */
int triad_pairsim_dS(const void* Q, const void* K, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad,
                     int Nk_eff, int D, const float* temp, float clamp_lo, int diag, int diag_off,
                     const int* argmax, const float* dclip, const float* qw, const float* dSdiag,
                     const float* coef, void* dS, long long CT, double* dt_part, hipStream_t stream);

/* Fast backward (only `total` differentiated): complete the forward's tiled unit l_nonneg
 * gradient (stored divided by su = |temp|, see triad_pairsim_fwd) in place, in the same units:
 * += ratio_max / su * dclip[i][j] * qw[r] at each row's argmax key (max backward,
 * model.py:389/507) and += ratio_diag / su * gdiag on the diagonal pairs; temp = the forward's
 * temperature (device, required). The GEMMs then take alpha = temp * c_nn * su. max_part[block] =
 * sum dclip*qw*rowmax (n_max_part blocks). */
int triad_dS_patch(void* dS, long long CT, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad, int Nk_eff,
                   int diag_off, const int* argmax, const float* rowmax, const float* dclip, const float* qw,
                   float ratio_max, const float* gdiag, float ratio_diag, double* max_part, int n_max_part,
                   const float* temp, hipStream_t stream);

/* triad_dS_patch over a dS holding only the stored key tiles (k_tiles = the stored-tile prefix sum
 * the forward was given, triad_pairsim_problem.k_tiles; NULL = triad_dS_patch): a term landing in
 * a sample's unstored all-zero last tile is dropped (it multiplies zero keys in dQ, and the keys'
 * own gradient rows are padding); max_part still counts it. Same reference lines as above. */
int triad_dS_patch_tiles(void* dS, long long CT, int R, int R_pad, int Nq, int Bq, int Bk, int Nk_pad, int Nk_eff,
                         int diag_off, const int* argmax, const float* rowmax, const float* dclip, const float* qw,
                         float ratio_max, const float* gdiag, float ratio_diag, double* max_part, int n_max_part,
                         const float* temp, const int* k_tiles, hipStream_t stream);

/* dL/dtemp = sum_k w[k]*sum(p_k) + w[3]*d l_cal/d temp (has_cal: AV, model.py:420-424). */
int triad_dtemp_finalize(const double* p0, int n0, const double* p1, int n1, const double* p2, int n2,
                         const float* temp, const float* w, int has_cal, float* out, hipStream_t stream);

/* dQ / dK of S = temp * Q K^T from the tiled dS (dk = 0: C = alpha * dS K, M = R_pad,
 * nkt = C_pad/32, B = K; dk = 1: C = alpha * dS^T Q, M = CT*32, nkt = R_pad/32, B = Q);
 * C bf16 [M][512]; splits > 1 uses fp32 slabs [splits][M][512]. */
int triad_tile_gemm(const void* Dt, long long CT, int dk, const void* B, int M, int nkt, const float* alpha,
                    int splits, float* slabs, void* C, hipStream_t stream);

/* The same GEMM into unscaled fp32 slabs [splits][M][512] only (no reduction): partial sums the
 * caller reduces with triad_sum_slabs, e.g. dQ over the key-sample chunks of the memory-bounded
 * (recompute) backward. */
int triad_tile_gemm_slabs(const void* Dt, long long CT, int dk, const void* B, int M, int nkt, int splits,
                          float* slabs, hipStream_t stream);

/* Direct-B form of triad_tile_gemm on v_mfma_f32_16x16x32_bf16: B's MFMA fragments pre-arranged
 * once (triad_bfrag_pack16, B [nkt*32][512] bf16 -> Bp of the same size, per dk) so each wave
 * streams its own columns into registers and only dS goes through LDS; faster at the c3 shapes
 * than the workspace-free triad_tile_gemm, results equal to fp32 accumulation order of the tile
 * (reference: the gradients of S = temp Q K^T, SajayR/TRIAD model.py:384-387 / 502-505). */
int triad_bfrag_pack16(const void* B, int nkt, int dk, void* Bp, hipStream_t stream);
int triad_tile_gemm_packed16(const void* Dt, long long CT, int dk, const void* Bp, int M, int nkt, const float* alpha,
                             int splits, float* slabs, void* C, hipStream_t stream);
int triad_tile_gemm_packed16_slabs(const void* Dt, long long CT, int dk, const void* Bp, int M, int nkt, int splits,
                                   float* slabs, hipStream_t stream);

/* C = alpha * op(A) . op(B): A [M][Kd] (a_kcontig=1) or [Kd][M] (0); B [N][Kd] (b_kcontig=1)
 * or [Kd][N] (0); C fp32 or bf16 (out_bf16). M, N multiples of 128, Kd of 64.
 * dQ = temp * dS . K and dK = temp * dS^T . Q of S = temp * Q K^T (model.py:387/505),
 * and the projection-head GEMMs (model.py:68/116/326). */
int triad_gemm_bf16(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                    int M, int N, int Kd, const float* alpha, void* C, long long ldc, int out_bf16,
                    hipStream_t stream);

/* C = op(A) . op(B) (+ bias[n], fp32, added before the single bf16 rounding), bf16 out, tile form
 * chosen from the shape: the backbone projections (F.linear / its input gradient under autocast)
 * without a vendor BLAS. M, N multiples of 128, Kd of 64; bias may be NULL. */
int triad_gemm_bf16_bias(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                         int M, int N, int Kd, const float* bias, void* C, long long ldc, hipStream_t stream);

/* triad_gemm_bf16_bias with the bias as the bf16 vector of the autocast model (what F.linear
 * under autocast adds, widened to fp32 in the epilogue): bit-identical to passing its fp32
 * widening, without that copy per call (model.py:68/116/326 heads, the backbone Linear layers). */
int triad_gemm_bf16_bias_bf16(const void* A, long long lda, int a_kcontig, const void* B, long long ldb,
                              int b_kcontig, int M, int N, int Kd, const void* bias, void* C, long long ldc,
                              hipStream_t stream);

/* Split-K GEMM (weight gradients of the projection heads, train.py:987 backward):
 * `splits` fp32 partial slabs [splits][M][N] in caller-owned `slabs`, then C = alpha * sum. */
int triad_gemm_bf16_splitk(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                           int M, int N, int Kd, int splits, const float* alpha, float* slabs, void* C,
                           int out_bf16, hipStream_t stream);

/* triad_gemm_bf16_splitk in an explicit tile form (1-4 as triad_gemm_bf16_form; 0 = the size
 * policy): the backbone weight gradients at >= 32,768 tokens run the eight-wave 256 x 256 form
 * with their own split counts (triad_amd/linear.py). form + 8: the workgroups of one split all on
 * one XCD (each split's token slab fetched into one L2 once; splits % 8 == 0, else TRIAD_EINVAL). */
int triad_gemm_bf16_splitk_form(const void* A, long long lda, int a_kcontig, const void* B, long long ldb,
                                int b_kcontig, int M, int N, int Kd, int splits, const float* alpha, float* slabs,
                                void* C, int out_bf16, int form, hipStream_t stream);

/* triad_gemm_bf16 in an explicit tile form, a per-call argument (there is no process-wide GEMM
 * state): 0 = size policy (what triad_gemm_bf16 uses), 1 = 128 x 128 tiles, 2 = 256 x 128 LDS ring,
 * 4 = 256 x 256 eight-wave tiles (3, the retired four-wave tile, runs as 4; M, N multiples of 256). */
int triad_gemm_bf16_form(const void* A, long long lda, int a_kcontig, const void* B, long long ldb, int b_kcontig,
                         int M, int N, int Kd, const float* alpha, void* C, long long ldc, int out_bf16, int form,
                         hipStream_t stream);

/* Projection head on row-panel GEMMs (model.py:32-34,68 / 81-83,116 / 253-255,326 under bf16
 * autocast; csrc/rowgemm.hip): a workgroup owns 128 token rows x all 512 columns, so the LayerNorm
 * and its backward run in the GEMM epilogues. Weights are pre-arranged in MFMA-fragment order:
 * triad_wpack(W, K, Bp) for C = A W^T with W [512][K] bf16 (Bp: K * 512 bf16); triad_wpack2 packs
 * both weights of a head in one launch. Outputs have triad_rowpanel_count(M) * 128 rows (rows >= M
 * written as zeros).
 *   projhead_fwd: the whole forward in one kernel -- y1 = bf16(h W1^T + b1), mean / rstd (fp32,
 *           biased variance + eps) of y1's rows, ln = bf16((y1 - mean) rstd gamma + beta), kept in
 *           LDS as the A operand of y = bf16(ln W2^T + b2); y1 / ln / mean / rstd are stored for the
 *           backward. h row r at h + (r / n_per) * bstride + (r % n_per) * lda (a strided view read
 *           in place). Bit-identical to ln_fwd followed by rowgemm_bias;
 *   ln_fwd: its first half (y1, mean / rstd, ln);
 *   rowgemm_bias: C = bf16(A W^T + bias) (projection2 from ln in HBM);
 *   ln_bwd: dln = bf16(dy W2) (W2p = triad_bfrag_pack16(W2, 16, 1, .)), dy1 = bf16(rstd (g -
 *           mean(g) - xh mean(g xh))), g = dln gamma, and part [panels][3][512] column sums of
 *           dln xh (dgamma), dln (dbeta), dy1 (db1) per panel (reduce with triad_sum_slabs).
 * Biases are the bf16 vectors autocast adds (b1, b2, bias: bf16 [512]); gamma / beta fp32. */
int triad_wpack(const void* W, int K, void* Bp, hipStream_t stream);
int triad_wpack2(const void* W1, int K1, void* Bp1, const void* W2, int K2, void* Bp2, hipStream_t stream);
int triad_rowpanel_count(long long M);
int triad_projhead_fwd(const void* h, long long M, int H, long long lda, long long n_per, long long bstride,
                       const void* W1p, const void* b1, const float* gamma, const float* beta, float eps,
                       const void* W2p, const void* b2, void* y1, void* ln, float* mean, float* rstd, void* y,
                       hipStream_t stream);
int triad_projhead_ln_fwd(const void* h, long long M, int H, long long lda, long long n_per, long long bstride,
                          const void* W1p, const void* b1, const float* gamma, const float* beta, float eps, void* y1,
                          void* ln, float* mean, float* rstd, hipStream_t stream);
int triad_rowgemm_bias(const void* A, long long M, int K, long long lda, const void* Bp, const void* bias, void* C,
                       hipStream_t stream);
int triad_projhead_ln_bwd(const void* dy, long long M, const void* W2p, const void* y1, const float* mean,
                          const float* rstd, const float* gamma, void* dy1, float* part, hipStream_t stream);

/* Inference similarity maps (model.py:355-368 compute_similarity_matrix; forward() 630-636,
 * viz.py:182): sim[b][i][j] = temp * <f1[b][i] / max(||f1[b][i]||, eps), f2[b][j] / max(||f2[b][j]||,
 * eps)>, f1 (B, N1, D), f2 (B, N2, D) contiguous bf16 16-byte aligned, D % 32 == 0, D <= 512, temp
 * a device scalar, sim (B, N1, N2) fp32 16-byte aligned. One launch over all samples: a workgroup
 * normalises 64 f1 rows and, block by block, 64 f2 rows into LDS (operands rounded to bf16 after
 * it, as F.normalize returns bf16) and applies the temperature in the epilogue. */
int triad_similarity_maps(const void* f1, const void* f2, int B, int N1, int N2, int D, const float* temp, float eps,
                          float* sim, hipStream_t stream);

/* LayerNorm(512) forward of the library-GEMM projection head (model.py:68/116/326 under
 * autocast): ln = bf16((y1 - mean) rstd gamma + beta) over bf16 y1 [M][512], fp32 statistics
 * (biased variance, eps) kept in mean / rstd [M]. */
int triad_ln_fwd(const void* y1, int M, const float* gamma, const float* beta, float eps, void* ln, float* mean,
                 float* rstd, hipStream_t stream);

/* Its backward from a bf16 dln: dy1 (bf16) and per-block column partials [nblocks][3][512] of
 * dgamma, dbeta, db1 (= column sums of dy1), reduced by triad_sum_slabs. */
int triad_ln_bwd3(const void* dln, const void* y1, const float* mean, const float* rstd, const float* gamma, int M,
                  void* dy1, float* part, int nblocks, hipStream_t stream);

/* out[c] = alpha * sum_r X[r][c] over bf16 X [rows][ld] (cols % 8 == 0), fp32 or bf16 out, at HBM rate:
 * row slices x 8-column 16-byte loads, partials in part (triad_colsum_splits(rows, cols) * cols floats). */
int triad_colsum_splits(long long rows, int cols);
int triad_colsum(const void* X, long long rows, int cols, long long ld, float* part, float alpha, int out_bf16,
                 void* out, hipStream_t stream);

/* The same column sums with the rows staged by 16-byte LDS-DMA (cols % 8 == 0, X 16-byte aligned;
 * the last 256-column tile masked): the form EVERY column sum of the step uses -- the bias
 * gradients of the heads and backbones, SpecAugment's masked_spec_embed (beside concurrent
 * streams' GEMMs, plain-load column sums returned disturbed values; reference:
 * autograd's bias gradients of model.py:32-34 / 81-83 / 253-255 and the backbones' Linear layers).
 * part: triad_colsum_dma_splits(rows, cols) * cols floats. */
int triad_colsum_dma_splits(long long rows, int cols);
int triad_colsum_dma(const void* X, long long rows, int cols, long long ld, float* part, float alpha, int out_bf16,
                     void* out, hipStream_t stream);

/* out[e] = alpha * sum_i slabs[i][e] (alpha may be NULL = 1), fp32 or bf16 out. */
int triad_sum_slabs(const float* slabs, int nslab, long long n, const float* alpha, int out_bf16, void* out,
                    hipStream_t stream);

/* x <- (x - mean) / sqrt(var + eps) over ALL n elements (population variance), fp32:
 * the Wav2Vec2/HuBERT processor normalisation of model.py:56-62 done on the device.
 * part: >= 2*nblocks doubles of scratch. */
int triad_global_znorm(const float* x, long long n, float eps, float* y, double* part, int nblocks,
                       hipStream_t stream);

/* Fused optimizer over flat fp32 buffers (train.py:990-1041; replaces the four
 * torch.optim.AdamW.step calls of train.py:1010-1040 and the norm/clip loops of 992-1006).
 * `chunks` is a device array of {int64 off; int32 n; int32 param} slices.
 * triad_grad_sumsq: out[c] = sum g^2 over chunk c (grad norms train.py:992-1002,
 * clip_grad_norm_ train.py:1004-1006).
 * triad_adamw_step: torch.optim.AdamW (decoupled weight decay) with g scaled by scale[param]
 * (the clip factor, NULL = 1); pp[3*param] = {lr/bc1, 1/sqrt(bc2), 1 - lr*wd}; omb1 / omb2 =
 * 1 - beta1 / 1 - beta2 rounded from double, as torch passes them (1 - float(beta2) loses 1.3e-5
 * of 1 - 0.999 to cancellation). shadow (may be
 * NULL): per parameter, (address of its bf16 model weight) - 2 * (flat offset), or 0; the step
 * then also writes bf16(p) there (mixed-precision model weights, the cast autocast would do).
 * triad_gather_grads: pieces = device array of {const void* src; int64 dst; int32 n; int32 f32};
 * g[dst + i] (+)= float(src[i]), src bf16 (f32 == 0) or fp32 (f32 == 1) -- the autograd
 * gradients of every flat-space parameter into the flat fp32 gradient buffer. */
int triad_grad_sumsq(const float* g, const void* chunks, int nchunks, double* out, hipStream_t stream);
int triad_adamw_step(float* p, const float* g, float* m, float* v, const void* chunks, int nchunks,
                     const float* pp, const float* scale, float beta1, float beta2, float omb1, float omb2,
                     float eps, const unsigned long long* shadow, hipStream_t stream);
int triad_gather_grads(const void* pieces, int npieces, float* g, int accumulate, hipStream_t stream);

/* dst[b][t] = idx[b][t] >= 0 ? src[b][idx[b][t]] : 0 (row_bytes per row). Patch-dropout
 * compaction with zero padding (model.py:282-307) and its backward scatter. */
int triad_gather_rows(const void* src, long long src_rows, const int* idx, int B, int M, int row_bytes, void* dst,
                      hipStream_t stream);

/* y = x / max(||x||_2, eps) per row, bf16 (F.normalize, model.py:363-364). */
int triad_l2norm_rows(const void* x, int rows, int D, float eps, void* y, hipStream_t stream);

/* Reference-precision retrieval (retrieval.py:106-114 aggregator_av_a2v / _v2a, the per-pair
 * `matmul(q, k.t()) / temperature -> max over the item's tokens -> mean` of its N^2 double loop,
 * retrieval.py:161-174 / 255-264), every pair in one launch, fp32 throughout:
 * sim[i][j] = mean_{q < qlen[i]} max_{k < klen[j]} <Q[i][q], K[j][k]> / temp, Q (Bq, nq_pad, D) and
 * K (Bk, nk_pad, D) contiguous fp32 16-byte aligned, zero-padded token lists (nq_pad, nk_pad
 * multiples of 64, D % 32 == 0), qlen / klen device int32, sim (Bq, Bk) fp32. For fp32
 * embeddings (model.use_amp == False, as the reference's retrieval embeds); the bf16 product
 * path is triad_pairsim_fwd + triad_clip_reduce. */
int triad_retrieval_maxmean_f32(const float* Q, const int* qlen, int Bq, int nq_pad, const float* K, const int* klen,
                                int Bk, int nk_pad, int D, float temp, float* sim, hipStream_t stream);

/* y = x / max(||x||_2, eps) per row, fp32 (F.normalize of the reference's fp32 retrieval embeddings,
 * retrieval.py:93-94); x, y 16-byte aligned, D % 4 == 0. */
int triad_l2norm_rows_f32(const float* x, int rows, int D, float eps, float* y, hipStream_t stream);

/* Audio front-end (model.py:29-30,66: the HuBERT conv feature encoder's layer 0,
 * transformers HubertGroupNormConvLayer = conv -> GroupNorm(C groups) -> GELU), fused
 * GroupNorm + exact GELU over channels-last x[B][Tp][C] bf16 (C % 8 == 0, 256 % (C/8) == 0); the
 * first T frames of each sample are valid, frames T .. Tp-1 padding (outputs written as 0).
 * fwd: y = bf16(gelu((x - mean[b][c]) * rstd[b][c] * gamma[c] + beta[c])), statistics over t < T
 *      in fp32/fp64, mean / rstd (B*C floats) saved for the backward.
 * bwd: dx (bf16) and dgamma / dbeta (C floats, overwritten) from dy (bf16).
 * ws: triad_chgn_workspace_bytes(B, T, C) bytes of scratch. */
long long triad_chgn_workspace_bytes(int B, int T, int C);
int triad_chgn_gelu_fwd(const void* x, int B, int T, int Tp, int C, const float* gamma, const float* beta,
                        float eps, float* mean, float* rstd, void* ws, void* y, hipStream_t stream);
int triad_chgn_gelu_bwd(const void* x, const void* dy, int B, int T, int Tp, int C, const float* gamma,
                        const float* beta, const float* mean, const float* rstd, void* ws, void* dx, float* dgamma,
                        float* dbeta, hipStream_t stream);

/* HuBERT conv layer 0 (1 -> C, kernel 10, stride 5, no bias) + GroupNorm(C groups) + GELU forward with
 * conv0 recomputed from the bf16 waveform wave[b][Lp] (Lp >= 5 (Tp - 1) + 10) in both passes; writes the
 * padded frame buffers out = bf16(gelu(gn(y0))) and y0out = y0 (frames T .. Tp-1 zero) and mean / rstd;
 * the backward is triad_chgn_gelu_bwd over y0out. ws: triad_chgn_workspace_bytes(B, T, C) bytes. */
int triad_c0gn_fwd(const void* wave, long long Lp, const void* w0, int B, int T, int Tp, int C, const float* gamma,
                   const float* beta, float eps, float* mean, float* rstd, void* ws, void* out, void* y0out,
                   hipStream_t stream);

/* conv0's weight gradient dw0[c][j] (fp32) = sum_{b, t < T} dy0[b*Tp + t][c] * wave[b][5t + j] (bf16 inputs);
 * ws: triad_conv0_dw_workspace_bytes(B, T, C) bytes. */
long long triad_conv0_dw_workspace_bytes(int B, int T, int C);
int triad_conv0_dw(const void* wave, long long Lp, const void* dy0, int B, int T, int Tp, int C, void* ws, float* dw0,
                   hipStream_t stream);

/* HuBERT positional convolution (model.py:29-30,66: transformers HubertPositionalConvEmbedding,
 * Conv1d(C, C, 128, padding 64, groups) + SamePad) as an implicit GEMM over channels-last bf16:
 * y[b][t][g*CG+n] = bias + sum_{j<128, c<CG} x[b][t+j-pad][g*CG+c] * wt[g][n][j*CG+c], t < T,
 * x zero outside [0, T); CG = C/groups in {48, 64}; bias f32 (may be NULL).
 * Forward: wt[g][n][j*CG+c] = W[g*CG+n][c][j], pad = 64. Input gradient: x = dy,
 * wt[g][c][j*CG+n] = W[g*CG+n][c][127-j], pad = 63. */
int triad_posconv(const void* x, const void* wt, const float* bias, void* y, int B, int T, int C, int groups,
                  int pad, hipStream_t stream);

/* Weight gradient of the same conv (C / groups == 48): fp32 partials part[s][g][j][n][c] over
 * `splits` contiguous sample ranges, dW[g*48 + n][c][j] = sum_s part[...]; part holds
 * triad_posconv_dw_part_bytes(C, groups, splits) bytes. Replaces aten's grouped-conv weight
 * gradient (transformers HubertPositionalConvEmbedding backward). */
long long triad_posconv_dw_part_bytes(int C, int groups, int splits);
int triad_posconv_dw(const void* x, const void* dy, int B, int T, int C, int groups, int pad, int splits, float* part,
                     hipStream_t stream);

/* Backbone self-attention (the DINOv2 / HuBERT / DistilBERT encoders of model.py:29-30,79-80,
 * 218-227; no dropout, no mask): O = softmax(Q K^T * scale) V per (sample, head), head dim D = 64,
 * N <= 320. Tensors are (B, N, H, 64) bf16 in memory with the head dim contiguous: element
 * (b, n, h, c) at b*sB + n*sN + h*64 + c. lse: [B*H][N] f32 log-sum-exp (forward output, backward
 * input); delta: [B*H][N] f32 scratch. */
int triad_attn_fwd(const void* q, long long q_sB, long long q_sN, const void* k, long long k_sB, long long k_sN,
                   const void* v, long long v_sB, long long v_sN, int B, int H, int N, int D, float scale, void* out,
                   long long out_sB, long long out_sN, float* lse, hipStream_t stream);
int triad_attn_bwd(const void* q, long long q_sB, long long q_sN, const void* k, long long k_sB, long long k_sN,
                   const void* v, long long v_sB, long long v_sN, const void* o, long long o_sB, long long o_sN,
                   const void* dout, long long do_sB, long long do_sN, const float* lse, int B, int H, int N, int D,
                   float scale, void* dq, long long dq_sB, long long dq_sN, void* dk, long long dk_sB,
                   long long dk_sN, void* dv, long long dv_sB, long long dv_sN, float* delta, hipStream_t stream);
/* Attention-probability dropout (HuBERT / DistilBERT attention_dropout, transformers' sdpa path):
 * O = (softmax(Q K^T scale) * keep / (1 - p)) V, lse of the undropped scores. Keep bits from the
 * common.h hash of element (bh N + q) N + key, stored by triad_attn_dropmask in two layouts of
 * ceil(N/32) words per row: wq[(bh N + q) nkt + kt] (bit j = key 32 kt + j) and wk[(bh N + key) nkt + qt]
 * (bit j = query 32 qt + j); B*H*N*nkt u32 each. NULL masks = no dropout. */
int triad_attn_dropmask(int B, int H, int N, float p, unsigned seed, unsigned* wq, unsigned* wk, hipStream_t stream);
int triad_attn_fwd_dropout(const void* q, long long q_sB, long long q_sN, const void* k, long long k_sB,
                           long long k_sN, const void* v, long long v_sB, long long v_sN, int B, int H, int N, int D,
                           float scale, const unsigned* wq, float p, void* out, long long out_sB, long long out_sN,
                           float* lse, hipStream_t stream);
int triad_attn_bwd_dropout(const void* q, long long q_sB, long long q_sN, const void* k, long long k_sB,
                           long long k_sN, const void* v, long long v_sB, long long v_sN, const void* o,
                           long long o_sB, long long o_sN, const void* dout, long long do_sB, long long do_sN,
                           const float* lse, int B, int H, int N, int D, float scale, const unsigned* wq,
                           const unsigned* wk, float p, void* dq, long long dq_sB, long long dq_sN, void* dk,
                           long long dk_sB, long long dk_sN, void* dv, long long dv_sB, long long dv_sN, float* delta,
                           hipStream_t stream);

/* LoRA skinny products (model.py:223-266, peft LoRA r = 8 on the ViT's attn.qkv / attn.proj):
 * triad_rows_nt: out[m][j] = sum_k X[m][k] * W[j][k], X [M][ldx] bf16, W [J][K] bf16, J <= 16,
 *                K % 32 == 0, out [M][J] bf16 (t = x A^T).
 */
int triad_rows_nt(const void* X, long long ldx, int M, int K, const void* W, int J, void* out, hipStream_t stream);
/* triad_lora_update: Y[m][o] += sum_j T[m][j] Bs[o][j] in place (Y [M][ldy] bf16, T [M][8], Bs [O][8] bf16;
 *                    y += t (sB)^T after the base GEMM, dx += dt A in the backward).
 * triad_lora_tn:     out[o][j] = alpha sum_m Y[m][o] T[m][j] (f32 [O][8]) and, if Wt != NULL,
 *                    dt[m][j] = sum_o Y[m][o] Wt[j][o] (Wt [16][O] bf16, rows 8..15 zero; dt [M][8] bf16),
 *                    in ONE pass over Y; O / 256 in {1,2,3,4,6,8,9,12}; slabs: triad_lora_tn_blocks(M) * O * 8. */
int triad_lora_update(void* Y, long long ldy, int M, int O, const void* T, const void* Bs, hipStream_t stream);
int triad_lora_tn_blocks(int M);
int triad_lora_tn(const void* Y, long long ldy, int M, int O, const void* T, const void* Wt, void* dt, float alpha,
                  float* slabs, float* out, hipStream_t stream);

/* ViT residual + LayerScale + LayerNorm (model.py:207-266, DINOv2 blocks; csrc/resid_ln.hip):
 * triad_addln_fwd: xn = x + g * y (y bf16, may be NULL: LN of x alone, xn not written), ln = LN(xn) w + b
 *                  as bf16 (out_f32 = 0) or fp32, per-row mean / rstd; x, xn, w, b, g fp32; D % 256 == 0.
 * triad_addln_bwd: dx = dres (may be NULL) + LN backward of dln (bf16 / fp32) at xn, dy = bf16(g dx). */
int triad_addln_fwd(const float* x, const void* y, const float* g, const float* w, const float* b, float eps, int M,
                    int D, float* xn, void* ln, int out_f32, float* mean, float* rstd, hipStream_t stream);
int triad_addln_bwd(const void* dln, int dln_f32, const float* dres, const float* xn, const float* mean,
                    const float* rstd, const float* w, const float* g, int M, int D, float* dx, void* dy,
                    hipStream_t stream);

/* HuBERT post-LN layer passes (transformers HubertEncoderLayer under bf16 autocast; csrc/postln.hip).
 * Dropout keep bits: counter hash of (seed, element pair), keep iff 16-bit uniform >= round(p * 65536).
 * triad_dropaddln_fwd: h = LN(res + bf16(y keep / (1-p))) fp32 and hb = bf16(h), mean / rstd per row (D % 256 == 0).
 * triad_dropaddln_bwd: dres = LN'(dh + dhb) (either NULL), dy = bf16(bf16(dres) keep / (1-p)); part:
 *                      triad_dropaddln_bwd_blocks(M) x 2 x D fp32 dgamma / dbeta partials.
 * triad_geludrop_fwd / _bwd: v = bf16(bf16(gelu(u)) keep / (1-p)) over n bf16 (n % 8 == 0) and its gradient.
 * triad_dropout_keep: the keep bits (u8) for n elements (tests). */
int triad_dropaddln_fwd(const float* res, const void* y, const float* w, const float* b, float eps, int M, int D,
                        float p, unsigned seed, float* h, void* hb, float* mean, float* rstd, hipStream_t stream);
int triad_dropaddln_bwd_blocks(int M);
int triad_dropaddln_bwd(const float* dh, const void* dhb, const float* res, const void* y, const float* mean,
                        const float* rstd, const float* w, int M, int D, float p, unsigned seed, float* dres, void* dy,
                        float* part, hipStream_t stream);
/* GELU table for the two passes below: triad_gelu_table_bytes() bytes of device memory built once by
 * triad_gelu_table (value and slope of every bf16 argument with |x| in [2^-40, 2^6)); table = NULL
 * makes the passes evaluate the formula. */
long long triad_gelu_table_bytes(void);
int triad_gelu_table(void* table, hipStream_t stream);
int triad_geludrop_fwd(const void* u, long long n, float p, unsigned seed, const void* table, void* v,
                       hipStream_t stream);
int triad_geludrop_bwd(const void* u, const void* dv, long long n, float p, unsigned seed, const void* table, void* du,
                       hipStream_t stream);
int triad_dropout_keep(long long n, float p, unsigned seed, void* out, hipStream_t stream);

/* Materialising debug path (csrc/dense.hip; SURVEY §8b keeps the reference's small-B methods):
 * S = token similarities fp32 (Bq, Bk, Nq, Nk) as model.py:384-387 / 502-505 return them.
 * triad_dense_nparts(n): number of per-block partials the reductions below write for n elements.
 * triad_dense_rowmax: rowmax[j][i*Nq+q] = max_k S, argmax = first max index (model.py:389 / 507);
 *                     feeds triad_clip_reduce for clip (model.py:391 / 509-512).
 * triad_nonneg_fwd:   part[b] = sum clamp(S, lo, 0)^2 (model.py:417-418 / 524-525).
 * triad_nonneg_bwd:   dS = coef[0] * scale * 2 clamp(S, lo, 0) [lo <= S <= 0] (coef may be NULL = 1).
 * triad_sims_bwd_pack: G = dtok (may be NULL) + [k == argmax] dclip[i][j] qw[r] (dclip may be NULL) as the
 *                     bf16 GEMM operand A[i*Nq+q][j*Nk+k] (row stride lda, caller zeroes the padding) and
 *                     part[b] = sum G * S / temp; dQ / dK are then two triad_gemm_bf16 calls.
 * triad_sum_parts:    out[0] = scale * sum part (float). */
int triad_dense_nparts(long long n);
int triad_dense_rowmax(const float* S, int Bq, int Bk, int Nq, int Nk, int R_pad, float* rowmax, int* argmax,
                       hipStream_t stream);
int triad_nonneg_fwd(const float* S, long long n, float lo, double* part, hipStream_t stream);
int triad_nonneg_bwd(const float* S, long long n, float lo, float scale, const float* coef, float* dS,
                     hipStream_t stream);
int triad_sims_bwd_pack(const float* S, const float* dtok, const float* dclip, const float* qw, const int* argmax,
                        int Bq, int Bk, int Nq, int Nk, int R_pad, const float* temp, void* A, long long lda,
                        double* part, hipStream_t stream);
int triad_sum_parts(const double* part, int n, double scale, float* out, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* TRIAD_HIP_H */

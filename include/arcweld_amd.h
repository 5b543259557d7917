/* arcweld_amd.h -- C ABI of the MI355X (gfx950) HIP kernels behind the VQ-VAE + Transformer training path.
 *
 * The reference (tmdt-buw/VQ-VAE-Transformer-Arc-Welding) is pure Python on stock PyTorch ops; it has no FFI.
 * Its drop-in boundary is the nn.Module surface.  This library sits BELOW that
 * surface: each entry point replaces the ATen work of one reference call site, cited per function.
 *
 * Conventions (all entry points):
 *   - plain device pointers + sizes/leading dimensions (in elements); caller owns every buffer;
 *   - `stream` is a hipStream_t passed as void*; nothing synchronises the host;
 *   - return 0 (AW_OK) or a negative status; aw_last_error() returns a thread-local message;
 *   - no allocation inside (graph-capture safe); accumulators that must start at zero are documented.
 */
#ifndef ARCWELD_AMD_H
#define ARCWELD_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { AW_OK = 0, AW_ERR_ARG = -1, AW_ERR_LAUNCH = -2 };
enum { AW_F32 = 0, AW_BF16 = 1 };
/* act: the activation of C2 modes 1 / 4 and of the epilogue's act'; AW_ACT_DERIV (with pre): pre already holds the
 * activation's derivative (saved by a c2_mode 4 forward), the epilogue multiplies by it as it is */
enum { AW_ACT_GELU_ERF = 0, AW_ACT_GELU_TANH = 1, AW_ACT_DERIV = 2 };

const char* aw_last_error(void);
int aw_version(void);

/* ------------------------------------------------------------------------------------------------ GEMM
 * C[M,N] = epilogue( alpha * op(A)[M,K] . op(B)[K,N] )  on MFMA (bf16 16x16x32 or exact-f32 16x16x4).
 * Replaces every conv1d / conv_transpose1d / addmm / mm of the hot path (SURVEY.md section 2 ATen table):
 *   model/vq_vae_patch_embedd.py:11,27,30,65,68,81,87,143 and model/transformer_block.py:30,32,78-79,
 *   model/transformer_decoder.py:29 -- forward, input-gradient and weight-gradient forms.
 * Operand storage (dtype = a_dtype for A and B; AW_F32 or AW_BF16):
 *   a_trans = 0: A[m*lda + k]        a_trans = 1: A[k*lda + m]
 *   b_trans = 0: B[n*ldb + k]        b_trans = 1: B[k*ldb + n]      (weights [out][in] are b_trans = 0)
 *   A transposed operand whose width (M or N) is not a multiple of 16 bytes but whose leading dimension is at
 *   least that width rounded up is read in whole 16-B chunks: every row, the last included, must be readable up
 *   to the rounded width (the padding values are never used).
 * Implicit k=3/pad=1 convolution along windows of `conv_seg` rows (conv_cin > 0):
 *   conv_operand = 0 (A, a_trans = 0): K = 3*conv_cin, A[m][j*cin+i] = src[(m + conv_dir*(j-1))*lda + i],
 *                  zero where the shifted row leaves its window;
 *   conv_operand = 1 (B, b_trans = 1): N = 3*conv_cin, B[k][j*cin+i] = src[(k + (j-1))*ldb + i], same mask.
 * Epilogue, per element (row r, col c), in this order:
 *   v = alpha*acc;  v += bias[c] (bias[c % bias_mod] if bias_mod > 0);  v *= act'(pre[r*ld_pre + c]) (pre f32/bf16);  v *= dropout(drop_seed, r*N+c, drop_p);
 *   v += resid[r*ld_resid + c] (resid f32/bf16);  v += beta * C_old (C must be f32 when beta != 0);  C[r*ldc + c] = v (c_dtype)
 *   C2 (c2_mode): 1 = act(v), 2 = v, 3 = v * dropout(drop2_seed, r*N+c, drop2_p); stored as c2_dtype;
 *   c2_mode 4: C = act(v) and C2 = act'(v) instead (from one exponential: the backward multiplies by the saved
 *   derivative, act = AW_ACT_DERIV, rather than evaluating act' of a saved pre-activation)
 *   colstats (f64, 2*stats_mod): += v and v*v into slot (c % stats_mod)      (BatchNorm batch statistics)
 *   a_rowsum (f32, M): += sum_k A[m][k]                                      (bias gradients, fused)
 */
typedef struct {
  int M, N, K;
  int a_dtype;
  const void* A; int64_t lda; int a_trans;
  const void* B; int64_t ldb; int b_trans;
  int conv_cin, conv_seg, conv_dir, conv_operand;
  float alpha, beta;
  const float* bias;
  int act;                       /* AW_ACT_GELU_ERF / _TANH (act' and C2 modes 1, 4) or AW_ACT_DERIV (pre = act') */
  const float* pre; int64_t ld_pre;
  const float* resid; int64_t ld_resid;
  float drop_p; uint64_t drop_seed;
  void* C; int64_t ldc; int c_dtype;
  void* C2; int64_t ldc2; int c2_mode; int c2_dtype;
  float drop2_p; uint64_t drop2_seed;
  double* colstats; int stats_mod;
  float* a_rowsum;
  int bias_mod;                  /* > 0: bias index is c % bias_mod (ConvT bias shared by the k taps) */
  /* accumulate = 1: C[r*ldc + colmap(c)] += alpha*acc with f32 atomics (split-K allowed; no other epilogue
   * field may be set).  colmap(c) = (c % col_mod)*col_mul + c/col_mod + col_off  (col_mod > 0)
   *                              =  c*col_mul + col_off                          (col_mod == 0)
   * so weight gradients land directly in the reference layouts (conv (O,I,3) taps, ConvT (I,O,k)). */
  int accumulate, col_mod, col_mul, col_off;
  /* seed_ptr != NULL: the dropout seeds become mix(drop_seed, *seed_ptr) and mix(drop2_seed, *seed_ptr), with
   * *seed_ptr read on the device (a per-step counter, so one captured HIP graph replays with fresh masks). */
  const uint64_t* seed_ptr;
  /* dtype of `pre` (AW_F32 or AW_BF16): bf16-mode forwards keep the GELU pre-activations in the operand dtype */
  int pre_dtype;
  /* epilogue store policy for C / C2: AW_STORE_NT (0, non-temporal; the lines stay in the XCD's L2 until the
   * end-of-kernel release writes them back) or AW_STORE_WT (1, write-through: the lines leave L2 at once, so the
   * next dependent launch does not wait for that write-back; the VQ-VAE step's GEMM chain, +3 % per step). */
  int store_policy;
  /* dtype of `resid` (AW_F32 or AW_BF16): the bf16-mode VQ-VAE keeps its ResBlock residual streams (activations and
   * their gradients) in bf16, as autocast would (model/vq_vae_patch_embedd.py:73-74 under bf16 autocast) */
  int resid_dtype;
} aw_gemm_args;
#define AW_STORE_NT 0
#define AW_STORE_WT 1

int aw_gemm(const aw_gemm_args* args, void* stream);
/* Same, with a caller-provided f32 workspace: when the shape is split over K (small M*N, long K: the weight
 * gradients), partial products go to plain-store slabs in `ws` and one reduce pass writes C (no atomics).
 * aw_gemm_workspace returns the number of f32 elements needed (0: no split). */
int64_t aw_gemm_workspace(const aw_gemm_args* args);
int aw_gemm_ws(const aw_gemm_args* args, float* ws, int64_t ws_elems, void* stream);
/* Grouped launch of n <= AW_GEMM_MAX_GROUPS accumulate-mode problems (weight gradients) that share every field
 * except A, B, C and a_rowsum: one kernel over all groups' tiles.  The backward defers the weight gradients of
 * the ResBlock stack and issues them as one launch per layer kind (model/vq_vae_patch_embedd.py:60-74 grads;
 * model/transformer_block.py:30,32,78-79 grads), so each tile runs the full token reduction without split-K. */
#define AW_GEMM_MAX_GROUPS 16
int aw_gemm_grouped(const aw_gemm_args* args, int n, void* stream);
/* Tile policy knob: 0 = automatic (256x128 tiles for bf16 launches that fill the chip, else 128x128), 128 or 256 =
 * force that tile for every eligible launch (bf16, non-ragged) -- used by the tests to cover both pipelines. */
int aw_gemm_set_tile(int bm);
/* Weight-gradient kernel policy for the grouped decoder k = 3 launches (model/vq_vae_patch_embedd.py:60-74 grads):
 * 0 = automatic (the 8-wave ping-pong kernel when the shape qualifies and fills the chip), 1 = force it whenever the
 * shape qualifies, -1 = always the generic grouped GEMM (tests, A/B). */
int aw_gemm_set_wgrad_policy(int mode);
/* Batched weight gradients of plain (1-tap) layers: n <= AW_WGRAD_BATCH_MAX accumulate-mode problems
 *   C_i[m*ldc + colmap(n)] += alpha * sum_k A_i[k*lda + m] * B_i[k*ldb + n],  a_rowsum_i[m] += alpha * sum_k A_i[k*lda + m]
 * with bf16 operands (a_trans = b_trans = 1), f32 C, any M_i / N_i that are multiples of 256, one K (any K: ragged
 * token counts) and one alpha for all problems.  Replaces the weight / bias gradients of the transformer's Linear
 * layers, one launch for the four kinds of all 8 blocks (half of them per launch when a data-parallel step reduces
 * the later half's gradients early) (model/transformer_block.py:28-30,76-77), and of the
 * VQ-VAE encoder's per-token convs (model/vq_vae_patch_embedd.py:65,68 via :108-110).  One stream-K launch (one
 * workgroup per CU, equal work per CU whatever the tile count); tiles split between workgroups are summed through
 * `ws` (aw_wgrad_batch_workspace bytes, 16-B aligned, no initial contents).  One batch at a time per device (the
 * per-tile arrival counters are the library's).  Each tile adds into C with one plain read-modify-write (not
 * atomics, unlike aw_gemm's accumulate mode): the problems' C ranges [C, C + M*ldc) must not overlap (rejected).
 * aw_wgrad_batch_workspace returns -1 when the batch is not eligible. */
#define AW_WGRAD_BATCH_MAX 32
int64_t aw_wgrad_batch_workspace(const aw_gemm_args* args, int n);
int aw_wgrad_batch(const aw_gemm_args* args, int n, void* ws, int64_t ws_bytes, void* stream);
/* Bound of the fix-up's poll for its sibling pieces (default 2^26 polls; a piece that runs out of it poisons its tile
 * with NaN instead of summing unpublished partials).  0 forces that path on every split tile: a test hook, after
 * which the per-tile hand-off counters of this process are stale (tests/test_gpu_kernels.py runs it in a child
 * process). */
int aw_wgrad_set_spin_limit(int polls);

/* Fused ResBlock chain, bf16 operands, H = 512, no BatchNorm: the whole ResBlock stack of the encoder or of the
 * decoder (model/vq_vae_patch_embedd.py:60-74 ResBlock, :103-110 CNNBlock) as ONE persistent launch of N / 64
 * workgroups, each walking a 64-token row block through the 2R convs with its activations resident in LDS; it
 * replaces the 2R aw_gemm launches of either direction.  The forward's operands a1 / a and keep bits are theirs bit for
 * bit; in place of their saved pre-activations h / x it saves GELU'(h) / GELU'(x) (f32 values rounded to bf16), and
 * the backward multiplies by those: its gh / gxo_out track the unfused backward to bf16 rounding.
 *   taps = 1: the encoder (CNNBlock(seperate=True)): every conv sees a length-1 token slice, so it is its centre tap,
 *             a [H][H] contraction per token; weights are [H][H] (packed).
 *   taps = 3: the decoder (CNNBlock(seperate=False)): k = 3, padding 1 convs along windows of seg = 16 consecutive
 *             rows (the rows of one welding window; rows outside the window read as zero, aw_gemm's implicit conv
 *             with conv_seg = 16); weights are [H][3H] with column j*H + i = tap j, input channel i (packed).
 * Forward, per block r (x_0 = x0, a_0 = a0 = GELU(x_0)), conv(W, v)[t] = sum_j W_j v[t + j - 1] (taps = 3) or W v[t]:
 *   h_r = conv(W1_r, a_r) + b1_r,  a1_r = GELU(h_r),  x_{r+1} = x_r + Dropout(conv(W2_r, a1_r) + b2_r; drop_seed[r],
 *   group row*H + c as aw_gemm's epilogue),  a_{r+1} = GELU(x_{r+1}) for r < R-1 and x_R for r = R-1.
 *   Stored: dgelu_h[r] = GELU'(h_r), a1[r] = a1_r, dgelu_x[r] = GELU'(x_{r+1}) (r < R-1), a[r] = a_{r+1} (GELU' of
 *   the f32 values, rounded to bf16: the backward's multipliers, in place of the unfused path's saved h_r / x_{r+1});
 *   dgelu_h / a1 / dgelu_x may be NULL (not stored: eval forwards).  Weights w1 / w2 are the forward copies of aw_res_pack_weights, biases f32.  With drop_p > 0
 *   and drop_masks != NULL the launch also writes the keep bits of every block there (aw_res_dropout_masks_bytes;
 *   the masks aw_res_dropout_masks makes), for the backward.
 * Backward, per block r = R-1 .. 0, from gx = dL/dx_R (bf16) and gxo = gx * mask_{R-1} (bf16), with
 * convT(W, v)[t] = sum_j W_j^T v[t - j + 1] (taps = 3) or W^T v[t]:
 *   gh_r = convT(W2_r, go_r) * GELU'(h_r),  gx_r = gx_{r+1} + convT(W1_r, gh_r) * GELU'(x_r),
 *   gxo_out[r] = gx_r * mask_{r-1} (r > 0: block r-1's conv2 operand) or gx_0 (r = 0); gh[r] = gh_r.
 *   w1t / w2t are the backward copies of aw_res_pack_weights; dgelu_h[r] = the forward's dgelu_h[r], dgelu_x[r] =
 *   the forward's dgelu_x[r-1] (r >= 1; dgelu_x[0] unused), x0 = x_0 (block 0's GELU'(x_0) is evaluated here, the
 *   erf form of aw_gemm's bf16 epilogues); drop_masks (drop_p > 0) = what the forward wrote.
 * All activations are [N][H] bf16 with row stride H, 16-B aligned; N * H * 2 < 2^31; 1 <= R <= AW_RES_CHAIN_MAX;
 * taps = 3 needs seg = 16 and N % 16 == 0.  drop_seed / seed_ptr select the masks (forward); store_policy AW_STORE_WT
 * (sc1) or AW_STORE_NT for every global store. */
#define AW_RES_CHAIN_MAX 16
typedef struct {
  int64_t N;
  int H, R;
  int taps, seg;
  const void* a0;
  const void* x0;
  const void* w1[AW_RES_CHAIN_MAX];
  const void* w2[AW_RES_CHAIN_MAX];
  const float* b1[AW_RES_CHAIN_MAX];
  const float* b2[AW_RES_CHAIN_MAX];
  void* dgelu_h[AW_RES_CHAIN_MAX];
  void* a1[AW_RES_CHAIN_MAX];
  void* dgelu_x[AW_RES_CHAIN_MAX];
  void* a[AW_RES_CHAIN_MAX];
  float drop_p;
  uint64_t drop_seed[AW_RES_CHAIN_MAX];
  const uint64_t* seed_ptr;
  int store_policy;
  uint64_t* drop_masks;
} aw_res_chain_fwd_args;
typedef struct {
  int64_t N;
  int H, R;
  int taps, seg;
  const void* gx;
  const void* gxo;
  const void* x0;
  const void* w1t[AW_RES_CHAIN_MAX];
  const void* w2t[AW_RES_CHAIN_MAX];
  const void* dgelu_h[AW_RES_CHAIN_MAX];
  const void* dgelu_x[AW_RES_CHAIN_MAX];
  void* gh[AW_RES_CHAIN_MAX];
  void* gxo_out[AW_RES_CHAIN_MAX];
  float drop_p;
  int store_policy;
  const uint64_t* drop_masks;
} aw_res_chain_bwd_args;
int aw_res_chain_fwd(const aw_res_chain_fwd_args* args, void* stream);
int aw_res_chain_bwd(const aw_res_chain_bwd_args* args, void* stream);
/* The chain's dropout keep bits for R blocks at N tokens: aw_res_dropout_masks_bytes(N, R) bytes (16-B aligned), one
 * 64-bit word per chain thread and block (block r's mask: the keep decision of aw_gemm's dropout epilogue with seed
 * drop_seed[r] mixed with *seed_ptr, on element row * 512 + c).  aw_res_chain_fwd writes the same words itself;
 * this standalone form serves a backward without a chain forward (and the tests). */
int64_t aw_res_dropout_masks_bytes(int64_t N, int R);
int aw_res_dropout_masks(int64_t N, int R, float drop_p, const uint64_t* drop_seed, const uint64_t* seed_ptr,
                         void* masks, void* stream);
/* Fragment-packed weight copies of the chain: n <= AW_RES_PACK_MAX bf16 matrices src[i] = W of shape
 * [512][taps * 512] ([out][(tap, in)], the forward operand layout; taps 1 or 3).  fwd[i] packs A = W, bwd[i] packs
 * the backward operand A[i][(j, o)] = W[o][j * 512 + i] (W^T for taps = 1); either may be NULL.  Packed layout of a
 * [512][K] A (row m, column k): the 1-KB block (m / 16, k / 32) at byte ((m / 16) * (K / 32) + k / 32) * 1024 holds
 * lane l = (m % 16) + 16 ((k % 32) / 8) at 16 l, element k % 8 within -- one MFMA A-fragment, so a wave reads each
 * fragment as one contiguous KB. */
#define AW_RES_PACK_MAX 32
int aw_res_pack_weights(const void* const* src, void* const* fwd, void* const* bwd, int n, int taps, void* stream);

/* -------------------------------------------------------------------------------- vector quantizer
 * VectorQuantizer.forward (model/vector_quantizer.py:76-119), fp32, codebook staged in LDS, no MFMA:
 *   dist = fl(fl(|z|^2 + |e_k|^2) - 2 * (k-ordered fmaf chain z.e_k)), argmin with first-index ties,
 *   z_q_ste = z + (e_idx - z), idx (int64), counts[k] += 1, sqerr[0] += sum (e_idx - z)^2 (f64).
 * counts (K floats) and sqerr (1 double) must be zero on entry.  D in {16,32,64,128,256}.
 */
int aw_vq_forward(const float* z, const float* E, int64_t N, int K, int D,
                  float* zq, int64_t* idx, float* counts, double* sqerr, void* stream);
/* aw_vq_forward that also writes z_q_ste into zq_copy (NULL = none; 16-B aligned, copy_dtype AW_BF16 or AW_F32):
 * the GEMM operand of the decoder's first conv, without a separate cast launch. */
int aw_vq_forward_ex(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx, float* counts,
                     double* sqerr, void* zq_copy, int copy_dtype, void* stream);
/* aw_vq_forward_ex with the code counts split over count_groups partial histograms (1..AW_VQ_COUNT_GROUPS_MAX):
 * counts holds count_groups x K floats, zero on entry; workgroup b adds into partial b % count_groups, so the adds
 * into any one address are count_groups times fewer (they serialise at the memory-side atomic units).  The partials
 * sum to the counts; aw_vq_finalize_ex takes them as they are. */
#define AW_VQ_COUNT_GROUPS_MAX 64
int aw_vq_forward_ex2(const float* z, const float* E, int64_t N, int K, int D, float* zq, int64_t* idx, float* counts,
                      int count_groups, double* sqerr, void* zq_copy, int copy_dtype, void* stream);
/* loss = m + beta*m with m = sqerr/(N*D) (vector_quantizer.py:107-108); perplexity = exp(-sum p log(p+1e-10)),
 * p = counts/N (:114-115).  Each output is one f32 device scalar. */
int aw_vq_finalize(const float* counts, const double* sqerr, int64_t N, int K, int D, float beta,
                   float* loss, float* perplexity, void* stream);
/* aw_vq_finalize over count_groups partial histograms (aw_vq_forward_ex2), summed per code in a fixed order. */
int aw_vq_finalize_ex(const float* counts, int count_groups, const double* sqerr, int64_t N, int K, int D, float beta,
                      float* loss, float* perplexity, void* stream);
/* Backward of the STE + loss: dz = g_zq + g_loss*2(z - z_q)/(N*D);  dE[idx] += g_loss*2*beta*(z_q - z)/(N*D).
 * g_zq may be NULL (treated as 0); g_loss is a device scalar.  dE is accumulated (not overwritten). */
int aw_vq_backward(const float* z, const float* E, const int64_t* idx, const float* g_zq, const float* g_loss,
                   int64_t N, int K, int D, float beta, float* dz, float* dE, void* stream);
/* aw_vq_backward that also writes dz into dz_copy (NULL = none; copy_dtype AW_BF16 or AW_F32): the operand of the
 * SepCNN backward GEMMs. */
int aw_vq_backward_ex(const float* z, const float* E, const int64_t* idx, const float* g_zq, const float* g_loss,
                      int64_t N, int K, int D, float beta, float* dz, float* dE, void* dz_copy, int copy_dtype,
                      void* stream);
/* ------------------------------------------------------------------ residual VQ with EMA codebooks (csrc/rvq.hip)
 * ResidualVQLightning (model/vector_quantizer.py:9-56) wraps vector-quantize-pytorch's ResidualVQ (third-party, not
 * installed here: its published algorithm is restated, parity unpinned).  Per layer i: aw_vq_forward on residual r_i
 * (counts = the EMA's bins, sqerr -> commitment loss via aw_vq_finalize with beta 0), then these:
 * sums[idx[n]][:] += z[n][:] (accumulated; zero on entry), f32, D % 4 == 0 (vector_quantizer.py:20-21 ema update). */
int aw_vq_cluster_sums(const float* z, const int64_t* idx, int64_t N, int K, int D, float* sums, void* stream);
/* One Lloyd step of the k-means init: means[k] = sums[k] / counts[k] where counts[k] > 0 (else unchanged);
 * avg (may be NULL) = the new means * counts (the init's embed_avg, written on the last step). */
int aw_kmeans_update(float* means, const float* sums, const float* counts, int K, int D, float* avg, void* stream);
/* EMA codebook update + dead-code replacement, in place (EuclideanCodebook training branch):
 *   cs = decay cs + (1-decay) counts;  avg = decay avg + (1-decay) sums;
 *   embed = avg / ((cs + eps) / (sum cs + K eps) * sum cs);
 *   codes with cs < threshold (threshold > 0) take a batch row z[r]: embed = z[r], avg = threshold z[r], cs = threshold.
 * Rows: the expired code of rank j (of n) draws uniformly from the j-th of n equal strata of the N rows (distinct rows),
 * hash seed mix(salt, *seed_ptr) (seed_ptr may be NULL).  ws: 2K floats of scratch. */
int aw_rvq_ema_update(float* embed, float* embed_avg, float* cluster_size, const float* counts, const float* sums,
                      const float* z, int64_t N, int K, int D, float decay, float eps, float threshold, uint64_t salt,
                      const uint64_t* seed_ptr, float* ws, void* stream);
/* out = (first ? 0 : out) + zq;  r_next = r - zq (r_next may be NULL).  n elements. */
int aw_rvq_residual(const float* r, const float* zq, int64_t n, float* out, int first, float* r_next, void* stream);
/* Backward of the stack: dz = nq * g_zq + sum_i g_loss[i] * commitment * 2 (res_i - q_i) / (N D);
 * res, q: (nq, N, D) -- each layer's input residual and its straight-through output; g_zq may be NULL. */
int aw_rvq_backward(const float* res, const float* q, const float* g_zq, const float* g_loss, int nq, int64_t N,
                    int D, float commitment, float* dz, void* stream);

/* min_encodings one-hot (N,K) f32 (vector_quantizer.py:98-100). */
int aw_vq_onehot(const int64_t* idx, int64_t N, int K, float* onehot, void* stream);
/* Gather E[idx] -> out (N, D) (get_embedding_from_one_hot, vector_quantizer.py:121-131). */
int aw_vq_gather(const float* E, const int64_t* idx, int64_t N, int D, float* out, void* stream);

/* --------------------------------------------------------------------------- VQ-VAE layout kernels
 * Patchify (model/vq_vae_patch_embedd.py:13-17): x (B, L, C) -> patches (B*S, ldp) with token t covering the
 * channel-major flat window [t*P, (t+1)*P); columns P..ldp-1 are zero.  S = L*C/P. */
int aw_patchify(const float* x, int64_t B, int L, int C, int P, void* patches, int64_t ldp, int dtype,
                void* stream);
/* Weight relayouts (+cast) for the GEMM operand forms; out dtype = `dtype`.
 * mode 0: conv (O,I,k) tap t -> [O][I]                        (centre tap of the per-token encoder convs)
 * mode 1: conv (O,I,3)     -> [O][3*I], col j*I+i              (decoder conv forward, b_trans=0)
 * mode 2: conv (O,I,3)     -> [3*O][I], row j*O+o = W[o][:,j]  (decoder conv input-gradient, b_trans=1)
 * mode 3: convT (I,O,k)    -> [k*O][I], row j*O+o              (un-patch ConvT forward b_trans=0 / dgrad b_trans=1)
 * mode 4: conv (O,I,k)     -> [O][ldo] zero padded, col i*k+j  (patch embed, 1 input channel)
 * `ldo` is the output row length (ignored except for mode 4).  Batched form only:
 * mode 5: plain cast of O*I elements;
 * (mode 6 is retired: it fed the round-2 fused encoder chain, deleted in round 3);
 * mode 7: conv stored tap-major (O,3,I) -> [3*O][I], row j*O+o (decoder conv input-gradient when the optimizer keeps
 *         the weight tap-major; the forward copy [O][3*I] of such a weight is mode 5 over O x 3I). */
int aw_weight_relayout(const float* W, int O, int I, int k, int tap, int mode, void* out, int64_t ldo,
                       int dtype, void* stream);
/* Batched form: up to AW_RELAYOUT_MAX_JOBS relayouts (modes 0-7 above; mode 5 casts e.g. the Linear weights of
 * model/transformer_block.py) into one output dtype, one launch per call. */
#define AW_RELAYOUT_MAX_JOBS 40
typedef struct {
  const float* W;
  void* out;
  int O, I, k, tap, mode;
  int64_t ldo;
} aw_relayout_job;
int aw_weight_relayout_batch(const aw_relayout_job* jobs, int n, int dtype, void* stream);
/* Inverse relayout of weight GRADIENTS, accumulated (+=) into the reference-layout gradient:
 * mode 0: g[O][I] -> G[o][i][tap];  mode 1: g[O][3I] -> G[o][i][j];  mode 3: g[kO][I] -> G[i][o][j];
 * mode 4: g[O][ldo] -> G[o][0][j]. */
int aw_weight_grad_scatter(const float* g, int O, int I, int k, int tap, int mode, int64_t ldg, float* G,
                           void* stream);
/* Elementwise cast/copy: out[i] = in[i] (f32 -> dtype). */
int aw_cast(const float* in, int64_t n, void* out, int dtype, void* stream);

/* Un-patch head forward (vq_vae_patch_embedd.py:27-30,52-57):
 * y (R = B*Q rows of H, f32, BN input) -> BN(stats) -> GELU(erf) -> ConvT(H->1, k5, s5) -> x_hat (B, 200, 2)
 * interleaved (flat position 5q+j of window b).  stats (f32 4*H): mean, invstd, gamma, beta (aw_bn_finalize). */
int aw_unpatch_head_fwd(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                        const float* b2, float* x_hat, void* stream);
/* BatchNorm finalize: colstats (f64 sum, sumsq over n rows) -> stats {mean, invstd, gamma, beta};
 * training: running_mean/var momentum update (unbiased var), *nbt += 1.  eval (training == 0): uses running. */
int aw_bn_finalize(const double* colstats, int64_t n, int H, const float* gamma, const float* beta,
                   float* running_mean, float* running_var, int64_t* nbt, float eps, float momentum,
                   int training, float* stats, void* stream);
/* Un-patch head backward from g_xhat (same layout as x_hat).
 * pass 1: per-channel sums sum_g, sum_g*xhat (f64 2H, zero on entry); grads of w2 (H*5), b2 (1), gamma, beta
 *         accumulated (+=).
 * pass 2: g_y (R x H, gy_dtype) = BatchNorm backward (batch stats if training, else running) of g*gelu'(.),
 *         db_y (H f32, +=) = channel sums of g_y (gradient of the ConvT bias feeding the BN). */
int aw_unpatch_head_bwd1(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                         const float* g_xhat, double* gsums, float* gw2, float* gb2, float* ggamma, float* gbeta,
                         void* stream);
int aw_unpatch_head_bwd2(const float* y, int64_t R, int H, int Q, const float* stats, const float* w2,
                         const float* g_xhat, const double* gsums, int training, void* g_y, int gy_dtype, float* db_y,
                         void* stream);
/* The same three passes with y in y_dtype (AW_F32, or AW_BF16 when H is a power of two in 64..2048): the bf16
 * operand mode stores the ConvT output in bf16, halving the head's three HBM passes over it; the BN statistics
 * still come from the f32 values in the ConvT epilogue. */
int aw_unpatch_head_fwd_ex(const void* y, int y_dtype, int64_t R, int H, int Q, const float* stats, const float* w2,
                           const float* b2, float* x_hat, void* stream);
int aw_unpatch_head_bwd1_ex(const void* y, int y_dtype, int64_t R, int H, int Q, const float* stats, const float* w2,
                            const float* g_xhat, double* gsums, float* gw2, float* gb2, float* ggamma, float* gbeta,
                            void* stream);
int aw_unpatch_head_bwd2_ex(const void* y, int y_dtype, int64_t R, int H, int Q, const float* stats, const float* w2,
                            const float* g_xhat, const double* gsums, int training, void* g_y, int gy_dtype,
                            float* db_y, void* stream);
/* Fused training-step form of the head forward and pass 1 (train_reconstruction_embedding.py's step: loss =
 * mse(x_hat, x) + embedding loss, autencoder_lightning_base.py:80-97; vq_vae_patch_embedd.py:27-30,52-57), H == 512:
 * one read of y computes x_hat (as aw_unpatch_head_fwd_ex), g_xhat = (2 / (R*5)) * gscale[0] * (x_hat - x) (as
 * aw_mse_bwd), sqerr (f64, +=) = sum (x_hat - x)^2 (as aw_mse_fwd), and pass 1 of the backward from that g_xhat
 * (as aw_unpatch_head_bwd1_ex: gsums, gw2, gb2, ggamma, gbeta).  x: the input windows, same layout as x_hat. */
int aw_unpatch_head_fwd_bwd1(const void* y, int y_dtype, int64_t R, int H, int Q, const float* stats, const float* w2,
                             const float* b2, const float* x, const float* gscale, float* x_hat, float* g_xhat,
                             double* sqerr, double* gsums, float* gw2, float* gb2, float* ggamma, float* gbeta,
                             void* stream);
/* BatchNorm1d of the `--batchnorm 1` ResBlocks (model/vq_vae_patch_embedd.py:60-74).  Activations h are
 * [N rows][H channels] f32; statistics are per (group, channel), group = row % G (decoder G = 1; encoder G = S
 * token positions, each its own batch of B rows: CNNBlock(seperate=True) runs the blocks per token slice).
 * stats sums: double [2][G][H] (sum, sum of squares), zero on entry.
 * finalize: stats f32 [4][G][H] = mean, invstd, gamma, beta; training: batch statistics (biased variance) and
 *   the running statistics moved once per group in group order (unbiased variance, momentum), *nbt += G;
 *   eval: the running statistics for every group.
 * apply: mode 0: out = BN(h), op = GELU(out); mode 1: out = resid + dropout(BN(h)) (mask of element r*H + c
 *   from aw_seed_mix(drop_seed, seed_ptr), as the GEMM epilogues), op = GELU(out) or NULL; mode 2: as mode 1
 *   with op = out (no GELU).  op in op_dtype.
 * bwd_reduce: t = g_in * dropout mask; sums [2][G][H] += (sum t, sum t * xhat), zero on entry.
 * bwd_apply: dh (dh_dtype) = gamma*invstd*(t - S1/n - xhat*S2/n) (training) or gamma*invstd*t (eval);
 *   dgamma += sum_g S2, dbeta += sum_g S1 (either may be NULL).  n = rows per group. */
int aw_bn_group_stats(const float* h, int64_t N, int H, int G, double* sums, void* stream);
int aw_bn_group_finalize(const double* sums, int64_t n, int H, int G, const float* gamma, const float* beta,
                         float* running_mean, float* running_var, int64_t* nbt, float eps, float momentum,
                         int training, float* stats, void* stream);
int aw_bn_apply(const float* h, int64_t N, int H, int G, const float* stats, int mode, const float* resid,
                float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr, float* out, void* op, int op_dtype,
                void* stream);
int aw_bn_bwd_reduce(const float* h, int64_t N, int H, int G, const float* stats, const float* g_in, float drop_p,
                     uint64_t drop_seed, const uint64_t* seed_ptr, double* sums, void* stream);
int aw_bn_bwd_apply(const float* h, int64_t N, int H, int G, const float* stats, const float* g_in, float drop_p,
                    uint64_t drop_seed, const uint64_t* seed_ptr, const double* sums, int64_t n, int training,
                    void* dh, int dh_dtype, float* dgamma, float* dbeta, void* stream);
/* Mean-squared error (F.mse_loss, autencoder_lightning_base.py:82): sqerr[0] (f64, zero on entry) += sum (a-b)^2;
 * backward: ga = 2(a-b)/n * g (device scalar g). */
int aw_mse_fwd(const float* a, const float* b, int64_t n, double* sqerr, void* stream);
int aw_mse_bwd(const float* a, const float* b, int64_t n, const float* g, float* ga, void* stream);

/* loss = a[0] + b[0] (both device scalars) -> out[0]; also used for the autograd scalar plumbing. */
int aw_scalar_add(const float* a, const float* b, float* out, void* stream);
/* recon = sqerr/numel as f32 -> out */
int aw_mse_finalize(const double* sqerr, int64_t numel, float* out, void* stream);
/* out = sqerr / numel and sum = out + addend in one launch (the training step's recon error and total loss,
 * autencoder_lightning_base.py:80-97: loss = recon_error + embedding_loss). */
int aw_mse_finalize_add(const double* sqerr, int64_t numel, const float* addend, float* out, float* sum, void* stream);

/* ------------------------------------------------------------------------------------- optimizer
 * Multi-tensor RAdam over one flat parameter buffer (torch.optim.RAdam semantics, L2 weight decay):
 * segments [seg_off[s], seg_off[s]+seg_len[s]) (sorted, within [0,total)) with weight decay seg_wd[s]; seg_active[s]==0
 * are skipped (grad None: model/transformer_decoder.py heads under find_unused_parameters).  The buffers are 16-B
 * aligned, total % 4 == 0 and every segment starts 16-B aligned; the padding after a segment (up to the next
 * multiple of 4 elements) must be zero in all four buffers and stays zero (same for aw_grad_norm_clip's grad).
 * scalars come from host (step count, lr, betas, eps); `gscale` is a device scalar multiplying the gradient
 * first (clip coefficient; NULL = 1). */
int aw_radam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_off,
                  const int64_t* seg_len, const float* seg_wd, const int* seg_active, int nseg, int64_t total, int64_t step,
                  float lr, float beta1, float beta2, float eps, const float* gscale, const int64_t* step_ptr,
                  int zero_grad, void* stream);
/* zero_grad != 0: the gradient of every updated element is zeroed after use (optimizer.zero_grad() fused into the
 * update; inactive segments are left as they are). */
/* aw_radam_step that also writes the operand copies of the updated weights (what aw_weight_relayout_batch would
 * produce from the new values), so the training step needs no relayout launch.  ops: device array of
 * AW_OPS_PER_SEG descriptors per segment (ops[AW_OPS_PER_SEG*s + j]; mode -1 = none): flat element l of segment s
 * (the parameter in its storage order: (O, I, k) contiguous; a declare_centre_tap segment is its [O][I] centre,
 * described as k = 1, tap = 0) goes to `out` at the index of relayout mode `mode` (0-7), cast to `dtype`. */
#define AW_OPS_PER_SEG 2
typedef struct {
  void* out;
  int O, I, k, tap, mode, dtype;
  int64_t ldo;
} aw_operand_desc;
int aw_radam_step_ops(float* param, float* grad, float* exp_avg, float* exp_avg_sq, const int64_t* seg_off,
                      const int64_t* seg_len, const float* seg_wd, const int* seg_active, int nseg, int64_t total,
                      int64_t step, float lr, float beta1, float beta2, float eps, const float* gscale,
                      const int64_t* step_ptr, const aw_operand_desc* ops, int zero_grad, void* stream);
/* Device step counter / RNG counter: *counter += v (one thread; graph-capture safe).  With step_ptr != NULL,
 * aw_radam_step reads the step number from the device (the host `step` is ignored) and derives the bias
 * corrections and rectification there, in double precision like torch's python-float scalars. */
int aw_counter_add(int64_t* counter, int64_t v, void* stream);
/* The same, also copying the new value to *snapshot (the per-forward dropout seed the backward re-reads). */
int aw_counter_add_snapshot(int64_t* counter, int64_t v, int64_t* snapshot, void* stream);
/* The same, also zeroing zero[0 .. nzero) in the one launch (a forward's f64 accumulator block). */
int aw_counter_add_snapshot_zero(int64_t* counter, int64_t v, int64_t* snapshot, double* zero, int64_t nzero,
                                 void* stream);
/* Global L2 norm of the active segments of `grad` -> out_norm (f32 device scalar) and the clip coefficient
 * min(max_norm/(norm+1e-6), 1) -> out_coef (Lightning gradient_clip_val -> clip_grad_norm_).
 * ws: f64[AW_NORM_WS] scratch (per-workgroup partial sums, reduced in a fixed order: the norm is deterministic). */
#define AW_NORM_WS 1024
int aw_grad_norm_clip(const float* grad, const int64_t* seg_off, const int64_t* seg_len, const int* seg_active,
                      int nseg, int64_t total, float max_norm, double* ws, float* out_norm, float* out_coef,
                      void* stream);
/* x[i] *= s (device scalar), over n elements. */
int aw_scale(float* x, int64_t n, const float* s, void* stream);

/* ------------------------------------------------------------------------------------ transformer
 * LayerNorm (model/transformer_block.py:71,73; transformer_decoder.py:28), eps, over the last dim D.
 * y = (x-mean)*rstd*w + b (y_dtype); mean/rstd saved (f32, R each). */
int aw_layernorm_fwd(const float* x, int64_t R, int D, const float* w, const float* b, float eps, void* y,
                     int y_dtype, float* mean, float* rstd, void* stream);
/* dx (+= if accumulate) and dw/db (accumulated, f32).  Optional second output dx2 (dx2_dtype) = the final dx
 * times the dropout mask (drop_seed, r*D + c, drop_p) of the residual branch that produced x -- the operand of
 * the preceding block's output-projection gradients (mask regenerated, never stored). */
int aw_layernorm_bwd(const float* x, const float* dy, int64_t R, int D, const float* w, const float* mean,
                     const float* rstd, float* dx, int accumulate, float* dw, float* db, void* dx2, int dx2_dtype,
                     float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr, void* stream);
/* Classification head (transformer_decoder.py:126-129): s[r] = xf[r].w1 (+b1), g = GELU_erf(s),
 * out[b][c] = sum_t g[b*T+t] W2[c][t] (+b2[c]).  b1/b2 may be NULL (class_h_bias=False). */
int aw_class_head_fwd(const float* xf, int64_t B, int T, int D, const float* w1, const float* b1, const float* W2,
                      const float* b2, float* s, float* out, void* stream);
/* Backward: dxf (R x D, written), dw1 (D), db1 (1), dW2 (2 x T), db2 (2) accumulated (+=); NULL grads skipped. */
int aw_class_head_bwd(const float* xf, const float* s, const float* dout, int64_t B, int T, int D, const float* w1,
                      const float* W2, float* dxf, float* dw1, float* db1, float* dW2, float* db2, void* stream);
/* Token embedding + sinusoidal PE (model/embedding.py:57-59): x[b,t,:] = Wtok[ids[b,t]] + pe[t] */
int aw_embed_fwd(const int64_t* ids, int64_t B, int T, int D, const float* wtok, const float* pe, float* x,
                 void* stream);
/* aw_embed_fwd followed by aw_layernorm_fwd(x, B*T, D, w, b, eps, y, y_dtype, mean, rstd) in one launch, bit-identical
   to the pair (the first block's ln_1, model/transformer_block.py:84); D = 256, 512, 768 or 1024, 16-B aligned rows */
int aw_embed_ln_fwd(const int64_t* ids, int64_t B, int T, int D, const float* wtok, const float* pe, float* x,
                    const float* w, const float* b, float eps, void* y, int y_dtype, float* mean, float* rstd,
                    void* stream);
int aw_embed_bwd(const int64_t* ids, int64_t B, int T, int D, const float* dx, float* dwtok, void* stream);
/* aw_embed_bwd for a table of V rows without global atomics: a counting sort of the rows by id, then one owner per
   table element (ids outside [0, V) are skipped).  work: V + 1 + B*T ints of device scratch.  Falls back to
   aw_embed_bwd when V > 15360, D is not 256 / 512 / 768 / 1024 or dx / dwtok are not 16-B aligned. */
int aw_embed_bwd_sorted(const int64_t* ids, int64_t B, int T, int D, int V, const float* dx, float* dwtok, int* work,
                        void* stream);
/* Its two halves, for a caller that sorts early (the ids are known at the forward): aw_embed_sort fills work (V + 1 + R ints; V <= 15360) from the R ids,
   aw_embed_bwd_segsum adds the rows of dx (R x D, D = 256/512/768/1024, 16-B aligned) into dwtok from it. */
int aw_embed_sort(const int64_t* ids, int64_t R, int V, int* work, void* stream);
int aw_embed_bwd_segsum(const int* work, int V, int D, const float* dx, float* dwtok, void* stream);
/* Causal self-attention core (model/transformer_block.py:44-60) on the packed qkv projection
 * (B*T, 3*d, dtype), heads of hs = d/n_head: y (B*T, d, dtype) = softmax(q k^T / sqrt(hs), causal) v;
 * lse (B*n_head*T f32) saved for the backward (flash-style, T x T never materialised). */
int aw_attn_fwd(const void* qkv, int64_t B, int T, int n_head, int d, int dtype, void* y, float* lse,
                void* stream);
/* dqkv (B*T, 3d, dtype) from dy (B*T, d, dtype), recomputing P from lse; ws: f32 B*n_head*T (delta). */
int aw_attn_bwd(const void* qkv, const void* y, const void* dy, const float* lse, int64_t B, int T, int n_head,
                int d, int dtype, void* dqkv, float* ws, void* stream);
/* The same two with attention-probability dropout (CausalSelfAttention.attn_dropout, transformer_block.py:44-57;
 * the reference default is 0.0): P_ij kept with probability 1 - drop_p and scaled by 1/(1 - drop_p); the mask of
 * element ((b*n_head + h)*T + i)*T + j comes from the counter hash of (drop_seed mixed with *seed_ptr when given),
 * so the backward regenerates the forward's mask.  drop_p = 0 is exactly aw_attn_fwd / aw_attn_bwd. */
int aw_attn_fwd_dropout(const void* qkv, int64_t B, int T, int n_head, int d, int dtype, void* y, float* lse,
                        float drop_p, uint64_t drop_seed, const uint64_t* seed_ptr, void* stream);
int aw_attn_bwd_dropout(const void* qkv, const void* y, const void* dy, const float* lse, int64_t B, int T,
                        int n_head, int d, int dtype, void* dqkv, float* ws, float drop_p, uint64_t drop_seed,
                        const uint64_t* seed_ptr, void* stream);
/* KV-cache decode attention (MyTransformerDecoder.generate, model/transformer_decoder.py:203-224):
 * n_new query rows per sequence at absolute positions pos0 .. pos0+n_new-1 (qkv_new (B*n_new, 3d, dtype), row
 * b*n_new + i).  Their K and V are appended to kv_cache (B, Tmax, 2d, dtype; row b*Tmax + t = [K | V]) and
 * y (B*n_new, d, dtype) = softmax(q k^T / sqrt(hs)) v over the cached positions 0 .. pos0+i (causal). */
int aw_attn_decode(const void* qkv_new, int64_t B, int n_new, int pos0, int n_head, int d, int dtype,
                   void* kv_cache, int Tmax, void* y, void* stream);
/* Cross entropy with ignore_index (transformer_decoder.py:226-230): logits (R, V) f32 with row stride ldl;
 * loss_sum (f64, zero on entry) += sum over kept rows of (lse - logit[y]); count (f64) += kept rows.
 * The backward writes dlogits = (softmax - onehot) * g / count (g device scalar) into dlogits (dtype) and zeros
 * into its padding columns V..ldd-1. */
int aw_ce_fwd(const float* logits, int64_t R, int V, int64_t ldl, const int64_t* y, int ignore_index,
              double* loss_sum, double* count, float* lse, void* stream);
int aw_ce_bwd(const float* logits, int64_t R, int V, int64_t ldl, const int64_t* y, int ignore_index,
              const float* lse, const double* count, const float* g, void* dlogits, int64_t ldd, int dtype,
              void* stream);
int aw_ce_finalize(const double* loss_sum, const double* count, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ARCWELD_AMD_H */

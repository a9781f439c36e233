/* mlvae.h -- C ABI of libmlvae.so, the MI355X (gfx950) kernels of the ML-VAE training step.
 *
 * Conventions
 *   - Every entry point returns int: 0 ok, 1 bad argument, 2 HIP launch/runtime error;
 *     the text of the last error of the calling thread is mlvae_last_error().
 *   - The caller owns every device buffer and workspace; the library never allocates.
 *   - Calls are stream-ordered on `stream` (a hipStream_t passed as void*) and reentrant.
 *   - Tensors are fp32, row-major [B*T, C] with row n = b*T + t (the reference's batch_first
 *     [B,T,C] layout, ref:src/modules/decoder.py:14), leading dimension in elements.
 *   - prec: 0 = fp32 (exact f32 MFMA, the parity mode), 1 = bf16 operands / fp32 accumulate.
 *
 * The reference is pure Python (SURVEY.md section 0): it has no FFI.  Each entry below names
 * the reference code whose work it replaces; the Python drop-in layer (ml-vae_amd/modules,
 * ml-vae_amd/models) binds these through ctypes (INTEGRATION.md).
 */
#ifndef MLVAE_H
#define MLVAE_H
#include <stddef.h>
#ifdef __cplusplus
extern "C" {
#endif

const char* mlvae_last_error(void);
int mlvae_abi_version(void);
int mlvae_device_check(char* arch_out, int len);

/* C = epi(alpha*op(A).op(B) + bias1 + bias2 + beta*C).  trans_a: A stored [K][M];
 * trans_b: B stored [N][K].  epi 0 none, 1 LeakyReLU(0.01), 2 multiply by lrelu'(aux).
 * kshift/kshift_T (trans_b = 0): B row k reads row k+kshift when 0 <= k%T + kshift < T, else 0.
 * Replaces nn.Linear forward/backward (ref:src/modules/fc_block.py:10-16,
 * ref:src/modules/vanilla_vae.py:18-24) and the LSTM input projections and weight
 * gradients (ref:src/modules/decoder.py:14-15,22). */
size_t mlvae_gemm_workspace_size(int M, int N, int K);
int mlvae_gemm(int prec, int trans_a, int trans_b, int M, int N, int K, float alpha,
               const float* A, int lda, const float* B, int ldb, float beta, float* C, int ldc,
               const float* bias1, const float* bias2, int epi, const float* aux, int ldaux,
               int kshift_T, int kshift, float* ws, size_t ws_bytes, void* stream);

/* bf16-MFMA GEMM over bf16 or fp32 operands (a_bf16 / b_bf16: operand stored as bf16),
 * fp32 C, same epilogues / kshift / split-K as mlvae_gemm.  The bf16 precision mode's GEMMs:
 * the step keeps bf16 copies of its GEMM operands (h, dropout output, dG, weights).  Operand
 * rows along the contiguous dimension must be 16-byte aligned. */
size_t mlvae_gemm_ex_workspace_size(int M, int N, int K);
int mlvae_gemm_ex(int trans_a, int trans_b, int M, int N, int K, float alpha, const void* A,
                  int a_bf16, int lda, const void* B, int b_bf16, int ldb, float beta, float* C,
                  int ldc, const float* bias1, const float* bias2, int epi, const float* aux,
                  int ldaux, int kshift_T, int kshift, float* ws, size_t ws_bytes, void* stream);
/* The same with epilogue 3 = inter-layer dropout backward: C *= mask(drop_seed, drop_offset +
 * row*ldc + col)
 * with the mask of mlvae_dropout_ex (keep prob 1 - drop_p, scale 1/(1 - drop_p)), so the dgrad
 * of the layer above writes the gradient of the dropout input directly
 * (ref:src/modules/decoder.py:14, nn.LSTM dropout between layers in train mode). */
int mlvae_gemm_ex_drop(int trans_a, int trans_b, int M, int N, int K, float alpha,
                       const void* A, int a_bf16, int lda, const void* B, int b_bf16, int ldb,
                       float beta, float* C, int ldc, const float* bias1, const float* bias2,
                       int epi, const float* aux, int ldaux, int kshift_T, int kshift,
                       unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                       float* ws, size_t ws_bytes, void* stream);
/* Large bf16 GEMMs (256 x 256 tiles, LDS-DMA staging, bf16 operands only, fp32 C):
 *   C_b = epi( op(A_b) op(B_b) + bias1 + bias2 + beta C_b ),  b = 0 .. batch-1
 * A_b = A + b*a_bstride (elements; strides may be negative), likewise B_b, C_b.  trans_a = 0: A [M,K] k-contiguous;
 * trans_a = 1: A stored [K,M].  trans_b = 1: B stored [N,K]; trans_b = 0: B stored [K,N].
 * kshift (+ b*kshift_bstep) time-shifts the rows of a [K,N] B operand as mlvae_gemm does.
 * epi as mlvae_gemm_ex_drop (3 = dropout mask of (drop_seed, row*ldc + col)); epi | 16
 * (EPI_OUT_F16) stores C as IEEE fp16 (C then points at fp16; beta 0, epi 0 or 3, N, ldc and
 * c_bstride multiples of 4 / 8, aligned C and biases): the input projection into the wide
 * recurrence's fp16 gate buffer (mlvae_lstm_gates_fp16).  Operands need
 * 16-byte aligned bases, lda/ldb and the contiguous extent multiples of 8.  Long-K products
 * split K into fp32 partial slabs (workspace: mlvae_gemm_bf16_workspace_size) reduced in a fixed
 * order.  Replaces the LSTM input projection, its dgrad and the weight gradients
 * (ref:src/modules/decoder.py:14-15,22). */
size_t mlvae_gemm_bf16_workspace_size(int M, int N, int K, int batch);
/* split-K planning target of mlvae_gemm_bf16 in workgroups (default 256, one per CU); returns
 * the previous value (values < 1 only query).  Host-side launch planning state: set it on the
 * launching thread right before the launches it should shape (the engine lowers it for weight
 * gradients that overlap a recurrence).  Workspace sizes assume the default or lower. */
int mlvae_gemm_bf16_set_split_target(int workgroups);
/* main-loop variant of mlvae_gemm_bf16 (0 = the default per operand layout; others are the
 * kernel's measured alternatives, for same-process A/B timing); returns the previous value
 * (values < 0 only query).  Initialised from MLVAE_GEMM_VAR.  Host-side planning state. */
int mlvae_gemm_bf16_set_variant(int var);
int mlvae_gemm_bf16(int trans_a, int trans_b, int M, int N, int K, int batch, const void* A,
                    int lda, long long a_bstride, const void* B, int ldb, long long b_bstride,
                    float* C, int ldc, long long c_bstride, float beta, const float* bias1,
                    const float* bias2, int epi, const float* aux, int ldaux, int kshift_T,
                    int kshift, int kshift_bstep, unsigned long long drop_seed,
                    unsigned long long drop_offset, float drop_p, float* ws, size_t ws_bytes,
                    void* stream);
/* y (bf16) = round-to-nearest-even(x), n elements. */
int mlvae_cast_bf16(size_t n, const float* x, void* y, void* stream);
/* y [cols, rows] (bf16) = transpose of x [rows, cols] (fp32, row-major): the k-contiguous copy of
 * an LSTM input weight that the dgrad dX = dG W_ih reads (ref:src/modules/decoder.py:14-15). */
int mlvae_cast_bf16_t(int rows, int cols, const float* x, void* y, void* stream);

/* Bidirectional LSTM layer recurrence, both directions in one persistent launch.
 * gates [B*T, 8H]: in = x W_ih^T + b_ih + b_hh (cols [0,4H) forward, [4H,8H) reverse);
 *                  out = activated gates i,f,g,o (saved for the backward).
 * cells [B*T, 2H], y [B*T, 2H] (forward half | reverse half) = nn.LSTM output.
 * xbuf: exchange workspace (size from mlvae_lstm_workspace_size); err: device int set to 1
 * if a hand-off wait timed out (the launch then completes with undefined outputs).
 * Replaces the recurrent part of nn.LSTM (ref:src/modules/decoder.py:22). */
int mlvae_lstm_workspace_size(int B, int H, int prec, size_t* xbytes);
int mlvae_lstm_fwd(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                   float* gates, float* cells, float* y, void* xbuf, size_t xbytes, int* err,
                   void* stream);
/* BPTT: gates in = activated gates from mlvae_lstm_fwd, out = pre-activation gate grads dG.
 * dy = gradient wrt the layer output y.  Weight/input grads follow as GEMMs on dG. */
int mlvae_lstm_bwd(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                   float* gates, const float* cells, const float* dy, void* xbuf, size_t xbytes,
                   int* err, void* stream);
/* _ex variants: the forward also writes h as bf16 (y_bf16 [B*T, 2H], may be NULL); the
 * backward writes dG as bf16 into dg_bf16 [B*T, 8H] instead of into gates (NULL: into gates).
 * The bf16 copies are the operands of the bf16-mode GEMMs (mlvae_gemm_ex). */
int mlvae_lstm_fwd_ex(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                      float* gates, float* cells, float* y, void* y_bf16, void* xbuf,
                      size_t xbytes, int* err, void* stream);
int mlvae_lstm_bwd_ex(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                      float* gates, const float* cells, const float* dy, void* dg_bf16,
                      void* xbuf, size_t xbytes, int* err, void* stream);
/* Unidirectional layer, nn.LSTM(bidirectional=False, batch_first=True): the phoneme
 * recogniser's and boundary detector's LSTMs (ref:src/modules/phoneme_recognizer.py:13,
 * ref:src/modules/boundary_detector.py:19) and the MD-VAE's 512-unit RNN (ref:src/models/MD_VAE/
 * model.yaml:78-83).  gates [B*T, 4H] fp32 (in: x W_ih^T + b_ih + b_hh; out: activated i,f,g,o;
 * the backward overwrites them with dG unless dg_bf16 != NULL), cells / y / dy [B*T, H].  Same
 * workspace, err word and batch chunking as mlvae_lstm_fwd. */
int mlvae_lstm1_fwd(int prec, int B, int T, int H, const float* w_hh, float* gates, float* cells,
                    float* y, void* y_bf16, void* xbuf, size_t xbytes, int* err, void* stream);
int mlvae_lstm1_bwd(int prec, int B, int T, int H, const float* w_hh, float* gates,
                    const float* cells, const float* dy, void* dg_bf16, void* xbuf, size_t xbytes,
                    int* err, void* stream);
/* Wide-batch recurrence (csrc/lstm_wide.hip): one launch per layer for the whole batch when B is
 * past one batch-group launch (bf16, H = 512).  mlvae_lstm_gates_fp16(B, H, prec) = 1 for such
 * shapes; their gate buffer is IEEE fp16 [B*T, 8H] (half the projection's write and the
 * recurrences' reads) and they run only through the _ex2 entry points with gates_fp16 = 1.
 * gates_fp16 = 0 (and every entry point above) always runs the batch-group kernels on fp32
 * gates, batch-chunked.
 * fwd_ex2: y (fp32) may be NULL on the wide path; y_bf16 as _ex; y_drop_bf16 (wide path only,
 *   may be NULL) = bf16 dropout(h) for the next layer, mask of element drop_offset + row*2H + col
 *   from Philox(drop_seed) with keep 1 - drop_p -- the same mask mlvae_dropout_ex and the
 *   dropout epilogues (epi 3) draw, so the dgrad GEMM's epilogue recomputes it.
 * bwd_ex2: gates are the forward's (fp16 when gates_fp16); the wide backward writes dG only as
 *   bf16 into dg_bf16 (required) and, when dbias_rows != NULL (wide path only), the fp32 sums of
 *   dG over each batch group's 16 utterances and all T steps: dbias_rows [ceil(B/16)][8H], whose
 *   column sums are the layer's b_ih / b_hh gradients (ref:src/modules/decoder.py:14-15). */
int mlvae_lstm_gates_fp16(int B, int H, int prec);
/* The same for sequence length T: also 0 where T exceeds the wide kernels' 32-bit batch-group
 * addressing (16 T 8H fp16 gates >= 4 GB); the engine picks its gate buffer with it. */
int mlvae_lstm_gates_fp16_t(int B, int T, int H, int prec);
int mlvae_lstm_fwd_ex2(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                       void* gates, int gates_fp16, float* cells, float* y, void* y_bf16,
                       void* y_drop_bf16, unsigned long long drop_seed,
                       unsigned long long drop_offset, float drop_p, void* xbuf, size_t xbytes,
                       int* err, void* stream);
int mlvae_lstm_bwd_ex2(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                       void* gates, int gates_fp16, const float* cells, const float* dy,
                       void* dg_bf16, float* dbias_rows, void* xbuf, size_t xbytes, int* err,
                       void* stream);
/* bwd_ex3: bwd_ex2 with dy given as bf16 [B*T, 2H] when dy_bf16 = 1 (wide path only: gates_fp16 = 1;
 *   not with the fp8 BPTT) -- the fused engine's heads and dgrad GEMMs write dY in bf16, halving
 *   its bytes in their epilogues and in the BPTT's cell-input stream.  dy_bf16 = 0: bwd_ex2. */
int mlvae_lstm_bwd_ex3(int prec, int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev,
                       void* gates, int gates_fp16, const float* cells, const void* dy, int dy_bf16,
                       void* dg_bf16, float* dbias_rows, void* xbuf, size_t xbytes, int* err,
                       void* stream);
/* fp8 mode (BASELINE.json configs[4]) of the wide-batch recurrences (gates_fp16 shapes, bf16):
 *   fwd: as mlvae_lstm_fwd_ex2 without the fp32 h, plus y_drop_fp8 = e4m3(dropout(h) * x8_scale):
 *        the next layer's fp8 input-projection operand, written by the recurrence itself
 *        (replaces a cast pass over the bf16 copy; ref:src/modules/decoder.py:14-15,22);
 *        y_drop_bf16 may be NULL (the e4m3 copy alone: a step whose weight gradient of the next
 *        layer runs on e4m3 too reads no bf16 dropout(h))
 *   bwd: as mlvae_lstm_bwd_ex2, plus dg_fp8 = e4m3(dG * *dg8_scale) (NULL: none) -- the fp8
 *        dgrad's operand under delayed scaling -- and max |dG| max-ed into *dg_amax (float bits) */
int mlvae_lstm_fwd_fp8(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev, void* gates,
                       float* cells, void* y_bf16, void* y_drop_bf16, void* y_drop_fp8, float x8_scale,
                       unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                       void* xbuf, size_t xbytes, int* err, void* stream);
/* Wide forward of the bottom layer with its input projection fused (replaces the skinny
 * projection + mlvae_lstm_fwd_ex2 pair for ref:src/modules/decoder.py:22, nn.LSTM layer 0 whose
 * input is the 32-wide latent z): each step's gate inputs z_t W_ih^T + b_ih + b_hh are computed
 * inside the recurrence from z (bf16 [B*T rows, ldz], Z = 32), so the 8H-wide projection is
 * never written or read; gates receives the activated gates (fp16) as from mlvae_lstm_fwd_ex2.
 * y (fp32 h), y_drop_bf16 and y_drop_fp8 (with x8_scale > 0) are optional, each on its own. */
int mlvae_lstm_fwd_z(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev, const void* z_bf16,
                     int ldz, int Z, const float* w_ih_fwd, const float* w_ih_rev, const float* b_ih_fwd,
                     const float* b_hh_fwd, const float* b_ih_rev, const float* b_hh_rev, void* gates,
                     float* cells, float* y, void* y_bf16, void* y_drop_bf16, void* y_drop_fp8, float x8_scale,
                     unsigned long long drop_seed, unsigned long long drop_offset, float drop_p, void* xbuf,
                     size_t xbytes, int* err, void* stream);
/* mlvae_lstm_fwd_z with y_bf16_prev = 1: y_bf16 row t receives the h ENTERING step t (h_{t-1} in
 * the forward direction, h_{t+1} in the reverse one, zeros at each utterance's first step) instead
 * of h_t -- the time-shifted operand of dW_hh_l0 = sum_t dG_t^T h_{t-/+1} pre-shifted, so that the
 * weight gradient runs as a plain (unshifted) product.  For a y_bf16 no other product reads (the
 * next layer's input is the dropout copy). */
int mlvae_lstm_fwd_z2(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev, const void* z_bf16,
                      int ldz, int Z, const float* w_ih_fwd, const float* w_ih_rev, const float* b_ih_fwd,
                      const float* b_hh_fwd, const float* b_ih_rev, const float* b_hh_rev, void* gates,
                      float* cells, float* y, void* y_bf16, int y_bf16_prev, void* y_drop_bf16, void* y_drop_fp8,
                      float x8_scale, unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                      void* xbuf, size_t xbytes, int* err, void* stream);
int mlvae_lstm_bwd_fp8(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev, void* gates,
                       const float* cells, const float* dy, void* dg_bf16, float* dbias_rows,
                       void* dg_fp8, const float* dg8_scale, unsigned* dg_amax, void* xbuf,
                       size_t xbytes, int* err, void* stream);
/* mlvae_lstm_bwd_fp8 with dy as bf16 [B*T, 2H] when dy_bf16 = 1 (as mlvae_lstm_bwd_ex3).  Both
 * forms: dg_bf16 may be NULL when dg_fp8 is given (every dG reader on e4m3: the dgrad, dW_ih and
 * dW_hh through mlvae_gemm_fp8_tn_ex); the bias rows still come from the fp32 dG. */
int mlvae_lstm_bwd_fp8_ex(int B, int T, int H, const float* w_hh_fwd, const float* w_hh_rev, void* gates,
                          const float* cells, const void* dy, int dy_bf16, void* dg_bf16,
                          float* dbias_rows, void* dg_fp8, const float* dg8_scale, unsigned* dg_amax,
                          void* xbuf, size_t xbytes, int* err, void* stream);
/* Workgroups (one per CU, co-resident) of the recurrence launch for this shape as the engine
 * runs it (fp16 gates where mlvae_lstm_gates_fp16): the wide kernels fill the chip. */
int mlvae_lstm_launch_workgroups(int B, int H, int prec, int fwd);
/* Diagnostics: record per-step phase stamps of workgroup 0 into buf (NULL disables). */
int mlvae_lstm_set_debug(void* buf);

/* MD-VAE upstream-LSTM losses (csrc/md.hip).
 * mlvae_phn_bce: PhonemeRecognizer.compute_losses (ref:src/modules/phoneme_recognizer.py:35-81).
 *   logits [B,T,C] (row stride ldl), feat_lens / phn_lens [B] relative, phn [B,L] int64 ids,
 *   boundary [B,T] 0/1 (float).  Frame t < T_i = round(T feat_len) gets target one-hot(phn[b, k])
 *   with k = (boundaries in [0, t]) - 1; loss [B,T,C] = BCE-with-logits, 0 past T_i (may be NULL);
 *   with dloss given, dlogits = dloss (sigmoid(x) - y).  The reference's asserts set *err bits:
 *   2 = boundaries do not give L_i = round(L phn_len) segments from frame 0, 4 = phoneme id
 *   outside [0, C).
 * mlvae_boundary_fwd / _bwd: BoundaryDetector after its FC heads (ref:src/modules/boundary_detector.py:
 *   42-97).  za, zb [n] = pre-Softplus head outputs, y [n] boundary targets, u [10][n] U(0,1) draws
 *   (NULL: Philox(seed) at element offset + s*n + i).  Forward: v = mean of the ten clamped
 *   Kumaraswamy draws, bce = their mean BCE, kld = KL(Beta(alpha, beta) || Beta(1, 9)) (any output
 *   may be NULL).  Backward: dza, dzb from the cotangents dv, dbce, dkld (NULL = 0). */
int mlvae_phn_bce(int B, int T, int C, const float* logits, int ldl, const float* feat_lens,
                  const long long* phn, int L, const float* phn_lens, const float* boundary,
                  float* loss, const float* dloss, float* dlogits, int* err, void* stream);
int mlvae_boundary_fwd(size_t n, const float* za, const float* zb, const float* y, const float* u,
                       unsigned long long seed, unsigned long long offset, float* v, float* bce,
                       float* kld, void* stream);
int mlvae_boundary_bwd(size_t n, const float* za, const float* zb, const float* y, const float* u,
                       unsigned long long seed, unsigned long long offset, const float* dv,
                       const float* dbce, const float* dkld, float* dza, float* dzb, void* stream);

/* MD-VAE Viterbi decode (csrc/decode.hip): decode_plvl_md_lbl_seqs_full
 * (ref:src/utils/decode_utils.py:374-565, run in the MD-VAE forward at ref:src/models/MD_VAE/
 * model.py:133-141).  logits [B,T,N] (phoneme recogniser output, row stride ldl), boundary_v
 * [B,T], pi_logits [B,T,2], prior [N], seqs [B,L] int64 canonical ids, feat_lens / seq_lens [B]
 * relative, weight = dec_weight.  Outputs (int32): boundary_out [B,T] decoded boundaries (0/1),
 * flvl_out [B,T] frame-level and plvl_out [B,L] phoneme-level mispronunciation labels (-1 past
 * T_i / L_i), lens_out [B,2] = (T_i, L_i).  ws: mlvae_viterbi_workspace_size(B,T,L) bytes (the
 * argmax path map).  *err bits: 8 = the backtrack did not end at (l, t) = (0, 0) (the reference's
 * assert), 16 = T_i or L_i empty / L_i > 1024.  L <= 1024. */
size_t mlvae_viterbi_workspace_size(int B, int T, int L);
int mlvae_viterbi_md(int B, int T, int N, int L, const float* logits, int ldl, const float* boundary_v,
                     const float* pi_logits, const float* prior, const long long* seqs,
                     const float* feat_lens, const float* seq_lens, float weight, void* ws,
                     size_t ws_bytes, int* boundary_out, int* flvl_out, int* plvl_out, int* lens_out,
                     int* err, void* stream);

/* fp8 GEMM mode (BASELINE.json configs[4], csrc/gemm_fast.hip VAR 8 + csrc/fp8.hip): the decoder's
 * layer-1 input projection (ref:src/modules/decoder.py:14-15,22, nn.LSTM's x W_ih^T) on fp8 e4m3
 * (OCP) operands with per-tensor scales, v_mfma_scale_f32_16x16x128_f8f6f4, fp32 accumulate.
 *   gemm_fp8:  C = (*alpha) * A . B^T + bias1 + bias2, A [M][K], B [N][K] fp8 (k-contiguous,
 *              K, lda, ldb % 16, 16-byte aligned); C fp32, or fp16 with epi = 16 (EPI_OUT_F16).
 *   fp8_scale: out[0] = q = 448 / max|x| (1 if 0 / non-finite), out[1] = 1 / (q * other_scale).
 *   cast_fp8:  dst = e4m3(clamp(src * scale, +-448)), RNE; scale = *scale_p if non-null. */
int mlvae_gemm_fp8(int M, int N, int K, const void* A, int lda, const void* B, int ldb, void* C, int ldc,
                   const float* alpha, const float* bias1, const float* bias2, int epi, void* stream);
/* As mlvae_gemm_fp8 with epi = EPI_DROPOUT allowed (fp32 or, with the EPI_OUT_BF16 flag 32, bf16
 * C): C *= the inter-layer dropout mask of element drop_offset + row * ldc + col -- the fp8
 * layer-1 dgrad with the dropout backward fused (ref:src/modules/decoder.py:14-15: the dropout
 * between the LSTM layers); bf16 C is the wide BPTT's dY input (mlvae_lstm_bwd_ex3). */
int mlvae_gemm_fp8_ex(int M, int N, int K, const void* A, int lda, const void* B, int ldb, void* C,
                      int ldc, const float* alpha, const float* bias1, const float* bias2, int epi,
                      unsigned long long drop_seed, unsigned long long drop_offset, float drop_p,
                      void* stream);
/* C [M][N] (fp32) = (*alpha) * A^T B over fp8 e4m3 operands stored [K][M] and [K][N] (m- and
 * n-contiguous rows of lda / ldb bytes): the layer-1 weight gradient dW_ih = dG^T X over the K
 * frames (ref:src/modules/decoder.py:14-15,22, nn.LSTM's W_ih gradient) on the e4m3 dG the fp8
 * BPTT writes and the e4m3 layer input the forward writes.  M, N, lda, ldb % 16, 16-byte aligned
 * operands; deterministic split-K through ws (mlvae_gemm_fp8_tn_workspace_size bytes). */
size_t mlvae_gemm_fp8_tn_workspace_size(int M, int N, int K);
int mlvae_gemm_fp8_tn(int M, int N, int K, const void* A, int lda, const void* B, int ldb, float* C, int ldc,
                      const float* alpha, float* ws, size_t ws_bytes, void* stream);
/* mlvae_gemm_fp8_tn batched (A + z a_bstride, B + z b_bstride bytes, C + z c_bstride floats) with
 * time-shifted B rows: row k of B_z is read at k + sh_z, sh_z = kshift + z kshift_bstep, when
 * 0 <= k % kshift_T + sh_z < kshift_T, else as zeros (K % kshift_T == 0): the recurrent weight
 * gradients dW_hh = sum_t dG_t^T h_{t-1} (forward) / h_{t+1} (reverse) of both directions in one
 * launch on e4m3 dG and h (ref:src/modules/decoder.py:14-15,22; the bf16 form: mlvae_gemm_bf16's
 * kshift arguments).  Strides % 16; workspace mlvae_gemm_fp8_tn_ex_workspace_size bytes. */
size_t mlvae_gemm_fp8_tn_ex_workspace_size(int M, int N, int K, int batch);
int mlvae_gemm_fp8_tn_ex(int M, int N, int K, int batch, const void* A, int lda, long long a_bstride,
                         const void* B, int ldb, long long b_bstride, float* C, int ldc, long long c_bstride,
                         const float* alpha, int kshift_T, int kshift, int kshift_bstep, float* ws,
                         size_t ws_bytes, void* stream);
size_t mlvae_fp8_scale_workspace_size(void);
int mlvae_fp8_scale(size_t n, const float* x, float other_scale, float* out, float* ws, size_t ws_bytes,
                    void* stream);
int mlvae_cast_fp8(size_t n, const void* src, int src_bf16, const float* scale_p, float scale, void* dst,
                   void* stream);
/* Delayed (previous-step) scaling: from an amax word a producer max-ed (float bits),
 * out[0] = q = 448 / (margin * amax_prev) (1 without a usable amax), out[1] = 1 / (q * *other_q)
 * (the fp8 GEMM's alpha); *amax_next (distinct word, optional) is cleared for this step's producer. */
int mlvae_fp8_delayed_scale(const unsigned* amax_prev, unsigned* amax_next, const float* other_q,
                            float margin, float* out, void* stream);

/* Conv1d encoder layers (csrc/conv.hip), BASELINE.json configs[3]'s "Conv1d encoder variant":
 * the reference has none (SURVEY.md Appendix A); semantics = torch.nn.Conv1d(Cin, Cout, K,
 * padding=(K-1)/2) over each utterance of the batch-first frames [B, T, C] (row b*T + t), zero
 * outside [0, T).  This replaces the encoder's Linear layers (ref:src/modules/vanilla_vae.py:13-16,
 * FCBlock ref:src/modules/fc_block.py:4-21) in modules/conv_vae.py.  w: torch layout
 * [Cout][Cin][K] fp32; activations fp32, bf16 MFMA operands, fp32 accumulate.
 *   fwd:   y = act(conv(x) + bias)                      act: 1 = LeakyReLU(0.01)
 *   dgrad: dx = conv^T(dy) [* lrelu'(aux)]              (aux = the layer input's LReLU output)
 *   wgrad: dw = sum over frames, db = column sums of dy  (overwritten; deterministic)
 * Limits: K odd <= 9, Cin % 4 == 0 and <= 128, Cout % 16 == 0 and <= 128, 16-byte aligned
 * rows; wgrad: Cout in {16, 32, 64}, K * roundup(Cin, 16) <= 512 (mlvae_conv1d_supported). */
int mlvae_conv1d_supported(int Cin, int Cout, int K);
int mlvae_conv1d_fwd(int B, int T, int Cin, int Cout, int K, const float* x, int ldx, const float* w,
                     const float* bias, int act, float* y, int ldy, void* stream);
int mlvae_conv1d_dgrad(int B, int T, int Cin, int Cout, int K, const float* dy, int lddy, const float* w,
                       const float* aux, int ldaux, float* dx, int lddx, void* stream);
size_t mlvae_conv1d_wgrad_workspace_size(int B, int T, int Cin, int Cout, int K);
int mlvae_conv1d_wgrad(int B, int T, int Cin, int Cout, int K, const float* dy, int lddy, const float* x,
                       int ldx, float* dw, float* db, void* ws, size_t ws_bytes, void* stream);
/* ELBO: reparameterise + KL (ref:src/modules/vanilla_vae.py:37-45) with masked partial
 * sums; ml = [mu | log_var] rows of width 2Z (leading dim ldml). */
int mlvae_elbo_partials_count(int B, int T, int C);
int mlvae_reparam_kl_fwd(int B, int T, int Z, const float* ml, int ldml, const float* eps,
                         const float* lens, float* z, float* kl_out, float* partials,
                         void* stream);
int mlvae_reparam_kl_bwd(int B, int T, int Z, const float* ml, int ldml, const float* eps,
                         const float* lens, const int* count, const float* dz, const float* dkl,
                         float kl_scale, float* dml, int lddml, void* stream);
/* Reconstruction term (ref:src/modules/decoder.py:37-53; loss_type 0 likelihood, 1 mse)
 * with masked partial sums and, when dmux != NULL, its gradient. */
int mlvae_recon(int B, int T, int F, int loss_type, const float* mux, int ldmu, const float* lvx,
                int ldlv, const float* x, int ldx, const float* lens, const int* count,
                float* rec_out, float* partials, const float* drec, float rec_scale, float* dmux,
                float* dlvx, void* stream);
/* Fused decoder heads (bf16 mode): both FCBlock([2H, C, C, F]) heads forward, the recon loss
 * (masked partial sums into partials[mlvae_heads_partials_count(B, T)], read by
 * mlvae_elbo_finalize) and, when train, its gradient (scale rec_scale / (count * F)), both heads
 * backward and dy = d loss / d rnn_out [B*T, 2H], in one launch.  y_bf16 [B*T, 2H] bf16 rnn output;
 * w1_bf16 [2C, 2H] the two heads' stacked first-layer weights (bf16), w1t_bf16 its transpose
 * [2H, 2C] (train); b1 [2C]; w2*/w3* fp32 [C, C] / [F, C].  Outputs fp32: p1 [B*T, 2C], p2m/p2v
 * [B*T, C], mux/lvx [B*T, F]; train: dmux/dlvx (dlvx NULL for mse), dp2m/dp2v, dp1, dy.
 * mlvae_heads_supported(C, F, 2H): C == 64, F in {64, 80}, 2H % 128 == 0.  Replaces
 * ref:src/modules/decoder.py:24-25,37-53 + ref:src/modules/fc_block.py:9-16 and their autograd. */
int mlvae_heads_partials_count(int B, int T);
int mlvae_heads_supported(int C, int F, int H2);
int mlvae_heads_fused(int B, int T, int F, int C, int H2, int loss_type, int train,
                      const void* y_bf16, const void* w1_bf16, const void* w1t_bf16, const float* b1,
                      const float* w2m, const float* b2m, const float* w3m, const float* b3m,
                      const float* w2v, const float* b2v, const float* w3v, const float* b3v,
                      const float* x, const float* lens, const int* count, float rec_scale,
                      float* p1, float* p2m, float* p2v, float* mux, float* lvx, float* dmux,
                      float* dlvx, float* dp2m, float* dp2v, float* dp1, float* dy,
                      float* partials, void* stream);
/* mlvae_heads_fused plus, when bias_ws is given (train only), the five head bias gradients from
 * in-kernel column sums: per-workgroup sums into bias_ws (>= mlvae_heads_bias_workspace_size
 * bytes), then a fixed-order reduce into db3m / db3v (mean_fc / log_var_fc blocks.4.bias [F]),
 * db2m / db2v (blocks.2.bias [C]) and db1 (the stacked blocks.0 biases [2C]; mse: the log_var
 * head gets no gradient, so db3v, db2v and db1[C:] are not written).  Replaces the autograd
 * bias sums of ref:src/modules/fc_block.py:9-16 without re-reading dOUT / dP2 / dP1.
 * saved_bf16: p1, p2m/p2v, dmux/dlvx, dp2m/dp2v and dp1 are written as bf16 (packed rows, the
 * weight-gradient GEMMs' operand precision) instead of fp32; mux / lvx / dy stay fp32.
 * With bias_ws and saved_bf16 in train mode the work runs in split form: P1 and dY as 256^2
 * GEMMs (bias + LReLU + bf16 epilogue; fp32 dY) around a persistent kernel for the middle stages
 * (same outputs).  saved_bf16 bit 1 (value 3): the split form writes
 * dY as bf16 [N, 2H] (mlvae_lstm_bwd_ex3's dy_bf16 input); an error without the split form. */
size_t mlvae_heads_bias_workspace_size(int B, int T, int F, int C);
int mlvae_heads_fused_ex(int B, int T, int F, int C, int H2, int loss_type, int train,
                         const void* y_bf16, const void* w1_bf16, const void* w1t_bf16, const float* b1,
                         const float* w2m, const float* b2m, const float* w3m, const float* b3m,
                         const float* w2v, const float* b2v, const float* w3v, const float* b3v,
                         const float* x, const float* lens, const int* count, float rec_scale,
                         float* p1, float* p2m, float* p2v, float* mux, float* lvx, float* dmux,
                         float* dlvx, float* dp2m, float* dp2v, float* dp1, float* dy,
                         float* partials, float* bias_ws, size_t bias_ws_bytes, float* db3m,
                         float* db3v, float* db2m, float* db2v, float* db1, int saved_bf16,
                         void* stream);
/* mlvae_heads_fused_ex plus, when wg_ws is given, the four small weight gradients of the heads
 * (ref:src/modules/fc_block.py:9-16 blocks.2 / blocks.4 of mean_fc and log_var_fc, the products
 * autograd forms for decoder.py:24-25): dw3m / dw3v = dOUT_h^T P2_h [F, C] and dw2m / dw2v =
 * dP2_h^T P1_h [C, C], accumulated inside the heads' middle kernel over its 64-frame tiles (the
 * frame rows as K, read transposed from the LDS images it already holds), per-workgroup slabs
 * reduced in a fixed order -- replacing four split-K GEMM launches over the saved intermediates.
 * Needs the split form (train, bias_ws, saved_bf16 bit 0) and wg_ws_bytes >=
 * mlvae_heads_wgrad_workspace_size(B, T, F, C); under mse (loss_type 1) dw3v / dw2v may be NULL
 * and are not written.  P2 / dOUT / dP2 (p2m, p2v, dmux, dlvx, dp2m, dp2v) are then not written. */
size_t mlvae_heads_wgrad_workspace_size(int B, int T, int F, int C);
/* The split form's two first-layer products (P1 = LReLU(Y W1^T + b1), dY = dP1 W1) run on a
 * 128-row kernel (mode 1, the default: from 64K frames; 2: at every size; 0: on the 256² GEMM).
 * Both compute each output with the same k-order, so the modes agree bit for bit. */
int mlvae_heads_set_nt_mode(int mode);
int mlvae_heads_fused_ex2(int B, int T, int F, int C, int H2, int loss_type, int train,
                          const void* y_bf16, const void* w1_bf16, const void* w1t_bf16, const float* b1,
                          const float* w2m, const float* b2m, const float* w3m, const float* b3m,
                          const float* w2v, const float* b2v, const float* w3v, const float* b3v,
                          const float* x, const float* lens, const int* count, float rec_scale,
                          float* p1, float* p2m, float* p2v, float* mux, float* lvx, float* dmux,
                          float* dlvx, float* dp2m, float* dp2v, float* dp1, float* dy,
                          float* partials, float* bias_ws, size_t bias_ws_bytes, float* db3m,
                          float* db3v, float* db2m, float* db2v, float* db1, int saved_bf16,
                          float* wg_ws, size_t wg_ws_bytes, float* dw3m, float* dw3v, float* dw2m,
                          float* dw2v, void* stream);
/* mlvae_heads_fused_ex2 with the split-bf16 forward when w1_split is given (split form only): the
 * forward products of ref:src/modules/fc_block.py:9-16 as bf16 hi + lo operand pairs -- P1 = LReLU(Y
 * (W1_hi + W1_lo)^T + b1) on the 128-row kernel, P2 = LReLU(P1 (W2_hi + W2_lo)^T + b2) and OUT =
 * P2_hi (W3_hi + W3_lo)^T + P2_lo W3_hi^T + b3 -- so mu_x / log_var_x (and the ELBO) carry no bf16
 * rounding of the heads' weights.  w1_split = mlvae_bf16_split_rows(W1 [2C, 2H], chunk 64).  The
 * backward products stay bf16. */
int mlvae_heads_fused_ex3(int B, int T, int F, int C, int H2, int loss_type, int train,
                          const void* y_bf16, const void* w1_bf16, const void* w1t_bf16, const float* b1,
                          const float* w2m, const float* b2m, const float* w3m, const float* b3m,
                          const float* w2v, const float* b2v, const float* w3v, const float* b3v,
                          const float* x, const float* lens, const int* count, float rec_scale,
                          float* p1, float* p2m, float* p2v, float* mux, float* lvx, float* dmux,
                          float* dlvx, float* dp2m, float* dp2v, float* dp1, float* dy,
                          float* partials, float* bias_ws, size_t bias_ws_bytes, float* db3m,
                          float* db3v, float* db2m, float* db2v, float* db1, int saved_bf16,
                          float* wg_ws, size_t wg_ws_bytes, float* dw3m, float* dw3v, float* dw2m,
                          float* dw2v, const void* w1_split, void* stream);
/* dst [rows][2 cols] bf16 = src [rows][cols] fp32 as split-bf16 pairs: each chunk-wide column block
 * c becomes [hi | lo] at columns 2 c chunk .. 2 (c + 1) chunk - 1 (x = hi + lo to ~2^-17).  cols %
 * chunk == 0. */
int mlvae_bf16_split_rows(const float* src, int rows, int cols, int chunk, void* dst, void* stream);
/* Skinny products of the bottom LSTM layer (bf16; one side is the latent width):
 * mlvae_skinny_nt: C [M, N] (fp32, ldc) = A [M, K] . Bt [N, K]^T, bf16 k-contiguous operands,
 *   N in {16, 32, 48, 64}, K % 32 == 0: dZ = dG W_ih over the k-contiguous W_ih^T copy.
 * mlvae_skinny_tn: W [M, nw] (fp32 row-major) = A^T B over K frames, A stored [K, M] (lda), B
 *   stored [K, NB] (ldb), NB in {16..64} % 16, M % 64 == 0; bias1/bias2 [M] (either may be NULL)
 *   = column nw of the product (B's column nw all ones: the bias gradient as MFMA work).  Frame
 *   splits go to fp32 slabs (workspace: mlvae_skinny_tn_workspace_size) summed in a fixed order.
 * Replace the autograd of layer 0's input projection (ref:src/modules/decoder.py:14-15,22). */
/* C[M, N] = A[M, K] B[N, K]^T + bias1 + bias2 (bf16 operands, k-contiguous, fp32 C), K in
 * {8, 16, 24, 32}, N % 16 == 0, 16-byte aligned rows; biases may be NULL.  The layer-0 LSTM
 * input projection z W_ih^T + b_ih + b_hh (ref:src/modules/decoder.py:14-15,22), K = latent. */
int mlvae_skinny_proj(int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                      const float* bias1, const float* bias2, float* C, int ldc, void* stream);
/* The same with C fp32 (c_fp16 = 0) or IEEE fp16 (c_fp16 = 1: the wide recurrence's gates). */
int mlvae_skinny_proj_ex(int M, int N, int K, const void* A, int lda, const void* B, int ldb,
                         const float* bias1, const float* bias2, void* C, int ldc, int c_fp16,
                         void* stream);
int mlvae_skinny_nt(int M, int N, int K, const void* A, int lda, const void* Bt, int ldb,
                    float* C, int ldc, void* stream);
size_t mlvae_skinny_tn_workspace_size(int M, int NB, int K);
int mlvae_skinny_tn(int M, int NB, int K, const void* A, int lda, const void* B, int ldb, int nw,
                    float* W, float* bias1, float* bias2, float* ws, size_t ws_bytes, void* stream);
/* fp8 mode (configs[4]), layer 0: the same two products on the e4m3 dG the fp8 BPTT writes (lda in
 * bytes, % 16) -- converted to bf16 in registers (exact), results times *alpha (1 / dG's scale).
 * mlvae_skinny_nt_fp8 needs K % 256 and M >= 4096; mlvae_skinny_tn_fp8 mlvae_skinny_tn's workspace. */
int mlvae_skinny_nt_fp8(int M, int N, int K, const void* A8, int lda, const void* Bt, int ldb, float* C, int ldc,
                        const float* alpha, void* stream);
int mlvae_skinny_tn_fp8(int M, int NB, int K, const void* A8, int lda, const void* B, int ldb, int nw, float* W,
                        float* bias1, float* bias2, const float* alpha, float* ws, size_t ws_bytes, void* stream);
/* dZ = dG W_ih_l0 (as mlvae_skinny_nt) and dW_ih_l0 | b_ih = b_hh gradients = dG^T [z | 1] (as
 * mlvae_skinny_tn) from ONE pass over the layer-0 dG (ref:src/modules/decoder.py:14-15,22, the
 * autograd of nn.LSTM's layer-0 input projection): dG [M][lda] bf16 with K8 = 8H columns
 * (K8 % 256 == 0), Wt = W_ih^T [32][ldw] bf16, zb = [z | 1 | 0] [M][ldz >= 48] bf16 (Z = 32), dZ
 * [M][lddz] fp32; W [K8][32], bias1 / bias2 [K8] (optional).  Deterministic (fixed-order slab
 * reduce). */
size_t mlvae_skinny_dzw_workspace_size(int M, int K8);
int mlvae_skinny_dzw(int M, int K8, const void* A, int lda, const void* Wt, int ldw, const void* zb, int ldz, int Z,
                     float* dZ, int lddz, float* W, float* bias1, float* bias2, float* ws, size_t ws_bytes,
                     void* stream);
/* Fused VanillaVAE encoder (bf16; mlvae_encoder_supported: E == 64, Z == 32, F in {64, 80}).
 * Forward: FC(F->E) LReLU FC(E->E) LReLU -> [mu | log_var] -> z = eps exp(lv/2) + mu, with the
 * masked KL sums in kl_partials[mlvae_encoder_partials_count] (read by mlvae_elbo_finalize).
 * eps_in NULL: eps = Philox(seed, offset + n*Z + k) (the mlvae_randn stream) -> eps_out.
 * z_bf16 [B*T, z_ld]: z_ld = Z, or >= Z + 16 with columns Z..Z+15 = [1, 0, ...] (the ones column
 * of mlvae_skinny_tn's bias gradient).  e1/e2 bf16 [B*T, E] are kept for the backward.
 * Backward: from dz (the gradient reaching z) the reparam/KL gradient, both LReLU dgrads and the
 * six encoder weight/bias gradients (overwritten; fixed-order reduce over the workspace
 * mlvae_encoder_workspace_size).  Replaces ref:src/modules/vanilla_vae.py:13-45 and its autograd. */
int mlvae_encoder_supported(int F, int E, int Z);
int mlvae_encoder_partials_count(int B, int T);
size_t mlvae_encoder_workspace_size(int B, int T, int F, int E, int Z);
int mlvae_encoder_fwd(int B, int T, int F, int E, int Z, const float* x, const float* w0,
                      const float* b0, const float* w1, const float* b1, const float* wml,
                      const float* bml, const float* eps_in, unsigned long long seed,
                      unsigned long long offset, const float* lens, void* e1_bf16, void* e2_bf16,
                      float* ml, float* z, void* z_bf16, int z_ld, float* eps_out,
                      float* kl_partials, void* stream);
/* mlvae_encoder_fwd with split = 1: every forward product as a_hi W_hi + a_hi W_lo + a_lo W_hi
 * (bf16 hi + lo pairs of the fp32 x, activations and weights: mu / log_var / z / KL to ~1e-5 of
 * fp32 at the same HBM traffic; e1 / e2 are still saved bf16).  split = 0 is mlvae_encoder_fwd. */
int mlvae_encoder_fwd_ex(int B, int T, int F, int E, int Z, const float* x, const float* w0,
                         const float* b0, const float* w1, const float* b1, const float* wml,
                         const float* bml, const float* eps_in, unsigned long long seed,
                         unsigned long long offset, const float* lens, void* e1_bf16, void* e2_bf16,
                         float* ml, float* z, void* z_bf16, int z_ld, float* eps_out,
                         float* kl_partials, int split, void* stream);
int mlvae_encoder_bwd(int B, int T, int F, int E, int Z, const float* dz, const float* ml,
                      const float* eps, const void* e1_bf16, const void* e2_bf16, const float* x,
                      const float* wml, const float* w1, const float* lens, const int* count,
                      float kl_scale, float* dwml, float* dbml, float* dw1, float* db1, float* dw0,
                      float* db0, float* ws, size_t ws_bytes, void* stream);
/* Data parallel: the step's scalars in a 4-float header before the flat gradient, summed by the
 * last gradient bucket's all-reduce (one collective instead of a loss-sum and an err-max).  pack =
 * 1: hdr = [loss3 | err != 0]; pack = 0 (after the sum): loss3 = hdr[0..2], err = 1 when any rank
 * set it.  ref:src/prepare_experiment.py:12,55 (SpeechBrain run_opts data parallel), the loss
 * sync of ref:src/models/md_model.py:77-88 fit_batch. */
int mlvae_dp_scalars(int pack, float* hdr, float* loss3, int* err, void* stream);
/* out[3] = {kld_loss, recon_loss, w_kl*kld + w_rec*recon}
 * (ref:src/utils/data_utils.py:67-104, ref:src/models/md_model.py:189-213). */
int mlvae_elbo_finalize(const float* kl_partials, int nk, const float* rec_partials, int nr,
                        const float* lens, const int* count, int B, int T, int Z, int F,
                        float w_kl, float w_rec, float* out, void* stream);
/* count (optional, device int) overrides the valid-frame count derived from lens: a
 * data-parallel shard passes the all-reduced global count so that its loss/gradients are
 * its exact share of the global masked mean (SURVEY.md 8(e)(i)). */
int mlvae_count_frames(const float* lens, int B, int T, int* out, void* stream);
/* eps ~ N(0,1) from Philox-4x32-10(seed, offset + i): shard-invariant reparameterisation noise
 * (replaces torch.randn_like at ref:src/modules/vanilla_vae.py:39). */
int mlvae_randn(size_t n, unsigned long long seed, unsigned long long offset, float* out,
                void* stream);
/* apply_lens_to_loss(loss[B,T,C], lens, reduction 0 mean / 1 batchmean / 2 batch);
 * out holds 2*B floats (results first). */
int mlvae_masked_mean(int B, int T, int C, const float* loss, const float* lens, int reduction,
                      float* out, void* stream);

/* InputNormalization(norm_type='global') inside the fused step: SpeechBrain's normaliser
 * (un-vendored; parity unpinned, restated in brain/features.py), built at
 * ref:src/models/test_vanilla_vae/model.yaml:14-15 and applied at
 * ref:src/models/test_vanilla_vae/model.py:24-25.  F % 4 == 0, 16-byte aligned buffers.
 *   stats:  per-utterance mean / std over the first round(rel_len*T) frames -> utt_stats [B][2F];
 *           sums [2F+1] = the sums of those over the utterances with frames, and their count
 *           (what a data-parallel run all-reduces before the update)
 *   update: mode 0 keep, 1 set the global statistics to the batch's, 2 running average with
 *           weight w of the batch (epoch < update_until_epoch): g = w_old g + w_new cur
 *   apply:  out = (x - glob_mean) / glob_std over rows x F */
int mlvae_norm_supported(int F);
int mlvae_norm_stats(int B, int T, int F, const float* x, const float* rel_lens, float* utt_stats,
                     float* sums, float eps, void* stream);
int mlvae_norm_update(int F, const float* sums, float* glob_mean, float* glob_std, int mode,
                      float w_old, float w_new, void* stream);  /* mode 2: w_old = 1 - w, w_new = w */
int mlvae_norm_apply(size_t rows, int F, const float* x, const float* glob_mean, const float* glob_std,
                     float* out, void* stream);

/* check_gradients + Adam (ref:src/models/md_model.py:82-86, model.yaml:45-47). */
int mlvae_sumsq_partials_count(size_t n);
int mlvae_grad_sumsq(const float* grads, size_t n, double* partials, void* stream);
/* advance: 1 = single-tensor step (prologue + update + step counter); for a multi-tensor
 * step over several buffers call with 0 for the first, -1 (reuse the prologue's hyp) for the
 * middle ones and 1 for the last (which advances the device step counter). */
int mlvae_adam_step(float* params, float* exp_avg, float* exp_avg_sq, const float* grads,
                    size_t n, const double* partials, int nparts, const float* loss, int* step,
                    int* nonfinite, float lr, float beta1, float beta2, float eps,
                    float max_norm, float* norm_out, float* hyp_scratch, int advance,
                    void* stream);
/* As mlvae_adam_step, plus the persistent recurrences' hand-off timeout word `err` (optional):
 * while *err != 0 the update is skipped (parameters and Adam state untouched, step counter not
 * advanced) and *err_skips (optional) counts the skipped steps, apart from non-finite losses. */
int mlvae_adam_step_ex(float* params, float* exp_avg, float* exp_avg_sq, const float* grads,
                       size_t n, const double* partials, int nparts, const float* loss, int* step,
                       int* nonfinite, const int* err, int* err_skips, float lr, float beta1,
                       float beta2, float eps, float max_norm, float* norm_out, float* hyp_scratch,
                       int advance, void* stream);

/* clip_grad_norm_ over several separately stored grads: every grad's sum-of-squares
 * partials go to one buffer (offsets), then each grad is scaled by min(max/(total+1e-6),1). */
int mlvae_clip_scale(float* grads, size_t n, const double* partials, int nparts, float max_norm,
                     float* norm_out, void* stream);

/* module-level autograd helpers: dx = dy * lrelu'(y); d apply_lens_to_loss / d loss */
int mlvae_lrelu_bwd(size_t n, const float* dy, const float* y, float* dx, void* stream);
int mlvae_masked_mean_bwd(int B, int T, int C, const float* lens, int reduction, const float* g,
                          float* dloss, void* stream);

/* bias gradients: out[c] = beta*out[c] + sum_n in[n][c]; out2 (optional) gets a copy. */
size_t mlvae_colsum_workspace_size(int N, int C);
int mlvae_colsum(int N, int C, const float* in, int ld, float* out, float* out2, float beta,
                 float* ws, size_t ws_bytes, void* stream);
/* the same over an fp32 (in_bf16 = 0) or bf16 (in_bf16 = 1) input */
int mlvae_colsum_ex(int N, int C, const void* in, int in_bf16, int ld, float* out, float* out2,
                    float beta, float* ws, size_t ws_bytes, void* stream);

/* y = x * mask; mask = given (already scaled) or Philox(seed, i) keep-prob 1-p scaled 1/(1-p).
 * Inter-layer dropout of nn.LSTM in train mode (ref:src/modules/decoder.py:14). */
int mlvae_dropout(size_t n, const float* x, float* y, const float* mask,
                  unsigned long long seed, float p, void* stream);
/* the same writing y (fp32, may be NULL) and/or y_bf16 (bf16, may be NULL); element i takes the
 * mask of index offset + i (offset a multiple of 4): a data-parallel shard passes the global
 * index of its first element, so every rank count draws the single-GPU run's masks */
int mlvae_dropout_ex(size_t n, const float* x, float* y, void* y_bf16, const float* mask,
                     unsigned long long seed, unsigned long long offset, float p, void* stream);

/* GMM-VAE latent block (SURVEY 8(f) rank 1; replaces ref:src/modules/gmm_vae.py:24-67).
 * P = the five heads as one stacked GEMM output, rows of width >= 4*N*Z + N:
 * [prior_mean | prior_log_var | mean | log_var] (N*Z each), then the N gmm logits.
 * Forward: z = eps*exp(lv/2) + mean; kl = -0.5(1 + lv - plv - (e^lv + (m-pm)^2)/(e^plv + 1e-5));
 * w = hard Gumbel-softmax(logits, tau) (straight-through value), ysoft = its soft sample.
 * expo = the Exp(1) draws [rows, N] or NULL: Philox(seed, offset + r*N + n) (ref :31).
 * Backward: dP from dz, dkl, dw (each NULL = 0); logits get the straight-through gradient. */
int mlvae_gmm_latent_fwd(int rows, int N, int Z, const float* P, int ldp, const float* eps,
                         const float* expo, unsigned long long seed, unsigned long long offset,
                         float tau, float* z, float* kl, float* w, float* ysoft, void* stream);
int mlvae_gmm_latent_bwd(int rows, int N, int Z, const float* P, int ldp, const float* eps,
                         const float* ysoft, float tau, const float* dz, const float* dkl,
                         const float* dw, float* dP, int lddp, void* stream);
/* apply_weight (ref:src/utils/data_utils.py:32-64): y[r,c] = sum_n w[r,n] x[r, n*C + c];
 * backward dx[r, n*C + c] = w[r,n] dy[r,c] and dw[r,n] = sum_c dy[r,c] x[r, n*C + c]
 * (dx or dw may be NULL). */
int mlvae_apply_weight_fwd(int rows, int N, int C, const float* x, int ldx, const float* w,
                           float* y, int ldy, void* stream);
int mlvae_apply_weight_bwd(int rows, int N, int C, const float* x, int ldx, const float* w,
                           const float* dy, int lddy, float* dx, int lddx, float* dw,
                           void* stream);

#ifdef __cplusplus
}
#endif
#endif

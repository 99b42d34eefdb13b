/*
 * statecatcher.h — C ABI of libstatecatcher_hip.so, the MI355X (gfx950) hot path of the
 * stateful recurrent ASR step (LucyRNN scan fwd/bwd, decay scan, CTC alpha-beta, greedy
 * CTC decode).
 *
 * Every entry point takes plain device pointers, element counts/strides (in ELEMENTS, as the
 * reference's Triton launches do) and a hipStream_t passed as void*.  No torch types cross
 * this boundary.  All calls are asynchronous on `stream` and never synchronise the host.
 *
 * Return value: 0 on success; SC_EINVAL (-1) for an invalid argument (message in
 * sc_last_error()); a positive hipError_t if the launch failed.
 *
 * Reference interfaces replaced (paths under speechcatcher-asr/statecatcher):
 *   sc_lucy_scan_fwd  <- lucyrnn_triton.py:179-244 `rnn_forward_unfused_rmsnorm`,
 *                        launched at lucyrnn_triton.py:61-73 with grid (B, D)
 *   sc_lucy_scan_bwd  <- (absent in the reference) adjoint of the above
 *   sc_decay_scan_fwd <- lucyrnn_triton.py:158-177 `fused_decay_scan`, launched at
 *                        lucyrnn.py:147-151; generalised with an optional initial state
 *   sc_decay_scan_bwd <- (absent) adjoint of the above
 *   sc_layernorm_*    <- nn.LayerNorm between layers, lucyrnn_triton.py:96-97, :136-137
 *   sc_ln_fold_*, sc_lucy_scan_*_ln <- the same LayerNorm folded into the next layer's gate
 *                        projection (LN(h) W^T + b = rstd (h W''^T - mean r) + b')
 *   sc_ctc_*          <- ATen ctc_loss behind nn.CTCLoss(blank=0, zero_infinity=True),
 *                        train.py:142 / model.py:68-71
 *   sc_ctc_greedy_decode <- decoder.py:3-30 `ctc_greedy_decoder`
 *   sc_ctc_greedy_step   <- decoder.py:3-30 applied one frame at a time (streaming)
 *   sc_ctc_greedy_frames <- the same over a block of frames in one launch
 *   sc_fbank          <- make_frontend (model.py:250-279, applied at train.py:473-475):
 *                        torchaudio MFCC / MelSpectrogram + AmplitudeToDB (unpinned, absent)
 *   sc_lucy_step_*    <- the native LucyRNN's infer-mode frame loop, lucyrnn.py:172-184, i.e.
 *                        LucyRNNCell.forward (lucyrnn.py:44-70) at T = 1 (streaming decode)
 *   sc_mlstm_*        <- the xLSTM encoder's mLSTM cell (model.py:214-229, :301-307; fork kernels
 *                        "chunkwise--native_autograd", train.py:643-645), math as
 *                        transformers/models/xlstm/modeling_xlstm.py:74-386 (parity vs the fork
 *                        unpinned)
 *   sc_rnnt_*         <- warp_rnnt `rnnt_loss(log_probs, labels, frames_lengths, labels_lengths,
 *                        blank, compact, gather=True)` called at model.py:97-105 (train.py:38-42,
 *                        :144); the log_softmax of model.py:93 optionally fused
 */
#ifndef STATECATCHER_H
#define STATECATCHER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SC_EINVAL (-1)

/* element types of floating tensors crossing the ABI */
#define SC_F32 0
#define SC_BF16 1
#define SC_F16 2

/* ABI version; bumped on any signature change */
int sc_abi_version(void);

/* Message for the last SC_EINVAL / launch failure on this thread ("" if none). */
const char* sc_last_error(void);

/* ---------------------------------------------------------------- LucyRNN scan ---------- */

/* Time steps per checkpointed super-chunk (state saved at each super-chunk start). */
int sc_lucy_scan_chunk(void);

/* Floats needed for the forward->backward state checkpoint: B * ceil(T/chunk) * 2 * D. */
int64_t sc_lucy_scan_ckpt_numel(int B, int T, int D);

/*
 * Forward scan.  Mirrors rnn_forward_unfused_rmsnorm(gates_ptr, h0_ptr, s0_ptr, out_ptr,
 * s_out_ptr, B, T, D, stride_g_bt, stride_g_td, stride_g_cd, stride_o_bt, stride_o_bd)
 * (lucyrnn_triton.py:180-194), plus one stride the reference does not have:
 *   gates  gate g (order r,z,k,v,h_pre,decay,alpha) of hidden unit d at step t of row b is at
 *            b*stride_g_bt + t*stride_g_td + g*stride_g_cd + (d/64)*stride_g_cb + d%64
 *          i.e. hidden units come in 64-wide column blocks.  The reference's [B,T,7,D] layout
 *          is stride_g_cb = 64.  The step-blocked layout [B,T,ceil(D/64),7,64] (stride_g_cd = 64,
 *          stride_g_cb = 448; what a projection GEMM writes when its weight rows are permuted
 *          accordingly) puts each step's 7 x 64 gates of one column block in one contiguous
 *          run, which the kernel streams in whole 16-byte pieces.
 *   gate_bias  NULL (gates already include the projection bias, as in the reference), or fp32
 *          [7,D] (logical order g*D + d) added to every step's gates on load (lets the
 *          projection GEMM skip its bias epilogue; the backward then needs the same pointer)
 *   h0,s0  [B,D] fp32 contiguous (read exactly as contiguous; the caller must not pass the
 *          strided out[:, -1] view the reference passes — SURVEY F3)
 *   out    [B,T,D] of gates_dtype, d-stride 1 (strides stride_o_bt, stride_o_bd)
 *   s_out  [B,D] fp32 contiguous: state after the last step
 *   h_out  NULL, or [B,D] fp32 contiguous: h after the last step in fp32 (the reference carries
 *          out[:, -1] in x.dtype = fp32; with a 16-bit out this keeps the carry unrounded)
 *   ckpt   NULL, or sc_lucy_scan_ckpt_numel() floats: (s,h) at every super-chunk start,
 *          consumed by sc_lucy_scan_bwd (training)
 * State arithmetic is fp32 for every gates_dtype.  Any element strides work; 16-byte aligned
 * gates with strides (and D) in multiples of 16 bytes take the wide-piece path.
 */
int sc_lucy_scan_fwd(const void* gates, int gates_dtype, const float* gate_bias,
                     const float* h0, const float* s0,
                     void* out, float* s_out, float* h_out, int B, int T, int D,
                     int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                     int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd, float* ckpt,
                     void* stream);

/*
 * sc_lucy_scan_fwd plus two 16-bit planes with out's strides: out_dup (the rounded h again) and
 * out_lo (h minus its rounding, rounded).  With out, out_dup, out_lo as the K blocks of one
 * [B*T][3D] operand, a bf16 GEMM against [W_hi | W_lo | W_hi] gives x.W with the error of an fp32
 * GEMM (the output projection before the CTC lattice, lucyrnn_triton.py:150 / model.py:70).
 * gates_dtype must be bf16 or f16.
 */
int sc_lucy_scan_fwd_split(const void* gates, int gates_dtype, const float* gate_bias,
                           const float* h0, const float* s0, void* out, void* out_dup, void* out_lo,
                           float* s_out, float* h_out, int B, int T, int D,
                           int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                           int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd,
                           float* ckpt, void* stream);

/*
 * sc_lucy_scan_fwd(_split) with the inter-layer LayerNorm (lucyrnn_triton.py:96-97, :136-137)
 * folded in.  16-bit gates, 16-byte pieces, D = 512 or 1024.  out_dup / out_lo: NULL, or the
 * split planes of sc_lucy_scan_fwd_split.
 *   ln_r       NULL, or fp32 [7,D]: this layer's gates are u = h W''^T of the RAW previous output h
 *              (W'' the bf16 image of sc_weight_images with col_scale = gamma, row_shift = the
 *              sc_ln_fold_prep shift) and r its row sums (sc_ln_fold_prep rowsum); each gate is
 *              rebuilt on load as rstd (u - mean r) + gate_bias, gate_bias = b' (sc_ln_fold_prep
 *              bias_out), which equals LN(h) W^T + b
 *   ln_rec_in  with ln_r: fp32 [B][T][D/64][2], (mean, M2) of h's 64-unit blocks (the previous
 *              layer's ln_rec_out); combined per row with Chan's formula, eps ln_eps
 *   ln_stat    NULL, or fp32 [B][T][2] out: the rows' (rstd, mean) (what sc_lucy_scan_bwd_ln and
 *              sc_ln_fold_bwd read)
 *   ln_rec_out NULL, or fp32 [B][T][D/64][2] out: (mean, M2) of this layer's 16-bit output
 *              values per 64-unit block, for the next layer's fold
 */
int sc_lucy_scan_fwd_ln(const void* gates, int gates_dtype, const float* gate_bias,
                        const float* h0, const float* s0, void* out, void* out_dup, void* out_lo,
                        float* s_out, float* h_out, int B, int T, int D,
                        int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                        int64_t stride_g_cb, int64_t stride_o_bt, int64_t stride_o_bd,
                        float* ckpt, const float* ln_r, const float* ln_rec_in, float* ln_stat,
                        float* ln_rec_out, float ln_eps, void* stream);

/*
 * Backward scan.  Inputs: the forward's gates and ckpt, dout = dL/d out (same dtype as gates,
 * strides stride_d_bt/stride_d_bd), ds_last = dL/d s_out (fp32 [B,D], may be NULL = zero).
 * Outputs: dgates (gates_dtype, laid out like gates with strides stride_dg_*), dh0, ds0 (fp32
 * [B,D]) and, if dbias is not NULL, dbias fp32 [B,7,D] = sum over t of the stored dgates (per
 * batch row; summing over b gives the gate-projection bias gradient without another pass over
 * dgates).
 */
int sc_lucy_scan_bwd(const void* gates, int gates_dtype, const float* gate_bias, const float* ckpt,
                     const void* dout, const float* ds_last,
                     void* dgates, float* dh0, float* ds0, float* dbias, int B, int T, int D,
                     int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                     int64_t stride_g_cb, int64_t stride_d_bt, int64_t stride_d_bd,
                     int64_t stride_dg_bt, int64_t stride_dg_td, int64_t stride_dg_cd,
                     int64_t stride_dg_cb, void* stream);

/*
 * Backward of sc_lucy_scan_fwd_ln's fold (16-bit, D = 512 or 1024, 16-byte aligned gates / dout /
 * dgates): the gates are rebuilt from ln_r, gate_bias and the forward's ln_stat; dgates =
 * dL/du = rstd dL/dgate (the input and weight gradients of u = h W''^T consume it); dbias keeps
 * dL/dgate (the gradient of b').  ln_r = NULL: the gates are sc_gemm_tn_ln_bf16's output, which
 * already holds rstd (u - mean r); the scan adds gate_bias (= b') alone, ln_stat is that GEMM's
 * stat, and dgates / dbias are as above.
 */
int sc_lucy_scan_bwd_ln(const void* gates, int gates_dtype, const float* gate_bias,
                        const float* ckpt, const void* dout, const float* ds_last, void* dgates,
                        float* dh0, float* ds0, float* dbias, int B, int T, int D,
                        int64_t stride_g_bt, int64_t stride_g_td, int64_t stride_g_cd,
                        int64_t stride_g_cb, int64_t stride_d_bt, int64_t stride_d_bd,
                        int64_t stride_dg_bt, int64_t stride_dg_td, int64_t stride_dg_cd,
                        int64_t stride_dg_cb, const float* ln_r, const float* ln_stat,
                        void* stream);

/* ---------------------------------------------------------------- decay scan ------------ */

/*
 * s_t = decay_t * s_{t-1} + kv_t with s_{-1} = init (init NULL -> 0, as fused_decay_scan).
 * Mirrors fused_decay_scan(kv_ptr, decay_ptr, output_ptr, B, T, D, stride_b, stride_t,
 * stride_d) (lucyrnn_triton.py:159-163); kv, decay and out share the strides, stride_d == 1.
 * init: fp32 [B,D] contiguous or NULL.  Accumulation fp32 (lucyrnn_triton.py:171).
 */
int sc_decay_scan_fwd(const void* kv, const void* decay, void* out, int dtype,
                      const float* init, int B, int T, int D,
                      int64_t stride_b, int64_t stride_t, int64_t stride_d, void* stream);

/*
 * Adjoint: g_t = dout_t + decay_{t+1} g_{t+1};  dkv_t = g_t;  ddecay_t = g_t * s_{t-1}
 * (s_{-1} = init).  s_all is the forward output.  dinit (fp32 [B,D]) may be NULL.
 */
int sc_decay_scan_bwd(const void* decay, const void* s_all, const void* dout, void* dkv,
                      void* ddecay, int dtype, const float* init, float* dinit,
                      int B, int T, int D, int64_t stride_b, int64_t stride_t, int64_t stride_d,
                      void* stream);

/* ---------------------------------------------------------------- LayerNorm ------------- */

/*
 * The stack's inter-layer nn.LayerNorm(D) (lucyrnn_triton.py:96-97, :136-137; eps 1e-5,
 * biased variance) in the activation dtype with fp32 statistics.  Rows of D contiguous
 * elements, 16-byte aligned; D must be 64 * (16 / element size) * {1, 2, 4, 8}
 * (sc_layernorm_supported).  gamma/beta fp32 [D]; mean/rstd fp32 [rows].
 */
int sc_layernorm_supported(int dtype, int D);
int sc_layernorm_fwd(const void* x, int dtype, const float* gamma, const float* beta, void* y,
                     float* mean, float* rstd, int64_t rows, int D, float eps, void* stream);

/* fp32 workspace floats needed by sc_layernorm_bwd (per-workgroup gamma/beta partial rows). */
int64_t sc_layernorm_bwd_workspace_numel(int64_t rows, int D);

/*
 * dx (dtype of x) and dgamma_dbeta fp32 [2, D] (row 0 dgamma, row 1 dbeta; fixed-order
 * reduction, deterministic) from x, dy and the forward's mean/rstd.
 */
int sc_layernorm_bwd(const void* x, const void* dy, int dtype, const float* gamma,
                     const float* mean, const float* rstd, void* dx, float* dgamma_dbeta,
                     float* workspace, int64_t rows, int D, void* stream);

/*
 * The LayerNorm fold around the scans (see sc_lucy_scan_fwd_ln).  Per job (one gate projection
 * W fp32 [rows = 7D][ld], the preceding LayerNorm's gamma / beta [D], the projection bias [rows]
 * or NULL), in one launch for up to 16 jobs:
 *   shift[n] = mean_k gamma_k W_nk   (row_shift of the W'' image; W''_nk = bf16(gamma_k W_nk -
 *                                     shift_n), computed unfused, as sc_weight_images computes it)
 *   bias_out[n] = b_n + sum_k W_nk beta_k
 *   rowsum[n] = sum_k W''_nk
 */
typedef struct {
  const float* w;
  const float* gamma;
  const float* beta;
  const float* bias;
  float* shift;
  float* bias_out;
  float* rowsum;
  int64_t ld, rows, D;
} sc_ln_fold_job;
int sc_ln_fold_prep(const sc_ln_fold_job* jobs, int njobs, void* stream);

/*
 * dL/dh [rows][D] bf16 of the LayerNorm input h from g = dL/du W'' (the gate projection's input
 * gradient with the scan's rstd-scaled dgates) and the forward's stat [rows][2] (rstd, mean):
 * dh = g - mean(g) - xhat mean(xhat g), xhat = (h - mean) rstd.  D = 512 or 1024.
 */
int sc_ln_fold_bwd(const void* g, const void* h, int dtype, const float* stat, void* dh,
                   int64_t rows, int D, void* stream);

/* fp32 workspace floats of sc_ln_fold_wgrad. */
int64_t sc_ln_fold_wgrad_workspace_numel(int rows, int D);

/*
 * From M = dL/dW'' fp32 [rows][D] (reference row order) and dL/db' fp32 [rows]:
 * dw [rows][D] = gamma (M - rowmean M) + dL/db' beta^T  (dL/dW), and dgamma_dbeta fp32 [2][D] =
 * (sum_n W (M - rowmean M), sum_n W dL/db') in a fixed order.  (dL/db = dL/db'.)
 */
int sc_ln_fold_wgrad(const float* M, const float* w, int64_t ld, const float* gamma,
                     const float* beta, const float* dbias, int rows, int D, float* dw,
                     float* dgamma_dbeta, float* workspace, void* stream);

/* ---------------------------------------------------------------- CTC ------------------- */

/* Workspace bytes for sc_ctc_fwd / sc_ctc_bwd (alpha, beta, row log-sum-exp, label chains). */
size_t sc_ctc_workspace_bytes(int B, int T, int max_target_len);

/*
 * CTC forward over x [B,T,V] (x_dtype, v-stride 1, strides stride_b/stride_t):
 *   is_logits = 1: x are logits, log_softmax is fused (model.py:70 + ATen ctc_loss);
 *   is_logits = 0: x are log-probabilities (the nn.CTCLoss input convention).
 * targets: int64 [B, max_target_len] padded (train.py:208), row stride target_stride;
 * max_target_len <= 1007.  in_lens/tgt_lens: int64 [B] device arrays.  Writes nll [B] fp32 (+inf when infeasible;
 * the zero_infinity reduction is the caller's) and fills the workspace for sc_ctc_bwd.
 */
int sc_ctc_fwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
               int64_t stride_b, int64_t stride_t,
               const int64_t* targets, int64_t target_stride, int max_target_len,
               const int64_t* in_lens, const int64_t* tgt_lens, int blank,
               float* nll, void* workspace, size_t workspace_bytes, void* stream);

/*
 * CTC backward: grad [B,T,V] (grad_dtype, contiguous) =
 *   scale[b] * (exp(lp) - exp(lcab + nll - lp))  for t < in_len[b], 0 otherwise,
 * ATen's formula; with is_logits = 1 it is the gradient w.r.t. the logits.  scale: fp32 [B]
 * (dL/dnll_b, already zero where the loss was zeroed).
 */
int sc_ctc_bwd(const void* x, int x_dtype, int is_logits, int B, int T, int V,
               int64_t stride_b, int64_t stride_t,
               const int64_t* targets, int64_t target_stride, int max_target_len,
               const int64_t* in_lens, const int64_t* tgt_lens, int blank,
               const float* nll, const float* scale, void* grad, int grad_dtype,
               const void* workspace, size_t workspace_bytes, void* stream);

/*
 * sc_ctc_fwd / sc_ctc_bwd with the emission columns given exactly (is_logits = 1): ex fp32
 * [B][T][max_target_len + 1] (strides ex_stride_b, ex_stride_t; column stride 1), ex[b][t][0] =
 * the blank's logit, ex[b][t][1 + u] = label u's, replace x's values at those columns in the
 * lattice's emissions and in the gradient row (softmax term and occupancy); the row's
 * log-sum-exp still reads x.  For a bf16 output projection whose emission columns were computed
 * to fp32 accuracy (statecatcher_amd.ops.CTCHeadFn): the same head, model.py:68-71 +
 * lucyrnn_triton.py:150, with the logits' bf16 rounding kept out of the lattice.
 */
int sc_ctc_fwd_ex(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                  int64_t stride_b, int64_t stride_t,
                  const int64_t* targets, int64_t target_stride, int max_target_len,
                  const int64_t* in_lens, const int64_t* tgt_lens, int blank,
                  const float* ex, int64_t ex_stride_b, int64_t ex_stride_t,
                  float* nll, void* workspace, size_t workspace_bytes, void* stream);
int sc_ctc_bwd_ex(const void* x, int x_dtype, int is_logits, int B, int T, int V,
                  int64_t stride_b, int64_t stride_t,
                  const int64_t* targets, int64_t target_stride, int max_target_len,
                  const int64_t* in_lens, const int64_t* tgt_lens, int blank,
                  const float* ex, int64_t ex_stride_b, int64_t ex_stride_t,
                  const float* nll, const float* scale, void* grad, int grad_dtype,
                  const void* workspace, size_t workspace_bytes, void* stream);

/*
 * The operand of the emission-logit GEMM of that head: out bf16 [B][max_target_len + 1][3 K],
 * row (b, c) = [bf16(w_r) | bf16(w_r - bf16(w_r)) | bf16(w_r)] with r = blank (c = 0) or
 * targets[b][c - 1] clamped into [0, V); bias_out fp32 [B][max_target_len + 1] = bias[r] (0 if
 * bias is NULL).  w fp32 [V][ldw], K % 4 == 0.  Against the last scan's [x_hi | x_hi | x_lo]
 * rows one bf16 GEMM gives the emission logits to ~2^-16 relative (lucyrnn_triton.py:150).
 */
int sc_ctc_split_rows(const float* w, int64_t ldw, const float* bias, int V, int K,
                      const int64_t* targets, int64_t target_stride, int max_target_len,
                      int blank, void* out, float* bias_out, int B, void* stream);

/*
 * The reduction nn.CTCLoss(reduction='mean', zero_infinity=True) applies to sc_ctc_fwd's nll
 * (train.py:142): loss[0] = mean_b(nll_b / max(U_b, 1)) with infinite nll_b counted as 0, and
 * factor[b] = d loss / d nll_b (0 for infinite nll_b), the `scale` sc_ctc_bwd takes times the
 * loss's upstream gradient.  nll, factor: fp32 [B]; tgt_lens int64 [B]; loss fp32 [1].
 */
int sc_ctc_mean(const float* nll, const int64_t* tgt_lens, int B, float* loss, float* factor,
                void* stream);

/* ---------------------------------------------------------------- greedy decode --------- */

/*
 * decoder.py:3-30 on device: argmax over V (first maximal index; NaN counts as maximal,
 * as torch.argmax), trim to lengths[b], collapse repeats, drop blank.
 * tokens: int32 [B,T] (first counts[b] entries valid), counts: int32 [B].
 */
int sc_ctc_greedy_decode(const void* log_probs, int dtype, int B, int T, int V,
                         int64_t stride_b, int64_t stride_t, const int64_t* lengths, int blank,
                         int32_t* tokens, int32_t* counts, void* stream);

/*
 * decoder.py:3-30 for ONE frame of B streams (streaming decode): tok = argmax of logits row b
 * (same tie/NaN rule); emit[b*emit_stride] = tok if the frame is live (mask null or mask[b] != 0)
 * and tok != blank and tok != prev[b], else -1; prev[b] = tok for live frames (start streams
 * with prev = -1, decoder.py's prev_token = None).  logits row stride stride_b (elements).
 */
int sc_ctc_greedy_step(const void* logits, int dtype, int B, int V, int64_t stride_b,
                       const float* mask, int blank, int32_t* prev, int32_t* emit,
                       int64_t emit_stride, void* stream);
/*
 * sc_ctc_greedy_step over F consecutive frames in one launch, frame f = 0 .. F-1 in order:
 * logits [F][B][V] (strides stride_f, stride_b), mask [F][B] (stride mask_f) or null, emit
 * [F][B] (strides emit_f, emit_b); prev carried from frame to frame as F calls would.
 */
int sc_ctc_greedy_frames(const void* logits, int dtype, int F, int B, int V, int64_t stride_f,
                         int64_t stride_b, const float* mask, int64_t mask_f, int blank,
                         int32_t* prev, int32_t* emit, int64_t emit_f, int64_t emit_b,
                         void* stream);

/* ---------------------------------------------------------------- streaming LucyRNN step -- */

/*
 * Native LucyRNN, infer mode, one frame (lucyrnn.py:172-184 -> LucyRNNCell.forward :44-70).
 * Per layer the caller runs a = input_proj(x) (GEMM), sc_lucy_step_ln (layernorm_in), the gate
 * GEMM, then sc_lucy_step_cell.  State h, s: fp32 [B,D] contiguous, updated in place.  All other
 * activations share `dtype` (f32/bf16/f16), rows contiguous except g (row stride g_stride).
 * 1 <= D <= 1024.  LayerNorm eps as given (nn.LayerNorm: 1e-5).
 */
int sc_lucy_step_supported(int dtype, int D);

/* y = LayerNorm(x; w, b) per row of D (layernorm_in, lucyrnn.py:45). */
int sc_lucy_step_ln(const void* x, int dtype, const float* w, const float* b, float eps, void* y,
                    int B, int D, void* stream);

/*
 * mode 0 (fused_ops, :47-54):  g = [z | k | v | h_pre | decay_logits] (5D per row; the
 *   reference's r chunk is computed and never used, so the caller drops W_fused's first D rows);
 *   s' = sigmoid(dl) s + k v;  c = tanh(LN_h(h_pre + s'));  h' = (1 - z~) c + z~ h with
 *   z~ = sigmoid(LN_z(z));  masked blend (:66-68) with mask[b];  out = new h.
 * mode 1 (unfused, :55-60):  g = [W_z u | W_k u | W_v u | W_decay u];  s updated as above;
 *   out = u + s' (the input of W_h).
 * mode 2 (unfused, :61-68):  hp = W_h(u + s');  c = tanh(LN_h(hp));  z~ from g as in mode 0;
 *   h updated and masked;  out = new h.
 * LayerNorm pointers null = layer_norm False (nn.Identity).  mask: fp32 [B] or null.
 */
int sc_lucy_step_cell(int mode, const void* g, int dtype, int64_t g_stride, const void* u,
                      const void* hp, const float* lnz_w, const float* lnz_b, const float* lnh_w,
                      const float* lnh_b, float eps, float* h, float* s, void* out,
                      const float* mask, int B, int D, void* stream);

/*
 * The same frame as a chain of fused kernels (csrc/lucy_frame.hip; no library GEMM, no separate
 * LayerNorm launch).  Activations fp32; weights fp32 (fp32 MFMA, the reference's arithmetic) or
 * bf16 (bf16 MFMA).  LayerNorm statistics travel as (n, mean, M2, -) float4 records, [nrec][B].
 *
 * sc_lucy_frame_gemm: y[b][j] = sum_k x~[b][k] w[j][k] + bias[j], x~ = x or, when ln_w is given,
 *   LayerNorm(x) from the nst_in records of st_in (lucyrnn.py:45 layernorm_in).  epi:
 *   0 plain; 1 plain + one statistics record of y per 32 columns into st_out ([ceil(N/32)][B]);
 *   2 unfused gates (N = 4D: z k v decay, lucyrnn.py:55-59): s' = sigmoid(decay) s + k v into s
 *     (masked), y = x~ + s' ([B][D], K == D), z ([B][D]), records of z per 16 units into st_z;
 *   3 fused gates (N = 5D: z k v h_pre decay; W_fused without its unused r rows, :47-53): s as
 *     above, y = h_pre + s', z, records of y into st_out and of z into st_z ([D/16][B] each).
 *   x 16-byte aligned with ldx % 4 == 0, K % 4 == 0; w 16-byte aligned with ldw % 8 == 0.
 * sc_lucy_frame_cellb: h = (1 - sigmoid(LN_z z)) tanh(LN_h hp) + sigmoid(LN_z z) h (masked,
 *   :61-68) in place, and out[b][:D] = h (the next layer's input).
 */
int sc_lucy_frame_gemm(int epi, const float* x, int64_t ldx, int K, const float* ln_w,
                       const float* ln_b, const void* st_in, int nst_in, float eps, const void* w,
                       int w_dtype, int64_t ldw, const float* bias, int B, int N, float* y,
                       int64_t ldy, void* st_out, float* z, void* st_z, float* s,
                       const float* mask, void* stream);
int sc_lucy_frame_cellb(const float* z, const void* st_z, int nst_z, const float* hp,
                        const void* st_h, int nst_h, const float* lnz_w, const float* lnz_b,
                        const float* lnh_w, const float* lnh_b, float eps, float* h, float* out,
                        int64_t ldo, const float* mask, int B, int D, void* stream);

/*
 * The same two kernels over up to 8 independent jobs in ONE launch each: a block of F frames of
 * an L-layer model runs as a wavefront over (frame, layer) -- stage tau computes layer l of frame
 * tau - l for every l at once, since layer l of frame j needs only layer l - 1 of frame j and
 * layer l of frame j - 1 -- so a block takes 4 (F + L - 1) launches instead of 4 F L (statecatcher
 * _amd/streaming.py).  Each job has the arguments of one sc_lucy_frame_gemm / _cellb call; the
 * jobs of one call share epi, w_dtype, eps and the presence of the LayerNorm prologue.
 */
typedef struct sc_frame_gemm_job {
  const float* x;
  int64_t ldx;
  int K;
  const float* ln_w;
  const float* ln_b;
  const void* st_in;
  int nst_in;
  const void* w;
  int64_t ldw;
  const float* bias;
  int B, N;
  float* y;
  int64_t ldy;
  void* st_out;
  float* z;
  void* st_z;
  float* s;
  const float* mask;
} sc_frame_gemm_job;
int sc_lucy_frame_gemm_multi(int epi, int w_dtype, float eps, const sc_frame_gemm_job* jobs,
                             int njobs, void* stream);
typedef struct sc_frame_cell_job {
  const float* z;
  const void* st_z;
  int nst_z;
  const float* hp;
  const void* st_h;
  int nst_h;
  const float *lnz_w, *lnz_b, *lnh_w, *lnh_b;
  float* h;
  float* out;
  int64_t ldo;
  const float* mask;
  int B, D;
} sc_frame_cell_job;
int sc_lucy_frame_cellb_multi(float eps, const sc_frame_cell_job* jobs, int njobs, void* stream);

/* ---------------------------------------------------------------- column sums ----------- */

/*
 * out[n] = sum_m x[m][n] in fp32, fixed summation order (deterministic), x row-major [M][ld]
 * (16-byte aligned rows) of dtype f32/bf16/f16.  The step's row reductions: the output
 * projection's bias gradient (dy.sum(0), lucyrnn_triton.py:8-25 Linear backward), split-K
 * weight-gradient partial sums, per-row gate-bias partials.  Optional block transpose of the
 * output index: with N = perm_a * perm_b * C, column (a, b, c) is written at (b, a, c)
 * (perm_a = perm_b = 1: identity).  workspace: sc_colsum_workspace_bytes(M, N) device bytes.
 */
size_t sc_colsum_workspace_bytes(int64_t M, int64_t N);
int sc_colsum(const void* x, int dtype, int64_t M, int64_t N, int64_t ld, int64_t perm_a,
              int64_t perm_b, float* out, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- weight-gradient GEMM -- */

/*
 * Split-L weight gradient of a projection: part[s] = A[Ls]^T B[Ls] (fp32 [I][J] slab per
 * L-split s) for A = dY bf16 [L][lda], B = X bf16 [L][ldb] — the backward of LinearSafe
 * (lucyrnn_triton.py:20-25: dW = dgates^T x) and of output_proj (lucyrnn_triton.py:107-109).
 * Sum the S slabs with sc_colsum (fixed order; it also un-permutes step-blocked rows).
 * Needs L % 64 == 0, J % 256 == 0, and I % 256 == 0 -- or I % 224 == 0 only at the 256-workgroup
 * shape (I/224)*(J/256)*8 == 256 (e.g. I = 3584 = 7 * 512 with J = 512) -- plus 16-byte aligned
 * operands and leading dimensions.  Gate on sc_gemm_wgrad_splits: it returns the split count
 * for a shape, 0 when unsupported (use a library GEMM).  part: S * I * J floats.
 */
int sc_gemm_wgrad_splits(int L, int I, int J);
int sc_gemm_wgrad_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, float* part, int L,
                       int I, int J, int S, void* stream);

/*
 * Frame-major projection GEMM C = A B^T, bf16 in / fp32 accumulate / bf16 out, for A [M][lda]
 * and B [N][ldb] both K-contiguous, C [M][ldc].  Replaces the library GEMMs of LinearSafe's
 * forward (lucyrnn_triton.py:20-25, gates = x W^T; layer 0's Din = 80 zero-padded to 128) and of
 * the input gradients (dx = dgates W as dgates (W^T)^T; output_proj's dh = dlogits Wo,
 * lucyrnn_triton.py:107-109).  Needs K % 64 == 0, N % 256 == 0, 16-byte aligned operands and
 * leading dimensions, every operand < 4 GiB.  tile_m: rows per tile, 0 (default 192), 128 or 192.
 * Deterministic (no atomics, fixed K order).  Returns 0, SC_EINVAL, or a HIP error code.
 */
int sc_gemm_tn_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc,
                    int M, int N, int K, int tile_m, void* stream);

/*
 * The gate projection of layers 1.. with the inter-layer LayerNorm folded in
 * (lucyrnn_triton.py:96-97 + :20-25: LinearSafe(LayerNorm(h))): C [M][ldc] bf16 =
 *   rstd (h W''^T - mean r) = LN(h) W^T - W beta      (the scan adds b' = b + W beta)
 * for H = the previous layer's RAW output [M][ldh] bf16 (K = D, the LayerNorm width), Wpp = the
 * W'' image [N][ldw] (sc_weight_images with a LayerNorm fold job, step-blocked rows), r [N] =
 * its row sums in the image's row order (sc_ln_fold_prep's rowsum, permuted like the rows).  Each
 * row's mean and rstd = 1 / sqrt(biased variance + eps) come from the rows as they stream
 * through the GEMM; stat [M] (float pairs (rstd, mean)) receives them for the backward
 * (sc_lucy_scan_bwd_ln with ln_r = NULL, sc_ln_fold_bwd).  K % 64 == 0, N % 256 == 0, 16-byte
 * aligned operands.  Replaces sc_layernorm_fwd + the projection GEMM.
 */
int sc_gemm_tn_ln_bf16(const void* H, int64_t ldh, const void* Wpp, int64_t ldw, void* C,
                       int64_t ldc, int M, int N, int K, const float* r, void* stat, float eps,
                       void* stream);

/* ---------------------------------------------------------------- optimizer step -------- */

/*
 * clip_grad_norm_(params, max_norm) followed by torch.optim.Adam / AdamW's step
 * (train.py:543-552, :119-136), fp32 tensors of any length, one launch per pass:
 *   sc_adam_sumsq  sum of squares of the gradients of the clipped tensors into
 *                  part[sc_adam_parts(t, nt)] (fixed order, no atomics);
 *   sc_adam_step   coef = max_norm / (sqrt(sum part) + 1e-6) clamped to <= 1 (part = NULL: 1;
 *                  NaN propagates like torch.clamp), then per element: g *= coef; AdamW
 *                  (decoupled = 1) p *= 1 - lr wd, Adam g += wd p; m = lerp(m, g, 1 - beta1);
 *                  v = v beta2 + (1 - beta2) g g; p -= step_size m / (sqrt(v) / bc2_sqrt + eps),
 *                  step_size = lr / (1 - beta1^step), bc2_sqrt = sqrt(1 - beta2^step).
 *                  norm_out (optional, one float): the total norm clip_grad_norm_ returns.
 * The gradients are only read (p.grad keeps its unclipped values; the step loop discards them).
 * Up to 24 tensors go into one launch's argument table; longer lists take several launches.
 */
typedef struct {
  float* p;        /* parameter */
  const float* g;  /* gradient */
  float* m;        /* exp_avg */
  float* v;        /* exp_avg_sq */
  int64_t n;       /* elements */
} sc_adam_tensor;
int64_t sc_adam_parts(const sc_adam_tensor* t, int nt);
int sc_adam_sumsq(const sc_adam_tensor* t, int nt, float* part, void* stream);
int sc_adam_step(const sc_adam_tensor* t, int nt, const float* part, int64_t nparts,
                 double max_norm, double lr, double beta1, double beta2, double eps,
                 double weight_decay, int decoupled, double step_size, double bc2_sqrt,
                 float* norm_out, void* stream);

/*
 * Per-step bf16 images of the fp32 projection weights, one launch for up to 16 weights: the
 * autocast casts of LinearSafe (lucyrnn_triton.py:20-25 under train.py's autocast) plus the
 * layouts the GEMMs want.  Per job: dst bf16 [rows][cols_pad] = src rows (stride ld_src) with
 * zero columns cols..cols_pad-1, rows in step-blocked order (block, gate, unit) when block_d = D
 * > 0 (rows = 7 D, D % 64 == 0; dst row (b, g, u) = src row g D + 64 b + u); dst_t (optional)
 * bf16 [cols][rows] = dst's first cols columns transposed.  Round to nearest even.
 * col_scale [cols] / row_shift [rows] (either may be NULL): the imaged value is
 * col_scale[c] * src - row_shift[source row], computed unfused (the folded LayerNorm's W'',
 * sc_ln_fold_prep).
 */
typedef struct {
  const float* src;
  void* dst;
  void* dst_t;
  int64_t rows, cols, cols_pad, ld_src, block_d;
  const float* col_scale;
  const float* row_shift;
} sc_image_job;
int sc_weight_images(const sc_image_job* jobs, int njobs, void* stream);

/* ---------------------------------------------------------------- xLSTM block glue ------ */

/*
 * The xLSTM-large block's elementwise / row-norm glue (C4 encoder, model.py:214-229; structure
 * as transformers' modeling_xlstm.py:870-1205), one HBM pass each, bf16 tensors, fp32 math,
 * bf16 roundings where the torch module rounds.  Weight gradients come back as fp32 partial rows
 * [sc_xlstm_part_rows(rows)][D] for a fixed-order sum (sc_colsum).
 *   RMSNorm (force_float32_reductions): y = bf16(bf16(x rsqrt(mean x^2 + eps)) w), x/y [rows][D]
 *     contiguous, D in {256, 512, 768, 1024}; rstd fp32 [rows] saved for the backward.
 *   gated head LayerNorm: out[m][n DH + e] = bf16(bf16(sigmoid(o[m][n DH + e])) *
 *     bf16(LN(h[b][n][t][:])[e]) * w[n DH + e]), m = b T + t: MultiHeadLayerNorm of the mLSTM
 *     cell output in the cell's [B][NH][T][DH] layout times sigmoid of the output gate (a
 *     row-strided view, ldo); NH <= 4, DH in {64, 128, 192, 256}; mean/rstd fp32 [M][NH].
 *     Backward: dh in the cell layout, d o into a [M][lddo] view (the fused projection's
 *     gradient).
 *   SwiGLU: y = bf16(bf16(silu(g)) u) for a = [g | u] rows of 2F; the backward writes [dg | du].
 */
int sc_xlstm_part_rows(int64_t rows);
int sc_rmsnorm_fwd(const void* x, const float* w, void* y, float* rstd, int64_t rows, int D,
                   float eps, void* stream);
int sc_rmsnorm_bwd(const void* x, const void* dy, const float* w, const float* rstd, void* dx,
                   float* part, int64_t rows, int D, void* stream);
/* The block's residual add folded into the next RMSNorm (xLSTM block: x + y then norm_ffn, and
 * the previous block's x + ffn(..) then norm_mlstm; modeling_xlstm.py block forward):
 * s = bf16(x + r) (written) and y = RMSNorm(s) as sc_rmsnorm_fwd.  The backward takes s as its x
 * and adds the residual branch's gradient: dx = bf16(bf16(dRMSNorm) + dres), the sum autograd
 * forms for the two bf16 gradients of s. */
int sc_rmsnorm_add_fwd(const void* x, const void* r, void* s, const float* w, void* y, float* rstd,
                       int64_t rows, int D, float eps, void* stream);
int sc_rmsnorm_add_bwd(const void* s, const void* dy, const void* dres, const float* w,
                       const float* rstd, void* dx, float* part, int64_t rows, int D, void* stream);
int sc_mhln_gate_fwd(const void* h, const void* o, int64_t ldo, const float* w, void* out,
                     float* mean, float* rstd, int B, int T, int NH, int DH, float eps,
                     void* stream);
int sc_mhln_gate_bwd(const void* h, const void* o, int64_t ldo, const float* w, const float* mean,
                     const float* rstd, const void* dy, int64_t ldy, void* dh, void* dgo,
                     int64_t lddo, float* part, int B, int T, int NH, int DH, void* stream);
/* The same with h in f16 (an f16 mLSTM cell's output), each element rounded to bf16 on load as
 * h.to(bfloat16) would; dh is written in bf16. */
int sc_mhln_gate_fwd_h16(const void* h, const void* o, int64_t ldo, const float* w, void* out,
                         float* mean, float* rstd, int B, int T, int NH, int DH, float eps,
                         void* stream);
int sc_mhln_gate_bwd_h16(const void* h, const void* o, int64_t ldo, const float* w,
                         const float* mean, const float* rstd, const void* dy, int64_t ldy,
                         void* dh, void* dgo, int64_t lddo, float* part, int B, int T, int NH,
                         int DH, void* stream);
int sc_swiglu_fwd(const void* a, void* y, int64_t rows, int F, void* stream);
int sc_swiglu_bwd(const void* a, const void* dy, void* da, int64_t rows, int F, void* stream);

/* ---------------------------------------------------------------- feature frontend ------ */

/* Frames of a row of n_samples (center=False): 1 + (n - 400) / 160, or 0 below 400 samples. */
int64_t sc_fbank_frames(int64_t n_samples);
size_t sc_fbank_workspace_bytes(void);

/*
 * make_frontend(kind)(audio).transpose(1, 2) (model.py:250-279, train.py:473-475):
 * audio fp32 [B][audio_stride] (n_samples used per row) -> out fp32 [B][frames][80].
 * n_fft = win = 400 (periodic Hann), hop 160, center=False, power 2, 80 HTK mel bands over
 * [0, sample_rate/2], no filter normalisation.
 *   kind 0 (mfcc): log(mel + 1e-6), orthonormal DCT-II, 80 coefficients;
 *   kind 1 (mel):  10 log10(max(mel, 1e-10)), then max(x, max over the whole call - 80)
 *                  (AmplitudeToDB(top_db=80) on a (B, 80, frames) spectrogram).
 * workspace: sc_fbank_workspace_bytes() device bytes (kind 1 only).
 */
int sc_fbank(const float* audio, int B, int64_t n_samples, int64_t audio_stride, int kind,
             float sample_rate, float* out, void* workspace, size_t workspace_bytes, void* stream);

/* ---------------------------------------------------------------- mLSTM ----------------- */

/* 1 if the mLSTM kernels are compiled for this compute dtype (bf16/f16) and head dims. */
int sc_mlstm_supported(int dtype, int DQ, int DV);

/* Elements of the forward's chunk-start state image states_C: BH * (T/64) * DQ * DV. */
int64_t sc_mlstm_chunk_state_numel(int BH, int T, int DQ, int DV);

/*
 * mLSTM cell forward over BH = batch x heads independent sequences, chunkwise (chunk 64,
 * T % 64 == 0).  q, k [BH][T][DQ], v [BH][T][DV] of dtype (bf16 or f16; MFMA with fp32
 * accumulation); igate, fgate fp32 [BH][T] pre-activations; optional initial state c0 fp32
 * [BH][DQ][DV], n0 [BH][DQ], m0 [BH] (NULL = zeros).  Outputs: h [BH][T][DV] (dtype);
 * states_C = the stabilised state C~_k at every chunk START k < T/64, in dtype and TRANSPOSED
 * ([BH][T/64][DV][DQ]: exactly the operand image the forward's q C~_k MFMA consumes; the
 * backward's dq reads it);
 * states_n / states_m fp32 at every chunk boundary ([BH][T/64+1][DQ], [BH][T/64+1]; index T/64
 * is the final state); c_last fp32 [BH][DQ][DV] the final state C~ (the carried segment state);
 * m_rows, den_rows fp32 [BH][T] (the row stabiliser and normaliser, consumed by the backward).
 * One launch: each (sequence, 64-column block of C~) walks its chunks with the state in MFMA
 * accumulators (the fp32 chunk states are never written to HBM).  h_t = q~_t C_t / (max(|q~_t n_t|,
 * e^{-m_t}) + eps) with q~ = q DQ^-1/2.
 * layout (optional, 7 int64): {NH, qb, qh, qt, vb, vh, vt} element strides of q / k (and dq /
 * dk) and v (dv) with sequence bh = b NH + h at step t at (bh / NH) qb + (bh % NH) qh + t qt:
 * the xLSTM layer reads them in place from its fused projection output [B][T][N] (qh = DQ,
 * qt = N) and the backward writes the gradients into the projection's gradient the same way.
 * NULL = contiguous [BH][T][D].  Strides multiples of 8 elements, bases 16-byte aligned.
 */
int sc_mlstm_fwd(const void* q, const void* k, const void* v, int dtype, const float* igate,
                 const float* fgate, const float* c0, const float* n0, const float* m0, int BH,
                 int T, int DQ, int DV, float eps, void* h, void* states_C, float* states_n,
                 float* states_m, float* c_last, float* m_rows, float* den_rows,
                 const int64_t* layout, void* stream);

/*
 * Backward of sc_mlstm_fwd given dh (dtype, [BH][T][DV]) and optional gradients of the final
 * state (dcT fp32 [BH][DQ][DV], dnT [BH][DQ]; NULL = zero).  Outputs dq, dk, dv (dtype),
 * dstates_C / dstates_n fp32 [BH][DQ][DV] / [BH][DQ] = the gradient w.r.t. the INITIAL state
 * (c0, n0; the per-chunk state gradients never leave the chip: one 8-wave workgroup per
 * sequence walks the chunks in reverse with dC~ in MFMA accumulators), and the
 * per-step gate terms qdq = q_t.dq_t, kdk = k_t.dk_t (fp32 [BH][T]): d igate = kdk,
 * d fgate_t = sigmoid(-f_t) sum_{r>=t} (qdq_r - kdk_r).  The stabiliser is not differentiated.
 * layout: as sc_mlstm_fwd's; dq / dk / dv are written with the same strides as q / k / v.
 */
int sc_mlstm_bwd(const void* q, const void* k, const void* v, int dtype, const float* igate,
                 const float* fgate, const void* h, const void* dh, const float* dcT,
                 const float* dnT, const void* states_C, const float* states_n,
                 const float* states_m, const float* m_rows, const float* den_rows, int BH, int T,
                 int DQ, int DV, float eps, float* dstates_C, float* dstates_n, void* dq,
                 void* dk, void* dv, float* qdq, float* kdk, const int64_t* layout,
                 void* stream);

/*
 * sc_mlstm_fwd / sc_mlstm_bwd with the operands in another dtype than the cell computes in:
 * io_dtype is the dtype of q, k, v (and dh, dq, dk, dv); dtype the cell's MFMA dtype and that of h
 * and the chunk-state image.  Supported pairs: (bf16, bf16), (f16, f16), and (f16, bf16) -- the
 * reference's float16 cell (autocast_kernel_dtype, model.py:227) reading a bf16-autocast
 * model's projection in place, each operand rounded to f16 on load as .to(float16) would, and
 * the gradients rounded through f16 to bf16 as the split path's casts are.
 */
int sc_mlstm_fwd_io(const void* q, const void* k, const void* v, int dtype, int io_dtype,
                    const float* igate, const float* fgate, const float* c0, const float* n0,
                    const float* m0, int BH, int T, int DQ, int DV, float eps, void* h,
                    void* states_C, float* states_n, float* states_m, float* c_last,
                    float* m_rows, float* den_rows, const int64_t* layout, void* stream);
int sc_mlstm_bwd_io(const void* q, const void* k, const void* v, int dtype, int io_dtype,
                    const float* igate, const float* fgate, const void* h, const void* dh,
                    const float* dcT, const float* dnT, const void* states_C,
                    const float* states_n, const float* states_m, const float* m_rows,
                    const float* den_rows, int BH, int T, int DQ, int DV, float eps,
                    float* dstates_C, float* dstates_n, void* dq, void* dk, void* dv,
                    float* qdq, float* kdk, const int64_t* layout, void* stream);

/*
 * Gate gradients of the mLSTM cell from sc_mlstm_bwd's qdq / kdk (fp32 [BH][T], T % 64 == 0)
 * and the forget-gate pre-activations fgate (fp32 [BH][T], after any soft cap):
 *   d igate = kdk,  d fgate_t = sigmoid(-fgate_t) sum_{r >= t} (qdq_r - kdk_r).
 * Either dfgate != NULL (fp32 [BH][T]; d igate is kdk itself), or da != NULL: both gradients
 * through the xLSTM gate soft cap (cap > 0; cap <= 0 = none): g (1 - tanh(x / cap)^2) in fp32,
 * rounded once to bf16, written into the projection gradient da at [b][t][io + h] and
 * [b][t][fo + h] (row stride ld elements), a holding the raw bf16 pre-activations at the same
 * positions; sequence bh = b NH + h.
 */
int sc_mlstm_gate_bwd(const float* qdq, const float* kdk, const float* fgate, int BH, int T,
                      float* dfgate, const void* a, void* da, int NH, int64_t ld, int io, int fo,
                      float cap, void* stream);

/* ---------------------------------------------------------------- RNN-T ----------------- */

/* Workspace bytes for sc_rnnt_fwd / sc_rnnt_bwd (gathered log-probs, alpha, beta, offsets). */
size_t sc_rnnt_workspace_bytes(int B, int T, int max_labels);

/*
 * RNN-T negative log-likelihood over the transducer lattice (gather semantics: the blank and
 * next-label log-probs of every node (t, u), t < frames_lengths[b], u <= labels_lengths[b]).
 * x: node (b,t,u)'s V-row (v-stride 1) is at
 *   dense   (row_offsets == NULL): b*stride_b + t*stride_t + u*stride_u   ([B,T,max_labels+1,V])
 *   compact (row_offsets != NULL): (row_offsets[b] + t*(labels_lengths[b]+1) + u) * stride_u,
 *           the packed (sum_b T_b (U_b+1), V) layout of RNNTCompactPredictorJoiner (model.py:147-200)
 *   is_logits = 1: x are joiner logits, log_softmax fused; 0: x are log-probs.
 * labels: int64 [B, max_labels] (row stride label_stride); lengths: int64 [B] device arrays.
 * nll: fp32 [B] (+inf when frames_lengths[b] == 0).  max_labels <= 1023.
 */
int sc_rnnt_fwd(const void* x, int x_dtype, int is_logits, int B, int T, int max_labels, int V,
                int64_t stride_b, int64_t stride_t, int64_t stride_u, const int64_t* row_offsets,
                const int64_t* labels, int64_t label_stride, const int64_t* frames_lengths,
                const int64_t* labels_lengths, int blank, float* nll, void* workspace,
                size_t workspace_bytes, void* stream);

/*
 * Gradient of sum_b scale[b] * nll[b] w.r.t. x, written to grad (grad_dtype = fp32 or x_dtype,
 * same layout as x; dense rows outside the lattice are zeroed).  Logits: the softmax-corrected
 * row; log-probs: non-zero only at the blank and label entries (warp_rnnt gather=True).
 */
int sc_rnnt_bwd(const void* x, int x_dtype, int is_logits, int B, int T, int max_labels, int V,
                int64_t stride_b, int64_t stride_t, int64_t stride_u, const int64_t* row_offsets,
                const int64_t* labels, int64_t label_stride, const int64_t* frames_lengths,
                const int64_t* labels_lengths, int blank, const float* scale, void* grad,
                int grad_dtype, const void* workspace, size_t workspace_bytes, void* stream);

/*
 * Fused joiner + RNN-T loss (C5): RNNTPredictorJoiner.forward (model.py:129-145) -> fp32
 * log_softmax (model.py:93) -> the gathered lattice, without the (B, T, U+1, V) logits.
 *   enc   fp32 [B][T][J]       enc_proj(enc_out), contiguous
 *   pred  fp32 [B][U1][J]      pred_proj(embedding(blank-prefixed labels)), U1 = max_labels + 1
 *   W     bf16 [V][J]          joiner.weight (MFMA operand); bias fp32 [V] = joiner.bias
 * J must be 64 (train.py:639's --rnnt-joiner-dim default), V a multiple of 32, <= 1024.
 * Forward: nll fp32 [B] as sc_rnnt_fwd (same workspace, sc_rnnt_workspace_bytes).
 * Backward (after the forward, same workspace) of sum_b scale[b] nll[b], one pass over the
 * logits (the workgroups split the vocabulary; t_blocks and u_splits count those splits too):
 *   d_enc   fp32 [u_splits][B][T][J]   partials (sum them: d enc)
 *   d_pred  fp32 [B][t_blocks][U1][J]  partials (sum over t_blocks: d pred); zero-filled by
 *                                      the caller (columns outside the lattice are not written)
 *   dW      fp32 [slices][V][J], db fp32 [slices][V]: partials of sum_n dlogits_n z_n^T and
 *           sum_n dlogits_n, dlogits_n = a_n softmax_n - w_blank,n e_blank - w_label,n e_y,
 *           a_n = scale (occ_blank + occ_label) (sum them in a fixed order: d W, d bias)
 * t_blocks / u_splits / slices: sc_rnnt_joint_geometry.
 */
int sc_rnnt_joint_geometry(int B, int T, int max_labels, int V, int* t_blocks, int* u_splits,
                           int* slices);
int sc_rnnt_joint_fwd(const float* enc, const float* pred, const void* W, const float* bias, int B,
                      int T, int max_labels, int V, int J, const int64_t* labels,
                      int64_t label_stride, const int64_t* frames_lengths,
                      const int64_t* labels_lengths, int blank, float* nll, void* workspace,
                      size_t workspace_bytes, void* stream);
int sc_rnnt_joint_bwd(const float* enc, const float* pred, const void* W, const float* bias, int B,
                      int T, int max_labels, int V, int J, const int64_t* labels,
                      int64_t label_stride, const int64_t* frames_lengths,
                      const int64_t* labels_lengths, int blank, const float* scale, float* d_enc,
                      float* d_pred, float* dW, float* db, const void* workspace,
                      size_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* STATECATCHER_H */

/*
 * ssq.h -- C ABI of libssq.so, the MI355X (gfx950) kernels of the shifted-scale
 * PTQ calibration path.  Plain pointers and sizes only: every pointer is DEVICE
 * memory owned by the caller (PyTorch's caching allocator in the Python host layer),
 * borrowed for the duration of the call.  Launches are asynchronous on `stream`
 * (a hipStream_t passed as void*); no entry point allocates or synchronizes, and none
 * keeps state except the opt-in deferred-finalize queue (ssq_set_deferred_finalize), the
 * opt-in deferred prepared forward (ssq_set_deferred_prep_fwd), the opt-in deferred
 * multi-tensor q/dq (ssq_set_deferred_fq_multi) and the armed optimizer step
 * (ssq_adam_arm), so
 * every call is graph-capturable.
 *
 * Return value: 0 on success; a negative SSQ_E* code for an argument error; otherwise
 * the hipError_t of a failed launch.  ssq_last_error() returns a thread-local message.
 *
 * Streams and workspaces (every entry point): calls on one stream run in issue order;
 * calls on different streams may run concurrently provided no two calls in flight share a
 * workspace (`ws`) or an output buffer.  The library holds no device-global state: every
 * reduction's partials -- and the one in-launch last-arriver counter (the epilogue
 * backward's act-delta reduction, zeroed by the launch that writes its partials) -- live in
 * the call's own workspace, which needs no initialisation.  The host-state deferrals and
 * the armed step below are per stream but not thread-safe: issue them from one host thread.
 *
 * The reference (jai1215snu/ShiftedScaleQuantization) is pure PyTorch: it has no FFI.
 * Each entry point below replaces the eager-op sequence cited beside it; the reference
 * "binding" that calls it is the quantizer module's forward/backward, whose Python
 * mirror (shiftedscalequantization_amd.quant) calls this ABI through ctypes
 * (INTEGRATION.md shows the binding).
 *
 * Common geometry: a weight tensor is viewed as (Co, Ci, K) with K = kh*kw (K = 1 for
 * Linear).  "delta_per_ci" selects a delta of shape (Co,) (0) or (Co, Ci) (1, after
 * ChannelQuant.update_delta).  Quantized codes are written as one byte per element:
 * uint8 for asymmetric ranges, int8 (two's complement) for symmetric ones.
 */
#ifndef SSQ_H_
#define SSQ_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SSQ_OK 0
#define SSQ_E_ARG (-1)      /* invalid size / pointer / enum */
#define SSQ_E_WS (-2)       /* workspace too small */

typedef void* ssq_stream_t; /* hipStream_t */

const char* ssq_last_error(void);
int ssq_version(void);
/* Cache-policy variant of the streaming kernels (0 plain, 1 non-temporal); returns the
 * previous value.  Used by bench.py for A/B measurements only.                        */
int ssq_set_variant(int variant);

/* ---------------------------------------------------------------- K1/K2 uniform affine q/dq
 * UniformAffineQuantizer.forward (quant_layer.py:77-98), with round_ste (:18-22):
 *   d = delta[c]*scale; t = x/d; q = clamp((rint(t) - t) + t + zp[c], qmin, qmax);
 *   y = (q - zp[c]) * d
 * (rint(t) - t) + t == rint(t) for finite t and NaN at t = +-inf, as the reference's
 * round_ste; clamp keeps NaN (torch.clamp).  Element i belongs to channel
 * c = (i / inner) % nch   (nch == 1: per-tensor).                                     */
int ssq_fq_fwd(const float* x, float* y, void* codes_or_null, const float* delta,
               const float* zp, int64_t n, int64_t inner, int64_t nch, float scale,
               int qmin, int qmax, ssq_stream_t stream);
/* The same q/dq with plain torch.round (t = +-inf clamps to an edge): ChannelQuant
 * opt_mode 'none' (channelQuant.py:79-94), ChannelQuantAct 'none'
 * (channelQuantAct.py:56-67), AdaRound 'nearest' (adaptive_rounding.py:40-41).       */
int ssq_fq_round_fwd(const float* x, float* y, void* codes_or_null, const float* delta,
                     const float* zp, int64_t n, int64_t inner, int64_t nch, float scale,
                     int qmin, int qmax, ssq_stream_t stream);

/* Several tensors in ONE launch (e.g. every conv weight of a network): segment s is
 * the tensor x[s] (n[s] elements, inner[s] per channel, nch[s] channels). Per-channel
 * delta/zp of the tile a workgroup covers are staged in LDS. Arrays are HOST arrays of
 * length nseg; the pointers they hold are device pointers.                          */
int ssq_fq_fwd_multi(int nseg, const float* const* x, float* const* y,
                     const float* const* delta, const float* const* zp,
                     const int64_t* n, const int64_t* inner, const int64_t* nch,
                     const int* qmin, const int* qmax, ssq_stream_t stream);
/* With this deferral on, ssq_fq_fwd_multi (<= 48 segments) does not launch: it queues its
 * table on its stream, and the next per-tensor ssq_fq_fwd on that stream (float4 path, no
 * codes, the default streaming geometry) runs the table's tiles in extra workgroups of its
 * own launch -- e.g. an activation cache and every weight of a network quantized in one
 * launch (bench.py's step).  Same code: bit-identical outputs.  One table is queued at a
 * time (a second call launches the first); ssq_flush_fq_multi launches a table still queued
 * on `stream`.  The caller must not read the queued outputs before that launch or flush.
 * Host state, not thread-safe; ssq_set_deferred_fq_multi returns the previous setting;
 * turning it off launches a table still queued (on its own stream), and only a table queued
 * under deferral rides on a per-tensor launch. */
int ssq_set_deferred_fq_multi(int on);
int ssq_flush_fq_multi(ssq_stream_t stream);

/* STE backward of ssq_fq_fwd (autograd of quant_layer.py:92-98):
 *   gx = where(qmin <= rint(x/d)+zp <= qmax, gy*d, 0) / d
 *   gdelta[c] = sum gy*(q-zp) - sum g_int*((x/d)/d) ; gzp[c] = sum g_int - sum gy*d
 * gx / gdelta / gzp may each be NULL. Channel reductions are deterministic (fixed
 * order partials in `ws`, reduced in double).                                         */
size_t ssq_fq_bwd_workspace_size(int64_t n, int64_t inner, int64_t nch);
int ssq_fq_bwd(const float* x, const float* gy, const float* delta, const float* zp,
               int64_t n, int64_t inner, int64_t nch, int qmin, int qmax,
               float* gx, float* gdelta, float* gzp, void* ws, size_t ws_bytes,
               ssq_stream_t stream);
/* Backward of q/dq with torch.round instead of round_ste: ChannelQuantAct 'none' mode
 * (quant/channelQuantAct.py:56-67; x / (delta*shiftedScale) rounded with no gradient).
 * Pass delta = the fp32 product delta*shiftedScale.  The gradient wrt x is zero (not
 * written); gdelta = sum gy*(q - zp) is the gradient wrt that product (the caller scales
 * it by shiftedScale, the product's backward); gzp as ssq_fq_bwd.  Workspace as
 * ssq_fq_bwd.                                                                          */
int ssq_fq_round_bwd(const float* x, const float* gy, const float* delta, const float* zp,
                     int64_t n, int64_t inner, int64_t nch, int qmin, int qmax, float* gdelta,
                     float* gzp, void* ws, size_t ws_bytes, ssq_stream_t stream);
/* Per-tensor ssq_fq_bwd for an x that is a ReLU output, with the ReLU backward folded in:
 * gx is written at the ReLU's input (x <= 0 -> 0, torch threshold_backward on the output),
 * bit-identical to ssq_fq_bwd followed by ssq_relu_bwd.  Workspace as ssq_fq_bwd with
 * nch = 1.  Replaces the act quantizer's backward (quant_layer.py:92-98) + the ReLU's
 * (quant_block.py:117, QuantModule activation quant_layer.py:270).                     */
int ssq_fq_relu_bwd(const float* x, const float* gy, const float* delta, const float* zp,
                    int64_t n, int qmin, int qmax, float* gx, float* gdelta, float* gzp,
                    void* ws, size_t ws_bytes, ssq_stream_t stream);
/* The same for x a ReLU6 output (MobileNetV2's QuantInvertedResidual, quant_block.py:
 * 205-239): gx = 0 where x <= 0 or x >= 6 (torch hardtanh_backward).                  */
int ssq_fq_relu6_bwd(const float* x, const float* gy, const float* delta, const float* zp,
                     int64_t n, int qmin, int qmax, float* gx, float* gdelta, float* gzp,
                     void* ws, size_t ws_bytes, ssq_stream_t stream);

/* ---------------------------------------------------------------- K3/K4 scale init
 * init_quantization_scale (quant_layer.py:100-166) for `rows` independent rows of
 * `inner` elements (rows = Co for channel-wise weights, 1 for a per-tensor activation).
 * method 0 = 'max' (fp64 finalize exactly as the host Python; scale_flag = 'scale' in
 * scale_method), 1 = 'mse' (80 shrink candidates, mean |x-q|^2.4, first strict min).
 * Outputs delta, zp, raw_zp: `rows` floats each.  `scores_or_null` receives the
 * rows x 80 candidate scores (mse only) for inspection.                                */
size_t ssq_scale_init_workspace_size(int64_t rows, int64_t inner, int method);
int ssq_scale_init(const float* x, int64_t rows, int64_t inner, int n_bits, int sym,
                   int method, int scale_flag, float* delta, float* zp, float* raw_zp,
                   double* scores_or_null, void* ws, size_t ws_bytes, ssq_stream_t stream);

/* ---------------------------------------------------------------- K5-K9 ChannelQuant
 * Shift-candidate floors are recomputed in-kernel from W:  F_i = floor(W / (delta*s_i)).
 * alpha layout: conv (Ci, S); Linear (Co, Ci, S)  (is_fc = 1).  S <= 8.
 * `shifts` (the shiftTarget list) is a HOST array of S floats; every other pointer is
 * device memory.                                                                      */

/* ChannelQuant.init_v_beta (channelQuant.py:279-294, mode 0) / init_v (:201-213, mode 1)
 * + init_alpha (:158-199) + get_delta (:221-237).  init_alpha's squared error compares W
 * with the integer floors F_i (mode 0, the reference's quirk) or with the dequantized
 * 'none'-mode candidates at delta*s_i (mode 1, uses zp/qmin/qmax).  Writes alpha (init
 * logits), beta (W-shaped, mode 0; may be NULL) and the per-(Ci,S) (conv) / per-element
 * (fc) squared-error table mse_out (may be NULL).                                      */
size_t ssq_shift_init_workspace_size(int64_t Co, int64_t Ci, int64_t K, int S, int is_fc);
int ssq_shift_init(const float* W, const float* delta, const float* zp, const float* shifts,
                   int S, int64_t Co, int64_t Ci, int64_t K, int is_fc, int mode, int qmin,
                   int qmax, float* alpha, float* beta, float* mse_out, void* ws,
                   size_t ws_bytes, ssq_stream_t stream);

/* ChannelQuant.init_beta (channelQuant.py:300-307) / AdaRoundQuantizer.init_alpha
 * (adaptive_rounding.py:66-74): beta = -log((zeta-gamma)/(rest-gamma) - 1).           */
int ssq_rect_init(const float* W, const float* delta, int delta_per_ci, int64_t Co,
                  int64_t Ci, int64_t K, float* beta, ssq_stream_t stream);

/* ChannelQuant.get_delta (channelQuant.py:221-237): out (Co, Ci) = delta * s[argmax p].*/
int ssq_get_delta(const float* delta, const float* alpha, const float* shifts, int S,
                  int64_t Co, int64_t Ci, int is_fc, float* out, ssq_stream_t stream);

/* ChannelQuant.forward 'adaShift' (channelQuant.py:51-64, shifted_x_quant :96-118):
 *   Xf = hard_targets ? F_{argmax p} : sum_i F_i * p_i   (separate fp32 roundings)
 *   Q  = clamp(Xf + (hard_round ? [beta>=0] : h(beta)) + zp, qmin, qmax)
 *   What = (Q - zp) * delta                                                           */
int ssq_adashift_fwd(const float* W, const float* alpha, const float* beta,
                     const float* delta, const float* zp, const float* shifts, int S,
                     int64_t Co, int64_t Ci, int64_t K, int is_fc, int hard_targets,
                     int hard_round, int qmin, int qmax, float* What, void* codes_or_null,
                     ssq_stream_t stream);

/* Backward of the soft-target adaShift forward wrt alpha (and beta if gbeta != NULL).
 * Conv alpha gradients are reduced over (Co, K) deterministically in two fixed-order
 * stages through `ws` (ssq_adashift_bwd_workspace_size bytes; 0 for Linear).
 * Fused shift regulariser (layer_recon_fused_shiftedScale.py:281-282), applied when
 * lambda != 0:  reg = lambda * sum(1 - |2p-1|^b);  its gradient is added to galpha and
 * per-alpha-row values are written to reg_vals (may be NULL).  (lambda, b) come from
 * reg_lambda/reg_b, or from the DEVICE pair reg_dev[0..1] when reg_dev != NULL (the
 * graph-capturable form: the schedule changes every iteration).
 * galpha is OVERWRITTEN (not accumulated).                                             */
size_t ssq_adashift_bwd_workspace_size(int64_t Co, int64_t Ci, int64_t K, int S, int is_fc);
int ssq_adashift_bwd(const float* gWhat, const float* W, const float* alpha,
                     const float* beta, const float* delta, const float* zp,
                     const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K,
                     int is_fc, int hard_round, int qmin, int qmax, float reg_lambda,
                     float reg_b, const float* reg_dev, float* galpha, float* gbeta,
                     float* reg_vals, void* ws, size_t ws_bytes, ssq_stream_t stream);

/* Prepared adaShift (conv weights, S <= 4, K <= 256).  In the fused loop W, delta, the shifts
 * and beta are frozen (layer_recon_fused_shiftedScale.py:59-66) and the reference computes
 * its floor candidates x_q once (channelQuant.py:284-286).  ssq_adashift_prepare does that
 * once: fpack[e] = the S floors floor(W/(delta*s_i)) as int8 bytes (byte i) of one 32-bit
 * word, hterm[e] = h(beta) (hard_round: [beta >= 0]).  *overflow (device int, zeroed by the
 * caller) becomes nonzero if a floor does not fit int8 -- the caller then keeps
 * ssq_adashift_fwd/bwd.  The prepared forward / backward give the same What and alpha
 * gradients as ssq_adashift_fwd / ssq_adashift_bwd (beta frozen: no gbeta) while streaming
 * 12 B per weight each.  The _multi forms take nseg weights (e.g. every conv of a block,
 * same S) in ONE forward launch and TWO backward launches; arrays are indexed by segment.
 * The backward reduces over (Co, K) in two fixed-order stages through `ws`; galpha
 * OVERWRITTEN; regulariser as ssq_adashift_bwd (reg_vals may be NULL, or entries NULL). */
int ssq_adashift_prepare(const float* W, const float* beta, const float* delta,
                         const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K,
                         int hard_round, uint32_t* fpack, float* hterm, int* overflow,
                         ssq_stream_t stream);
int ssq_adashift_fwd_prepared(const uint32_t* fpack, const float* hterm, const float* alpha,
                              const float* delta, const float* zp, int S, int64_t Co,
                              int64_t Ci, int64_t K, int hard_targets, int qmin, int qmax,
                              float* What, ssq_stream_t stream);
int ssq_adashift_fwd_prepared_multi(int nseg, const uint32_t* const* fpack,
                                    const float* const* hterm, const float* const* alpha,
                                    const float* const* delta, const float* const* zp,
                                    const int64_t* Co, const int64_t* Ci, const int64_t* K,
                                    const int* qmin, const int* qmax, int S, int hard_targets,
                                    float* const* What, ssq_stream_t stream);
size_t ssq_adashift_bwd_prepared_workspace_size(int64_t Co, int64_t Ci, int64_t K, int S);
int ssq_adashift_bwd_prepared(const float* gWhat, const uint32_t* fpack, const float* hterm,
                              const float* alpha, const float* delta, const float* zp, int S,
                              int64_t Co, int64_t Ci, int64_t K, int qmin, int qmax,
                              float reg_lambda, float reg_b, const float* reg_dev,
                              float* galpha, float* reg_vals, void* ws, size_t ws_bytes,
                              ssq_stream_t stream);
size_t ssq_adashift_bwd_prepared_multi_workspace_size(int nseg, const int64_t* Co,
                                                      const int64_t* Ci, const int64_t* K, int S);
int ssq_adashift_bwd_prepared_multi(int nseg, const float* const* gWhat,
                                    const uint32_t* const* fpack, const float* const* hterm,
                                    const float* const* alpha, const float* const* delta,
                                    const float* const* zp, const int64_t* Co, const int64_t* Ci,
                                    const int64_t* K, const int* qmin, const int* qmax, int S,
                                    float reg_lambda, float reg_b, const float* reg_dev,
                                    float* const* galpha, float* const* reg_vals, void* ws,
                                    size_t ws_bytes, ssq_stream_t stream);

/* Shift-regulariser alone (value + gradient wrt alpha), for iterations where the
 * reconstruction gradient is not wanted.  mode 0: lambda*sum(1-|2p-1|^b)
 * (fused loss); mode 1: entropy lambda*-sum(p log(p+1e-10))
 * (layer_recon_shiftedScale.py:393,467).  galpha is ACCUMULATED (+=) if not NULL.     */
int ssq_shift_reg(const float* alpha, int S, int64_t rows, int mode, float lambda, float b,
                  float* galpha, float* reg_vals, ssq_stream_t stream);

/* 'learned_hard_sigmoid' (channelQuant.py:81-82): What = sum_i Xq_i * p_i (or Xq_{argmax})
 * where Xq_i are the DEQUANTIZED candidates of init_v (channelQuant.py:201-213), i.e.
 * 'none'-mode q/dq of W at delta*s_i, recomputed in-kernel.  galpha OVERWRITTEN.      */
int ssq_lhs_fwd(const float* W, const float* alpha, const float* delta, const float* zp,
                const float* shifts, int S, int64_t Co, int64_t Ci, int64_t K, int is_fc,
                int hard_targets, int qmin, int qmax, float* What, ssq_stream_t stream);
int ssq_lhs_bwd(const float* gWhat, const float* W, const float* alpha, const float* delta,
                const float* zp, const float* shifts, int S, int64_t Co, int64_t Ci,
                int64_t K, int is_fc, int qmin, int qmax, float* galpha, void* ws,
                size_t ws_bytes, ssq_stream_t stream);

/* 'adaround' mode (channelQuant.py:65-78) and AdaRoundQuantizer 'learned_hard_sigmoid'
 * (adaptive_rounding.py:38-67):  Q = clamp(floor(W/d) + (hard ? [beta>=0] : h(beta)) + zp)
 * What = (Q - zp)*d, d = delta*scale.  Backward gives gbeta (W-shaped, OVERWRITTEN); with
 * reg_lambda != 0 (or reg_dev != NULL: (lambda, b) read from that DEVICE pair, the
 * graph-capturable form) the gradient of the rounding regulariser
 * lambda*sum(1-|2h(beta)-1|^b) (block_recon.py:171-174) is added in the same pass.      */
int ssq_adaround_fwd(const float* W, const float* beta, const float* delta, int delta_per_ci,
                     const float* zp, float scale, int64_t Co, int64_t Ci, int64_t K,
                     int hard_round, int qmin, int qmax, float* What, void* codes_or_null,
                     ssq_stream_t stream);
int ssq_adaround_bwd(const float* gWhat, const float* W, const float* beta,
                     const float* delta, int delta_per_ci, const float* zp, float scale,
                     int64_t Co, int64_t Ci, int64_t K, int qmin, int qmax, float reg_lambda,
                     float reg_b, const float* reg_dev, float* gbeta, ssq_stream_t stream);
/* Several AdaRound weights (a block's quantizers) in one launch each way: arrays of nseg
 * (<= 8) per-weight arguments as in ssq_adaround_fwd / _bwd (scale, qmin, qmax per weight);
 * results bit-identical to one call per weight. */
int ssq_adaround_fwd_multi(int nseg, const float* const* W, const float* const* beta,
                           const float* const* delta, const int* delta_per_ci,
                           const float* const* zp, const float* scale, const int64_t* Co,
                           const int64_t* Ci, const int64_t* K, int hard_round, const int* qmin,
                           const int* qmax, float* const* What, ssq_stream_t stream);
int ssq_adaround_bwd_multi(int nseg, const float* const* gWhat, const float* const* W,
                           const float* const* beta, const float* const* delta,
                           const int* delta_per_ci, const float* const* zp, const float* scale,
                           const int64_t* Co, const int64_t* Ci, const int64_t* K, const int* qmin,
                           const int* qmax, float reg_lambda, float reg_b, const float* reg_dev,
                           float* const* gbeta, ssq_stream_t stream);

/* Rounding regulariser lambda*sum(1-|2h(v)-1|^b) over h = rect_sigmoid(v)
 * (layer_recon_fused_shiftedScale.py:278-279, block_recon.py:171-174,
 * layer_recon_shiftedScale.py:386-387).  loss_out: one float (deterministic).
 * gv (may be NULL) is ACCUMULATED (+=).                                               */
size_t ssq_round_reg_workspace_size(int64_t n);
int ssq_round_reg(const float* v, int64_t n, float lambda, float b, float* loss_out,
                  float* gv, void* ws, size_t ws_bytes, ssq_stream_t stream);

/* ---------------------------------------------------------------- K10 ChannelQuantMSE
 * init_scale 'max' mode (channelQuantMSE.py:203-241): per column j of W viewed as
 * (Co, J) keep the LAST candidate c = k/level (k = level..1) whose normalized codes
 * ((W/c)/delta + zero)/(2^b-1), zero = rint(raw_zp/delta), lie in the open range
 * (-0.5*thr/(2^b-1), 1+0.5*thr/(2^b-1)) over all Co.  inp_scale: J floats.           */
int ssq_inpscale_search(const float* W, const float* delta, const float* raw_zp,
                        int64_t Co, int64_t J, int n_bits, int level, float threshold,
                        float* inp_scale, ssq_stream_t stream);
/* ChannelQuantMSE.forward (channelQuantMSE.py:267-276). */
int ssq_inpscale_fwd(const float* W, const float* inp_scale, const float* delta,
                     const float* raw_zp, int64_t Co, int64_t J, int n_bits, float* What,
                     ssq_stream_t stream);

/* ---------------------------------------------------------------- K11 reconstruction loss
 * lp_loss (quant_layer.py:25-32) value and its gradient wrt pred in one pass:
 *   loss = sum |pred-tgt|^p / M ;  grad = gscale * ((1/M) * (p*|d|^(p-1)) * sgn(d))
 * M = n / C for reduction 'none' (sum over dim 1, mean over the rest), n for 'all'.
 * loss_out / grad / gscale (a DEVICE scalar, the upstream gradient) may each be NULL.
 * relu_mask != 0: pred is the output of a ReLU and grad is written at the ReLU's input
 * (grad = 0 where pred <= 0, torch's threshold_backward) -- the block's final ReLU
 * backward folded into the loss pass.  The loss reduction is deterministic: workgroup
 * partials in ws, summed in index order by a finalize launch (or task, with deferral on). */
size_t ssq_lp_loss_workspace_size(int64_t n);
int ssq_lp_loss(const float* pred, const float* tgt, int64_t n, int64_t M, float p,
                float* loss_out, float* grad, const float* gscale, int relu_mask, void* ws,
                size_t ws_bytes, ssq_stream_t stream);

/* ssq_lp_loss with the target rows read straight from the cached outputs: target element
 * i is tgt_cache[idx[i / row] * row + i % row] (the loop's cached_outs[idx] batch,
 * layer_recon_fused_shiftedScale.py:95-97, without materialising it).  n % row == 0,
 * n < 2^31.  Same values as ssq_gather_rows2 + ssq_lp_loss.                             */
int ssq_lp_loss_rows(const float* pred, const float* tgt_cache, const int64_t* idx, int64_t row,
                     int64_t n, int64_t M, float p, float* loss_out, float* grad,
                     const float* gscale, int relu_mask, void* ws, size_t ws_bytes,
                     ssq_stream_t stream);

/* ---------------------------------------------------------------- K14 batch gather
 * dst_k[r] = src_k[idx[r]] for two sources at once (cached block input and output,
 * layer_recon_fused_shiftedScale.py:95-97). src1/dst1 may be NULL.                    */
int ssq_gather_rows2(const float* src0, float* dst0, int64_t row0, const float* src1,
                     float* dst1, int64_t row1, const int64_t* idx, int64_t nidx,
                     ssq_stream_t stream);
/* The same gather with the indices read from `slot` (one iteration's row of a device ring
 * the host filled for several iterations at once: nidx indices, then the iteration's other
 * words) and slot[0:stage_words] copied to stage_dst in the same launch -- the static words
 * the iteration's later launches read (the loss rows' indices, Adam's step constants).  A
 * loop captured as several iterations per graph replay starts each with this launch
 * (quant/block_recon.py).                                                              */
int ssq_gather_rows2_staged(const float* src0, float* dst0, int64_t row0, const float* src1,
                            float* dst1, int64_t row1, const int64_t* slot, int64_t nidx,
                            int64_t* stage_dst, int64_t stage_words, ssq_stream_t stream);

/* ---------------------------------------------------------------- K19 fused fc iteration
 * One BRECQ AdaRound iteration of a Linear layer (the network's last layer: layer_recon.py
 * :10-104 with its LossFunction :107-170, adaptive_rounding.py:38-67, lp_loss p = 2,
 * quant_layer.py:25-32) in two launches: y = x[idx] What^T + bias and the loss gradient
 * g = dL/dy; then dW = g^T x[idx], V's gradient (AdaRound backward + the rounding
 * regulariser), V's Adam step (exp_avg / exp_avg_sq; ssq_adam's ops), What = AdaRound(W, V)
 * of the updated V for the next call (per-row delta / zp, soft rounding, clamp to
 * [qmin, qmax]; ssq_adaround_fwd's ops -- which also provides the first call's What), and
 * the loss value into loss_out.  `slot` (device) holds the bs batch indices (rows of
 * x_cache [N, Ci] and tgt_cache [N, Co]) followed by the iteration's words as fp32 pairs:
 * (lambda, b) of the regulariser, then Adam's (-lr/bc1, sqrt(bc2)).  g ([bs, Co]) is
 * scratch (and readable); gv_out may receive V's gradient.  1 <= bs <= 64, Ci a multiple
 * of 64 up to 4096; x_cache and What 16-B aligned.  fp32 MFMA (v_mfma_f32_16x16x4_f32):
 * the forward as 16 x 16 output tiles with the K range split over 8 waves, the weight
 * gradient as one 16 x 16 tile per wave; fixed summation orders.                      */
size_t ssq_fc_recon_workspace_size(int64_t Co, int64_t Ci, int64_t bs);
int ssq_fc_recon_iter(const float* x_cache, const float* tgt_cache, const int64_t* slot,
                      int64_t bs, const float* W, float* V, float* What, const float* delta,
                      const float* zp, int qmin, int qmax, const float* bias, int64_t Co,
                      int64_t Ci, float one_minus_beta1, float beta2, float one_minus_beta2,
                      float eps, float* exp_avg, float* exp_avg_sq, float* g, float* gv_out,
                      float* loss_out, void* ws, size_t ws_bytes, ssq_stream_t stream);

/* ---------------------------------------------------------------- K13 fused epilogue
 * QuantModule conv bias add (quant_layer.py:250), the block's residual add and ReLU
 * (quant_block.py:99-117) in one pass, in the reference's op order:
 *   out = act((y + bias[c]) + res),  c = (i / hw) % C,
 * act by the `relu` code of every K13 entry point: 0 identity, 1 ReLU, 2 ReLU6 (torch
 * clamp semantics: -0.0 and NaN kept).  bias / res may be NULL.  ssq_relu_bwd: gin =
 * out <= 0 ? 0 : g (torch's ReLU backward on its output); ssq_relu6_bwd: gin = 0 where
 * out <= 0 or out >= 6 (hardtanh_backward).  n < 2^31.                                   */
int ssq_bias_act(const float* y, const float* bias, const float* res, float* out, int64_t n,
                 int64_t hw, int64_t C, int relu, ssq_stream_t stream);
int ssq_relu_bwd(const float* g, const float* out, float* gin, int64_t n, ssq_stream_t stream);
int ssq_relu6_bwd(const float* g, const float* out, float* gin, int64_t n, ssq_stream_t stream);
/* F.max_pool2d forward, NCHW fp32, square K x K window (K <= 7), stride, pad <= K/2, no
 * dilation, floor mode: torch's rule (a larger value or a NaN replaces the running max, ties
 * keep the first, window walked row-major), bit-identical to torch.  The ResNet stem's pool
 * (models/resnet.py's maxpool after the stem; validation common.py:153-221). */
int ssq_maxpool2d_fwd(const float* x, float* y, int64_t N, int64_t C, int64_t H, int64_t W,
                      int64_t K, int64_t stride, int64_t pad, ssq_stream_t stream);
/* ssq_bias_act with the following per-tensor activation fake-quant (quant_layer.py:92-98,
 * applied at quant_layer.py:272 / quant_block.py:118) in the same pass:
 *   yq = (clamp(rint(out/delta[0]) + zp[0], qmin, qmax) - zp[0]) * delta[0]
 * bit-identical to ssq_bias_act + ssq_fq_fwd.  out (the pre-quant activation, needed only
 * by the backward) may be NULL: then the pass reads y (+res) and writes yq alone.        */
int ssq_bias_act_fq(const float* y, const float* bias, const float* res, float* out, float* yq,
                    int64_t n, int64_t hw, int64_t C, int relu, const float* delta,
                    const float* zp, int qmin, int qmax, ssq_stream_t stream);

/* The general epilogue: out = act(((y + bias[c]) * gamma[c] + phi[c]) + res), the
 * QuantModule's gamma^z/phi^z affine (quant_layer.py:266-267, learned with --bias_cal)
 * included, optionally followed by the per-tensor act fake-quant (yq; then out may be
 * NULL).  gamma/phi (both or neither), bias, res, delta/zp may be NULL.  Bit-identical to
 * the reference's separate fp32 ops.                                                     */
int ssq_epilogue_fwd(const float* y, const float* bias, const float* gamma, const float* phi,
                     const float* res, float* out, float* yq, int64_t n, int64_t hw, int64_t C,
                     int relu, const float* delta, const float* zp, int qmin, int qmax,
                     ssq_stream_t stream);
/* Its backward from g = dL/d(output), recomputing the pre-activation from y (NCHW, N x C
 * planes of hw): gy = g_t * gamma[c] (or g_t), gres = g_t, ggamma[c] = sum g_t*(y+bias[c]),
 * gphi[c] = sum g_t, gdelta/gzp as ssq_fq_bwd, where g_t is the act quantizer's STE and the
 * ReLU mask applied to g.  Every output may be NULL (gy: dL/dy not wanted, only the
 * per-channel / quantizer sums are produced).  Per-(n, c) partials in ws
 * (ssq_epilogue_bwd_workspace_size(N*C)), reduced in a fixed order.                     */
size_t ssq_epilogue_bwd_workspace_size(int64_t rows);
int ssq_epilogue_bwd(const float* g, const float* y, const float* bias, const float* gamma,
                     const float* phi, const float* res, int64_t N, int64_t C, int64_t hw,
                     int relu, const float* delta, const float* zp, int qmin, int qmax, float* gy,
                     float* gres, float* ggamma, float* gphi, float* gdelta, float* gzp, void* ws,
                     size_t ws_bytes, ssq_stream_t stream);
/* The fused tail of a reconstruction iteration: the block's final epilogue forward, the
 * reconstruction loss (power p: 2 in the shifted-scale loops, 2.4 in BRECQ's act phase)
 * against the cached target rows and the epilogue backward, in one pass
 * (layer_recon_fused_shiftedScale.py's quant_out -> lp_loss -> backward; block_recon.py's
 * act branch).  The output is recomputed from y with the forward's ops and never stored;
 * dL/d(output) is ssq_lp_loss_rows's gradient at the same p (mean over M) bit for bit; the
 * loss value Sum|out - tgt|^p / M (row partials summed in row order) goes to loss_out.
 * tgt_cache is [*, C, hw], idx holds the N cached rows of this batch.  Outputs and
 * workspace as ssq_epilogue_bwd.  res_bias / res_gamma+res_phi (any may be NULL; ReLU or
 * identity only): res is the raw output of the block's downsample conv and its own epilogue
 * (bias add, gamma^z/phi^z, no activation: ssq_epilogue_fwd's ops) is applied in the pass;
 * gres is then dL/d(that raw output) and gres_gamma / gres_phi its gamma / phi gradients --
 * bit-identical to running that epilogue forward and backward as two more passes. */
int ssq_epilogue_loss_bwd(const float* tgt_cache, const int64_t* idx, int64_t M, float p,
                          float* loss_out, const float* y, const float* bias, const float* gamma,
                          const float* phi, const float* res, const float* res_bias,
                          const float* res_gamma, const float* res_phi, int64_t N, int64_t C,
                          int64_t hw, int relu, const float* delta, const float* zp, int qmin,
                          int qmax, float* gy, float* gres, float* ggamma, float* gphi,
                          float* gres_gamma, float* gres_phi, float* gdelta, float* gzp,
                          void* ws, size_t ws_bytes, ssq_stream_t stream);
/* The three above reading y and / or res in place from per-sample row caches: with a map,
 * y / res is a [*, C, hw] cache and sample n of the batch is its row y_rows[n] / res_rows[n]
 * (either map may be NULL: that operand is the batch itself).  BRECQ's act phase hands its
 * frozen convs' precomputed outputs and the cached block input to the epilogues this way
 * instead of gathering a batch copy of each (block_recon.py:62-73's cached[idx]); the values
 * and their order are those of the gathered batch, so the results are bit-identical.       */
/* stage_dst (may be NULL): workgroup 0 also copies stage_n int64 words (<= 4096) from
 * stage_src to stage_dst -- a loop replaying several iterations per graph hands each
 * iteration's device words (a ring row, from which this launch takes its row maps) to the
 * static slot its later launches read, without a copy launch of its own.                  */
int ssq_epilogue_fwd_rows(const float* y, const int64_t* y_rows, const float* bias,
                          const float* gamma, const float* phi, const float* res,
                          const int64_t* res_rows, float* out, float* yq, int64_t n, int64_t hw,
                          int64_t C, int relu, const float* delta, const float* zp, int qmin,
                          int qmax, const int64_t* stage_src, int64_t* stage_dst,
                          int64_t stage_n, ssq_stream_t stream);
int ssq_epilogue_bwd_rows(const float* g, const float* y, const int64_t* y_rows,
                          const float* bias, const float* gamma, const float* phi,
                          const float* res, const int64_t* res_rows, int64_t N, int64_t C,
                          int64_t hw, int relu, const float* delta, const float* zp, int qmin,
                          int qmax, float* gy, float* gres, float* ggamma, float* gphi,
                          float* gdelta, float* gzp, void* ws, size_t ws_bytes,
                          ssq_stream_t stream);
int ssq_epilogue_loss_bwd_rows(const float* tgt_cache, const int64_t* idx, int64_t M, float p,
                               float* loss_out, const float* y, const int64_t* y_rows,
                               const float* bias, const float* gamma, const float* phi,
                               const float* res, const int64_t* res_rows,
                               const float* res_bias, const float* res_gamma,
                               const float* res_phi, int64_t N, int64_t C, int64_t hw, int relu,
                               const float* delta, const float* zp, int qmin, int qmax,
                               float* gy, float* gres, float* ggamma, float* gphi,
                               float* gres_gamma, float* gres_phi, float* gdelta, float* gzp,
                               void* ws, size_t ws_bytes, ssq_stream_t stream);

/* ---------------------------------------------------------------- Adam
 * torch.optim.Adam's single-tensor step (the reference's optimizer; block_recon.py:57-60,
 * layer_recon_fused_shiftedScale.py:57/73) over nseg parameter tensors in one launch:
 *   m = m + (1-b1)*(g-m);  v = v*b2 + ((1-b2)*g)*g;  p = p + (nss*m)/(sqrt(v)/bc2s + eps)
 * with nss = -lr/(1-b1^t), bc2s = sqrt(1-b2^t) taken from the DEVICE pair `hyper` when it
 * is not NULL (graph-capturable), else from the scalar arguments.  Arrays are HOST arrays
 * of length nseg holding device pointers.                                               */
int ssq_adam(int nseg, float* const* p, const float* const* g, float* const* m,
             float* const* v, const int64_t* n, float one_minus_beta1, float beta2,
             float one_minus_beta2, float eps, const float* hyper, float neg_step_size,
             float bias_correction2_sqrt, ssq_stream_t stream);
/* The same step, armed instead of launched: ssq_adam_arm records the nseg parameters
 * (p, m, v, n; hyper is required) for `stream`; the next prepared alpha backward on that
 * stream applies the step where each gradient is finalised -- the alpha segments of that
 * launch in their finalisers, gamma^z / phi^z (parameters whose gradients the epilogue
 * backward entry points of that stream produce) in their finalize tasks -- when it can
 * cover EVERY armed parameter, and attaches nothing otherwise.  Same update, same fp32
 * operations as ssq_adam: bit-identical.  ssq_adam_take returns 1 when the armed step ran
 * inside a launch (nothing left to do) and 0 when it did not (the caller launches ssq_adam);
 * either way it disarms.  The gradients are still written.  Host state, not thread-safe. */
int ssq_adam_arm(int nseg, float* const* p, float* const* m, float* const* v, const int64_t* n,
                 float one_minus_beta1, float beta2, float one_minus_beta2, float eps,
                 const float* hyper, ssq_stream_t stream);
int ssq_adam_take(ssq_stream_t stream);

/* ---------------------------------------------------------------- deferred finalizes
 * With deferral on, ssq_lp_loss[_rows] (loss value) and ssq_epilogue_bwd (gamma/phi and act
 * delta/zp gradients) queue their small finalize reduction on the stream instead of
 * launching it; the next ssq_epilogue_bwd or prepared alpha backward on that stream runs
 * the queue in extra workgroups of its own launch (same code and order: bit-identical).
 * ssq_adam, the lp_loss entry points and ssq_flush_finalize launch what is still queued.
 * The caller must give each producer's workspace a slot no other launch writes before the
 * flush, and must flush before reading a queued output on the host or with other kernels
 * (the reconstruction loop: deferral on for its body, flush at its end).  Host state,
 * not thread-safe.  ssq_set_deferred_finalize returns the previous setting; it launches
 * nothing (it takes no stream), so flush every stream with queued tasks before turning
 * deferral off. */
int ssq_set_deferred_finalize(int on);
int ssq_flush_finalize(ssq_stream_t stream);

/* ---------------------------------------------------------------- deferred prepared forward
 * The fused loop's iteration start in one launch (csrc/prep_ride.h).  With this deferral on,
 * ssq_adashift_fwd_prepared_multi (<= 8 segments) does not launch: it queues its table on
 * its stream, and the next ssq_gather_rows2 on that stream runs it in extra workgroups of
 * the gather launch (same code: bit-identical What).  One table is queued at a time (a second
 * call launches the first); ssq_flush_prep_fwd launches a table still queued on `stream`.
 * The caller must not read the queued What before that gather or flush.  Host state, not
 * thread-safe; ssq_set_deferred_prep_fwd returns the previous setting; turning it off
 * launches a forward still queued (on its own stream).  Replaces nothing in the reference: the iteration start of
 * layer_recon_fused_shiftedScale.py:94-100 (batch draw, then the quantized forward). */
int ssq_set_deferred_prep_fwd(int on);
int ssq_flush_prep_fwd(ssq_stream_t stream);

/* ---------------------------------------------------------------- K17 conv weight gradient
 * Deterministic fp32 conv weight gradient (NCHW, dilation 1) on the fp32 matrix cores:
 *   dw[co, ci, r, s] = sum_{n,oh,ow} dy[n, co, oh, ow] * x[n, g*Cig + ci, oh*st + r - pad,
 *                                                          ow*st + s - pad]
 * (the autograd of the reconstruction loops' F.conv2d weight, quant_layer.py:250, under
 * the reference's cudnn.deterministic = True, common.py:77-85).  Split-K partials in ws,
 * summed in a fixed order: bit-identical run to run.  OW <= 128, tensors < 2^31 elements. */
/* A/B knob (returns the previous value; out-of-range values only query): non-depthwise
 * weight-gradient form, 0 auto, 1 input-row-tile kernel (+ 1x1 GEMM), 2 im2col-DMA kernel,
 * 3 band kernel (3x3 / pad 1 / stride 1-2 / Cin, Cout multiples of 32; others as 1), 4 the
 * band kernel at 4 waves per workgroup instead of 8 (same bits). */
int ssq_conv_wgrad_set_form(int form);
/* The kernel ssq_conv_wgrad runs for a shape under the current form: 0 unsupported,
 * 1 input-row tile, 2 im2col-DMA, 3 band (16-byte staging), 4 1x1 GEMM, 5 depthwise
 * reduction, 6 band (4-byte staging: planes whose rows are not 16-B aligned). */
int ssq_conv_wgrad_kind(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                        int64_t S, int64_t stride, int64_t pad, int64_t groups);
size_t ssq_conv_wgrad_workspace_size(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co,
                                     int64_t R, int64_t S, int64_t stride, int64_t pad,
                                     int64_t groups);
int ssq_conv_wgrad(const float* x, const float* dy, int64_t Nb, int64_t C, int64_t H, int64_t W,
                   int64_t Co, int64_t R, int64_t S, int64_t stride, int64_t pad, int64_t groups,
                   float* dw, void* ws, size_t ws_bytes, ssq_stream_t stream);
/* The same weight gradient as one fp32 library GEMM (small output planes, where it beats
 * the band kernel): the two operands, written in one launch,
 *   dy2[co][n*P + p] = dy[n][co][p]                                  (Co x N*P)
 *   col[n*P + p][(ci*R + r)*S + s] = x[n][ci][oh*st+r-pad][ow*st+s-pad] (N*P x C*R*S, 0 outside)
 * with P = OH*OW; then dw = dy2 @ col (Co x C*R*S = dw's layout) by the caller's GEMM.
 * Either output may be NULL (with its input): the forward GEMM y2 = W @ col^T needs col
 * only, a backward with a saved col needs dy2 only.  Ungrouped convs; every operand
 * < 2^31 elements. */
int ssq_wgrad_gemm_operands(const float* x, const float* dy, int64_t Nb, int64_t C, int64_t H,
                            int64_t W, int64_t Co, int64_t R, int64_t S, int64_t stride,
                            int64_t pad, float* col, float* dy2, ssq_stream_t stream);
/* The im2col matrix col (N*OH*OW x C*R*S) of epilogue(y): y is the previous conv's raw
 * output and the epilogue the K13 one (ssq_epilogue_fwd's bias, gamma^z / phi^z, activation
 * and per-tensor act fake-quant, each optional: bias / gamma+phi / delta+zp may be NULL),
 * applied on the fly with the same fp32 ops -- col is bit for bit the im2col of the
 * materialised epilogue output, which is never written (ResNet BasicBlock conv1 -> conv2 on
 * the small planes: quant_layer.py:250-272 then conv2's F.conv2d, quant_block.py:99-117). */
int ssq_gemm_col_epilogue(const float* y, const float* bias, const float* gamma,
                          const float* phi, int relu, const float* delta, const float* zp,
                          int qmin, int qmax, int64_t Nb, int64_t C, int64_t H, int64_t W,
                          int64_t R, int64_t S, int64_t stride, int64_t pad, float* col,
                          ssq_stream_t stream);

/* ---------------------------------------------------------------- K18 depthwise conv
 * Depthwise (groups == C == Co) fp32 NCHW conv, dilation 1, R*S <= 25, zero padding:
 *   y[n,c,oh,ow] = sum_{r,s} w[c,r,s] * x[n,c,oh*st+r-pad, ow*st+s-pad]
 * and its input gradient dx (the same sum transposed).  The MobileNetV2 blocks' depthwise
 * F.conv2d of QuantModule.forward (quant_layer.py:250) and its autograd; one plane per
 * workgroup staged in LDS ((H+2pad)*(W+2pad)*4 <= 128 KiB).  Deterministic.           */
/* 1 when both the forward and the input-gradient plan of this depthwise shape fit the
 * 128 KiB LDS stage (weight rows + zero-padded / margined planes), else 0 -- the caller
 * then keeps MIOpen.                                                                    */
int ssq_dwconv_supported(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t R, int64_t S,
                         int64_t stride, int64_t pad);
int ssq_dwconv_fwd(const float* x, const float* w, float* y, int64_t Nb, int64_t C, int64_t H,
                   int64_t W, int64_t R, int64_t S, int64_t stride, int64_t pad,
                   ssq_stream_t stream);
int ssq_dwconv_bwd_data(const float* dy, const float* w, float* dx, int64_t Nb, int64_t C,
                        int64_t H, int64_t W, int64_t R, int64_t S, int64_t stride, int64_t pad,
                        ssq_stream_t stream);

/* ---------------------------------------------------------------- K15/K16 packed export
 * Low-bit weight export (replaces the fp32 state_dict + pickled shift
 * choice of main_cifar10.py:86 / myScaledMethods.py:204-205).  A hard weight quantizer's
 * output is W_hat = ((q - zp[co]) * d1) (* d2[j]) with d1 per co (d1_per_ci = 0) or per
 * (co, ci) (= 1) and the optional column scale d2 (ChannelQuantMSE's inp_scale, j in
 * [0, Ci*K)).  Codes are stored as q - qmin in ssq_pack_bits(n_bits) = 2 / 4 / 8 bits each,
 * little-endian, ssq_pack_bytes(n, n_bits) bytes for n codes.
 * ssq_pack_encode recovers q from W_hat and ADDS to *mismatch (device u32, caller-zeroed)
 * the number of elements whose decode is not bit-identical to W_hat (0 = exact export).
 * ssq_pack_decode writes W_hat back.  Co*Ci*K < 2^31.                                    */
int ssq_pack_bits(int n_bits);
size_t ssq_pack_bytes(int64_t n, int n_bits);
int ssq_pack_encode(const float* What, const float* zp, const float* d1, int d1_per_ci,
                    const float* d2, int64_t Co, int64_t Ci, int64_t K, int n_bits, int qmin,
                    int qmax, void* packed, uint32_t* mismatch, ssq_stream_t stream);
int ssq_pack_decode(const void* packed, const float* zp, const float* d1, int d1_per_ci,
                    const float* d2, int64_t Co, int64_t Ci, int64_t K, int n_bits, int qmin,
                    float* What, ssq_stream_t stream);

/* ---------------------------------------------------------------- bandwidth probe
 * float4 device copy, used by bench.py to report the measured stream bandwidth.      */
int ssq_stream_copy(const float* src, float* dst, int64_t n, ssq_stream_t stream);
/* HBM read-only (kind 1: nt loads of src, dst receives nothing) / write-only (kind 2: nt
 * stores into dst) probe over n floats, K1's geometry.  Bench context only. */
int ssq_stream_probe(const float* src, float* dst, int64_t n, int kind, ssq_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* SSQ_H_ */

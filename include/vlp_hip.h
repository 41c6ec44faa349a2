/*
 * vlp_hip.h — C ABI of libvlp_hip.so, the MI355X (gfx950) implementation of the
 * CLIP-style contrastive pretraining step of
 * schusterbenjamin/Vision-Language-Pretraining-for-Bone-Tumor-Detection.
 *
 * The reference is pure Python: its hot path is VisionLanguageModule
 * (src/models/pretrain/VisionLanguageModule.py) whose arithmetic is delegated to
 * timm resnet34 (:30-35), HF BertModel/TinyBERT (:38-60), the head in forward
 * (:441-461), _compute_loss (:532-554) and torch.optim.AdamW (:130-184).  Each
 * entry point below replaces one of the device operations those calls dispatch
 * to; the Python host layer (vlp_amd/, src/models/pretrain/VisionLanguageModule.py
 * in this package) binds them with ctypes exactly as INTEGRATION.md shows.
 *
 * Conventions
 *  - All tensor arguments are DEVICE pointers (caller-allocated, e.g. by the
 *    PyTorch caching allocator); `stream` is a hipStream_t passed as void*.
 *    Every call only enqueues work on `stream`; none synchronises.
 *  - `dtype`: 0 = fp32 (parity mode), 1 = bf16 (throughput mode) storage of
 *    activations/gradients.  Weight gradients, BN statistics, and optimizer
 *    state are always fp32 (fp64 for BN sums).
 *  - Activations are NHWC ([N][H][W][C], C innermost); token hidden states are
 *    row-major [B*T][D].
 *  - Return value: 0 on success, otherwise a hipError_t code.
 *  - Stateless and re-entrant; "accumulate" outputs require the caller to zero
 *    them first (documented per call).
 */
#ifndef VLP_HIP_H
#define VLP_HIP_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* 3 since r5 (r4's 2 plus role_w on vlp_clip_loss_fused / vlp_ce_sym; the dy^T
 * operands of vlp_conv_wgrad / vlp_stem_wgrad / vlp_bn_bwd_apply removed); the
 * Python binding refuses any other value. */
int vlp_abi_version(void);
/* Diagnostic: register-only v_mfma_f32_16x16x32_bf16 chains (8 independent
 * accumulators per wave, 4 waves per block) to measure the card's dense bf16
 * MFMA ceiling next to the vendor figure.
 * FLOP = blocks * 4 * iters * 8 * 16384; out: blocks * 256 floats. */
int vlp_mfma_peak_probe(int blocks, int iters, float* out, void* stream);
/* Diagnostic: an empty kernel dispatch (end = 0: begin marker, 1: end marker)
 * that brackets bench.py's isolated roofline pass in a rocprofv3 kernel trace
 * (tools/roofline_window.py).  No reference counterpart. */
int vlp_trace_marker(int end, void* stream);

/* ---------------- image tower: convolutions ----------------
 * Replace the cuDNN conv fwd/dgrad/wgrad calls made by timm resnet34
 * (VisionLanguageModule.py:30-35 -> ImageEncoder.forward).
 * Weight operands are produced by vlp_pack_conv:
 *   wp = [Co][KH][KW][C]   (forward),  wt = [C][KH][KW][Co]   (data gradient).
 */
/* y[N][Ho][Wo][Co] = conv(x, w); optionally x := relu(in_scale*x + in_shift)
 * per input channel on load (previous BN+ReLU); accumulates per-channel
 * sum / sum of squares of y into stat_sum / stat_sumsq (fp64, zeroed by caller). */
int vlp_conv_fwd(int dtype, const void* x, const void* wp, void* y, int N, int H, int W, int C,
                 int Co, int KH, int KW, int S, int P, const float* in_scale,
                 const float* in_shift, double* stat_sum, double* stat_sumsq, int stat_rep,
                 void* stream);
/* Conv forward with BN-apply + ReLU of its input fused (timm BasicBlock
 * act1(bn1(conv1(x))) -> conv2, VisionLanguageModule.py:30-32): x is the raw
 * output of the previous conv; each input element becomes
 * relu(in_scale[c]*x + in_shift[c]) once, and that activation is also written to
 * x_act (what this conv's weight gradient reads), so no separate BN pass runs.
 * Bit-identical to vlp_bn_add_relu (no residual) followed by vlp_conv_fwd.
 * Layer-1 geometry only: vlp_conv_fwd_act_ok(...) = 1 when the shape is taken
 * (bf16, C = Co = 64, 3x3, stride 1, pad 1, W = 128); otherwise
 * vlp_conv_fwd_act returns hipErrorInvalidValue. */
int vlp_conv_fwd_act_ok(int dtype, int N, int H, int W, int C, int Co, int KH, int KW, int S, int P);
int vlp_conv_fwd_act(int dtype, const void* x, const void* wp, void* y, void* x_act, int N, int H, int W,
                     int C, int Co, int KH, int KW, int S, int P, const float* in_scale,
                     const float* in_shift, double* stat_sum, double* stat_sumsq, int stat_rep,
                     void* stream);
/* dx[N][H][W][C] = conv^T(dy, w).  If y_bn != NULL: dx := dx * (bn_scale*y_bn +
 * bn_shift > 0) (ReLU mask of the producing BN+ReLU) and stat1 += sum(dx),
 * stat2 += sum(dx * (y_bn - bn_mean) * bn_invstd); else if addend != NULL:
 * dx += addend (residual-branch gradient). */
int vlp_conv_dgrad(int dtype, const void* dy, const void* wt, void* dx, int N, int H, int W, int C,
                   int Co, int KH, int KW, int S, int P, const void* addend, const void* y_bn,
                   const float* bn_scale, const float* bn_shift, const float* bn_mean,
                   const float* bn_invstd, double* stat1, double* stat2, int stat_rep,
                   void* stream);
/* dgrad fused with the next block's output ReLU and BN2 backward sums:
 * g = (dgrad + addend) * (relu_out > 0); stat1 += sum g, stat2 += sum g*(y-mean)*invstd
 * (replaces the separate bn_bwd_reduce pass over dx, out, y2).  Exactly one of
 * relu_out (the activation) and relu_mask (its sign bits as written by
 * vlp_bn_add_relu / vlp_maxpool_fwd: bit e&7 of byte e>>3 for element e) is given. */
int vlp_conv_dgrad_relu(int dtype, const void* dy, const void* wt, void* g, int N, int H, int W,
                        int C, int Co, int KH, int KW, int S, int P, const void* addend,
                        const void* relu_out, const uint8_t* relu_mask, const void* y,
                        const float* mean, const float* invstd, double* stat1, double* stat2,
                        int stat_rep, void* stream);
/* Layer-1 data gradients with their input's BatchNorm backward folded in (timm
 * BasicBlock backward, VisionLanguageModule.py:30-32; replaces vlp_bn_bwd_apply +
 * vlp_conv_dgrad / vlp_conv_dgrad_relu).  The input dy = k*g_in + b*y_in + c (per
 * channel, in_coef = [k | b | c] from vlp_bn_bwd_coef) is formed once per input row
 * in the rows kernel's LDS ring and written to dy_out (the weight gradient's
 * operand); the epilogues are those of vlp_conv_dgrad (y_bn) and vlp_conv_dgrad_relu.
 * Shapes: vlp_conv_dgrad_act_ok (bf16, C = Co = 64, 3x3 stride 1 pad 1, W = 128),
 * else hipErrorInvalidValue.  Bit-identical to the separate pass + data gradient. */
int vlp_conv_dgrad_act_ok(int dtype, int N, int H, int W, int C, int Co, int KH, int KW, int S, int P);
int vlp_conv_dgrad_bn_act(int dtype, const void* g_in, const void* y_in, const float* in_coef, void* dy_out,
                          const void* wt, void* dx, int N, int H, int W, int C, int Co, int KH, int KW,
                          int S, int P, const void* y_bn, const float* bn_scale, const float* bn_shift,
                          const float* bn_mean, const float* bn_invstd, double* stat1, double* stat2,
                          int stat_rep, void* stream);
int vlp_conv_dgrad_relu_act(int dtype, const void* g_in, const void* y_in, const float* in_coef,
                            void* dy_out, const void* wt, void* gout, int N, int H, int W, int C, int Co,
                            int KH, int KW, int S, int P, const void* addend, const void* relu_out,
                            const uint8_t* relu_mask, const void* y, const float* mean,
                            const float* invstd, double* stat1, double* stat2, int stat_rep, void* stream);
/* Second block of layers 2-4 (timm BasicBlock backward, VisionLanguageModule.py:30-32): conv1's
 * data gradient (+ addend) through the previous block's output ReLU (relu_mask sign bits),
 * with that block's bn2 (y, mean, invstd) and downsample-BN (yd, meand, invstdd) backward
 * sums stat1 = sum g, stat2 = sum g*xhat, stat3 = sum g*xhatd in the epilogue (replaces
 * vlp_bn_bwd_reduce over dout, out, y2, yd).  bf16, stride 1, C >= 128, C % 64 == 0. */
int vlp_conv_dgrad_relu2(int dtype, const void* dy, const void* wt, void* g, int N, int H, int W, int C, int Co,
                         int KH, int KW, int S, int P, const void* addend, const uint8_t* relu_mask, const void* y,
                         const float* mean, const float* invstd, const void* yd, const float* meand,
                         const float* invstdd, double* stat1, double* stat2, double* stat3, int stat_rep,
                         void* stream);
/* First block of layers 2-4 (timm BasicBlock with downsample, VisionLanguageModule.py:30-32):
 * conv1's 3x3/2 data gradient with the 1x1/2 downsample's data gradient folded into
 * pixel-parity class (0, 0) as extra K-steps -- replaces vlp_conv_dgrad of the
 * downsample and the addend of vlp_conv_dgrad_relu.  dyd = dy + N*Ho*Wo*Co and
 * wtd = wt + C*KH*KW*Co (one allocation each), bf16, KH = KW = 3, S = 2, P = 1. */
int vlp_conv_dgrad_relu_ds(int dtype, const void* dy, const void* dyd, const void* wt, const void* wtd, void* g,
                           int N, int H, int W, int C, int Co, int KH, int KW, int S, int P,
                           const void* relu_out, const uint8_t* relu_mask, const void* y, const float* mean,
                           const float* invstd, double* stat1, double* stat2, int stat_rep, void* stream);
/* Weight gradient as split-K fp32 slabs: split s of the pixel reduction writes
 * split_ws[s][Co][KH][KW][C] (plain stores, no atomics); *nsplit receives the
 * split count (<= ws_floats / (Co*KH*KW*C)).  vlp_conv_wgrad_fold then sums the
 * slabs into grad[Co][C][KH][KW], the layout of the reference's conv weight
 * gradient (timm resnet34 convs, VisionLanguageModule.py:34-35), overwriting it.
 * Replaces vlp_conv_wgrad + vlp_unpack_conv_grad on the training path. */
int vlp_conv_wgrad_ws(int dtype, const void* dy, const void* x, float* split_ws, long long ws_floats,
                      int* nsplit, int N, int H, int W, int C, int Co, int KH, int KW, int S, int P,
                      void* stream);
int vlp_conv_wgrad_fold(int Co, int C, int KH, int KW, int nsplit, const float* split_ws, float* grad,
                        void* stream);
/* vlp_conv_wgrad_ws takes the layer-1 row-streaming kernel (bf16, C = Co = 64,
 * 3x3/1 pad 1, W = 128; one workgroup per image, one slab each) when the batch
 * holds at least this many images, else the im2col GEMM.  n < 0 restores the
 * default (3/4 of the device's CUs: below it the per-image workgroups leave the
 * chip idle).  *prev (may be null) receives the previous setting (-1 = default).
 * Returns 0.  Host-only, no GPU work. */
int vlp_set_wgrad_rows_min_images(int n, int* prev);
/* dw_ws[Co][KH][KW][C] += sum over pixels dy x_patch (fp32 atomics; zero first).
 * Optional BN+ReLU-on-load of x as in vlp_conv_fwd. */
int vlp_conv_wgrad(int dtype, const void* dy, const void* x, float* dw_ws, int N, int H, int W,
                   int C, int Co, int KH, int KW, int S, int P, const float* in_scale,
                   const float* in_shift, void* stream);

/* stem conv 7x7/2 pad 3, 3 -> 64 channels (timm resnet34 conv1, called from
 * ImageEncoder.forward, VisionLanguageModule.py:34-35), on a zero-padded NHWC4
 * image xp of size [N][Hp][Wp][4] (vlp_stem_geom); the caller zeroes xp once.
 * vlp_stem_prep_u8 also folds the collation's normalise + 3-channel replicate
 * (PretrainDataModule.py:167-171) into the upload of 1-channel uint8 images. */
void vlp_stem_geom(int H, int W, int* Ho, int* Wo, int* Hp, int* Wp);
int vlp_stem_prep(int dtype, const float* x_nchw, void* xp, int N, int H, int W, void* stream);
int vlp_stem_prep_u8(int dtype, const uint8_t* x_u8, void* xp, int N, int H, int W, float mean,
                     float std, void* stream);
int vlp_stem_fwd(int dtype, const void* xp, const void* wp, void* y, int N, int H, int W,
                 double* stat_sum, double* stat_sumsq, int stat_rep, void* stream);
int vlp_stem_wgrad(int dtype, const void* dy, const void* xp, float* dw_ws, int N, int H, int W,
                   void* stream);
/* the same through per-split fp32 slabs split_ws[s][64][256] (plain stores, no
 * atomics; *nsplit receives the split count), then vlp_stem_wgrad_fold sums
 * them into grad[64][3][7][7] (timm conv1.weight layout), overwriting it */
int vlp_stem_wgrad_ws(int dtype, const void* dy, const void* xp, float* split_ws, long long ws_floats,
                      int* nsplit, int N, int H, int W, void* stream);
int vlp_stem_wgrad_fold(int nsplit, const float* split_ws, float* grad, void* stream);

/* single-channel stem for the 1-channel uint8 upload (the reference replicates
 * the grayscale radiograph to 3 identical channels, PretrainDataModule.py:167-171,
 * so conv1 = a 1-channel 7x7/2 conv with the channel-summed weights: K = 64
 * instead of 256).  Image: 4 copies shifted by 0/2/4/6 pixels,
 * xs[4][N][Hp][Wp1] (vlp_stem1_geom; returns non-zero when Wo % 4 != 0, then the
 * caller uses the 3-channel path); weights W1[64][8][8] (vlp_pack_stem1);
 * vlp_stem1_wgrad_ws + vlp_stem1_wgrad_fold give the [64][3][7][7] gradient
 * (identical for the three channels). */
int vlp_stem1_geom(int H, int W, int* Ho, int* Wo, int* Hp, int* Wp1);
int vlp_stem1_prep_u8(int dtype, const uint8_t* x_u8, void* xs, int N, int H, int W, float mean, float std,
                      void* stream);
int vlp_pack_stem1(int dtype, const float* w, void* wp, void* stream);
int vlp_stem1_fwd(int dtype, const void* xs, const void* wp, void* y, int N, int H, int W,
                  double* stat_sum, double* stat_sumsq, int stat_rep, void* stream);
int vlp_stem1_wgrad_ws(int dtype, const void* dy, const void* xs, float* split_ws, long long ws_floats,
                       int* nsplit, int N, int H, int W, void* stream);
int vlp_stem1_wgrad_fold(int nsplit, const float* split_ws, float* grad, void* stream);
/* Fused stem (bf16, single-channel upload): replaces timm's conv1 -> bn1 ->
 * act1 -> maxpool (VisionLanguageModule.py:30-32) without ever writing the
 * full-resolution conv output.  vlp_stem1_pool_fwd computes the conv per
 * output row on MFMA, the BatchNorm sums (stat_* may be NULL: eval mode) and
 * the 3x3/2 pad-1 max-pool of sign(gamma)*y0, i.e. the window's max (gamma >= 0)
 * or min (gamma < 0) of y0, which is where relu(bn(y0)) peaks; it stores the
 * raw y0 there (yarg [N][Ho/2][Wo/2][64]) and the tap kh*3+kw (idx).  Then
 * p = relu(sc*yarg + sh) is vlp_bn_add_relu over the pooled tensor.
 * vlp_stem1_route_bwd writes dy = dBN(route(dp)) for the stem weight gradient,
 * recomputing y0 instead of reading it; dp must be ReLU-masked (p > 0, as the
 * layer-1 data-gradient epilogue produces it).  vlp_stem1_fused_ok(H, W) = 1 when the
 * shape qualifies (Wo a multiple of 64 up to 256, Ho even). */
int vlp_stem1_fused_ok(int H, int W);
int vlp_stem1_pool_fwd(const void* xs, const void* wp1, const float* gamma, void* yarg, uint8_t* idx, int N,
                       int H, int W, double* stat_sum, double* stat_sumsq, int stat_rep, void* stream);
int vlp_stem1_route_bwd(const void* xs, const void* wp1, const void* dp, const uint8_t* idx, const float* sc,
                        const float* sh, const float* mean, const float* istd, const float* gamma,
                        const double* sum_g, const double* sum_gx, void* dy, int N, int H, int W, void* stream);
/* The whole stem backward in one pass (routing + BN backward + weight gradient;
 * replaces the stem's autograd backward behind VisionLanguageModule.py:30-32):
 * dW1 = k R + b W1 G + c S with R = sum g P^T (the pooled gradient routed to its
 * arg-max pixel), G = sum P P^T, S = sum P over the conv-output pixels, so neither
 * y0 nor dy is formed.  grad [64][3][7][7] is overwritten (the same gradient for
 * the 3 identical input channels).  dp ReLU-masked as above; ws holds
 * vlp_stem1_bwd_fused_ws_floats fp32 elements. */
int vlp_stem1_bwd_fused_ws_floats(int N, int H, int W, long long* n);
int vlp_stem1_bwd_fused(const void* xs, const void* wp1, const void* dp, const uint8_t* idx, const float* mean,
                        const float* istd, const float* gamma, const double* sum_g, const double* sum_gx, float* ws,
                        long long ws_floats, float* grad, int N, int H, int W, void* stream);

/* ---------------- image tower: BatchNorm / residual / pooling ----------------
 * Replace timm resnet34's BatchNorm2d (train-mode batch statistics), ReLU,
 * residual add, maxpool 3x3/2 and global average pool (VisionLanguageModule.py:30-35).
 * Per-channel statistic outputs (fp64) are REPLICATED: a producer called with
 * stat_rep = R adds into R copies laid out [R][C] (copy = workgroup % R) so
 * that ~1e5 workgroups do not serialise on C addresses; vlp_stat_reduce folds
 * them into copy 0, which is what every consumer reads.  stat_rep = 1 means a
 * plain [C] buffer. */
int vlp_stat_reduce(int rep, int C, double* a, double* b, double* c, void* stream);
int vlp_bn_finalize(int C, double count, const double* sum, const double* sumsq,
                    const float* gamma, const float* beta, float eps, float momentum,
                    float* running_mean, float* running_var, float* scale, float* shift,
                    float* mean, float* invstd, void* stream);
/* vlp_stat_reduce + vlp_bn_finalize in one launch (sum / sumsq: [rep][C]
 * replicas, folded into copy 0 as a side effect) */
int vlp_bn_finalize_rep(int rep, int C, double count, double* sum, double* sumsq,
                        const float* gamma, const float* beta, float eps, float momentum,
                        float* running_mean, float* running_var, float* scale, float* shift,
                        float* mean, float* invstd, void* stream);
/* vlp_stat_reduce + vlp_bn_param_grad in one launch: dgamma = sum g*xhat,
 * dbeta = sum g; sum_gxd / dgamma_d / dbeta_d (all or none): the downsample BN
 * that shares g (BasicBlock bn2 + downsample.1).  Sums folded into copy 0. */
int vlp_bn_grad_rep(int rep, int C, double* sum_g, double* sum_gx, double* sum_gxd, float* dgamma,
                    float* dbeta, float* dgamma_d, float* dbeta_d, void* stream);
int vlp_bn_eval_coeffs(int C, const float* gamma, const float* beta, const float* running_mean,
                       const float* running_var, float eps, float* scale, float* shift,
                       void* stream);
/* out = relu(sc*y + sh + idt'), idt' = idt (scd == NULL) or scd*idt + shd; idt == NULL: relu(sc*y + sh).
 * relu_mask (optional, bf16 only): out's sign bits, byte e>>3 bit e&7 = (out[e] > 0) */
int vlp_bn_add_relu(int dtype, long long M, int C, const void* y, const float* sc, const float* sh,
                    const void* idt, const float* scd, const float* shd, void* out, uint8_t* relu_mask,
                    void* stream);
/* g = dout * (mask > 0) (dout may be a broadcast [N][C]/HW gradient `dbc`);
 * sum_g += sum g, sum_ga += sum g*xhat(ya), sum_gb += sum g*xhat(yb) */
int vlp_bn_bwd_reduce(int dtype, long long M, int C, const void* dout, const float* dbc, int HW,
                      const void* mask, const void* ya, const float* mean_a, const float* istd_a,
                      const void* yb, const float* mean_b, const float* istd_b, double* sum_g,
                      double* sum_ga, double* sum_gb, int stat_rep, void* stream);
/* coef[3][C] = (k, b, c) of dy = k*g + b*y + c over M rows (the folded BN backward;
 * sums already folded, as vlp_bn_bwd_apply reads them) */
int vlp_bn_bwd_coef(long long M, int C, const float* gamma, const float* istd, const float* mean,
                    const double* sum_g, const double* sum_gx, float* coef, void* stream);
/* dy_s = gamma_s*istd_s*(g - mean(g) - xhat_s*mean(g*xhat_s)) for sides a, b; g_out = g. */
int vlp_bn_bwd_apply(int dtype, long long M, int C, const void* dout, const float* dbc, int HW,
                     const void* mask, const void* ya, const float* mean_a, const float* istd_a,
                     const float* gamma_a, const double* sum_g_a, const double* sum_gx_a,
                     void* dy_a, const void* yb, const float* mean_b, const float* istd_b,
                     const float* gamma_b, const double* sum_g_b, const double* sum_gx_b,
                     void* dy_b, void* g_out, void* stream);
int vlp_bn_param_grad(int C, const double* sum_g, const double* sum_gx, float* dgamma,
                      float* dbeta, void* stream);
/* out = maxpool3x3/2(relu(sc*y + sh)), idx = argmax tap (0..8) per element;
 * yarg (optional): y at the argmax, so the stem BN's backward sums can be taken
 * per pooled output (g*[out>0]*xhat(yarg)) by the layer-1 data-gradient
 * epilogue (vlp_conv_dgrad_relu with relu_out = out, y = yarg) instead of a
 * pass over the full-resolution y */
int vlp_maxpool_fwd(int dtype, int N, int H, int W, int C, const void* y, const float* sc,
                    const float* sh, void* out, uint8_t* idx, void* yarg, uint8_t* relu_mask,
                    void* stream);
/* stem backward, pass 1: g = dp routed to each window's recorded argmax, masked by
 * the stem ReLU; accumulates sum g and sum g*xhat(y) (g itself is not stored) */
int vlp_maxpool_bwd(int dtype, int N, int H, int W, int C, const void* dp, const uint8_t* idx,
                    const void* y, const float* sc, const float* sh, const float* mean,
                    const float* istd, double* sum_g, double* sum_gx, int stat_rep,
                    void* stream);
/* stem backward, pass 2: recomputes g and writes the BatchNorm input gradient
 * dy = gamma*istd*(g - mean(g) - xhat*mean(g*xhat)) in one stream over y */
int vlp_maxpool_bwd_apply(int dtype, int N, int H, int W, int C, const void* dp,
                          const uint8_t* idx, const void* y, const float* sc, const float* sh,
                          const float* mean, const float* istd, const float* gamma,
                          const double* sum_g, const double* sum_gx, void* dy, void* stream);
int vlp_avgpool_fwd(int dtype, int N, int HW, int C, const void* x, void* feat, void* stream);

/* ---------------- text tower (TinyBERT) ----------------
 * Replace the cuBLAS/ATen kernels of HF BertModel (VisionLanguageModule.py:45, :57-60). */
/* y = x W^T + bias; mode 0 plain, 1 aux = pre-activation & y = gelu(aux),
 * 2 y = dropout_p(x W^T + bias) + res.  bf16 (also _rs and vlp_linear_dgrad): the
 * output width and every output/operand leading dimension a multiple of 8 and the
 * rows 16-byte aligned (8-column epilogue groups), else hipErrorInvalidValue. */
int vlp_linear_fwd(int dtype, int M, int N, int K, const void* x, int ldx, const void* w,
                   const float* bias, void* y, int ldy, int mode, void* aux, const void* res,
                   int ldr, float p, unsigned long long seed, void* stream);
/* y = res + rscale[row / rps] * (x W^T + bias): a residual branch under DropPath (NesT
 * TransformerLayer, timm nest.py: x + drop_path(attn(norm1(x))); per-sample scale 0 or 1/(1-p)) */
int vlp_linear_fwd_rs(int dtype, int M, int N, int K, const void* x, int ldx, const void* w,
                      const float* bias, void* y, int ldy, const void* res, int ldr, const float* rscale,
                      int rps, void* stream);
/* dx = dy W; mode 1: dx *= gelu'(aux); mode 0: dx += addend (if non-NULL) */
int vlp_linear_dgrad(int dtype, int M, int Kin, int Nout, const void* dy, int lddy, const void* w,
                     void* dx, int lddx, int mode, const void* aux, int ldaux, const void* addend,
                     int ldad, void* stream);
/* dw[Nout][Kin] += dy^T x (fp32 atomics; zero first) */
int vlp_linear_wgrad(int dtype, int M, int Nout, int Kin, const void* dy, int lddy, const void* x,
                     int ldx, float* dw, void* stream);
/* the same through a split-K workspace ws[ks][Nout][Kin] fp32 (bf16 only, Kin % 4 == 0):
 * split partials are plain stores, then one pass folds them into dw (no atomics) */
int vlp_linear_wgrad_ws(int dtype, int M, int Nout, int Kin, const void* dy, int lddy, const void* x,
                        int ldx, float* dw, float* ws, long long ws_elems, void* stream);
/* fp32 elements of the workspace vlp_linear_wgrad_ws uses at its full split count
 * for this shape (host-side query; a smaller workspace trims the splits) */
int vlp_linear_wgrad_ws_floats(int M, int Nout, int Kin, long long* n);
/* out[n] += sum_m x[m][n] (bias gradients; fp32 atomics) */
int vlp_colsum(int dtype, int M, int N, const void* x, int ld, float* out, void* stream);
int vlp_layernorm_fwd(int dtype, int M, int D, const void* x, const float* gamma,
                      const float* beta, float eps, void* y, float* mean, float* rstd, float p,
                      unsigned long long seed, void* stream);
int vlp_layernorm_bwd(int dtype, int M, int D, const void* dy, float p_out,
                      unsigned long long seed_out, const void* x, const float* mean,
                      const float* rstd, const float* gamma, void* dx, void* dxd, float p_in,
                      unsigned long long seed_in, float* dgamma, float* dbeta, void* stream);
/* dx = LayerNorm backward + addend (pre-norm residual: NesT's x + attn(norm1(x))) */
int vlp_layernorm_bwd_add(int dtype, int M, int D, const void* dy, const void* x, const float* mean,
                          const float* rstd, const float* gamma, const void* addend, void* dx,
                          float* dgamma, float* dbeta, void* stream);
/* the same, also writing dxs = rscale[row / rps] * dx: the DropPath-scaled gradient of the
 * residual branch that produced x (NesT; saves a separate scaling pass) */
int vlp_layernorm_bwd_add_rs(int dtype, int M, int D, const void* dy, const void* x, const float* mean,
                             const float* rstd, const float* gamma, const void* addend, void* dx, void* dxs,
                             const float* rscale, int rps, float* dgamma, float* dbeta, void* stream);
int vlp_attn_fwd(int dtype, int B, int T, int H, int dh, const void* qkv, const long long* amask,
                 void* ctx, float* P, float scale, float p, unsigned long long seed, void* stream);
int vlp_attn_bwd(int dtype, int B, int T, int H, int dh, const void* qkv, const float* P,
                 const void* dctx, void* dqkv, float scale, float p, unsigned long long seed,
                 void* stream);
int vlp_embed_fwd(int dtype, int M, int T, int D, const long long* ids, const long long* tt,
                  const float* wemb, const float* pemb, const float* temb, void* e_out,
                  void* stream);
int vlp_embed_bwd(int dtype, int M, int T, int D, const long long* ids, const long long* tt,
                  const void* de, float* dwemb, float* dpemb, float* dtemb, void* stream);
int vlp_scatter_rows(int dtype, int R, int D, const void* in, int ldi, void* out, int ldo,
                     void* stream);

/* ---------------- retrieval metrics ----------------
 * Replace the topk over the full similarity matrix in
 * precision_at_k_on_image_embeddings (VisionLanguageModule.py:364-400) and
 * recall_at_k_on_image_text_retreival (:402-439).  vals/idx[R][K] = the K
 * largest entries of each row x[r][0..N) in descending order, ties to the
 * lower column; K <= 16.  The caller builds x one query chunk at a time
 * (fp32 vlp_linear_fwd of normalised embeddings). */
int vlp_row_topk(int R, int N, const float* x, long long ldx, int K, float* vals, int* idx, void* stream);

/* ---------------- NesT image encoder (BASELINE configs[3]) ----------------
 * Replace timm nest.py's pieces behind ImageEncoder's timm.create_model("nest_small", ...)
 * (VisionLanguageModule.py:27-35).  Blocked local attention: qkv[BT*N][3C] rows (q | k | v,
 * head h at h*32), out[BT*N][C] head-major (h*32 + d; timm's d*H + h order is folded into
 * the proj weight with vlp_nest_permute_cols), lse[BT*H*N] (log2 domain), head dim 32.
 * Backward: delta[BT*H*N] scratch; writes every column of dqkv. */
int vlp_nest_attn_fwd(int dtype, int BT, int H, int N, int dh, const void* qkv, void* out, float* lse,
                      float scale, void* stream);
int vlp_nest_attn_bwd(int dtype, int BT, int H, int N, int dh, const void* qkv, const void* out,
                      const void* dout, const float* lse, float* delta, void* dqkv, float scale, void* stream);
/* blockify (timm nest.blockify, + pos[Hg*Wg][bs*bs][C] when non-NULL): NHWC image
 * x[B][Hg*bs][Wg*bs][C] -> tokens y[B][Hg*Wg][bs*bs][C]; inverse = deblockify (y <- x tokens) */
int vlp_nest_blockify(int dtype, int B, int Hg, int Wg, int bs, int C, const void* x, const float* pos,
                      void* y, int inverse, void* stream);
/* dpos[t][c] = sum_b dy[b][t][c] over the B samples of a level input [B][TN][C] */
int vlp_nest_pos_grad(int dtype, int B, int TN, int C, const void* dy, float* dpos, void* stream);
/* ConvPool's max pool 3x3 / 2, padding 1 (NHWC); idx = window tap 0..8 */
int vlp_nest_maxpool_fwd(int dtype, int B, int H, int W, int C, const void* x, void* y, uint8_t* idx,
                         void* stream);
int vlp_nest_maxpool_bwd(int dtype, int B, int H, int W, int C, const void* dy, const uint8_t* idx,
                         void* dx, void* stream);
/* patch-embed im2col: 4x4/4 patches -> out[B*(H/4)*(W/4)][48] in level-0 blocked token order;
 * exactly one of x (fp32 [B][3][H][W], normalised) / x_u8 ([B][1][H][W], (v-mean)/std) */
int vlp_nest_patch_prep(int dtype, int B, int H, int W, int bs, const float* x, const uint8_t* x_u8,
                        float mean, float std_, void* out, void* stream);
/* y[m][n] += bias[n] */
int vlp_nest_add_bias(int dtype, long long M, int N, void* y, const float* bias, void* stream);
/* proj weight input columns: dst[n][h*Dh + d] = src[n][d*H + h] (fp32 -> dtype_out), and back */
int vlp_nest_permute_cols(int dtype_out, int Nr, int H, int Dh, const float* src, void* dst, void* stream);
int vlp_nest_unpermute_cols(int Nr, int H, int Dh, const float* src, float* dst, void* stream);
/* DropPath: mode 0 x += s[m / rows] * y; mode 1 y = s[m / rows] * x */
int vlp_nest_rowscale(int dtype, long long M, int N, int rows, const float* s, void* x, void* y, int mode,
                      void* stream);
/* global average pool backward: dy[b*HW + p][c] = dfeat[b][c] * inv */
int vlp_nest_bcast(int dtype, int B, int HW, int C, const float* dfeat, float inv, void* dy, void* stream);

/* ---------------- contrastive head ----------------
 * Replace VisionLanguageModule.forward (VisionLanguageModule.py:441-461: projections,
 * F.normalize, logit_scale.exp().clamp(max=100) * img @ txt.T) and
 * VisionLanguageModule._compute_loss (VisionLanguageModule.py:532-554: symmetric CE). */
int vlp_l2norm_fwd(int R, int E, const float* x, float* y, float* norm, void* stream);
/* dx = gscale[0] * d normalize(x) (gscale may be NULL = 1); optional compute-dtype copy */
int vlp_l2norm_bwd(int dtype, int R, int E, const float* y, const float* norm, const float* dy,
                   const float* gscale, float* dx, void* dx_t, void* stream);
/* y = x * s[0] (+ y if accumulate); s may be NULL (= 1) */
int vlp_scale(int n, const float* x, const float* s, float* y, int accumulate, void* stream);
/* out[3] = {(parts0 + parts1) / (2N), parts0 / N, parts1 / N} */
int vlp_clip_loss_finish(const float* parts, int N, float* out, void* stream);
/* Fused global-batch symmetric InfoNCE, forward + backward (replaces the
 * logits matmul and the two F.cross_entropy calls of VisionLanguageModule.py
 * :456-459 / :550-552 with their autograd backward).  img_all/txt_all: [N][E]
 * gathered normalised embeddings (E <= 256, E % 4 == 0); this rank owns rows
 * [offset, offset+B).  Written (not accumulated): g_img_all/g_txt_all, d loss /
 * d embeddings for all N rows; d_logit_scale; loss_parts[0] the sum of the
 * image->text CE terms of the local rows, loss_parts[1] text->image; lse_out
 * (optional) [2][B].  role_w (optional, device, 2 floats): the gradients are those
 * of (role_w[0] image_loss + role_w[1] text_loss) / 2 (NULL: {1, 1}, the
 * reference's loss; other weights carry gradients of image_loss / text_loss).  ws: vlp_clip_loss_ws_floats(B, N, E) floats of scratch
 * (cosines / softmax weights, split-key partials, dq slabs; every product on fp32
 * MFMA; no atomics, bitwise reproducible).  ABI 3 (vlp_abi_version). */
int vlp_clip_loss_ws_floats(int B, int N, int E, long long* n);
int vlp_clip_loss_fused(int B, int N, int E, int offset, const float* img_all,
                        const float* txt_all, const float* logit_scale, float* g_img_all,
                        float* g_txt_all, float* d_logit_scale, float* loss_parts,
                        float* lse_out, const float* role_w, float* ws, long long ws_floats,
                        void* stream);
/* symmetric CE over explicit logits [B][B]: out = {loss, image_loss, text_loss} (+=);
 * dlogits (+=, optional) = d (role_w[0] image_loss + role_w[1] text_loss) / 2 / d logits
 * (role_w NULL: {1, 1}, the reference's loss, :550-552) */
int vlp_ce_sym(int B, const float* logits, float* out, float* dlogits, const float* role_w, void* stream);
/* C[M][N] (=|+=) alpha * sum_k A(m,k) B(n,k) on MFMA; a_kc / b_kc: K-contiguous
 * operand ([rows][ld]) else MN-contiguous ([K][ld]).  Every contiguous extent and
 * leading dimension a multiple of 16 B (4 fp32 / 8 bf16), N and ldc multiples of 4;
 * otherwise hipErrorInvalidValue */
int vlp_matmul(int dtype, int M, int N, int K, const void* A, int lda, int a_kc, const void* B,
               int ldb, int b_kc, void* C, int ldc, int out_f32, float alpha, int accumulate,
               void* stream);
int vlp_cast(int dtype, long long n, const float* x, void* y, void* stream);

/* ---------------- optimizer / packing ----------------
 * Replace torch.optim.AdamW as built by configure_optimizers
 * (VisionLanguageModule.py:130-184, configs/optimizer/adamw.yaml:1-3). */
int vlp_adamw(long long n, float* p, const float* g, float* m, float* v, float lr, float beta1,
              float beta2, float eps, float wd, float step_size, float bc2_sqrt, void* stream);
int vlp_pack_conv(int dtype, int Co, int C, int KH, int KW, const float* w, void* wp, void* wt,
                  void* stream);
/* vlp_pack_conv for n <= 48 convolutions in one launch: desc holds n rows of
 * 6 values {w, wp, wt (device pointers; wp / wt may be 0), Co, C, KH*KW}
 * (host memory, read during the call) */
int vlp_pack_conv_batch(int dtype, int n, const long long* desc, void* stream);
int vlp_pack_stem(int dtype, const float* w, void* wp, void* stream);
int vlp_unpack_conv_grad(int Co, int C, int KH, int KW, const float* ws, float* g, void* stream);
int vlp_unpack_stem_grad(const float* ws, float* g, void* stream);

/* ---------------- radiograph preprocessing / augmentation ----------------
 * Replace the reference's CPU DataLoader transforms (src/data/PretrainDataModule.py:157-198).
 * vlp_prep_images: n grayscale images of any size packed back to back in src (uint8 when
 * src_u8, else fp32; element offsets off[n] and sizes hw[n][2] in DEVICE memory) ->
 * HistogramNormalized (MONAI, 256 bins) -> CropLargerDimension(0.05) ->
 * PadToSquaredEdgeAverage -> Resized(S, area) -> (x - mean) / std, written to out fp32
 * [n][C][S][S] (channels identical, as the reference's 3-channel repeat).
 * work: n * 1544 bytes of device scratch. */
int vlp_prep_images(int n, const void* src, int src_u8, const long long* off, const int* hw, int S,
                    float mean, float std_, int C, float* out, void* work, void* stream);
/* One resample per sample for RandAffined + RandRotated + RandFlipd + RandZoomd, then
 * RandGaussianNoised: out[b][c] = bilinear(in[b][ci]) at source (row, col) =
 * M_b (p - centre) + centre + t_b (border clamp) + N(0, noise_std[b]);
 * maps[b] = {m00, m01, t0, m10, m11, t1} drawn on the host.  in: fp32 [B][Cin][H][W]
 * (Cin 1 or C), or uint8 [B][1][H][W] normalised on load with (v - mean) / std. */
int vlp_aug_warp(int B, int Cin, int C, int H, int W, const void* in, int in_u8, float mean, float std_,
                 const float* maps, const float* noise_std, unsigned long long seed, float* out,
                 void* stream);

#ifdef __cplusplus
}
#endif
#endif /* VLP_HIP_H */

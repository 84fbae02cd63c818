/* seg_hip.h — C ABI of libseg_hip.so, the MI355X (gfx950) training path for the
 * hierarchical weak-label segmentation model of pmeletis/IV2019-boosting-semantic-
 * segmentation-with-weak-labels.
 *
 * The reference exposes this path through Python/TF plugin functions; each entry point
 * below replaces the TF graph that one of them builds (paths relative to the reference's
 * code/ directory):
 *
 *   seg_create / seg_destroy      model(...) graph construction + variable creation
 *                                 (models/resnet50_extended_model_hierarchical.py:17-141,
 *                                  models/resnet50_extended_feature_extractor.py:8-51)
 *   seg_forward                   the TRAIN-mode forward pass of model(...) up to the
 *                                 low-resolution logits (hierarchical.py:102-134)
 *   seg_loss                      upsampler + softmax/argmax/decision fusion
 *                                 (hierarchical.py:135-168) and define_losses(TRAIN)
 *                                 (estimator/define_losses_hierarchical.py:14-217)
 *   seg_backward                  tf.gradients inside create_train_op
 *                                 (estimator/define_estimator_hierarchical.py:120-129)
 *   seg_apply_update              MomentumOptimizer.apply_gradients + UPDATE_OPS (BN moving
 *                                 averages, EMA) (estimator/define_optimizer.py:3-26,
 *                                 define_estimator_hierarchical.py:96-111)
 *   seg_confusion                 define_metrics.mean_iou's confusion matrix
 *                                 (estimator/define_metrics.py:5-20)
 *
 * Conventions: every function returns 0 on success or a negative errno-style code;
 * seg_last_error() describes the failure. Device buffers passed in are caller-owned; the
 * context owns activations and workspace. NHWC layout. Every launch goes to the explicit
 * stream argument; no call allocates, frees or synchronises inside a step, so a step can
 * be captured in a hipGraph. One context per device; not re-entrant per context.
 */
#ifndef SEG_HIP_H
#define SEG_HIP_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct seg_ctx seg_ctx;

enum { SEG_PYRAMID_NONE = 0, SEG_PYRAMID_PSP = 1, SEG_PYRAMID_ASPP = 2 };
enum { SEG_DTYPE_F32 = 0, SEG_DTYPE_BF16 = 1, SEG_DTYPE_F16 = 2 };
enum { SEG_DATASET_CITYSCAPES = 0, SEG_DATASET_VISTAS = 1 };
enum { SEG_PARAM_WEIGHTS = 0, SEG_PARAM_GAMMA = 1, SEG_PARAM_BETA = 2,
       SEG_PARAM_MOVING_MEAN = 3, SEG_PARAM_MOVING_VAR = 4, SEG_PARAM_BIASES = 5 };
enum { SEG_UPSAMPLING_BILINEAR = 0, SEG_UPSAMPLING_HYBRID = 1 };
enum { SEG_NORM_BATCH = 0, SEG_NORM_GROUP = 1 };

typedef struct seg_cfg {
  int depth;            /* 50 | 101 (name_feature_extractor) */
  int pyramid;          /* SEG_PYRAMID_* (psp_module; ASPP is the commented spec) */
  int height, width;    /* height/width_feature_extractor */
  int nb_pp, nb_pb, nb_pi;  /* per-GPU per-pixel / per-bbox / per-image sub-batches */
  int dtype;            /* SEG_DTYPE_*: compute/storage dtype (accumulation is fp32) */
  int dataset;          /* SEG_DATASET_* (per_pixel_dataset_name) */
  int output_stride;    /* stride_feature_extractor (8) */
  int feature_dims;     /* feature_dims_decreased (256) */
  float bn_decay;       /* batch_norm_decay (0.9) */
  int train_bn;         /* norm_train_variables */
  float weight_decay;   /* regularization_weight (0.00017): l2_regularizer scale */
  int fov_k, fov_rate;  /* fov_expansion_kernel_size / _rate: the optional extension/increase_fov
                           conv (resnet50_extended_feature_extractor.py:44-49); 0 = off */
  int upsampling;       /* SEG_UPSAMPLING_* (upsampling_method, hierarchical.py:143-184): hybrid
                           adds a 3x3 conv2d_transpose + bias per logits head before the resize */
  int norm;             /* SEG_NORM_* (norm_layer, hierarchical.py:293-333): group = per-image
                           tf.contrib.layers.group_norm after every conv, no moving statistics */
  int groups;           /* group-norm groups of the network's convs (0 = 32); the logits convs
                           use 1 (the softmax_classifier arg scope) */
} seg_cfg;

/* lifecycle -------------------------------------------------------------------------- */
int seg_create(int device, const seg_cfg* cfg, seg_ctx** out);
int seg_destroy(seg_ctx* ctx);
const char* seg_last_error(seg_ctx* ctx);   /* ctx may be NULL (creation errors) */

/* parameters: flat fp32 buffers, allocated by the caller (sizes from seg_sizes) --------
 * params  [n_train]            conv weights ([Co][KH][KW][Ci]) then BN gamma/beta
 * grads   [n_train + n_stats]  gradient of the segmentation loss; the tail holds this
 *                              step's BN batch statistics (mean, Bessel variance) so one
 *                              all-reduce averages both across data-parallel ranks
 * momentum[n_train], ema[n_train] (optional, may be NULL), moving[n_moving] */
int seg_sizes(seg_ctx* ctx, int64_t* n_train, int64_t* n_decay, int64_t* n_moving,
              int64_t* n_stats);
int seg_bind_buffers(seg_ctx* ctx, float* params, float* grads, float* momentum, float* ema,
                     float* moving);
int64_t seg_param_count(seg_ctx* ctx);
int seg_param_info(seg_ctx* ctx, int64_t i, const char** name, int64_t* offset,
                   int64_t* numel, int* kind);
/* dims[4]: weights (Co, KH, KW, Ci); BN vectors and biases (C, 1, 1, 1). The hybrid
 * upsampler's conv2d_transpose weights are (Cin, 3, 3, Cout) so that the OHWI -> HWIO export
 * gives TF's [h][w][out][in] filter layout */
int seg_param_shape(seg_ctx* ctx, int64_t i, int64_t* dims);
/* re-derive compute copies (bf16 weights, flipped dgrad weights) after a host write */
int seg_params_updated(seg_ctx* ctx, void* stream);

/* one training step -------------------------------------------------------------------- */
/* images_nhwc [N][H][W][3] fp32 is read (copied / converted into the context) on `stream`;
 * the caller's buffer may be released once the forward's work on that stream is done */
int seg_forward(seg_ctx* ctx, const float* images_nhwc, void* stream);
int seg_loss(seg_ctx* ctx, const int32_t* px_labels, const float* bbox_soft,
             const float* tag_soft, int32_t* decisions_out, void* stream);
int seg_backward(seg_ctx* ctx, void* stream);
/* lr, momentum; ema_decay_eff = min(ema_decay, (1+step)/(10+step)) or 0 to skip EMA;
 * grad_scale multiplies the gradient (1/world_size after a SUM all-reduce) */
int seg_apply_update(seg_ctx* ctx, float lr, float momentum, float ema_decay_eff,
                     float grad_scale, void* stream);
/* tf.train.MomentumOptimizer(use_nesterov=on) for later updates (define_optimizer.py:17-20):
 * var -= lr * (g + momentum * accum) instead of var -= lr * accum; off by default */
int seg_set_nesterov(seg_ctx* ctx, int on);
/* Overlap the update with the backward's last kernel (single-process training loops: nothing
 * may read the gradients between seg_backward and seg_apply_update). With on, seg_backward
 * returns with the stream joined to every weight gradient except the stem's, which is still
 * running on the weight-gradient stream; seg_apply_update updates every other parameter beside
 * it and joins before the stem's weights. Every other call that takes a stream joins first.
 * No reference counterpart (scheduling only; results are unchanged). Off by default.
 * seg_flush_grads makes `stream` wait for that last weight gradient, for a caller that reads
 * the gradient buffer before seg_apply_update. */
int seg_set_defer_stem(seg_ctx* ctx, int on);
int seg_flush_grads(seg_ctx* ctx, void* stream);
/* pre-masked identity-unit gradients (on by default): when an identity unit follows another,
 * its conv1 data gradient stores the previous unit's output gradient already ReLU-masked, and
 * that unit's c3 BN backward skips the mask bits and the separate masked-gradient store.
 * Scheduling of bytes only: results are bitwise identical either way (tests/test_gpu_step.py).
 * No reference counterpart. */
int seg_set_premask(seg_ctx* ctx, int on);
/* linear BN-backward fold (on by default): the training BN backward of a 16-bit bottleneck's
 * expanding conv3 is affine in the gated output gradient and in the conv input, so its apply
 * pass is folded into the conv3 data gradient (a K-concatenated GEMM) and weight gradient
 * (a second GEMM + an fp32 combine); 0 runs the separate BN-backward apply pass (the fold's
 * reference path in the parity tests). Same math, different rounding order. No reference
 * counterpart. */
int seg_set_lbf(seg_ctx* ctx, int on);
/* runtime counters since seg_create (diagnostics; no reference counterpart):
 * "premask_launches" = data gradients stored pre-masked (seg_set_premask): identity units'
 *   conv1, and at block boundaries a projection unit's conv1 + shortcut and decrease_fdims';
 * "lbf_layers" = conv3 layers whose BN-backward apply was folded into their data / weight
 * gradients by linearity (seg_set_lbf);
 * "loss_yf_launches" = seg_loss calls whose loss head ran the y-first kernel (the full-res
 *   columns of every block fit one 256-thread chunk: the 512 x 1024 and 1024 x 2048 shapes).
 * -ENOENT for an unknown name. */
int seg_counter(seg_ctx* ctx, const char* name, int64_t* value);

/* outputs ------------------------------------------------------------------------------
 * losses: device float[10] = {segmentation, l1, l2_vehicle, l2_human, n1, n2v, n2h,
 *         f1, f2v, f2h}; reg: device float[1] regularisation value of the last update
 *         (weights before the update) */
int seg_outputs(seg_ctx* ctx, const float** losses, const float** reg,
                const float** logits_lowres, int* ld_logits, int* h_low, int* w_low);
int seg_confusion(seg_ctx* ctx, const int32_t* labels, const int32_t* decisions, int64_t n,
                  int num_classes, int32_t* cm, void* stream);

/* EVAL / PREDICT (define_estimator_hierarchical.py:161-232) ------------------------------
 * seg_set_bn_inference(ctx, 1): later seg_forward calls normalise with the moving statistics
 * (tf.contrib.layers.batch_norm is_training = batch_norm_accumulate_statistics = False,
 * models/resnet50_extended_model_hierarchical.py:40-49,306-307); 0 restores training BN.
 * Turning it on snapshots the bound buffers (call it again after seg_bind_buffers); the
 * statistics of every layer are then set by one launch at the start of each forward.
 * seg_predict: decisions of the last seg_forward at out_h x out_w: fused hierarchical argmax
 * (hierarchical.py:88-130) -> cid_map[n_map] (training -> evaluation/inference cids, -1 =
 * void -> max+1; _map_predictions_to_new_cids :490-522) -> optional _replace_voids
 * (:577-630) -> NEAREST_NEIGHBOR align_corners resize to out_h x out_w (_resize_predictions
 * :524-575). decisions_out: device int32 [N][out_h][out_w].
 * replace_voids: 0 = none; 1 = the EVAL order above (replace at network resolution, then the
 * nearest resize); 2 = the PREDICT order (:227-231): nearest-resize the decisions and
 * ResizeBilinear(align_corners) the l1 probabilities to out_h x out_w first, then replace
 * voids from the top-2 of the RESIZED probabilities. 1 and 2 agree when out = network size. */
int seg_set_bn_inference(seg_ctx* ctx, int on);
int seg_predict(seg_ctx* ctx, const int32_t* cid_map, int n_map, int replace_voids, int out_h,
                int out_w, int32_t* decisions_out, void* stream);
/* seg_full_predictions: the model's full-resolution `predictions` of the last seg_forward
 * (hierarchical.py:84-130) at network resolution H x W, C = c1 + c2 + c3 channels (l1 | l2
 * vehicle | l2 human): logits_out f32 [N][H][W][C] (align-corners bilinear upsampling of the
 * low-res logits), probs_out f32 [N][H][W][C] (per-head softmax), head_decisions_out int32
 * [N][H][W][3] (per-head argmax), decisions_out int32 [N][H][W] (fused, common cids). Every
 * output is optional (NULL skips it); float outputs 16-byte aligned. */
int seg_full_predictions(seg_ctx* ctx, float* logits_out, float* probs_out,
                         int32_t* head_decisions_out, int32_t* decisions_out, void* stream);

/* input preprocessing (input_cityscapes.py:66-96,190-209), after the host
 * decodes TFRecord -> tf.train.Example -> PNG (input_pipelines/tfrecords.py):
 * seg_prepare_images: raw uint8 [n][src_h][src_w][3] -> convert_image_dtype -> bilinear
 *   resize_images (align_corners = False) to H x W -> from_0_1_to_m1_1 -> fp32 [n][H][W][3]
 * seg_prepare_labels: raw uint8 label ids [n][src_h][src_w] -> lids2cids[n_lids] (-1 = void
 *   -> max + 1) -> nearest resize to H x W -> int32 [n][H][W] (-1 for ids outside the table) */
int seg_prepare_images(const uint8_t* raw, int n, int src_h, int src_w, int H, int W, float* out,
                       void* stream);
int seg_prepare_labels(const uint8_t* raw, int n, int src_h, int src_w, int H, int W,
                       const int32_t* lids2cids, int n_lids, int32_t* out, void* stream);
/* seg_prepare_images_crop: the weak-label streams' image path (resize_images_and_labels with
 *   preserve_aspect_ratio, input_pipelines/utils.py:181-241, under the OpenImages train inputs,
 *   input_subset_bboxes_v2.py:111-125): convert_image_dtype -> bilinear resize (align_corners =
 *   False) to resized_h x resized_w -> the H x W window at (crop_y, crop_x) -> from_0_1_to_m1_1.
 *   Only the window is computed; bitwise the same values as resizing and slicing. */
int seg_prepare_images_crop(const uint8_t* raw, int n, int src_h, int src_w, int resized_h,
                            int resized_w, int crop_y, int crop_x, int H, int W, float* out,
                            void* stream);

/* checkpoint interop (define_initializers.py:72-131, define_savers.py:38-66): CRC-32C of
 * host bytes, continuing from `crc` (0 to start) — the checksum TF tensor bundles
 * (<prefix>.index / <prefix>.data-*) keep per tensor and per table block. Host-only. */
uint32_t seg_crc32c(uint32_t crc, const void* data, size_t n);

/* loss scaling (fp16 storage, BASELINE config C5: fp16 with fp32 master gradients). The
 * gradient seed of seg_loss is multiplied by `scale`; seg_apply_update first flags non-finite
 * weight/BN gradients (device int, seg_found_inf), unscales them by grad_scale / scale (the BN
 * batch-statistics tail by grad_scale only) and skips the parameter update of a flagged step.
 * The caller adjusts the scale from the flag (dynamic loss scaling). */
int seg_set_loss_scale(seg_ctx* ctx, float scale);
int seg_found_inf(seg_ctx* ctx, const int32_t** flag_device);

/* cross-replica (synchronised) batch norm, the reference's --cross_replica_norm
 * (models/resnet50_extended_model_hierarchical.py:327-328 -> utils/cross_replica_batch_
 * normalization.py:393-476). With a hook set, every BN layer of seg_forward exchanges its
 * per-channel [mean | E[x^2]] (2C floats) and normalises with the replica average: mean,
 * variance E[x^2] - mean^2 (biased; it also feeds the moving variance, as the reference's
 * non-fused path does); every BN layer of seg_backward exchanges [mean(dyhat) |
 * mean(dyhat * xhat)] so dx is the gradient through the global statistics. `allreduce` must
 * SUM `n` floats at the device pointer `buf` in place across the `world` replicas, ordered
 * on `stream` (e.g. torch.distributed.all_reduce on that stream, RCCL or gloo), and return 0;
 * a nonzero return fails the step. fn = NULL turns synchronisation off; world = 1 with a hook
 * still calls it (a one-replica exchange: the sync-BN arithmetic over one replica). */
typedef int (*seg_allreduce_fn)(void* user, float* buf, int64_t n, void* stream);
int seg_set_bn_sync(seg_ctx* ctx, seg_allreduce_fn allreduce, void* user, int world);

/* gradient all-reduce buckets, in the order the backward completes them: n buckets
 * [lo[i], hi[i]) of the flat [grads | BN stats] buffer (conv-weight ranges cut at layer
 * boundaries, about SEG_BUCKET_MB = 32 MB each, then the BN-parameter + statistics tail);
 * returns n (fills at most max_buckets). seg_backward records one event per bucket when its
 * gradients are written; seg_stream_wait_bucket makes `stream` wait for it (the caller's
 * collective for bucket i then overlaps the rest of the backward). */
int seg_grad_buckets(seg_ctx* ctx, int max_buckets, int64_t* lo, int64_t* hi);
int seg_stream_wait_bucket(seg_ctx* ctx, int bucket, void* stream);

/* weak-label maps on the device (input_subset_bboxes_v2.py:74-98 rasterisation fused with the
 * aspect-preserving nearest-neighbour resize + crop of input_pipelines/utils.py:181-241;
 * input_subset_image_labels.py:73-107 for tags). All pointers are device memory:
 *   boxes [total][4] (xmin, xmax, ymin, ymax) normalised to [0,1], cids [total] in [0,13],
 *   box_off [n+1] per-image prefix offsets into boxes, geom [n][6] = (src_h, src_w, resized_h,
 *   resized_w, crop_y, crop_x); max_boxes = the largest per-image count (<= 1024);
 *   out [n][H][W][15] fp32 multinomials (channel 14 = void). tags [n][15] normalised. */
int seg_bbox_labels(const float* boxes, const int32_t* cids, const int32_t* box_off,
                    const int32_t* geom, int n, int max_boxes, int H, int W, float* out,
                    void* stream);
int seg_tag_labels(const float* tags, int n, int H, int W, float* out, void* stream);

/* internal tensors for parity tests: "logits", "grad_un", "dzscale", "feat", "dfeat", "z0",
 * "head<h>_out", "head<h>_dout", "pyr<b>_z" (pyramid branch b's BN + ReLU output at its pooled
 * resolution), "conv<i>_x" (input of the last forward), "conv<i>_y", "conv<i>_dy" (i =
 * creation index).
 * dims = N, H, W, C; ld = pixel stride; dtype = SEG_DTYPE_* of the storage */
int seg_debug_tensor(seg_ctx* ctx, const char* name, void** ptr, int* dims, int* ld, int* dtype);

/* kernel-time profiling: conv classes 0 fwd, 1 dgrad, 2 wgrad (gflop = algorithmic flops);
 * BN classes 3 apply, 4 bwd reduce, 5 bwd apply (gflop field = algorithmic GB moved) ---- */
int seg_profile(seg_ctx* ctx, int enable);
int seg_profile_read(seg_ctx* ctx, int cls, double* ms_total, double* gflop_total,
                     int64_t* launches, double* ms_max_layer, char* layer_name, int name_len);
/* one text line per recorded launch: cls name ci co k rate Ho Wo gflop ms gbytes
 * (gbytes = the launch's compulsory HBM GB: every operand read / written once) */
int seg_profile_dump(seg_ctx* ctx, char* buf, int len);

/* single-op entry points (parity tests of individual kernels) -------------------------- */
int seg_op_conv_fwd(int dtype, const void* x, int N, int H, int W, int C, int ldx,
                    const void* w, int Co, int k, int stride, int rate, int explicit_pad,
                    void* y, int ldy, float* stats, void* stream);
/* rows per BN-statistics partial written by seg_op_conv_fwd for this shape (128 or 256) */
int seg_op_conv_stat_rows(int dtype, int N, int H, int W, int C, int ldx, int Co, int ldy, int k,
                          int stride, int rate, int explicit_pad);
int seg_op_conv_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                      const void* w, int Ci, int k, int stride, int rate, int explicit_pad,
                      int H, int W, void* dx, int lddx, void* stream);
/* a 1 x 1 stride-1 data gradient with the identity units' epilogue: dx = dgrad(dy) + r (r may
 * be NULL; it may alias dx), stored masked by omask (ReLU bits [M][Ci/8], bit e of byte n/8 =
 * channel n; NULL = unmasked) -- the launches of the pre-masked residual chain (DESIGN.md §5b'',
 * §5f); 16-bit dtypes take the ping-pong kernel for Ci > 128: with r, persistent with the
 * residual tile by LDS-DMA and one rounding of dgrad + r (RQP); without, one tile per
 * workgroup */
int seg_op_conv_dgrad_res(int dtype, const void* dy, int N, int H, int W, int Co, int lddy,
                          const void* wt, int Ci, void* dx, int lddx, const void* r, int ldr,
                          const uint8_t* omask, void* stream);
int seg_op_conv_wgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                      const void* x, int H, int W, int Ci, int ldx, int k, int stride, int rate,
                      int explicit_pad, float* dw, void* workspace, int64_t ws_bytes,
                      void* stream);
/* bf16 weight gradient with an explicit tile (bm co x bn columns, each 64/128/256) and
 * split count: reaches every kernel configuration at test sizes (256 x 256 = ping-pong) */
int seg_op_conv_wgrad_cfg(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                          const void* x, int H, int W, int Ci, int ldx, int k, int stride, int rate,
                          int explicit_pad, float* dw, void* workspace, int64_t ws_bytes, int bm,
                          int bn, int splits, void* stream);

#ifdef __cplusplus
}
#endif
#endif

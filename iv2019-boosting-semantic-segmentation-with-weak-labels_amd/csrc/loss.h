// Fused hierarchical multi-loss head (define_losses_hierarchical.py:98-210 +
// resnet50_extended_model_hierarchical.py:84-117): align-corners bilinear upsampling of the
// low-res logits computed on the fly, softmax, l1 sparse CE (strong images), l2 soft CE
// (strong one-hot + weak segment-summed bbox/tag labels), weak-weight gating by the l1
// argmax, SUM_BY_NONZERO_WEIGHTS partial sums, and the gradient pushed back through the
// upsampler to low resolution without ever materialising full-resolution logits.
#pragma once
#include "seg_common.h"

#define SEG_MAX_PP 66
#define SEG_MAX_PB 15
struct LossTables {
  int c1, c2, c3;          // logits channels per head (14,7,3 cityscapes / 53,12,5 vistas)
  int n_pp, n_pb;          // per-pixel label classes (20/66), per-bbox classes (15)
  int cid_l1_vehicle, cid_l1_human;
  int l1_wmax;             // l1 weight = (l1 label <= l1_wmax)
  int pp2l1[SEG_MAX_PP], pp2veh[SEG_MAX_PP], pp2hum[SEG_MAX_PP];
  int pb2veh[SEG_MAX_PB], pb2hum[SEG_MAX_PB];
  int l1_to_common[64], veh_to_common[16], hum_to_common[8];
};

struct LossArgs {
  const float* logits;     // [N][Hl][Wl][ldl]: l1 | l2v | l2h channels
  int N, Hl, Wl, ldl;
  int H, W;                // full resolution
  int npp, npb, npi;       // sub-batch sizes: strong, bbox, tag (strong first)
  const int* px_labels;    // [npp][H][W] per-pixel class ids
  const float* bbox_soft;  // [npb][H][W][n_pb]
  const float* tag_soft;   // [npi][H][W][n_pb]
  float* grad_un;          // [N][Hl][Wl][ldl] unnormalised dL/dlogits (every channel written)
  float* part;             // [nblocks][8] partial sums {S1,S2v,S2h,n1,n2v,n2h}
  int* decisions;          // optional [N][H][W] fused decisions
  int* l1_decisions;       // optional [N][H][W]
};

// EVAL / PREDICT decisions (define_estimator_hierarchical.py:161-194,215-232): per output
// pixel, the NEAREST_NEIGHBOR align_corners source pixel of the network-resolution decision
// map (_resize_predictions :524-575), recomputed from the low-res logits exactly as the loss
// head does (bilinear, softmax, argmax, hierarchical fusion), mapped through the training ->
// evaluation/inference cid table (_map_predictions_to_new_cids :490-522) and, optionally,
// void decisions replaced by the l1 top-k rule (_replace_voids :577-630).
struct EvalArgs {
  const float* logits;     // [N][Hl][Wl][ldl]
  int N, Hl, Wl, ldl;
  int H, W;                // network resolution (where decisions are formed)
  int Ho, Wo;              // output (label) resolution
  int replace_voids;       // 0 no, 1 EVAL order (replace, then resize), 2 PREDICT order
  int n_map;               // entries of map (= training classes)
  int map[SEG_MAX_PP];     // training cid -> new cid (voids already replaced)
  int* out;                // [N][Ho][Wo]
};

// Full-resolution predictions of the model (hierarchical.py:84-130) at network resolution;
// each output is optional (nullptr skips it)
struct FullPredArgs {
  const float* logits;     // [N][Hl][Wl][ldl]
  int N, Hl, Wl, ldl;
  int H, W;                // network resolution
  float* logits_out;       // [N][H][W][c1+c2+c3] upsampled logits (l1 | l2v | l2h)
  float* probs_out;        // [N][H][W][c1+c2+c3] per-head softmax
  int* head_decs_out;      // [N][H][W][3] per-head argmax (l1, l2v, l2h)
  int* decs_out;           // [N][H][W] fused decisions in common cids
};

int loss_head_blocks(int N, int Hl, int Wl);
hipError_t launch_eval_decisions(const EvalArgs& a, const LossTables& t, hipStream_t s);
hipError_t launch_full_predictions(const FullPredArgs& a, const LossTables& t, hipStream_t s);
hipError_t launch_loss_head(const LossArgs& a, const LossTables& t, hipStream_t s);
// true when launch_loss_head takes the y-first kernel for this geometry (Cityscapes tables)
bool loss_head_yf(int W, int Wl);
// out[0..9] = {seg, l1, l2v, l2h, n1, n2v, n2h, f1, f2v, f2h}; dzscale[ldl] per-channel
// factors (1/n1 | 0.1/n2v | 0.1/n2h; 0 where the count is 0)
hipError_t launch_loss_finalize(const float* part, int nblocks, const LossTables& t, int ldl,
                                float loss_scale,
                                float* out, float* dzscale, hipStream_t s);
hipError_t launch_confusion(const int* labels, const int* decisions, long n, int num_classes,
                            int* cm, hipStream_t s);

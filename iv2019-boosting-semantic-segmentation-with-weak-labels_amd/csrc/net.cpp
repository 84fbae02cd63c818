// Native runtime of the training step: builds the dilated-ResNet + pyramid + hierarchical
// heads graph (slim resnet_v1 unit schedule, reference models/*), owns activations and
// workspace, sequences the HIP kernels for forward / loss / backward / update, and exports
// the C ABI declared in include/seg_hip.h.
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "../../include/seg_hip.h"
#include "bn.h"
#include "lbf.h"
#include "input.h"
#include "conv.h"
#include "deconv.h"
#include "gn.h"
#include "loss.h"
#include "labels.h"
#include "optim.h"
#include "pool.h"

namespace {

thread_local std::string g_err;

int set_err(std::string* dst, int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  if (dst) *dst = buf;
  g_err = buf;
  return code;
}

struct Act {
  void* p = nullptr;
  int N = 0, H = 0, W = 0, C = 0, ld = 0;
  uint8_t* mask = nullptr;   // ReLU bits [M][C/8] of a BN+ReLU output (read by the backward)
  long M() const { return (long)N * H * W; }
};

struct ConvL {
  std::string name;
  int ci, co, k, stride, rate;
  bool explicit_pad, relu;
  long w_off = 0, g_off = 0, b_off = 0, mv_off = 0;  // flat offsets
  int N = 0, H = 0, W = 0, Ho = 0, Wo = 0, pad_h = 0, pad_w = 0;
  int co_pad = 0;                 // wgrad row padding (co % 8 != 0)
  void* w_lp = nullptr;           // compute-dtype weights [co][k][k][ci]
  void* wt_lp = nullptr;          // flipped transpose [ci][k][k][co] (dgrad)
  bool need_dgrad = true;
  Act x;                          // input of the last forward (not owned)
  Act y, dy;                      // conv output and its gradient
  BnState st{};
  float* stats_part = nullptr;    // [mtiles][co][2]
  float* bwd_part = nullptr;      // [rb][co][2] (group norm: [N][rb][co][2], rb per image)
  int rb = 1;
  // linear BN-backward fold (lbf.h; an identity unit's expansion conv3): per-channel (A, B, D)
  // [3][co] of the last backward, the gated gradient it read (seg_debug_tensor materialises dy
  // from it on request: the step itself never writes dy of such a layer)
  float* lbf_coef = nullptr;
  float* lbf_cs = nullptr;        // [rb of the unit's conv2 BN][ci] column-sum partials of y2
  bool lbf_done = false;          // folded in the last backward
  bool lbf_dy_ready = false;      // ... and dy materialised since (seg_debug_tensor)
  Act lbf_dyhat;
  // group norm: groups, per-image states (host copies of the device array st_dev) and the
  // forward chunk partials
  int groups = 0;
  std::vector<BnState> st_img;
  BnState* st_dev = nullptr;
  float* gn_part = nullptr;
};

enum ShortcutKind { SC_IDENTITY = 0, SC_SUBSAMPLE = 1, SC_CONV = 2 };

struct Unit {
  int sc = -1, c1 = -1, c2 = -1, c3 = -1;
  ShortcutKind kind = SC_IDENTITY;
  int stride = 1;
  Act in, out;        // in is not owned (previous output)
  Act z1, z2;         // post BN+ReLU of conv1/conv2
  Act dz1, dz2, dpre; // gradients; dpre = relu-masked gradient of out (identity/subsample)
  Act dout;           // gradient wrt out (owned)
  // this step's dout was written already ReLU-masked by the next unit's conv1 data gradient
  // (unit_backward): the c3 BN backward reads it without the bits and dout serves as dpre
  bool dout_masked = false;
};

struct Prof {
  bool on = false;
  std::vector<hipEvent_t> ev;
  // gflop: algorithmic work (conv classes) or algorithmic GB (BN classes); gbytes: the
  // launch's compulsory HBM bytes (every operand read / written once) in GB
  struct Rec { int cls; int layer; double gflop; int e0, e1; double gbytes; };
  std::vector<Rec> recs;
  int next = 0;
};

}  // namespace

static int dt_of(int abi_dtype) {
  return abi_dtype == SEG_DTYPE_BF16 ? SEG_BF16 : (abi_dtype == SEG_DTYPE_F16 ? SEG_F16 : SEG_F32);
}

struct seg_ctx {
  seg_cfg cfg{};
  int device = 0;
  int dt = SEG_BF16;
  size_t esz = 2;
  std::string err;
  std::vector<void*> allocs;

  // parameters
  std::vector<ConvL> convs;
  long n_train = 0, n_decay = 0, n_moving = 0, n_stats = 0;
  struct PInfo { std::string name; long off, numel; int kind; int dims[4]; };
  std::vector<PInfo> pinfo;
  float* params = nullptr;
  float* grads = nullptr;
  float* mom = nullptr;
  float* ema = nullptr;
  float* moving = nullptr;
  void* w_lp_flat = nullptr;      // bf16 copy of the conv-weight region (bf16 mode)

  // graph
  Act img;                        // compute-dtype images
  int stem = -1;
  // 16-bit stem as a 4 x 4 conv over the space-to-depth image (conv.h): img [N][Ho+3][Wo+3][16],
  // weights [64][256] (stem_wpad); img_dbg = the [N][H][W][8] image view for seg_debug_tensor
  bool stem_s2d = false;
  void* img_dbg = nullptr;
  FlipJob* flip_jobs = nullptr;   // device table: every dgrad weight flip in one launch
  int n_flip = 0;
  long flip_total = 0;
  bf16_t* stem_wpad = nullptr;
  Act z0, dz0, p0, dp0;
  bool z0_stale = false;   // the fused stem BN + ReLU + max-pool did not store z0 (see forward)
  uint8_t* pool_arg = nullptr;    // max-pool first-max window index per output element
  int pool_ph = 0, pool_pw = 0;
  std::vector<Unit> units;
  int dfd = -1;
  Act z_dfd, dz_dfd;              // extension output (pyramid input); may be a slice of concat
  int fov = -1;                   // optional extension/increase_fov conv after decrease_fdims
  Act z_pre, dz_pre;              // decrease_fdims BN/ReLU output when fov >= 0
  // pyramid
  std::vector<int> pyr_conv;      // per branch conv index
  std::vector<int> pyr_k;         // grid size per branch
  std::vector<Act> pooled, dpooled, zb, dzb;
  int pyr_final = -1;
  Act concat, dconcat;
  Act feat, dfeat;
  GridSpec pool_grids{};          // avg-pool grids over z_dfd
  std::vector<GridSpec> up_grids; // resize-transpose per branch
  float* grid_part = nullptr;     // [N][Hf][cells][C]
  // heads
  Unit heads[3];
  int logit_conv[3] = {-1, -1, -1};
  Act logits;                     // fp32 [N][Hl][Wl][ldl]
  float* grad_un = nullptr;       // fp32 same shape (gradient w.r.t. head_in)
  bool gn = false;                // norm_layer = group (gn.h)
  float* gn_gscaled = nullptr;    // group norm: the logits gradient times the loss factors
  // 'hybrid' upsampling: per-head 3x3 conv2d_transpose + bias on the logits (deconv.h)
  bool hybrid = false;
  long dc_w_off[3] = {0, 0, 0}, dc_b_off[3] = {0, 0, 0}, dc_b_lo = 0;
  float* up_in = nullptr;         // deconv output [N][Hl][Wl][ldl]
  float* dc_dx = nullptr;         // gradient w.r.t. the logits [N][Hl][Wl][ldl]
  float* dc_part = nullptr;       // weight-gradient tile partials
  const float* head_in = nullptr; // what the bilinear upsampler reads: logits or up_in
  int ldl = 0, nc[3] = {0, 0, 0};
  LossTables tables{};
  float* loss_part = nullptr;
  int loss_blocks = 0;
  float* loss_out = nullptr;      // [10]
  // gradient all-reduce buckets in ready order: conv-weight ranges [lo, hi) cut at layer
  // boundaries walking the layers in reverse (the backward's order), then the BN-parameter +
  // batch-statistics tail. An event is recorded on the backward stream as soon as every
  // weight gradient of a bucket has been written, so a collective on another stream can
  // start while the rest of the backward runs.
  std::vector<long> bk_lo, bk_hi;
  std::vector<std::vector<int>> bk_convs;
  std::vector<hipEvent_t> bk_ev;
  std::vector<char> wg_done;
  int bk_next = 0;
  // backward on two streams: every weight gradient runs on `side` (waiting for its layer's
  // dy on the compute stream), so the dgrad -> BN-backward chain and the wgrads overlap
  // cross-replica BN (seg_set_bn_sync): per-layer moment exchange through the caller's hook
  seg_allreduce_fn sync_fn = nullptr;
  int bn_infer = 0;   // seg_set_bn_inference: forward normalises with the moving statistics
  BnInferJob* infer_jobs = nullptr;   // device table: every layer's moving stats -> BnState
  void* sync_user = nullptr;
  int sync_world = 1;
  float* sync_pack = nullptr;     // [2 * max C]
  float loss_scale = 1.f;         // gradient seed multiplier (fp16 dynamic loss scaling)
  int nesterov = 0;               // MomentumOptimizer use_nesterov (seg_set_nesterov)
  int* skip_flag = nullptr;       // device: non-finite scaled gradients this step (update skipped)
  bool side_on = false;
  bool side_active = false;        // this backward: side_on and not profiling (kernel-alone timing)
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> ev_dy;   // per conv: dy written on the compute stream
  hipEvent_t ev_join = nullptr;
  // seg_set_defer_stem: the backward's compute stream joins the weight-gradient stream before the
  // stem's weight gradient (ev_prestem) instead of after it; seg_apply_update updates every other
  // parameter beside that last kernel and joins (ev_join) before the stem's weights
  hipEvent_t ev_prestem = nullptr;
  bool defer_stem = false;
  bool premask = true;             // seg_set_premask: pre-masked identity-unit gradients (unit_backward)
  int64_t premask_launches = 0;    // conv1 data gradients stored pre-masked (seg_counter)
  int64_t loss_yf_launches = 0;    // loss heads run by the y-first kernel (seg_counter)
  bool prestem_rec = false;
  bool stem_pending = false;
  float* dzscale = nullptr;       // [ldl]
  float* reg_part = nullptr;
  float* reg_out = nullptr;
  // workspace
  float* slab = nullptr;
  size_t slab_floats = 0;
  // linear BN-backward fold (lbf.h), on unless seg_set_lbf(ctx, 0): 16-bit bottleneck units
  // whose conv3 expands (co >= 2 ci, ci % 64 == 0: every unit of R50). Compute-stream scratch (used in
  // order by one layer at a time): the scaled data-gradient weights, the D-scaled weights, H
  // and its split-K slab, the data gradient's constant; weight-gradient-stream scratch: the
  // two GEMM results and the column-sum partials of the conv input
  bool lbf_on = true;
  void* lbf_wts = nullptr;
  void* lbf_xd = nullptr;
  void* lbf_h = nullptr;
  float* lbf_hslab = nullptr;
  float* lbf_bias = nullptr;
  float* lbf_bpart = nullptr;
  float* lbf_p1 = nullptr;
  int64_t lbf_launches = 0;        // layers folded (seg_counter)
  float* stat_scratch = nullptr;
  size_t stat_scratch_floats = 0;
  Prof prof;
  bool bound = false;
};

namespace {

int hip_fail(seg_ctx* c, hipError_t e, const char* where) {
  return set_err(c ? &c->err : nullptr, -EIO, "%s: %s", where, hipGetErrorString(e));
}
#define HIPCALL(c, expr)                                    \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return hip_fail((c), _e, #expr);  \
  } while (0)

template <typename T>
int dalloc(seg_ctx* c, T** p, size_t count) {
  void* q = nullptr;
  size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess) return hip_fail(c, e, "hipMalloc");
  (void)hipMemset(q, 0, bytes);
  c->allocs.push_back(q);
  *p = (T*)q;
  return 0;
}

int alloc_act(seg_ctx* c, Act& a, int N, int H, int W, int C, int ld = 0, size_t esz = 0) {
  a.N = N; a.H = H; a.W = W; a.C = C; a.ld = ld ? ld : C;
  size_t e = esz ? esz : c->esz;
  char* p = nullptr;
  int r = dalloc(c, &p, (size_t)a.M() * a.ld * e);
  a.p = p;
  return r;
}

// ReLU-output activation with its bit mask (C % 8 == 0)
int alloc_relu_act(seg_ctx* c, Act& a, int N, int H, int W, int C, int ld = 0) {
  if (int r = alloc_act(c, a, N, H, W, C, ld)) return r;
  if (C % 8) return 0;
  return dalloc(c, &a.mask, (size_t)a.M() * (C / 8));
}

Act slice(const seg_ctx* c, const Act& a, int c_off, int C) {
  Act v = a;
  v.p = (char*)a.p + (size_t)c_off * c->esz;
  v.C = C;
  return v;
}

// ------------------------------------------------------------------------------------------
// architecture (slim resnet_v1 / stack_blocks_dense; reference models/* — see oracle/tfseg)
// ------------------------------------------------------------------------------------------
int add_conv(seg_ctx* c, const std::string& name, int ci, int co, int k, int stride, int rate,
             bool explicit_pad, bool relu) {
  ConvL L;
  L.name = name; L.ci = ci; L.co = co; L.k = k; L.stride = stride; L.rate = rate;
  L.explicit_pad = explicit_pad; L.relu = relu;
  c->convs.push_back(L);
  return (int)c->convs.size() - 1;
}

struct UnitSpec { std::string scope; int din, d, dbn, s, r; };

std::vector<UnitSpec> resnet_units(int depth, int output_stride) {
  const int n3 = depth == 101 ? 23 : 6;
  struct B { const char* n; int base, units, stride; } blocks[4] = {
      {"block1", 64, 3, 2}, {"block2", 128, 4, 2}, {"block3", 256, n3, 2}, {"block4", 512, 3, 1}};
  const int target = output_stride / 4;
  int current = 1, rate = 1, din = 64;
  std::vector<UnitSpec> out;
  for (auto& b : blocks) {
    for (int i = 0; i < b.units; ++i) {
      int us = i == b.units - 1 ? b.stride : 1;
      std::string scope = std::string(b.n) + "/unit_" + std::to_string(i + 1) + "/bottleneck_v1";
      if (current == target) {
        out.push_back({scope, din, b.base * 4, b.base, 1, rate});
        rate *= us;
      } else {
        out.push_back({scope, din, b.base * 4, b.base, us, 1});
        current *= us;
      }
      din = b.base * 4;
    }
  }
  return out;
}

void add_bottleneck(seg_ctx* c, Unit& u, const std::string& scope, int din, int d, int dbn, int s,
                    int r) {
  if (d != din) {
    u.sc = add_conv(c, scope + "/shortcut", din, d, 1, s, 1, false, false);
    u.kind = SC_CONV;
  } else {
    u.kind = s > 1 ? SC_SUBSAMPLE : SC_IDENTITY;
  }
  u.stride = s;
  u.c1 = add_conv(c, scope + "/conv1", din, dbn, 1, 1, 1, false, true);
  u.c2 = add_conv(c, scope + "/conv2", dbn, dbn, 3, s, r, s > 1, true);
  u.c3 = add_conv(c, scope + "/conv3", dbn, d, 1, 1, 1, false, false);
}

void fill_tables(LossTables& t, int dataset) {
  memset(&t, 0, sizeof(t));
  if (dataset == SEG_DATASET_VISTAS) {
    // define_losses_hierarchical.py:37-74; hierarchical.py:146-156
    t.c1 = 53; t.c2 = 12; t.c3 = 5; t.n_pp = 66; t.n_pb = 15;
    t.cid_l1_vehicle = 49; t.cid_l1_human = 19; t.l1_wmax = 51;
    const int pp2l1[66] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19,
                           19, 19, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34,
                           35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47, 48, 49, 49, 49, 49,
                           49, 49, 49, 49, 49, 49, 49, 50, 51, 52};
    const int pb2l1[15] = {49, 49, 49, 49, 49, 49, 19, 19, 19, 19, 19, 52, 52, 52, 52};
    (void)pb2l1;
    int pp2veh[66], pp2hum[66];
    for (int i = 0; i < 66; ++i) { pp2veh[i] = 11; pp2hum[i] = 4; }
    for (int i = 0; i < 11; ++i) pp2veh[52 + i] = i;
    pp2hum[19] = 0; pp2hum[20] = 1; pp2hum[21] = 2; pp2hum[22] = 3;
    const int pb2veh[15] = {0, 2, 3, 5, 6, 9, 11, 11, 11, 11, 11, 11, 11, 11, 11};
    const int pb2hum[15] = {4, 4, 4, 4, 4, 4, 0, 0, 0, 0, 0, 4, 4, 4, 4};
    for (int i = 0; i < 66; ++i) { t.pp2l1[i] = pp2l1[i]; t.pp2veh[i] = pp2veh[i]; t.pp2hum[i] = pp2hum[i]; }
    for (int i = 0; i < 15; ++i) { t.pb2veh[i] = pb2veh[i]; t.pb2hum[i] = pb2hum[i]; }
    for (int i = 0; i < 20; ++i) t.l1_to_common[i] = i;
    for (int i = 20; i < 50; ++i) t.l1_to_common[i] = i + 3;
    t.l1_to_common[50] = 63; t.l1_to_common[51] = 64; t.l1_to_common[52] = 65;
    for (int i = 0; i < 11; ++i) t.veh_to_common[i] = 52 + i;
    t.veh_to_common[11] = 65;
    const int h2c[5] = {19, 20, 21, 22, 65};
    for (int i = 0; i < 5; ++i) t.hum_to_common[i] = h2c[i];
  } else {
    // define_losses_hierarchical.py:75-93; hierarchical.py:157-162
    t.c1 = 14; t.c2 = 7; t.c3 = 3; t.n_pp = 20; t.n_pb = 15;
    t.cid_l1_vehicle = 12; t.cid_l1_human = 11; t.l1_wmax = 12;
    const int pp2l1[20] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 11, 12, 12, 12, 12, 12, 12, 13};
    const int pp2veh[20] = {6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 6, 0, 1, 2, 3, 4, 5, 6};
    const int pp2hum[20] = {2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 0, 1, 2, 2, 2, 2, 2, 2, 2};
    const int pb2veh[15] = {5, 2, 0, 4, 3, 1, 6, 6, 6, 6, 6, 6, 6, 6, 6};
    const int pb2hum[15] = {2, 2, 2, 2, 2, 2, 0, 0, 0, 0, 0, 2, 2, 2, 2};
    for (int i = 0; i < 20; ++i) { t.pp2l1[i] = pp2l1[i]; t.pp2veh[i] = pp2veh[i]; t.pp2hum[i] = pp2hum[i]; }
    for (int i = 0; i < 15; ++i) { t.pb2veh[i] = pb2veh[i]; t.pb2hum[i] = pb2hum[i]; }
    const int l1c[14] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 19};
    const int vc[7] = {13, 14, 15, 16, 17, 18, 19};
    const int hc[3] = {11, 12, 19};
    for (int i = 0; i < 14; ++i) t.l1_to_common[i] = l1c[i];
    for (int i = 0; i < 7; ++i) t.veh_to_common[i] = vc[i];
    for (int i = 0; i < 3; ++i) t.hum_to_common[i] = hc[i];
  }
}

// TF ResizeBilinear(align_corners=True) legacy index/lerp (float arithmetic)
void tf_lerp_host(int o, int n_in, int n_out, int& lo, int& hi, float& l) {
  float scale = n_out > 1 ? (float)(n_in - 1) / (float)(n_out - 1) : 0.f;
  float fin = (float)o * scale;
  lo = (int)fin;
  hi = std::min(lo + 1, n_in - 1);
  l = fin - (float)lo;
}

// geometry of a conv on an input of spatial size (H, W)
void conv_geom(ConvL& L, int N, int H, int W) {
  L.N = N; L.H = H; L.W = W;
  const int keff = L.k + (L.k - 1) * (L.rate - 1);
  if (L.explicit_pad) {  // conv2d_same, stride > 1: pad (keff-1)//2 before, rest after, VALID
    L.pad_h = L.pad_w = (keff - 1) / 2;
    L.Ho = (H + keff - 1 - keff) / L.stride + 1;
    L.Wo = (W + keff - 1 - keff) / L.stride + 1;
  } else {               // SAME (only stride 1 here): out = ceil(n/s)
    L.Ho = (H + L.stride - 1) / L.stride;
    L.Wo = (W + L.stride - 1) / L.stride;
    int tot_h = std::max((L.Ho - 1) * L.stride + keff - H, 0);
    int tot_w = std::max((L.Wo - 1) * L.stride + keff - W, 0);
    L.pad_h = tot_h / 2;
    L.pad_w = tot_w / 2;
  }
}

int alloc_conv(seg_ctx* c, ConvL& L, int N, int H, int W, int ldy = 0) {
  conv_geom(L, N, H, W);
  L.co_pad = (L.co % 8) ? ((L.co + 15) / 16) * 16 : L.co;
  int ld = ldy ? ldy : L.co_pad;
  if (int r = alloc_act(c, L.y, N, L.Ho, L.Wo, L.co, ld)) return r;
  if (int r = alloc_act(c, L.dy, N, L.Ho, L.Wo, L.co, ld)) return r;
  float* v;
  if (int r = dalloc(c, &v, (size_t)6 * L.co)) return r;
  L.st.mean = v; L.st.invstd = v + L.co; L.st.scale = v + 2 * L.co; L.st.var_unb = v + 3 * L.co;
  L.st.sdy = v + 4 * L.co; L.st.sdyx = v + 5 * L.co;
  long M = (long)N * L.Ho * L.Wo;
  if (int r = dalloc(c, &L.stats_part, (size_t)conv_nt_mtiles(M) * L.co * 2)) return r;
  if (c->gn) {
    const long hw = (long)L.Ho * L.Wo;
    L.rb = bn_bwd_rowblocks(hw, L.co);
    if (int r = dalloc(c, &L.bwd_part, (size_t)N * L.rb * L.co * 2)) return r;
    if (int r = dalloc(c, &L.gn_part, (size_t)N * gn_chunks(hw) * L.co * 2)) return r;
    float* sv;
    if (int r = dalloc(c, &sv, (size_t)N * 6 * L.co)) return r;
    L.st_img.resize(N);
    for (int n = 0; n < N; ++n) {
      float* b = sv + (size_t)n * 6 * L.co;
      L.st_img[n] = BnState{b, b + L.co, b + 2 * L.co, b + 3 * L.co, b + 4 * L.co, b + 5 * L.co};
    }
    if (int r = dalloc(c, &L.st_dev, (size_t)N)) return r;
    HIPCALL(c, hipMemcpy(L.st_dev, L.st_img.data(), N * sizeof(BnState), hipMemcpyHostToDevice));
  } else {
    L.rb = bn_bwd_rowblocks(M, L.co);
    if (int r = dalloc(c, &L.bwd_part, (size_t)L.rb * L.co * 2)) return r;
  }
  size_t need = (size_t)((conv_nt_mtiles(M) + 63) / 64) * L.co * 3;
  c->stat_scratch_floats = std::max(c->stat_scratch_floats, need);
  return 0;
}

// concurrent = the weight gradient runs on the side stream beside the dgrad -> BN chain:
// at most ~128 workgroups (half the CUs, the chain keeps the other half: 90.4 -> 92.9 img/s
// on C2 against 512, and half the split-K slab traffic); alone (profiled, single stream,
// seg_op_*): at most one wave of the 256 CUs (one workgroup per CU, LDS-bound). The weight-
// gradient kernels run one workgroup per CU, so a launch of 256 + a few workgroups pays a
// whole second wave for the few: tools/wgrad_sweep.py PP_ONLY=1 on the C2 shapes, e.g. block3
// 3x3 (9 tiles) 24 splits 188 us, 32 splits (288 workgroups) 266 us; block3 1x1 (4 tiles) 64
// splits 97 us against the former 2-wave 128 splits 121 us.
int wgrad_splits(const WgradArgs& a, int dt, bool concurrent = false) {
  const int ci = a.C, k = a.KH, co = a.Co;   // Co = co_pad; 16 / 4 for the space-to-depth stem
  int BM = co <= 64 ? 64 : 128;
  int BN = 128;
  long P = (long)a.N * a.Ho * a.Wo;
  if (ci % 8 == 0) conv_wgrad_v2_tile(co, k * k * ci, P, &BM, &BN);
  long tiles = (long)((co + BM - 1) / BM) * ((k * k * ci + BN - 1) / BN);
  // the small-channel 3 x 3 patch kernel: the same predicate launch_conv_wgrad dispatches on
  if (seg_half(dt) && conv_wgrad_patch_ok(a)) tiles = conv_wgrad_patch_blocks(a);
  // workgroups = tiles x splits <= one wave of the CUs the launch may use; each split >= 32
  // K-steps of 64 pixels beside the dgrad chain, >= 16 alone
  const long target = concurrent ? 128 : 256;
  long s = std::max<long>(1, target / std::max<long>(tiles, 1));
  long maxs = std::max<long>(1, P / (concurrent ? 2048 : 1024));
  s = std::min(s, maxs);
  return (int)std::min<long>(s, 256);
}

// the weight-gradient problem of layer L (x / dy pixel strides: the activations' layout,
// channels padded to a multiple of 8); the space-to-depth stem is a 4 x 4 VALID conv over 16
// channels
WgradArgs wgrad_problem(const ConvL& L, bool s2d) {
  WgradArgs a{};
  a.N = L.N; a.H = L.H; a.W = L.W; a.C = s2d ? 16 : L.ci; a.ldx = (a.C + 7) / 8 * 8;
  a.Ho = L.Ho; a.Wo = L.Wo; a.Co = L.co_pad; a.lddy = (L.co_pad + 7) / 8 * 8;
  a.KH = a.KW = s2d ? 4 : L.k; a.sf = s2d ? 1 : L.stride; a.dil = s2d ? 1 : L.rate;
  a.pad_h = s2d ? 0 : L.pad_h; a.pad_w = s2d ? 0 : L.pad_w;
  return a;
}

// ------------------------------------------------------------------------------------------
// kernel sequencing helpers
// ------------------------------------------------------------------------------------------
struct Step {
  seg_ctx* c;
  hipStream_t s;
  int dt;
};

int prof_begin(seg_ctx* c, hipStream_t s, int cls, int layer, double gflop, int* slot,
               double gbytes = -1.0) {
  *slot = -1;
  if (!c->prof.on) return 0;
  if (c->prof.next + 2 > (int)c->prof.ev.size()) return 0;
  int e0 = c->prof.next++, e1 = c->prof.next++;
  HIPCALL(c, hipEventRecord(c->prof.ev[e0], s));
  c->prof.recs.push_back({cls, layer, gflop, e0, e1, gbytes < 0 ? gflop : gbytes});
  *slot = (int)c->prof.recs.size() - 1;
  return 0;
}
int prof_end(seg_ctx* c, hipStream_t s, int slot) {
  if (slot < 0) return 0;
  HIPCALL(c, hipEventRecord(c->prof.ev[c->prof.recs[slot].e1], s));
  return 0;
}

// one cross-replica exchange (SUM in place, ordered on stream s) through the caller's hook
int sync_exchange(seg_ctx* c, float* buf, long n, hipStream_t s) {
  const int r = c->sync_fn(c->sync_user, buf, (int64_t)n, s);
  if (r) return set_err(&c->err, -EIO, "cross-replica BN exchange failed (hook returned %d)", r);
  return 0;
}

int conv_forward(Step& S, int li, const Act& x) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  L.x = x;
  ConvArgs a{};
  a.x = x.p; a.N = x.N; a.H = x.H; a.W = x.W; a.C = x.C; a.ldx = x.ld;
  a.w = L.w_lp; a.ldw = L.k * L.k * L.ci;
  a.y = L.y.p; a.Ho = L.Ho; a.Wo = L.Wo; a.Co = L.co; a.ldy = L.y.ld;
  a.KH = a.KW = L.k; a.sf = L.stride; a.st = 1; a.pad_h = L.pad_h; a.pad_w = L.pad_w;
  a.dil = L.rate; a.stats = L.stats_part;
  if (li == c->stem && c->stem_s2d) {   // 4 x 4 VALID over the space-to-depth image
    a.C = 16; a.ldx = 16; a.tap8 = 2; a.w = c->stem_wpad; a.ldw = 256;
    a.KH = a.KW = 4; a.sf = 1; a.pad_h = a.pad_w = 0; a.dil = 1;
  }
  long M = (long)x.N * L.Ho * L.Wo;
  int slot;
  const double esz = c->esz;   // x + w + y, each once
  const double gbx = ((double)L.N * L.H * L.W * L.ci + (double)L.co * L.k * L.k * L.ci +
                      (double)M * L.co) * esz * 1e-9;
  if (int r = prof_begin(c, S.s, 0, li, 2.0 * M * L.co * L.k * L.k * L.ci * 1e-9, &slot, gbx)) return r;
  HIPCALL(c, launch_conv_nt(S.dt, 0, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  if (c->gn) {   // group norm: per-image statistics in every mode (no moving statistics)
    GnPartArgs g{};
    g.y = L.y.p; g.ldy = L.y.ld; g.N = x.N; g.hw = (long)L.Ho * L.Wo; g.C = L.co; g.part = L.gn_part;
    HIPCALL(c, launch_gn_partial(S.dt, 0, g, S.s));
    HIPCALL(c, launch_gn_stats_final(L.gn_part, x.N, g.hw, L.co, L.groups, c->params + L.g_off,
                                     L.st_dev, S.s));
    return 0;
  }
  if (c->bn_infer) return 0;   // is_training=False: the statistics were set for every layer
                               // by one launch at the start of the forward
  const bool sync = c->sync_fn != nullptr;
  HIPCALL(c, launch_bn_stats_finalize(L.stats_part, M, L.co, conv_nt_stat_rows(S.dt, 0, a), c->stat_scratch,
                                      c->params + L.g_off, L.st, S.s, sync ? c->sync_pack : nullptr));
  if (sync) {
    if (int r = sync_exchange(c, c->sync_pack, 2L * L.co, S.s)) return r;
    HIPCALL(c, launch_bn_sync_unpack(c->sync_pack, L.co, 1.f / c->sync_world, c->params + L.g_off,
                                     L.st, S.s));
  }
  return 0;
}

// out = act(bn(y) [+ residual])
int bn_apply_one(Step& S, int li, const Act& out, int out_f32, const Act* res, int rs, int li2,
                 int relu, int img);

int bn_apply(Step& S, int li, const Act& out, int out_f32, const Act* res = nullptr, int rs = 1,
             int li2 = -1, int relu = -1) {
  if (!S.c->gn) return bn_apply_one(S, li, out, out_f32, res, rs, li2, relu, -1);
  // group norm: the per-image affine is per channel; one launch per image on row offsets
  for (int n = 0; n < out.N; ++n)
    if (int r = bn_apply_one(S, li, out, out_f32, res, rs, li2, relu, n)) return r;
  return 0;
}

// one image's rows of an activation (img < 0: all of it)
Act image_rows(const Act& a, int img, size_t esz) {
  if (img < 0) return a;
  Act v = a;
  const size_t hw = (size_t)a.H * a.W;
  v.p = (char*)a.p + (size_t)img * hw * a.ld * esz;
  if (a.mask) v.mask = a.mask + (size_t)img * hw * (a.C / 8);
  v.N = 1;
  return v;
}

int bn_apply_one(Step& S, int li, const Act& out0, int out_f32, const Act* res0, int rs, int li2,
                 int relu, int img) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  const Act out = image_rows(out0, img, out_f32 ? 4 : c->esz);
  Act res_img;
  const Act* res = res0;
  if (res0 && img >= 0) { res_img = image_rows(*res0, img, c->esz); res = &res_img; }
  const Act Y = image_rows(L.y, img, c->esz);
  const BnState& st = img >= 0 ? L.st_img[img] : L.st;
  BnApplyArgs a{};
  a.y = Y.p; a.ldy = Y.ld; a.M = Y.M(); a.C = L.co;
  a.mean = st.mean; a.scale = st.scale; a.beta = c->params + L.b_off;
  a.relu = relu < 0 ? (L.relu ? 1 : 0) : relu;
  if (res) {
    a.res = res->p; a.ldres = res->ld; a.rs = rs; a.Ho = L.Ho; a.Wo = L.Wo; a.Hr = res->H;
    a.Wr = res->W;
  }
  if (li2 >= 0) {
    ConvL& L2 = c->convs[li2];
    const Act Y2 = image_rows(L2.y, img, c->esz);
    const BnState& st2 = img >= 0 ? L2.st_img[img] : L2.st;
    a.y2 = Y2.p; a.ldy2 = Y2.ld; a.mean2 = st2.mean; a.scale2 = st2.scale;
    a.beta2 = c->params + L2.b_off;
  }
  a.out = out.p; a.ldo = out.ld;
  a.mask = a.relu ? out.mask : nullptr;
  const double esz = seg_half(S.dt) ? 2.0 : 4.0;
  const double gb = a.M * (double)a.C * (esz * (1 + (a.res || a.y2 ? 1 : 0)) +
                                         (out_f32 ? 4.0 : esz)) * 1e-9;
  int slot;
  if (int r = prof_begin(c, S.s, 3, li, gb, &slot)) return r;
  HIPCALL(c, launch_bn_apply(S.dt, out_f32, a, S.s));
  return prof_end(c, S.s, slot);
}

int gn_backward(Step& S, int li, const Act& dz, int dz_f32, const Act* z, const Act* dyhat_out,
                const float* dzscale);

// BN backward for layer li: dz (gradient wrt BN output), z (mask source or null). dshift: a
// per-channel term of dz its producer left out (added before the gate; bits only);
// reduce_only: reduce + finalize (the linear BN-backward fold replaces the apply), the gated
// gradient stored by the reduce when dyhat_out is given
int bn_backward(Step& S, int li, const Act& dz, int dz_f32, const Act* z, const Act* dyhat_out,
                const float* dzscale = nullptr, const float* dshift = nullptr,
                bool reduce_only = false, float* cs_out = nullptr) {
  seg_ctx* c = S.c;
  if (c->gn) return gn_backward(S, li, dz, dz_f32, z, dyhat_out, dzscale);
  ConvL& L = c->convs[li];
  BnBwdArgs a{};
  a.dz = dz.p; a.lddz = dz.ld;
  if (z) { a.z = z->p; a.ldz = z->ld; }
  if (z && z->mask && !dz_f32 && !dzscale && z->C == L.co) { a.mask = z->mask; a.z = nullptr; }
  a.y = L.y.p; a.ldy = L.y.ld; a.M = L.y.M(); a.C = L.co;
  a.mean = L.st.mean; a.invstd = L.st.invstd; a.scale = L.st.scale;
  a.sdy = L.st.sdy; a.sdyx = L.st.sdyx;
  a.dy = L.dy.p; a.lddy = L.dy.ld;
  if (dyhat_out) { a.dyhat = dyhat_out->p; a.lddyhat = dyhat_out->ld; }
  a.part = L.bwd_part; a.rb = L.rb;
  a.dzscale = dzscale;
  a.dshift = dshift;
  a.reduce_dyhat = reduce_only && dyhat_out ? 1 : 0;
  if (cs_out) { a.cs_part = cs_out; a.beta = c->params + L.b_off; }
  if ((dshift || a.reduce_dyhat || cs_out) && !a.mask)
    return set_err(&c->err, -EINVAL, "bn_backward %s: shift / reduce-side dyhat need the ReLU bits", L.name.c_str());
  const double esz = seg_half(S.dt) ? 2.0 : 4.0, zsz = dz_f32 ? 4.0 : esz;
  const double me = a.M * (double)a.C * 1e-9;
  const double gb_in = me * (zsz + (a.mask ? 0.125 : (z ? zsz : 0.0)) + esz);
  int slot;
  if (int r = prof_begin(c, S.s, 4, li, gb_in + (a.reduce_dyhat ? me * esz : 0.0), &slot)) return r;
  HIPCALL(c, launch_bn_bwd_reduce(S.dt, dz_f32, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  const bool tb = c->cfg.train_bn != 0;
  // a backward after a moving-statistics forward (TRAIN without
  // batch_norm_accumulate_statistics) differentiates through constant statistics
  HIPCALL(c, launch_bn_bwd_finalize(L.bwd_part, L.rb, a.M, L.co, L.st,
                                    tb ? c->grads + L.g_off : nullptr,
                                    tb ? c->grads + L.b_off : nullptr, S.s, c->bn_infer));
  if (c->sync_fn && !c->bn_infer) {
    // [mean(dyhat) | mean(dyhat * xhat)] (contiguous in the layer's state) averaged over the
    // replicas: dx is the gradient through the global statistics; dgamma / dbeta stay this
    // replica's sums (the gradient all-reduce averages them)
    if (int r = sync_exchange(c, L.st.sdy, 2L * L.co, S.s)) return r;
    HIPCALL(c, launch_scale2(L.st.sdy, 2L * L.co, 1.f / c->sync_world, 0, 1.f, S.s));
  }
  if (reduce_only) return 0;
  const double gb_apply = gb_in + me * esz * (dyhat_out ? 2 : 1);
  if (int r = prof_begin(c, S.s, 5, li, gb_apply, &slot)) return r;
  HIPCALL(c, launch_bn_bwd_apply(S.dt, dz_f32, a, S.s));
  return prof_end(c, S.s, slot);
}

// BN backward of two layers gated by the same dz / ReLU bits (a projection unit's conv3 and
// shortcut BN): one dual reduce and one dual apply read dz and the bits once for both; each
// layer keeps its own finalize. Batch norm, 16-bit or fp32 dz of the storage type, no
// cross-replica exchange (that path runs the two layers through bn_backward)
// second_only: dz arrived pre-masked and the first layer's apply is folded (lbf.h): after the
// dual reduce and both finalizes only the second layer's apply runs (ungated)
int bn_backward_dual(Step& S, int li, int li2, const Act& dz, const Act& z, bool second_only = false) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  ConvL& L2 = c->convs[li2];
  BnBwdArgs a{};
  a.dz = dz.p; a.lddz = dz.ld; a.mask = z.mask;
  a.y = L.y.p; a.ldy = L.y.ld; a.M = L.y.M(); a.C = L.co;
  a.mean = L.st.mean; a.invstd = L.st.invstd; a.scale = L.st.scale;
  a.sdy = L.st.sdy; a.sdyx = L.st.sdyx;
  a.dy = L.dy.p; a.lddy = L.dy.ld;
  a.part = L.bwd_part; a.rb = L.rb;
  a.y2 = L2.y.p; a.ldy2 = L2.y.ld;
  a.mean2 = L2.st.mean; a.invstd2 = L2.st.invstd; a.scale2 = L2.st.scale;
  a.sdy2 = L2.st.sdy; a.sdyx2 = L2.st.sdyx;
  a.dy2 = L2.dy.p; a.lddy2 = L2.dy.ld;
  a.part2 = L2.bwd_part;
  const double esz = seg_half(S.dt) ? 2.0 : 4.0;
  const double me = a.M * (double)a.C * 1e-9;
  const double gb_in = me * (esz + 0.125 + 2 * esz);   // dz + bits + both y
  int slot;
  if (int r = prof_begin(c, S.s, 4, li, gb_in, &slot)) return r;
  HIPCALL(c, launch_bn_bwd_reduce_dual(S.dt, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  const bool tb = c->cfg.train_bn != 0;
  HIPCALL(c, launch_bn_bwd_finalize(L.bwd_part, L.rb, a.M, L.co, L.st, tb ? c->grads + L.g_off : nullptr,
                                    tb ? c->grads + L.b_off : nullptr, S.s, c->bn_infer));
  HIPCALL(c, launch_bn_bwd_finalize(L2.bwd_part, L2.rb, a.M, L2.co, L2.st,
                                    tb ? c->grads + L2.g_off : nullptr,
                                    tb ? c->grads + L2.b_off : nullptr, S.s, c->bn_infer));
  if (second_only) {
    BnBwdArgs b{};
    b.dz = dz.p; b.lddz = dz.ld;
    b.y = L2.y.p; b.ldy = L2.y.ld; b.M = a.M; b.C = L2.co;
    b.mean = L2.st.mean; b.invstd = L2.st.invstd; b.scale = L2.st.scale;
    b.sdy = L2.st.sdy; b.sdyx = L2.st.sdyx;
    b.dy = L2.dy.p; b.lddy = L2.dy.ld;
    if (int r = prof_begin(c, S.s, 5, li2, me * 3 * esz, &slot)) return r;
    HIPCALL(c, launch_bn_bwd_apply(S.dt, 0, b, S.s));
    return prof_end(c, S.s, slot);
  }
  if (int r = prof_begin(c, S.s, 5, li, gb_in + me * 2 * esz, &slot)) return r;
  HIPCALL(c, launch_bn_bwd_apply_dual(S.dt, a, S.s));
  return prof_end(c, S.s, slot);
}

// group norm backward (gn.h): per image the batch-norm reduce (S1, S2 per channel) into
// its slice of the partials, one finalize for the layer (dgamma / dbeta, per-image group
// means), per image the batch-norm apply with scale = invstd and the gradient times gamma
int gn_backward(Step& S, int li, const Act& dz0, int dz_f32, const Act* z0, const Act* dyhat0,
                const float* dzscale) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  const size_t zsz = dz_f32 ? 4 : c->esz;
  Act dzl = dz0;
  if (dzscale) {   // the logits: the loss normalisation first (gamma mixes into it below)
    HIPCALL(c, launch_gn_chscale((const float*)dz0.p, c->gn_gscaled, dz0.M(), dz0.ld, L.co, dzscale, S.s));
    dzl.p = c->gn_gscaled;
  }
  const float* gamma = c->params + L.g_off;
  const bool tb = c->cfg.train_bn != 0;
  for (int pass = 0; pass < 2; ++pass) {
    if (pass == 1)
      HIPCALL(c, launch_gn_bwd_final(L.bwd_part, dz0.N, L.rb, (long)L.Ho * L.Wo, L.co, L.groups, gamma,
                                     L.st_dev, tb ? c->grads + L.g_off : nullptr,
                                     tb ? c->grads + L.b_off : nullptr, S.s));
    for (int n = 0; n < dz0.N; ++n) {
      const Act dz = image_rows(dzl, n, zsz);
      const Act Y = image_rows(L.y, n, c->esz);
      const Act DY = image_rows(L.dy, n, c->esz);
      const BnState& st = L.st_img[n];
      BnBwdArgs a{};
      a.dz = dz.p; a.lddz = dz.ld;
      if (z0) {
        const Act z = image_rows(*z0, n, zsz);
        a.z = z.p; a.ldz = z.ld;
        if (z.mask && !dz_f32 && z.C == L.co) { a.mask = z.mask; a.z = nullptr; }
      }
      a.y = Y.p; a.ldy = Y.ld; a.M = Y.M(); a.C = L.co;
      a.mean = st.mean; a.invstd = st.invstd; a.sdy = st.sdy; a.sdyx = st.sdyx;
      a.dy = DY.p; a.lddy = DY.ld;
      a.part = L.bwd_part + (size_t)n * L.rb * L.co * 2; a.rb = L.rb;
      if (pass == 0) {
        HIPCALL(c, launch_bn_bwd_reduce(S.dt, dz_f32, a, S.s));
      } else {
        if (dyhat0) {
          const Act dh = image_rows(*dyhat0, n, c->esz);
          a.dyhat = dh.p; a.lddyhat = dh.ld;
        }
        a.scale = st.invstd;   // dx = invstd (gamma dyhat - sdy - xhat sdyx)
        a.dzscale = gamma;
        HIPCALL(c, launch_bn_bwd_apply(S.dt, dz_f32, a, S.s));
      }
    }
  }
  return 0;
}

// dx = dgrad(dy) [+ r1] [+ r2]
ConvArgs dgrad_args(seg_ctx* c, int li, const Act& dx, const Act* r1, const Act* r2);

// dx = dgrad(dy) [+ r1] [+ r2]; omask: ReLU bits to store dx masked by (premask)
int conv_dgrad(Step& S, int li, const Act& dx, const Act* r1 = nullptr, const Act* r2 = nullptr,
               const uint8_t* omask = nullptr) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  ConvArgs a = dgrad_args(c, li, dx, r1, r2);
  if (omask) { a.omask = omask; a.ldm = a.Co / 8; }
  long M = (long)L.N * L.H * L.W;
  int slot;
  // dy + w + dx (+ each residual read once)
  const double nres = (r1 ? 1.0 : 0.0) + (r2 ? 1.0 : 0.0);
  const double gbx = ((double)L.N * L.Ho * L.Wo * L.co + (double)L.co * L.k * L.k * L.ci +
                      (double)M * L.ci * (1.0 + nres)) * c->esz * 1e-9;
  if (int r = prof_begin(c, S.s, 1, li, 2.0 * M * L.ci * L.k * L.k * L.co * 1e-9 / L.stride / L.stride,
                         &slot, gbx)) return r;
  HIPCALL(c, launch_conv_nt(S.dt, 0, a, S.s));
  return prof_end(c, S.s, slot);
}

// dx = dgrad(li) + dgrad(li2) in one K-concatenated ping-pong launch: a projection unit's conv1
// and shortcut (both 1 x 1, stride 1, the unit input's geometry). Returns 1 when the shapes do
// not fit that path (the caller then runs the two data gradients with the residual add).
// omask (in / out): ReLU bits to store dx masked by (premask_bits), reset to nullptr when the
// launch cannot take them
int conv_dgrad_dual(Step& S, int li, int li2, const Act& dx, const uint8_t** omask = nullptr) {
  seg_ctx* c = S.c;
  const ConvL& L = c->convs[li];
  const ConvL& L2 = c->convs[li2];
  if (!seg_half(S.dt) || L.k != 1 || L2.k != 1 || L.stride != 1 || L2.stride != 1 ||
      L.ci != L2.ci || L.Ho != L2.Ho || L.Wo != L2.Wo || L.H != L.Ho || L.W != L.Wo ||
      !L.wt_lp || !L2.wt_lp)
    return 1;
  ConvArgs a = dgrad_args(c, li, dx, nullptr, nullptr);
  a.x2 = L2.dy.p; a.ldx2 = L2.dy.ld; a.C2 = L2.co;
  a.w2 = L2.wt_lp; a.ldw2 = L2.co;
  if (a.st != 1 || a.sf != 1 || a.pad_h || a.pad_w || !conv_nt_pp_ok(a)) return 1;
  if (omask && *omask) {   // stored masked by the consumer's ReLU bits where that launch exists
    a.omask = *omask; a.ldm = a.Co / 8;
    if (!conv_nt_omask_ok(S.dt, a)) { a.omask = nullptr; *omask = nullptr; }
  }
  const long M = (long)L.N * L.H * L.W;
  const double gbx = ((double)M * (L.co + L2.co) + (double)(L.co + L2.co) * L.ci + (double)M * L.ci) *
                     c->esz * 1e-9;
  int slot;
  if (int r = prof_begin(c, S.s, 1, li, 2.0 * M * L.ci * (L.co + L2.co) * 1e-9, &slot, gbx)) return r;
  HIPCALL(c, launch_conv_nt_pp(S.dt, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  return 0;
}

ConvArgs dgrad_args(seg_ctx* c, int li, const Act& dx, const Act* r1, const Act* r2) {
  ConvL& L = c->convs[li];
  ConvArgs a{};
  a.x = L.dy.p; a.N = L.N; a.H = L.Ho; a.W = L.Wo; a.C = L.co; a.ldx = L.dy.ld;
  a.w = L.wt_lp; a.ldw = L.k * L.k * L.co;
  a.y = dx.p; a.Ho = L.H; a.Wo = L.W; a.Co = L.ci; a.ldy = dx.ld;
  if (r1) { a.r = r1->p; a.ldr = r1->ld; }
  if (r2) { a.r2 = r2->p; a.ldr2 = r2->ld; }
  a.KH = a.KW = L.k;
  const int keff = L.k + (L.k - 1) * (L.rate - 1);
  a.sf = 1; a.st = L.stride;
  a.pad_h = (keff - 1) - L.pad_h; a.pad_w = (keff - 1) - L.pad_w;
  a.dil = L.rate; a.stats = nullptr;
  return a;
}

// record (on the weight-gradient stream ws) the events of every conv-weight bucket whose
// gradients are all written, in order; `final` flushes the remaining weight buckets
int bucket_progress(seg_ctx* c, hipStream_t ws, bool final) {
  const int nw = (int)c->bk_convs.size();
  while (c->bk_next < nw) {
    const int b = c->bk_next;
    bool ok = true;
    for (int li : c->bk_convs[b]) ok = ok && c->wg_done[li];
    if (!ok && !final) return 0;
    HIPCALL(c, hipEventRecord(c->bk_ev[b], ws));
    ++c->bk_next;
  }
  return 0;
}

int conv_wgrad_impl(Step& S, int li, const Act& x);
int conv_wgrad(Step& S, int li, const Act& x) {
  seg_ctx* c = S.c;
  Step W = S;
  if (c->side_active) {   // the layer's dy (and the wgrad input x) are ready on the compute stream
    if (li == c->stem && c->defer_stem) {   // every other weight gradient is queued before it
      HIPCALL(c, hipEventRecord(c->ev_prestem, c->side));
      c->prestem_rec = true;
    }
    HIPCALL(c, hipEventRecord(c->ev_dy[li], S.s));
    HIPCALL(c, hipStreamWaitEvent(c->side, c->ev_dy[li], 0));
    W.s = c->side;
  }
  if (int r = conv_wgrad_impl(W, li, x)) return r;
  c->wg_done[li] = 1;
  return bucket_progress(c, W.s, false);
}

int conv_wgrad_impl(Step& S, int li, const Act& x) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[li];
  WgradArgs a{};
  a.dy = L.dy.p; a.lddy = L.dy.ld;
  a.x = x.p; a.N = x.N; a.H = x.H; a.W = x.W; a.C = x.C; a.ldx = x.ld;
  a.Ho = L.Ho; a.Wo = L.Wo; a.Co = L.co_pad;
  a.KH = a.KW = L.k; a.sf = L.stride; a.pad_h = L.pad_h; a.pad_w = L.pad_w; a.dil = L.rate;
  const bool s2d = li == c->stem && c->stem_s2d;
  if (s2d) { a.KH = a.KW = 4; a.sf = 1; a.pad_h = a.pad_w = 0; a.dil = 1; }
  // the stem's weight gradient is the last work of the step (its dgrad is skipped): nothing
  // runs beside it, so it takes the whole chip (tools/timeline.py: the compute stream idled
  // ~0.75 ms waiting for it)
  a.splits = wgrad_splits(a, S.dt, c->side_active && li != c->stem);
  const long per = (long)a.Co * a.KH * a.KW * a.C;
  // the shared slab was sized at creation for these shapes; never exceed it
  a.splits = (int)std::max<long>(1, std::min<long>(a.splits, (long)c->slab_floats / per));
  a.out = c->slab;
  long P = (long)L.N * L.Ho * L.Wo;
  int slot;
  // dy + x (16-bit) + the fp32 weight gradient; split-K slab traffic is overhead, not algorithmic
  const double gbx = (((double)P * L.co + (double)L.N * L.H * L.W * L.ci) * c->esz +
                      (double)L.co * L.k * L.k * L.ci * 4.0) * 1e-9;
  if (int r = prof_begin(c, S.s, 2, li, 2.0 * P * L.co * L.k * L.k * L.ci * 1e-9, &slot, gbx)) return r;
  HIPCALL(c, launch_conv_wgrad(S.dt, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  if (s2d) {
    HIPCALL(c, launch_splitk_reduce_s2d(c->slab, a.splits, (long)L.co_pad * 256, L.co,
                                        c->grads + L.w_off, S.s));
    return 0;
  }
  const long n = (long)L.co * L.k * L.k * L.ci;
  // slab rows are co_pad wide only in the Co dimension: rows 0..co-1 are the real ones
  // split z of the slab starts at z*co_pad*ncol; rows >= co are padding and never reduced
  HIPCALL(c, launch_splitk_reduce(c->slab, a.splits, (long)L.co_pad * L.k * L.k * L.ci, n,
                                  c->grads + L.w_off, 0, S.s));
  return 0;
}

}  // namespace

namespace {

// ------------------------------------------------------------------------------------------
// pyramid tables
// ------------------------------------------------------------------------------------------
int upload_grid(seg_ctx* c, GridSpec& g, const std::vector<float>& rt, const std::vector<float>& ct) {
  float *drt, *dct;
  if (int r = dalloc(c, &drt, rt.size())) return r;
  if (int r = dalloc(c, &dct, ct.size())) return r;
  HIPCALL(c, hipMemcpy(drt, rt.data(), rt.size() * 4, hipMemcpyHostToDevice));
  HIPCALL(c, hipMemcpy(dct, ct.data(), ct.size() * 4, hipMemcpyHostToDevice));
  g.rowtab = drt;
  g.coltab = dct;
  return 0;
}

// VALID avg pools with (kh, kw) windows over an (H, W) map (remainders dropped)
int make_pool_grids(seg_ctx* c, GridSpec& g, int H, int W, const std::vector<std::pair<int, int>>& win) {
  memset(&g, 0, sizeof(g));
  g.n = (int)win.size();
  for (int i = 0; i < g.n; ++i) {
    g.kh[i] = win[i].first; g.kw[i] = win[i].second;
    g.kr[i] = (H - g.kh[i]) / g.kh[i] + 1;
    g.kc[i] = (W - g.kw[i]) / g.kw[i] + 1;
    g.ccell_off[i] = g.total_ccells; g.total_ccells += g.kc[i];
    g.rcell_off[i] = g.total_rcells; g.total_rcells += g.kr[i];
    g.scale[i] = 1.f / (float)(g.kh[i] * g.kw[i]);
  }
  if (g.total_ccells > SEG_MAX_CELLS) return set_err(&c->err, -EINVAL, "too many pyramid cells");
  std::vector<float> rt((size_t)g.total_ccells * W, 0.f), ct((size_t)g.total_rcells * H, 0.f);
  for (int i = 0; i < g.n; ++i) {
    for (int j = 0; j < g.kc[i]; ++j)
      for (int w = j * g.kw[i]; w < (j + 1) * g.kw[i]; ++w) rt[(size_t)(g.ccell_off[i] + j) * W + w] = 1.f;
    for (int r = 0; r < g.kr[i]; ++r)
      for (int h = r * g.kh[i]; h < (r + 1) * g.kh[i]; ++h) ct[(size_t)(g.rcell_off[i] + r) * H + h] = 1.f;
  }
  return upload_grid(c, g, rt, ct);
}

// transpose of an align-corners resize (kr, kc) -> (H, W)
int make_resize_grid(seg_ctx* c, GridSpec& g, int kr, int kc, int H, int W) {
  memset(&g, 0, sizeof(g));
  g.n = 1; g.kr[0] = kr; g.kc[0] = kc; g.total_ccells = kc; g.total_rcells = kr; g.scale[0] = 1.f;
  std::vector<float> rt((size_t)kc * W, 0.f), ct((size_t)kr * H, 0.f);
  for (int w = 0; w < W; ++w) {
    int lo, hi; float l;
    tf_lerp_host(w, kc, W, lo, hi, l);
    rt[(size_t)lo * W + w] += 1.f - l;
    rt[(size_t)hi * W + w] += l;
  }
  for (int h = 0; h < H; ++h) {
    int lo, hi; float l;
    tf_lerp_host(h, kr, H, lo, hi, l);
    ct[(size_t)lo * H + h] += 1.f - l;
    ct[(size_t)hi * H + h] += l;
  }
  return upload_grid(c, g, rt, ct);
}

// ------------------------------------------------------------------------------------------
// graph construction + allocation
// ------------------------------------------------------------------------------------------
// linear BN-backward fold (lbf.h): the unit shapes it applies to -- a 16-bit batch-norm
// bottleneck (identity, subsample, or projection with its output gradient pre-masked) whose conv3 is an expansion 1 x 1 (co >= 2 ci, ci a multiple of 64; its data
// gradient is a ping-pong launch for ci > 128, a v2 launch otherwise: C2 = ci, Co = ci) and whose
// conv2 output gate is kept as bits
int lbf_hsplits(const ConvL& L3) { return std::max(1, L3.co / 128); }   // H: 128 channels per split

bool lbf_shape_ok(const seg_ctx* c, const Unit& u) {
  if (!seg_half(c->dt) || c->gn || u.c3 < 0 || u.c2 < 0) return false;
  const ConvL& L3 = c->convs[u.c3];
  const ConvL& L2 = c->convs[u.c2];
  return L3.k == 1 && L3.stride == 1 && L3.rate == 1 && L3.co >= 2 * L3.ci && L3.ci >= 64 &&
         L3.co <= 2048 && L3.ci % 64 == 0 && L3.co % 128 == 0 && L2.co == L3.ci && L2.relu;
}

int alloc_unit(seg_ctx* c, Unit& u, const Act& in) {
  u.in = in;
  if (u.sc >= 0)
    if (int r = alloc_conv(c, c->convs[u.sc], in.N, in.H, in.W)) return r;
  ConvL& c1 = c->convs[u.c1];
  if (int r = alloc_conv(c, c1, in.N, in.H, in.W)) return r;
  if (int r = alloc_relu_act(c, u.z1, in.N, c1.Ho, c1.Wo, c1.co)) return r;
  if (int r = alloc_act(c, u.dz1, in.N, c1.Ho, c1.Wo, c1.co)) return r;
  ConvL& c2 = c->convs[u.c2];
  if (int r = alloc_conv(c, c2, in.N, c1.Ho, c1.Wo)) return r;
  if (int r = alloc_relu_act(c, u.z2, in.N, c2.Ho, c2.Wo, c2.co)) return r;
  if (int r = alloc_act(c, u.dz2, in.N, c2.Ho, c2.Wo, c2.co)) return r;
  ConvL& c3 = c->convs[u.c3];
  if (int r = alloc_conv(c, c3, in.N, c2.Ho, c2.Wo)) return r;
  if (int r = alloc_relu_act(c, u.out, in.N, c3.Ho, c3.Wo, c3.co)) return r;
  if (int r = alloc_act(c, u.dout, in.N, c3.Ho, c3.Wo, c3.co)) return r;
  if (u.kind != SC_CONV)
    if (int r = alloc_act(c, u.dpre, in.N, c3.Ho, c3.Wo, c3.co)) return r;
  return 0;
}

int build(seg_ctx* c) {
  const seg_cfg& g = c->cfg;
  const int N = g.nb_pp + g.nb_pb + g.nb_pi;
  const int fd = g.feature_dims;
  if (N <= 0 || g.height < 32 || g.width < 32) return set_err(&c->err, -EINVAL, "bad batch/size");
  if (g.depth != 50 && g.depth != 101) return set_err(&c->err, -EINVAL, "depth must be 50|101");
  if (g.output_stride != 8) return set_err(&c->err, -EINVAL, "output_stride must be 8");
  if (fd % 8) return set_err(&c->err, -EINVAL, "feature_dims must be a multiple of 8");
  const std::string rn = "feature_extractor/base/resnet_v1_" + std::to_string(g.depth);

  // ---- layers in TF variable-creation order ----
  c->stem = add_conv(c, rn + "/conv1", 3, 64, 7, 2, 1, true, true);
  for (auto& us : resnet_units(g.depth, g.output_stride)) {
    Unit u;
    add_bottleneck(c, u, rn + "/" + us.scope, us.din, us.d, us.dbn, us.s, us.r);
    c->units.push_back(u);
  }
  c->dfd = add_conv(c, "feature_extractor/extension/decrease_fdims", 2048, fd, 1, 1, 1, false, true);
  if (g.fov_k < 0 || g.fov_rate < 0 || (g.fov_k > 0) != (g.fov_rate > 0))
    return set_err(&c->err, -EINVAL, "fov_k and fov_rate must both be set (hierarchical.py:272-274)");
  if (g.fov_k > 0)   // slim.conv2d(fe, fd, fov_k, rate=fov_rate): SAME, BN, ReLU
    c->fov = add_conv(c, "feature_extractor/extension/increase_fov", fd, fd, g.fov_k, 1, g.fov_rate,
                      false, true);
  if (g.pyramid == SEG_PYRAMID_PSP) {
    const char* nm[4] = {"Conv", "Conv_1", "Conv_2", "Conv_3"};
    for (int i = 0; i < 4; ++i)
      c->pyr_conv.push_back(add_conv(c, std::string("feature_extractor/pyramid_module/") + nm[i], fd, fd, 1, 1, 1, false, true));
    c->pyr_final = add_conv(c, "feature_extractor/pyramid_module/Conv_4", 5 * fd, fd, 1, 1, 1, false, true);
  } else if (g.pyramid == SEG_PYRAMID_ASPP) {
    // the commented _create_aspp_module (hierarchical.py:209-226), in the PSP call site's scope
    const std::string sc = "feature_extractor/pyramid_module/";
    c->pyr_conv.push_back(add_conv(c, sc + "Conv", fd, fd, 1, 1, 1, false, true));     // image pool
    c->pyr_conv.push_back(add_conv(c, sc + "Conv_1", fd, fd, 1, 1, 1, false, true));   // 1x1
    const int rates[3] = {6, 12, 18};
    for (int i = 0; i < 3; ++i)
      c->pyr_conv.push_back(add_conv(c, sc + "Conv_" + std::to_string(i + 2), fd, fd, 3, 1, rates[i], false, true));
    c->pyr_final = add_conv(c, sc + "Conv_5", 5 * fd, fd, 1, 1, 1, false, true);
  }
  const char* hn[3] = {"l1", "l2_vehicle", "l2_human"};
  for (int h = 0; h < 3; ++h)
    add_bottleneck(c, c->heads[h], std::string("adaptation_module/") + hn[h] + "_features", fd, fd, fd, 1, 1);
  fill_tables(c->tables, g.dataset);
  c->nc[0] = c->tables.c1; c->nc[1] = c->tables.c2; c->nc[2] = c->tables.c3;
  for (int h = 0; h < 3; ++h)
    c->logit_conv[h] = add_conv(c, std::string("softmax_classifier/") + hn[h] + "_logits", fd, c->nc[h], 1, 1, 1, false, false);
  c->convs[c->stem].need_dgrad = false;

  if (g.upsampling != SEG_UPSAMPLING_BILINEAR && g.upsampling != SEG_UPSAMPLING_HYBRID)
    return set_err(&c->err, -EINVAL, "upsampling must be bilinear or hybrid");
  c->hybrid = g.upsampling == SEG_UPSAMPLING_HYBRID;
  if (g.norm != SEG_NORM_BATCH && g.norm != SEG_NORM_GROUP)
    return set_err(&c->err, -EINVAL, "norm must be batch or group");
  c->gn = g.norm == SEG_NORM_GROUP;
  if (c->gn) {   // module_arg_scope groups (32), the softmax_classifier scope's groups=1
    const int G = g.groups > 0 ? g.groups : 32;
    for (auto& L : c->convs) {
      const bool logit = &L == &c->convs[c->logit_conv[0]] || &L == &c->convs[c->logit_conv[1]] ||
                         &L == &c->convs[c->logit_conv[2]];
      L.groups = logit ? 1 : G;
      if (L.co % L.groups || L.co / L.groups > 256)
        return set_err(&c->err, -EINVAL, "group norm: %s has %d channels for %d groups", L.name.c_str(),
                       L.co, L.groups);
    }
  }

  // ---- flat parameter layout ----
  // [conv weights | hybrid deconv weights] (weight decay) [BN gamma/beta | deconv biases]
  long off = 0;
  for (auto& L : c->convs) { L.w_off = off; off += (long)L.co * L.k * L.k * L.ci; }
  if (c->hybrid)
    for (int h = 0; h < 3; ++h) { c->dc_w_off[h] = off; off += 9L * c->nc[h] * c->nc[h]; }
  c->n_decay = off;
  for (auto& L : c->convs) { L.g_off = off; off += L.co; L.b_off = off; off += L.co; }
  c->dc_b_lo = off;
  if (c->hybrid)
    for (int h = 0; h < 3; ++h) { c->dc_b_off[h] = off; off += c->nc[h]; }
  c->n_train = off;
  long moff = 0;
  for (auto& L : c->convs) { L.mv_off = moff; moff += L.co; }
  c->n_moving = 2 * moff;
  c->n_stats = c->n_moving;
  {
    // runtime knob (deliberate): the all-reduce bucket size, a property of the interconnect
    // rather than of the kernels (seg_grad_buckets); results are identical for any value
    const char* e = getenv("SEG_BUCKET_MB");
    const long cap = (e ? std::max(1L, atol(e)) : 32L) * (1L << 20) / 4;   // floats per bucket
    long hi = c->n_decay;
    std::vector<int> cur;
    for (int li = (int)c->convs.size() - 1; li >= 0; --li) {
      cur.push_back(li);
      const long lo = c->convs[li].w_off;
      if (hi - lo >= cap || li == 0) {
        c->bk_lo.push_back(lo); c->bk_hi.push_back(hi); c->bk_convs.push_back(cur);
        cur.clear();
        hi = lo;
      }
    }
    c->bk_lo.push_back(c->n_decay); c->bk_hi.push_back(c->n_train + c->n_stats);
    c->bk_ev.resize(c->bk_lo.size());
    for (auto& ev : c->bk_ev) HIPCALL(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->wg_done.assign(c->convs.size(), 0);
    // runtime knob (deliberate): SEG_SIDE_STREAM=0 runs the backward on one stream, so a
    // rocprofv3 trace sees kernel-alone durations (tools/session.sh stats, pmc_traffic.sh);
    // results are bitwise identical either way
    const char* se = getenv("SEG_SIDE_STREAM");
    c->side_on = !(se && se[0] == '0');
    if (c->side_on) {
      HIPCALL(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
      c->ev_dy.resize(c->convs.size());
      for (auto& ev : c->ev_dy) HIPCALL(c, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
      HIPCALL(c, hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming));
      HIPCALL(c, hipEventCreateWithFlags(&c->ev_prestem, hipEventDisableTiming));
    }
  }
  for (auto& L : c->convs) {
    c->pinfo.push_back({L.name + "/weights", L.w_off, (long)L.co * L.k * L.k * L.ci, SEG_PARAM_WEIGHTS, {L.co, L.k, L.k, L.ci}});
    if (c->gn) {   // tf.contrib.layers.group_norm variables: no moving statistics
      c->pinfo.push_back({L.name + "/GroupNorm/beta", L.b_off, L.co, SEG_PARAM_BETA, {L.co, 1, 1, 1}});
      c->pinfo.push_back({L.name + "/GroupNorm/gamma", L.g_off, L.co, SEG_PARAM_GAMMA, {L.co, 1, 1, 1}});
      continue;
    }
    c->pinfo.push_back({L.name + "/BatchNorm/beta", L.b_off, L.co, SEG_PARAM_BETA, {L.co, 1, 1, 1}});
    c->pinfo.push_back({L.name + "/BatchNorm/gamma", L.g_off, L.co, SEG_PARAM_GAMMA, {L.co, 1, 1, 1}});
    c->pinfo.push_back({L.name + "/BatchNorm/moving_mean", L.mv_off, L.co, SEG_PARAM_MOVING_MEAN, {L.co, 1, 1, 1}});
    c->pinfo.push_back({L.name + "/BatchNorm/moving_variance", moff + L.mv_off, L.co, SEG_PARAM_MOVING_VAR, {L.co, 1, 1, 1}});
  }
  if (c->hybrid) {
    // slim.conv2d_transpose default scopes inside softmax_classifier/upsampling, created after
    // the three logits convs (hierarchical.py:84-86,168-180)
    const char* sfx[3] = {"", "_1", "_2"};
    for (int h = 0; h < 3; ++h) {
      const std::string nm = std::string("softmax_classifier/upsampling/Conv2d_transpose") + sfx[h];
      const int C = c->nc[h];
      c->pinfo.push_back({nm + "/weights", c->dc_w_off[h], 9L * C * C, SEG_PARAM_WEIGHTS, {C, 3, 3, C}});
      c->pinfo.push_back({nm + "/biases", c->dc_b_off[h], C, SEG_PARAM_BIASES, {C, 1, 1, 1}});
    }
  }

  // ---- activations ----
  const int H = g.height, W = g.width;
  // the stem input is context-owned in every dtype (the 16-bit space-to-depth image, or an fp32
  // copy): the stem's weight gradient reads it in seg_backward, after the caller's buffer may
  // be gone
  c->stem_s2d = seg_half(c->dt);
  ConvL& st = c->convs[c->stem];
  if (int r = alloc_conv(c, st, N, H, W)) return r;
  if (c->stem_s2d) {
    if (st.k != 7 || st.stride != 2 || st.ci != 3)
      return set_err(&c->err, -EINVAL, "space-to-depth stem expects a 7x7/2 conv of 3 channels");
    if (int r = alloc_act(c, c->img, N, st.Ho + 3, st.Wo + 3, 16)) return r;
  } else {
    if (int r = alloc_act(c, c->img, N, H, W, 3)) return r;
  }
  if (int r = alloc_relu_act(c, c->z0, N, st.Ho, st.Wo, 64)) return r;
  if (int r = alloc_act(c, c->dz0, N, st.Ho, st.Wo, 64)) return r;
  {  // max_pool2d 3x3/2 SAME
    int Ho = (st.Ho + 1) / 2, Wo = (st.Wo + 1) / 2;
    int th = std::max((Ho - 1) * 2 + 3 - st.Ho, 0), tw = std::max((Wo - 1) * 2 + 3 - st.Wo, 0);
    c->pool_ph = th / 2; c->pool_pw = tw / 2;
    if (int r = alloc_act(c, c->p0, N, Ho, Wo, 64)) return r;
    if (int r = dalloc(c, &c->pool_arg, (size_t)N * Ho * Wo * 64)) return r;
    if (int r = alloc_act(c, c->dp0, N, Ho, Wo, 64)) return r;
  }
  Act x = c->p0;
  for (auto& u : c->units) {
    if (int r = alloc_unit(c, u, x)) return r;
    x = u.out;
  }
  ConvL& dfd = c->convs[c->dfd];
  if (int r = alloc_conv(c, dfd, N, x.H, x.W)) return r;
  const int Hf = dfd.Ho, Wf = dfd.Wo;
  if (int r = alloc_act(c, c->dz_dfd, N, Hf, Wf, fd)) return r;
  if (c->fov >= 0) {
    if (int r = alloc_relu_act(c, c->z_pre, N, Hf, Wf, fd)) return r;
    if (int r = alloc_act(c, c->dz_pre, N, Hf, Wf, fd)) return r;
    if (int r = alloc_conv(c, c->convs[c->fov], N, Hf, Wf)) return r;
  }
  if (g.pyramid == SEG_PYRAMID_PSP) {
    if (int r = alloc_act(c, c->concat, N, Hf, Wf, 5 * fd)) return r;
    if (int r = alloc_act(c, c->dconcat, N, Hf, Wf, 5 * fd)) return r;
    c->z_dfd = slice(c, c->concat, 0, fd);
    // _create_psp_module: spatial dims = (hf, wf) // stride; kernel = stride = dims // k
    const int sh = H / g.output_stride, sw = W / g.output_stride;
    std::vector<std::pair<int, int>> win;
    for (int k : {1, 2, 3, 6}) win.push_back({sh / k, sw / k});
    if (int r = make_pool_grids(c, c->pool_grids, Hf, Wf, win)) return r;
    size_t gp = (size_t)N * Hf * c->pool_grids.total_ccells * fd;
    for (int b = 0; b < 4; ++b) {
      const int kr = c->pool_grids.kr[b], kc = c->pool_grids.kc[b];
      Act pa, dpa, za, dza;
      if (int r = alloc_act(c, pa, N, kr, kc, fd)) return r;
      if (int r = alloc_act(c, dpa, N, kr, kc, fd)) return r;
      if (int r = alloc_act(c, za, N, kr, kc, fd)) return r;
      if (int r = alloc_act(c, dza, N, kr, kc, fd)) return r;
      c->pooled.push_back(pa); c->dpooled.push_back(dpa); c->zb.push_back(za); c->dzb.push_back(dza);
      if (int r = alloc_conv(c, c->convs[c->pyr_conv[b]], N, kr, kc)) return r;
      GridSpec ug;
      if (int r = make_resize_grid(c, ug, kr, kc, Hf, Wf)) return r;
      c->up_grids.push_back(ug);
      gp = std::max(gp, (size_t)N * Hf * kc * fd);
    }
    if (int r = dalloc(c, &c->grid_part, gp)) return r;
    if (int r = alloc_conv(c, c->convs[c->pyr_final], N, Hf, Wf)) return r;
    if (int r = alloc_relu_act(c, c->feat, N, Hf, Wf, fd)) return r;
    if (int r = alloc_act(c, c->dfeat, N, Hf, Wf, fd)) return r;
  } else if (g.pyramid == SEG_PYRAMID_ASPP) {
    if (int r = alloc_relu_act(c, c->z_dfd, N, Hf, Wf, fd)) return r;
    if (int r = alloc_act(c, c->concat, N, Hf, Wf, 5 * fd)) return r;
    if (int r = alloc_act(c, c->dconcat, N, Hf, Wf, 5 * fd)) return r;
    std::vector<std::pair<int, int>> win{{Hf, Wf}};   // global average pool
    if (int r = make_pool_grids(c, c->pool_grids, Hf, Wf, win)) return r;
    Act pa, dpa, za, dza;
    if (int r = alloc_act(c, pa, N, 1, 1, fd)) return r;
    if (int r = alloc_act(c, dpa, N, 1, 1, fd)) return r;
    if (int r = alloc_act(c, za, N, 1, 1, fd)) return r;
    if (int r = alloc_act(c, dza, N, 1, 1, fd)) return r;
    c->pooled.push_back(pa); c->dpooled.push_back(dpa); c->zb.push_back(za); c->dzb.push_back(dza);
    if (int r = alloc_conv(c, c->convs[c->pyr_conv[0]], N, 1, 1)) return r;
    GridSpec ug;
    if (int r = make_resize_grid(c, ug, 1, 1, Hf, Wf)) return r;
    c->up_grids.push_back(ug);
    if (int r = dalloc(c, &c->grid_part, (size_t)N * Hf * fd)) return r;
    for (int b = 1; b < 5; ++b)
      if (int r = alloc_conv(c, c->convs[c->pyr_conv[b]], N, Hf, Wf)) return r;
    if (int r = alloc_conv(c, c->convs[c->pyr_final], N, Hf, Wf)) return r;
    if (int r = alloc_relu_act(c, c->feat, N, Hf, Wf, fd)) return r;
    if (int r = alloc_act(c, c->dfeat, N, Hf, Wf, fd)) return r;
  } else {
    if (int r = alloc_relu_act(c, c->z_dfd, N, Hf, Wf, fd)) return r;
    c->feat = c->z_dfd;
    c->dfeat = c->dz_dfd;
  }
  for (int h = 0; h < 3; ++h) {
    if (int r = alloc_unit(c, c->heads[h], c->feat)) return r;
    if (int r = alloc_conv(c, c->convs[c->logit_conv[h]], N, Hf, Wf)) return r;
  }
  c->ldl = ((c->nc[0] + c->nc[1] + c->nc[2] + 3) / 4) * 4;
  if (int r = alloc_act(c, c->logits, N, Hf, Wf, c->nc[0] + c->nc[1] + c->nc[2], c->ldl, 4)) return r;
  if (int r = dalloc(c, &c->grad_un, (size_t)N * Hf * Wf * c->ldl)) return r;
  c->head_in = (const float*)c->logits.p;
  if (c->gn)
    if (int r = dalloc(c, &c->gn_gscaled, (size_t)N * Hf * Wf * c->ldl)) return r;
  if (c->hybrid) {
    if (int r = dalloc(c, &c->up_in, (size_t)N * Hf * Wf * c->ldl)) return r;
    if (int r = dalloc(c, &c->dc_dx, (size_t)N * Hf * Wf * c->ldl)) return r;
    const size_t np = (size_t)deconv_wgrad_blocks(N, Hf, Wf, c->nc[0] + c->nc[1] + c->nc[2]) * deconv_nw(c->nc);
    if (int r = dalloc(c, &c->dc_part, np)) return r;
    c->head_in = c->up_in;
  }
  c->loss_blocks = loss_head_blocks(N, Hf, Wf);
  if (int r = dalloc(c, &c->loss_part, (size_t)c->loss_blocks * 8)) return r;
  if (int r = dalloc(c, &c->loss_out, 16)) return r;
  if (int r = dalloc(c, &c->dzscale, c->ldl)) return r;
  if (int r = dalloc(c, &c->reg_part, sgdm_blocks(c->n_decay) + 2)) return r;   // + the split update's
  if (int r = dalloc(c, &c->reg_out, 4)) return r;

  // ---- compute weight copies and workspace ----
  if (seg_half(c->dt))
    if (int r = dalloc(c, (bf16_t**)&c->w_lp_flat, c->n_decay)) return r;
  size_t slab = 0;
  for (auto& L : c->convs) {
    if (L.need_dgrad) {
      char* p;
      if (int r = dalloc(c, &p, (size_t)L.co * L.k * L.k * L.ci * c->esz)) return r;
      L.wt_lp = p;
    }
    if (seg_half(c->dt)) L.w_lp = (uint16_t*)c->w_lp_flat + L.w_off;   // bf16 or fp16 bits
    const bool s2d = &L == &c->convs[c->stem] && c->stem_s2d;
    const WgradArgs a = wgrad_problem(L, s2d);
    const int sp = std::max(wgrad_splits(a, c->dt, false), wgrad_splits(a, c->dt, true));
    slab = std::max(slab, (size_t)sp * a.Co * a.KH * a.KW * a.C);
  }
  if (c->stem_s2d) {
    const ConvL& st = c->convs[c->stem];
    if (int r = dalloc(c, &c->stem_wpad, (size_t)st.co * 256)) return r;
  }
  c->slab_floats = slab;
  if (int r = dalloc(c, &c->slab, slab)) return r;
  if (int r = dalloc(c, &c->stat_scratch, std::max<size_t>(c->stat_scratch_floats, 16))) return r;
  {  // linear BN-backward fold: per-layer coefficients and the shared scratch (lbf.h)
    size_t wts = 0, hh = 0, hs = 0, ci_max = 0;
    for (auto& u : c->units) {
      if (!lbf_shape_ok(c, u)) continue;
      ConvL& L3 = c->convs[u.c3];
      if (int r = dalloc(c, &L3.lbf_coef, 3 * (size_t)L3.co)) return r;
      // per layer: conv2's BN reduce writes it on the compute stream while the side stream may
      // still be combining an earlier unit's gradient
      if (int r = dalloc(c, &L3.lbf_cs, (size_t)c->convs[u.c2].rb * L3.ci)) return r;
      wts = std::max(wts, (size_t)L3.co * L3.ci);
      hh = std::max(hh, (size_t)L3.ci * L3.ci);
      hs = std::max(hs, (size_t)lbf_hsplits(L3) * L3.ci * L3.ci);
      ci_max = std::max(ci_max, (size_t)L3.ci);
    }
    if (wts) {
      char* p;
      if (int r = dalloc(c, &p, wts * c->esz)) return r;
      c->lbf_wts = p;
      if (int r = dalloc(c, &p, wts * c->esz)) return r;
      c->lbf_xd = p;
      if (int r = dalloc(c, &p, hh * c->esz)) return r;
      c->lbf_h = p;
      if (int r = dalloc(c, &c->lbf_hslab, hs)) return r;
      if (int r = dalloc(c, &c->lbf_bias, ci_max)) return r;
      if (int r = dalloc(c, &c->lbf_bpart, (wts / 128) + ci_max)) return r;   // [co / 128][ci]
      if (int r = dalloc(c, &c->lbf_p1, wts + hh)) return r;   // [P1 (co x ci) | G (ci x ci)]
    }
  }
  return 0;
}

// ------------------------------------------------------------------------------------------
// step
// ------------------------------------------------------------------------------------------
int unit_forward(Step& S, Unit& u) {
  seg_ctx* c = S.c;
  if (u.sc >= 0)
    if (int r = conv_forward(S, u.sc, u.in)) return r;
  if (int r = conv_forward(S, u.c1, u.in)) return r;
  if (int r = bn_apply(S, u.c1, u.z1, 0)) return r;
  if (int r = conv_forward(S, u.c2, u.z1)) return r;
  if (int r = bn_apply(S, u.c2, u.z2, 0)) return r;
  if (int r = conv_forward(S, u.c3, u.z2)) return r;
  // out = relu(shortcut + bn3(conv3))
  if (u.kind == SC_CONV) return bn_apply(S, u.c3, u.out, 0, nullptr, 1, u.sc, 1);
  (void)c;
  return bn_apply(S, u.c3, u.out, 0, &u.in, u.kind == SC_SUBSAMPLE ? u.stride : 1, -1, 1);
}

// pred = the unit whose output is u's input (nullptr: none). When both are identity units,
// u's conv1 data gradient (+ the residual dpre) is stored already masked by pred's output ReLU
// bits: everything that reads pred's dout wants it masked (pred's c3 BN backward and, as
// pred's dpre, pred's own conv1 residual), so pred's c3 BN backward neither reads the bits nor
// writes dpre (one M x C store pass fewer per such unit)
bool premask_ok(seg_ctx* c, const Unit& u, const Unit* pred, bool accumulate) {
  if (!c->premask || !pred || accumulate || u.kind != SC_IDENTITY || pred->kind == SC_SUBSAMPLE || c->gn)
    return false;
  if (!pred->out.mask || pred->out.C != c->convs[u.c1].ci || c->convs[pred->c3].co != pred->out.C) return false;
  ConvArgs a = dgrad_args(c, u.c1, pred->dout, &u.dpre, nullptr);
  a.ldm = a.Co / 8;
  return conv_nt_omask_ok(c->dt, a);
}

// the ReLU bits of pred's output when the data gradient into it (of C channels) may be stored
// masked by them: pred an identity or subsample unit, so its c3 BN backward then reads dout
// ungated and writes no dpre (block boundaries: a projection unit's dual data gradient,
// decrease_fdims')
const uint8_t* premask_bits(seg_ctx* c, const Unit* pred, int C) {
  if (!c->premask || !pred || pred->kind == SC_CONV || c->gn || !pred->out.mask ||
      pred->out.C != C || c->convs[pred->c3].co != C)
    return nullptr;
  return pred->out.mask;
}

// ---- linear BN-backward fold of an identity unit's conv3 (lbf.h) ----
// in_masked: u.dout arrived pre-masked (a projection unit folds only then: its gated gradient
// is dout itself, and its dual BN reduce cannot store one)
bool lbf_ok(seg_ctx* c, const Unit& u, bool in_masked) {
  if (!c->lbf_on || !c->lbf_wts || !lbf_shape_ok(c, u)) return false;
  if (u.kind == SC_CONV) {
    const ConvL& L3 = c->convs[u.c3];
    const ConvL& Ls = c->convs[u.sc];
    if (!in_masked || c->sync_fn || Ls.co != L3.co || Ls.rb != L3.rb || Ls.y.M() != L3.y.M()) return false;
  }
  const ConvL& L3 = c->convs[u.c3];
  if (!L3.lbf_coef || !L3.wt_lp || !u.out.mask || u.out.C != L3.co || !u.z2.mask ||
      u.z2.C != L3.ci || u.dz2.C != L3.ci)
    return false;
  ConvArgs a{};
  a.x = u.dout.p; a.N = L3.N; a.H = L3.Ho; a.W = L3.Wo; a.C = L3.co; a.ldx = u.dout.ld;
  a.w = c->lbf_wts; a.ldw = L3.co;
  a.y = u.dz2.p; a.Ho = L3.H; a.Wo = L3.W; a.Co = L3.ci; a.ldy = u.dz2.ld;
  a.x2 = u.z2.p; a.ldx2 = u.z2.ld; a.C2 = L3.ci; a.w2 = c->lbf_h; a.ldw2 = L3.ci;
  a.KH = a.KW = 1; a.sf = 1; a.st = 1; a.dil = 1;
  if (u.kind != SC_CONV && u.dpre.ld != u.dout.ld) return false;
  return L3.ci > 128 ? conv_nt_pp_ok(a) : conv_nt_v2_ok(a) && conv_nt_v2_dual_ok(a);
}

// the weight gradient of a folded conv3 (on the weight-gradient stream when it is active):
// P1 = dyhat^T y2 and G = y2^T y2 by the weight-gradient kernel, the column sums of y2, then
// dW3 = A o P1 + B (x) colsum + D o (W3 G) into the gradient buffer
int lbf_wgrad(Step& S, Unit& u, const Act& dyhat) {
  seg_ctx* c = S.c;
  const int li = u.c3;
  ConvL& L = c->convs[li];
  Step W = S;
  if (c->side_active) {   // dyhat, y2 and this layer's coefficients are ready on the compute stream
    HIPCALL(c, hipEventRecord(c->ev_dy[li], S.s));
    HIPCALL(c, hipStreamWaitEvent(c->side, c->ev_dy[li], 0));
    W.s = c->side;
  }
  const Act& y2 = u.z2;
  const long P = (long)L.N * L.Ho * L.Wo;
  const long n1 = (long)(L.co + L.ci) * L.ci;
  int slot;
  // algorithmic work of the layer's weight gradient; the G rows are time of this class too
  // (the combine is recorded with the BN-backward apply class, lbf_combine)
  const double gbx = (((double)P * L.co + (double)P * L.ci) * c->esz + (double)L.co * L.ci * 4.0) * 1e-9;
  if (int r = prof_begin(c, W.s, 2, li, 2.0 * P * L.co * L.ci * 1e-9, &slot, gbx)) return r;
  if (L.ci < 256) {   // narrow ci: P1 and G as one launch of the tile shape the v2 heuristic picks
    WgradArgs a{};
    a.dy = dyhat.p; a.lddy = dyhat.ld;
    a.dy2 = y2.p; a.lddy2 = y2.ld; a.Co1 = L.co;
    a.x = y2.p; a.N = y2.N; a.H = y2.H; a.W = y2.W; a.C = y2.C; a.ldx = y2.ld;
    a.Ho = L.Ho; a.Wo = L.Wo; a.Co = L.co + L.ci;
    a.KH = a.KW = 1; a.sf = 1; a.dil = 1;
    a.splits = wgrad_splits(a, S.dt, c->side_active);
    a.splits = (int)std::max<long>(1, std::min<long>(a.splits, (long)c->slab_floats / n1));
    a.out = c->slab;
    HIPCALL(c, launch_conv_wgrad(S.dt, a, W.s));
    HIPCALL(c, launch_splitk_reduce(c->slab, a.splits, n1, n1, c->lbf_p1, 0, W.s));
  } else {
    // P1 = dyhat^T y2 and G = y2^T y2 as one launch: output rows co.. co + ci - 1 take y2 as dy
    WgradArgs a{};
    a.dy = dyhat.p; a.lddy = dyhat.ld;
    a.dy2 = y2.p; a.lddy2 = y2.ld; a.Co1 = L.co;
    a.x = y2.p; a.N = y2.N; a.H = y2.H; a.W = y2.W; a.C = y2.C; a.ldx = y2.ld;
    a.Ho = L.Ho; a.Wo = L.Wo; a.Co = L.co + L.ci;
    a.KH = a.KW = 1; a.sf = 1; a.dil = 1;
    a.splits = wgrad_splits(a, S.dt, c->side_active);
    a.splits = (int)std::max<long>(1, std::min<long>(a.splits, (long)c->slab_floats / ((long)a.Co * a.C)));
    a.out = c->slab;
    if (!conv_wgrad_pp_ok(a)) return set_err(&c->err, -EINVAL, "lbf weight gradient %s: shape", L.name.c_str());
    HIPCALL(c, launch_conv_wgrad_pp(S.dt, a, W.s));
    HIPCALL(c, launch_splitk_reduce(c->slab, a.splits, n1, n1, c->lbf_p1, 0, W.s));
  }
  return prof_end(c, W.s, slot);
}

// dW3 = A o P1 + B (x) colsum + D o (W3 G) into the gradient buffer, after the unit's conv2
// BN-backward reduce has written the column sums of y2 (recomputed there from z2 exactly as
// the forward BN apply formed y2: a separate pass over y2 measured the same step time,
// profiles/r05_s26_premask_cs_wg_ab.txt), on the weight-gradient stream when it is active
int lbf_combine(Step& S, Unit& u) {
  seg_ctx* c = S.c;
  const int li = u.c3;
  ConvL& L = c->convs[li];
  Step W = S;
  if (c->side_active) {
    HIPCALL(c, hipEventRecord(c->ev_dy[li], S.s));
    HIPCALL(c, hipStreamWaitEvent(c->side, c->ev_dy[li], 0));
    W.s = c->side;
  }
  int slot;
  // profiled as BN-backward apply time with the prep and H (the B and D terms it adds are that
  // pass's affine part); its bytes: P1, G, W3, the column-sum partials and the result
  const double gbc = ((double)L.co * L.ci * (4.0 + c->esz + 4.0) + (double)L.ci * L.ci * 4.0 +
                      (double)c->convs[u.c2].rb * L.ci * 4.0) * 1e-9;
  if (int r = prof_begin(c, W.s, 5, li, gbc, &slot)) return r;
  LbfCombineArgs cb{};
  cb.co = L.co; cb.ci = L.ci; cb.w = L.w_lp; cb.g = c->lbf_p1 + (size_t)L.co * L.ci; cb.p1 = c->lbf_p1;
  cb.cspart = L.lbf_cs; cb.rb = c->convs[u.c2].rb;
  cb.coef = L.lbf_coef; cb.out = c->grads + L.w_off;
  HIPCALL(c, launch_lbf_combine(S.dt, cb, W.s));
  if (int r = prof_end(c, W.s, slot)) return r;
  c->wg_done[li] = 1;
  return bucket_progress(c, W.s, false);
}

// after the conv3 BN reduce + finalize: the coefficients, the scaled weights, H, the weight
// gradient (side stream) and the conv3 data gradient as one K-concatenated GEMM
// [dyhat | y2] x [A o W3 ; H] into u.dz2 (its constant b is left to c2's BN backward)
int lbf_backward(Step& S, Unit& u, const Act& dyhat) {
  seg_ctx* c = S.c;
  ConvL& L = c->convs[u.c3];
  const int co = L.co, ci = L.ci;
  int slot;
  // profiled as BN-backward apply time (the pass they replace), in two records so that the
  // weight gradient queued between them (one stream when profiling) is not counted twice:
  // the prep's bytes (both weight copies read and written), then H's (its operands, slab and
  // 16-bit result)
  if (int r = prof_begin(c, S.s, 5, u.c3, 4.0 * co * ci * c->esz * 1e-9, &slot)) return r;
  LbfPrepArgs p{};
  p.co = co; p.ci = ci;
  p.mean = L.st.mean; p.invstd = L.st.invstd; p.scale = L.st.scale; p.sdy = L.st.sdy; p.sdyx = L.st.sdyx;
  p.w = L.w_lp; p.wt = L.wt_lp; p.wts = c->lbf_wts; p.xd = c->lbf_xd; p.bpart = c->lbf_bpart;
  p.coef = L.lbf_coef;
  HIPCALL(c, launch_lbf_prep(S.dt, p, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  if (int r = lbf_wgrad(S, u, dyhat)) return r;
  const double gbh = (2.0 * co * ci * c->esz + (double)ci * ci * (c->esz + 8.0 * lbf_hsplits(L))) * 1e-9;
  if (int r = prof_begin(c, S.s, 5, u.c3, gbh, &slot)) return r;
  WgradArgs h{};   // H[k][k'] = sum_c (D_c W3[c][k]) W3[c][k']: the channels c are the "pixels"
  h.dy = c->lbf_xd; h.lddy = ci;
  h.x = L.w_lp; h.N = 1; h.H = 1; h.W = co; h.C = ci; h.ldx = ci;
  h.Ho = 1; h.Wo = co; h.Co = ci; h.KH = h.KW = 1; h.sf = 1; h.dil = 1;
  h.splits = lbf_hsplits(L); h.out = c->lbf_hslab;
  HIPCALL(c, launch_conv_wgrad(S.dt, h, S.s));
  HIPCALL(c, launch_lbf_hreduce(S.dt, c->lbf_hslab, h.splits, (long)ci * ci, c->lbf_h, c->lbf_bpart,
                                co / 128, ci, c->lbf_bias, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  ConvArgs a{};
  a.x = dyhat.p; a.N = L.N; a.H = L.Ho; a.W = L.Wo; a.C = co; a.ldx = dyhat.ld;
  a.w = c->lbf_wts; a.ldw = co;
  a.y = u.dz2.p; a.Ho = L.H; a.Wo = L.W; a.Co = ci; a.ldy = u.dz2.ld;
  a.x2 = u.z2.p; a.ldx2 = u.z2.ld; a.C2 = ci; a.w2 = c->lbf_h; a.ldw2 = ci;
  a.KH = a.KW = 1; a.sf = 1; a.st = 1; a.dil = 1;
  const long M = (long)L.N * L.H * L.W;
  const double gbx = ((double)M * (co + ci) + (double)co * ci + (double)ci * ci + (double)M * ci) * c->esz * 1e-9;
  if (int r = prof_begin(c, S.s, 1, u.c3, 2.0 * M * ci * co * 1e-9, &slot, gbx)) return r;
  if (ci > 128) HIPCALL(c, launch_conv_nt_pp(S.dt, a, S.s));
  else HIPCALL(c, launch_conv_nt_v2(S.dt, a, S.s));
  if (int r = prof_end(c, S.s, slot)) return r;
  L.lbf_done = true;
  L.lbf_dyhat = dyhat;
  ++c->lbf_launches;
  return 0;
}

int unit_backward(Step& S, Unit& u, const Act& dx, bool accumulate, Unit* pred = nullptr) {
  seg_ctx* c = S.c;
  // identity / subsample shortcuts: the c3 BN backward also writes the ReLU-masked dout
  // (dpre), the residual of the unit's input gradient -- unless dout arrived masked
  // (dout_masked, premask_ok). (Measured and rejected: reading dout + the bits as the
  // residual in conv1's dgrad epilogue instead of dpre, 1.8 % slower per step.)
  const bool in_masked = u.dout_masked;
  u.dout_masked = false;
  const Act* dpre = u.kind != SC_CONV && !in_masked ? &u.dpre : nullptr;
  const Act& dres = in_masked ? u.dout : u.dpre;   // the masked dout, wherever it lives
  const ConvL& L3 = c->convs[u.c3];
  const ConvL& Ls = c->convs[u.kind == SC_CONV ? u.sc : u.c3];
  const bool lbf = lbf_ok(c, u, in_masked);
  if (lbf) {
    // linear BN-backward fold: reduce + finalize of conv3's BN (the gated gradient into dpre
    // by the reduce itself when dout is not pre-masked; a projection unit's dual reduce, then
    // the shortcut BN's apply alone), then no conv3 apply pass (lbf_backward)
    if (u.kind == SC_CONV) {
      if (int r = bn_backward_dual(S, u.c3, u.sc, u.dout, u.out, true)) return r;
    } else if (int r = bn_backward(S, u.c3, u.dout, 0, in_masked ? nullptr : &u.out, dpre, nullptr, nullptr,
                                   true)) {
      return r;
    }
    if (int r = lbf_backward(S, u, u.kind == SC_CONV ? u.dout : dres)) return r;
  } else {
    if (u.kind == SC_CONV && !c->gn && !c->sync_fn && u.out.mask && u.out.C == L3.co &&
        Ls.co == L3.co && Ls.rb == L3.rb && Ls.y.M() == L3.y.M()) {
      if (int r = bn_backward_dual(S, u.c3, u.sc, u.dout, u.out)) return r;
    } else {
      if (int r = bn_backward(S, u.c3, u.dout, 0, in_masked ? nullptr : &u.out, dpre)) return r;
      if (u.kind == SC_CONV)
        if (int r = bn_backward(S, u.sc, u.dout, 0, &u.out, nullptr)) return r;
    }
    if (int r = conv_wgrad(S, u.c3, u.z2)) return r;
    if (int r = conv_dgrad(S, u.c3, u.dz2)) return r;
  }
  if (int r = bn_backward(S, u.c2, u.dz2, 0, &u.z2, nullptr, nullptr, lbf ? c->lbf_bias : nullptr, false,
                         lbf ? L3.lbf_cs : nullptr))
    return r;
  if (lbf)
    if (int r = lbf_combine(S, u)) return r;
  if (int r = conv_wgrad(S, u.c2, u.z1)) return r;
  if (int r = conv_dgrad(S, u.c2, u.dz1)) return r;
  if (int r = bn_backward(S, u.c1, u.dz1, 0, &u.z1, nullptr)) return r;
  if (int r = conv_wgrad(S, u.c1, u.in)) return r;
  switch (u.kind) {
    case SC_IDENTITY:
      if (accumulate) return conv_dgrad(S, u.c1, dx, &dx, &dres);
      if (premask_ok(c, u, pred, accumulate)) {
        if (int r = conv_dgrad(S, u.c1, dx, &dres, nullptr, pred->out.mask)) return r;
        pred->dout_masked = true;   // only once the masked store is enqueued
        ++c->premask_launches;
        return 0;
      }
      return conv_dgrad(S, u.c1, dx, &dres);
    case SC_SUBSAMPLE: {
      if (accumulate) return set_err(&c->err, -EINVAL, "accumulating subsample unit");
      if (int r = conv_dgrad(S, u.c1, dx)) return r;
      HIPCALL(c, launch_add_strided(S.dt, dx.p, dx.H, dx.W, dx.ld, dres.p, dres.N, dres.H,
                                    dres.W, dres.C, dres.ld, u.stride, S.s));
      return 0;
    }
    case SC_CONV: {
      if (int r = conv_wgrad(S, u.sc, u.in)) return r;
      if (!accumulate) {   // one K-concatenated GEMM when both are 1 x 1 stride-1 ping-pong shapes
        const uint8_t* pm = premask_bits(c, pred, c->convs[u.c1].ci);
        const int r = conv_dgrad_dual(S, u.c1, u.sc, dx, &pm);
        if (r == 0 && pm) {
          pred->dout_masked = true;   // only once the masked store is enqueued
          ++c->premask_launches;
        }
        if (r <= 0) return r;
      }
      if (int r = conv_dgrad(S, u.c1, dx, accumulate ? &dx : nullptr)) return r;
      return conv_dgrad(S, u.sc, dx, &dx);
    }
  }
  return 0;
}

DeconvArgs deconv_args(seg_ctx* c) {
  DeconvArgs a{};
  a.x = (const float*)c->logits.p; a.y = c->up_in; a.g = c->grad_un; a.gscale = c->dzscale;
  a.dx = c->dc_dx; a.part = c->dc_part;
  a.N = c->logits.N; a.H = c->logits.H; a.W = c->logits.W; a.ld = c->ldl;
  for (int h = 0; h < 3; ++h) {
    a.c[h] = c->nc[h];
    a.w[h] = c->params + c->dc_w_off[h]; a.b[h] = c->params + c->dc_b_off[h];
    a.gw[h] = c->grads + c->dc_w_off[h]; a.gb[h] = c->grads + c->dc_b_off[h];
  }
  return a;
}

Act logits_slice(seg_ctx* c, int h) {
  int off = 0;
  for (int i = 0; i < h; ++i) off += c->nc[i];
  Act a = c->logits;
  a.p = (float*)c->logits.p + off;
  a.C = c->nc[h];
  return a;
}

int forward(Step& S, const float* images) {
  seg_ctx* c = S.c;
  if (c->bn_infer)
    HIPCALL(c, launch_bn_infer_finalize_all(c->infer_jobs, (int)c->convs.size(), S.s));
  if (c->stem_s2d) {
    const ConvL& st = c->convs[c->stem];
    HIPCALL(c, launch_cast_s2d(S.dt, images, c->img.p, st.N, st.H, st.W, c->img.H, c->img.W, st.pad_h,
                               st.pad_w, S.s));
  } else {
    HIPCALL(c, hipMemcpyAsync(c->img.p, images, (size_t)c->img.M() * 3 * sizeof(float),
                              hipMemcpyDeviceToDevice, S.s));
  }
  if (int r = conv_forward(S, c->stem, c->img)) return r;
  const ConvL& stl = c->convs[c->stem];
  if (!c->gn && c->z0.mask && c->pool_ph == 0 && c->pool_pw == 0 && c->z0.H == 2 * c->p0.H &&
      c->z0.W == 2 * c->p0.W) {
    // stem BN + ReLU fused into the max-pool: y0 is read once, z0 (the max-pool input) is never
    // written; its ReLU bits (the BN backward's gate) are
    const double esz = c->esz;
    const double gb = (c->z0.M() * 64.0 * (esz + 0.125) + c->p0.M() * 64.0 * (esz + 1.0)) * 1e-9;
    int slot;
    if (int r = prof_begin(c, S.s, 3, c->stem, gb, &slot)) return r;
    HIPCALL(c, launch_bn_relu_maxpool_fwd(S.dt, stl.y.p, c->z0.N, c->z0.H, c->z0.W, stl.y.ld,
                                          stl.st.mean, stl.st.scale, c->params + stl.b_off,
                                          c->z0.mask, c->p0.p, c->p0.H, c->p0.W, c->p0.ld,
                                          c->pool_ph, c->pool_pw, c->pool_arg, S.s));
    if (int r = prof_end(c, S.s, slot)) return r;
    c->z0_stale = true;
  } else {
    if (int r = bn_apply(S, c->stem, c->z0, 0)) return r;
    HIPCALL(c, launch_maxpool_fwd(S.dt, c->z0.p, c->z0.N, c->z0.H, c->z0.W, 64, c->z0.ld, c->p0.p,
                                  c->p0.H, c->p0.W, c->p0.ld, c->pool_ph, c->pool_pw, c->pool_arg,
                                  S.s));
    c->z0_stale = false;
  }
  for (auto& u : c->units)
    if (int r = unit_forward(S, u)) return r;
  if (int r = conv_forward(S, c->dfd, c->units.back().out)) return r;
  if (c->fov >= 0) {
    if (int r = bn_apply(S, c->dfd, c->z_pre, 0)) return r;
    if (int r = conv_forward(S, c->fov, c->z_pre)) return r;
    if (int r = bn_apply(S, c->fov, c->z_dfd, 0)) return r;
  } else if (int r = bn_apply(S, c->dfd, c->z_dfd, 0)) {
    return r;
  }
  if (c->cfg.pyramid == SEG_PYRAMID_PSP) {
    const Act& z = c->z_dfd;
    HIPCALL(c, launch_grid_rowreduce(S.dt, z.p, z.N, z.H, z.W, z.C, z.ld, c->pool_grids,
                                     c->grid_part, S.s));
    void* outs[SEG_MAX_GRIDS];
    for (int b = 0; b < 4; ++b) outs[b] = c->pooled[b].p;
    HIPCALL(c, launch_grid_colreduce(S.dt, c->grid_part, z.N, z.H, z.W, z.C, c->pool_grids, outs, S.s));
    const int fd = c->cfg.feature_dims;
    for (int b = 0; b < 4; ++b) {
      if (int r = conv_forward(S, c->pyr_conv[b], c->pooled[b])) return r;
      if (int r = bn_apply(S, c->pyr_conv[b], c->zb[b], 0)) return r;
      Act dst = slice(c, c->concat, (b + 1) * fd, fd);
      HIPCALL(c, launch_resize_fwd(S.dt, c->zb[b].p, c->zb[b].N, c->zb[b].H, c->zb[b].W, fd,
                                   c->zb[b].ld, dst.p, dst.H, dst.W, dst.ld, S.s));
    }
    if (int r = conv_forward(S, c->pyr_final, c->concat)) return r;
    if (int r = bn_apply(S, c->pyr_final, c->feat, 0)) return r;
  } else if (c->cfg.pyramid == SEG_PYRAMID_ASPP) {
    const Act& z = c->z_dfd;
    const int fd = c->cfg.feature_dims;
    // image-pool branch: global mean -> 1x1 conv/BN/ReLU -> align-corners broadcast (slice 0)
    HIPCALL(c, launch_grid_rowreduce(S.dt, z.p, z.N, z.H, z.W, z.C, z.ld, c->pool_grids,
                                     c->grid_part, S.s));
    void* outs[SEG_MAX_GRIDS] = {c->pooled[0].p, nullptr, nullptr, nullptr};
    HIPCALL(c, launch_grid_colreduce(S.dt, c->grid_part, z.N, z.H, z.W, z.C, c->pool_grids, outs, S.s));
    if (int r = conv_forward(S, c->pyr_conv[0], c->pooled[0])) return r;
    if (int r = bn_apply(S, c->pyr_conv[0], c->zb[0], 0)) return r;
    Act d0 = slice(c, c->concat, 0, fd);
    HIPCALL(c, launch_resize_fwd(S.dt, c->zb[0].p, c->zb[0].N, 1, 1, fd, c->zb[0].ld, d0.p, d0.H,
                                 d0.W, d0.ld, S.s));
    // 1x1 and the rate-6/12/18 3x3 branches write their BN/ReLU outputs into slices 1..4
    for (int b = 1; b < 5; ++b) {
      if (int r = conv_forward(S, c->pyr_conv[b], z)) return r;
      if (int r = bn_apply(S, c->pyr_conv[b], slice(c, c->concat, b * fd, fd), 0)) return r;
    }
    if (int r = conv_forward(S, c->pyr_final, c->concat)) return r;
    if (int r = bn_apply(S, c->pyr_final, c->feat, 0)) return r;
  }
  for (int h = 0; h < 3; ++h) {
    if (int r = unit_forward(S, c->heads[h])) return r;
    if (int r = conv_forward(S, c->logit_conv[h], c->heads[h].out)) return r;
    if (int r = bn_apply(S, c->logit_conv[h], logits_slice(c, h), 1)) return r;
  }
  if (c->hybrid) HIPCALL(c, launch_deconv_fwd(deconv_args(c), S.s));
  return 0;
}

int backward_layers(Step& S);
int backward(Step& S) {
  seg_ctx* c = S.c;
  std::fill(c->wg_done.begin(), c->wg_done.end(), 0);
  c->bk_next = 0;
  // a profiled backward runs on one stream so the HIP-event kernel timings are kernel-alone
  c->side_active = c->side_on && !c->prof.on;
  c->prestem_rec = false;
  if (c->side_active) {   // the side stream must not run ahead of the previous use of its buffers
    HIPCALL(c, hipEventRecord(c->ev_join, S.s));
    HIPCALL(c, hipStreamWaitEvent(c->side, c->ev_join, 0));
  }
  if (int r = backward_layers(S)) return r;
  if (int r = bucket_progress(c, c->side_active ? c->side : S.s, true)) return r;
  if (c->side_active) {   // join: the update (and the next forward) follow every weight gradient
    HIPCALL(c, hipEventRecord(c->ev_join, c->side));
    if (c->prestem_rec) {   // deferred: only the gradients before the stem's (see seg_apply_update)
      HIPCALL(c, hipStreamWaitEvent(S.s, c->ev_prestem, 0));
      c->stem_pending = true;
    } else {
      HIPCALL(c, hipStreamWaitEvent(S.s, c->ev_join, 0));
    }
  }
  // BN-parameter + statistics tail bucket: written on the compute stream
  HIPCALL(c, hipEventRecord(c->bk_ev.back(), S.s));
  return 0;
}

int backward_layers(Step& S) {
  seg_ctx* c = S.c;
  // no pre-masked gradient survives a backward that stopped part-way (unit_backward)
  for (auto& u : c->units) u.dout_masked = false;
  for (auto& u : c->heads) u.dout_masked = false;
  for (auto& L : c->convs) L.lbf_done = L.lbf_dy_ready = false;
  // hybrid: the loss-normalised gradient goes back through the deconvolution first (its
  // weight / bias gradients and dx), then into the logits BN without a further scale
  if (c->hybrid) HIPCALL(c, launch_deconv_bwd(deconv_args(c), S.s));
  for (int h = 0; h < 3; ++h) {
    Act gz = logits_slice(c, h);
    int off = (int)((float*)gz.p - (float*)c->logits.p);
    gz.p = (c->hybrid ? c->dc_dx : c->grad_un) + off;
    if (int r = bn_backward(S, c->logit_conv[h], gz, 1, nullptr, nullptr,
                            c->hybrid ? nullptr : c->dzscale + off)) return r;
    if (int r = conv_wgrad(S, c->logit_conv[h], c->heads[h].out)) return r;
    if (int r = conv_dgrad(S, c->logit_conv[h], c->heads[h].dout)) return r;
    if (int r = unit_backward(S, c->heads[h], c->dfeat, h > 0)) return r;
  }
  if (c->cfg.pyramid == SEG_PYRAMID_PSP) {
    const int fd = c->cfg.feature_dims;
    if (int r = bn_backward(S, c->pyr_final, c->dfeat, 0, &c->feat, nullptr)) return r;
    if (int r = conv_wgrad(S, c->pyr_final, c->concat)) return r;
    if (int r = conv_dgrad(S, c->pyr_final, c->dconcat)) return r;
    for (int b = 0; b < 4; ++b) {
      Act d = slice(c, c->dconcat, (b + 1) * fd, fd);
      HIPCALL(c, launch_grid_rowreduce(S.dt, d.p, d.N, d.H, d.W, fd, d.ld, c->up_grids[b],
                                       c->grid_part, S.s));
      void* outs[SEG_MAX_GRIDS] = {c->dzb[b].p, nullptr, nullptr, nullptr};
      HIPCALL(c, launch_grid_colreduce(S.dt, c->grid_part, d.N, d.H, d.W, fd, c->up_grids[b], outs, S.s));
      if (int r = bn_backward(S, c->pyr_conv[b], c->dzb[b], 0, &c->zb[b], nullptr)) return r;
      if (int r = conv_wgrad(S, c->pyr_conv[b], c->pooled[b])) return r;
      if (int r = conv_dgrad(S, c->pyr_conv[b], c->dpooled[b])) return r;
    }
    const void* dps[SEG_MAX_GRIDS];
    for (int b = 0; b < 4; ++b) dps[b] = c->dpooled[b].p;
    Act d0 = slice(c, c->dconcat, 0, fd);
    HIPCALL(c, launch_psp_input_bwd(S.dt, d0.p, d0.ld, c->pool_grids, dps, d0.N, d0.H, d0.W, fd,
                                    c->dz_dfd.p, c->dz_dfd.ld, S.s));
  } else if (c->cfg.pyramid == SEG_PYRAMID_ASPP) {
    const int fd = c->cfg.feature_dims;
    if (int r = bn_backward(S, c->pyr_final, c->dfeat, 0, &c->feat, nullptr)) return r;
    if (int r = conv_wgrad(S, c->pyr_final, c->concat)) return r;
    if (int r = conv_dgrad(S, c->pyr_final, c->dconcat)) return r;
    // image-pool branch: transpose of the broadcast = sum over the map
    Act s0 = slice(c, c->dconcat, 0, fd);
    HIPCALL(c, launch_grid_rowreduce(S.dt, s0.p, s0.N, s0.H, s0.W, fd, s0.ld, c->up_grids[0],
                                     c->grid_part, S.s));
    void* outs[SEG_MAX_GRIDS] = {c->dzb[0].p, nullptr, nullptr, nullptr};
    HIPCALL(c, launch_grid_colreduce(S.dt, c->grid_part, s0.N, s0.H, s0.W, fd, c->up_grids[0], outs, S.s));
    if (int r = bn_backward(S, c->pyr_conv[0], c->dzb[0], 0, &c->zb[0], nullptr)) return r;
    if (int r = conv_wgrad(S, c->pyr_conv[0], c->pooled[0])) return r;
    if (int r = conv_dgrad(S, c->pyr_conv[0], c->dpooled[0])) return r;
    // conv branches: dz_dfd = sum of their data gradients (fixed branch order)
    for (int b = 1; b < 5; ++b) {
      Act db = slice(c, c->dconcat, b * fd, fd);
      Act zb = slice(c, c->concat, b * fd, fd);
      if (int r = bn_backward(S, c->pyr_conv[b], db, 0, &zb, nullptr)) return r;
      if (int r = conv_wgrad(S, c->pyr_conv[b], c->z_dfd)) return r;
      if (int r = conv_dgrad(S, c->pyr_conv[b], c->dz_dfd, b > 1 ? &c->dz_dfd : nullptr)) return r;
    }
    // + the global-average-pool transpose, in place
    const void* dps[SEG_MAX_GRIDS] = {c->dpooled[0].p, nullptr, nullptr, nullptr};
    HIPCALL(c, launch_psp_input_bwd(S.dt, c->dz_dfd.p, c->dz_dfd.ld, c->pool_grids, dps, c->dz_dfd.N,
                                    c->dz_dfd.H, c->dz_dfd.W, fd, c->dz_dfd.p, c->dz_dfd.ld, S.s));
  }
  if (c->fov >= 0) {
    if (int r = bn_backward(S, c->fov, c->dz_dfd, 0, &c->z_dfd, nullptr)) return r;
    if (int r = conv_wgrad(S, c->fov, c->z_pre)) return r;
    if (int r = conv_dgrad(S, c->fov, c->dz_pre)) return r;
    if (int r = bn_backward(S, c->dfd, c->dz_pre, 0, &c->z_pre, nullptr)) return r;
  } else if (int r = bn_backward(S, c->dfd, c->dz_dfd, 0, &c->z_dfd, nullptr)) {
    return r;
  }
  if (int r = conv_wgrad(S, c->dfd, c->units.back().out)) return r;
  {
    Unit& last = c->units.back();
    const uint8_t* pm = premask_bits(c, &last, c->convs[c->dfd].ci);
    if (pm) {
      ConvArgs a = dgrad_args(c, c->dfd, last.dout, nullptr, nullptr);
      a.omask = pm; a.ldm = a.Co / 8;
      if (!conv_nt_omask_ok(S.dt, a)) pm = nullptr;
    }
    if (int r = conv_dgrad(S, c->dfd, last.dout, nullptr, nullptr, pm)) return r;
    if (pm) { last.dout_masked = true; ++c->premask_launches; }
  }
  for (int i = (int)c->units.size() - 1; i >= 0; --i) {
    const Act& dx = i == 0 ? c->dp0 : c->units[i - 1].dout;
    if (int r = unit_backward(S, c->units[i], dx, false, i == 0 ? nullptr : &c->units[i - 1])) return r;
  }
  HIPCALL(c, launch_maxpool_bwd(S.dt, c->pool_arg, c->z0.N, c->z0.H, c->z0.W, 64, c->dp0.p,
                                c->dp0.H, c->dp0.W, c->dp0.ld, c->dz0.p, c->dz0.ld, c->pool_ph,
                                c->pool_pw, S.s));
  if (int r = bn_backward(S, c->stem, c->dz0, 0, &c->z0, nullptr)) return r;
  return conv_wgrad(S, c->stem, c->img);
}

int refresh_stem_pad(seg_ctx* c, hipStream_t s) {
  if (!c->stem_s2d) return 0;
  const ConvL& st = c->convs[c->stem];
  HIPCALL(c, launch_stem_s2d_weights((const bf16_t*)st.w_lp, c->stem_wpad, st.co, s));
  return 0;
}

// a deferred stem weight gradient (seg_set_defer_stem) must be complete before anything else
// on stream s reads or rewrites the step's buffers. The pending state is kept until the
// gradient is consumed (seg_apply_update) or superseded (seg_backward): a join on another
// stream must not let a later seg_apply_update skip its own join
int join_stem(seg_ctx* c, hipStream_t s, bool consume = false) {
  if (!c->stem_pending) return 0;
  HIPCALL(c, hipStreamWaitEvent(s, c->ev_join, 0));
  if (consume) c->stem_pending = false;
  return 0;
}

int refresh_compute_weights(seg_ctx* c, hipStream_t s) {
  if (seg_half(c->dt))
    HIPCALL(c, launch_cast_f32_half(c->dt, c->params, c->w_lp_flat, c->n_decay, s));
  if (c->n_flip) HIPCALL(c, launch_weight_flip_batched(c->dt, c->flip_jobs, c->n_flip, c->flip_total, s));
  return refresh_stem_pad(c, s);
}

}  // namespace

// ==========================================================================================
// C ABI
// ==========================================================================================
extern "C" {

const char* seg_last_error(seg_ctx* ctx) { return ctx ? ctx->err.c_str() : g_err.c_str(); }
int seg_set_loss_scale(seg_ctx* c, float scale);

int seg_create(int device, const seg_cfg* cfg, seg_ctx** out) {
  if (!cfg || !out) return set_err(nullptr, -EINVAL, "null argument");
  *out = nullptr;
  // host-side validation first: a bad configuration fails the same way with or without a GPU
  if (cfg->dtype < SEG_DTYPE_F32 || cfg->dtype > SEG_DTYPE_F16)
    return set_err(nullptr, -EINVAL, "dtype %d (SEG_DTYPE_F32 / _BF16 / _F16)", cfg->dtype);
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return set_err(nullptr, -ENODEV, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
  seg_ctx* c = new seg_ctx();
  c->cfg = *cfg;
  c->device = device;
  c->dt = dt_of(cfg->dtype);
  c->esz = seg_half(c->dt) ? 2 : 4;
  int r = build(c);
  if (!r && c->dt == SEG_F16) r = seg_set_loss_scale(c, 1.f);   // overflow flag of fp16 steps
  if (r) {
    std::string msg = c->err;
    seg_destroy(c);
    return set_err(nullptr, r, "%s", msg.c_str());
  }
  *out = c;
  return 0;
}

int seg_destroy(seg_ctx* c) {
  if (!c) return 0;
  (void)hipSetDevice(c->device);
  if (c->side) (void)hipStreamSynchronize(c->side);   // a deferred stem weight gradient
  (void)hipDeviceSynchronize();
  for (void* p : c->allocs) (void)hipFree(p);
  if (c->infer_jobs) (void)hipFree(c->infer_jobs);
  for (auto ev : c->prof.ev) (void)hipEventDestroy(ev);
  for (auto ev : c->bk_ev) (void)hipEventDestroy(ev);
  for (auto ev : c->ev_dy) (void)hipEventDestroy(ev);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->ev_prestem) (void)hipEventDestroy(c->ev_prestem);
  if (c->side) (void)hipStreamDestroy(c->side);
  delete c;
  return 0;
}

int seg_sizes(seg_ctx* c, int64_t* n_train, int64_t* n_decay, int64_t* n_moving, int64_t* n_stats) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (n_train) *n_train = c->n_train;
  if (n_decay) *n_decay = c->n_decay;
  if (n_moving) *n_moving = c->n_moving;
  if (n_stats) *n_stats = c->n_stats;
  return 0;
}

int seg_bind_buffers(seg_ctx* c, float* params, float* grads, float* momentum, float* ema,
                     float* moving) {
  if (!c || !params || !grads || !momentum || !moving)
    return set_err(c ? &c->err : nullptr, -EINVAL, "params/grads/momentum/moving required");
  c->params = params; c->grads = grads; c->mom = momentum; c->ema = ema; c->moving = moving;
  const long half = c->n_moving / 2;
  for (auto& L : c->convs) {
    if (c->dt == SEG_F32) L.w_lp = params + L.w_off;
    // batch statistics land directly in the gradient tail (one all-reduce covers them)
    L.st.mean = grads + c->n_train + L.mv_off;
    L.st.var_unb = grads + c->n_train + half + L.mv_off;
  }
  // the batched flip table needs the compute-weight pointers (fp32: the bound params)
  std::vector<FlipJob> jobs;
  long tot = 0;
  for (auto& L : c->convs)
    if (L.wt_lp) {
      jobs.push_back({L.w_lp, L.wt_lp, L.co, L.k, L.ci, tot});
      tot += flip_tiles(L.co, L.k, L.ci);
    }
  c->n_flip = (int)jobs.size();
  c->flip_total = tot;
  if (c->n_flip) {
    if (!c->flip_jobs)
      if (int r = dalloc(c, &c->flip_jobs, jobs.size())) return r;
    HIPCALL(c, hipMemcpy(c->flip_jobs, jobs.data(), jobs.size() * sizeof(FlipJob), hipMemcpyHostToDevice));
  }
  c->bound = true;
  return 0;
}

int64_t seg_param_count(seg_ctx* c) { return c ? (int64_t)c->pinfo.size() : -1; }

int seg_param_info(seg_ctx* c, int64_t i, const char** name, int64_t* offset, int64_t* numel,
                   int* kind) {
  if (!c || i < 0 || i >= (int64_t)c->pinfo.size()) return set_err(c ? &c->err : nullptr, -EINVAL, "bad index");
  const auto& p = c->pinfo[i];
  if (name) *name = p.name.c_str();
  if (offset) *offset = p.off;
  if (numel) *numel = p.numel;
  if (kind) *kind = p.kind;
  return 0;
}

int seg_param_shape(seg_ctx* c, int64_t i, int64_t* dims) {
  if (!c || !dims || i < 0 || i >= (int64_t)c->pinfo.size())
    return set_err(c ? &c->err : nullptr, -EINVAL, "bad index");
  for (int k = 0; k < 4; ++k) dims[k] = c->pinfo[i].dims[k];
  return 0;
}

#define NEED_BOUND(c) \
  if (!(c) || !(c)->bound) return set_err((c) ? &(c)->err : nullptr, -EINVAL, "context not bound")

int seg_params_updated(seg_ctx* c, void* stream) {
  NEED_BOUND(c);
  if (int r = join_stem(c, (hipStream_t)stream)) return r;
  return refresh_compute_weights(c, (hipStream_t)stream);
}

int seg_forward(seg_ctx* c, const float* images, void* stream) {
  NEED_BOUND(c);
  if (!images) return set_err(&c->err, -EINVAL, "images required");
  Step S{c, (hipStream_t)stream, c->dt};
  if (int r = join_stem(c, S.s)) return r;
  return forward(S, images);
}

int seg_loss(seg_ctx* c, const int32_t* px, const float* bbox, const float* tag, int32_t* decisions,
             void* stream) {
  NEED_BOUND(c);
  if (int r = join_stem(c, (hipStream_t)stream)) return r;
  const seg_cfg& g = c->cfg;
  if ((g.nb_pp && !px) || (g.nb_pb && !bbox) || (g.nb_pi && !tag))
    return set_err(&c->err, -EINVAL, "missing labels for a non-empty sub-batch");
  LossArgs a{};
  a.logits = c->head_in; a.N = c->logits.N; a.Hl = c->logits.H; a.Wl = c->logits.W;
  a.ldl = c->ldl; a.H = g.height; a.W = g.width;
  a.npp = g.nb_pp; a.npb = g.nb_pb; a.npi = g.nb_pi;
  a.px_labels = px; a.bbox_soft = bbox; a.tag_soft = tag;
  a.grad_un = c->grad_un; a.part = c->loss_part; a.decisions = decisions;
  hipStream_t s = (hipStream_t)stream;
  HIPCALL(c, launch_loss_head(a, c->tables, s));
  if (c->tables.c1 == 14 && loss_head_yf(a.W, a.Wl)) ++c->loss_yf_launches;
  HIPCALL(c, launch_loss_finalize(c->loss_part, c->loss_blocks, c->tables, c->ldl, c->loss_scale,
                                  c->loss_out, c->dzscale, s));
  return 0;
}

int seg_set_bn_inference(seg_ctx* c, int on) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (c->gn) return 0;   // group norm normalises every image by its own statistics in all modes
  if (on) {   // (re)build the per-layer job table from the bound buffers (outside any step)
    NEED_BOUND(c);
    std::vector<BnInferJob> jobs;
    const long half = c->n_moving / 2;
    for (const ConvL& L : c->convs)
      jobs.push_back({c->moving + L.mv_off, c->moving + half + L.mv_off, c->params + L.g_off,
                      L.st, L.co});
    if (!c->infer_jobs) {
      HIPCALL(c, hipMalloc(&c->infer_jobs, jobs.size() * sizeof(BnInferJob)));
    }
    HIPCALL(c, hipMemcpy(c->infer_jobs, jobs.data(), jobs.size() * sizeof(BnInferJob),
                         hipMemcpyHostToDevice));
  }
  c->bn_infer = on ? 1 : 0;
  return 0;
}

int seg_predict(seg_ctx* c, const int32_t* cid_map, int n_map, int replace_voids, int out_h,
                int out_w, int32_t* decisions_out, void* stream) {
  NEED_BOUND(c);
  if (int r = join_stem(c, (hipStream_t)stream)) return r;
  const seg_cfg& g = c->cfg;
  if (!cid_map || !decisions_out) return set_err(&c->err, -EINVAL, "null cid_map / decisions_out");
  if (n_map != c->tables.n_pp)
    return set_err(&c->err, -EINVAL, "cid map has %d entries, the model has %d training classes",
                   n_map, c->tables.n_pp);
  if (out_h < 1 || out_w < 1) return set_err(&c->err, -EINVAL, "bad output size %dx%d", out_h, out_w);
  if (replace_voids < 0 || replace_voids > 2)
    return set_err(&c->err, -EINVAL, "replace_voids = %d (0, 1 or 2)", replace_voids);
  EvalArgs a{};
  a.logits = c->head_in; a.N = c->logits.N; a.Hl = c->logits.H; a.Wl = c->logits.W;
  a.ldl = c->ldl; a.H = g.height; a.W = g.width; a.Ho = out_h; a.Wo = out_w;
  a.replace_voids = replace_voids; a.n_map = n_map; a.out = decisions_out;
  int mx = -1;
  for (int i = 0; i < n_map; ++i) mx = std::max(mx, (int)cid_map[i]);
  for (int i = 0; i < n_map; ++i) {   // utils._replacevoids: -1 -> max + 1
    if (cid_map[i] < -1) return set_err(&c->err, -EINVAL, "cid_map[%d] = %d", i, cid_map[i]);
    a.map[i] = cid_map[i] == -1 ? mx + 1 : cid_map[i];
  }
  HIPCALL(c, launch_eval_decisions(a, c->tables, (hipStream_t)stream));
  return 0;
}

int seg_full_predictions(seg_ctx* c, float* logits_out, float* probs_out,
                         int32_t* head_decisions_out, int32_t* decisions_out, void* stream) {
  NEED_BOUND(c);
  if (int r = join_stem(c, (hipStream_t)stream)) return r;
  FullPredArgs a{};
  a.logits = c->head_in; a.N = c->logits.N; a.Hl = c->logits.H; a.Wl = c->logits.W;
  a.ldl = c->ldl; a.H = c->cfg.height; a.W = c->cfg.width;
  a.logits_out = logits_out; a.probs_out = probs_out;
  a.head_decs_out = head_decisions_out; a.decs_out = decisions_out;
  if ((reinterpret_cast<uintptr_t>(logits_out) | reinterpret_cast<uintptr_t>(probs_out)) & 15)
    return set_err(&c->err, -EINVAL, "logits_out / probs_out must be 16-byte aligned");
  HIPCALL(c, launch_full_predictions(a, c->tables, (hipStream_t)stream));
  return 0;
}

int seg_backward(seg_ctx* c, void* stream) {
  NEED_BOUND(c);
  Step S{c, (hipStream_t)stream, c->dt};
  if (int r = join_stem(c, S.s, true)) return r;
  return backward(S);
}

int seg_apply_update(seg_ctx* c, float lr, float momentum, float ema_decay_eff, float grad_scale,
                     void* stream) {
  NEED_BOUND(c);
  hipStream_t s = (hipStream_t)stream;
  const ConvL& stl = c->convs[c->stem];
  const long st_lo = stl.w_off, st_hi = stl.w_off + (long)stl.co * stl.k * stl.k * stl.ci;
  // deferred stem (seg_set_defer_stem): every parameter but the stem's conv weights is updated
  // while the stem's weight gradient still runs on the weight-gradient stream; not with loss
  // scaling (one overflow check covers all gradients) or a gradient scale (the all-reduce path)
  const bool split = c->stem_pending && !c->skip_flag && grad_scale == 1.f && !stl.wt_lp &&
                     st_hi <= c->n_decay;
  if (!split)
    if (int r = join_stem(c, s, true)) return r;
  if (c->skip_flag) {   // loss-scaled (fp16) step: unscale, and skip it if anything overflowed
    HIPCALL(c, hipMemsetAsync(c->skip_flag, 0, sizeof(int), s));
    HIPCALL(c, launch_nonfinite(c->grads, c->n_train, c->skip_flag, s));
    HIPCALL(c, launch_scale2(c->grads, c->n_train, grad_scale / c->loss_scale, c->n_stats, grad_scale, s));
  } else if (grad_scale != 1.f) {
    HIPCALL(c, launch_scale_inplace(c->grads, c->n_train + c->n_stats, grad_scale, s));
  }
  SgdmArgs a{};
  a.w = c->params; a.g = c->grads; a.v = c->mom;
  a.ema = ema_decay_eff > 0.f ? c->ema : nullptr;
  a.w_lp = seg_half(c->dt) ? c->w_lp_flat : nullptr;
  a.lp_f16 = c->dt == SEG_F16;
  a.skip = c->skip_flag;
  a.n = c->n_decay; a.lr = lr; a.momentum = momentum; a.wd = c->cfg.weight_decay;
  a.ema_decay = ema_decay_eff; a.reg_part = c->reg_part; a.nesterov = c->nesterov;
  int nparts = sgdm_blocks(c->n_decay);
  SgdmArgs st_a = a;   // the stem's range (split): [st_lo, st_hi), partials after the others'
  if (split) {
    // [0, st_lo) and [st_hi, n_decay) now, partials packed in that order, then the stem's
    SgdmArgs r0 = a, r1 = a;
    r0.n = st_lo;
    r1.w = a.w + st_hi; r1.g = a.g + st_hi; r1.v = a.v + st_hi;
    r1.ema = a.ema ? a.ema + st_hi : nullptr;
    r1.w_lp = a.w_lp ? (char*)a.w_lp + st_hi * c->esz : nullptr;
    r1.n = c->n_decay - st_hi;
    r1.reg_part = a.reg_part + sgdm_blocks(r0.n);
    HIPCALL(c, launch_sgdm(r0, s));
    HIPCALL(c, launch_sgdm(r1, s));
    st_a.w = a.w + st_lo; st_a.g = a.g + st_lo; st_a.v = a.v + st_lo;
    st_a.ema = a.ema ? a.ema + st_lo : nullptr;
    st_a.w_lp = a.w_lp ? (char*)a.w_lp + st_lo * c->esz : nullptr;
    st_a.n = st_hi - st_lo;
    st_a.reg_part = r1.reg_part + sgdm_blocks(r1.n);
    nparts = sgdm_blocks(r0.n) + sgdm_blocks(r1.n) + sgdm_blocks(st_a.n);
  } else {
    HIPCALL(c, launch_sgdm(a, s));
    HIPCALL(c, launch_sum_partials(c->reg_part, nparts, c->reg_out, s));
  }
  if (c->cfg.train_bn) {
    SgdmArgs b = a;
    b.w = c->params + c->n_decay; b.g = c->grads + c->n_decay; b.v = c->mom + c->n_decay;
    b.ema = a.ema ? c->ema + c->n_decay : nullptr; b.w_lp = nullptr; b.n = c->n_train - c->n_decay;
    b.wd = 0.f; b.reg_part = nullptr;
    HIPCALL(c, launch_sgdm(b, s));
  } else if (c->hybrid) {   // frozen BN parameters: the deconv biases still train
    SgdmArgs b = a;
    b.w = c->params + c->dc_b_lo; b.g = c->grads + c->dc_b_lo; b.v = c->mom + c->dc_b_lo;
    b.ema = a.ema ? c->ema + c->dc_b_lo : nullptr; b.w_lp = nullptr; b.n = c->n_train - c->dc_b_lo;
    b.wd = 0.f; b.reg_part = nullptr;
    HIPCALL(c, launch_sgdm(b, s));
  }
  const long half = c->n_moving / 2;
  // group norm keeps no moving statistics; a moving-statistics (frozen) step updates none
  if (!c->gn && !c->bn_infer)
    HIPCALL(c, launch_moving_update(c->moving, c->moving + half, c->grads + c->n_train,
                                    c->grads + c->n_train + half, (int)half, c->cfg.bn_decay, s));
  if (c->n_flip) HIPCALL(c, launch_weight_flip_batched(c->dt, c->flip_jobs, c->n_flip, c->flip_total, s));
  if (split) {   // the stem's weight gradient is done: its update, then the regulariser sum
    if (int r = join_stem(c, s, true)) return r;
    HIPCALL(c, launch_sgdm(st_a, s));
    HIPCALL(c, launch_sum_partials(c->reg_part, nparts, c->reg_out, s));
  }
  return refresh_stem_pad(c, s);
}

int seg_flush_grads(seg_ctx* c, void* stream) {
  NEED_BOUND(c);
  // a deferred stem weight gradient may still run on the weight-gradient stream: the caller's
  // stream waits for it (without consuming the join seg_apply_update takes)
  return join_stem(c, (hipStream_t)stream, false);
}

int seg_set_defer_stem(seg_ctx* c, int on) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  c->defer_stem = on != 0;
  return 0;
}

int seg_set_premask(seg_ctx* c, int on) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  c->premask = on != 0;
  return 0;
}

int seg_set_lbf(seg_ctx* c, int on) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  c->lbf_on = on != 0;
  return 0;
}

int seg_counter(seg_ctx* c, const char* name, int64_t* value) {
  if (!c || !name || !value) return set_err(c ? &c->err : nullptr, -EINVAL, "null argument");
  const std::string n(name);
  if (n == "premask_launches") *value = c->premask_launches;
  else if (n == "lbf_layers") *value = c->lbf_launches;
  else if (n == "loss_yf_launches") *value = c->loss_yf_launches;
  else return set_err(&c->err, -ENOENT, "unknown counter '%s'", name);
  return 0;
}

int seg_outputs(seg_ctx* c, const float** losses, const float** reg, const float** logits,
                int* ld, int* hl, int* wl) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (losses) *losses = c->loss_out;
  if (reg) *reg = c->reg_out;
  if (logits) *logits = c->head_in;
  if (ld) *ld = c->ldl;
  if (hl) *hl = c->logits.H;
  if (wl) *wl = c->logits.W;
  return 0;
}

int seg_confusion(seg_ctx* c, const int32_t* labels, const int32_t* decisions, int64_t n,
                  int num_classes, int32_t* cm, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = hipMemsetAsync(cm, 0, (size_t)num_classes * num_classes * 4, s);
  if (e == hipSuccess) e = launch_confusion(labels, decisions, n, num_classes, cm, s);
  if (e != hipSuccess) return hip_fail(c, e, "seg_confusion");
  return 0;
}

int seg_set_nesterov(seg_ctx* c, int on) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  c->nesterov = on ? 1 : 0;
  return 0;
}

int seg_set_loss_scale(seg_ctx* c, float scale) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (!(scale > 0.f)) return set_err(&c->err, -EINVAL, "loss scale must be > 0");
  c->loss_scale = scale;
  if (!c->skip_flag && (scale != 1.f || c->dt == SEG_F16))
    if (int r = dalloc(c, &c->skip_flag, 1)) return r;
  return 0;
}

int seg_set_bn_sync(seg_ctx* c, seg_allreduce_fn fn, void* user, int world) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (c->gn && fn && world > 1)   // module_arg_scope :329-331
    return set_err(&c->err, -EINVAL, "cross_replica_norm is supported only for batch normalization");
  if (world < 1) return set_err(&c->err, -EINVAL, "world must be >= 1");
  if (!fn) {   // world == 1 with a hook still exchanges (a one-replica collective)
    c->sync_fn = nullptr;
    c->sync_user = nullptr;
    c->sync_world = 1;
    return 0;
  }
  if (!c->sync_pack) {
    int cmax = 1;
    for (const ConvL& L : c->convs) cmax = std::max(cmax, L.co);
    if (int r = dalloc(c, &c->sync_pack, 2 * (size_t)cmax)) return r;
  }
  c->sync_fn = fn;
  c->sync_user = user;
  c->sync_world = world;
  return 0;
}

int seg_found_inf(seg_ctx* c, const int32_t** flag) {
  if (!c || !flag) return set_err(c ? &c->err : nullptr, -EINVAL, "null argument");
  *flag = c->skip_flag;
  return 0;
}

int seg_grad_buckets(seg_ctx* c, int max_buckets, int64_t* lo, int64_t* hi) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  const int n = (int)c->bk_lo.size();
  for (int i = 0; i < n && i < max_buckets; ++i) {
    if (lo) lo[i] = c->bk_lo[i];
    if (hi) hi[i] = c->bk_hi[i];
  }
  return n;
}

int seg_stream_wait_bucket(seg_ctx* c, int bucket, void* stream) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (bucket < 0 || bucket >= (int)c->bk_ev.size()) return set_err(&c->err, -EINVAL, "bad bucket %d", bucket);
  HIPCALL(c, hipStreamWaitEvent((hipStream_t)stream, c->bk_ev[bucket], 0));
  return 0;
}

int seg_bbox_labels(const float* boxes, const int32_t* cids, const int32_t* box_off,
                    const int32_t* geom, int n, int max_boxes, int H, int W, float* out,
                    void* stream) {
  if (n < 0 || H <= 0 || W <= 0 || (n > 0 && (!box_off || !geom || !out)))
    return set_err(nullptr, -EINVAL, "seg_bbox_labels: bad arguments");
  if (max_boxes < 0 || max_boxes > 1024)
    return set_err(nullptr, -E2BIG, "seg_bbox_labels: at most 1024 boxes per image (reference 516)");
  static_assert(sizeof(BboxGeom) == 6 * sizeof(int32_t), "geom layout");
  hipError_t e = launch_bbox_labels(boxes, cids, box_off, (const BboxGeom*)geom, n, H, W, out,
                                    (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_bbox_labels");
}

int seg_tag_labels(const float* tags, int n, int H, int W, float* out, void* stream) {
  if (n < 0 || H <= 0 || W <= 0 || (n > 0 && (!tags || !out)))
    return set_err(nullptr, -EINVAL, "seg_tag_labels: bad arguments");
  hipError_t e = launch_tag_labels(tags, n, H, W, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_tag_labels");
}

int seg_prepare_images(const uint8_t* raw, int n, int src_h, int src_w, int H, int W, float* out,
                       void* stream) {
  if (n < 0 || src_h <= 0 || src_w <= 0 || H <= 0 || W <= 0 || (n > 0 && (!raw || !out)))
    return set_err(nullptr, -EINVAL, "seg_prepare_images: bad arguments");
  hipError_t e = launch_prepare_images(raw, n, src_h, src_w, H, W, 0, 0, H, W, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_prepare_images");
}

int seg_prepare_images_crop(const uint8_t* raw, int n, int src_h, int src_w, int resized_h,
                            int resized_w, int crop_y, int crop_x, int H, int W, float* out,
                            void* stream) {
  if (n < 0 || src_h <= 0 || src_w <= 0 || H <= 0 || W <= 0 || (n > 0 && (!raw || !out)) ||
      crop_y < 0 || crop_x < 0 || crop_y + H > resized_h || crop_x + W > resized_w)
    return set_err(nullptr, -EINVAL, "seg_prepare_images_crop: bad arguments (window %d,%d + %dx%d "
                   "outside the resized %dx%d)", crop_y, crop_x, H, W, resized_h, resized_w);
  hipError_t e = launch_prepare_images(raw, n, src_h, src_w, resized_h, resized_w, crop_y, crop_x,
                                       H, W, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_prepare_images_crop");
}

int seg_prepare_labels(const uint8_t* raw, int n, int src_h, int src_w, int H, int W,
                       const int32_t* lids2cids, int n_lids, int32_t* out, void* stream) {
  if (n < 0 || src_h <= 0 || src_w <= 0 || H <= 0 || W <= 0 || (n > 0 && (!raw || !out)) ||
      !lids2cids || n_lids <= 0 || n_lids > SEG_MAX_LIDS)
    return set_err(nullptr, -EINVAL, "seg_prepare_labels: bad arguments");
  LidMap m{};
  m.n = n_lids;
  int mx = -1;
  for (int i = 0; i < n_lids; ++i) mx = std::max(mx, (int)lids2cids[i]);
  for (int i = 0; i < n_lids; ++i)   // utils._replacevoids: -1 -> max + 1
    m.cid[i] = lids2cids[i] == -1 ? mx + 1 : lids2cids[i];
  hipError_t e = launch_prepare_labels(raw, n, src_h, src_w, H, W, m, out, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_prepare_labels");
}

int seg_debug_tensor(seg_ctx* c, const char* name, void** ptr, int* dims, int* ld, int* dtype) {
  if (!c || !name) return set_err(c ? &c->err : nullptr, -EINVAL, "null argument");
  if (c->stem_pending)   // the caller reads on its own stream: a deferred stem gradient first
    HIPCALL(c, hipEventSynchronize(c->ev_join));
  std::string n(name);
  Act a;
  int dt = c->dt == SEG_BF16 ? SEG_DTYPE_BF16 : (c->dt == SEG_F16 ? SEG_DTYPE_F16 : SEG_DTYPE_F32);
  if (n == "logits") { a = c->logits; dt = SEG_DTYPE_F32; }
  else if (n == "head_in") { a = c->logits; a.p = (void*)c->head_in; dt = SEG_DTYPE_F32; }
  else if (n == "grad_un") { a = c->logits; a.p = c->grad_un; dt = SEG_DTYPE_F32; }
  else if (n == "dzscale") { a.p = c->dzscale; a.N = a.H = a.W = 1; a.C = a.ld = c->ldl; dt = SEG_DTYPE_F32; }
  else if (n == "feat") a = c->feat;
  else if (n == "dfeat") a = c->dfeat;
  else if (n == "z0") {   // stem BN + ReLU output (the max-pool input)
    if (c->z0_stale) {   // fused forward: materialise it (same kernel, this step's statistics)
      HIPCALL(c, hipDeviceSynchronize());   // the step's streams may be non-blocking
      Step S{c, nullptr, c->dt};
      if (int r = bn_apply(S, c->stem, c->z0, 0)) return r;
      HIPCALL(c, hipStreamSynchronize(nullptr));
      c->z0_stale = false;
    }
    a = c->z0;
  }
  else if (n.rfind("pyr", 0) == 0 && n.size() == 6 && n.substr(4) == "_z") {
    // a pyramid branch's BN + ReLU output at its pooled resolution (PSP: grids 1, 2, 3, 6;
    // ASPP: 0 = the image pool), the input of its align-corners resize into the concat
    const int b = n[3] - '0';
    if (b < 0 || b >= (int)c->zb.size() || !c->zb[b].p) return set_err(&c->err, -EINVAL, "bad pyramid branch");
    a = c->zb[b];
  }
  else if (n.rfind("head", 0) == 0 && n.size() > 5) {
    int h = n[4] - '0';
    if (h < 0 || h > 2) return set_err(&c->err, -EINVAL, "bad head");
    if (n.substr(5) == "_out") a = c->heads[h].out;
    else if (n.substr(5) == "_dout") a = c->heads[h].dout;
    else return set_err(&c->err, -EINVAL, "unknown tensor %s", name);
  } else if (n.rfind("conv", 0) == 0) {
    size_t us = n.find('_');
    int i = atoi(n.substr(4, us - 4).c_str());
    if (i < 0 || i >= (int)c->convs.size() || us == std::string::npos) return set_err(&c->err, -EINVAL, "bad conv");
    if (n.substr(us) == "_x" && i == c->stem && c->stem_s2d) {
      // the stem reads the space-to-depth image: present the [N][H][W][8] view of it
      const ConvL& st = c->convs[c->stem];
      if (!c->img_dbg) {
        char* p;
        if (int r = dalloc(c, &p, (size_t)st.N * st.H * st.W * 8 * 2)) return r;
        c->img_dbg = p;
      }
      HIPCALL(c, hipDeviceSynchronize());   // the s2d image is written on the step's stream
      HIPCALL(c, launch_unshuffle_s2d(c->img.p, c->img_dbg, st.N, st.H, st.W, c->img.H, c->img.W,
                                      st.pad_h, st.pad_w, 0));
      HIPCALL(c, hipDeviceSynchronize());
      a.p = c->img_dbg; a.N = st.N; a.H = st.H; a.W = st.W; a.C = 3; a.ld = 8;
    } else if (n.substr(us) == "_x") a = c->convs[i].x;
    else if (n.substr(us) == "_y") a = c->convs[i].y;
    else if (n.substr(us) == "_dy") {
      ConvL& L = c->convs[i];
      if (L.lbf_done && !L.lbf_dy_ready) {   // folded (lbf.h): the step never wrote it; the apply it replaced, now
        HIPCALL(c, hipDeviceSynchronize());
        BnBwdArgs b{};
        b.dz = L.lbf_dyhat.p; b.lddz = L.lbf_dyhat.ld;
        b.y = L.y.p; b.ldy = L.y.ld; b.M = L.y.M(); b.C = L.co;
        b.mean = L.st.mean; b.invstd = L.st.invstd; b.scale = L.st.scale;
        b.sdy = L.st.sdy; b.sdyx = L.st.sdyx;
        b.dy = L.dy.p; b.lddy = L.dy.ld;
        HIPCALL(c, launch_bn_bwd_apply(c->dt, 0, b, nullptr));
        HIPCALL(c, hipDeviceSynchronize());
        L.lbf_dy_ready = true;
      }
      a = L.dy;
    }
    else if (n.substr(us) == "_dyhat" && c->convs[i].lbf_done) a = c->convs[i].lbf_dyhat;
    else if (n.substr(us) == "_lbfcoef" && c->convs[i].lbf_done) {   // [3][co] = A, B, D (lbf.h)
      a.p = c->convs[i].lbf_coef; a.N = 1; a.H = 1; a.W = 3; a.C = a.ld = c->convs[i].co;
      dt = SEG_DTYPE_F32;
    }
    else return set_err(&c->err, -EINVAL, "unknown tensor %s", name);
  } else {
    return set_err(&c->err, -EINVAL, "unknown tensor %s", name);
  }
  if (ptr) *ptr = a.p;
  if (dims) { dims[0] = a.N; dims[1] = a.H; dims[2] = a.W; dims[3] = a.C; }
  if (ld) *ld = a.ld;
  if (dtype) *dtype = dt;
  return 0;
}

int seg_profile(seg_ctx* c, int enable) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  if (enable && c->prof.ev.empty()) {
    c->prof.ev.resize(16384);
    for (auto& ev : c->prof.ev) HIPCALL(c, hipEventCreate(&ev));
  }
  c->prof.on = enable != 0;
  c->prof.recs.clear();
  c->prof.next = 0;
  return 0;
}

int seg_profile_read(seg_ctx* c, int cls, double* ms_total, double* gflop_total,
                     int64_t* launches, double* ms_max_layer, char* layer_name, int name_len) {
  if (!c) return set_err(nullptr, -EINVAL, "null ctx");
  double tot = 0, gf = 0;
  int64_t n = 0;
  std::vector<double> per_layer(c->convs.size(), 0.0);
  for (auto& r : c->prof.recs) {
    if (r.cls != cls) continue;
    HIPCALL(c, hipEventSynchronize(c->prof.ev[r.e1]));
    float ms = 0;
    HIPCALL(c, hipEventElapsedTime(&ms, c->prof.ev[r.e0], c->prof.ev[r.e1]));
    tot += ms; gf += r.gflop; ++n;
    per_layer[r.layer] += ms;
  }
  int best = -1;
  for (size_t i = 0; i < per_layer.size(); ++i)
    if (best < 0 || per_layer[i] > per_layer[best]) best = (int)i;
  if (ms_total) *ms_total = tot;
  if (gflop_total) *gflop_total = gf;
  if (launches) *launches = n;
  if (ms_max_layer) *ms_max_layer = best >= 0 ? per_layer[best] : 0;
  if (layer_name && name_len > 0) {
    snprintf(layer_name, name_len, "%s", best >= 0 ? c->convs[best].name.c_str() : "");
  }
  return 0;
}

int seg_profile_dump(seg_ctx* c, char* buf, int len) {
  if (!c || !buf || len <= 0) return set_err(c ? &c->err : nullptr, -EINVAL, "bad argument");
  std::string out;
  char line[512];
  for (auto& r : c->prof.recs) {
    HIPCALL(c, hipEventSynchronize(c->prof.ev[r.e1]));
    float ms = 0;
    HIPCALL(c, hipEventElapsedTime(&ms, c->prof.ev[r.e0], c->prof.ev[r.e1]));
    const ConvL& L = c->convs[r.layer];
    snprintf(line, sizeof(line), "%d %s %d %d %d %d %d %d %.6f %.6f %.6f\n", r.cls, L.name.c_str(),
             L.ci, L.co, L.k, L.rate, L.Ho, L.Wo, r.gflop, (double)ms, r.gbytes);
    out += line;
  }
  snprintf(buf, len, "%s", out.c_str());
  return (int)out.size() >= len ? -ENOSPC : 0;
}

static void op_geom(int H, int W, int k, int stride, int rate, int explicit_pad, int* Ho, int* Wo,
                    int* ph, int* pw) {
  ConvL L;
  L.k = k; L.stride = stride; L.rate = rate; L.explicit_pad = explicit_pad != 0;
  conv_geom(L, 1, H, W);
  *Ho = L.Ho; *Wo = L.Wo; *ph = L.pad_h; *pw = L.pad_w;
}

int seg_op_conv_fwd(int dtype, const void* x, int N, int H, int W, int C, int ldx, const void* w,
                    int Co, int k, int stride, int rate, int explicit_pad, void* y, int ldy,
                    float* stats, void* stream) {
  int Ho, Wo, ph, pw;
  op_geom(H, W, k, stride, rate, explicit_pad, &Ho, &Wo, &ph, &pw);
  ConvArgs a{};
  a.x = x; a.N = N; a.H = H; a.W = W; a.C = C; a.ldx = ldx;
  a.w = w; a.ldw = k * k * C; a.y = y; a.Ho = Ho; a.Wo = Wo; a.Co = Co; a.ldy = ldy;
  a.KH = a.KW = k; a.sf = stride; a.st = 1; a.pad_h = ph; a.pad_w = pw; a.dil = rate; a.stats = stats;
  hipError_t e = launch_conv_nt(dt_of(dtype), 0, a, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_op_conv_fwd");
}

int seg_op_conv_stat_rows(int dtype, int N, int H, int W, int C, int ldx, int Co, int ldy, int k,
                          int stride, int rate, int explicit_pad) {
  int Ho, Wo, ph, pw;   // the ConvArgs seg_op_conv_fwd builds (the kernel choice is shape-dependent)
  op_geom(H, W, k, stride, rate, explicit_pad, &Ho, &Wo, &ph, &pw);
  ConvArgs a{};
  a.N = N; a.H = H; a.W = W; a.C = C; a.ldx = ldx; a.ldw = k * k * C; a.Ho = Ho; a.Wo = Wo;
  a.Co = Co; a.ldy = ldy; a.KH = a.KW = k; a.sf = stride; a.st = 1; a.pad_h = ph; a.pad_w = pw;
  a.dil = rate;
  return conv_nt_stat_rows(dt_of(dtype), 0, a);
}

int seg_op_conv_dgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                      const void* wt, int Ci, int k, int stride, int rate, int explicit_pad, int H,
                      int W, void* dx, int lddx, void* stream) {
  int ho, wo, ph, pw;
  op_geom(H, W, k, stride, rate, explicit_pad, &ho, &wo, &ph, &pw);
  if (ho != Ho || wo != Wo) return set_err(nullptr, -EINVAL, "dgrad geometry mismatch");
  const int keff = k + (k - 1) * (rate - 1);
  ConvArgs a{};
  a.x = dy; a.N = N; a.H = Ho; a.W = Wo; a.C = Co; a.ldx = lddy;
  a.w = wt; a.ldw = k * k * Co; a.y = dx; a.Ho = H; a.Wo = W; a.Co = Ci; a.ldy = lddx;
  a.KH = a.KW = k; a.sf = 1; a.st = stride; a.pad_h = keff - 1 - ph; a.pad_w = keff - 1 - pw;
  a.dil = rate;
  hipError_t e = launch_conv_nt(dt_of(dtype), 0, a, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_op_conv_dgrad");
}

int seg_op_conv_dgrad_res(int dtype, const void* dy, int N, int H, int W, int Co, int lddy,
                          const void* wt, int Ci, void* dx, int lddx, const void* r, int ldr,
                          const uint8_t* omask, void* stream) {
  if (!r && !omask) return set_err(nullptr, -EINVAL, "dgrad_res: a residual or a mask is required");
  if (omask && Ci % 8) return set_err(nullptr, -EINVAL, "dgrad_res: masked outputs need Ci %% 8 == 0");
  ConvArgs a{};
  a.x = dy; a.N = N; a.H = H; a.W = W; a.C = Co; a.ldx = lddy;
  a.w = wt; a.ldw = Co; a.y = dx; a.Ho = H; a.Wo = W; a.Co = Ci; a.ldy = lddx;
  a.KH = a.KW = 1; a.sf = 1; a.st = 1; a.dil = 1;
  if (r) { a.r = r; a.ldr = ldr; }
  if (omask) { a.omask = omask; a.ldm = Ci / 8; }
  hipError_t e = launch_conv_nt(dt_of(dtype), 0, a, (hipStream_t)stream);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_op_conv_dgrad_res");
}

int seg_op_conv_wgrad(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                      const void* x, int H, int W, int Ci, int ldx, int k, int stride, int rate,
                      int explicit_pad, float* dw, void* workspace, int64_t ws_bytes, void* stream) {
  int ho, wo, ph, pw;
  op_geom(H, W, k, stride, rate, explicit_pad, &ho, &wo, &ph, &pw);
  if (ho != Ho || wo != Wo) return set_err(nullptr, -EINVAL, "wgrad geometry mismatch");
  WgradArgs a{};
  a.dy = dy; a.lddy = lddy; a.x = x; a.N = N; a.H = H; a.W = W; a.C = Ci; a.ldx = ldx;
  a.Ho = Ho; a.Wo = Wo; a.Co = Co; a.KH = a.KW = k; a.sf = stride; a.pad_h = ph; a.pad_w = pw;
  a.dil = rate; a.splits = wgrad_splits(a, dt_of(dtype));
  const long n = (long)Co * k * k * Ci;
  if ((int64_t)a.splits * n * 4 > ws_bytes) a.splits = (int)std::max<int64_t>(1, ws_bytes / (n * 4));
  a.out = (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = launch_conv_wgrad(dt_of(dtype), a, s);
  if (e == hipSuccess) e = launch_splitk_reduce((float*)workspace, a.splits, n, n, dw, 0, s);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_op_conv_wgrad");
}

int seg_op_conv_wgrad_cfg(int dtype, const void* dy, int N, int Ho, int Wo, int Co, int lddy,
                          const void* x, int H, int W, int Ci, int ldx, int k, int stride, int rate,
                          int explicit_pad, float* dw, void* workspace, int64_t ws_bytes, int bm,
                          int bn, int splits, void* stream) {
  if (dtype != SEG_DTYPE_BF16 && dtype != SEG_DTYPE_F16)
    return set_err(nullptr, -EINVAL, "wgrad_cfg: 16-bit dtypes only");
  if ((bm != 64 && bm != 128 && bm != 256) || (bn != 64 && bn != 128 && bn != 256) || splits < 1)
    return set_err(nullptr, -EINVAL, "wgrad_cfg: tile must be 64/128/256, splits >= 1");
  int ho, wo, ph, pw;
  op_geom(H, W, k, stride, rate, explicit_pad, &ho, &wo, &ph, &pw);
  if (ho != Ho || wo != Wo) return set_err(nullptr, -EINVAL, "wgrad geometry mismatch");
  WgradArgs a{};
  a.dy = dy; a.lddy = lddy; a.x = x; a.N = N; a.H = H; a.W = W; a.C = Ci; a.ldx = ldx;
  a.Ho = Ho; a.Wo = Wo; a.Co = Co; a.KH = a.KW = k; a.sf = stride; a.pad_h = ph; a.pad_w = pw;
  a.dil = rate; a.splits = splits;
  const long n = (long)Co * k * k * Ci;
  if ((int64_t)splits * n * 4 > ws_bytes) return set_err(nullptr, -EINVAL, "wgrad_cfg: workspace");
  if (!conv_wgrad_v2_ok(a)) return set_err(nullptr, -EINVAL, "wgrad_cfg: shape not on the v2 path");
  a.out = (float*)workspace;
  hipStream_t s = (hipStream_t)stream;
  hipError_t e = launch_conv_wgrad_v2_tile(dt_of(dtype), a, bm, bn, s);
  if (e == hipSuccess) e = launch_splitk_reduce((float*)workspace, splits, n, n, dw, 0, s);
  return e == hipSuccess ? 0 : hip_fail(nullptr, e, "seg_op_conv_wgrad_cfg");
}

}  // extern "C"

// ---- checkpoint interop: CRC-32C (Castagnoli) of host bytes, the checksum TF 1.12 tensor
// bundles store per tensor and per table block (tensorflow/core/lib/hash/crc32c.h), used by
// utils/tf_checkpoint.py to read / write <prefix>.index + <prefix>.data-* checkpoints
namespace {
struct Crc32cTables {
  uint32_t t[8][256];
  Crc32cTables() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
  }
};
const Crc32cTables& crc_tables() {
  static const Crc32cTables tb;
  return tb;
}
}  // namespace

extern "C" uint32_t seg_crc32c(uint32_t crc, const void* data, size_t n) {
  const uint32_t(*t)[256] = crc_tables().t;
  const uint8_t* p = (const uint8_t*)data;
  uint32_t c = ~crc;
  while (n >= 8) {   // slicing-by-8
    uint32_t lo, hi;
    memcpy(&lo, p, 4);
    memcpy(&hi, p + 4, 4);
    lo ^= c;
    c = t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
        t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = t[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
  return ~c;
}

"""One full training step driven from C: a C program that includes only
include/seg_hip.h (plus HIP's C runtime API for its own device buffers) creates a context,
binds caller-owned buffers, uploads the parameters, runs seg_forward -> seg_loss ->
seg_backward -> seg_apply_update on its own stream and prints the loss terms; they, the
regularisation value and the updated parameters / momentum / moving statistics must be
BITWISE equal to the same step run through the Python/ctypes wrapper (seg_hip.SegContext).

Reference binding point: the plugin surface that system_factory.py:178-187 binds
(define_estimator -> model_fn / define_losses / create_train_op); the C consumer is the step
a non-Python host would run through the same library.

The consumer runs as a fresh child process (never an exec of this GPU-initialised process),
after the Python context has been destroyed."""
import os
import struct
import subprocess

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER_DIR = os.path.join(REPO, "include")
LIBDIR = os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")

H, W, NPP, NPB = 64, 128, 1, 1
LR, MOM = 0.01, 0.9

C_SRC = r"""
#include "seg_hip.h"
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x) do { int rc_ = (int)(x); if (rc_ != 0) { \
  fprintf(stderr, "%s:%d %s -> %d (%s)\n", __FILE__, __LINE__, #x, rc_, seg_last_error(ctx)); \
  return 1; } } while (0)

static void* read_file(const char* dir, const char* name, size_t bytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "rb");
  if (!f) return NULL;
  void* p = malloc(bytes);
  size_t got = fread(p, 1, bytes, f);
  fclose(f);
  if (got != bytes) { free(p); return NULL; }
  return p;
}

static int write_file(const char* dir, const char* name, const void* p, size_t bytes) {
  char path[4096];
  snprintf(path, sizeof path, "%s/%s", dir, name);
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  size_t put = fwrite(p, 1, bytes, f);
  fclose(f);
  return put != bytes;
}

static void* upload(const void* host, size_t bytes) {
  void* d = NULL;
  if (hipMalloc(&d, bytes) != hipSuccess) return NULL;
  if (hipMemcpy(d, host, bytes, hipMemcpyHostToDevice) != hipSuccess) return NULL;
  return d;
}

int main(int argc, char** argv) {
  seg_ctx* ctx = NULL;
  if (argc != 7) { fprintf(stderr, "usage: dir H W nb_pp nb_pb lr\n"); return 2; }
  const char* dir = argv[1];
  const int H = atoi(argv[2]), W = atoi(argv[3]), npp = atoi(argv[4]), npb = atoi(argv[5]);
  const float lr = (float)atof(argv[6]);
  const int N = npp + npb;

  seg_cfg cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.depth = 50; cfg.pyramid = SEG_PYRAMID_NONE; cfg.height = H; cfg.width = W;
  cfg.nb_pp = npp; cfg.nb_pb = npb; cfg.nb_pi = 0; cfg.dtype = SEG_DTYPE_F32;
  cfg.dataset = SEG_DATASET_CITYSCAPES; cfg.output_stride = 8; cfg.feature_dims = 256;
  cfg.bn_decay = 0.9f; cfg.train_bn = 1; cfg.weight_decay = 0.00017f;
  cfg.upsampling = SEG_UPSAMPLING_BILINEAR; cfg.norm = SEG_NORM_BATCH;
  CK(hipSetDevice(0));
  CK(seg_create(0, &cfg, &ctx));

  int64_t n_train = 0, n_decay = 0, n_moving = 0, n_stats = 0;
  CK(seg_sizes(ctx, &n_train, &n_decay, &n_moving, &n_stats));
  float* params_h = (float*)read_file(dir, "params.f32", (size_t)n_train * 4);
  float* moving_h = (float*)read_file(dir, "moving.f32", (size_t)n_moving * 4);
  float* images_h = (float*)read_file(dir, "images.f32", (size_t)N * H * W * 3 * 4);
  int32_t* px_h = (int32_t*)read_file(dir, "px.i32", (size_t)npp * H * W * 4);
  float* bbox_h = (float*)read_file(dir, "bbox.f32", (size_t)npb * H * W * 15 * 4);
  if (!params_h || !moving_h || !images_h || !px_h || !bbox_h) {
    fprintf(stderr, "input files missing or of the wrong size\n");
    return 3;
  }
  /* caller-owned device buffers (the context never allocates them) */
  float* params = (float*)upload(params_h, (size_t)n_train * 4);
  float* moving = (float*)upload(moving_h, (size_t)n_moving * 4);
  float *grads = NULL, *momentum = NULL;
  CK(hipMalloc((void**)&grads, (size_t)(n_train + n_stats) * 4));
  CK(hipMalloc((void**)&momentum, (size_t)n_train * 4));
  CK(hipMemset(grads, 0, (size_t)(n_train + n_stats) * 4));
  CK(hipMemset(momentum, 0, (size_t)n_train * 4));
  float* images = (float*)upload(images_h, (size_t)N * H * W * 3 * 4);
  int32_t* px = (int32_t*)upload(px_h, (size_t)npp * H * W * 4);
  float* bbox = (float*)upload(bbox_h, (size_t)npb * H * W * 15 * 4);
  if (!params || !moving || !images || !px || !bbox) { fprintf(stderr, "upload\n"); return 4; }

  hipStream_t s;
  CK(hipStreamCreate(&s));
  CK(seg_bind_buffers(ctx, params, grads, momentum, NULL, moving));
  CK(seg_params_updated(ctx, s));
  /* one training step: forward -> fused loss head -> backward -> SGDM + L2 + BN moving averages */
  CK(seg_forward(ctx, images, s));
  CK(seg_loss(ctx, px, bbox, NULL, NULL, s));
  CK(seg_backward(ctx, s));
  CK(seg_apply_update(ctx, lr, 0.9f, 0.0f, 1.0f, s));
  CK(hipStreamSynchronize(s));

  const float *losses_d = NULL, *reg_d = NULL, *logits_d = NULL;
  int ld = 0, hl = 0, wl = 0;
  CK(seg_outputs(ctx, &losses_d, &reg_d, &logits_d, &ld, &hl, &wl));
  float losses[10], reg = 0.f;
  CK(hipMemcpy(losses, losses_d, sizeof losses, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&reg, reg_d, sizeof reg, hipMemcpyDeviceToHost));
  for (int i = 0; i < 10; ++i) {
    unsigned u;
    memcpy(&u, &losses[i], 4);
    printf("loss %d %08x %.9g\n", i, u, losses[i]);
  }
  { unsigned u; memcpy(&u, &reg, 4); printf("reg %08x %.9g\n", u, reg); }

  float* out = (float*)malloc((size_t)n_train * 4);
  CK(hipMemcpy(out, params, (size_t)n_train * 4, hipMemcpyDeviceToHost));
  if (write_file(dir, "params_after.f32", out, (size_t)n_train * 4)) return 5;
  CK(hipMemcpy(out, momentum, (size_t)n_train * 4, hipMemcpyDeviceToHost));
  if (write_file(dir, "momentum_after.f32", out, (size_t)n_train * 4)) return 5;
  float* mv = (float*)malloc((size_t)n_moving * 4);
  CK(hipMemcpy(mv, moving, (size_t)n_moving * 4, hipMemcpyDeviceToHost));
  if (write_file(dir, "moving_after.f32", mv, (size_t)n_moving * 4)) return 5;
  CK(seg_destroy(ctx));
  ctx = NULL;
  hipFree(params); hipFree(moving); hipFree(grads); hipFree(momentum);
  hipFree(images); hipFree(px); hipFree(bbox);
  CK(hipStreamDestroy(s));
  printf("ok\n");
  return 0;
}
"""


def _hex(v: float) -> str:
    """The C side's printf("%08x") of the float's bits."""
    return "%08x" % struct.unpack("<I", struct.pack("<f", v))[0]


def test_c_consumer_runs_a_training_step_bitwise(cuda, tmp_path):
    from input_pipelines.synthetic import batch
    from oracle.tfseg import SegConfig, init_params
    from seg_hip import SegContext

    lib = os.path.join(LIBDIR, "libseg_hip.so")
    assert os.path.exists(lib), "libseg_hip.so is not built"
    exe = tmp_path / "c_step"
    src = tmp_path / "c_step.c"
    src.write_text(C_SRC)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__",
                    "-I", HEADER_DIR, "-I", "/opt/rocm/include", str(src), "-o", str(exe),
                    "-L", LIBDIR, "-lseg_hip", "-L", "/opt/rocm/lib", "-lamdhip64",
                    f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"], check=True, timeout=120)

    # the same step through the ctypes wrapper
    cfg = SegConfig(height=H, width=W, nb_pp=NPP, nb_pb=NPB, nb_pi=0, pyramid="none")
    p0 = {k: v.astype(np.float32) for k, v in init_params(cfg, seed=3).items()}
    d = batch(7, NPP, NPB, 0, H, W)
    dev = torch.device("cuda", 0)
    ctx = SegContext(pyramid="none", height=H, width=W, nb_pp=NPP, nb_pb=NPB, dtype="fp32")
    ctx.load_params(p0)
    torch.cuda.synchronize()
    ctx.params.cpu().numpy().tofile(tmp_path / "params.f32")
    ctx.moving.cpu().numpy().tofile(tmp_path / "moving.f32")
    np.ascontiguousarray(d["images"], np.float32).tofile(tmp_path / "images.f32")
    np.ascontiguousarray(d["px"], np.int32).tofile(tmp_path / "px.i32")
    np.ascontiguousarray(d["bbox"], np.float32).tofile(tmp_path / "bbox.f32")
    ctx.forward(torch.as_tensor(d["images"]).to(dev))
    ctx.loss(torch.as_tensor(d["px"]).to(dev), torch.as_tensor(d["bbox"]).to(dev))
    ctx.backward()
    ctx.apply_update(LR, MOM)
    torch.cuda.synchronize()
    losses, reg, _ = ctx.outputs()
    py_losses = losses.cpu().numpy().astype(np.float32).copy()
    py_reg = float(reg.cpu().numpy()[0])
    py_params = ctx.params.cpu().numpy().copy()
    py_mom = ctx.momentum.cpu().numpy().copy()
    py_moving = ctx.moving.cpu().numpy().copy()
    ctx.close()
    torch.cuda.synchronize()

    out = subprocess.run([str(exe), str(tmp_path), str(H), str(W), str(NPP), str(NPB), repr(LR)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    lines = out.stdout.split("\n")
    assert "ok" in lines, out.stdout
    c_losses = {}
    for ln in lines:
        f = ln.split()
        if f and f[0] == "loss":
            c_losses[int(f[1])] = f[2]
        elif f and f[0] == "reg":
            c_reg = f[1]
    assert [c_losses[i] for i in range(10)] == [_hex(float(v)) for v in py_losses], \
        (out.stdout, py_losses)
    assert c_reg == _hex(py_reg), (c_reg, py_reg)
    assert py_losses[0] > 0 and py_losses[4] > 0   # a real loss over real pixel counts
    for name, ref in (("params_after", py_params), ("momentum_after", py_mom),
                      ("moving_after", py_moving)):
        got = np.fromfile(tmp_path / f"{name}.f32", dtype=np.float32)
        assert got.shape == ref.shape and np.array_equal(got.view(np.uint32), ref.view(np.uint32)), name
    assert not np.array_equal(py_params, np.fromfile(tmp_path / "params.f32", dtype=np.float32))

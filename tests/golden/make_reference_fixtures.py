"""Generates tests/golden/reference_fixtures.npz from the REFERENCE's own numpy helpers.

Run in the build container only (it reads /root/reference, which does not exist on the GPU
box). TensorFlow 1.12 is absent; the helpers below are TF-free numpy code, so
the `tensorflow` import of their modules is satisfied with a MagicMock stub — nothing from
TF is executed. Outputs are committed as data (inputs + expected outputs):

  * input_subset_bboxes_v2._generate_rla      (open_images/input_subset_bboxes_v2.py:74-98)
  * input_subset_image_labels._generate_rla   (open_images/input_subset_image_labels.py:73-96)
  * utils.utils._replacevoids                 (utils/utils.py:286-289)
  * utils.utils.print_metrics_from_confusion_matrix (utils/utils.py:385-446)
"""
import io
import json
import os
import sys
from contextlib import redirect_stdout
from unittest import mock

import numpy as np

REF = "/root/reference/code"


def _import_reference():
    for name in ("tensorflow", "tensorflow.python", "tensorflow.python.util",
                 "tensorflow.python.util.deprecation", "tensorflow.image",
                 "tensorflow.contrib", "tensorflow.contrib.slim", "PIL", "PIL.Image"):
        sys.modules.setdefault(name, mock.MagicMock())
    sys.modules["tensorflow.python.util.deprecation"].deprecated = lambda *a, **k: (lambda f: f)
    sys.path.insert(0, REF)
    import input_pipelines.open_images.input_subset_bboxes_v2 as bb
    import input_pipelines.open_images.input_subset_image_labels as il
    import utils.utils as uu
    return bb, il, uu


def main(out=os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_fixtures.npz")):
    bb, il, uu = _import_reference()
    rng = np.random.default_rng(20191009)
    fx = {}
    # --- bbox rasterisation: 8 cases, ragged sizes, 0..12 boxes, overlapping classes ---
    mids = list(bb.mid2cid.keys())
    for case in range(8):
        h, w = int(rng.integers(5, 40)), int(rng.integers(5, 50))
        k = int(rng.integers(0, 13))
        names = [mids[int(i)] for i in rng.integers(0, 14, size=k)]
        if case == 7 and k:
            names[0] = "/m/unknown"  # mid not in mid2cid: ignored by the reference
        a, b = rng.random((k, 2)).astype(np.float32), rng.random((k, 2)).astype(np.float32)
        coords = np.stack([np.minimum(a[:, 0], b[:, 0]), np.maximum(a[:, 0], b[:, 0]),
                           np.minimum(a[:, 1], b[:, 1]), np.maximum(a[:, 1], b[:, 1])], 1)
        rla = bb._generate_rla(b"id", [n.encode() for n in names], coords, np.array([h, w]))
        fx[f"bbox{case}_size"] = np.array([h, w])
        fx[f"bbox{case}_cids"] = np.array([bb.mid2cid.get(n, -1) for n in names], dtype=np.int64)
        fx[f"bbox{case}_coords"] = coords
        fx[f"bbox{case}_rla"] = rla
    # --- image-level tags ---
    for case in range(6):
        k = int(rng.integers(0, 5))
        names = [mids[int(i)] for i in rng.integers(0, 14, size=k)]
        rla = il._generate_rla(b"id", [n.encode() for n in names], np.array([4, 4]))
        fx[f"tag{case}_cids"] = np.array(sorted({bb.mid2cid[n] for n in names}), dtype=np.int64)
        fx[f"tag{case}_rla"] = rla
    # --- _replacevoids on the shipped problem definitions ---
    for ds in ("cityscapes", "vistas"):
        with open(os.path.join(REF, "problem_definitions", ds, "problem01.json")) as f:
            lids2cids = json.load(f)["lids2cids"]
        fx[f"replacevoids_{ds}_in"] = np.array(lids2cids)
        fx[f"replacevoids_{ds}_out"] = np.array(uu._replacevoids(lids2cids))
    # --- eval metrics from confusion matrices (incl. an empty GT row) ---
    for case in range(4):
        cm = rng.integers(0, 500, size=(20, 20)).astype(np.int32)
        if case == 1:
            cm[3, :] = 0
        if case == 2:
            cm[:, 5] = 0
            cm[5, :] = 0
        s = io.StringIO()
        with redirect_stdout(s):
            buf = io.StringIO()
            uu.print_metrics_from_confusion_matrix(cm, printfile=buf)
        vals = buf.getvalue().split()[:3]
        fx[f"cm{case}"] = cm
        fx[f"cm{case}_metrics"] = np.array([float(v) for v in vals])
    np.savez_compressed(out, **fx)
    print("wrote", out, len(fx), "arrays")


if __name__ == "__main__":
    main()

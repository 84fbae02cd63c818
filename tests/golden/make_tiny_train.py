"""Writes tests/golden/tiny_train/: a tiny real-data training set in the reference's formats, for
the real-data TRAIN path (input_pipelines/train_inputs.py) — generated data, no reference code:

* cityscapes.tfrecord: 4 tf.train.Example records (KEYS2FEATURES_v5: image/label PNGs + paths,
  input_cityscapes.py:25-36), 96 x 192 images, Cityscapes label ids in blocks (void ids included);
* bboxes.json + images/<id>.jpg: OpenImages-style box index (mid, (xmin, xmax, ymin, ymax)),
  images of three sizes, some unknown mids and one image without boxes;
* tags.json: image-level mids for the same images (one with none).

python tests/golden/make_tiny_train.py   (deterministic; seed 7)"""
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "iv2019-boosting-semantic-segmentation-with-weak-labels_amd")]

OUT = os.path.join(HERE, "tiny_train")
MIDS = ['/m/0199g', '/m/01bjv', '/m/0k4j', '/m/04_sv', '/m/07jdr', '/m/07r04', '/m/01g317',
        '/m/04yx4', '/m/03bt1vf', '/m/01bl7v', '/m/05r655', '/m/015qff', '/m/01mqdt', '/m/02pv19']


def smooth_image(rng, h, w):
    """Low-frequency colour field (compresses well; bilinear resizes exercise fractions)."""
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    img = np.zeros((h, w, 3), np.float32)
    for c in range(3):
        a, b, p, q = rng.uniform(0.02, 0.2, 4)
        img[..., c] = 127.5 + 60 * np.sin(a * yy + p * 7) + 60 * np.cos(b * xx + q * 5)
    img += rng.integers(-6, 7, img.shape)
    return np.clip(img, 0, 255).astype(np.uint8)


def main():
    from PIL import Image
    from input_pipelines.tfrecords import encode_example, encode_png, write_records
    rng = np.random.default_rng(7)
    os.makedirs(os.path.join(OUT, "images"), exist_ok=True)
    recs = []
    for i in range(4):
        img = smooth_image(rng, 96, 192)
        lab = np.kron(rng.integers(0, 34, (6, 12)), np.ones((16, 16), np.int64)).astype(np.uint8)
        recs.append(encode_example({
            'image/encoded': [encode_png(img)], 'image/format': [b'png'],
            'image/shape': [96, 192, 3], 'image/path': [f'img_{i}.png'.encode()],
            'label/encoded': [encode_png(lab[..., None])], 'label/format': [b'png'],
            'label/shape': [96, 192, 1], 'label/path': [f'lab_{i}.png'.encode()]}))
    write_records(os.path.join(OUT, "cityscapes.tfrecord"), recs)
    boxes, tags = {}, {}
    for i, (h, w) in enumerate([(80, 120), (100, 100), (70, 150), (90, 200)]):
        iid = f"oi_{i:03d}"
        buf = io.BytesIO()
        Image.fromarray(smooth_image(rng, h, w)).save(buf, "JPEG", quality=90)
        with open(os.path.join(OUT, "images", iid + ".jpg"), "wb") as f:
            f.write(buf.getvalue())
        k = 0 if i == 1 else int(rng.integers(2, 7))
        bl = []
        for _ in range(k):
            a, b = np.sort(rng.uniform(0, 1, 2)), np.sort(rng.uniform(0, 1, 2))
            mid = MIDS[int(rng.integers(len(MIDS)))] if rng.uniform() > 0.15 else '/m/unknown'
            bl.append([mid, [round(float(a[0]), 4), round(float(a[1]), 4),
                             round(float(b[0]), 4), round(float(b[1]), 4)]])
        boxes[iid] = bl
        tags[iid] = [] if i == 2 else sorted({MIDS[int(j)] for j in rng.integers(0, 14, 3)})
    with open(os.path.join(OUT, "bboxes.json"), "w") as f:
        json.dump(boxes, f, indent=0, sort_keys=True)
    with open(os.path.join(OUT, "tags.json"), "w") as f:
        json.dump(tags, f, indent=0, sort_keys=True)


if __name__ == "__main__":
    main()

"""TFRecord input without TensorFlow: the reference's Cityscapes /
Vistas readers (input_pipelines/cityscapes/input_cityscapes.py:25-96,190-240) as

  host:   TFRecord framing -> tf.train.Example (KEYS2FEATURES_v5,
          utils/keys2features_specs_v5.py:8-19) -> PNG decode (PIL, on the CPU like
          tf.image.decode_png) -> one pinned uint8 batch copied to the device
  device: seg_prepare_images / seg_prepare_labels (csrc/input.hip): convert_image_dtype,
          bilinear resize (align_corners = False), from_0_1_to_m1_1; lids2cids gather and
          nearest resize — producing ``proimages`` / ``prolabels`` in HBM.

TFRecord framing: uint64 length, uint32 masked CRC-32C of the length bytes, the record,
uint32 masked CRC-32C of the record (tensorflow/core/lib/io/record_writer.cc). No TF-written
file is available here: reading one is parity unpinned beyond the published format; the
tests pin the writer/reader round trip and the CRC known answers.
"""
from __future__ import annotations

import io
import struct
from typing import Dict, Iterator, List, Tuple

import numpy as np

from utils.tf_checkpoint import (_fields, _key, _read_varint, _varint, crc32c, mask_crc,
                                 unmask_crc)


# ---- TFRecord framing ---------------------------------------------------------------------
def read_records(path: str, verify: bool = True) -> Iterator[bytes]:
    with open(path, 'rb') as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise ValueError(f'{path}: truncated record header')
            n, lcrc = struct.unpack('<QI', head)
            if verify and unmask_crc(lcrc) != crc32c(head[:8]):
                raise ValueError(f'{path}: corrupted record length')
            data = f.read(n)
            tail = f.read(4)
            if len(data) < n or len(tail) < 4:
                raise ValueError(f'{path}: truncated record')
            if verify and unmask_crc(struct.unpack('<I', tail)[0]) != crc32c(data):
                raise ValueError(f'{path}: corrupted record data')
            yield data


def write_records(path: str, records: List[bytes]):
    with open(path, 'wb') as f:
        for r in records:
            ln = struct.pack('<Q', len(r))
            f.write(ln + struct.pack('<I', mask_crc(crc32c(ln))) + r +
                    struct.pack('<I', mask_crc(crc32c(r))))


# ---- tf.train.Example ----------------------------------------------------------------------
def parse_example(b: bytes) -> Dict[str, list]:
    """Example{features{feature: map<string, Feature{bytes_list|float_list|int64_list}>}}
    -> name -> list of values (bytes / float / int)."""
    out = {}
    for f, _, feats in _fields(b):
        if f != 1:
            continue
        for g, _, entry in _fields(feats):
            if g != 1:
                continue
            name, vals = None, []
            for h, _, v in _fields(entry):
                if h == 1:
                    name = v.decode()
                elif h == 2:
                    for kind, _, lst in _fields(v):
                        for k, wt, x in _fields(lst):
                            if k != 1:
                                continue
                            if kind == 1:
                                vals.append(bytes(x))
                            elif kind == 2:
                                vals.extend(np.frombuffer(x, '<f4').tolist() if wt == 2
                                            else [struct.unpack('<f', struct.pack('<I', x))[0]])
                            elif kind == 3:
                                if wt == 2:
                                    i = 0
                                    while i < len(x):
                                        u, i = _read_varint(x, i)
                                        vals.append(u - (1 << 64) if u >= 1 << 63 else u)
                                else:
                                    vals.append(x - (1 << 64) if x >= 1 << 63 else x)
            out[name] = vals
    return out


def encode_example(features: Dict[str, list]) -> bytes:
    """The inverse of parse_example (bytes -> bytes_list, float -> float_list, int ->
    int64_list; packed repeated scalars like protobuf's serializer)."""
    def msg(field, payload):
        return _key(field, 2) + _varint(len(payload)) + payload
    entries = b''
    for name in sorted(features):
        vals = list(features[name])
        if vals and isinstance(vals[0], (bytes, bytearray)):
            lst = b''.join(msg(1, bytes(v)) for v in vals)
            feat = msg(1, lst)
        elif vals and isinstance(vals[0], float):
            feat = msg(2, msg(1, np.asarray(vals, '<f4').tobytes()))
        else:
            feat = msg(3, msg(1, b''.join(_varint(int(v)) for v in vals)))
        entries += msg(1, msg(1, name.encode()) + msg(2, feat))
    return msg(1, entries)


# ---- PNG --------------------------------------------------------------------------------------
def decode_png(b: bytes, channels: int = 0) -> np.ndarray:
    """tf.image.decode_png (CPU): uint8 [H, W, C] (C from the file when channels == 0)."""
    from PIL import Image
    im = Image.open(io.BytesIO(b))
    if channels == 3:
        im = im.convert('RGB')
    elif channels == 1:
        im = im.convert('L')
    a = np.asarray(im, dtype=np.uint8)
    return a[..., None] if a.ndim == 2 else a


def encode_png(a: np.ndarray) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(a.squeeze(-1) if a.ndim == 3 and a.shape[-1] == 1 else a).save(buf, 'PNG')
    return buf.getvalue()


def parse_cityscapes_example(b: bytes) -> Tuple[np.ndarray, np.ndarray, bytes, bytes]:
    """_parse_tfexample (input_cityscapes.py:40-64): image uint8 [H,W,3], label ids uint8
    [H,W] (first channel of the decoded label PNG), image and label paths."""
    e = parse_example(b)
    image = decode_png(e['image/encoded'][0])
    label = decode_png(e['label/encoded'][0])[..., 0]
    return image, label, e.get('image/path', [b''])[0], e.get('label/path', [b''])[0]


# ---- device preprocessing ------------------------------------------------------------------------
def prepare_images(raw, H: int, W: int, stream=None):
    """raw: device uint8 [n, h, w, 3] -> fp32 proimages [n, H, W, 3] in [-1, 1)."""
    import torch
    from seg_hip import LIB, _ptr, _stream, check
    assert raw.dtype == torch.uint8 and raw.dim() == 4 and raw.shape[-1] == 3 and raw.is_cuda
    raw = raw.contiguous()
    out = torch.empty((raw.shape[0], H, W, 3), dtype=torch.float32, device=raw.device)
    check(LIB.seg_prepare_images(_ptr(raw), raw.shape[0], raw.shape[1], raw.shape[2], H, W,
                                 _ptr(out), _stream(stream)))
    return out


def prepare_images_crop(raw, resized, offset, H: int, W: int, stream=None):
    """raw: device uint8 [n, h, w, 3] -> bilinear resize to `resized` (h, w) -> the H x W window
    at `offset` (y, x) -> fp32 [n, H, W, 3] in [-1, 1) (the aspect-preserving resize + random
    crop of the weak-label streams, input_pipelines/utils.py:181-241)."""
    import torch
    from seg_hip import LIB, _ptr, _stream, check
    assert raw.dtype == torch.uint8 and raw.dim() == 4 and raw.shape[-1] == 3 and raw.is_cuda
    raw = raw.contiguous()
    out = torch.empty((raw.shape[0], H, W, 3), dtype=torch.float32, device=raw.device)
    check(LIB.seg_prepare_images_crop(_ptr(raw), raw.shape[0], raw.shape[1], raw.shape[2],
                                      int(resized[0]), int(resized[1]), int(offset[0]),
                                      int(offset[1]), H, W, _ptr(out), _stream(stream)))
    return out


def prepare_labels(raw, H: int, W: int, lids2cids, stream=None):
    """raw: device uint8 label ids [n, h, w] -> int32 prolabels [n, H, W] in training cids."""
    import ctypes
    import torch
    from seg_hip import LIB, _ptr, _stream, check
    assert raw.dtype == torch.uint8 and raw.dim() == 3 and raw.is_cuda
    raw = raw.contiguous()
    out = torch.empty((raw.shape[0], H, W), dtype=torch.int32, device=raw.device)
    m = (ctypes.c_int32 * len(lids2cids))(*[int(v) for v in lids2cids])
    check(LIB.seg_prepare_labels(_ptr(raw), raw.shape[0], raw.shape[1], raw.shape[2], H, W, m,
                                 len(lids2cids), _ptr(out), _stream(stream)))
    return out


def tfrecord_input(paths, lids2cids, H: int, W: int, nb: int, device=None, repeat=False):
    """Batches of ({'proimages', 'rawimagespaths'}, {'prolabels'}) from TFRecord files, the
    evaluate_input contract (input_cityscapes.py:217-240; all images of a batch share one
    size, as the reference requires for Nb > 1)."""
    import torch
    dev = device or torch.device('cuda', torch.cuda.current_device())
    paths = [paths] if isinstance(paths, str) else list(paths)
    while True:
        ims, las, ips = [], [], []
        for p in paths:
            for rec in read_records(p):
                im, la, ip, _ = parse_cityscapes_example(rec)
                ims.append(im)
                las.append(la)
                ips.append(ip)
                if len(ims) == nb:
                    raw_i = torch.from_numpy(np.stack(ims)).pin_memory().to(dev, non_blocking=True)
                    raw_l = torch.from_numpy(np.stack(las)).pin_memory().to(dev, non_blocking=True)
                    yield ({'proimages': prepare_images(raw_i, H, W), 'rawimagespaths': ips},
                           {'prolabels': prepare_labels(raw_l, H, W, lids2cids)})
                    ims, las, ips = [], [], []
        if not repeat:
            return

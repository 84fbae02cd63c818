"""TF 1.12 checkpoint interop without TensorFlow.

The reference saves and restores ``tf.train.Saver`` V2 checkpoints (define_savers.py:38-66)
and warm-starts from ImageNet checkpoints such as slim's ``resnet_v1_50.ckpt`` through
``replace_initializers`` (define_initializers.py:72-131). This module reads and writes that
on-disk format (a "tensor bundle") directly:

* ``<prefix>.index``: a LevelDB-format table (tensorflow/core/lib/io/table*.cc): data blocks of
  prefix-compressed (key, value) entries with restart points, a metaindex block, an index
  block of BlockHandles, every block followed by a 1-byte compression type (0 = none,
  1 = snappy) and a masked CRC-32C; a 48-byte footer ending in the magic 0xdb4775248b80fb57.
  Key "" holds a BundleHeaderProto {num_shards, endianness, version}; every other key is a
  tensor name with a BundleEntryProto {dtype, shape, shard_id, offset, size, crc32c}.
* ``<prefix>.data-SSSSS-of-NNNNN``: the raw little-endian tensor bytes.

Conv weights are HWIO in TF ([KH, KW, Ci, Co]) and OHWI in the native context; the conversion
is done here. The CRC-32C runs in libseg_hip.so (``seg_crc32c``, host code).

Parity: the format is restated from TensorFlow's published sources (tensor_bundle.proto,
table_format); no TF-written checkpoint is available in this environment, so reading one is
"parity unpinned" — tests pin the writer/reader round trip and the table/CRC known answers.
"""
from __future__ import annotations

import ctypes
import os
import struct
import warnings
from typing import Dict, Iterable, List, Tuple

import numpy as np

TABLE_MAGIC = 0xdb4775248b80fb57
_MASK_DELTA = 0xa282ead8

# tensorflow/core/framework/types.proto
_DT = {1: np.float32, 2: np.float64, 3: np.int32, 4: np.uint8, 5: np.int16, 6: np.int8,
       9: np.int64, 10: np.bool_, 17: np.uint16, 19: np.float16, 22: np.uint32, 23: np.uint64}
_DT_INV = {np.dtype(v): k for k, v in _DT.items()}


# ---- checksums ----------------------------------------------------------------------------
def crc32c(data, crc: int = 0) -> int:
    """CRC-32C of bytes-like data (libseg_hip.so seg_crc32c, slicing-by-8 host code)."""
    from seg_hip import LIB
    arr = np.frombuffer(data, np.uint8)
    return int(LIB.seg_crc32c(crc, arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes))


def mask_crc(crc: int) -> int:
    return ((((crc >> 15) | (crc << 17)) & 0xFFFFFFFF) + _MASK_DELTA) & 0xFFFFFFFF


def unmask_crc(masked: int) -> int:
    rot = (masked - _MASK_DELTA) & 0xFFFFFFFF
    return ((rot >> 17) | (rot << 15)) & 0xFFFFFFFF


# ---- protobuf wire format (the few messages a bundle uses) --------------------------------
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(b: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        c = b[i]
        i += 1
        v |= (c & 0x7F) << shift
        if not c & 0x80:
            return v, i
        shift += 7


def _fields(b: bytes):
    """(field number, wire type, value) of a serialized message."""
    i = 0
    while i < len(b):
        key, i = _read_varint(b, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = struct.unpack_from('<Q', b, i)[0]
            i += 8
        elif wt == 2:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        elif wt == 5:
            v = struct.unpack_from('<I', b, i)[0]
            i += 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield f, wt, v


def _key(f: int, wt: int) -> bytes:
    return _varint((f << 3) | wt)


def _encode_entry(dtype: int, shape: Iterable[int], shard: int, offset: int, size: int,
                  crc: int) -> bytes:
    dims = b''.join(_key(2, 2) + _varint(len(d)) + d
                    for d in (_key(1, 0) + _varint(int(s)) for s in shape))
    out = _key(1, 0) + _varint(dtype) + _key(2, 2) + _varint(len(dims)) + dims
    if shard:
        out += _key(3, 0) + _varint(shard)
    if offset:
        out += _key(4, 0) + _varint(offset)
    out += _key(5, 0) + _varint(size) + _key(6, 5) + struct.pack('<I', crc)
    return out


def _decode_entry(b: bytes) -> dict:
    e = {'dtype': 0, 'shape': [], 'shard_id': 0, 'offset': 0, 'size': 0, 'crc32c': None}
    for f, _, v in _fields(b):
        if f == 1:
            e['dtype'] = v
        elif f == 2:
            for g, _, dim in _fields(v):
                if g == 2:
                    size = 0
                    for h, _, x in _fields(dim):
                        if h == 1:
                            size = x - (1 << 64) if x >= 1 << 63 else x
                    e['shape'].append(size)
        elif f == 3:
            e['shard_id'] = v
        elif f == 4:
            e['offset'] = v
        elif f == 5:
            e['size'] = v
        elif f == 6:
            e['crc32c'] = v
        elif f == 7:
            raise NotImplementedError('partitioned (sliced) variables are not supported')
    return e


def _encode_header(num_shards: int) -> bytes:
    version = _key(1, 0) + _varint(1)   # VersionDef{producer: kTensorBundleVersion = 1}
    return _key(1, 0) + _varint(num_shards) + _key(3, 2) + _varint(len(version)) + version


# ---- table (LevelDB format) ----------------------------------------------------------------
def _snappy_decompress(b: bytes) -> bytes:
    n, i = _read_varint(b, 0)
    out = bytearray()
    while i < len(b):
        tag = b[i]
        i += 1
        t = tag & 3
        if t == 0:
            ln = tag >> 2
            if ln >= 60:
                nb = ln - 59
                ln = int.from_bytes(b[i:i + nb], 'little')
                i += nb
            ln += 1
            out += b[i:i + ln]
            i += ln
            continue
        if t == 1:
            ln = ((tag >> 2) & 7) + 4
            off = ((tag >> 5) << 8) | b[i]
            i += 1
        elif t == 2:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[i:i + 2], 'little')
            i += 2
        else:
            ln = (tag >> 2) + 1
            off = int.from_bytes(b[i:i + 4], 'little')
            i += 4
        start = len(out) - off
        for k in range(ln):   # copies may overlap their own output
            out.append(out[start + k])
    if len(out) != n:
        raise ValueError('corrupt snappy block')
    return bytes(out)


def _read_block(data: bytes, offset: int, size: int, verify: bool = True) -> bytes:
    contents = data[offset:offset + size]
    ctype = data[offset + size]
    if verify:
        stored = struct.unpack_from('<I', data, offset + size + 1)[0]
        if unmask_crc(stored) != crc32c(data[offset:offset + size + 1]):
            raise ValueError(f'block checksum mismatch at offset {offset}')
    if ctype == 0:
        return contents
    if ctype == 1:
        return _snappy_decompress(contents)
    raise ValueError(f'unknown block compression type {ctype}')


def _block_entries(block: bytes) -> List[Tuple[bytes, bytes]]:
    nrest = struct.unpack_from('<I', block, len(block) - 4)[0]
    end = len(block) - 4 - 4 * nrest
    out, i, last = [], 0, b''
    while i < end:
        shared, i = _read_varint(block, i)
        non_shared, i = _read_varint(block, i)
        vlen, i = _read_varint(block, i)
        key = last[:shared] + block[i:i + non_shared]
        i += non_shared
        out.append((key, block[i:i + vlen]))
        i += vlen
        last = key
    return out


def _handle(b: bytes, i: int = 0) -> Tuple[int, int, int]:
    off, i = _read_varint(b, i)
    size, i = _read_varint(b, i)
    return off, size, i


def read_table(path: str, verify: bool = True) -> List[Tuple[bytes, bytes]]:
    with open(path, 'rb') as f:
        data = f.read()
    if len(data) < 48 or struct.unpack_from('<Q', data, len(data) - 8)[0] != TABLE_MAGIC:
        raise ValueError(f'{path}: not a TF table (bad magic)')
    footer = data[len(data) - 48:]
    _, _, j = _handle(footer)          # metaindex (unused)
    ioff, isize, _ = _handle(footer, j)
    out = []
    for _, h in _block_entries(_read_block(data, ioff, isize, verify)):
        off, size, _ = _handle(h)
        out.extend(_block_entries(_read_block(data, off, size, verify)))
    return out


def _build_block(entries: List[Tuple[bytes, bytes]], restart_interval: int = 16) -> bytes:
    out, restarts, last = bytearray(), [], b''
    for n, (k, v) in enumerate(entries):
        if n % restart_interval == 0:
            restarts.append(len(out))
            shared = 0
        else:
            shared = 0
            while shared < min(len(k), len(last)) and k[shared] == last[shared]:
                shared += 1
        out += _varint(shared) + _varint(len(k) - shared) + _varint(len(v)) + k[shared:] + v
        last = k
    if not restarts:
        restarts = [0]
    for r in restarts:
        out += struct.pack('<I', r)
    out += struct.pack('<I', len(restarts))
    return bytes(out)


def write_table(path: str, entries: List[Tuple[bytes, bytes]], block_bytes: int = 4096):
    """Sorted (key, value) pairs -> an uncompressed table (TF's BundleWriter uses no
    compression for the index file)."""
    entries = sorted(entries)
    out = bytearray()
    index = []

    def emit(block: bytes) -> bytes:
        off = len(out)
        out.extend(block)
        trailer = bytes([0])
        out.extend(trailer + struct.pack('<I', mask_crc(crc32c(block + trailer))))
        return _varint(off) + _varint(len(block))

    cur, cur_size = [], 0
    for k, v in entries:
        cur.append((k, v))
        cur_size += len(k) + len(v) + 8
        if cur_size >= block_bytes:
            index.append((cur[-1][0], emit(_build_block(cur))))
            cur, cur_size = [], 0
    if cur:
        index.append((cur[-1][0], emit(_build_block(cur))))
    meta = emit(_build_block([]))
    idx = emit(_build_block(index, restart_interval=1))
    footer = (meta + idx).ljust(40, b'\0') + struct.pack('<Q', TABLE_MAGIC)
    out.extend(footer)
    with open(path, 'wb') as f:
        f.write(out)


# ---- bundles ---------------------------------------------------------------------------------
def _data_path(prefix: str, shard: int, num_shards: int) -> str:
    return f'{prefix}.data-{shard:05d}-of-{num_shards:05d}'


def list_variables(prefix: str) -> List[Tuple[str, List[int]]]:
    """tf.train.list_variables: sorted (name, shape)."""
    out = []
    for k, v in read_table(prefix + '.index'):
        if k:
            out.append((k.decode(), _decode_entry(v)['shape']))
    return out


def load_checkpoint(prefix: str, names: Iterable[str] = None,
                    verify: bool = True) -> Dict[str, np.ndarray]:
    """name -> ndarray (TF layouts) for every (or the given) tensor of a V2 checkpoint."""
    want = None if names is None else set(names)
    entries = read_table(prefix + '.index', verify)
    num_shards = 1
    for f, _, v in _fields(dict(entries).get(b'', b'')):
        if f == 1:
            num_shards = v
    files, out = {}, {}
    try:
        for k, v in entries:
            if not k or (want is not None and k.decode() not in want):
                continue
            e = _decode_entry(v)
            if e['dtype'] not in _DT:
                raise NotImplementedError(f"{k.decode()}: dtype enum {e['dtype']}")
            sh = e['shard_id']
            if sh not in files:
                files[sh] = open(_data_path(prefix, sh, num_shards), 'rb')
            files[sh].seek(e['offset'])
            raw = files[sh].read(e['size'])
            if verify and e['crc32c'] is not None and unmask_crc(e['crc32c']) != crc32c(raw):
                raise ValueError(f'{k.decode()}: tensor checksum mismatch')
            out[k.decode()] = np.frombuffer(raw, _DT[e['dtype']]).reshape(tuple(e['shape'])).copy()
    finally:
        for f in files.values():
            f.close()
    return out


def save_checkpoint(prefix: str, tensors: Dict[str, np.ndarray]):
    """One-shard V2 checkpoint of named arrays (written in sorted name order like
    BundleWriter), readable by tf.train.load_checkpoint / Saver.restore."""
    os.makedirs(os.path.dirname(os.path.abspath(prefix)), exist_ok=True)
    entries = [(b'', _encode_header(1))]
    off = 0
    with open(_data_path(prefix, 0, 1), 'wb') as f:
        for name in sorted(tensors):
            a = np.asarray(tensors[name]) if np.ndim(tensors[name]) == 0 \
                else np.ascontiguousarray(tensors[name])   # keeps 0-d scalars 0-d
            if a.dtype not in _DT_INV:
                raise TypeError(f'{name}: dtype {a.dtype} not supported')
            raw = a.astype(a.dtype.newbyteorder('<'), copy=False).tobytes()
            f.write(raw)
            entries.append((name.encode(), _encode_entry(_DT_INV[a.dtype], a.shape, 0, off,
                                                         len(raw), mask_crc(crc32c(raw)))))
            off += len(raw)
    write_table(prefix + '.index', entries)


# ---- native context <-> TF variable names ------------------------------------------------------
def _tf_layout(p, arr):
    """native (OHWI weights) -> TF (HWIO)"""
    if p.kind == 'weights':
        return np.ascontiguousarray(arr.reshape(p.shape).transpose(1, 2, 3, 0))
    return arr.reshape(p.shape)


def _native_layout(p, arr):
    if p.kind == 'weights':
        return np.ascontiguousarray(np.asarray(arr).transpose(3, 0, 1, 2))
    return np.asarray(arr)


def tf_shapes(ctx) -> Dict[str, Tuple[int, ...]]:
    """TF variable shapes of the context's parameters (weights HWIO)."""
    out = {}
    for p in ctx.param_info:
        out[p.name] = (p.shape[1], p.shape[2], p.shape[3], p.shape[0]) if p.kind == 'weights' \
            else tuple(p.shape)
    return out


EMA_SCOPE = 'exponential_moving_averages/'


def ema_name(var: str) -> str:
    """TF name of a variable's EMA shadow: ExponentialMovingAverage.apply under
    variable_scope('exponential_moving_averages') (define_estimator_hierarchical.py:96-111),
    the key predict_saver restores with --restore_emas (define_savers.py:44-47)."""
    return EMA_SCOPE + var + '/ExponentialMovingAverage'


def export_checkpoint(ctx, prefix: str, global_step: int = 0):
    """Saver-style checkpoint of the context: every model variable under its TF name, its
    Momentum slot (``<var>/Momentum``), the EMA shadows when kept (``ema_name(var)``) and
    ``global_step`` (int64)."""
    params, mom = ctx.named('params'), ctx.named('momentum')
    ema = ctx.named('ema') if ctx.ema is not None else {}
    out = {'global_step': np.array(global_step, np.int64)}
    for p in ctx.param_info:
        out[p.name] = _tf_layout(p, params[p.name])
        if p.name in mom:
            out[p.name + '/Momentum'] = _tf_layout(p, mom[p.name])
        if p.name in ema:
            out[ema_name(p.name)] = _tf_layout(p, ema[p.name])
    save_checkpoint(prefix, out)


def import_checkpoint(ctx, prefix: str, momentum: bool = True, restore_emas: bool = False) -> int:
    """Restore a checkpoint written with the model's own variable names; returns global_step.

    Training restart (momentum=True): parameters, moving statistics, Momentum slots and, when
    the context keeps them, the EMA shadows. Evaluation / prediction (momentum=False): with
    ``restore_emas`` every variable except the BN moving statistics is read from its EMA
    shadow (predict_saver, define_savers.py:38-66); a missing shadow is an error, as the
    reference's Saver restore would be."""
    import torch
    shapes = tf_shapes(ctx)
    vals = load_checkpoint(prefix)

    def src(p):
        if restore_emas and p.kind not in ('moving_mean', 'moving_variance'):
            return ema_name(p.name)
        return p.name
    missing = [src(p) for p in ctx.param_info if src(p) not in vals]
    if missing:
        raise KeyError(f'{len(missing)} variables missing from {prefix}: {missing[:3]}')
    ctx.load_params({p.name: _native_layout(p, vals[src(p)]) for p in ctx.param_info})

    def fill(buf, *keys):
        hit = 0
        for p in ctx.param_info:
            if p.kind in ('moving_mean', 'moving_variance'):
                continue
            v = next((vals[k(p.name)] for k in keys if k(p.name) in vals), None)
            if v is not None:
                hit += 1
                buf[p.offset:p.offset + p.numel].copy_(
                    torch.as_tensor(_native_layout(p, v).reshape(-1).astype(np.float32)))
        return hit
    if momentum:
        # the reference builds its optimizer inside variable_scope('train_ops')
        # (define_estimator_hierarchical.py:114-117), so its slots may carry that prefix; the
        # slot name is not pinned by any reference artefact (parity unpinned): accept both
        n_slots = fill(ctx.momentum, lambda n: n + '/Momentum', lambda n: 'train_ops/' + n + '/Momentum')
        n_train = sum(p.kind not in ('moving_mean', 'moving_variance') for p in ctx.param_info)
        if n_slots == 0 and n_train:
            warnings.warn(f'{prefix}: no Momentum slot found for {n_train} trainable variables; '
                          'training resumes with zero momentum')
        if ctx.ema is not None:   # after load_params, which reset the shadows to the weights
            fill(ctx.ema, ema_name)
    return int(vals.get('global_step', 0))


def warm_start_map(ckpt_vars: List[Tuple[str, List[int]]], model_vars: List[Tuple[str, tuple]],
                   psp_module: bool) -> Dict[str, str]:
    """checkpoint name -> model name, as replace_initializers builds var_dict
    (define_initializers.py:94-112): a model variable whose name contains an excluded
    substring is skipped; otherwise every checkpoint name that is a SUBSTRING of the model
    name with a compatible shape maps to it (later model variables overwrite earlier ones)."""
    exclude = ['global_step', 'train_ops', 'ExponentialMovingAverage', 'Momentum',
               'classifier', 'extension']
    if not psp_module:
        exclude.append('psp')
    out = {}
    for gname, gshape in model_vars:
        if any(exc in gname for exc in exclude):
            continue
        for cvn, cvs in ckpt_vars:
            if cvn in gname and _compatible(cvs, gshape):
                out[cvn] = gname
    return out


def _compatible(a, b) -> bool:
    return len(a) == len(b) and all(x == y or x < 0 or y < 0 for x, y in zip(a, b))


def warm_start(ctx, prefix: str, psp_module: bool = False) -> Dict[str, str]:
    """--init_ckpt_path: initialise every model variable the mapping reaches (e.g. the
    encoder from slim's ImageNet resnet_v1_50.ckpt); the rest keep their initialisers."""
    shapes = tf_shapes(ctx)
    mapping = warm_start_map(list_variables(prefix),
                             [(p.name, shapes[p.name]) for p in ctx.param_info], psp_module)
    vals = load_checkpoint(prefix, names=mapping.keys())
    by_name = {p.name: p for p in ctx.param_info}
    ctx.load_params({g: _native_layout(by_name[g], vals[c]) for c, g in mapping.items()})
    return mapping

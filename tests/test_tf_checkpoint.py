"""TF 1.12 checkpoint interop (utils/tf_checkpoint.py): CRC-32C / table / snappy known
answers, V2 bundle write -> read round trips, and the warm-start name mapping of
replace_initializers (define_initializers.py:72-131). No TF-written checkpoint exists in
this environment: reading one is parity unpinned beyond the published format."""
import struct

import numpy as np
import pytest


def test_crc32c_known_answers():
    from utils.tf_checkpoint import crc32c, mask_crc, unmask_crc
    assert crc32c(b"123456789") == 0xE3069283          # the CRC-32C check value
    assert crc32c(b"") == 0
    assert crc32c(bytes(32)) == 0x8A9136AA               # RFC 3720 B.4: 32 zero bytes
    assert crc32c(bytes([0xFF] * 32)) == 0x62A8AB43      # RFC 3720 B.4: 32 0xFF bytes
    assert crc32c(bytes(range(32))) == 0x46DD794E        # RFC 3720 B.4: incrementing
    data = np.random.default_rng(0).integers(0, 256, 100003, dtype=np.uint8).tobytes()
    assert crc32c(data[50000:], crc32c(data[:50000])) == crc32c(data)   # streaming
    for c in (0, 1, 0xE3069283, 0xFFFFFFFF):
        assert unmask_crc(mask_crc(c)) == c and mask_crc(c) != c


def test_snappy_known_answer():
    from utils.tf_checkpoint import _snappy_decompress
    # len 12; literal "abc"; copy (1-byte offset) of 9 bytes from offset 3 (overlapping)
    assert _snappy_decompress(bytes([12, 0x08]) + b"abc" + bytes([0x15, 3])) == b"abcabcabcabc"
    # 2-byte-offset copy
    assert _snappy_decompress(bytes([8, 0x0C]) + b"wxyz" + bytes([(4 - 1) << 2 | 2, 4, 0])) == b"wxyzwxyz"


def test_table_round_trip_many_blocks(tmp_path):
    from utils.tf_checkpoint import TABLE_MAGIC, read_table, write_table
    rng = np.random.default_rng(1)
    entries = [(f"scope/{i:05d}/var".encode(), rng.bytes(int(rng.integers(0, 300))))
               for i in range(500)]
    p = str(tmp_path / "t.index")
    write_table(p, entries + [(b"", b"hdr")])
    got = read_table(p)
    assert got == sorted(entries + [(b"", b"hdr")])
    raw = open(p, "rb").read()
    assert struct.unpack_from("<Q", raw, len(raw) - 8)[0] == TABLE_MAGIC
    # a flipped byte in a block is caught by its masked CRC
    bad = bytearray(raw)
    bad[10] ^= 1
    open(p, "wb").write(bytes(bad))
    with pytest.raises(ValueError):
        read_table(p)


def test_bundle_round_trip(tmp_path):
    from utils.tf_checkpoint import list_variables, load_checkpoint, save_checkpoint
    rng = np.random.default_rng(2)
    t = {"feature_extractor/base/resnet_v1_50/conv1/weights":
         rng.standard_normal((7, 7, 3, 64)).astype(np.float32),
         "feature_extractor/base/resnet_v1_50/conv1/BatchNorm/gamma":
         rng.standard_normal(64).astype(np.float32),
         "global_step": np.array(1234, np.int64),
         "some/int": np.arange(10, dtype=np.int32).reshape(2, 5),
         "some/double": rng.standard_normal((3,)),
         "some/empty": np.zeros((0, 4), np.float32)}
    pre = str(tmp_path / "model.ckpt-1234")
    save_checkpoint(pre, t)
    assert [n for n, _ in list_variables(pre)] == sorted(t)
    assert dict(list_variables(pre))["feature_extractor/base/resnet_v1_50/conv1/weights"] == [7, 7, 3, 64]
    back = load_checkpoint(pre)
    for k, v in t.items():
        assert back[k].dtype == v.dtype and back[k].shape == v.shape
        np.testing.assert_array_equal(back[k], v)
    # tensor bytes are checksummed
    with open(pre + ".data-00000-of-00001", "r+b") as f:
        f.seek(5)
        b = f.read(1)
        f.seek(5)
        f.write(bytes([b[0] ^ 0x40]))
    with pytest.raises(ValueError):
        load_checkpoint(pre)


def _model_vars(cfg):
    from oracle.tfseg import build_specs
    out = []
    for s in build_specs(cfg):
        out.append((f"{s.name}/weights", (s.k, s.k, s.ci, s.co)))
        for b in ("beta", "gamma", "moving_mean", "moving_variance"):
            out.append((f"{s.name}/BatchNorm/{b}", (s.co,)))
    return out


def test_warm_start_map_imagenet_like():
    """A slim ImageNet resnet_v1_50 checkpoint (names without the feature_extractor/base/
    prefix, plus its 1000-way logits and global_step) initialises exactly the encoder."""
    from oracle.tfseg import SegConfig
    from utils.tf_checkpoint import warm_start_map
    cfg = SegConfig(height=64, width=128, nb_pp=1, pyramid="psp")
    model = _model_vars(cfg)
    pre = "feature_extractor/base/"
    ckpt = [(n[len(pre):], list(s)) for n, s in model if n.startswith(pre)]
    ckpt += [("resnet_v1_50/logits/weights", [1, 1, 2048, 1000]),
             ("resnet_v1_50/logits/biases", [1000]), ("global_step", [])]
    m = warm_start_map(ckpt, model, psp_module=True)
    enc = [n for n, _ in model if n.startswith(pre)]
    assert sorted(m.values()) == sorted(enc)
    assert all(pre + c == g for c, g in m.items())
    # a shape mismatch is not mapped; excluded scopes never are
    ckpt2 = [("resnet_v1_50/conv1/weights", [7, 7, 3, 32]),
             ("softmax_classifier/l1_logits/weights", [1, 1, 256, 14]),
             ("feature_extractor/extension/decrease_fdims/weights", [1, 1, 2048, 256])]
    assert warm_start_map(ckpt2, model, psp_module=True) == {}

"""TFRecord / tf.train.Example / PNG input on the host, and the oracle's
preprocessing restatement (input_cityscapes.py:66-96,190-209). Known answers are hand-encoded
protobuf bytes and TF 1.12 resize index rules; reading a TF-written file is parity unpinned
(none is available here)."""
import numpy as np
import pytest


def test_record_round_trip_and_corruption(tmp_path):
    from input_pipelines.tfrecords import read_records, write_records
    recs = [b"", b"x", bytes(range(256)) * 40]
    p = str(tmp_path / "a.tfrecord")
    write_records(p, recs)
    assert list(read_records(p)) == recs
    raw = bytearray(open(p, "rb").read())
    raw[12 + 4 + 12 + 1 + 4 + 12 + 3] ^= 1        # a byte inside the third record's data
    open(p, "wb").write(bytes(raw))
    with pytest.raises(ValueError):
        list(read_records(p))


def test_example_known_bytes_and_round_trip():
    from input_pipelines.tfrecords import encode_example, parse_example
    # Example{features{feature{key: "a" value{int64_list{value: [1]}}}}}
    want = bytes([0x0a, 0x0c, 0x0a, 0x0a, 0x0a, 0x01, 0x61, 0x12, 0x05, 0x1a, 0x03, 0x0a, 0x01, 0x01])
    assert encode_example({"a": [1]}) == want
    assert parse_example(want) == {"a": [1]}
    ex = {"image/encoded": [b"\x89PNG..."], "image/shape": [1024, 2048, 3],
          "label/path": [b"aachen_000000_000019_gtFine_labelIds.png"], "f": [0.5, -2.0],
          "neg": [-3]}
    assert parse_example(encode_example(ex)) == ex


def test_png_example_parse(tmp_path):
    from input_pipelines.tfrecords import encode_example, encode_png, parse_cityscapes_example
    rng = np.random.default_rng(0)
    im = rng.integers(0, 256, (17, 23, 3), dtype=np.uint8)
    la = rng.integers(0, 34, (17, 23), dtype=np.uint8)
    b = encode_example({"image/encoded": [encode_png(im)], "label/encoded": [encode_png(la)],
                        "image/path": [b"i.png"], "label/path": [b"l.png"],
                        "image/shape": [17, 23, 3], "label/shape": [17, 23, 1]})
    im2, la2, ip, lp = parse_cityscapes_example(b)
    np.testing.assert_array_equal(im2, im)
    np.testing.assert_array_equal(la2, la)
    assert (ip, lp) == (b"i.png", b"l.png")


def test_oracle_prepare_known_answers():
    from oracle.tfseg import prepare_images_np, prepare_labels_np
    rng = np.random.default_rng(1)
    raw = rng.integers(0, 256, (2, 8, 12, 3), dtype=np.uint8)
    same = prepare_images_np(raw, 8, 12)
    x = raw.astype(np.float32) * np.float32(1 / 255)
    np.testing.assert_array_equal(same, (x - np.float32(0.5)) / np.float32(0.5))
    # 2x down-sampling with the legacy scaler lands exactly on even pixels (lerp 0)
    np.testing.assert_array_equal(prepare_images_np(raw, 4, 6), same[:, ::2, ::2])
    lab = rng.integers(0, 34, (1, 6, 9), dtype=np.uint8)
    l2c = [-1] * 7 + list(range(19)) + [-1] * 8        # 34 Cityscapes-like label ids
    got = prepare_labels_np(lab, 3, 3, l2c)
    m = np.array([19 if c == -1 else c for c in l2c])
    np.testing.assert_array_equal(got, m[lab[:, ::2, ::3]])
    # up-sampling repeats source pixels: src = floor(o * in/out)
    np.testing.assert_array_equal(prepare_labels_np(lab, 12, 18, l2c),
                                  np.repeat(np.repeat(m[lab], 2, 1), 2, 2))

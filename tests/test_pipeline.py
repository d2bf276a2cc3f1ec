"""CPU tests of the entry-point host side (SURVEY.md §8 B CLI surface, F2-F4):
TFRecord framing + tf.train.Example codec, read_test_data semantics, the
shuffle-batch input queue, the detection metrics against the scalar oracle
(oracle/eval_ref.py), offline dataset synthesis and the entry-point CLI."""
import os
import struct

import numpy as np
import pytest

from mog_air import datasets, records
from mog_air.evaluation import evaluation, iou_matrix
from oracle import eval_ref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_crc32c_known_answers():
    # CRC-32C check value (RFC 3720 B.4) and the all-zero 32-byte vector
    assert records.crc32c(b"123456789") == 0xE3069283
    assert records.crc32c(bytes(32)) == 0x8A9136AA
    assert records.crc32c(bytes([0xFF] * 32)) == 0x62A8AB43


def test_tfrecord_framing_and_example_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    imgs = [rng.uniform(0, 1, (50, 50)).astype(np.float32) for _ in range(5)]
    ids = [[1, 2], [3], [], [4, 5, 6], [7]]
    pos = [[1, 2, 10, 20], [3, 4], [], [1, 1, 2, 2, 3, 3], [9, 9]]
    box = [[17, 17, 20, 20], [18, 18], [], [17, 17, 17, 17, 17, 17], [23, 23]]
    lab = [[0, 1], [2], [], [3, 4, 5], [6]]
    dig = [2, 1, 0, 3, 1]
    base = str(tmp_path / "common13")
    records.write_to_records(base, imgs, ids, pos, box, lab, dig)
    raw = list(records.iter_records(base + ".tfrecords", verify=True))
    assert len(raw) == 5
    ex = records.parse_example(raw[3])
    assert list(ex["digits"]) == [3] and list(ex["height"]) == [50]
    assert np.array_equal(np.frombuffer(ex["positions"][0], np.int32), pos[3])
    x, k = records.load_images(base + ".tfrecords")
    assert x.shape == (5, 2500) and np.array_equal(x[0], imgs[0].ravel())
    assert list(k) == dig
    # read_test_data: the first empty image moves to the front (images and
    # digits only, as multi_mnist.py:343-352)
    im, dg, ind, ps, bx, lb = records.read_test_data(base + ".tfrecords",
                                                     shift_zero_digits_images=True)
    assert list(dg) == [0, 2, 1, 3, 1]
    assert np.array_equal(im[0], imgs[2].ravel())
    assert np.array_equal(ps[3], pos[3]) and len(ps[2]) == 0
    # corrupted payload is caught by the CRC check
    data = bytearray(open(base + ".tfrecords", "rb").read())
    data[20] ^= 0xFF
    open(base + "_bad.tfrecords", "wb").write(bytes(data))
    with pytest.raises(records.RecordError):
        list(records.iter_records(base + "_bad.tfrecords", verify=True))


def test_example_parses_unpacked_int64_and_float_lists():
    # hand-encoded Example: int64 field unpacked (wire type 0), floats packed
    def ld(fn, b):
        return records._enc_varint(fn << 3 | 2) + records._enc_varint(len(b)) + b
    i64 = ld(1, b"") [:0] + records._enc_varint(1 << 3) + records._enc_varint(7) + \
        records._enc_varint(1 << 3) + records._enc_varint((1 << 64) - 2)
    feat_i = ld(3, i64)
    feat_f = ld(2, ld(1, struct.pack("<2f", 1.5, -2.0)))
    entries = ld(1, ld(1, b"n") + ld(2, feat_i)) + ld(1, ld(1, b"f") + ld(2, feat_f))
    ex = records.parse_example(ld(1, entries))
    assert list(ex["n"]) == [7, -2]
    assert np.array_equal(ex["f"], np.float32([1.5, -2.0]))


def test_shuffle_batcher_epochs_and_end_of_data():
    x = np.arange(10, dtype=np.float32)[:, None]
    k = np.arange(10, dtype=np.int32)
    b = records.ShuffleBatcher(x, k, batch_size=4, num_epochs=2, min_after_dequeue=3, seed=1)
    seen = []
    with pytest.raises(StopIteration):
        while True:
            bx, bk = b.next_batch()
            assert np.array_equal(bx[:, 0], bk)
            seen.extend(bk.tolist())
    assert len(seen) == 20 - 20 % 4
    counts = np.bincount(seen, minlength=10)
    assert counts.max() <= 2


def _random_case(rng, n, T=6, csize=50):
    pos, size, nums = [], [], []
    for _ in range(n):
        g = int(rng.integers(0, 4))
        p = rng.integers(0, csize - 20, 2 * g)
        pos.append(p)
        size.append(rng.integers(10, 24, 2 * g))
        nums.append(int(rng.integers(0, 4)))
    shifts = rng.uniform(-0.8, 0.8, (n, T, 2))
    scales = rng.uniform(0.2, 0.6, (n, T, 1))
    return pos, size, shifts, scales, np.asarray(nums)


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_evaluation_matches_scalar_oracle(seed):
    rng = np.random.default_rng(seed)
    case = _random_case(rng, 40)
    got = evaluation(*case, csize=50)
    ref = eval_ref.evaluation(*case, csize=50)
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=0, atol=1e-12)


def test_evaluation_edge_cases():
    # no gt & no detection -> all ones; gt only -> zeros; detection only -> recall 1
    pos = [np.zeros(0), np.asarray([10, 10]), np.zeros(0)]
    size = [np.zeros(0), np.asarray([20, 20]), np.zeros(0)]
    sh = np.zeros((3, 2, 2))
    sc = np.full((3, 2, 1), 0.4)
    p, r, gi, di, gl = evaluation(pos, size, sh, sc, np.asarray([0, 0, 1]), csize=50)
    assert np.allclose(p, 1 / 3) and np.allclose(r, 2 / 3)
    assert gi == di == gl == pytest.approx(1 / 3)
    # a perfect detection: a hit at every threshold but the last (IoU > 1.0 is
    # never true: the reference compares strictly)
    box = np.asarray([[15.0, 15.0, 35.0, 35.0]])
    assert iou_matrix(box, box)[0, 0] == 1.0
    p, r, gi, di, gl = evaluation([np.asarray([15, 15])], [np.asarray([20, 20])],
                                  np.zeros((1, 1, 2)), np.full((1, 1, 1), 0.4),
                                  np.asarray([1]), csize=50)
    assert np.all(p[:10] == 1) and p[10] == 0 and np.all(r[:10] == 1) and gl == 1.0


def test_synthesis_layout():
    sets = datasets.synthesize("mnist", [1, 3], images_per_count=6, test_set_size=4, seed=3)
    tr, te = sets["train"], sets["test"]
    assert len(te["images"]) == 4 and len(tr["images"]) == 8
    for img, n, p, b in zip(tr["images"], tr["digits"], tr["positions"], tr["boxes"]):
        assert img.shape == (50, 50) and img.min() >= 0 and img.max() <= 1
        assert len(p) == len(b) == 2 * n
        for j in range(n):  # every object lies inside the canvas
            assert 0 <= p[2 * j] and p[2 * j] + b[2 * j] <= 50
    ds = datasets.synthesize("dsprites", [2, 4], images_per_count=2, test_set_size=1, seed=4,
                             dsprites_npz=os.path.join(ROOT, "data", "multi_dsprites", "data.npz"))
    assert ds["train"]["images"][0].shape == (64, 64)


def test_entry_point_cli_surface():
    import argparse
    from mog_air import trainer
    p = argparse.ArgumentParser()
    trainer.add_common_args(p, reader_threads=4)
    a = p.parse_args(["-r", "x", "-k", "kk", "-gpu", "0", "-data", "dsprites", "-o", "1", "-t",
                      "2", "-dn", "24", "-dl", "right_half", "-ds", "20k"])
    tr, te, canvas, name, digits = trainer.dataset_files(a, "e")
    assert canvas == 64 and digits == [2, 4] and name == "right_half20k24"
    assert tr.endswith("multi_dsprites/commonright_half20k24.tfrecords")
    assert te.endswith("multi_dsprites/testright_half20k24.tfrecords")
    a.dig_location = "left"
    with pytest.raises(ValueError):
        trainer.dataset_files(a, "e")


def test_results_folder_suffixes(tmp_path):
    import argparse
    from mog_air import trainer
    p = argparse.ArgumentParser()
    trainer.add_common_args(p, reader_threads=1)
    base = str(tmp_path / "res")
    f1 = trainer.results_folder(p.parse_args(["-r", base, "-k", "a"]), "e", "13")
    f2 = trainer.results_folder(p.parse_args(["-r", base, "-k", "a"]), "e", "13")
    f3 = trainer.results_folder(p.parse_args(["-r", base, "-k", "a", "-o", "1"]), "e", "13")
    assert f1 == base + "_(a)" and f2 == base + "_(a)_0" and f3 == f1
    for sub in ("models", "summary", "source"):
        assert os.path.isdir(os.path.join(f2, sub))

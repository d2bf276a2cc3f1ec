"""TFRecord files of ``tf.train.Example`` records, read and written without
TensorFlow, so the entry points consume the reference's
on-disk datasets: ``common*.tfrecords`` / ``test*.tfrecords`` written by
multi_mnist.py:224-260 (``write_to_records``; fields height, width, digits
[int64], indices / positions / boxes / labels [int32 bytes], image [float32
bytes]) and read by multi_mnist.py:274-301 (``read_and_decode``: shuffled
training batches) and :304-361 (``read_test_data``).

Record framing (TFRecord): uint64 little-endian length, uint32 masked CRC-32C
of the length bytes, the payload, uint32 masked CRC-32C of the payload;
mask(c) = ((c >> 15) | (c << 17)) + 0xa282ead8 (mod 2^32).

Example wire format (tensorflow/core/example/{example,feature}.proto):
Example{1: Features}; Features{1: repeated MapEntry{1: key, 2: Feature}};
Feature{1: BytesList, 2: FloatList, 3: Int64List}; each list's values are
field 1 (bytes repeated; floats / int64 packed, unpacked also accepted).
"""
from __future__ import annotations

import struct
from typing import Dict, Iterator, List, Optional, Tuple

import numpy as np

# ------------------------------------------------------------------ CRC ----
_CRC_TABLE = None


def _crc_table() -> List[int]:
    global _CRC_TABLE
    if _CRC_TABLE is None:
        poly = 0x82F63B78  # Castagnoli, reflected
        tab = []
        for i in range(256):
            c = i
            for _ in range(8):
                c = (c >> 1) ^ poly if c & 1 else c >> 1
            tab.append(c)
        _CRC_TABLE = tab
    return _CRC_TABLE


def crc32c(data: bytes) -> int:
    tab = _crc_table()
    c = 0xFFFFFFFF
    for b in data:
        c = tab[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return ((((c >> 15) | (c << 17)) & 0xFFFFFFFF) + 0xA282EAD8) & 0xFFFFFFFF


class RecordError(ValueError):
    pass


def iter_records(path: str, verify: bool = False) -> Iterator[bytes]:
    """Payloads of a TFRecord file (``tf.python_io.tf_record_iterator``).
    ``verify`` checks both CRCs (pure Python: slow on large files)."""
    with open(path, "rb") as f:
        while True:
            head = f.read(12)
            if not head:
                return
            if len(head) < 12:
                raise RecordError(f"{path}: truncated record header")
            (n,) = struct.unpack("<Q", head[:8])
            payload = f.read(n)
            tail = f.read(4)
            if len(payload) < n or len(tail) < 4:
                raise RecordError(f"{path}: truncated record")
            if verify:
                if struct.unpack("<I", head[8:])[0] != masked_crc(head[:8]):
                    raise RecordError(f"{path}: length CRC mismatch")
                if struct.unpack("<I", tail)[0] != masked_crc(payload):
                    raise RecordError(f"{path}: payload CRC mismatch")
            yield payload


def write_records(path: str, payloads) -> None:
    with open(path, "wb") as f:
        for p in payloads:
            head = struct.pack("<Q", len(p))
            f.write(head + struct.pack("<I", masked_crc(head)) + p +
                    struct.pack("<I", masked_crc(p)))


# ------------------------------------------------------------- protobuf ----
def _varint(buf: bytes, i: int) -> Tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if b < 0x80:
            return v, i
        shift += 7
        if shift > 63:
            raise RecordError("malformed varint")


def _fields(buf: bytes):
    """(field number, wire type, value) of one message; value is an int for
    varints, bytes for length-delimited fields, raw bytes for fixed32/64."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        fn, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 2:
            ln, i = _varint(buf, i)
            v = buf[i:i + ln]
            i += ln
        elif wt == 5:
            v = buf[i:i + 4]
            i += 4
        elif wt == 1:
            v = buf[i:i + 8]
            i += 8
        else:
            raise RecordError(f"unsupported wire type {wt}")
        yield fn, wt, v


def _signed64(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def parse_example(payload: bytes) -> Dict[str, object]:
    """tf.train.Example -> {name: list[bytes] | np.float32 array | np.int64 array}."""
    out: Dict[str, object] = {}
    for fn, _, features in _fields(payload):
        if fn != 1:
            continue
        for efn, _, entry in _fields(features):
            if efn != 1:
                continue
            key, feat = None, b""
            for kfn, _, kv in _fields(entry):
                if kfn == 1:
                    key = kv.decode("utf-8")
                elif kfn == 2:
                    feat = kv
            if key is None:
                continue
            value: object = []
            for kind, _, lst in _fields(feat):
                if kind == 1:  # BytesList
                    value = [v for f, _, v in _fields(lst) if f == 1]
                elif kind == 2:  # FloatList
                    vals: List[float] = []
                    for f, wt, v in _fields(lst):
                        if f != 1:
                            continue
                        if wt == 2:
                            vals.extend(np.frombuffer(v, "<f4").tolist())
                        else:
                            vals.append(struct.unpack("<f", v)[0])
                    value = np.asarray(vals, np.float32)
                elif kind == 3:  # Int64List
                    ivals: List[int] = []
                    for f, wt, v in _fields(lst):
                        if f != 1:
                            continue
                        if wt == 2:
                            j = 0
                            while j < len(v):
                                x, j = _varint(v, j)
                                ivals.append(_signed64(x))
                        else:
                            ivals.append(_signed64(v))
                    value = np.asarray(ivals, np.int64)
            out[key] = value
    return out


def _len_field(fn: int, data: bytes) -> bytes:
    return _enc_varint((fn << 3) | 2) + _enc_varint(len(data)) + data


def _enc_varint(v: int) -> bytes:
    if v < 0:
        v += 1 << 64
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def build_example(features: Dict[str, object]) -> bytes:
    """Inverse of parse_example: bytes / list of bytes -> BytesList, integer
    sequences -> Int64List (packed), float arrays -> FloatList (packed)."""
    entries = b""
    for key in sorted(features):
        v = features[key]
        if isinstance(v, (bytes, bytearray)):
            v = [bytes(v)]
        if isinstance(v, list) and v and isinstance(v[0], (bytes, bytearray)):
            lst = b"".join(_len_field(1, bytes(x)) for x in v)
            feat = _len_field(1, lst)
        else:
            arr = np.asarray(v)
            if arr.dtype.kind == "f":
                lst = _len_field(1, arr.astype("<f4").tobytes())
                feat = _len_field(2, lst)
            else:
                lst = _len_field(1, b"".join(_enc_varint(int(x)) for x in arr.ravel()))
                feat = _len_field(3, lst)
        entries += _len_field(1, _len_field(1, key.encode("utf-8")) + _len_field(2, feat))
    return _len_field(1, entries)


# ----------------------------------------------------- AIR dataset files ----
def write_to_records(filename: str, images, indices, positions, boxes, labels, digits) -> None:
    """multi_mnist.py:224-260 (``write_to_records``): one Example per image
    into ``filename + '.tfrecords'``."""
    payloads = []
    for i in range(len(images)):
        img = np.asarray(images[i], np.float32)
        rows, cols = img.shape
        payloads.append(build_example({
            "height": [rows], "width": [cols], "digits": [int(digits[i])],
            "indices": np.asarray(indices[i], np.int32).tobytes(),
            "positions": np.asarray(positions[i], np.int32).tobytes(),
            "boxes": np.asarray(boxes[i], np.int32).tobytes(),
            "labels": np.asarray(labels[i], np.int32).tobytes(),
            "image": img.ravel().tobytes(),
        }))
    write_records(filename + ".tfrecords", payloads)


def load_images(path: str, verify: bool = False) -> Tuple[np.ndarray, np.ndarray]:
    """All (image [N, C*C] f32, digits [N] i32) of a file (the two fields
    read_and_decode parses, multi_mnist.py:278-284)."""
    imgs, digs = [], []
    for rec in iter_records(path, verify):
        ex = parse_example(rec)
        imgs.append(np.frombuffer(ex["image"][0], np.float32))
        digs.append(int(ex["digits"][0]))
    if not imgs:
        return np.zeros((0, 0), np.float32), np.zeros((0,), np.int32)
    return np.stack(imgs).astype(np.float32), np.asarray(digs, np.int32)


def read_test_data(filename: str, shift_zero_digits_images: bool = False, verify: bool = False):
    """multi_mnist.py:304-361: (images, digits, indices, positions, boxes,
    labels); per-object fields truncated to the image's digit count.  With
    ``shift_zero_digits_images`` the first empty image moves to the front and
    the other empty images to the back — images and digits only, exactly as
    the reference does (the per-object lists keep the file order)."""
    images, digits, indices, positions, boxes, labels = [], [], [], [], [], []
    for rec in iter_records(filename, verify):
        ex = parse_example(rec)
        n = int(ex["digits"][0])
        images.append(np.frombuffer(ex["image"][0], np.float32))
        digits.append(n)
        indices.append(np.frombuffer(ex["indices"][0], np.int32)[:n])
        positions.append(np.frombuffer(ex["positions"][0], np.int32)[:2 * n])
        boxes.append(np.frombuffer(ex["boxes"][0], np.int32)[:2 * n])
        labels.append(np.frombuffer(ex["labels"][0], np.int32)[:n])
    empty = [i for i, d in enumerate(digits) if d == 0]
    if shift_zero_digits_images and empty:
        full = [i for i, d in enumerate(digits) if d > 0]
        order = [empty[0]] + full + empty[1:]
        images = np.asarray(images)[order]
        digits = np.asarray(digits)[order]
    return images, digits, indices, positions, boxes, labels


class ShuffleBatcher:
    """``tf.train.shuffle_batch`` over ``num_epochs`` passes of a dataset held
    in memory (multi_mnist.py:274-301 with string_input_producer's
    num_epochs, training_air_original.py:144-147): a RandomShuffleQueue of
    ``min_after_dequeue`` examples filled in file order, each dequeued
    example drawn uniformly from it.  ``next_batch`` raises StopIteration
    (the reference's OutOfRangeError) once fewer than ``batch_size``
    examples remain."""

    def __init__(self, images: np.ndarray, digits: np.ndarray, batch_size: int,
                 num_epochs: Optional[int], min_after_dequeue: int = 10000, seed: int = 12345):
        self.images, self.digits = images, digits
        self.batch_size = batch_size
        self.num_epochs = num_epochs
        self.rng = np.random.default_rng(seed)
        self.cap = max(1, min_after_dequeue)
        self._src = self._source()
        self._buf: List[int] = []
        self._exhausted = False

    def _source(self) -> Iterator[int]:
        ep = 0
        n = len(self.digits)
        while n and (self.num_epochs is None or ep < self.num_epochs):
            for i in range(n):
                yield i
            ep += 1

    def _fill(self):
        while not self._exhausted and len(self._buf) < self.cap + self.batch_size:
            try:
                self._buf.append(next(self._src))
            except StopIteration:
                self._exhausted = True

    def next_batch(self) -> Tuple[np.ndarray, np.ndarray]:
        self._fill()
        if len(self._buf) < self.batch_size:
            raise StopIteration
        picks = []
        for _ in range(self.batch_size):
            j = int(self.rng.integers(len(self._buf)))
            self._buf[j], self._buf[-1] = self._buf[-1], self._buf[j]
            picks.append(self._buf.pop())
        idx = np.asarray(picks)
        return self.images[idx], self.digits[idx].astype(np.int32)

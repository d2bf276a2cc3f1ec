"""Offline dataset synthesis for the entry points.

Multi-MNIST (multi_mnist.py:90-221, :371-555) needs MNIST, which is fetched
from the internet by the reference and is not obtainable here; the stand-in
places procedural glyphs (random pen strokes of MNIST-digit scale, 17-23 px
sides, or 11-15 px for the ``bbox`` datasets, train_air_pr.py:84-87) on the
50x50 canvas.  Multi-dSprites (multi_dsprites.py:451-594) is built from the
reference's own shape file ``data/multi_dsprites/data.npz`` (120 64x64
sprites, cropped to 30x30 as IMAGE_SIZE there) on 64x64 canvases.

Placement follows generate_multi_image (multi_mnist.py:90-221): each object
is cropped to its non-empty square, tried at up to 100 uniform positions,
rejected on pixel overlap with the objects already placed, and the whole
canvas is redrawn if an object finds no place.  Returned per image: the
canvas, the object ids, positions [x, y, ...], boxes [w, h, ...], labels and
the object count — the fields write_to_records stores.
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional, Sequence

import numpy as np


def crop_non_empty(image: np.ndarray) -> np.ndarray:
    """Square crop around the non-empty pixels (multi_mnist.py:38-50)."""
    cols = np.nonzero(image.sum(axis=0))[0]
    rows = np.nonzero(image.sum(axis=1))[0]
    if cols.size == 0 or rows.size == 0:
        return image
    cx, lx = (cols[0] + cols[-1]) / 2.0, cols[-1] - cols[0]
    cy, ly = (rows[0] + rows[-1]) / 2.0, rows[-1] - rows[0]
    half = max(lx, ly) / 2.0
    y0, y1 = int(cy - half), int(cy + half)
    x0, x1 = int(cx - half), int(cx + half)
    return image[max(y0, 0):y1 + 1, max(x0, 0):x1 + 1]


def stroke_glyphs(n: int, rng: np.random.Generator, size_min: int = 17,
                  size_max: int = 23) -> List[np.ndarray]:
    """Procedural digit stand-ins: 2-4 thick random strokes in a square of a
    random side, intensities in (0.05, 1] like normalised MNIST pixels."""
    out = []
    for _ in range(n):
        s = int(rng.integers(size_min, size_max + 1))
        img = np.zeros((s, s), np.float32)
        yy, xx = np.mgrid[0:s, 0:s].astype(np.float32)
        for _ in range(int(rng.integers(2, 5))):
            p0, p1 = rng.uniform(0.1, 0.9, 2) * (s - 1), rng.uniform(0.1, 0.9, 2) * (s - 1)
            d = p1 - p0
            t = np.clip(((xx - p0[0]) * d[0] + (yy - p0[1]) * d[1]) / max(d @ d, 1e-6), 0, 1)
            dist = np.hypot(xx - (p0[0] + t * d[0]), yy - (p0[1] + t * d[1]))
            img = np.maximum(img, np.clip(1.6 - dist / (0.06 * s + 0.5), 0, 1))
        img[0, :] = img[-1, :] = 0
        img[:, 0] = img[:, -1] = 0
        img[img < 0.05] = 0
        out.append(img)
    return out


def dsprite_glyphs(path: str, image_size: int = 30):
    d = np.load(path)  # plain arrays only (allow_pickle defaults to False)
    return [im[:image_size, :image_size].astype(np.float32) for im in d["imgs"]], d["label"]


def generate_multi_image(glyphs: Sequence[np.ndarray], num: int, canvas: int,
                         rng: np.random.Generator, order: List[int],
                         max_attempts: int = 100):
    """One canvas with `num` non-overlapping objects (multi_mnist.py:90-221,
    pixel-overlap test, no buffer, no margin)."""
    while True:
        img = np.zeros((canvas, canvas), np.float32)
        ids, pos, box = [], [], []
        ok = True
        for _ in range(num):
            if not order:
                order.extend(rng.permutation(len(glyphs)).tolist())
            idx = order.pop()
            g = crop_non_empty(glyphs[idx])
            h, w = g.shape
            if h > canvas or w > canvas:
                ok = False
                break
            placed = False
            for _ in range(max_attempts):
                x = int(rng.integers(0, canvas - w + 1))
                y = int(rng.integers(0, canvas - h + 1))
                win = img[y:y + h, x:x + w]
                if ids and not np.array_equal(np.maximum(g, win), g + win):
                    continue
                placed = True
                break
            if not placed:
                ok = False
                break
            img[y:y + h, x:x + w] += g
            ids.append(idx)
            pos += [x, y]
            box += [w, h]
        if ok:
            return np.clip(img, 0.0, 1.0), ids, pos, box


def synthesize(kind: str, num_in_common: Sequence[int], images_per_count: int,
               test_set_size: int, seed: int = 0, bbox: bool = False,
               dsprites_npz: Optional[str] = None) -> Dict[str, Dict[str, list]]:
    """Train / test splits shaped like the reference's common*/test* files:
    ``images_per_count`` canvases per object count in ``num_in_common``,
    shuffled together, the first ``test_set_size`` forming the test split
    (multi_mnist.py:489-555)."""
    rng = np.random.default_rng(seed)
    if kind == "mnist":
        lo, hi = (11, 15) if bbox else (17, 23)
        glyphs = stroke_glyphs(512, rng, lo, hi)
        labels = rng.integers(0, 10, len(glyphs))
        canvas = 50
    else:
        path = dsprites_npz or os.path.join("data", "multi_dsprites", "data.npz")
        if not os.path.exists(path):  # the copy shipped with this repository
            path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "data",
                                "multi_dsprites", "data.npz")
        glyphs, lab = dsprite_glyphs(path)
        labels = lab[:, 1] if lab.ndim == 2 else lab
        canvas = 64
    order: List[int] = []
    rows = []
    for n in num_in_common:
        for _ in range(images_per_count):
            img, ids, pos, box = generate_multi_image(glyphs, n, canvas, rng, order)
            rows.append((img, ids, pos, box, [int(labels[i]) for i in ids], n))
    perm = rng.permutation(len(rows))
    rows = [rows[i] for i in perm]

    def split(rs):
        return {"images": [r[0] for r in rs], "indices": [r[1] for r in rs],
                "positions": [r[2] for r in rs], "boxes": [r[3] for r in rs],
                "labels": [r[4] for r in rs], "digits": [r[5] for r in rs]}

    return {"test": split(rows[:test_set_size]), "train": split(rows[test_set_size:])}

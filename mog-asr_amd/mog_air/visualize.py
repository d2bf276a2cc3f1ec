"""Reconstruction / generation image grids written as PNG files at the
reference's cadence (training_air_original.py:368-411, :445-490): the test
model's ``visualized_image`` (air_model.py:266-347 ``_visualize_reconstructions``:
original and reconstruction enlarged 2x, each object's attention window drawn
in its step's colour, 4-pixel white stripes), the misclassified subset, and
the generation grids with and without windows (air_model.py:349-420,
1137-1146), tiled by ``pile_image`` (utils/checkpoints.py:104-140).

Host-side presentation only (not on the per-step path).  The
window outlines are warped into the enlarged canvas with the HIP STN
(``ops.stn_forward``), exactly as the reference runs its ``transformer`` on
a ``draw_bounding_boxes`` image; PNG encoding is plain zlib (PIL is not
available here).
"""
from __future__ import annotations

import os
import struct
import zlib
from typing import Optional

import numpy as np
import torch

from . import ops

# air_model.py:197-198
COLORS = np.array([[1., 0., 0.], [0., 1., 0.], [0., 0., 1.], [1., 1., 0.], [1., 0., 1.],
                   [0., 1., 1.]], np.float32)


def write_png(path: str, rgb: np.ndarray) -> None:
    """8-bit RGB PNG (filter 0 per scanline)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w, c = rgb.shape
    assert c == 3
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(h))

    def chunk(tag, data):
        body = tag + data
        return struct.pack(">I", len(data)) + body + struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF)

    png = b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0))
    png += chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b"")
    with open(path, "wb") as f:
        f.write(png)


def pile_image(images: np.ndarray, path: str, shape=None) -> None:
    """utils/checkpoints.py:104-140: a unit x unit grid (unit = floor(sqrt(n)))
    filled column by column; images [N, H, W, 3] (or [N, H, W, 1]) in [0, 1]."""
    images = np.asarray(images, np.float32)
    if images.shape[-1] == 1:
        images = np.repeat(images, 3, axis=-1)
    n, h, w, _ = images.shape
    if shape is None:
        unit = max(1, int(n ** 0.5))
        shape = (unit, unit)
    grid = np.zeros((shape[1] * h, shape[0] * w, 3), np.float32)
    for i in range(min(n, shape[0] * shape[1])):
        col, row = i // shape[0], i % shape[1]
        grid[row * h:(row + 1) * h, col * w:(col + 1) * w] = images[i]
    write_png(path, np.clip(grid * 255.0 + 0.5, 0, 255).astype(np.uint8))


def resize_bilinear(img: np.ndarray, out: int) -> np.ndarray:
    """tf.image.resize_images (TF 1.12 bilinear, align_corners=False) of
    [N, S, S] to [N, out, out]: source coordinate = dst * S / out."""
    n, s, _ = img.shape
    c = np.arange(out, dtype=np.float32) * (s / out)
    lo = np.floor(c).astype(np.int64)
    hi = np.minimum(lo + 1, s - 1)
    f = (c - lo).astype(np.float32)
    rows = img[:, lo, :] * (1 - f)[None, :, None] + img[:, hi, :] * f[None, :, None]
    return rows[:, :, lo] * (1 - f)[None, None, :] + rows[:, :, hi] * f[None, None, :]


def window_boxes(st_back: torch.Tensor, window: int, size: int) -> np.ndarray:
    """[N, T, 6] backward transforms -> [N, T, size, size] window outlines:
    a window-sized image with a 1-pixel border (draw_bounding_boxes of the box
    [0, 0, 1, 1]) warped by the STN, clipped to [0, 1] and sharpened > 0.01
    (air_model.py:289-332)."""
    n, t = st_back.shape[0], st_back.shape[1]
    box = torch.zeros((window, window), device=st_back.device)
    box[0, :] = 1.0
    box[-1, :] = 1.0
    box[:, 0] = 1.0
    box[:, -1] = 1.0
    U = box.reshape(1, -1).expand(n * t, -1).contiguous()
    out = torch.empty((n * t, size * size), device=st_back.device)
    th = st_back.reshape(n * t, 6).contiguous().float()
    ops.stn_forward(U.view(n * t, window, window), th, (size, size), out=out)
    b = out.clamp(0.0, 1.0).cpu().numpy().reshape(n, t, size, size)
    return (b > 0.01).astype(np.float32)


def colored(images: np.ndarray, boxes: np.ndarray, steps: np.ndarray) -> np.ndarray:
    """_draw_colored_bounding_boxes (air_model.py:195-214): [N, S, S] grey
    images, [N, T, S, S] boxes, [N] executed steps -> [N, S, S, 3]."""
    out = np.repeat(images[..., None], 3, axis=-1).astype(np.float32)
    for s in range(boxes.shape[1]):
        m = (boxes[:, s] > 0) & (s < steps)[:, None, None]
        out[m] = COLORS[s % len(COLORS)]
    return out


def reconstruction_images(model, images, zoom: int = 2, num: Optional[int] = None) -> np.ndarray:
    """The test model's visualized_image_all after ``model.infer``: [N, zC,
    2 zC + 8, 3] (original with windows | stripe | reconstruction with
    windows | stripe)."""
    C = model.canvas_size
    x = torch.as_tensor(images, dtype=torch.float32).reshape(-1, C, C).cpu().numpy()
    rec = model.reconstruction.reshape(-1, C, C).float().cpu().numpy()
    n = x.shape[0] if num is None else min(num, x.shape[0])
    x, rec = x[:n], rec[:n]
    st = model.rec_st_back[:n]                              # [n, T_exec, 2, 3]
    T = model.max_steps
    pad = torch.zeros((n, T, 6), device=st.device)
    pad[:, :st.shape[1]] = st.reshape(n, st.shape[1], 6)
    steps = model.rec_num_digits[:n].cpu().numpy()
    boxes = window_boxes(pad, model.windows_size, zoom * C)
    big_x, big_r = resize_bilinear(x, zoom * C), resize_bilinear(rec, zoom * C)
    stripe = np.ones((n, zoom * C, 4, 3), np.float32)
    return np.concatenate([colored(big_x, boxes, steps), stripe, colored(big_r, boxes, steps),
                           stripe], axis=2)


def generation_images(model, num_steps: int, zoom: int = 2):
    """``generated_samples`` and ``generated_samples_bbox`` (air_model.py:1001-1146):
    ([G, C, C, 1] canvas, [G, zC, zC, 3] enlarged canvas with windows)."""
    C = model.canvas_size
    canvas = model.generate(num_steps).reshape(-1, C, C).float().cpu().numpy()
    G = canvas.shape[0]
    st = model.generated_st_back                             # [G, T, 2, 3]
    T = model.max_steps
    pad = torch.zeros((G, max(T, st.shape[1]), 6), device=st.device)
    pad[:, :st.shape[1]] = st.reshape(G, st.shape[1], 6)
    steps = model.generated_num_digits.cpu().numpy()
    boxes = window_boxes(pad, model.windows_size, zoom * C)
    return canvas[..., None], colored(resize_bilinear(canvas, zoom * C), boxes, steps)


def save_visualizations(model, images, targets, folder: str, tag, digits=(), num: int = 60,
                        generations: bool = True, gen_tag=None) -> None:
    """training_air_original.py:368-411 for one test batch: visualize_{tag}.png
    (first ``num``), visualize_{tag}_wrong.png (misclassified, up to 100) and,
    per digit count i, visualize_gen{gen_tag}_{i}.png / visualize_genbbox{gen_tag}_{i}.png
    (gen_tag defaults to tag; the final dump uses the step number there)."""
    model.infer(images, targets)
    allv = reconstruction_images(model, images)
    pile_image(allv[:num], os.path.join(folder, "visualize_{}.png".format(tag)))
    acc = model.accuracy_instance.cpu().numpy()
    wrong = allv[acc[:allv.shape[0]] == 0]
    if wrong.shape[0] > 0:
        pile_image(wrong[:100], os.path.join(folder, "visualize_{}_wrong.png".format(tag)))
    if not generations:
        return
    for i in digits:
        gen, gen_box = generation_images(model, int(i))
        gt = tag if gen_tag is None else gen_tag
        pile_image(gen, os.path.join(folder, "visualize_gen{}_{}.png".format(gt, i)))
        pile_image(gen_box, os.path.join(folder, "visualize_genbbox{}_{}.png".format(gt, i)))

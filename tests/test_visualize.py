"""Image grids of the entry points (mog_air.visualize; reference
training_air_original.py:368-411, air_model.py:195-347, utils/checkpoints.py:
104-140): the PNG writer round-trips, the grid layout and bilinear 2x
enlargement follow the reference; on the GPU the full reconstruction and
generation grids are written for a trained-from-init model."""
import struct
import zlib

import numpy as np
import pytest

import sys, os  # noqa: E401
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "mog-asr_amd"))
from mog_air import visualize as V  # noqa: E402


def _read_png(path):
    data = open(path, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, idat, w = 8, b"", None
    while pos < len(data):
        n, = struct.unpack(">I", data[pos:pos + 4])
        tag, body = data[pos + 4:pos + 8], data[pos + 8:pos + 8 + n]
        crc, = struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])
        assert crc == zlib.crc32(tag + body) & 0xFFFFFFFF
        if tag == b"IHDR":
            w, h = struct.unpack(">II", body[:8])
        if tag == b"IDAT":
            idat += body
        pos += 12 + n
    raw = zlib.decompress(idat)
    rows = [raw[y * (3 * w + 1) + 1:(y + 1) * (3 * w + 1)] for y in range(h)]
    return np.frombuffer(b"".join(rows), np.uint8).reshape(h, w, 3)


def test_png_roundtrip(tmp_path):
    img = (np.random.default_rng(0).random((7, 11, 3)) * 255).astype(np.uint8)
    V.write_png(str(tmp_path / "a.png"), img)
    np.testing.assert_array_equal(_read_png(str(tmp_path / "a.png")), img)


def test_pile_image_column_major_grid(tmp_path):
    # 5 images -> 2 x 2 grid, filled column by column (checkpoints.py:135-137)
    ims = np.stack([np.full((3, 4, 3), v / 10.0) for v in range(5)])
    V.pile_image(ims, str(tmp_path / "g.png"))
    g = _read_png(str(tmp_path / "g.png")).astype(np.float32) / 255.0
    assert g.shape == (6, 8, 3)
    assert abs(g[0, 0, 0] - 0.0) < 1e-2 and abs(g[3, 0, 0] - 0.1) < 1e-2
    assert abs(g[0, 4, 0] - 0.2) < 1e-2 and abs(g[3, 4, 0] - 0.3) < 1e-2


def test_resize_bilinear_tf1_asymmetric():
    x = np.arange(4, dtype=np.float32).reshape(1, 2, 2)
    y = V.resize_bilinear(x, 4)
    # source coordinate = dst / 2: 0, 0.5, 1, 1.5 (clamped to the last pixel)
    np.testing.assert_allclose(y[0, 0], [0.0, 0.5, 1.0, 1.0])
    np.testing.assert_allclose(y[0, :, 0], [0.0, 1.0, 2.0, 2.0])


@pytest.mark.gpu
def test_grids_written_on_gpu(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    from oracle import air_oracle as ao
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=3, cnn=False, train=False, scope="vis", device="cuda:0")
    x, k = ao.synthetic_canvases(16, seed=3)
    V.save_visualizations(m, x, k, str(tmp_path), 500, digits=(1, 2), num=9)
    for name in ("visualize_500.png", "visualize_gen500_1.png", "visualize_genbbox500_2.png"):
        img = _read_png(str(tmp_path / name))
        assert img.ndim == 3 and img.shape[2] == 3 and img.size > 0
    rec = _read_png(str(tmp_path / "visualize_500.png"))
    # 9 images -> 3 x 3 grid of [2C, 2*(2C) + 8] panels
    assert rec.shape == (3 * 100, 3 * 208, 3)

"""The pipelined fused step (vae_pipe.hip: persistent role-split workgroups,
the dense layers of tile i beside the STN read of tile i+1 and the STN write
of tile i-1) against the lockstep kernel (vae_step.hip) and the unfused bf16
sequence: every saved activation, r, z, the KL, the canvas parts and their
row ranges bit for bit (the same k-ordered MFMA chains and epilogues, only the
schedule differs).  air_model.py:500-588, vae.py:5-48, transformer.py:18-175."""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SAVED = ("canvas", "runloss", "vkl", "gb", "a1b", "a2b", "mu", "lv", "z", "zb", "d1b", "d2b", "r")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _setup(batch, seed):
    cfg = ao.AirConfig(batch=batch, max_steps=3, scale_prior_variance=0.05,
                       z_pres_prior_log_odds=-0.01)
    P = ao.init_params(cfg, seed=100 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=200 + seed)
    x, k = ao.synthetic_canvases(batch, seed=300 + seed)
    return cfg, P, nz, x, k


def _model(P, scope, fused=True):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=3, scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                 learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=True,
                 scope=scope, device=DEV, precision="bf16", fused_step=fused)
    m.params.load_dict(P)
    return m


def _bits(a):
    return a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)


def _same(ma, mb, names=SAVED):
    for name in names:
        a, b = getattr(ma._ws, name), getattr(mb._ws, name)
        assert torch.equal(_bits(a), _bits(b)), name


@pytest.mark.parametrize("batch", [150, 640])
def test_pipe_matches_unfused_bitwise(batch, monkeypatch):
    """Forced pipelined form: 150 images (one launch per loop step, running
    loss in the kernel, a ragged last tile, one tile per workgroup) and 640
    (all three steps' rows in one launch: x indexed by row % B)."""
    monkeypatch.setenv("MOG_VS_PIPE", "1")
    cfg, P, nz, x, k = _setup(batch, seed=11)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    mf, mu = _model(P, "pipe%d" % batch), _model(P, "pipeu%d" % batch, fused=False)
    G = torch.zeros((batch, cfg.canvas_size ** 2), device=DEV)
    mf.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    mu.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    torch.cuda.synchronize()
    _same(mf, mu)
    rows = mf._ws.prows.cpu().numpy()
    lo, hi = rows & 0xffff, rows >> 16
    assert (lo % 2 == 0).all() and (lo <= hi).all() and (hi <= 50).all()
    if mu._ws.prows is not None:  # (the unfused per-step form keeps one running canvas)
        np.testing.assert_array_equal(rows, mu._ws.prows.cpu().numpy())
    assert mf.loss == mu.loss


def test_pipe_inkernel_noise_several_tiles_per_workgroup(monkeypatch):
    """Perf mode (eps_x from in-kernel Philox) at 16,384 images: the batched
    VAE's 49,152 rows are three tiles per workgroup, so the S role samples
    tile i+1 and writes tile i-1 while the M role computes tile i; equal to the
    lockstep kernel bit for bit."""
    import bench
    x, k = bench.synthetic(16384, 77)
    X, K = torch.as_tensor(x).to(DEV), torch.as_tensor(k).to(DEV)
    cfg, P, _, _, _ = _setup(8, seed=12)
    mp, ml = _model(P, "pipe_big"), _model(P, "lock_big")
    mp.noise_seed = ml.noise_seed = 99
    monkeypatch.setenv("MOG_VS_PIPE", "1")
    mp.compute_gradients(X, K)
    monkeypatch.setenv("MOG_VS_PIPE", "0")
    ml.compute_gradients(X, K)
    torch.cuda.synchronize()
    assert mp._ws.eps_x_offset is not None
    _same(mp, ml, SAVED + ("cparts", "prows"))
    assert mp.loss == ml.loss


@pytest.mark.parametrize("canvas", [50, 64])
def test_pipe_roofline_launch_bitwise(canvas, monkeypatch):
    """The bench's north-star launch (bench.fused_step_roofline: 65,536 images,
    one loop step, training form) in both forms, outputs compared bit for
    bit, C = 50 and the Multi-dSprites C = 64."""
    import bench
    from mog_air.air_model import AIRModel  # noqa: F401
    dev = torch.device(DEV)
    B = 65536
    m = bench.make_model("bf16", dev, 1, 0, "pipe_roof%d" % canvas, canvas=canvas)
    m.noise_seed = 78
    x, k = bench.synthetic(B, 4321, canvas)
    X = torch.from_numpy(x).to(dev)
    m.infer(torch.from_numpy(x).to(dev), torch.from_numpy(k).to(dev))
    ws = m._ws
    outs = {}
    for form in ("1", "0"):
        monkeypatch.setenv("MOG_VS_PIPE", form)
        m._step_fused(X, ws, 1, 0.3, save=True)
        torch.cuda.synchronize()
        outs[form] = {n: getattr(ws, n)[1].clone() for n in
                      ("gb", "a1b", "a2b", "mu", "lv", "z", "zb", "d1b", "d2b", "r", "cparts",
                       "prows", "vkl")}
    for n in outs["1"]:
        assert torch.equal(_bits(outs["1"][n]), _bits(outs["0"][n])), n

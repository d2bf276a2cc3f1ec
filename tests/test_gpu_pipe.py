"""The pipelined persistent form of the fused STN-read -> VAE -> STN-write
kernel (vae_step.hip stn_vae_pipe_kernel: sampler / DMA / MFMA / STN-write
wave roles over 64-image tiles, LDS-counter hand-offs) against the unfused
bf16 sequence (stn_forward + bf16 GEMMs + vae_sample + stn accumulate) and the
lockstep form, bit for bit.

MOG_VS_PIPE=1 forces the form at test sizes, MOG_VS_PIPE_GRID gives each
workgroup several tiles (the cross-tile pipeline: ring reuse, arena hand-back,
S running ahead of M, W behind it), MOG_VS_CHECK=1 makes a role wait that
timed out fail the call instead of passing silently.
Reference: air/air_model.py:523-588, air/vae.py:5-48, air/transformer.py:18-175.
"""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


@pytest.fixture
def pipe(monkeypatch):
    def on(grid):
        monkeypatch.setenv("MOG_VS_PIPE", "1")
        monkeypatch.setenv("MOG_VS_CHECK", "1")
        monkeypatch.setenv("MOG_VS_PIPE_GRID", str(grid))
    return on


def _setup(batch, seed, canvas=50):
    cfg = ao.AirConfig(batch=batch, max_steps=3, scale_prior_variance=0.05,
                       z_pres_prior_log_odds=-0.01, canvas_size=canvas)
    P = ao.init_params(cfg, seed=1100 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=1200 + seed)
    if canvas == 50:
        x, k = ao.synthetic_canvases(batch, seed=1300 + seed)
    else:
        x, k = ao.synthetic_canvases(batch, canvas=canvas, seed=1300 + seed, counts=(2, 4),
                                     side=(22, 30))
    return cfg, P, nz, x, k


def _model(cfg, P, scope, fused, batched=True):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=3, canvas_size=cfg.canvas_size, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=True, scope=scope, device=DEV, precision="bf16",
                 fused_step=fused, batch_vae=batched)
    m.params.load_dict(P)
    return m


def _bits(a):
    return a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)


SAVED = ("runloss", "vkl", "gb", "a1b", "a2b", "mu", "lv", "z", "zb", "d1b", "d2b", "r")


def _compare(mf, mu, names):
    torch.cuda.synchronize()
    for n in names:
        assert torch.equal(_bits(getattr(mf._ws, n)), _bits(getattr(mu._ws, n))), n
    np.testing.assert_array_equal(mf.canvas.cpu().numpy(), mu.canvas.cpu().numpy())
    assert mf.loss == mu.loss


@pytest.mark.parametrize("batch,grid,batched", [(150, 1, False), (300, 2, False),
                                                (257, 3, False), (128, 1, True),
                                                (192, 4, True)])
def test_pipe_matches_unfused_bitwise(batch, grid, batched, pipe):
    """Training form (saved activations written): per-step launches (the
    running loss updated in the kernel; ragged last tiles at 150 / 300 / 257)
    and the all-steps launch over T*B rows (x_period = B, several tiles per
    workgroup)."""
    pipe(grid)
    cfg, P, nz, x, k = _setup(batch=batch, seed=batch + grid)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    tag = "%d_%d_%d" % (batch, grid, batched)
    mf = _model(cfg, P, "pf" + tag, True, batched)
    mu = _model(cfg, P, "pu" + tag, False, batched)
    G = torch.zeros((batch, cfg.canvas_size ** 2), device=DEV)
    mf.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    mu.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    _compare(mf, mu, SAVED)
    rows = mf._ws.prows.cpu().numpy()
    lo, hi = rows & 0xffff, rows >> 16
    assert (lo % 2 == 0).all() and (lo <= hi).all() and (hi <= cfg.canvas_size).all()


def test_pipe_forward_only_matches_lockstep_bitwise(monkeypatch):
    """Forward-only form (evaluation: the glimpse staged through the gb
    workspace, no other saved activation) against the lockstep kernel."""
    cfg, P, nz, x, k = _setup(batch=320, seed=3)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    monkeypatch.setenv("MOG_VS_PIPE", "0")
    ml = _model(cfg, P, "pfo_l", True)
    ml.infer(x, k, noise=noise)
    torch.cuda.synchronize()
    monkeypatch.setenv("MOG_VS_PIPE", "1")
    monkeypatch.setenv("MOG_VS_CHECK", "1")
    monkeypatch.setenv("MOG_VS_PIPE_GRID", "2")
    mp = _model(cfg, P, "pfo_p", True)
    mp.infer(x, k, noise=noise)
    _compare(mp, ml, ("vkl", "z", "r"))


def test_pipe_inkernel_noise_matches_filled_noise(pipe):
    """Perf mode (eps_x from the Philox counters inside the kernel) against
    the unfused sequence reading the filled buffer."""
    pipe(2)
    cfg, P, nz, x, k = _setup(batch=256, seed=4)
    mf = _model(cfg, P, "pn_f", True)
    mu = _model(cfg, P, "pn_u", False)
    mf.noise_seed = mu.noise_seed = 777
    mf.compute_gradients(x, k)
    mu.compute_gradients(x, k)
    assert mf._ws.eps_x_offset is not None
    _compare(mf, mu, ("runloss", "vkl", "r", "z", "d2b", "gb"))


def test_pipe_c64_matches_unfused_bitwise(pipe):
    """configs[3] canvas (C = 64: the STN write tables at their largest)."""
    pipe(2)
    cfg, P, nz, x, k = _setup(batch=192, seed=5, canvas=64)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    mf = _model(cfg, P, "p64f", True)
    mu = _model(cfg, P, "p64u", False)
    G = torch.zeros((192, 64 * 64), device=DEV)
    mf.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    mu.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    _compare(mf, mu, SAVED)


def test_pipe_gradients_match_lockstep(monkeypatch):
    """A whole train-step backward on the pipelined form's saved activations
    equals the lockstep form's (same bits in, same launches after)."""
    cfg, P, nz, x, k = _setup(batch=128, seed=6)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    monkeypatch.setenv("MOG_VS_PIPE", "0")
    gl = _model(cfg, P, "pg_l", True).compute_gradients(x, k, noise=noise)
    monkeypatch.setenv("MOG_VS_PIPE", "1")
    monkeypatch.setenv("MOG_VS_CHECK", "1")
    monkeypatch.setenv("MOG_VS_PIPE_GRID", "2")
    gp = _model(cfg, P, "pg_p", True).compute_gradients(x, k, noise=noise)
    # split-K atomics make the weight-gradient sums order-dependent
    for n in gl:
        d = np.linalg.norm(gp[n] - gl[n]) / max(np.linalg.norm(gl[n]), 1e-30)
        assert d < 1e-5, (n, d)

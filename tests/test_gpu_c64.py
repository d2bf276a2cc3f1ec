"""configs[3] (Multi-dSprites, C = 64: multi_dsprites.py:391-392,
training_air_original.py:89 canvas 64) on the GPU: the larger-canvas STN
gather path and the C = 64 tables of the fused step kernel.

* fp32: the full model forward bit-exact against the C oracle (oracle/air_ref.c)
  at C = 64 (counts, scales, shifts, windows, latents, KLs, canvas), train
  and test models, and gradients against float64 autograd.
* bf16: the fused STN-read -> VAE -> STN-write kernel against the unfused
  sequence bit for bit at C = 64, for every compiled tile shape, with a ragged
  last workgroup (batch 150).
"""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao
from oracle import air_torch as at

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
C = 64


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _setup(batch, seed, train=True, T=3):
    cfg = ao.AirConfig(batch=batch, max_steps=T, train=train, canvas_size=C,
                       scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01)
    P = ao.init_params(cfg, seed=500 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=600 + seed)
    x, k = ao.synthetic_canvases(batch, canvas=C, seed=700 + seed, counts=(2, 4), side=(22, 30))
    return cfg, P, nz, x, k


def _model(cfg, P, scope, precision="fp32", fused=True):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=C, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=cfg.train, scope=scope, device=DEV, precision=precision,
                 fused_step=fused)
    m.params.load_dict(P)
    return m


def _noise(nz):
    return {k: torch.as_tensor(v).to(DEV) for k, v in nz.items()}


@pytest.mark.parametrize("train", [True, False])
def test_fp32_forward_c64_bit_exact(train):
    cfg, P, nz, x, k = _setup(batch=24, seed=1 if train else 2, train=train)
    ro = ao.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, "c64fwd%d" % train)
    m.infer(x, k, noise=_noise(nz))
    assert m.executed_steps == ro["T"]
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ro["digits"])
    np.testing.assert_array_equal(m.rec_scales.cpu().numpy()[..., 0], ro["scale"].T)
    np.testing.assert_array_equal(m.rec_shifts.cpu().numpy(), ro["shift"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_windows.cpu().numpy(), ro["window"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_latents.cpu().numpy(), ro["latent"].transpose(1, 0, 2))
    for key in ("z_pres_kls", "scale_kls", "shift_kls"):
        np.testing.assert_array_equal(getattr(m, key).cpu().numpy(),
                                      ro[key.replace("kls", "kl")].T, err_msg=key)
    np.testing.assert_array_equal(m.vae_kls.cpu().numpy(), ro["vae_kl"].T)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ro["canvas"])
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ro["loss"], rtol=1e-5)
    # batch mean of per-image losses in the thousands: the per-image bar
    # (1e-5 relative; block-tree BCE sums) carries over to the mean
    assert abs(m.loss - ro["loss_mean"]) <= max(1e-3, 1e-5 * abs(ro["loss_mean"]))


def test_fp32_gradients_c64_vs_float64_autograd():
    cfg, P, nz, x, k = _setup(batch=6, seed=3)
    Gc = (np.random.default_rng(19).standard_normal((cfg.batch, C * C)) * 0.01).astype(np.float32)
    m = _model(cfg, P, "c64grad")
    grads = m.compute_gradients(x, k, noise=_noise(nz),
                                canvas_cotangent=torch.as_tensor(Gc).to(DEV))
    Pt = at.to_torch(P, requires_grad=True)
    out = at.air_forward(cfg, Pt, at.to_torch(nz), torch.tensor(x, dtype=torch.float64),
                         z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                         canvas_cotangent=torch.tensor(Gc, dtype=torch.float64),
                         fixed_steps=True)
    out["loss"].backward()
    for name, p in Pt.items():
        ref = p.grad.numpy() if p.grad is not None else np.zeros(p.shape)
        got = grads[name]
        err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-12)
        assert err < 2e-3 or np.linalg.norm(got - ref) < 1e-6, (name, err)


def _bits(a):
    return a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)


@pytest.mark.parametrize("variant", ["2", "3", "4"])
def test_bf16_fused_step_c64_matches_unfused_bitwise(variant, monkeypatch):
    monkeypatch.setenv("MOG_VS_MT", variant)
    cfg, P, nz, x, k = _setup(batch=150, seed=4)
    noise = _noise(nz)
    mf = _model(cfg, P, "c64f%s" % variant, precision="bf16", fused=True)
    mu = _model(cfg, P, "c64u%s" % variant, precision="bf16", fused=False)
    assert mf.fused_step and not mu.fused_step
    mf.compute_gradients(x, k, noise=noise)  # the training form: saved activations written
    mu.compute_gradients(x, k, noise=noise)
    torch.cuda.synchronize()
    for name in ("canvas", "runloss", "vkl", "gb", "a1b", "a2b", "mu", "lv", "z", "zb", "d1b",
                 "d2b", "r"):
        assert torch.equal(_bits(getattr(mf._ws, name)), _bits(getattr(mu._ws, name))), name
    rows = mf._ws.prows.cpu().numpy()
    lo, hi = rows & 0xffff, rows >> 16
    assert (lo % 2 == 0).all() and (lo <= hi).all() and (hi <= C).all()
    assert mf.loss == mu.loss
    # the count chain never touches the VAE: bf16 counts equal the fp32 oracle's
    ro = ao.forward(cfg, P, nz, x, k)
    np.testing.assert_array_equal(mf.rec_num_digits.cpu().numpy(), ro["digits"])

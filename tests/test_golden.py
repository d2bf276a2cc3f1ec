"""Golden vectors (tests/golden/*.npz, written by scripts/make_golden.py from
the CPU oracle).  The reference ships no fixtures and TensorFlow is absent
(SURVEY.md §8c), so the vectors pin the oracle restatement against drift and
give the HIP path committed expected outputs:

* CPU: the C oracle reproduces every forward vector bit for bit; the float64
  torch restatement reproduces the one-step Adam deltas.
* GPU: AIRModel (fp32) reproduces the forward vectors bit for bit (counts,
  scales, shifts, KLs, windows, latents, canvas), per-image loss within
  1e-5 relative; the bf16 configuration keeps the counts bit-exact; one
  clipped TF-Adam step under the golden canvas cotangent moves every small
  parameter tensor by the golden delta within 2 % of the step size.
"""
import glob
import os

import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FWD = sorted(glob.glob(os.path.join(GOLD, "air_fwd_*.npz")))
EXACT = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob", "z_pres_kl",
         "scale_kl", "shift_kl", "vae_kl", "canvas", "digits")


def _load(path):
    g = dict(np.load(path))
    cfg_kw = {k[4:]: g[k] for k in g if k.startswith("cfg_")}
    kw = {}
    for k, v in cfg_kw.items():
        if k == "num_prior":
            kw[k] = None if np.ndim(v) == 0 else tuple(int(x) for x in v)
        elif k == "train":
            kw[k] = bool(v)
        else:
            kw[k] = int(v)
    cfg = ao.AirConfig(scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01, **kw)
    P = ao.init_params(cfg, seed=int(g["param_seed"]), bias_scale=0.05)
    from scripts.make_golden import param_checksum
    assert param_checksum(P) == g["param_checksum"], "oracle weight init drifted"
    noise = {k[6:]: g[k] for k in g if k.startswith("noise_")}
    return cfg, P, noise, g


def test_golden_files_present():
    assert len(FWD) >= 3 and os.path.exists(os.path.join(GOLD, "air_adam_step_b4.npz"))


@pytest.mark.parametrize("path", FWD, ids=os.path.basename)
def test_oracle_reproduces_golden_forward(path):
    cfg, P, noise, g = _load(path)
    ref = ao.forward(cfg, P, noise, g["x"], g["targets"])
    assert ref["T"] == int(g["T"])
    for k in EXACT + ("bce", "mse", "loss"):
        np.testing.assert_array_equal(ref[k], g["out_" + k], err_msg=k)


def _adam_case():
    g = dict(np.load(os.path.join(GOLD, "air_adam_step_b4.npz")))
    cfg = ao.AirConfig(batch=4, max_steps=3, scale_prior_variance=0.05,
                       z_pres_prior_log_odds=-0.01)
    P0 = ao.init_params(cfg, seed=int(g["param_seed"]), bias_scale=0.05)
    noise = {k[6:]: g[k] for k in g if k.startswith("noise_")}
    return cfg, P0, noise, g


def test_torch_oracle_reproduces_golden_adam_step():
    from oracle import air_torch as at
    cfg, P0, noise, g = _adam_case()
    P = at.to_torch(P0, requires_grad=True)
    out = at.air_forward(cfg, P, at.to_torch(noise), torch.tensor(g["x"], dtype=torch.float64),
                         z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                         canvas_cotangent=torch.tensor(g["canvas_cotangent"], dtype=torch.float64),
                         fixed_steps=True)
    out["loss"].backward()
    assert float(out["loss"]) == pytest.approx(float(g["loss"]), rel=1e-12)
    grads = {n: p.grad if p.grad is not None else torch.zeros_like(p) for n, p in P.items()}
    m = {n: torch.zeros_like(v) for n, v in P.items()}
    v = {n: torch.zeros_like(t) for n, t in P.items()}
    with torch.no_grad():
        at.tf_clip_adam_step(P, grads, m, v, 1, lr=1e-4, clip=1.0)
    for k in g:
        if k.startswith("delta_"):
            n = k[6:].replace("__", "/")
            np.testing.assert_allclose(P[n].detach().numpy() - P0[n], g[k], rtol=1e-9,
                                       atol=1e-15, err_msg=n)


def _gpu_model(cfg, P, scope, precision="fp32"):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=cfg.canvas_size, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=cfg.train, scope=scope, device="cuda:0",
                 num_prior=list(cfg.num_prior) if cfg.num_prior else None, precision=precision)
    m.params.load_dict(P)
    return m


@pytest.mark.gpu
@pytest.mark.parametrize("path", FWD, ids=os.path.basename)
def test_hip_reproduces_golden_forward(path):
    cfg, P, noise, g = _load(path)
    m = _gpu_model(cfg, P, "gold_" + os.path.basename(path))
    m.infer(g["x"], g["targets"], noise={k: torch.as_tensor(v).cuda() for k, v in noise.items()})
    assert m.executed_steps == int(g["T"])
    got = {"scale": m.rec_scales[..., 0], "shift": m.rec_shifts, "st_back": m.rec_st_back,
           "window": m.rec_windows, "latent": m.rec_latents, "z_pres_prob": m.z_pres_probs,
           "z_pres_kl": m.z_pres_kls, "scale_kl": m.scale_kls, "shift_kl": m.shift_kls,
           "vae_kl": m.vae_kls}
    for k, v in got.items():  # model outputs are [B, T, ...]; golden step records [T, B, ...]
        ref = g["out_" + k]
        ref = np.moveaxis(ref, 0, 1).reshape(v.shape)
        np.testing.assert_array_equal(v.cpu().numpy(), ref, err_msg=k)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), g["out_canvas"])
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), g["out_digits"])
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), g["out_loss"], rtol=1e-5)
    # batch-mean -ELBO: 1e-3 absolute or, for losses in the
    # thousands (fp32 ulp 5e-4 at 6,000), the per-image 1e-5 relative bar
    ref = float(g["loss_mean"])
    assert abs(m.loss - ref) <= max(1e-3, 1e-5 * abs(ref))


@pytest.mark.gpu
@pytest.mark.parametrize("path", FWD, ids=os.path.basename)
def test_hip_bf16_golden_counts(path):
    cfg, P, noise, g = _load(path)
    m = _gpu_model(cfg, P, "goldbf_" + os.path.basename(path), precision="bf16")
    m.infer(g["x"], g["targets"], noise={k: torch.as_tensor(v).cuda() for k, v in noise.items()})
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), g["out_digits"])
    np.testing.assert_array_equal(m.rec_scales[..., 0].cpu().numpy(),
                                  np.moveaxis(g["out_scale"], 0, 1))


@pytest.mark.gpu
def test_hip_train_step_follows_golden_adam_deltas():
    """fp32 gradients (GPU) vs float64 (golden) through one clipped TF-Adam
    step: every delta within 2 % of the 1e-4 step (plus float32 rounding of
    the parameter itself)."""
    cfg, P0, noise, g = _adam_case()
    m = _gpu_model(cfg, P0, "gold_adam")
    m.compute_gradients(g["x"], g["targets"],
                        noise={k: torch.as_tensor(v).cuda() for k, v in noise.items()},
                        canvas_cotangent=torch.as_tensor(g["canvas_cotangent"]).cuda())
    m.params.apply_adam(1e-4, 1.0)
    after = m.params.state_dict()
    n_checked = 0
    for k in g:
        if not k.startswith("delta_"):
            continue
        n = k[6:].replace("__", "/")
        d = after[n].astype(np.float64) - P0[n].astype(np.float64)
        tol = 2e-6 + np.spacing(np.abs(P0[n]).astype(np.float32)).astype(np.float64)
        np.testing.assert_array_less(np.abs(d - g[k]), tol, err_msg=n)
        n_checked += d.size
    assert n_checked > 1000

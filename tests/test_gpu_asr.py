"""AIR-ASR on the GPU: the HIP path
(mog_air.asr_model.AIRModel) against the C oracle (oracle/asr_ref.c) on
identical injected noise — counts, steps, scales, shifts, z_pres
probabilities, masked KL records and the canvas bit for bit, per-image loss
within 1e-5 relative, margin within 1e-6 relative — and its gradients
against float64 torch autograd (oracle/asr_torch.py) under a well-conditioned
canvas cotangent, for the learned z_pres prior and fix_steps, train and test
models, fp32 and the bf16 glimpse-VAE configuration."""
import os

import numpy as np
import pytest
import torch

from oracle import air_oracle as ao
from oracle import asr_oracle as so
from oracle import asr_torch as st

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _cfg(**kw):
    base = dict(batch=12, max_steps=4, constrains_num=(1, 3), constrains_num_gamma=0.5,
                constrains_margin_gamma=100.0, constrains_num_element_gamma=10.0,
                constrains_bbox_gamma=1.0, constrains_sharesize_gamma=0.3,
                constrains_area_gamma=0.2, constrains_area_minmax=(17.0, 23.0))
    base.update(kw)
    return so.AsrConfig(**base)


def _model(cfg, P, scope, precision="fp32"):
    from mog_air.asr_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, max_digits=cfg.max_steps, canvas_size=cfg.canvas_size,
                 vae_likelihood_std=cfg.vae_likelihood_std, z_pres_prior_log_odds=-0.01,
                 z_pres_temperature=cfg.z_pres_temperature,
                 stopping_threshold=cfg.stopping_threshold, learning_rate=1e-4,
                 gradient_clipping_norm=1.0, cnn=False, train=cfg.train, scope=scope,
                 constrains_num=list(cfg.constrains_num),
                 constrains_num_gamma=cfg.constrains_num_gamma,
                 constrains_margin_gamma=cfg.constrains_margin_gamma,
                 constrains_num_element_gamma=cfg.constrains_num_element_gamma,
                 constrains_bbox_gamma=cfg.constrains_bbox_gamma,
                 constrains_sharesize_gamma=cfg.constrains_sharesize_gamma,
                 constrains_area_gamma=cfg.constrains_area_gamma,
                 constrains_area_minmax=list(cfg.constrains_area_minmax),
                 fix_steps=cfg.fix_steps, device=DEV, precision=precision)
    m.params.load_dict(P)
    return m


def _setup(seed, **kw):
    cfg = _cfg(**kw)
    P = so.init_params(cfg, seed=seed, bias_scale=0.05)
    nz = so.make_noise(cfg, seed=seed + 1)
    x, k = ao.synthetic_canvases(cfg.batch, seed=seed + 2)
    return cfg, P, nz, x, k


@pytest.mark.parametrize("kw,fused", [(dict(), False), (dict(train=False), False),
                                      (dict(fix_steps=2), False),
                                      (dict(z_pres_temperature=1.0, stopping_threshold=0.99), False),
                                      (dict(), True), (dict(fix_steps=2), True)])
def test_asr_forward_bit_exact_vs_oracle(kw, fused):
    """fused: each step's glimpse VAE through the fused fp32 step kernel
    (forced at this small batch; the model uses it from 8192 rows per step),
    the canvas from per-step parts -- the same bits."""
    cfg, P, nz, x, k = _setup(20, **kw)
    ref = so.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, "asrf%d%d" % (hash(tuple(sorted(kw.items()))), fused))
    if fused:
        m.FUSED_F32_MIN_ROWS = 0
    m.infer(x, k, noise={n: torch.as_tensor(v).to(DEV) for n, v in nz.items()})
    T = ref["T"]
    assert m.executed_steps == T
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ref["digits"])
    np.testing.assert_array_equal(m.rec_scales[..., 0].cpu().numpy(), ref["scale"].T)
    np.testing.assert_array_equal(m.rec_shifts.cpu().numpy(), ref["shift"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.z_pres_probs.cpu().numpy(), ref["z_pres_prob"].T)
    np.testing.assert_array_equal(m.z_pres_kls.cpu().numpy(), ref["z_pres_kl"].T)
    np.testing.assert_array_equal(m.scale_kls.cpu().numpy(), ref["scale_kl"].T)
    np.testing.assert_array_equal(m.shift_kls.cpu().numpy(), ref["shift_kl"].T)
    np.testing.assert_array_equal(m.vae_kls.cpu().numpy(), ref["vae_kl"].T)
    np.testing.assert_array_equal(m.rec_windows.cpu().numpy(), ref["window"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ref["canvas"])
    ws = m._ws
    for key, buf in (("area", ws.area), ("out", ws.outl), ("size", ws.size),
                     ("overlap", ws.over), ("element", ws.element), ("pr_loss", ws.pr)):
        np.testing.assert_array_equal(buf.cpu().numpy(), ref[key], err_msg=key)
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ref["loss"], rtol=1e-5)
    assert float(ws.margin[0]) == pytest.approx(ref["margin"], rel=1e-6, abs=1e-6)
    assert abs(m.loss - ref["loss_mean"]) <= max(1e-3, 1e-6 * abs(ref["loss_mean"]))


@pytest.mark.parametrize("kw,precision,tol,cos_min,global_tol",
                         [(dict(), "fp32", 2e-3, 0.999, 2e-3),
                          (dict(fix_steps=2), "fp32", 2e-3, 0.999, 2e-3),
                          # the fused fp32 step kernel's saved activations into the
                          # same backward (forced at this batch)
                          (dict(), "fp32-fused", 2e-3, 0.999, 2e-3),
                          # bf16: the bf16 VAE latents feed the next step's LSTM input
                          # and the shift / scale heads in ASR (unlike AIR), so the bf16
                          # forward trajectory itself drifts from the float64 one.  Some
                          # head gradients are ill-conditioned: perturbing only the VAE
                          # weights by 0.4 % (float64, no bf16 anywhere) moves
                          # inf_shift/dense_3/bias by 120 % (cosine 0.17).  Gate: every
                          # tensor whose float64 gradient moves < 10 % under that
                          # perturbation within 20 %, cosine >= 0.99 (an indexing or
                          # missing-term bug gives ~100 % / cosine ~0), and the whole
                          # concatenated gradient within 8 %.  Measured on MI355X
                          # (profiles/r03_asr_bf16_grad_report.json): worst checked
                          # tensor 11.3 % / cosine 0.9948 (inf_shift/dense_1/kernel),
                          # 42 of 49 tensors checked, global 4.95 % / cosine 0.9988.
                          (dict(), "bf16", 2e-1, 0.99, 8e-2)])
def test_asr_gradients_vs_float64_autograd(kw, precision, tol, cos_min, global_tol):
    cfg, P, nz, x, k = _setup(30, **kw)
    rng = np.random.default_rng(31)
    Gc = (rng.standard_normal((cfg.batch, cfg.canvas_size ** 2)) * 0.01).astype(np.float32)
    fused = precision == "fp32-fused"
    precision = "fp32" if fused else precision
    m = _model(cfg, P, "asrg%s%s%d" % (precision, cfg.fix_steps, fused), precision)
    if fused:
        m.FUSED_F32_MIN_ROWS = 0
    grads = m.compute_gradients(x, k, noise={n: torch.as_tensor(v).to(DEV) for n, v in nz.items()},
                                canvas_cotangent=torch.as_tensor(Gc).to(DEV))
    Pt = {n: torch.tensor(v, dtype=torch.float64, requires_grad=True) for n, v in P.items()}
    out = st.asr_forward(cfg, Pt, nz, torch.tensor(x, dtype=torch.float64),
                         canvas_cotangent=torch.tensor(Gc, dtype=torch.float64))
    out["loss"].backward()
    conditioned = {name: True for name in Pt}
    if precision == "bf16":
        r2 = np.random.default_rng(5)
        Pp = {n: torch.tensor(v * (1 + 4e-3 * r2.standard_normal(v.shape)) if "/vae/" in n else v,
                              dtype=torch.float64, requires_grad=True) for n, v in P.items()}
        st.asr_forward(cfg, Pp, nz, torch.tensor(x, dtype=torch.float64),
                       canvas_cotangent=torch.tensor(Gc, dtype=torch.float64))["loss"].backward()
        for name, p in Pt.items():
            if p.grad is None or Pp[name].grad is None:
                continue
            a, b = p.grad.numpy(), Pp[name].grad.numpy()
            conditioned[name] = np.linalg.norm(a - b) < 0.1 * np.linalg.norm(a)
    worst, checked = 0.0, 0
    got_all, ref_all = [], []
    report = []
    for name, p in Pt.items():
        ref = p.grad.numpy() if p.grad is not None else np.zeros(p.shape)
        got_all.append(np.asarray(grads[name], np.float64).ravel())
        ref_all.append(ref.ravel())
        if np.linalg.norm(ref) < 1e-6:
            assert np.linalg.norm(grads[name]) < 1e-4, name
            continue
        err = np.linalg.norm(grads[name] - ref) / np.linalg.norm(ref)
        cos = float(np.dot(grads[name].ravel(), ref.ravel()) /
                    (np.linalg.norm(grads[name]) * np.linalg.norm(ref) + 1e-30))
        report.append((name, float(err), cos, bool(conditioned[name])))
        if not conditioned[name]:
            continue
        worst = max(worst, err)
        checked += 1
        assert err < tol and cos > cos_min, (name, err, cos)
    g, r = np.concatenate(got_all), np.concatenate(ref_all)
    gerr = np.linalg.norm(g - r) / np.linalg.norm(r)
    gcos = float(np.dot(g, r) / (np.linalg.norm(g) * np.linalg.norm(r)))
    assert gerr < global_tol and gcos > 0.99, (gerr, gcos)
    assert checked >= 40  # (bf16: 42 of 49 conditioned tensors measured)
    print(f"ASR {precision} worst relative gradient error {worst:.2e}, global {gerr:.2e}")
    if os.environ.get("MOG_GRAD_REPORT"):
        import json
        with open(os.environ["MOG_GRAD_REPORT"] + f"_{precision}{cfg.fix_steps}.json", "w") as f:
            json.dump({"per_tensor": report, "global_rel": float(gerr), "global_cos": gcos}, f,
                      indent=1)


def test_asr_train_steps_finite():
    cfg, P, nz, x, k = _setup(40, batch=64, max_steps=6)
    m = _model(cfg, P, "asrtrain", "bf16")
    for i in range(3):
        loss, acc, mse, gs = m.step(x, k)
        assert np.isfinite(loss) and 0.0 <= acc <= 1.0
    assert gs == 3 and np.all(np.isfinite(m.params.flat.cpu().numpy()))
    lv = m.log_variables
    assert set(("num_margin", "num_min_KL", "area_loss", "over_loss")) <= set(lv)

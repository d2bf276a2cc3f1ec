"""TEST INFRASTRUCTURE ONLY — pure-torch CPU restatement of the reference AIR
train step (forward with autograd, TF-style clip + Adam).

Roles:
  1. an independent (float64-capable) restatement that pins the C oracle's
     forward (tests/test_oracle.py);
  2. the gradient oracle for the HIP backward (tests/test_gpu_parity.py);
  3. the CPU baseline timed by bench.py (``cpu_baseline.kind = "port"``):
     "CPU restatement, not TF-1.12" (BASELINE.md §3).

Follows: air/air_model.py:426-900 (loop, masks, loss), :941-999 (optimizer),
air/transformer.py:48-171, air/vae.py:5-48, air/concrete.py:20-64, TF-1.12
BasicLSTMCell / Adam semantics.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from .air_oracle import AirConfig, f32log, marginal_objective, param_specs


def _linspace(n: int, dtype) -> torch.Tensor:
    # TF LinSpace in fp32: start + step*i, last = stop (transformer.py:119-136)
    i = np.arange(n, dtype=np.float32)
    v = np.float32(-1.0) + np.float32(2.0 / (n - 1)) * i if n > 1 else np.array([-1.0])
    v = v.astype(np.float32)
    v[-1] = 1.0
    return torch.from_numpy(v).to(dtype)


def transformer(U: torch.Tensor, theta: torch.Tensor, out_hw) -> torch.Tensor:
    """transformer.py:18-175.  U [N,Hin,Win], theta [N,6] -> [N,Hout,Wout]."""
    N, Hin, Win = U.shape
    Ho, Wo = out_hw
    dt = U.dtype
    xt = _linspace(Wo, dt).view(1, Wo).expand(Ho, Wo).reshape(-1)
    yt = _linspace(Ho, dt).view(Ho, 1).expand(Ho, Wo).reshape(-1)
    th = theta.view(N, 6)
    xs = (th[:, 0:1] * xt + th[:, 1:2] * yt) + th[:, 2:3]
    ys = (th[:, 3:4] * xt + th[:, 4:5] * yt) + th[:, 5:6]
    wm = float(np.float32(Win) - np.float32(1.001)) if dt == torch.float32 else Win - 1.001
    hm = float(np.float32(Hin) - np.float32(1.001)) if dt == torch.float32 else Hin - 1.001
    x = (xs + 1.0) * wm / 2.0
    y = (ys + 1.0) * hm / 2.0
    x0 = torch.floor(x).detach().clamp(-2 ** 30, 2 ** 30).long()
    y0 = torch.floor(y).detach().clamp(-2 ** 30, 2 ** 30).long()
    x1, y1 = x0 + 1, y0 + 1
    x0, x1 = x0.clamp(0, Win - 1), x1.clamp(0, Win - 1)
    y0, y1 = y0.clamp(0, Hin - 1), y1.clamp(0, Hin - 1)
    flat = U.reshape(N, Hin * Win)
    Ia = torch.gather(flat, 1, y0 * Win + x0)
    Ib = torch.gather(flat, 1, y1 * Win + x0)
    Ic = torch.gather(flat, 1, y0 * Win + x1)
    Id = torch.gather(flat, 1, y1 * Win + x1)
    x0f, x1f, y0f, y1f = x0.to(dt), x1.to(dt), y0.to(dt), y1.to(dt)
    wa = (x1f - x) * (y1f - y)
    wb = (x1f - x) * (y - y0f)
    wc = (x - x0f) * (y1f - y)
    wd = (x - x0f) * (y - y0f)
    out = ((wa * Ia + wb * Ib) + wc * Ic) + wd * Id
    return out.view(N, Ho, Wo)


def softplus_tf(x: torch.Tensor) -> torch.Tensor:
    """TF-1.12 Softplus functor thresholds (vae.py:11)."""
    t = float(np.log(np.finfo(np.float32).eps) + 2.0)
    ex = torch.exp(torch.clamp(x, max=-t))
    mid = torch.log(ex + 1.0)
    return torch.where(x > -t, x, torch.where(x < t, ex, mid))


def concrete_kl(y, plo, pT, qlo, qT):
    """concrete.py:30-64 (reduce_logsumexp of [0, a] with a stop-gradient max)."""
    eps = 1e-9

    def lse0(a):
        m = torch.clamp(a, min=0.0).detach()
        return torch.log(torch.exp(-m) + torch.exp(a - m)) + m

    lp = (np.log(pT + eps) - y * (pT + 1.0) + plo) - 2.0 * lse0(-y * pT + plo)
    lq = (np.log(qT + eps) - y * (qT + 1.0) + qlo) - 2.0 * lse0(-y * qT + qlo)
    return lq - lp


def _dense(x, P, name, act=None):
    y = x @ P[name + "/weights"] + P[name + "/biases"]
    return act(y) if act is not None else y


def air_forward(cfg: AirConfig, P: Dict[str, torch.Tensor], noise: Dict[str, torch.Tensor],
                images: torch.Tensor, targets: Optional[torch.Tensor] = None,
                z_pres_prior_log_odds: Optional[float] = None,
                canvas_cotangent: Optional[torch.Tensor] = None,
                fixed_steps: bool = False) -> Dict[str, torch.Tensor]:
    """Reference loop (air_model.py:426-900).  ``canvas_cotangent`` replaces the
    BCE term by <G, canvas> (well-conditioned surrogate used for gradient
    parity).  ``fixed_steps`` runs all max_steps with
    the loop predicate folded into a per-step 'live' mask (the HIP schedule);
    losses and counts are identical to the data-dependent exit."""
    dt = images.dtype
    B, T, H = cfg.batch, cfg.max_steps, cfg.rnn_units
    C, W = cfg.canvas_size, cfg.windows_size
    thr = cfg.stopping_threshold
    Tz = cfg.z_pres_temperature
    prior_lo = cfg.z_pres_prior_log_odds if z_pres_prior_log_odds is None else z_pres_prior_log_odds
    mo = marginal_objective(cfg.num_prior, T) if cfg.num_prior is not None else None
    p = "air/rnn/"
    K = P[p + "rnn/basic_lstm_cell/kernel"]
    bK = P[p + "rnn/basic_lstm_cell/bias"]
    h = torch.zeros(B, H, dtype=dt)
    c = torch.zeros(B, H, dtype=dt)
    stop = torch.zeros(B, dtype=dt)
    runloss = torch.zeros(B, dtype=dt)
    digits = torch.zeros(B, dtype=torch.int32)
    canvas = torch.zeros(B, C * C, dtype=dt)
    recs = {k: [] for k in ("scale", "shift", "window", "latent", "z_pres_prob", "z_pres_kl",
                            "scale_kl", "shift_kl", "vae_kl", "z_pres")}
    relu = torch.relu
    slv_p = float(f32log(cfg.scale_prior_variance))
    hlv_p = float(f32log(cfg.shift_prior_variance))
    vlv_p = float(f32log(cfg.vae_prior_variance))
    xk = images @ K[: C * C]  # hoisted x-projection (identical math)
    step = 0
    while step < T:
        live_any = bool((stop < thr).any())
        if not fixed_steps and not live_any:
            break
        live = 1.0 if live_any else 0.0
        g = xk + h @ K[C * C:] + bK
        i_, j_, f_, o_ = g.split(H, dim=1)
        c = c * torch.sigmoid(f_ + 1.0) + torch.sigmoid(i_) * torch.tanh(j_)
        h = torch.tanh(c) * torch.sigmoid(o_)
        sm = _dense(_dense(h, P, p + "scale/mean/hidden", relu), P, p + "scale/mean/output")
        sv = _dense(_dense(h, P, p + "scale/log_variance/hidden", relu), P,
                    p + "scale/log_variance/output")
        hm = _dense(_dense(h, P, p + "shift/mean/hidden", relu), P, p + "shift/mean/output")
        hv = _dense(_dense(h, P, p + "shift/log_variance/hidden", relu), P,
                    p + "shift/log_variance/output")
        svar, hvar = torch.exp(sv), torch.exp(hv)
        scale = torch.sigmoid(sm + noise["eps_scale"][step].view(B, 1) * torch.sqrt(svar))
        shift = torch.tanh(hm + noise["eps_shift"][step] * torch.sqrt(hvar))
        s, tx, ty = scale[:, 0], shift[:, 0], shift[:, 1]
        zero = torch.zeros_like(s)
        theta = torch.stack([s, zero, tx, zero, s, ty], 1)
        window = transformer(images.view(B, C, C), theta, (W, W)).reshape(B, W * W)
        v = p + "vae/"
        a1 = _dense(window, P, v + "recognition_1", softplus_tf)
        a2 = _dense(a1, P, v + "recognition_2", softplus_tf)
        mu = _dense(a2, P, v + "rec_mean")
        lv = _dense(a2, P, v + "rec_log_variance")
        z = mu + noise["eps_z"][step] * torch.sqrt(torch.exp(lv))
        d1 = _dense(z, P, v + "generative_1", softplus_tf)
        d2 = _dense(d1, P, v + "generative_2", softplus_tf)
        m = _dense(d2, P, v + "gen_mean")
        r = torch.sigmoid(m + noise["eps_x"][step] * cfg.vae_likelihood_std)
        theta_r = torch.stack([1.0 / s, zero, -tx / s, zero, 1.0 / s, -ty / s], 1)
        wr = transformer(r.view(B, W, W), theta_r, (C, C)).reshape(B, C * C)
        lo = _dense(_dense(h, P, p + "z_pres/log_odds/hidden", relu), P,
                    p + "z_pres/log_odds/output")[:, 0]
        u = noise["u"][step]
        y = (lo + (torch.log(u + 1e-9) - torch.log(1.0 - u + 1e-9))) / Tz
        zp = torch.sigmoid(y)
        if not cfg.train:
            zp = torch.round(zp)
        bias = float(mo[step]) if mo is not None else 0.0
        zkl = concrete_kl(y, prior_lo + bias, Tz, lo, Tz)
        zkl_end = (concrete_kl(y, -100.0, Tz, lo, Tz) if mo is not None
                   else torch.zeros_like(zkl))
        runloss = runloss + live * torch.where(stop < thr, zkl, zkl_end)
        stop = stop + (1.0 - zp)
        active = stop < thr
        digits = digits + active.to(torch.int32)
        canvas = canvas + torch.where(active.view(B, 1), zp.view(B, 1) * wr,
                                      torch.zeros_like(wr))
        skl = 0.5 * ((slv_p - sv - 1.0 + svar / cfg.scale_prior_variance +
                      (sm - cfg.scale_prior_mean) ** 2 / cfg.scale_prior_variance).sum(1))
        hkl = 0.5 * ((hlv_p - hv - 1.0 + hvar / cfg.shift_prior_variance +
                      (hm - cfg.shift_prior_mean) ** 2 / cfg.shift_prior_variance).sum(1))
        vkl = 0.5 * ((vlv_p - lv - 1.0 + torch.exp(lv) / cfg.vae_prior_variance +
                      (mu - cfg.vae_prior_mean) ** 2 / cfg.vae_prior_variance).sum(1))
        zero_b = torch.zeros_like(skl)
        runloss = runloss + torch.where(active, skl, zero_b)
        runloss = runloss + torch.where(active, hkl, zero_b)
        runloss = runloss + torch.where(active, vkl, zero_b)
        for k, val in (("scale", scale), ("shift", shift), ("window", r), ("latent", z),
                       ("z_pres_prob", torch.sigmoid(lo)), ("z_pres_kl", zkl),
                       ("scale_kl", skl), ("shift_kl", hkl), ("vae_kl", vkl),
                       ("z_pres", zp)):
            recs[k].append(val)
        step += 1
    out = {k: torch.stack(v, 0) for k, v in recs.items() if v}
    out["T"] = step
    out["digits"] = digits
    out["canvas"] = canvas
    out["running_loss"] = runloss
    rec = torch.clamp(canvas, 0.0, 1.0)  # TF Min/Max grads pass at equality
    if canvas_cotangent is None:
        x = images
        bce = -(x * torch.log(rec + 1e-10) + (1.0 - x) * torch.log(1.0 - rec + 1e-10)).sum(1)
        out["bce"] = bce
        out["mse"] = ((x - rec) ** 2).sum(1)
        per_image = runloss + bce
        out["loss_b"] = per_image
        out["loss"] = per_image.mean()
    else:
        out["loss"] = runloss.mean() + (canvas_cotangent * canvas).sum()
    if targets is not None:
        out["accuracy"] = (targets.to(torch.int32) == digits).to(dt).mean()
    return out


def tf_clip_adam_step(params: Dict[str, torch.Tensor], grads: Dict[str, torch.Tensor],
                      m: Dict[str, torch.Tensor], v: Dict[str, torch.Tensor], t: int,
                      lr: float = 1e-4, clip: float = 1.0, beta1=0.9, beta2=0.999,
                      eps=1e-8) -> None:
    """air_model.py:941-999: per-tensor inf->0, nan->0, clip_by_norm, then TF
    ApplyAdam (epsilon outside the bias correction).  ``t`` starts at 1."""
    b1p = np.float32(beta1) ** np.float32(t)
    b2p = np.float32(beta2) ** np.float32(t)
    lr_t = lr * np.sqrt(1.0 - b2p) / (1.0 - b1p)
    with torch.no_grad():
        for name, p in params.items():
            g = grads[name]
            g = torch.where(torch.isinf(g), torch.zeros_like(g), g)
            g = torch.where(torch.isnan(g), torch.zeros_like(g), g)
            l2 = (g * g).sum()
            norm = torch.sqrt(l2) if float(l2) > 0 else l2
            g = g * clip / torch.clamp(norm, min=clip)
            m[name] += (g - m[name]) * (1.0 - beta1)
            v[name] += (g * g - v[name]) * (1.0 - beta2)
            p -= (m[name] * lr_t) / (torch.sqrt(v[name]) + eps)


def to_torch(d: Dict[str, np.ndarray], dtype=torch.float64, requires_grad=False):
    return {k: torch.tensor(np.asarray(v), dtype=dtype, requires_grad=requires_grad)
            for k, v in d.items()}


def train_step(cfg: AirConfig, P, m, v, t, noise, images, targets, prior_lo):
    """One CPU train step (forward, backward, clip, Adam). Returns the loss."""
    for p_ in P.values():
        p_.grad = None
    out = air_forward(cfg, P, noise, images, targets, z_pres_prior_log_odds=prior_lo)
    out["loss"].backward()
    grads = {k: p_.grad if p_.grad is not None else torch.zeros_like(p_) for k, p_ in P.items()}
    tf_clip_adam_step(P, grads, m, v, t)
    return float(out["loss"].detach())


__all__ = ["transformer", "air_forward", "tf_clip_adam_step", "to_torch", "train_step",
           "param_specs", "softplus_tf", "concrete_kl"]

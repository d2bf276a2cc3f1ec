"""TEST INFRASTRUCTURE ONLY — float64-capable torch restatement of the AIR-ASR
forward pass (air/air_number_bbox_location.py:384-1079, same semantics as
oracle/asr_ref.c) whose autograd backward is the gradient oracle of the HIP
ASR path.  ``canvas_cotangent`` replaces the reconstruction BCE by <G, canvas>
(the BCE is bit-fragile at canvas pixels that are exactly 0; DESIGN.md
§Numerics); ``fixed_steps`` folds the loop predicate into a live mask (the
HIP schedule) — losses are identical to the data-dependent exit.
"""
from __future__ import annotations

import numpy as np
import torch

from .air_torch import concrete_kl, softplus_tf, transformer
from .asr_oracle import P_ROOT, AsrConfig


def _sce(z, x):
    """tf.nn.sigmoid_cross_entropy_with_logits(labels=z, logits=x)."""
    return torch.clamp(x, min=0.0) - x * z + torch.log1p(torch.exp(-torch.abs(x)))


def _logit8(p):
    return torch.log(p + 1e-8) - torch.log(1.0 - p + 1e-8)


def asr_forward(cfg: AsrConfig, P, noise, images, targets=None, canvas_cotangent=None,
                fixed_steps=True, live_reduce=None, zsum_reduce=None, global_batch=None):
    """``live_reduce(local_any) -> global_any`` and ``zsum_reduce(local [T] sum)
    -> global [T] sum`` restate one data-parallel shard: the
    loop predicate is global over the batch (air_number_bbox_location.py:386-390)
    and the margin uses the batch-mean z_pres probabilities (:982-998) of
    ``global_batch`` images; the returned loss is this shard's share
    (B_local / global_batch of its mean) plus the full margin, so the sum of
    the shards' gradients is the full-batch gradient."""
    dt = images.dtype
    B, T, H, Z = cfg.batch, cfg.max_steps, cfg.rnn_units, cfg.vae_latent_dimensions
    C, W = cfg.canvas_size, cfg.windows_size
    C2, W2 = C * C, W * W
    p = P_ROOT

    def dense(x, scope, act=None):
        y = x @ P[p + scope + "/kernel"] + P[p + scope + "/bias"]
        return act(y) if act is not None else y

    def vdense(x, name, act=None):
        y = x @ P[p + "vae/" + name + "/weights"] + P[p + "vae/" + name + "/biases"]
        return act(y) if act is not None else y

    def lstm(x, h, c, scope):
        g = torch.cat([x, h], 1) @ P[p + scope + "/kernel"] + P[p + scope + "/bias"]
        gi, gj, gf, go = torch.split(g, H, 1)
        c = c * torch.sigmoid(gf + 1.0) + torch.sigmoid(gi) * torch.tanh(gj)
        return torch.tanh(c) * torch.sigmoid(go), c

    z0 = lambda *s: torch.zeros(s, dtype=dt)  # noqa: E731
    h, c, hg, cg = z0(B, H), z0(B, H), z0(B, H), z0(B, H)
    hg_prev, zprev, ssprev = z0(B, H), z0(B, Z), z0(B, 3)
    stop = z0(B)
    canvas = z0(B, C2)
    digits = torch.zeros(B, dtype=torch.int64)
    gclv = float(np.log(np.float32(cfg.scale_prior_variance), dtype=np.float32)) \
        if dt == torch.float32 else float(np.log(cfg.scale_prior_variance))
    gcvar, gcm = cfg.scale_prior_variance, cfg.scale_prior_mean
    vplv = float(np.log(cfg.vae_prior_variance))
    rec = {k: [] for k in ("scale", "shift", "zprob", "zkl", "skl", "shkl", "vkl", "prn")}
    thr, Tq = cfg.stopping_threshold, cfg.z_pres_temperature
    steps = 0
    for t in range(T):
        live = bool((stop < thr).any())
        if live_reduce is not None:
            live = bool(live_reduce(live))
        if not live:
            if not fixed_steps:
                break
        steps += int(live)
        tn = lambda k: torch.as_tensor(noise[k][t], dtype=dt)  # noqa: E731
        x_in = torch.cat([images, zprev, ssprev], 1)
        h, c = lstm(x_in, h, c, "infer_rnn_running")
        sm = dense(dense(h, "inf_shift/dense", torch.relu), "inf_shift/dense_1")
        slv = dense(dense(h, "inf_shift/dense_2", torch.relu), "inf_shift/dense_3")
        svar = torch.exp(slv)
        sl = sm + tn("eps_shift") * torch.sqrt(svar)
        shift = torch.tanh(sl)
        hin = torch.cat([h, sl], 1)
        cm = dense(torch.cat([dense(hin, "inf_scale/dense", torch.relu), sl], 1),
                   "inf_scale/dense_1")
        clv = dense(torch.cat([dense(hin, "inf_scale/dense_2", torch.relu), sl], 1),
                    "inf_scale/dense_3")
        cvar = torch.exp(clv)
        cl = cm + tn("eps_scale")[:, None] * torch.sqrt(cvar)
        s = torch.sigmoid(cl)[:, 0]
        ss = torch.cat([sl, cl], 1)
        hg, cg = lstm(torch.cat([zprev, ssprev], 1), hg, cg, "gen_rnn_running")
        gsm = dense(dense(hg, "gen_shift/dense", torch.relu), "gen_shift/dense_1")
        gslv = dense(dense(hg, "gen_shift/dense_2", torch.relu), "gen_shift/dense_3")
        tx, ty = shift[:, 0], shift[:, 1]
        zr = torch.zeros_like(s)
        th = torch.stack([s, zr, tx, zr, s, ty], 1)
        g = transformer(images.view(B, C, C), th, (W, W)).reshape(B, W2)
        a1 = vdense(g, "recognition_1", softplus_tf)
        a2 = vdense(a1, "recognition_2", softplus_tf)
        mu, lv = vdense(a2, "rec_mean"), vdense(a2, "rec_log_variance")
        zl = mu + tn("eps_z") * torch.sqrt(torch.exp(lv))
        d2 = vdense(vdense(zl, "generative_1", softplus_tf), "generative_2", softplus_tf)
        r = torch.sigmoid(vdense(d2, "gen_mean") + tn("eps_x") * cfg.vae_likelihood_std)
        thb = torch.stack([1.0 / s, zr, -tx / s, zr, 1.0 / s, -ty / s], 1)
        wr = transformer(r.view(B, W, W), thb, (C, C)).reshape(B, C2)
        if cfg.fix_steps is not None:
            plo = torch.full((B,), 100.0 if t < cfg.fix_steps else -100.0, dtype=dt)
        else:
            plo = dense(dense(hg_prev, "z_pres/prior/dense", torch.relu),
                        "z_pres/prior/dense_1")[:, 0]
        lo = dense(dense(h, "z_pres/log_odds/dense", torch.relu), "z_pres/log_odds/dense_1")[:, 0]
        u = tn("u")
        y = (lo + (torch.log(u + 1e-9) - torch.log(1.0 - u + 1e-9))) / Tq
        zp = torch.sigmoid(y)
        if not cfg.train:
            zp = torch.round(zp).detach()
        zprob = torch.sigmoid(lo)
        if cfg.constrains_num_gamma > 1e-8:
            ent = zprob * softplus_tf(-lo) + (1.0 - zprob) * softplus_tf(lo)
            prn = ent * cfg.constrains_num_gamma
        else:
            prn = torch.zeros_like(lo)
        zkl = concrete_kl(y, plo, Tq, lo, Tq)
        zkl = torch.where(stop < thr, zkl, torch.zeros_like(zkl))
        stop = stop + (1.0 - zp)
        act = stop < thr
        digits = digits + act.long()
        canvas = canvas + torch.where(act[:, None], zp[:, None] * wr, torch.zeros_like(wr))
        skl = 0.5 * ((((gclv - clv) - 1.0) + cvar / gcvar) + (cm - gcm) ** 2 / gcvar)[:, 0]
        gv = torch.exp(gslv)
        shkl = 0.5 * ((((gslv - slv) - 1.0) + svar / gv) + (sm - gsm) ** 2 / gv).sum(1)
        vkl = 0.5 * ((((vplv - lv) - 1.0) + torch.exp(lv) / cfg.vae_prior_variance) +
                     (mu - cfg.vae_prior_mean) ** 2 / cfg.vae_prior_variance).sum(1)
        mask = lambda v: torch.where(act, v, torch.zeros_like(v))  # noqa: E731
        lw = 1.0 if live else 0.0  # steps past the global exit contribute nothing
        for k, v in (("scale", s), ("shift", shift), ("zprob", zprob), ("zkl", zkl * lw),
                     ("skl", mask(skl) * lw), ("shkl", mask(shkl) * lw),
                     ("vkl", mask(vkl) * lw), ("prn", prn * lw)):
            rec[k].append(v)
        zprev, ssprev, hg_prev = zl, ss, hg
    Tx = steps
    S = {k: torch.stack(v[:Tx], 1) for k, v in rec.items()}  # [B, Tx, ...]
    elbo = S["zkl"].sum(1) + S["skl"].sum(1) + S["shkl"].sum(1) + S["vkl"].sum(1)
    kl = elbo
    if canvas_cotangent is None:
        rc = torch.clamp(canvas, 0.0, 1.0)
        bce = -(images * torch.log(rc + 1e-10) + (1.0 - images) * torch.log(1.0 - rc + 1e-10)).sum(1)
        elbo = elbo + bce
    Cf = float(C)
    sc = S["scale"] * Cf
    amin, amax = cfg.constrains_area_minmax
    area = (torch.clamp(amax - sc, min=0.0) + torch.clamp(sc - amin, min=0.0)).mean(1)
    cx = (S["shift"][..., 0] + 1.0) * Cf / 2.0
    cy = (S["shift"][..., 1] + 1.0) * Cf / 2.0
    outl = (torch.clamp(-(cx - 0.5 * sc), min=0) + torch.clamp(-(cy - 0.5 * sc), min=0) +
            torch.clamp(cx + 0.5 * sc - Cf, min=0) + torch.clamp(cy + 0.5 * sc - Cf, min=0)).sum(1)
    size = torch.clamp((sc[:, :, None] - sc[:, None, :]).abs() - 3.0, min=0).sum((1, 2))
    md = torch.maximum((cx[:, :, None] - cx[:, None, :]).abs(),
                       (cy[:, :, None] - cy[:, None, :]).abs())
    smean = (sc[:, :, None] + sc[:, None, :]) / 2.0
    eye = torch.eye(Tx, dtype=dt)
    over = (torch.clamp(smean - md, min=0) * (1.0 - eye)).sum((1, 2))
    pr = (S["prn"].sum(1) + cfg.constrains_area_gamma * area + over * cfg.constrains_bbox_gamma +
          outl * cfg.constrains_bbox_gamma + size * cfg.constrains_sharesize_gamma)
    margin = torch.zeros((), dtype=dt)
    elem = torch.zeros(B, dtype=dt)
    if cfg.constrains_margin_gamma > 1e-8:
        cons = list(cfg.constrains_num)
        obj = torch.tensor([[1.0 if t < k else 0.0 for t in range(Tx)] for k in cons], dtype=dt)
        mo = obj.mean(0)
        if zsum_reduce is None:
            pm = S["zprob"].mean(0)
        else:  # global value, gradient through this shard's own terms only
            zl = S["zprob"].sum(0)
            zg = torch.as_tensor(zsum_reduce(zl.detach().clone()), dtype=dt)
            pm = (zl + (zg - zl.detach())) / float(global_batch or B)
        margin = (_sce(mo, _logit8(pm)) * cfg.constrains_margin_gamma).sum()
        ce = _sce(obj[None], _logit8(S["zprob"])[:, None, :]).sum(2)
        elem = ce.min(1).values * cfg.constrains_num_element_gamma
    loss_b = elbo + pr + elem
    loss = loss_b.mean() * (B / float(global_batch or B)) + margin
    if canvas_cotangent is not None:
        loss = loss + (canvas_cotangent * canvas).sum()
    return {"loss": loss, "loss_b": loss_b, "kl": kl, "pr": pr, "T": Tx, "digits": digits, "canvas": canvas,
            "scale": S["scale"], "shift": S["shift"], "z_pres_prob": S["zprob"],
            "margin": margin, "element": elem, "area": area, "out": outl, "size": size,
            "overlap": over}

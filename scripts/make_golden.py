"""Generates the committed golden vectors under tests/golden/ from the CPU
oracle (oracle/air_ref.c forward, oracle/air_torch.py train step).

TensorFlow 1.12 — the reference's arithmetic — is not installed and the
reference ships no tests or fixtures, so these vectors pin
the oracle restatement itself (any later change to it or to the weight /
noise generators shows up as a golden mismatch) and give the GPU tests
committed expected outputs.  Weights are not stored: they are regenerated
from the recorded seeds by oracle.air_oracle.init_params (numpy
default_rng, platform independent), guarded by a recorded checksum.

usage: python scripts/make_golden.py   (writes tests/golden/*.npz)
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import air_oracle as ao  # noqa: E402
from oracle import air_torch as at  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
FWD_KEYS = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob", "z_pres_kl",
            "scale_kl", "shift_kl", "vae_kl", "canvas", "bce", "mse", "loss", "digits")


def param_checksum(P):
    return np.float64(sum(float(np.sum(P[n].astype(np.float64) * (i + 1)))
                          for i, n in enumerate(sorted(P))))


CASES = {
    # train model, 3 steps (BASELINE metric), all noise injected
    "air_fwd_train_b6": dict(cfg=dict(batch=6, max_steps=3, train=True), pseed=11, nseed=12,
                             xseed=13),
    # test model (rounded z_pres), 6 steps as the entry points, -ap prior
    "air_fwd_test_ap_b5": dict(cfg=dict(batch=5, max_steps=6, train=False, num_prior=(1, 3)),
                               pseed=21, nseed=22, xseed=23),
    # Multi-dSprites canvas (configs[3]: C = 64, multi_dsprites.py:391-392), train model
    "air_fwd_train_c64_b4": dict(cfg=dict(batch=4, max_steps=3, train=True, canvas_size=64),
                                 pseed=41, nseed=42, xseed=43, side=(22, 30)),
}


def make_forward(name, spec):
    cfg = ao.AirConfig(scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01, **spec["cfg"])
    P = ao.init_params(cfg, seed=spec["pseed"], bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=spec["nseed"])
    x, k = ao.synthetic_canvases(cfg.batch, canvas=cfg.canvas_size, seed=spec["xseed"],
                                 side=spec.get("side", (17, 23)))
    ref = ao.forward(cfg, P, nz, x, k)
    out = {"x": x, "targets": k, "param_seed": spec["pseed"], "param_checksum": param_checksum(P),
           "T": ref["T"], "loss_mean": ref["loss_mean"], "accuracy": ref["accuracy"]}
    for kname, v in nz.items():
        out["noise_" + kname] = v
    for kname in FWD_KEYS:
        out["out_" + kname] = ref[kname]
    for kname, v in spec["cfg"].items():
        out["cfg_" + kname] = np.asarray(v if v is not None else -1)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), **out)
    print(name, "T =", ref["T"], "loss", ref["loss_mean"], "digits", ref["digits"])


def make_adam_step():
    """One TF-Adam step (clip 1.0, lr 1e-4) of the float64 torch restatement
    (batch 4) under the well-conditioned canvas cotangent G (loss = mean KLs +
    <G, canvas>, DESIGN.md §Numerics: the BCE itself is bit-fragile at canvas
    pixels that are exactly 0, so an fp64 BCE gradient is not a stable
    target): the parameter deltas of the small tensors (heads, LSTM bias,
    VAE biases)."""
    cfg = ao.AirConfig(batch=4, max_steps=3, scale_prior_variance=0.05,
                       z_pres_prior_log_odds=-0.01)
    P0 = ao.init_params(cfg, seed=31, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=32)
    x, k = ao.synthetic_canvases(cfg.batch, seed=33)
    Gc = (np.random.default_rng(34).standard_normal((cfg.batch, 2500)) * 0.01).astype(np.float32)
    P = at.to_torch(P0, requires_grad=True)
    out = at.air_forward(cfg, P, at.to_torch(nz), torch.tensor(x, dtype=torch.float64),
                         z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                         canvas_cotangent=torch.tensor(Gc, dtype=torch.float64),
                         fixed_steps=True)
    out["loss"].backward()
    grads = {n: p.grad if p.grad is not None else torch.zeros_like(p) for n, p in P.items()}
    m = {n: torch.zeros_like(v) for n, v in P.items()}
    v = {n: torch.zeros_like(t) for n, t in P.items()}
    with torch.no_grad():
        at.tf_clip_adam_step(P, grads, m, v, 1, lr=1e-4, clip=1.0)
    res = {"x": x, "targets": k, "canvas_cotangent": Gc, "param_seed": 31,
           "param_checksum": param_checksum(P0), "loss": np.float64(out["loss"].detach())}
    for kname, val in nz.items():
        res["noise_" + kname] = val
    for n, t in P.items():
        if int(np.prod(t.shape)) <= 1100:
            res["delta_" + n.replace("/", "__")] = (t.detach().numpy() - P0[n].astype(np.float64))
    np.savez_compressed(os.path.join(OUT, "air_adam_step_b4.npz"), **res)
    print("air_adam_step_b4 loss", res["loss"], "deltas",
          sum(1 for kk in res if kk.startswith("delta_")))


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    ao.build()
    for n, s in CASES.items():
        make_forward(n, s)
    make_adam_step()

"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the AIR-ASR C oracle
(oracle/asr_ref.c) plus its parameter table, noise layout and defaults.

Only tests/ and tooling may import this module; the product never does.

Shapes follow air/air_number_bbox_location.py: inference LSTMCell on
[x, z_prev, shift/scale latents] (:403-412, :863-867), generative LSTMCell on
[z_prev, latents] (:457-463, :868-873), tf.layers.dense heads (:414-474,
:590-609), the glimpse VAE (vae.py:5-48).  Variable names are the TF scope
paths under "air/air_model" (dense layers numbered in creation order).
Hyper-parameters: train_air_pr.py:160-213 (threshold 0.9, temperature 0.1,
likelihood std 0.0, fixed scale prior -1 / 0.05).  Parity against TF-1.12 is
unpinned (TF absent, no reference tests or fixtures).
"""
from __future__ import annotations

import ctypes
import dataclasses
from typing import Dict, List, Optional, Tuple

import numpy as np

from . import air_oracle as ao

_FP = ao._FP


@dataclasses.dataclass
class AsrConfig:
    batch: int = 64
    canvas_size: int = 50
    windows_size: int = 28
    max_steps: int = 6
    rnn_units: int = 256
    vae_latent_dimensions: int = 50
    vae_recognition_units: Tuple[int, int] = (512, 256)
    vae_generative_units: Tuple[int, int] = (256, 512)
    scale_hidden_units: int = 64
    z_pres_hidden_units: int = 64
    train: bool = True
    vae_likelihood_std: float = 0.0
    stopping_threshold: float = 0.9
    z_pres_temperature: float = 0.1
    scale_prior_mean: float = -1.0
    scale_prior_variance: float = 0.05
    vae_prior_mean: float = 0.0
    vae_prior_variance: float = 1.0
    fix_steps: Optional[int] = None
    constrains_num: Tuple[int, ...] = (1, 3)
    constrains_num_gamma: float = 0.0
    constrains_margin_gamma: float = 0.0
    constrains_num_element_gamma: float = 0.0
    constrains_bbox_gamma: float = 0.0
    constrains_sharesize_gamma: float = 0.0
    constrains_area_gamma: float = 0.0
    constrains_area_minmax: Tuple[float, float] = (17.0, 23.0)


P_ROOT = "air/air_model/"


def param_specs(cfg: AsrConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """(TF variable name, shape) in asr_ref.c slot order."""
    C2, H, Z = cfg.canvas_size ** 2, cfg.rnn_units, cfg.vae_latent_dimensions
    W2 = cfg.windows_size ** 2
    HS, HZ = cfg.scale_hidden_units, cfg.z_pres_hidden_units
    R1, R2 = cfg.vae_recognition_units
    G1, G2 = cfg.vae_generative_units
    p = P_ROOT
    specs = [(p + "infer_rnn_running/kernel", (C2 + Z + 3 + H, 4 * H)),
             (p + "infer_rnn_running/bias", (4 * H,)),
             (p + "gen_rnn_running/kernel", (Z + 3 + H, 4 * H)),
             (p + "gen_rnn_running/bias", (4 * H,))]

    def four(scope, kin, kout, extra):
        return [(p + scope + "/dense/kernel", (kin, HS)), (p + scope + "/dense/bias", (HS,)),
                (p + scope + "/dense_1/kernel", (HS + extra, kout)),
                (p + scope + "/dense_1/bias", (kout,)),
                (p + scope + "/dense_2/kernel", (kin, HS)), (p + scope + "/dense_2/bias", (HS,)),
                (p + scope + "/dense_3/kernel", (HS + extra, kout)),
                (p + scope + "/dense_3/bias", (kout,))]

    specs += four("inf_shift", H, 2, 0)
    specs += four("inf_scale", H + 2, 1, 2)
    specs += four("gen_shift", H, 2, 0)
    for scope in ("z_pres/prior", "z_pres/log_odds"):
        specs += [(p + scope + "/dense/kernel", (H, HZ)), (p + scope + "/dense/bias", (HZ,)),
                  (p + scope + "/dense_1/kernel", (HZ, 1)), (p + scope + "/dense_1/bias", (1,))]
    v = p + "vae/"
    specs += [
        (v + "recognition_1/weights", (W2, R1)), (v + "recognition_1/biases", (R1,)),
        (v + "recognition_2/weights", (R1, R2)), (v + "recognition_2/biases", (R2,)),
        (v + "rec_mean/weights", (R2, Z)), (v + "rec_mean/biases", (Z,)),
        (v + "rec_log_variance/weights", (R2, Z)), (v + "rec_log_variance/biases", (Z,)),
        (v + "generative_1/weights", (Z, G1)), (v + "generative_1/biases", (G1,)),
        (v + "generative_2/weights", (G1, G2)), (v + "generative_2/biases", (G2,)),
        (v + "gen_mean/weights", (G2, W2)), (v + "gen_mean/biases", (W2,)),
    ]
    return specs


def init_params(cfg: AsrConfig, seed: int = 1235, bias_scale: float = 0.0):
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_specs(cfg):
        if len(shape) == 2:
            lim = np.sqrt(6.0 / (shape[0] + shape[1]))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = (rng.uniform(-bias_scale, bias_scale, size=shape).astype(np.float32)
                         if bias_scale > 0 else np.zeros(shape, np.float32))
    return out


def make_noise(cfg: AsrConfig, seed: int = 7) -> Dict[str, np.ndarray]:
    rng = np.random.default_rng(seed)
    T, B = cfg.max_steps, cfg.batch
    W2, Z = cfg.windows_size ** 2, cfg.vae_latent_dimensions
    f = np.float32
    return {"eps_shift": rng.standard_normal((T, B, 2)).astype(f),
            "eps_scale": rng.standard_normal((T, B)).astype(f),
            "eps_z": rng.standard_normal((T, B, Z)).astype(f),
            "eps_x": rng.standard_normal((T, B, W2)).astype(f),
            "u": rng.uniform(0.0, 1.0, (T, B)).astype(f)}


class _Cfg(ctypes.Structure):
    _fields_ = ([(n, ctypes.c_int) for n in
                 ("B", "C", "W", "max_steps", "H", "Z", "R1", "R2", "G1", "G2", "HS", "HZ",
                  "train", "fix_steps", "n_constrains")] +
                [("constrains", ctypes.c_int * 8)] +
                [(n, ctypes.c_float) for n in
                 ("lik_std", "thr", "temperature", "scale_prior_mean", "scale_prior_var",
                  "scale_prior_logvar", "vae_prior_mean", "vae_prior_var", "vae_prior_logvar",
                  "g_num", "g_margin", "g_element", "g_bbox", "g_size", "g_area", "area_min",
                  "area_max")])


class _Noise(ctypes.Structure):
    _fields_ = [(n, _FP) for n in ("eps_shift", "eps_scale", "eps_z", "eps_x", "u")]


_OUT = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob", "z_pres", "z_pres_kl",
        "scale_kl", "shift_kl", "vae_kl", "pr_num", "canvas", "bce", "mse", "elbo", "pr_loss",
        "element", "loss", "area", "out", "size", "overlap", "margin")
STEP_KEYS = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob", "z_pres",
             "z_pres_kl", "scale_kl", "shift_kl", "vae_kl", "pr_num")


class _Out(ctypes.Structure):
    _fields_ = [(n, _FP) for n in _OUT] + [("digits", ctypes.POINTER(ctypes.c_int))]


def _cfg(cfg: AsrConfig) -> _Cfg:
    c = _Cfg()
    c.B, c.C, c.W, c.max_steps = cfg.batch, cfg.canvas_size, cfg.windows_size, cfg.max_steps
    c.H, c.Z = cfg.rnn_units, cfg.vae_latent_dimensions
    c.R1, c.R2 = cfg.vae_recognition_units
    c.G1, c.G2 = cfg.vae_generative_units
    c.HS, c.HZ = cfg.scale_hidden_units, cfg.z_pres_hidden_units
    c.train = int(cfg.train)
    c.fix_steps = -1 if cfg.fix_steps is None else int(cfg.fix_steps)
    assert 1 <= len(cfg.constrains_num) <= 8
    c.n_constrains = len(cfg.constrains_num)
    for i, v in enumerate(cfg.constrains_num):
        c.constrains[i] = int(v)
    c.lik_std, c.thr, c.temperature = (cfg.vae_likelihood_std, cfg.stopping_threshold,
                                       cfg.z_pres_temperature)
    c.scale_prior_mean, c.scale_prior_var = cfg.scale_prior_mean, cfg.scale_prior_variance
    c.scale_prior_logvar = ao.f32log(cfg.scale_prior_variance)
    c.vae_prior_mean, c.vae_prior_var = cfg.vae_prior_mean, cfg.vae_prior_variance
    c.vae_prior_logvar = ao.f32log(cfg.vae_prior_variance)
    c.g_num, c.g_margin = cfg.constrains_num_gamma, cfg.constrains_margin_gamma
    c.g_element, c.g_bbox = cfg.constrains_num_element_gamma, cfg.constrains_bbox_gamma
    c.g_size, c.g_area = cfg.constrains_sharesize_gamma, cfg.constrains_area_gamma
    c.area_min, c.area_max = cfg.constrains_area_minmax
    return c


def forward(cfg: AsrConfig, params, noise, images, targets=None) -> Dict[str, np.ndarray]:
    lib = ao._load()
    lib.oracle_asr_forward.restype = ctypes.c_int
    B, T = cfg.batch, cfg.max_steps
    C2, W2, Z = cfg.canvas_size ** 2, cfg.windows_size ** 2, cfg.vae_latent_dimensions
    images = np.ascontiguousarray(images, np.float32).reshape(B, C2)
    c = _cfg(cfg)
    specs = param_specs(cfg)
    plist = [np.ascontiguousarray(params[n], np.float32) for n, _ in specs]
    for (n, shp), a in zip(specs, plist):
        assert a.shape == tuple(shp), (n, a.shape, shp)
    parr = (_FP * len(plist))(*[a.ctypes.data_as(_FP) for a in plist])
    nzk = {k: np.ascontiguousarray(noise[k], np.float32)
           for k in ("eps_shift", "eps_scale", "eps_z", "eps_x", "u")}
    nz = _Noise(*[nzk[k].ctypes.data_as(_FP)
                  for k in ("eps_shift", "eps_scale", "eps_z", "eps_x", "u")])
    shapes = {"scale": (T, B), "shift": (T, B, 2), "st_back": (T, B, 6), "window": (T, B, W2),
              "latent": (T, B, Z), "z_pres_prob": (T, B), "z_pres": (T, B), "z_pres_kl": (T, B),
              "scale_kl": (T, B), "shift_kl": (T, B), "vae_kl": (T, B), "pr_num": (T, B),
              "canvas": (B, C2), "bce": (B,), "mse": (B,), "elbo": (B,), "pr_loss": (B,),
              "element": (B,), "loss": (B,), "area": (B,), "out": (B,), "size": (B,),
              "overlap": (B,), "margin": (1,)}
    res = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
    res["digits"] = np.zeros(B, np.int32)
    out = _Out(*([res[k].ctypes.data_as(_FP) for k in _OUT] +
                 [res["digits"].ctypes.data_as(ctypes.POINTER(ctypes.c_int))]))
    tg = None if targets is None else np.ascontiguousarray(targets, np.int32)
    acc = ctypes.c_float(0.0)
    texec = lib.oracle_asr_forward(ctypes.byref(c), parr, ctypes.byref(nz),
                                   images.ctypes.data_as(_FP),
                                   None if tg is None else tg.ctypes.data_as(
                                       ctypes.POINTER(ctypes.c_int)),
                                   ctypes.byref(out), ctypes.byref(acc))
    for k in STEP_KEYS:
        res[k] = res[k][:texec]
    res["T"] = int(texec)
    res["accuracy"] = float(acc.value)
    res["margin"] = float(res["margin"][0])
    res["loss_mean"] = float(np.float32(np.mean(res["loss"], dtype=np.float32)) +
                             np.float32(res["margin"]))
    return res

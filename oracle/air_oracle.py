"""TEST INFRASTRUCTURE ONLY — ctypes front-end of the C restatement oracle.

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline leg
may import this module.  The product (``mog-asr_amd/mog_air``) never does.

It owns an *independent* statement of the reference's parameter shapes and
hyper-parameters so the parity tests can map product parameters onto the
oracle by TF variable name:

* parameter shapes: ``air/air_model.py:454-498,594-600`` (LSTM kernel
  ``[C*C+H, 4H]``, heads fc 256->64->k), ``air/vae.py:15-46``;
* AIR-baseline hyper-parameters: ``training_air_original.py:158-209``;
* annealed z_pres prior: ``air/air_model.py:164-184`` with the schedule at
  ``training_air_original.py:193-201``.

Parity against TF-1.12 is unpinned (TF is absent and the reference ships no
tests or golden files — SURVEY.md §4, §8c).  The oracle is pinned instead by
known-answer properties of the reference STN (tests/test_oracle.py) and by an
independent float64 torch restatement (oracle/air_torch.py).
"""
from __future__ import annotations

import ctypes
import dataclasses
import os
import subprocess
from typing import Dict, List, Optional, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liboracle_air.so")


@dataclasses.dataclass
class AirConfig:
    """Hyper-parameters of one AIRModel (reference kwargs, air_model.py:15-51)."""

    batch: int = 64
    canvas_size: int = 50
    windows_size: int = 28
    max_steps: int = 3
    rnn_units: int = 256
    vae_latent_dimensions: int = 50
    vae_recognition_units: Tuple[int, int] = (512, 256)
    vae_generative_units: Tuple[int, int] = (256, 512)
    scale_hidden_units: int = 64
    shift_hidden_units: int = 64
    z_pres_hidden_units: int = 64
    train: bool = True
    vae_likelihood_std: float = 0.3
    stopping_threshold: float = 0.99
    z_pres_temperature: float = 1.0
    scale_prior_mean: float = -1.0
    scale_prior_variance: float = 0.05
    shift_prior_mean: float = 0.0
    shift_prior_variance: float = 1.0
    vae_prior_mean: float = 0.0
    vae_prior_variance: float = 1.0
    z_pres_prior_log_odds: float = -0.01
    num_prior: Optional[Tuple[int, ...]] = None


def annealed_log_odds(global_step: int, init=10000.0, factor=0.1, iters=3000,
                      vmin=1e-9) -> np.float32:
    """tf.train.exponential_decay (non-staircase) + max + log(v + 1e-9) in fp32
    (air_model.py:164-184; schedule training_air_original.py:193-201)."""
    f32 = np.float32
    p = f32(global_step) / f32(iters)
    v = f32(init) * np.power(f32(factor), p, dtype=np.float32)
    v = np.maximum(v, f32(vmin))
    return np.log(v + f32(1e-9), dtype=np.float32)


def marginal_objective(num_prior, max_steps) -> np.ndarray:
    """air_model.py:86-107 (the ``-ap`` prior)."""
    objective = np.zeros([max_steps])
    buffer = 1.0 - 1.0 / len(num_prior)
    for ind in range(max_steps):
        if ind not in num_prior and ind < max(num_prior):
            objective[ind] = 1.0
        else:
            if ind == max(num_prior):
                break
            objective[ind] = buffer
            if ind in num_prior:
                buffer -= 1.0 / len(num_prior)
    for ind in range(max_steps):
        if objective[ind] == 1.0:
            objective[ind] = 100
        elif objective[ind] == 0.0:
            objective[ind] = -100.0
        else:
            objective[ind] = np.log(objective[ind] / (1.0 - objective[ind]))
    return objective.astype(np.float32)


def param_specs(cfg: AirConfig) -> List[Tuple[str, Tuple[int, ...]]]:
    """(TF variable name, shape) in the oracle's slot order (air_ref.c enum).

    Names are the ones the reference's scopes produce: the loop body runs
    inside ``variable_scope("air")`` -> ``variable_scope("rnn")``
    (air_model.py:127,812-851)."""
    C2 = cfg.canvas_size ** 2
    H = cfg.rnn_units
    W2 = cfg.windows_size ** 2
    R1, R2 = cfg.vae_recognition_units
    G1, G2 = cfg.vae_generative_units
    Z = cfg.vae_latent_dimensions
    HS, HZ = cfg.scale_hidden_units, cfg.z_pres_hidden_units
    HH = cfg.shift_hidden_units
    assert HS == HH, "oracle assumes equal scale/shift hidden widths"
    p = "air/rnn/"
    specs = [
        (p + "rnn/basic_lstm_cell/kernel", (C2 + H, 4 * H)),
        (p + "rnn/basic_lstm_cell/bias", (4 * H,)),
    ]
    for head, k in (("scale/mean", 1), ("scale/log_variance", 1),
                    ("shift/mean", 2), ("shift/log_variance", 2)):
        specs += [
            (p + head + "/hidden/weights", (H, HS)),
            (p + head + "/hidden/biases", (HS,)),
            (p + head + "/output/weights", (HS, k)),
            (p + head + "/output/biases", (k,)),
        ]
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
    specs += [
        (p + "z_pres/log_odds/hidden/weights", (H, HZ)),
        (p + "z_pres/log_odds/hidden/biases", (HZ,)),
        (p + "z_pres/log_odds/output/weights", (HZ, 1)),
        (p + "z_pres/log_odds/output/biases", (1,)),
    ]
    return specs


def init_params(cfg: AirConfig, seed: int = 1235, bias_scale: float = 0.0
                ) -> Dict[str, np.ndarray]:
    """Glorot/Xavier-uniform kernels (TF default for BasicLSTMCell and
    contrib fully_connected), zero biases unless ``bias_scale`` > 0 (tests use
    non-zero biases so bias paths are exercised)."""
    rng = np.random.default_rng(seed)
    out = {}
    for name, shape in param_specs(cfg):
        if len(shape) == 2:
            lim = np.sqrt(6.0 / (shape[0] + shape[1]))
            out[name] = rng.uniform(-lim, lim, size=shape).astype(np.float32)
        else:
            out[name] = (rng.uniform(-bias_scale, bias_scale, size=shape)
                         .astype(np.float32) if bias_scale > 0
                         else np.zeros(shape, np.float32))
    return out


def make_noise(cfg: AirConfig, seed: int = 7) -> Dict[str, np.ndarray]:
    """Injected noise for the 5 random draws per step (SURVEY.md §7 'RNG')."""
    rng = np.random.default_rng(seed)
    T, B = cfg.max_steps, cfg.batch
    W2, Z = cfg.windows_size ** 2, cfg.vae_latent_dimensions
    f = np.float32
    return {
        "eps_scale": rng.standard_normal((T, B)).astype(f),
        "eps_shift": rng.standard_normal((T, B, 2)).astype(f),
        "eps_z": rng.standard_normal((T, B, Z)).astype(f),
        "eps_x": rng.standard_normal((T, B, W2)).astype(f),
        "u": rng.uniform(0.0, 1.0, (T, B)).astype(f),
    }


def synthetic_canvases(batch: int, canvas: int = 50, seed: int = 1234,
                       counts=(1, 3), side=(17, 23)) -> Tuple[np.ndarray, np.ndarray]:
    """Multi-MNIST-like synthetic canvases: K glyphs of
    side U{17..23} px, pixel values U(0,1) thresholded below 0.05
    (multi_mnist.py:155), clipped to [0,1]."""
    rng = np.random.default_rng(seed)
    imgs = np.zeros((batch, canvas, canvas), np.float32)
    ks = rng.integers(counts[0], counts[1] + 1, size=batch)
    for b in range(batch):
        for _ in range(ks[b]):
            s = int(rng.integers(side[0], side[1] + 1))
            y = int(rng.integers(0, canvas - s + 1))
            x = int(rng.integers(0, canvas - s + 1))
            g = rng.uniform(0.0, 1.0, (s, s)).astype(np.float32)
            # stroke-like sparsity: keep ~35% of the glyph box
            g = np.where(rng.uniform(size=(s, s)) < 0.35, g, 0.0)
            g = np.where(g >= 0.05, g, 0.0)
            imgs[b, y:y + s, x:x + s] += g
    imgs = np.clip(imgs, 0.0, 1.0).reshape(batch, canvas * canvas)
    return imgs.astype(np.float32), ks.astype(np.int32)


# ---------------------------------------------------------------- ctypes ---

class _Cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in
                ("B", "C", "W", "max_steps", "H", "Z", "R1", "R2", "G1", "G2", "HS", "HZ",
                 "train", "use_num_prior")] + \
               [(n, ctypes.c_float) for n in
                ("lik_std", "thr", "temperature", "scale_prior_mean", "scale_prior_var",
                 "scale_prior_logvar", "shift_prior_mean", "shift_prior_var",
                 "shift_prior_logvar", "vae_prior_mean", "vae_prior_var",
                 "vae_prior_logvar", "z_pres_prior_log_odds")] + \
               [("marginal_objective", ctypes.POINTER(ctypes.c_float))]


_FP = ctypes.POINTER(ctypes.c_float)


class _Noise(ctypes.Structure):
    _fields_ = [(n, _FP) for n in ("eps_scale", "eps_shift", "eps_z", "eps_x", "u")]


_OUT_FIELDS = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob",
               "z_pres_kl", "scale_kl", "shift_kl", "vae_kl", "glimpse", "z_pres", "mu",
               "logvar", "h", "canvas", "recon", "bce", "mse", "running_loss", "loss")


STEP_KEYS = ("scale", "shift", "st_back", "window", "latent", "z_pres_prob", "z_pres_kl",
             "scale_kl", "shift_kl", "vae_kl", "glimpse", "z_pres", "mu", "logvar", "h")


class _Out(ctypes.Structure):
    _fields_ = [(n, _FP) for n in _OUT_FIELDS] + [("digits", ctypes.POINTER(ctypes.c_int))]


_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def _load():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.oracle_air_forward.restype = ctypes.c_int
        _lib.oracle_stn.restype = None
        _lib.oracle_concrete_kl.restype = ctypes.c_float
        _lib.oracle_concrete_kl.argtypes = [ctypes.c_float] * 5
    return _lib


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_FP)


def f32log(v: float) -> np.float32:
    """tf.log(python_float) evaluated in fp32 (air_model.py:133-138)."""
    return np.log(np.float32(v), dtype=np.float32)


def stn(U: np.ndarray, theta: np.ndarray, out_hw: Tuple[int, int]) -> np.ndarray:
    """Reference STN for a batch: U [N,Hin,Win], theta [N,6] -> [N,Hout,Wout]."""
    lib = _load()
    U = np.ascontiguousarray(U, np.float32)
    theta = np.ascontiguousarray(theta, np.float32).reshape(-1, 6)
    N, Hin, Win = U.shape
    out = np.zeros((N, out_hw[0], out_hw[1]), np.float32)
    for n in range(N):
        lib.oracle_stn(_ptr(U[n]), ctypes.c_int(Hin), ctypes.c_int(Win), _ptr(theta[n]),
                       ctypes.c_int(out_hw[0]), ctypes.c_int(out_hw[1]), _ptr(out[n]))
    return out


def dense_chain(x: np.ndarray, w: np.ndarray, b: Optional[np.ndarray] = None) -> np.ndarray:
    """out = chain_k(x w) (+ b): one fp32 fma chain per output in k order."""
    lib = _load()
    x = np.ascontiguousarray(x, np.float32)
    w = np.ascontiguousarray(w, np.float32)
    B, K = x.shape
    N = w.shape[1]
    out = np.zeros((B, N), np.float32)
    bb = None if b is None else np.ascontiguousarray(b, np.float32)
    lib.oracle_dense(_ptr(x), ctypes.c_int(B), ctypes.c_int(K), _ptr(w),
                     None if bb is None else _ptr(bb), ctypes.c_int(N), _ptr(out))
    return out


def concrete_kl(y, plo, pT, qlo, qT) -> float:
    return float(_load().oracle_concrete_kl(y, plo, pT, qlo, qT))


def forward(cfg: AirConfig, params: Dict[str, np.ndarray], noise: Dict[str, np.ndarray],
            images: np.ndarray, targets: Optional[np.ndarray] = None,
            z_pres_prior_log_odds: Optional[float] = None) -> Dict[str, np.ndarray]:
    """Run the reference forward loop. Returns [T_exec, B, ...]-shaped step
    records plus per-image results; ``T`` = executed steps."""
    lib = _load()
    B, T = cfg.batch, cfg.max_steps
    C2, W2 = cfg.canvas_size ** 2, cfg.windows_size ** 2
    Z, H = cfg.vae_latent_dimensions, cfg.rnn_units
    images = np.ascontiguousarray(images, np.float32).reshape(B, C2)
    c, mo = _make_cfg(cfg, z_pres_prior_log_odds)
    specs = param_specs(cfg)
    plist = [np.ascontiguousarray(params[n], np.float32) for n, _ in specs]
    for (n, shp), a in zip(specs, plist):
        assert a.shape == tuple(shp), (n, a.shape, shp)
    parr = (_FP * len(plist))(*[_ptr(a) for a in plist])
    nzk = {k: np.ascontiguousarray(v, np.float32) for k, v in noise.items()}
    nz = _Noise(*[_ptr(nzk[k]) for k in ("eps_scale", "eps_shift", "eps_z", "eps_x", "u")])
    return _run_forward(lib, cfg, c, parr, nz, images, targets, B, T, C2, W2, Z, H, mo)


def generate(cfg: AirConfig, params: Dict[str, np.ndarray], noise: Dict[str, np.ndarray],
             batch: int, n_steps: int) -> Dict[str, np.ndarray]:
    """Generation loop (air_model.py:1001-1146): canvas [G, C2] and the
    backward transforms [n_steps, G, 6] for injected prior noise
    (eps_scale [T,G], eps_shift [T,G,2], eps_z [T,G,Z], eps_x [T,G,W2])."""
    lib = _load()
    c, _ = _make_cfg(cfg, None)
    specs = param_specs(cfg)
    plist = [np.ascontiguousarray(params[n], np.float32) for n, _ in specs]
    parr = (_FP * len(plist))(*[_ptr(a) for a in plist])
    nzk = {k: np.ascontiguousarray(noise[k], np.float32)
           for k in ("eps_scale", "eps_shift", "eps_z", "eps_x")}
    dummy = np.zeros(1, np.float32)
    nz = _Noise(*[_ptr(nzk[k]) for k in ("eps_scale", "eps_shift", "eps_z", "eps_x")] +
                [_ptr(dummy)])
    canvas = np.zeros((batch, cfg.canvas_size ** 2), np.float32)
    st = np.zeros((n_steps, batch, 6), np.float32)
    lib.oracle_air_generate(ctypes.byref(c), parr, ctypes.byref(nz), ctypes.c_int(batch),
                            ctypes.c_int(n_steps), _ptr(canvas), _ptr(st))
    return {"canvas": canvas, "st_back": st, "digits": np.full(batch, n_steps, np.int32)}


def _make_cfg(cfg: AirConfig, z_pres_prior_log_odds):
    B, T = cfg.batch, cfg.max_steps
    Z, H = cfg.vae_latent_dimensions, cfg.rnn_units
    c = _Cfg()
    c.B, c.C, c.W, c.max_steps, c.H, c.Z = B, cfg.canvas_size, cfg.windows_size, T, H, Z
    c.R1, c.R2 = cfg.vae_recognition_units
    c.G1, c.G2 = cfg.vae_generative_units
    c.HS, c.HZ = cfg.scale_hidden_units, cfg.z_pres_hidden_units
    c.train = int(cfg.train)
    c.lik_std, c.thr, c.temperature = (cfg.vae_likelihood_std, cfg.stopping_threshold,
                                       cfg.z_pres_temperature)
    c.scale_prior_mean, c.scale_prior_var = cfg.scale_prior_mean, cfg.scale_prior_variance
    c.scale_prior_logvar = f32log(cfg.scale_prior_variance)
    c.shift_prior_mean, c.shift_prior_var = cfg.shift_prior_mean, cfg.shift_prior_variance
    c.shift_prior_logvar = f32log(cfg.shift_prior_variance)
    c.vae_prior_mean, c.vae_prior_var = cfg.vae_prior_mean, cfg.vae_prior_variance
    c.vae_prior_logvar = f32log(cfg.vae_prior_variance)
    c.z_pres_prior_log_odds = (cfg.z_pres_prior_log_odds if z_pres_prior_log_odds is None
                               else z_pres_prior_log_odds)
    mo = None
    if cfg.num_prior is not None:
        mo = marginal_objective(cfg.num_prior, T)
        c.use_num_prior = 1
        c.marginal_objective = _ptr(mo)
    else:
        c.use_num_prior = 0
    return c, mo


def _run_forward(lib, cfg, c, parr, nz, images, targets, B, T, C2, W2, Z, H, mo):
    shapes = {
        "scale": (T, B), "shift": (T, B, 2), "st_back": (T, B, 6), "window": (T, B, W2),
        "latent": (T, B, Z), "z_pres_prob": (T, B), "z_pres_kl": (T, B),
        "scale_kl": (T, B), "shift_kl": (T, B), "vae_kl": (T, B), "glimpse": (T, B, W2),
        "z_pres": (T, B), "mu": (T, B, Z), "logvar": (T, B, Z), "h": (T, B, H),
        "canvas": (B, C2), "recon": (B, C2), "bce": (B,), "mse": (B,),
        "running_loss": (B,), "loss": (B,),
    }
    res = {k: np.zeros(s, np.float32) for k, s in shapes.items()}
    res["digits"] = np.zeros(B, np.int32)
    out = _Out(*([_ptr(res[k]) for k in _OUT_FIELDS] +
                 [res["digits"].ctypes.data_as(ctypes.POINTER(ctypes.c_int))]))
    tg = None if targets is None else np.ascontiguousarray(targets, np.int32)
    acc = ctypes.c_float(0.0)
    texec = lib.oracle_air_forward(
        ctypes.byref(c), parr, ctypes.byref(nz), _ptr(images),
        None if tg is None else tg.ctypes.data_as(ctypes.POINTER(ctypes.c_int)),
        ctypes.byref(out), ctypes.byref(acc))
    for k in STEP_KEYS:
        res[k] = res[k][:texec]
    res["T"] = int(texec)
    res["accuracy"] = float(acc.value)
    res["loss_mean"] = float(np.mean(res["loss"], dtype=np.float32))
    res["mse_mean"] = float(np.mean(res["mse"], dtype=np.float32))
    return res

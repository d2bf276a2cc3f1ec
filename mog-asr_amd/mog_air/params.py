"""Parameter store of one AIR scope: every trainable variable of the reference
lives in ONE flat fp32 HBM buffer (params), with gradients, Adam moments and
the per-tensor table the fused clip+Adam kernel walks.

Variable names and shapes restate the reference: LSTM kernel/bias of
BasicLSTMCell (air_model.py:812-815, [C*C+H, 4H]), the four scale/shift heads
and the z_pres head (fc 256->64 relu -> fc k, air_model.py:458-498,594-600)
and the glimpse VAE (vae.py:15-46).  The body of the reference while-loop runs
under variable_scope("air")/("rnn") (air_model.py:127,812), hence the
``air/rnn/`` prefix.  Tensors are stored in TF layout ([in, out] row-major) and
each starts on a 256-byte boundary for vector loads.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np
import torch

from . import _lib

ALIGN = 64  # floats


def param_specs(C2: int, H: int, W2: int, R: Tuple[int, int], G: Tuple[int, int], Z: int,
                HS: int, HZ: int) -> List[Tuple[str, Tuple[int, ...]]]:
    p = "air/rnn/"
    specs = [(p + "rnn/basic_lstm_cell/kernel", (C2 + H, 4 * H)),
             (p + "rnn/basic_lstm_cell/bias", (4 * H,))]
    for head, k in (("scale/mean", 1), ("scale/log_variance", 1), ("shift/mean", 2),
                    ("shift/log_variance", 2)):
        specs += [(p + head + "/hidden/weights", (H, HS)), (p + head + "/hidden/biases", (HS,)),
                  (p + head + "/output/weights", (HS, k)), (p + head + "/output/biases", (k,))]
    v = p + "vae/"
    R1, R2 = R
    G1, G2 = G
    specs += [(v + "recognition_1/weights", (W2, R1)), (v + "recognition_1/biases", (R1,)),
              (v + "recognition_2/weights", (R1, R2)), (v + "recognition_2/biases", (R2,)),
              (v + "rec_mean/weights", (R2, Z)), (v + "rec_mean/biases", (Z,)),
              (v + "rec_log_variance/weights", (R2, Z)),
              (v + "rec_log_variance/biases", (Z,)),
              (v + "generative_1/weights", (Z, G1)), (v + "generative_1/biases", (G1,)),
              (v + "generative_2/weights", (G1, G2)), (v + "generative_2/biases", (G2,)),
              (v + "gen_mean/weights", (G2, W2)), (v + "gen_mean/biases", (W2,))]
    specs += [(p + "z_pres/log_odds/hidden/weights", (H, HZ)),
              (p + "z_pres/log_odds/hidden/biases", (HZ,)),
              (p + "z_pres/log_odds/output/weights", (HZ, 1)),
              (p + "z_pres/log_odds/output/biases", (1,))]
    return specs


class ParamStore:
    """Flat parameters + grads + Adam state for one scope (shared on reuse)."""

    def __init__(self, specs, device, seed: int = 1235, pad: Dict[str, int] = None):
        """pad[name]: zero elements kept behind variable `name` (not part of
        any variable: no view, optimizer entry or checkpoint covers them), for
        kernels that read / accumulate a few rows past a matrix (the AIR-ASR
        LSTM kernels at the 16-byte-aligned packed-row count)."""
        self.specs = list(specs)
        self.device = device
        self._views: Dict[Tuple[str, str], Tuple[torch.Tensor, torch.Tensor]] = {}
        self.offsets: Dict[str, int] = {}
        self.shapes: Dict[str, Tuple[int, ...]] = {}
        pad = dict(pad or {})
        off = 0
        for name, shape in self.specs:
            self.offsets[name] = off
            self.shapes[name] = tuple(shape)
            n = int(np.prod(shape)) + pad.get(name, 0)
            off += (n + ALIGN - 1) // ALIGN * ALIGN
        self.total = off
        self.n_params = sum(int(np.prod(s)) for _, s in self.specs)
        f32 = dict(device=device, dtype=torch.float32)
        self.flat = torch.zeros(self.total, **f32)
        self.grad = torch.zeros(self.total, **f32)
        self.m = torch.zeros(self.total, **f32)
        self.v = torch.zeros(self.total, **f32)
        self.global_step = 0
        self.version = 0  # bumped on every parameter write (bf16 packs key on it)
        self.adam_t = 0
        self.beta1_power = np.float32(0.9)
        self.beta2_power = np.float32(0.999)
        self._build_optim_table()
        self.init_glorot(seed)

    # ------------------------------------------------------------ views ---
    def view(self, name: str, buf: str = "flat") -> torch.Tensor:
        """View of one variable inside a flat buffer.  Cached per (buffer,
        name) while the buffer object stays the same: the train step asks for
        ~100 views per step, and at the reference's batch of 64 the host-side
        launch sequence, not the GPU, sets the step time."""
        t = getattr(self, buf)
        key = (buf, name)
        hit = self._views.get(key)
        if hit is not None and hit[0] is t:
            return hit[1]
        o = self.offsets[name]
        shape = self.shapes[name]
        v = t[o:o + int(np.prod(shape))].view(shape)
        self._views[key] = (t, v)
        return v

    def g(self, name: str) -> torch.Tensor:
        return self.view(name, "grad")

    # ------------------------------------------------------------ init ----
    def init_glorot(self, seed: int) -> None:
        """Xavier/Glorot-uniform kernels, zero biases (TF defaults of
        BasicLSTMCell and contrib.layers.fully_connected)."""
        rng = np.random.default_rng(seed)
        host = np.zeros(self.total, np.float32)
        for name, shape in self.specs:
            o = self.offsets[name]
            n = int(np.prod(shape))
            if len(shape) == 2:
                lim = np.sqrt(6.0 / (shape[0] + shape[1]))
                host[o:o + n] = rng.uniform(-lim, lim, n).astype(np.float32)
        self.flat.copy_(torch.from_numpy(host))
        self.version += 1

    def load_dict(self, d: Dict[str, np.ndarray]) -> None:
        host = self.flat.detach().cpu().numpy().copy()
        for name, shape in self.specs:
            if name in d:
                a = np.asarray(d[name], np.float32)
                assert a.shape == shape, (name, a.shape, shape)
                o = self.offsets[name]
                host[o:o + a.size] = a.reshape(-1)
        self.flat.copy_(torch.from_numpy(host))
        self.version += 1

    def state_dict(self) -> Dict[str, np.ndarray]:
        host = self.flat.detach().cpu().numpy()
        out = {}
        for name, shape in self.specs:
            o = self.offsets[name]
            out[name] = host[o:o + int(np.prod(shape))].reshape(shape).copy()
        return out

    def grad_dict(self) -> Dict[str, np.ndarray]:
        host = self.grad.detach().cpu().numpy()
        return {name: host[self.offsets[name]:self.offsets[name] + int(np.prod(s))]
                .reshape(s).copy() for name, s in self.specs}

    # ------------------------------------------------------- optimizer ----
    def _build_optim_table(self) -> None:
        chunk = _lib.load().mog_optim_chunk_elems()
        offs, lens, btens, bstart = [], [], [], []
        for i, (name, shape) in enumerate(self.specs):
            n = int(np.prod(shape))
            offs.append(self.offsets[name])
            lens.append(n)
            for c0 in range(0, n, chunk):
                btens.append(i)
                bstart.append(c0)
        dev = self.device
        self.t_off = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.t_len = torch.tensor(lens, dtype=torch.int64, device=dev)
        self.t_bt = torch.tensor(btens, dtype=torch.int32, device=dev)
        self.t_bs = torch.tensor(bstart, dtype=torch.int64, device=dev)
        self.n_blocks = len(btens)
        # per-chunk sums of squares (clip_adam scratch: one per block)
        self.sumsq = torch.zeros(self.n_blocks, dtype=torch.float32, device=dev)

    def apply_adam(self, lr: float, clip, beta1=0.9, beta2=0.999, eps=1e-8) -> None:
        """TF AdamOptimizer.apply_gradients after the reference's per-tensor
        sanitize + clip_by_norm (air_model.py:944-999).  beta powers are fp32
        variables starting at beta (t = 1) and multiplied after each update."""
        from . import ops  # noqa: F401  (registers torch.ops.mog_air)
        lr_t = np.float32(lr) * np.sqrt(np.float32(1) - self.beta2_power,
                                        dtype=np.float32) / (np.float32(1) - self.beta1_power)
        # clip None (gradient_clipping_norm=None): the reference applies the
        # gradients as they are, without NaN/Inf zeroing (air_model.py:948)
        torch.ops.mog_air.clip_adam_(self.flat, self.grad, self.m, self.v, self.t_off, self.t_len,
                                     self.t_bt, self.t_bs, self.n_blocks,
                                     self.sumsq if clip is not None else None,
                                     float(clip) if clip is not None else 0.0, float(lr_t),
                                     float(beta1), float(beta2), float(eps))
        self.beta1_power = np.float32(self.beta1_power * np.float32(beta1))
        self.beta2_power = np.float32(self.beta2_power * np.float32(beta2))
        self.adam_t += 1
        self.version += 1

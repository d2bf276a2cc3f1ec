"""PyTorch-ROCm custom ops over the HIP kernels: the
``mog_air::`` operator namespace, so the hot-path pieces are callable (and
differentiable) from ordinary torch code the way the reference's TF graph
uses transformer() / vae() / BasicLSTMCell / AdamOptimizer.  Each op launches
the same HIP kernel the AIRModel host drives through the C ABI, on torch's
current HIP stream; there is no CPU implementation (a CPU tensor raises).

    import mog_air.torch_ops                          # registers the ops
    g = torch.ops.mog_air.stn(canvas, theta, 28, 28)  # transformer() read
    g.sum().backward()                                # mog_stn_backward

Ops (reference counterpart):
  stn(U[N,Hin,Win] f32, theta[N,6], Hout, Wout) -> [N,Hout,Wout]   transformer.py:18-175
  stn_accumulate_(canvas[N,C*C], U, theta, z[N], mask[N]) (in place)  air_model.py:580-588,665-675
  lstm_cell(G[B,4H], c_prev[B,H]) -> (c, h)                         BasicLSTMCell gates
  dense(x, W, b, act) -> act(x W + b)  act: 0 none, 1 relu, 2 softplus  fully_connected
  tf_adam_clip_(flat params, grads, m, v, lr, clip, beta1, beta2, eps, step)  air_model.py:941-999
"""
from __future__ import annotations

from typing import Tuple

import torch

from . import _lib, ops
from .ops import EPI_RELU, EPI_SOFTPLUS, EPI_STORE, dp, stream_ptr


def _need_hip(*ts):
    for t in ts:
        if t.device.type != "cuda":
            raise RuntimeError("mog_air ops run on a HIP device only (no CPU implementation)")
        if t.dtype != torch.float32 or not t.is_contiguous():
            raise ValueError("mog_air ops take contiguous float32 tensors")


# ------------------------------------------------------------------ STN ----
@torch.library.custom_op("mog_air::stn", mutates_args=())
def stn(U: torch.Tensor, theta: torch.Tensor, Hout: int, Wout: int) -> torch.Tensor:
    _need_hip(U, theta)
    N, Hin, Win = U.shape
    out = torch.empty((N, Hout * Wout), device=U.device, dtype=torch.float32)
    _lib.call("mog_stn_forward", dp(U), N, Hin, Win, dp(theta), Hout, Wout, dp(out), None, None,
              0, stream_ptr())
    return out.view(N, Hout, Wout)


@stn.register_fake
def _(U, theta, Hout, Wout):
    return U.new_empty((U.shape[0], Hout, Wout))


@torch.library.custom_op("mog_air::stn_backward", mutates_args=())
def stn_backward(U: torch.Tensor, theta: torch.Tensor, G: torch.Tensor
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    _need_hip(U, theta, G)
    N, Hin, Win = U.shape
    Ho, Wo = G.shape[1], G.shape[2]
    dU, dth, _ = ops.stn_backward(U.reshape(N, Hin * Win), theta, (Ho, Wo), G.contiguous())
    return dU.view(N, Hin, Win), dth


@stn_backward.register_fake
def _(U, theta, G):
    return U.new_empty(U.shape), theta.new_empty(theta.shape)


def _stn_setup(ctx, inputs, output):
    U, theta, _, _ = inputs
    ctx.save_for_backward(U, theta)


def _stn_bwd(ctx, grad):
    U, theta = ctx.saved_tensors
    dU, dth = torch.ops.mog_air.stn_backward(U, theta, grad.contiguous())
    return dU, dth, None, None


stn.register_autograd(_stn_bwd, setup_context=_stn_setup)


@torch.library.custom_op("mog_air::stn_accumulate_", mutates_args=("canvas",))
def stn_accumulate_(canvas: torch.Tensor, U: torch.Tensor, theta: torch.Tensor, z: torch.Tensor,
                    mask: torch.Tensor) -> None:
    _need_hip(canvas, U, theta, z, mask)
    N, Hin, Win = U.shape
    C2 = canvas.shape[1]
    C = int(round(C2 ** 0.5))
    _lib.call("mog_stn_forward", dp(U), N, Hin, Win, dp(theta), C, C, dp(canvas), dp(z),
              dp(mask), 1, stream_ptr())


# ----------------------------------------------------------------- LSTM ----
@torch.library.custom_op("mog_air::lstm_cell", mutates_args=())
def lstm_cell(G: torch.Tensor, c_prev: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    _need_hip(G, c_prev)
    B, H = c_prev.shape
    c = torch.empty_like(c_prev)
    h = torch.empty_like(c_prev)
    _lib.call("mog_lstm_cell_forward", dp(G), None, dp(c_prev), dp(c), dp(h), B, H, stream_ptr())
    return c, h


@lstm_cell.register_fake
def _(G, c_prev):
    return c_prev.new_empty(c_prev.shape), c_prev.new_empty(c_prev.shape)


@torch.library.custom_op("mog_air::lstm_cell_backward", mutates_args=())
def lstm_cell_backward(G: torch.Tensor, c_prev: torch.Tensor, c: torch.Tensor, dh: torch.Tensor,
                       dc: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    _need_hip(G, c_prev, c, dh, dc)
    B, H = c_prev.shape
    dG = torch.empty_like(G)
    dc_prev = torch.empty_like(c_prev)
    _lib.call("mog_lstm_cell_backward", dp(G), None, dp(c_prev), dp(c), dp(dh), dp(dc), dp(dG),
              dp(dc_prev), None, B, H, stream_ptr())
    return dG, dc_prev


@lstm_cell_backward.register_fake
def _(G, c_prev, c, dh, dc):
    return G.new_empty(G.shape), c_prev.new_empty(c_prev.shape)


def _lstm_setup(ctx, inputs, output):
    G, c_prev = inputs
    c, _ = output
    ctx.save_for_backward(G, c_prev, c)


def _lstm_bwd(ctx, dc, dh):
    G, c_prev, c = ctx.saved_tensors
    dc = torch.zeros_like(c) if dc is None else dc.contiguous()
    dh = torch.zeros_like(c) if dh is None else dh.contiguous()
    return torch.ops.mog_air.lstm_cell_backward(G, c_prev, c, dh, dc)


lstm_cell.register_autograd(_lstm_bwd, setup_context=_lstm_setup)


# ---------------------------------------------------------------- dense ----
@torch.library.custom_op("mog_air::dense", mutates_args=())
def dense(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor, act: int) -> torch.Tensor:
    """act(x W + b): one k-ordered fp32 MFMA chain per output, bias added
    after (TF matmul + bias_add), act 0 none / 1 relu / 2 TF softplus."""
    _need_hip(x, W, b)
    M, K = x.shape
    N = W.shape[1]
    out = torch.empty((M, N), device=x.device, dtype=torch.float32)
    epi = {0: EPI_STORE, 1: EPI_RELU, 2: EPI_SOFTPLUS}[int(act)]
    ops.gemm([x], [W], [out], M, N, K, K, N, N, epi=epi, bias=[b])
    return out


@dense.register_fake
def _(x, W, b, act):
    return x.new_empty((x.shape[0], W.shape[1]))


# ----------------------------------------------------------- optimizer ----
@torch.library.custom_op("mog_air::tf_adam_clip_", mutates_args=("params", "grads", "m", "v"))
def tf_adam_clip_(params: torch.Tensor, grads: torch.Tensor, m: torch.Tensor, v: torch.Tensor,
                  lr: float, clip: float, beta1: float, beta2: float, eps: float,
                  step: int) -> None:
    """One tensor: inf/nan -> 0, clip_by_norm(clip), TF ApplyAdam at step
    `step` (1-based; lr_t = lr sqrt(1 - b2^t) / (1 - b1^t))."""
    _need_hip(params, grads, m, v)
    n = params.numel()
    chunk = _lib.load().mog_optim_chunk_elems()
    nblk = (n + chunk - 1) // chunk
    dev = params.device
    off = torch.zeros(1, device=dev, dtype=torch.int64)
    ln = torch.full((1,), n, device=dev, dtype=torch.int64)
    bt = torch.zeros(nblk, device=dev, dtype=torch.int32)
    bs = torch.arange(nblk, device=dev, dtype=torch.int64) * chunk
    sumsq = torch.zeros(1, device=dev, dtype=torch.float32)
    import numpy as np
    f = np.float32
    b1p, b2p = f(1), f(1)
    for _ in range(int(step)):  # TF keeps the beta powers as fp32 variables
        b1p, b2p = f(b1p * f(beta1)), f(b2p * f(beta2))
    lr_t = f(lr) * np.sqrt(f(1) - b2p, dtype=np.float32) / (f(1) - b1p)
    _lib.call("mog_clip_adam", dp(params), dp(grads), dp(m), dp(v), dp(off), dp(ln), dp(bt),
              dp(bs), nblk, dp(sumsq), float(clip), float(lr_t), float(beta1), float(beta2),
              float(eps), stream_ptr())

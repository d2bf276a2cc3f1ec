"""Differentiable PyTorch-ROCm custom ops over the HIP kernels:
functional ``mog_air::`` operators with autograd, so the hot-path pieces are
callable from ordinary torch code the way the reference's TF graph uses
transformer() / vae() / BasicLSTMCell / AdamOptimizer.  Every op is a
composition of the launch-level C++ operators of csrc/torch_ops.cpp
(torch.ops.mog_air.*_ -- the same launches the AIRModel schedules), on torch's
current HIP stream; there is no CPU implementation (a CPU tensor raises).

    import mog_air.torch_ops                          # registers the ops
    g = torch.ops.mog_air.stn(canvas, theta, 28, 28)  # transformer() read
    g.sum().backward()                                # mog_stn_backward

Ops (reference counterpart):
  stn(U[N,Hin,Win] f32, theta[N,6], Hout, Wout) -> [N,Hout,Wout]   transformer.py:18-175
  stn_accumulate_(canvas[N,C*C], U, theta, z[N], mask[N]) (in place)  air_model.py:580-588,665-675
  lstm_cell(G[B,4H], c_prev[B,H]) -> (c, h)                         BasicLSTMCell gates
  dense(x, W, b, act) -> act(x W + b)  act: 0 none, 1 relu, 2 softplus  fully_connected
  glimpse_vae(g[B,784], W[7], b[7], eps_z, eps_x, lik_std)            vae.py:5-48 (fp32)
      -> [r, mu, logvar, z, *saved]   differentiable in g, W, b through r, mu, logvar, z
  stn_vae_step(x[B,C*C], theta_f, theta_b, z_pres[B], mask[B], eps_z, eps_x, W[7], b[7],
               lik_std) -> [canvas_part[B,C*C], r, mu, logvar, z, vae_kl, *saved]
      the fused bf16 STN-read -> VAE -> STN-write step (air_model.py:523-588, vae.py:5-48);
      differentiable in theta_f, theta_b, z_pres, W, b through canvas_part
  air_step(h[B,H], W1[5], b1[5], W2[5], b2[5], eps_scale, eps_shift, u, stop, runloss, digits,
           live, cfg[10], train, use_num_prior) -> [theta_f, theta_b, zc, zmask, runloss, ...]
      one loop step's five heads + concrete z_pres + KLs (air_model.py:458-520, 552-705);
      differentiable in h, W1, b1, W2, b2 through theta_f, theta_b, zc and runloss
  tf_adam_clip_(flat params, grads, m, v, lr, clip, beta1, beta2, eps, step)  air_model.py:941-999
"""
from __future__ import annotations

from typing import List, Tuple

import numpy as np
import torch

from . import _lib, ops
from .air_model import R_NREC
from .ops import (BF_ATOMIC, BF_SOFTPLUS_BWD, BF_STORE, EPI_ATOMIC, EPI_RELU, EPI_SIGMOID_NOISE,
                  EPI_SOFTPLUS, EPI_SOFTPLUS_BWD, EPI_STORE, gemm, gemm_bf16)

_ops = ops._ops


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
    _ops.stn_forward_(U, N, Hin, Win, theta, Hout, Wout, out, None, None, 0)
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
    _ops.stn_forward_(U, N, Hin, Win, theta, C, C, canvas, z, mask, 1)


# ----------------------------------------------------------------- LSTM ----
@torch.library.custom_op("mog_air::lstm_cell", mutates_args=())
def lstm_cell(G: torch.Tensor, c_prev: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    _need_hip(G, c_prev)
    B, H = c_prev.shape
    c = torch.empty_like(c_prev)
    h = torch.empty_like(c_prev)
    _ops.lstm_cell_forward_(G, None, c_prev, c, h, B, H)
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
    _ops.lstm_cell_backward_(G, None, c_prev, c, dh, dc, dG, dc_prev, None, B, H)
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
    gemm([x], [W], [out], M, N, K, K, N, N, epi=epi, bias=[b])
    return out


@dense.register_fake
def _(x, W, b, act):
    return x.new_empty((x.shape[0], W.shape[1]))


# ------------------------------------------------------------ glimpse VAE ----
_VAE_SHAPES = ((784, 512), (512, 256), (256, 50), (256, 50), (50, 256), (256, 512), (512, 784))


def _check_vae(weights, biases):
    if len(weights) != 7 or len(biases) != 7:
        raise ValueError("7 VAE layers: recognition_1, recognition_2, rec_mean, "
                         "rec_log_variance, generative_1, generative_2, gen_mean")
    for w, b, s in zip(weights, biases, _VAE_SHAPES):
        if tuple(w.shape) != s or tuple(b.shape) != (s[1],):
            raise ValueError(f"VAE layer shape {tuple(w.shape)} / {tuple(b.shape)}, expected {s}")
    _need_hip(*weights, *biases)


@torch.library.custom_op("mog_air::glimpse_vae", mutates_args=())
def glimpse_vae(g: torch.Tensor, weights: List[torch.Tensor], biases: List[torch.Tensor],
                eps_z: torch.Tensor, eps_x: torch.Tensor, lik_std: float
                ) -> List[torch.Tensor]:
    """vae() of air/vae.py:5-48 in fp32 (the reference's precision): every
    dense layer one k-ordered fma chain, TF softplus / sigmoid epilogues,
    z = mu + eps_z sqrt(exp(logvar)), r = sigmoid(gen_mean + lik_std eps_x).
    Returns [r, mu, logvar, z] and the saved pre- / post-activations (a1pre,
    a1, a2pre, a2, d1pre, d1, d2pre, d2) the backward uses."""
    _need_hip(g, eps_z, eps_x)
    _check_vae(weights, biases)
    B = g.shape[0]
    e = lambda n: torch.empty((B, n), device=g.device, dtype=torch.float32)  # noqa: E731
    a1p, a1, a2p, a2 = e(512), e(512), e(256), e(256)
    mu, lv, z = e(50), e(50), e(50)
    d1p, d1, d2p, d2, r = e(256), e(256), e(512), e(512), e(784)
    W, b = weights, biases
    gemm([g], [W[0]], [a1], B, 512, 784, 784, 512, 512, epi=EPI_SOFTPLUS, bias=[b[0]], Cpre=[a1p])
    gemm([a1], [W[1]], [a2], B, 256, 512, 512, 256, 256, epi=EPI_SOFTPLUS, bias=[b[1]],
         Cpre=[a2p])
    gemm([a2, a2], [W[2], W[3]], [mu, lv], B, 50, 256, 256, 50, 50, bias=[b[2], b[3]])
    zero = torch.zeros(B, device=g.device, dtype=torch.float32)
    _ops.vae_sample_forward_(B, 50, 0.0, 1.0, 0.0, mu, lv, eps_z, z, None, 0, zero, zero.clone(),
                             zero.clone())
    gemm([z], [W[4]], [d1], B, 256, 50, 50, 256, 256, epi=EPI_SOFTPLUS, bias=[b[4]], Cpre=[d1p])
    gemm([d1], [W[5]], [d2], B, 512, 256, 256, 512, 512, epi=EPI_SOFTPLUS, bias=[b[5]],
         Cpre=[d2p])
    gemm([d2], [W[6]], [r], B, 784, 512, 512, 784, 784, epi=EPI_SIGMOID_NOISE, bias=[b[6]],
         aux=[eps_x], ldaux=784, aux_scale=float(lik_std))
    return [r, mu, lv, z, a1p, a1, a2p, a2, d1p, d1, d2p, d2]


@glimpse_vae.register_fake
def _(g, weights, biases, eps_z, eps_x, lik_std):
    B = g.shape[0]
    e = lambda n: g.new_empty((B, n))  # noqa: E731
    return [e(784), e(50), e(50), e(50), e(512), e(512), e(256), e(256), e(256), e(256), e(512),
            e(512)]


def _gv_setup(ctx, inputs, output):
    g, weights, biases, eps_z, eps_x, lik_std = inputs
    ctx.save_for_backward(g, eps_z, *output, *weights)


def _gv_bwd(ctx, grads):
    g, eps_z, r, mu, lv, z, a1p, a1, a2p, a2, d1p, d1, d2p, d2, *W = ctx.saved_tensors
    dr, dmu, dlv, dz = grads[:4]
    B, dev = g.shape[0], g.device
    e = lambda *s: torch.empty(s, device=dev, dtype=torch.float32)  # noqa: E731
    zeros = lambda *s: torch.zeros(s, device=dev, dtype=torch.float32)  # noqa: E731
    dr = zeros(B, 784) if dr is None else dr.contiguous()
    dm, dd2, dd1, dzt = e(B, 784), e(B, 512), e(B, 256), e(B, 50)
    _ops.sigmoid_backward_(r, dr, dm, B * 784)
    # (epi 4 reads the softplus OUTPUT: sigmoid(x) = 1 - exp(-softplus(x)))
    gemm([dm], [W[6]], [dd2], B, 512, 784, 784, 784, 512, transB=True, epi=EPI_SOFTPLUS_BWD,
         aux=[d2], ldaux=512)
    gemm([dd2], [W[5]], [dd1], B, 256, 512, 512, 512, 256, transB=True, epi=EPI_SOFTPLUS_BWD,
         aux=[d1], ldaux=256)
    gemm([dd1], [W[4]], [dzt], B, 50, 256, 256, 256, 50, transB=True)
    if dz is not None:
        _ops.add_(dzt, dz.contiguous(), dzt, B * 50)
    dmut, dlvt = e(B, 50), e(B, 50)
    zero = torch.zeros(B, device=dev, dtype=torch.float32)
    _ops.vae_sample_backward_(B, 50, 0.0, 1.0, 0.0, mu, lv, eps_z, dzt, zero, dmut, dlvt, None,
                              None, 0)
    if dmu is not None:
        _ops.add_(dmut, dmu.contiguous(), dmut, B * 50)
    if dlv is not None:
        _ops.add_(dlvt, dlv.contiguous(), dlvt, B * 50)
    tmp, da2, da1, dg = e(B, 256), e(B, 256), e(B, 512), e(B, 784)
    gemm([dmut], [W[2]], [tmp], B, 256, 50, 50, 50, 256, transB=True)
    gemm([dlvt], [W[3]], [da2], B, 256, 50, 50, 50, 256, transB=True, epi=EPI_SOFTPLUS_BWD,
         Cin=[tmp], aux=[a2], ldaux=256)
    gemm([da2], [W[1]], [da1], B, 512, 256, 256, 256, 512, transB=True, epi=EPI_SOFTPLUS_BWD,
         aux=[a1], ldaux=512)
    gemm([da1], [W[0]], [dg], B, 784, 512, 512, 512, 784, transB=True)
    # weight / bias gradients: dW = X^T dY (fp32 atomics), db = colsum(dY)
    xs = (g, a1, a2, a2, z, d1, d2)
    dys = (da1, da2, dmut, dlvt, dd1, dd2, dm)
    gW = [zeros(*w.shape) for w in W]
    gb = [zeros(w.shape[1]) for w in W]
    for x, dy, gw, gbi in zip(xs, dys, gW, gb):
        K, M = x.shape
        N = dy.shape[1]
        gemm([x], [dy], [gw], M, N, K, M, N, N, transA=True, epi=EPI_ATOMIC, colsum=[gbi])
    return dg, gW, gb, None, None, None


glimpse_vae.register_autograd(_gv_bwd, setup_context=_gv_setup)


# -------------------------------------- fused STN read -> VAE -> STN write ----
def _pack_vae_bf16(weights):
    """bf16 packs of the 7 VAE matrices: W^T in MFMA B-fragment order (the
    fused kernel's operand, mog_cvt_bf16_batch transpose 2) and W [in][out8]
    (the backward GEMMs' dX operand), one batched launch."""
    dev = weights[0].device
    bf = dict(device=dev, dtype=torch.bfloat16)
    wf, wn, srcs, dsts, dims = [], [], [], [], []
    for w in weights:
        I, O = w.shape
        Np, Kp = (O + 15) // 16 * 16, (I + 31) // 32 * 32
        f = torch.zeros((Np, Kp), **bf)
        n = torch.zeros((I, (O + 7) // 8 * 8), **bf)
        wf.append(f)
        wn.append(n)
        srcs += [w, w]
        dsts += [f, n]
        dims += [I, O, O, Np, Kp, Kp, 2, I, O, O, I, n.shape[1], n.shape[1], 0]
    _ops.cvt_bf16_batch_(srcs, dsts, dims)
    return wf, wn


@torch.library.custom_op("mog_air::stn_vae_step", mutates_args=())
def stn_vae_step(x: torch.Tensor, theta_f: torch.Tensor, theta_b: torch.Tensor,
                 z_pres: torch.Tensor, mask: torch.Tensor, eps_z: torch.Tensor,
                 eps_x: torch.Tensor, weights: List[torch.Tensor], biases: List[torch.Tensor],
                 lik_std: float) -> List[torch.Tensor]:
    """One loop step's glimpse path (air_model.py:523-588, vae.py:5-48) in the
    fused bf16 kernel (vae_step.hip), functional form: canvas_part =
    mask ? z_pres * STN(r, theta_b) : 0 over the C x C canvas, and r, mu,
    logvar, z, vae_kl (the per-image VAE KL of vae.py:27-30), then the saved
    bf16 activations (g, a1, a2, z, d1, d2) of the backward."""
    _need_hip(x, theta_f, theta_b, z_pres, mask, eps_z, eps_x)
    _check_vae(weights, biases)
    B, C2 = x.shape
    C = int(round(C2 ** 0.5))
    dev = x.device
    f32 = dict(device=dev, dtype=torch.float32)
    bf = dict(device=dev, dtype=torch.bfloat16)
    wf, _ = _pack_vae_bf16(weights)
    part = torch.zeros((B, C2), **f32)
    rows = torch.empty(B, device=dev, dtype=torch.int32)
    runloss, vkl = torch.zeros(B, **f32), torch.empty(B, **f32)
    gb, a1b, a2b = torch.empty((B, 784), **bf), torch.empty((B, 512), **bf), torch.empty((B, 256), **bf)
    zb = torch.zeros((B, 56), **bf)
    d1b, d2b = torch.empty((B, 256), **bf), torch.empty((B, 512), **bf)
    mu, lv, z = torch.empty((B, 50), **f32), torch.empty((B, 50), **f32), torch.empty((B, 50), **f32)
    r = torch.empty((B, 784), **f32)
    _ops.stn_vae_step_(B, C, x, theta_f, theta_b, mask, z_pres, eps_z, eps_x, 0, 0, False, wf,
                       list(biases), float(lik_std), 0.0, 1.0, 0.0, part, rows, runloss, vkl, gb,
                       a1b, a2b, mu, lv, z, zb, d1b, d2b, r)
    return [part, r, mu, lv, z, vkl, gb, a1b, a2b, zb, d1b, d2b]


@stn_vae_step.register_fake
def _(x, theta_f, theta_b, z_pres, mask, eps_z, eps_x, weights, biases, lik_std):
    B, C2 = x.shape
    f = lambda *s: x.new_empty(s)  # noqa: E731
    b = lambda *s: x.new_empty(s, dtype=torch.bfloat16)  # noqa: E731
    return [f(B, C2), f(B, 784), f(B, 50), f(B, 50), f(B, 50), f(B), b(B, 784), b(B, 512),
            b(B, 256), b(B, 56), b(B, 256), b(B, 512)]


def _svs_setup(ctx, inputs, output):
    x, theta_f, theta_b, z_pres, mask, eps_z, eps_x, weights, biases, lik_std = inputs
    part, r, mu, lv, z, vkl, gb, a1b, a2b, zb, d1b, d2b = output
    ctx.save_for_backward(x, theta_f, theta_b, z_pres, mask, eps_z, r, mu, lv, gb, a1b, a2b, zb,
                          d1b, d2b, *weights)


def _svs_bwd(ctx, grads):
    """Gradient from canvas_part (the other outputs are treated as
    non-differentiable here): STN write backward with the output sigmoid
    folded (bf16 dm), the bf16 VAE backward GEMM chain, the STN read backward
    for d theta_f, and fp32 weight / bias gradients (split-K atomics)."""
    (x, theta_f, theta_b, z_pres, mask, eps_z, r, mu, lv, gb, a1b, a2b, zb, d1b, d2b,
     *W) = ctx.saved_tensors
    dpart = grads[0]
    B, C2 = x.shape
    C = int(round(C2 ** 0.5))
    dev = x.device
    f32 = dict(device=dev, dtype=torch.float32)
    bf = dict(device=dev, dtype=torch.bfloat16)
    zeros = lambda *s: torch.zeros(s, **f32)  # noqa: E731
    if dpart is None:
        dpart = zeros(B, C2)
    _, wn = _pack_vae_bf16(W)
    zc = z_pres * (mask != 0).to(torch.float32)
    dmb = torch.empty((B, 784), **bf)
    dth_b, dot = torch.empty((B, 6), **f32), torch.empty(B, **f32)
    ops.stn_backward(r, theta_b, (C, C), dpart.contiguous(), gscale=zc.contiguous(), want_dot=True,
                     dtheta=dth_b, dot=dot, dm_bf16=dmb)
    dd2b, dd1b = torch.empty((B, 512), **bf), torch.empty((B, 256), **bf)
    dz = torch.empty((B, 50), **f32)
    gemm_bf16([dmb], [wn[6]], [dd2b], B, 512, 784, 784, 784, 512, epi=BF_SOFTPLUS_BWD, aux=[d2b],
              ldaux=512)
    gemm_bf16([dd2b], [wn[5]], [dd1b], B, 256, 512, 512, 512, 256, epi=BF_SOFTPLUS_BWD,
              aux=[d1b], ldaux=256)
    gemm_bf16([dd1b], [wn[4]], [dz], B, 50, 256, 256, 256, 50, epi=BF_STORE)
    dmub, dlvb = torch.zeros((B, 56), **bf), torch.zeros((B, 56), **bf)
    _ops.vae_sample_backward_(B, 50, 0.0, 1.0, 0.0, mu, lv, eps_z, dz, torch.zeros(B, **f32),
                              None, None, dmub, dlvb, 56)
    tmp, da2b, da1b = torch.empty((B, 256), **f32), torch.empty((B, 256), **bf), \
        torch.empty((B, 512), **bf)
    dg = torch.empty((B, 784), **f32)
    gemm_bf16([dmub], [wn[2]], [tmp], B, 256, 56, 56, 56, 256, epi=BF_STORE)
    gemm_bf16([dlvb], [wn[3]], [da2b], B, 256, 56, 56, 56, 256, epi=BF_SOFTPLUS_BWD, Cin=[tmp],
              aux=[a2b], ldaux=256)
    gemm_bf16([da2b], [wn[1]], [da1b], B, 512, 256, 256, 256, 512, epi=BF_SOFTPLUS_BWD,
              aux=[a1b], ldaux=512)
    gemm_bf16([da1b], [wn[0]], [dg], B, 784, 512, 512, 512, 784, epi=BF_STORE)
    dth_f = torch.empty((B, 6), **f32)
    ops.stn_backward(x, theta_f, (28, 28), dg, want_dU=False, dtheta=dth_f)
    xs = (gb, a1b, a2b, a2b, zb, d1b, d2b)
    dys = (da1b, da2b, dmub, dlvb, dd1b, dd2b, dmb)
    lds = (784, 512, 256, 256, 56, 256, 512)
    ldy = (512, 256, 56, 56, 256, 512, 784)
    gW = [zeros(*w.shape) for w in W]
    gbias = [zeros(w.shape[1]) for w in W]
    for xq, dy, gw, gbi, la, lb in zip(xs, dys, gW, gbias, lds, ldy):
        M, N = gw.shape
        gemm_bf16([xq], [dy], [gw], M, N, B, la, lb, N, tn=True, epi=BF_ATOMIC, colsum=[gbi])
    dz_pres = dot * (mask != 0).to(torch.float32)
    return None, dth_f, dth_b, dz_pres, None, None, None, gW, gbias, None


stn_vae_step.register_autograd(_svs_bwd, setup_context=_svs_setup)


# ------------------------------------------- heads + concrete z_pres step ----
# cfg order of air_step (floats): stopping threshold, concrete temperature,
# z_pres prior log-odds, its per-step bias (num prior), scale prior mean /
# variance / log-variance, shift prior mean / variance / log-variance
AIR_STEP_CFG = ("thr", "temperature", "prior_lo", "prior_bias", "s_pm", "s_pv", "s_plv", "h_pm",
                "h_pv", "h_plv")


@torch.library.custom_op("mog_air::air_step", mutates_args=())
def air_step(h: torch.Tensor, W1: List[torch.Tensor], b1: List[torch.Tensor],
             W2: List[torch.Tensor], b2: List[torch.Tensor], eps_scale: torch.Tensor,
             eps_shift: torch.Tensor, u: torch.Tensor, stop: torch.Tensor, runloss: torch.Tensor,
             digits: torch.Tensor, live: torch.Tensor, cfg: List[float], train: bool,
             use_num_prior: bool) -> List[torch.Tensor]:
    """One loop step's heads and concrete z_pres (SURVEY §8 B heads_fwd +
    concrete_fwd; air_model.py:458-520 heads, scale / shift sampling and theta,
    :552-577 theta^-1, :590-663 concrete z_pres and its KL, :677-705 scale /
    shift KLs): the five ReLU hidden layers in one batched launch, then the
    step kernel.  h [B,H] is the LSTM output; W1/b1 [H,HS]/[HS] and W2/b2
    [HS,k]/[k] are the five heads (scale-mean, scale-logvar, shift-mean,
    shift-logvar, z_pres log-odds; k = 2 for the shift heads).  State in:
    stop / runloss [B] f32, digits [B] int32, live [1] int32 (is step t live).
    Returns [theta_f, theta_b, zc, zmask, runloss, stop, digits, live, zprob,
    scale, shift, zkl, skl, shkl, rec, hid]: zc = active ? z_pres : 0 is the
    canvas coefficient.  Differentiable in h, W1, b1, W2, b2 (and runloss)
    through theta_f, theta_b, zc and runloss; the discrete state and the
    reporting outputs carry no gradient."""
    _need_hip(h, eps_scale, eps_shift, u, stop, runloss, *W1, *b1, *W2, *b2)
    if len(W1) != 5 or len(b1) != 5 or len(W2) != 5 or len(b2) != 5 or len(cfg) != 10:
        raise ValueError("air_step takes five heads and ten cfg floats")
    if digits.dtype != torch.int32 or live.dtype != torch.int32 or live.numel() != 1:
        raise ValueError("air_step: digits [B] and live [1] are int32")
    B, H = h.shape
    HS = W1[0].shape[1]
    dev = h.device
    f32 = dict(device=dev, dtype=torch.float32)
    hid = torch.empty((5, B, HS), **f32)
    gemm([h] * 5, list(W1), [hid[z] for z in range(5)], B, HS, H, H, HS, HS, epi=EPI_RELU,
         bias=list(b1))
    stop_o, rl_o, dig_o = stop.clone(), runloss.clone(), digits.clone()
    live_o = torch.zeros(2, device=dev, dtype=torch.int32)
    live_o[:1] = live
    rec = torch.empty((R_NREC, B), **f32)
    th_f, th_b = torch.empty((B, 6), **f32), torch.empty((B, 6), **f32)
    e = lambda *sh: torch.empty(sh, **f32)  # noqa: E731
    scale, shift, zprob, zkl, skl, shkl = e(B), e(B, 2), e(B), e(B), e(B), e(B)
    zmask, zval, zc = e(B), e(B), e(B)
    thr, temp, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = (float(c) for c in cfg)
    _ops.air_step_forward_(B, HS, HS, 0, train, use_num_prior, thr, temp, plo, pb, s_pm, s_pv,
                           s_plv, h_pm, h_pv, h_plv, [hid[z] for z in range(5)], list(W2),
                           list(b2), eps_scale, eps_shift, u, stop_o, rl_o, dig_o, live_o, rec,
                           th_f, th_b, scale, shift, zprob, zkl, skl, shkl, zmask, zval, zc)
    return [th_f, th_b, zc, zmask, rl_o, stop_o, dig_o, live_o[1:].clone(), zprob, scale, shift,
            zkl, skl, shkl, rec, hid]


@air_step.register_fake
def _(h, W1, b1, W2, b2, eps_scale, eps_shift, u, stop, runloss, digits, live, cfg, train,
      use_num_prior):
    B, HS = h.shape[0], W1[0].shape[1]
    n = lambda *sh: h.new_empty(sh)  # noqa: E731
    return [n(B, 6), n(B, 6), n(B), n(B), n(B), n(B), digits.new_empty(B), live.new_empty(1),
            n(B), n(B), n(B, 2), n(B), n(B), n(B), n(R_NREC, B), n(5, B, HS)]


def _as_setup(ctx, inputs, output):
    h, W1, b1, W2, b2, eps_scale, eps_shift, u, stop, runloss, digits, live, cfg, train, \
        use_num_prior = inputs
    ctx.cfg, ctx.train, ctx.use_num_prior = list(cfg), train, use_num_prior
    ctx.ks = [w.shape[1] for w in W2]
    ctx.save_for_backward(h, eps_scale, eps_shift, output[14], output[15], *W1, *W2)
    ctx.set_materialize_grads(False)


def _as_bwd(ctx, grads):
    """mog_air_step_backward with the per-image cotangent of the running loss
    (dloss) weighting this step's KL terms, then the heads: dh = sum_z dhid_z
    W1_z^T (one k-ordered chain), dW1 / db1 = h^T dhid, dW2 / db2 = hid^T dout
    (split-K atomics with fused column sums)."""
    h, eps_scale, eps_shift, rec, hid, *W = ctx.saved_tensors
    W1, W2 = W[:5], W[5:]
    B, H = h.shape
    HS = hid.shape[2]
    f32 = dict(device=h.device, dtype=torch.float32)
    zeros = lambda *s: torch.zeros(s, **f32)  # noqa: E731
    g = lambda i, *s: zeros(*s) if grads[i] is None else grads[i].contiguous()  # noqa: E731
    dth_f, dth_b, dzc, drl = g(0, B, 6), g(1, B, 6), g(2, B), g(4, B)
    thr, temp, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = (float(c) for c in ctx.cfg)
    dout, dhid = torch.empty((5, B, 2), **f32), torch.empty((5, B, HS), **f32)
    hid_l = [hid[z] for z in range(5)]
    _ops.air_step_backward_(B, HS, ctx.train, ctx.use_num_prior, temp, plo, pb, s_pm, s_pv, h_pm,
                            h_pv, 0.0, drl, rec, eps_scale, eps_shift, dth_f, dth_b, dzc, hid_l,
                            list(W2), dout[0], B * 2, dhid[0], B * HS)
    dh = torch.empty((B, H), **f32)
    ops.gemm_kseg([dhid[z] for z in range(5)], list(W1), dh, B, H, HS, HS, HS, H, transB=True)
    gW1, gb1 = [zeros(H, HS) for _ in range(5)], [zeros(HS) for _ in range(5)]
    splitk = max(1, B // 256)
    gemm([h] * 5, [dhid[z] for z in range(5)], gW1, H, HS, B, H, HS, HS, transA=True,
         epi=EPI_ATOMIC, splitk=splitk, colsum=gb1)
    gW2, gb2 = [zeros(HS, k) for k in ctx.ks], [zeros(k) for k in ctx.ks]
    for k in (1, 2):
        sel = [z for z in range(5) if ctx.ks[z] == k]
        if sel:
            gemm([hid[z] for z in sel], [dout[z] for z in sel], [gW2[z] for z in sel], HS, k, B,
                 HS, 2, k, transA=True, epi=EPI_ATOMIC, splitk=splitk,
                 colsum=[gb2[z] for z in sel])
    return (dh, gW1, gb1, gW2, gb2, None, None, None, None, drl, None, None, None, None, None)


air_step.register_autograd(_as_bwd, setup_context=_as_setup)


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
    sumsq = torch.zeros(nblk, device=dev, dtype=torch.float32)  # per-chunk scratch
    f = np.float32
    b1p, b2p = f(1), f(1)
    for _ in range(int(step)):  # TF keeps the beta powers as fp32 variables
        b1p, b2p = f(b1p * f(beta1)), f(b2p * f(beta2))
    lr_t = f(lr) * np.sqrt(f(1) - b2p, dtype=np.float32) / (f(1) - b1p)
    _ops.clip_adam_(params, grads, m, v, off, ln, bt, bs, nblk, sumsq, float(clip), float(lr_t),
                    float(beta1), float(beta2), float(eps))

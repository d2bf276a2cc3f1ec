"""The PyTorch custom-op surface (mog_air::*) over the HIP kernels: each op
against the CPU oracle (bit-exact where the C ABI path is) and its autograd
against float64 torch."""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao
from oracle import air_torch as at

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _ops():
    import mog_air.torch_ops  # noqa: F401


def _theta(rng, N):
    s = rng.uniform(0.3, 0.8, N)
    t = rng.uniform(-0.5, 0.5, (N, 2))
    return np.stack([s, 0 * s, t[:, 0], 0 * s, s, t[:, 1]], 1).astype(np.float32)


def test_stn_op_bit_exact_and_autograd():
    rng = np.random.default_rng(0)
    N = 9
    U = rng.uniform(0, 1, (N, 50, 50)).astype(np.float32)
    th = _theta(rng, N)
    ref = ao.stn(U, th, (28, 28))
    Ug = torch.tensor(U, device=DEV, requires_grad=True)
    tg = torch.tensor(th, device=DEV, requires_grad=True)
    out = torch.ops.mog_air.stn(Ug, tg, 28, 28)
    np.testing.assert_array_equal(out.detach().cpu().numpy(), ref.reshape(N, 28, 28))
    G = torch.tensor(rng.standard_normal((N, 28, 28)).astype(np.float32), device=DEV)
    (out * G).sum().backward()
    U64 = torch.tensor(U, dtype=torch.float64, requires_grad=True)
    t64 = torch.tensor(th, dtype=torch.float64, requires_grad=True)
    (at.transformer(U64, t64, (28, 28)) * G.double().cpu()).sum().backward()
    np.testing.assert_allclose(Ug.grad.cpu().numpy(), U64.grad.numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(tg.grad.cpu().numpy(), t64.grad.numpy(), rtol=1e-3, atol=1e-3)


def test_lstm_cell_op_autograd():
    rng = np.random.default_rng(1)
    B, H = 7, 256
    G = torch.tensor(rng.standard_normal((B, 4 * H)).astype(np.float32), device=DEV,
                     requires_grad=True)
    c0 = torch.tensor(rng.standard_normal((B, H)).astype(np.float32), device=DEV,
                      requires_grad=True)
    c, h = torch.ops.mog_air.lstm_cell(G, c0)
    w = torch.tensor(rng.standard_normal((B, H)).astype(np.float32), device=DEV)
    (h * w + c).sum().backward()
    G64 = G.detach().cpu().double().requires_grad_()
    c64 = c0.detach().cpu().double().requires_grad_()
    gi, gj, gf, go = torch.split(G64, H, 1)
    cr = c64 * torch.sigmoid(gf + 1.0) + torch.sigmoid(gi) * torch.tanh(gj)
    hr = torch.tanh(cr) * torch.sigmoid(go)
    np.testing.assert_allclose(h.detach().cpu().numpy(), hr.detach().numpy(), rtol=1e-5,
                               atol=1e-6)
    (hr * w.cpu().double() + cr).sum().backward()
    np.testing.assert_allclose(G.grad.cpu().numpy(), G64.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(c0.grad.cpu().numpy(), c64.grad.numpy(), rtol=1e-4, atol=1e-6)


@pytest.mark.parametrize("act", [0, 1, 2])
def test_dense_op_bit_exact(act):
    rng = np.random.default_rng(2 + act)
    x = rng.standard_normal((37, 300)).astype(np.float32)
    W = (rng.standard_normal((300, 70)) * 0.1).astype(np.float32)
    b = rng.standard_normal(70).astype(np.float32)
    ref = ao.dense_chain(x, W, b)
    if act == 1:
        ref = np.maximum(ref, 0)
    elif act == 2:
        lib = ao._load()
        y = np.zeros_like(ref)
        lib.oracle_math_vec(5, ref.ctypes.data_as(ao._FP), y.ctypes.data_as(ao._FP), ref.size)
        ref = y
    got = torch.ops.mog_air.dense(torch.tensor(x, device=DEV), torch.tensor(W, device=DEV),
                                  torch.tensor(b, device=DEV), act)
    np.testing.assert_array_equal(got.cpu().numpy(), ref)


def test_tf_adam_clip_op():
    rng = np.random.default_rng(5)
    p = rng.standard_normal(5000).astype(np.float32)
    g = (rng.standard_normal(5000) * 3).astype(np.float32)
    g[7] = np.inf
    g[9] = np.nan
    P = {"w": torch.tensor(p, dtype=torch.float64)}
    Gd = {"w": torch.tensor(np.nan_to_num(g, nan=0.0, posinf=0.0), dtype=torch.float64)}
    m = {"w": torch.zeros(5000, dtype=torch.float64)}
    v = {"w": torch.zeros(5000, dtype=torch.float64)}
    at.tf_clip_adam_step(P, Gd, m, v, 1, lr=1e-3, clip=1.0)
    tp, tg = torch.tensor(p, device=DEV), torch.tensor(g, device=DEV)
    tm, tv = torch.zeros(5000, device=DEV), torch.zeros(5000, device=DEV)
    torch.ops.mog_air.tf_adam_clip_(tp, tg, tm, tv, 1e-3, 1.0, 0.9, 0.999, 1e-8, 1)
    np.testing.assert_allclose(tp.cpu().numpy(), P["w"].numpy(), rtol=1e-6, atol=1e-7)


def test_ops_refuse_cpu_tensors():
    with pytest.raises(RuntimeError):
        torch.ops.mog_air.stn(torch.zeros(1, 50, 50), torch.zeros(1, 6), 28, 28)

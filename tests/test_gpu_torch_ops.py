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


# ---------------------------------------------------------------------------
# glimpse VAE / fused step as functional ops; the AIRModel's dispatch
def _vae_params(rng, scale=0.08):
    shapes = ((784, 512), (512, 256), (256, 50), (256, 50), (50, 256), (256, 512), (512, 784))
    W = [torch.tensor((rng.standard_normal(s) * scale).astype(np.float32), device=DEV)
         for s in shapes]
    b = [torch.tensor((rng.standard_normal(s[1]) * 0.05).astype(np.float32), device=DEV)
         for s in shapes]
    return W, b


def _vae64(g, W, b, eps_z, eps_x, lik_std):
    """float64 torch restatement of vae() (air/vae.py:5-48, TF softplus)."""
    a1 = at.softplus_tf(g @ W[0] + b[0])
    a2 = at.softplus_tf(a1 @ W[1] + b[1])
    mu, lv = a2 @ W[2] + b[2], a2 @ W[3] + b[3]
    z = mu + eps_z * torch.sqrt(torch.exp(lv))
    d1 = at.softplus_tf(z @ W[4] + b[4])
    d2 = at.softplus_tf(d1 @ W[5] + b[5])
    r = torch.sigmoid((d2 @ W[6] + b[6]) + lik_std * eps_x)
    return r, mu, lv, z


def test_glimpse_vae_op_forward_and_autograd():
    rng = np.random.default_rng(21)
    B = 33
    W, b = _vae_params(rng)
    g = torch.tensor(rng.uniform(0, 1, (B, 784)).astype(np.float32), device=DEV,
                     requires_grad=True)
    ez = torch.tensor(rng.standard_normal((B, 50)).astype(np.float32), device=DEV)
    ex = torch.tensor(rng.standard_normal((B, 784)).astype(np.float32), device=DEV)
    for t in W + b:
        t.requires_grad_()
    out = torch.ops.mog_air.glimpse_vae(g, W, b, ez, ex, 0.3)
    r, mu, lv, z = out[:4]
    # the same dense layers as the model's bit-exact fp32 chains
    a1 = torch.ops.mog_air.dense(g.detach(), W[0].detach(), b[0].detach(), 2)
    np.testing.assert_array_equal(out[5].detach().cpu().numpy(), a1.cpu().numpy())
    G = [torch.tensor(rng.standard_normal(s).astype(np.float32), device=DEV)
         for s in ((B, 784), (B, 50), (B, 50), (B, 50))]
    (sum((o * w).sum() for o, w in zip((r, mu, lv, z), G))).backward()
    d = lambda t: t.detach().cpu().double().requires_grad_()  # noqa: E731
    g64, W64, b64 = d(g), [d(t) for t in W], [d(t) for t in b]
    ref = _vae64(g64, W64, b64, ez.cpu().double(), ex.cpu().double(), 0.3)
    for o, rr in zip((r, mu, lv, z), ref):
        np.testing.assert_allclose(o.detach().cpu().numpy(), rr.detach().numpy(), rtol=1e-4,
                                   atol=1e-5)
    (sum((o * w.cpu().double()).sum() for o, w in zip(ref, G))).backward()
    for got, want in [(g, g64)] + list(zip(W, W64)) + list(zip(b, b64)):
        err = np.linalg.norm(got.grad.cpu().numpy() - want.grad.numpy()) / \
            max(np.linalg.norm(want.grad.numpy()), 1e-12)
        assert err < 1e-4, err


def _step_inputs(rng, B, C=50):
    x = torch.tensor(ao.synthetic_canvases(B, canvas=C, seed=5)[0], device=DEV)
    s = rng.uniform(0.3, 0.7, B)
    t = rng.uniform(-0.5, 0.5, (B, 2))
    thf = np.stack([s, 0 * s, t[:, 0], 0 * s, s, t[:, 1]], 1).astype(np.float32)
    thb = np.stack([1 / s, 0 * s, -t[:, 0] / s, 0 * s, 1 / s, -t[:, 1] / s], 1).astype(np.float32)
    zp = rng.uniform(0.2, 1.0, B).astype(np.float32)
    mask = (rng.uniform(size=B) < 0.8).astype(np.float32)
    ez = rng.standard_normal((B, 50)).astype(np.float32)
    ex = rng.standard_normal((B, 784)).astype(np.float32)
    c = lambda a: torch.tensor(a, device=DEV)  # noqa: E731
    return x, c(thf), c(thb), c(zp), c(mask), c(ez), c(ex)


def test_stn_vae_step_op_matches_c_abi_bitwise():
    """torch.ops.mog_air.stn_vae_step against a direct ctypes call of the C
    entry point mog_stn_vae_step_forward on the same packed weights."""
    from mog_air import _lib
    from mog_air.torch_ops import _pack_vae_bf16
    rng = np.random.default_rng(31)
    B = 150
    W, b = _vae_params(rng)
    x, thf, thb, zp, mask, ez, ex = _step_inputs(rng, B)
    out = torch.ops.mog_air.stn_vae_step(x, thf, thb, zp, mask, ez, ex, W, b, 0.3)
    wf, _ = _pack_vae_bf16(W)
    f32 = dict(device=DEV, dtype=torch.float32)
    bf = dict(device=DEV, dtype=torch.bfloat16)
    ref = [torch.zeros((B, 2500), **f32), torch.empty((B, 784), **f32),
           torch.empty((B, 50), **f32), torch.empty((B, 50), **f32), torch.empty((B, 50), **f32),
           torch.empty(B, **f32), torch.empty((B, 784), **bf), torch.empty((B, 512), **bf),
           torch.empty((B, 256), **bf), torch.zeros((B, 56), **bf), torch.empty((B, 256), **bf),
           torch.empty((B, 512), **bf)]
    part, r, mu, lv, z, vkl, gb, a1b, a2b, zb, d1b, d2b = ref
    rows = torch.empty(B, device=DEV, dtype=torch.int32)
    runloss = torch.zeros(B, **f32)
    dp = lambda t: t.data_ptr()  # noqa: E731
    _lib.call("mog_stn_vae_step_forward", B, 50, 28, 512, 256, 50, 256, 512, dp(x), dp(thf),
              dp(thb), dp(mask), dp(zp), dp(ez), dp(ex), 0, 0, 0,
              _lib.ptr_array([dp(w) for w in wf]), _lib.ptr_array([dp(t) for t in b]), 0.3, 0.0,
              1.0, 0.0, dp(part), dp(rows), dp(runloss), dp(vkl), dp(gb), dp(a1b), dp(a2b),
              dp(mu), dp(lv), dp(z), dp(zb), dp(d1b), dp(d2b), dp(r), 0,
              torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for i, (a, e) in enumerate(zip(out, ref)):
        ai = a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)
        ei = e.view(torch.int16) if e.dtype == torch.bfloat16 else e.view(torch.int32)
        assert torch.equal(ai, ei), i


def test_stn_vae_step_op_autograd_vs_float64():
    """Gradients of the fused bf16 step (through canvas_part) against a
    float64 torch restatement of STN read -> vae() -> STN write; the bar is
    the bf16 configuration's."""
    rng = np.random.default_rng(41)
    B = 24
    W, b = _vae_params(rng)
    x, thf, thb, zp, mask, ez, ex = _step_inputs(rng, B)
    for t in W + b + [thf, thb, zp]:
        t.requires_grad_()
    out = torch.ops.mog_air.stn_vae_step(x, thf, thb, zp, mask, ez, ex, W, b, 0.3)
    G = torch.tensor(rng.standard_normal((B, 2500)).astype(np.float32) * 0.01, device=DEV)
    (out[0] * G).sum().backward()
    d = lambda t: t.detach().cpu().double().requires_grad_()  # noqa: E731
    W64, b64 = [d(t) for t in W], [d(t) for t in b]
    thf64, thb64, zp64 = d(thf), d(thb), d(zp)
    g = at.transformer(x.cpu().double().view(B, 50, 50), thf64, (28, 28)).reshape(B, 784)
    r = _vae64(g, W64, b64, ez.cpu().double(), ex.cpu().double(), 0.3)[0]
    w = at.transformer(r.view(B, 28, 28), thb64, (50, 50)).reshape(B, 2500)
    part = (mask.cpu().double() * zp64)[:, None] * w
    np.testing.assert_allclose(out[0].detach().cpu().numpy(), part.detach().numpy(), atol=3e-2)
    (part * G.cpu().double()).sum().backward()
    for name, got, want in ([("theta_b", thb, thb64), ("z_pres", zp, zp64)]
                            + [(f"W{i}", a, e) for i, (a, e) in enumerate(zip(W, W64))]):
        err = np.linalg.norm(got.grad.cpu().numpy() - want.grad.numpy()) / \
            max(np.linalg.norm(want.grad.numpy()), 1e-12)
        assert err < 6e-2, (name, err)


def test_air_model_dispatches_through_torch_ops():
    """Every hot-path launch of an AIRModel train step (fused bf16 and fp32)
    goes through torch.ops.mog_air (recorded with a TorchDispatchMode)."""
    from torch.utils._python_dispatch import TorchDispatchMode

    from mog_air.air_model import AIRModel

    class Rec(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.names = set()

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            self.names.add(str(func.overloadpacket))
            return func(*args, **(kwargs or {}))

    x, k = ao.synthetic_canvases(64, seed=3)
    for prec in ("bf16", "fp32"):
        m = AIRModel(max_steps=3, scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                     learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=True,
                     scope="disp" + prec, device=DEV, precision=prec)
        X, K = torch.tensor(x, device=DEV), torch.tensor(k, device=DEV)
        with Rec() as rec:
            m.train_step_async(X, K)
        torch.cuda.synchronize()
        want = {"mog_air.gemm_f32_", "mog_air.lstm_cell_forward_", "mog_air.air_step_forward_",
                "mog_air.recon_loss_", "mog_air.air_step_backward_",
                "mog_air.lstm_cell_backward_", "mog_air.clip_adam_", "mog_air.stn_backward_"}
        want |= ({"mog_air.stn_vae_step_", "mog_air.gemm_bf16_",
                  "mog_air.stn_backward_sigmoid_"} if prec == "bf16"
                 else {"mog_air.stn_forward_", "mog_air.vae_sample_forward_"})
        assert want <= rec.names, sorted(want - rec.names)

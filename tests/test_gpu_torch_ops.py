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
        # (batch 64 runs the batched VAE: every loop step's scalars in one launch)
        want = {"mog_air.gemm_f32_", "mog_air.lstm_cell_forward_",
                "mog_air.air_step_forward_steps_", "mog_air.air_runloss_",
                "mog_air.recon_loss_", "mog_air.air_step_backward_",
                "mog_air.lstm_cell_backward_", "mog_air.clip_adam_", "mog_air.stn_backward_"}
        want |= ({"mog_air.stn_vae_step_", "mog_air.gemm_bf16_",
                  "mog_air.stn_backward_sigmoid_"} if prec == "bf16"
                 else {"mog_air.stn_vae_step_f32_"} if m.fused_f32 and 3 * 64 >= m.FUSED_F32_MIN_ROWS
                 else {"mog_air.stn_forward_", "mog_air.vae_sample_forward_"})
        assert want <= rec.names, sorted(want - rec.names)


def test_asr_model_dispatches_through_torch_ops():
    """Every hot-path launch of an AIR-ASR train step (train_air_pr.py config:
    learned z_pres prior, number regularisers) goes through torch.ops.mog_air,
    the ASR cells and structural losses (air_number_bbox_location.py:384-1084)
    included; no ctypes launch remains on the step."""
    from torch.utils._python_dispatch import TorchDispatchMode

    from mog_air import _lib
    from mog_air.asr_model import AIRModel as AsrModel

    class Rec(TorchDispatchMode):
        def __init__(self):
            super().__init__()
            self.names = set()

        def __torch_dispatch__(self, func, types, args=(), kwargs=None):
            self.names.add(str(func.overloadpacket))
            return func(*args, **(kwargs or {}))

    calls = []
    real = _lib.call
    _lib.call = lambda name, *a: (calls.append(name), real(name, *a))[1]
    try:
        x, k = ao.synthetic_canvases(32, seed=4)
        for prec in ("bf16", "fp32"):
            m = AsrModel(None, None, max_steps=3, max_digits=3, cnn=False, train=True,
                         scope="asrdisp" + prec, device=DEV, precision=prec,
                         learning_rate=1e-4, gradient_clipping_norm=1.0,
                         constrains_num=[1, 3], constrains_margin_gamma=100.0,
                         constrains_num_element_gamma=10.0, constrains_area_minmax=[17, 23],
                         z_pres_temperature=0.1, stopping_threshold=0.9)
            X, K = torch.tensor(x, device=DEV), torch.tensor(k, device=DEV)
            with Rec() as rec:
                m.train_step_async(X, K)
            torch.cuda.synchronize()
            want = {"mog_air.asr_pack_", "mog_air.asr_step_forward_", "mog_air.asr_terms_",
                    "mog_air.asr_finalize_", "mog_air.asr_terms_backward_",
                    "mog_air.asr_step_backward_", "mog_air.add_",
                    "mog_air.gemm_f32_", "mog_air.lstm_cell_forward2_", "mog_air.recon_loss_",
                    "mog_air.lstm_cell_backward2_", "mog_air.clip_adam_"}
            assert want <= rec.names, sorted(want - rec.names)
            # (a batch of 32: the recurrent-input gradient in K parts, summed
            # by the parts form of the unpack)
            assert {"mog_air.asr_unpack_", "mog_air.asr_unpack_parts_"} & rec.names
    finally:
        _lib.call = real
    assert not calls, calls


def test_ops_validate_operands():
    """The launch-level ops reject, before any launch, an operand that is too
    small for the extent the kernel touches, of the wrong dtype, or on the
    host (ADVICE: a wrongly shaped tensor must be an error, not an
    out-of-bounds device write)."""
    ops = torch.ops.mog_air
    r = torch.empty(10, device=DEV)
    with pytest.raises(RuntimeError, match="touches"):
        ops.add_(r, r, torch.empty(5, device=DEV), 10)
    with pytest.raises(RuntimeError, match="must be"):
        ops.add_(r, r.to(torch.bfloat16), torch.empty(10, device=DEV), 10)
    with pytest.raises((RuntimeError, NotImplementedError)):
        ops.add_(r.cpu(), r.cpu(), r.cpu(), 10)
    A = torch.empty((64, 32), device=DEV)
    with pytest.raises(RuntimeError, match="touches"):  # C needs (64-1)*64+64 elements
        ops.gemm_f32_([A], [torch.empty((32, 64), device=DEV)], [torch.empty((64, 32), device=DEV)],
                      [None], [None], [None], [None], [None], 64, 64, 32, 32, 64, 64, 64, False,
                      False, 0, 0.0, 1)


def test_opcheck_launch_level_ops():
    """torch.library.opcheck on launch-level ops: the schemas' (x!)
    annotations match what the kernels write (test_schema) and the ops
    behave under fake / functionalized dispatch."""
    from torch.library import opcheck
    ops = torch.ops.mog_air
    n = 1000
    a, b = torch.randn(n, device=DEV), torch.randn(n, device=DEV)
    opcheck(ops.add_.default, (a, b, torch.empty(n, device=DEV), n),
            test_utils=("test_schema",))
    opcheck(ops.rng_fill_.default, (torch.empty(n, device=DEV), 7, 0, True),
            test_utils=("test_schema",))
    B, Z = 40, 50
    mu, lv, ep = (torch.randn(B, Z, device=DEV) * 0.3 for _ in range(3))
    act = torch.ones(B, device=DEV)
    opcheck(ops.vae_sample_forward_.default,
            (B, Z, 0.0, 1.0, 0.0, mu, lv, ep, torch.empty(B, Z, device=DEV),
             torch.zeros(B, 56, device=DEV, dtype=torch.bfloat16), 56, act,
             torch.zeros(B, device=DEV), torch.empty(B, device=DEV)),
            test_utils=("test_schema",))
    G = torch.randn(B, 4 * 256, device=DEV)
    opcheck(ops.lstm_cell_forward_.default,
            (G, None, torch.randn(B, 256, device=DEV), torch.empty(B, 256, device=DEV),
             torch.empty(B, 256, device=DEV), B, 256),
            test_utils=("test_schema",))


def test_lstm_cell_pair_ops_match_single_cells_bitwise():
    """lstm_cell_forward2_ / lstm_cell_backward2_ (both AIR-ASR cells in one
    launch) write exactly what two single-cell launches write, the optional
    operands (c_prev, dc, dGsum) absent in one cell and present in the other;
    the schemas' mutation annotations hold (opcheck)."""
    from torch.library import opcheck
    ops = torch.ops.mog_air
    g = torch.Generator(device="cpu").manual_seed(11)
    B, H = 77, 256

    def rn(*s):
        return torch.randn(*s, generator=g).to(DEV)

    G0, G1, cp1 = rn(B, 4 * H), rn(B, 4 * H), rn(B, H)
    single = [torch.empty(B, H, device=DEV) for _ in range(4)]
    ops.lstm_cell_forward_(G0, None, None, single[0], single[1], B, H)
    ops.lstm_cell_forward_(G1, None, cp1, single[2], single[3], B, H)
    pair = [torch.empty(B, H, device=DEV) for _ in range(4)]
    ops.lstm_cell_forward2_(G0, None, pair[0], pair[1], G1, cp1, pair[2], pair[3], B, H)
    for a, b in zip(single, pair):
        assert torch.equal(a, b)
    cc0, cc1, dh0, dh1, dc1 = rn(B, H), rn(B, H), rn(B, H), rn(B, H), rn(B, H)
    s0, s1 = rn(B, 4 * H), rn(B, 4 * H)
    outs_s = [torch.empty(B, 4 * H, device=DEV), torch.empty(B, H, device=DEV),
              torch.empty(B, 4 * H, device=DEV), torch.empty(B, H, device=DEV)]
    gs_s = s1.clone()
    ops.lstm_cell_backward_(G0, None, None, cc0, dh0, None, outs_s[0], outs_s[1], None, B, H)
    ops.lstm_cell_backward_(G1, None, cp1, cc1, dh1, dc1, outs_s[2], outs_s[3], gs_s, B, H)
    outs_p = [torch.empty_like(x) for x in outs_s]
    gs_p = s1.clone()
    ops.lstm_cell_backward2_(G0, None, cc0, dh0, None, outs_p[0], outs_p[1], None,
                             G1, cp1, cc1, dh1, dc1, outs_p[2], outs_p[3], gs_p, B, H)
    torch.cuda.synchronize()
    for a, b in zip(outs_s + [gs_s], outs_p + [gs_p]):
        assert torch.equal(a, b)
    assert not torch.equal(gs_p, s1)
    opcheck(ops.lstm_cell_forward2_.default,
            (G0, None, pair[0], pair[1], G1, cp1, pair[2], pair[3], B, H),
            test_utils=("test_schema",))
    opcheck(ops.lstm_cell_backward2_.default,
            (G0, cp1, cc0, dh0, dc1, outs_p[0], outs_p[1], s0.clone(),
             G1, cp1, cc1, dh1, dc1, outs_p[2], outs_p[3], s1.clone(), B, H),
            test_utils=("test_schema",))


def test_gemm_kseg_group_matches_single_chains_bitwise():
    """gemm_f32_kseg_group_ (AIR-ASR's three head-gradient chains of one loop
    step in one launch, segment counts 5 / 2 / 1) writes exactly what one
    gemm_f32_kseg_ per problem writes, Cin and a missing Cin included, and the
    chains match a float64 restatement to fp32 accuracy."""
    from mog_air import ops as mops
    g = torch.Generator(device="cpu").manual_seed(5)
    M, N, KS = 70, 256, 64

    def rn(*s):
        return torch.randn(*s, generator=g).to(DEV)

    segs = [([rn(M, KS) for _ in range(n)], [rn(N + 8, KS)[:N] for _ in range(n)]) for n in (5, 2, 1)]
    cin = [rn(M, N), None, rn(M, N)]
    want = []
    for (A, Bs), c in zip(segs, cin):
        out = torch.empty(M, N, device=DEV)
        mops.gemm_kseg(A, Bs, out, M, N, KS, KS, KS, N, transB=True, Cin=c)
        want.append(out)
    got = [torch.empty(M, N, device=DEV) for _ in segs]
    mops.gemm_kseg_group([(A, Bs, o, c) for (A, Bs), o, c in zip(segs, got, cin)], M, N, KS, KS,
                         KS, N, transB=True)
    torch.cuda.synchronize()
    for (A, Bs), c, w, o in zip(segs, cin, want, got):
        assert torch.equal(w, o)
        ref = sum(a.double() @ b.double().T for a, b in zip(A, Bs))
        if c is not None:
            ref = ref + c.double()
        assert (o.double() - ref).abs().max() <= 1e-5 * ref.abs().max()


# ------------------------------------------------ heads + concrete step op ----
_STEP_CFG = [0.99, 1.0, -2.0, 0.3, -1.0, 0.05, float(np.log(0.05)), 0.0, 1.0, 0.0]


def _air_step_inputs(seed, B=96, H=256, HS=64):
    rng = np.random.default_rng(seed)
    t = lambda a: torch.tensor(np.asarray(a, np.float32), device=DEV)  # noqa: E731
    h = t(rng.standard_normal((B, H)) * 0.5)
    W1 = [t(rng.standard_normal((H, HS)) * 0.08) for _ in range(5)]
    b1 = [t(rng.standard_normal(HS) * 0.05) for _ in range(5)]
    ks = (1, 1, 2, 2, 1)
    W2 = [t(rng.standard_normal((HS, k)) * 0.1) for k in ks]
    b2 = [t(rng.standard_normal(k) * 0.1) for k in ks]
    es, eh = t(rng.standard_normal(B)), t(rng.standard_normal((B, 2)))
    u = t(rng.uniform(0.05, 0.95, B))
    stop = t(rng.choice([0.0, 0.4, 1.5], B))
    rl = t(rng.standard_normal(B))
    dig = torch.tensor(rng.integers(0, 3, B).astype(np.int32), device=DEV)
    live = torch.ones(1, device=DEV, dtype=torch.int32)
    return h, W1, b1, W2, b2, es, eh, u, stop, rl, dig, live


def _step_c_abi(h, W1, b1, W2, b2, es, eh, u, stop, rl, dig, live, cfg, num_prior):
    """The AIRModel's launch sequence for one step (hidden GEMM + step kernel)."""
    from mog_air import ops
    from mog_air.air_model import R_NREC
    B, H = h.shape
    HS = W1[0].shape[1]
    e = lambda *s: torch.empty(s, device=DEV)  # noqa: E731
    hid = e(5, B, HS)
    ops.gemm([h] * 5, W1, [hid[z] for z in range(5)], B, HS, H, H, HS, HS, epi=ops.EPI_RELU,
             bias=b1)
    st, r, d = stop.clone(), rl.clone(), dig.clone()
    lv = torch.zeros(2, device=DEV, dtype=torch.int32)
    lv[0] = live[0]
    outs = dict(rec=e(R_NREC, B), th_f=e(B, 6), th_b=e(B, 6), scale=e(B), shift=e(B, 2),
                zprob=e(B), zkl=e(B), skl=e(B), shkl=e(B), zmask=e(B), zval=e(B), zc=e(B))
    torch.ops.mog_air.air_step_forward_(
        B, HS, HS, 0, True, num_prior, *cfg, [hid[z] for z in range(5)], W2, b2, es, eh, u, st, r,
        d, lv, outs["rec"], outs["th_f"], outs["th_b"], outs["scale"], outs["shift"],
        outs["zprob"], outs["zkl"], outs["skl"], outs["shkl"], outs["zmask"], outs["zval"],
        outs["zc"])
    outs.update(hid=hid, stop=st, runloss=r, digits=d, live=lv[1:])
    return outs


def _step64(h, W1, b1, W2, b2, es, eh, u, stop, rl, cfg, num_prior):
    """float64 torch restatement of one step (air_model.py:458-520, 552-705)."""
    thr, T, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = cfg
    hid = [torch.relu(h @ W1[z] + b1[z]) for z in range(5)]
    o = [hid[z] @ W2[z] + b2[z] for z in range(5)]
    sm, slv, lo, hm, hv = o[0][:, 0], o[1][:, 0], o[4][:, 0], o[2], o[3]
    s = torch.sigmoid(sm + es * torch.sqrt(torch.exp(slv)))
    tt = torch.tanh(hm + eh * torch.sqrt(torch.exp(hv)))
    tx, ty = tt[:, 0], tt[:, 1]
    zero = torch.zeros_like(s)
    thf = torch.stack([s, zero, tx, zero, s, ty], 1)
    thb = torch.stack([1 / s, zero, -tx / s, zero, 1 / s, -ty / s], 1)
    y = (lo + (torch.log(u + 1e-9) - torch.log((1 - u) + 1e-9))) / T
    z = torch.sigmoid(y)
    zkl = at.concrete_kl(y, plo + pb, T, lo, T)
    kl_end = at.concrete_kl(y, -100.0, T, lo, T) if num_prior else zero
    act = (stop + (1 - z.detach())) < thr
    skl = 0.5 * ((((s_plv - slv) - 1) + torch.exp(slv) / s_pv) + (sm - s_pm) ** 2 / s_pv)
    g = lambda m, v: (((h_plv - v) - 1) + torch.exp(v) / h_pv) + (m - h_pm) ** 2 / h_pv  # noqa
    shkl = 0.5 * (g(hm[:, 0], hv[:, 0]) + g(hm[:, 1], hv[:, 1]))
    rl_out = rl + torch.where(stop < thr, zkl, kl_end) + torch.where(act, skl + shkl, zero)
    return thf, thb, torch.where(act, z, zero), rl_out, act


@pytest.mark.parametrize("num_prior", [False, True])
def test_air_step_op_matches_c_abi_bitwise(num_prior):
    """torch.ops.mog_air.air_step (heads + concrete z_pres step) against the
    AIRModel's C-ABI launch sequence: every output bitwise; its autograd
    against mog_air_step_backward with the scalar grad_scale (dh bitwise,
    the split-K weight gradients to fp32 rounding)."""
    from mog_air import ops
    ins = _air_step_inputs(5 + num_prior)
    h, W1, b1, W2, b2, es, eh, u, stop, rl, dig, live = ins
    ref = _step_c_abi(*ins, _STEP_CFG, num_prior)
    hq = h.clone().requires_grad_()
    W1q = [w.clone().requires_grad_() for w in W1]
    W2q = [w.clone().requires_grad_() for w in W2]
    b1q = [w.clone().requires_grad_() for w in b1]
    b2q = [w.clone().requires_grad_() for w in b2]
    out = torch.ops.mog_air.air_step(hq, W1q, b1q, W2q, b2q, es, eh, u, stop, rl, dig, live,
                                     _STEP_CFG, True, num_prior)
    names = ["th_f", "th_b", "zc", "zmask", "runloss", "stop", "digits", "live", "zprob", "scale",
             "shift", "zkl", "skl", "shkl", "rec", "hid"]
    for n, o in zip(names, out):
        np.testing.assert_array_equal(o.detach().cpu().numpy(), ref[n].cpu().numpy(), err_msg=n)
    B = h.shape[0]
    rng = np.random.default_rng(9)
    Gf = torch.tensor(rng.standard_normal((B, 6)).astype(np.float32), device=DEV)
    Gb = torch.tensor(rng.standard_normal((B, 6)).astype(np.float32), device=DEV)
    Gz = torch.tensor(rng.standard_normal(B).astype(np.float32), device=DEV)
    gs = 1.0 / B
    loss = (out[0] * Gf).sum() + (out[1] * Gb).sum() + (out[2] * Gz).sum() + out[4].sum() * gs
    grads = torch.autograd.grad(loss, [hq, *W1q, *b1q, *W2q, *b2q])
    HS = W1[0].shape[1]
    dout, dhid = torch.empty((5, B, 2), device=DEV), torch.empty((5, B, HS), device=DEV)
    thr, T, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = _STEP_CFG
    hid_l = [ref["hid"][z] for z in range(5)]
    torch.ops.mog_air.air_step_backward_(B, HS, True, num_prior, T, plo, pb, s_pm, s_pv, h_pm,
                                         h_pv, gs, None, ref["rec"], es, eh, Gf, Gb, Gz, hid_l,
                                         W2, dout[0], B * 2, dhid[0], B * HS)
    dh = torch.empty_like(h)
    ops.gemm_kseg([dhid[z] for z in range(5)], W1, dh, B, h.shape[1], HS, HS, HS, h.shape[1],
                  transB=True)
    np.testing.assert_array_equal(grads[0].cpu().numpy(), dh.cpu().numpy())
    for z in range(5):
        np.testing.assert_allclose(grads[1 + z].cpu().numpy(),
                                   (h.T @ dhid[z]).cpu().numpy(), rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(grads[11 + z].cpu().numpy(),
                                   (ref["hid"][z].T @ dout[z][:, :W2[z].shape[1]]).cpu().numpy(),
                                   rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(grads[16 + z].cpu().numpy(),
                                   dout[z][:, :W2[z].shape[1]].sum(0).cpu().numpy(),
                                   rtol=1e-4, atol=1e-6)


def test_air_step_op_autograd_vs_float64():
    """Per-image running-loss cotangents (dloss) included: gradients of the op
    against float64 autograd of the restated step."""
    ins = _air_step_inputs(11)
    h, W1, b1, W2, b2, es, eh, u, stop, rl, dig, live = ins
    req = lambda ts: [t.clone().requires_grad_() for t in ts]  # noqa: E731
    hq, W1q, b1q, W2q, b2q = req([h])[0], req(W1), req(b1), req(W2), req(b2)
    out = torch.ops.mog_air.air_step(hq, W1q, b1q, W2q, b2q, es, eh, u, stop, rl, dig, live,
                                     _STEP_CFG, True, True)
    B = h.shape[0]
    rng = np.random.default_rng(12)
    G = [torch.tensor(rng.standard_normal(s).astype(np.float32), device=DEV)
         for s in ((B, 6), (B, 6), (B,), (B,))]
    loss = sum((o * g).sum() for o, g in zip((out[0], out[1], out[2], out[4]), G))
    grads = torch.autograd.grad(loss, [hq, *W1q, *b1q, *W2q, *b2q])
    d = lambda ts: [t.detach().cpu().double().requires_grad_() for t in ts]  # noqa: E731
    h6, W16, b16, W26, b26 = d([h])[0], d(W1), d(b1), d(W2), d(b2)
    c = lambda t: t.cpu().double()  # noqa: E731
    thf, thb, zc, rlo, act = _step64(h6, W16, b16, W26, b26, c(es), c(eh), c(u), c(stop), c(rl),
                                     _STEP_CFG, True)
    np.testing.assert_array_equal(act.numpy(), out[3].detach().cpu().numpy() != 0)
    np.testing.assert_allclose(out[4].detach().cpu().numpy(), rlo.detach().numpy(), rtol=1e-4,
                               atol=1e-4)
    l64 = sum((o * c(g)).sum() for o, g in zip((thf, thb, zc, rlo), G))
    g64 = torch.autograd.grad(l64, [h6, *W16, *b16, *W26, *b26])
    for i, (a, b) in enumerate(zip(grads, g64)):
        bn = b.numpy()
        tol = 2e-3 * max(1.0, float(np.abs(bn).max()))
        np.testing.assert_allclose(a.cpu().numpy(), bn, rtol=2e-3, atol=tol, err_msg=str(i))


def test_air_step_backward_per_image_dloss():
    """mog_air_step_backward's dloss: each image's head-output gradient equals
    the one a uniform grad_scale of that image's value gives (bitwise)."""
    ins = _air_step_inputs(13)
    h, W1, b1, W2, b2, es, eh, u, stop, rl, dig, live = ins
    ref = _step_c_abi(*ins, _STEP_CFG, True)
    B, HS = h.shape[0], W1[0].shape[1]
    rng = np.random.default_rng(14)
    Gf = torch.tensor(rng.standard_normal((B, 6)).astype(np.float32), device=DEV)
    Gb = torch.tensor(rng.standard_normal((B, 6)).astype(np.float32), device=DEV)
    Gz = torch.tensor(rng.standard_normal(B).astype(np.float32), device=DEV)
    thr, T, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = _STEP_CFG
    hid_l = [ref["hid"][z] for z in range(5)]

    def run(gs, dl):
        dout, dhid = torch.empty((5, B, 2), device=DEV), torch.empty((5, B, HS), device=DEV)
        torch.ops.mog_air.air_step_backward_(B, HS, True, True, T, plo, pb, s_pm, s_pv, h_pm,
                                             h_pv, gs, dl, ref["rec"], es, eh, Gf, Gb, Gz, hid_l,
                                             W2, dout[0], B * 2, dhid[0], B * HS)
        return dout.cpu().numpy(), dhid.cpu().numpy()

    odd = np.arange(B) % 2 == 1
    dl = torch.tensor(np.where(odd, 2.0, 0.5).astype(np.float32), device=DEV)
    mix = run(0.0, dl)
    for v, rows in ((0.5, ~odd), (2.0, odd)):
        uni = run(v, None)
        for a, b in zip(mix, uni):
            np.testing.assert_array_equal(a[:, rows], b[:, rows])


def test_air_step_backward_steps_match_single_steps_bitwise():
    """air_step_backward_ over T loop steps in one launch (steps=T: records
    [T][17][B], the other operands over T*B rows, the dloss per image) writes
    exactly what T single-step launches write."""
    T_ = 3
    steps = [_air_step_inputs(21 + t) for t in range(T_)]
    refs = [_step_c_abi(*ins, _STEP_CFG, False) for ins in steps]
    B, HS = steps[0][0].shape[0], steps[0][1][0].shape[1]
    W2 = steps[0][3]
    rng = np.random.default_rng(22)

    def rn(*s):
        return torch.tensor(rng.standard_normal(s).astype(np.float32), device=DEV)

    Gf, Gb, Gz = rn(T_, B, 6), rn(T_, B, 6), rn(T_, B)
    es = torch.stack([ins[5] for ins in steps])
    eh = torch.stack([ins[6] for ins in steps])
    rec = torch.stack([r["rec"] for r in refs]).contiguous()
    hid = [torch.stack([r["hid"][z] for r in refs]).contiguous() for z in range(5)]
    dl = torch.tensor(rng.uniform(0.5, 2.0, B).astype(np.float32), device=DEV)
    thr, tmp, plo, pb, s_pm, s_pv, s_plv, h_pm, h_pv, h_plv = _STEP_CFG
    for dloss in (None, dl):
        d1, h1 = torch.empty((5, T_, B, 2), device=DEV), torch.empty((T_, B, 5 * HS), device=DEV)
        for t in range(T_):
            torch.ops.mog_air.air_step_backward_(
                B, HS, True, False, tmp, plo, 0.0, s_pm, s_pv, h_pm, h_pv, 1.0 / B, dloss, rec[t],
                es[t], eh[t], Gf[t], Gb[t], Gz[t], [x[t] for x in hid], W2, d1[0, t], T_ * B * 2,
                h1[t], HS)
        d2, h2 = torch.empty_like(d1), torch.empty_like(h1)
        torch.ops.mog_air.air_step_backward_(
            B, HS, True, False, tmp, plo, 0.0, s_pm, s_pv, h_pm, h_pv, 1.0 / B, dloss, rec, es, eh,
            Gf, Gb, Gz, hid, W2, d2[0], T_ * B * 2, h2, HS, None, T_)
        torch.cuda.synchronize()
        assert torch.equal(d1, d2) and torch.equal(h1, h2)
        assert float(h2.abs().sum()) > 0


def test_stn_forward_periodic_matches_per_step_reads_bitwise():
    """stn_forward with n = T*B images over a B-image U (image i reads U[i % B]:
    every loop step's glimpse read of the shared canvas in one launch) writes
    exactly what T reads of B images write, fp32 and bf16 outputs."""
    from mog_air import ops as mops
    rng = np.random.default_rng(31)
    B, T_ = 37, 3
    U = torch.tensor(rng.random((B, 2500)).astype(np.float32), device=DEV)
    th = torch.tensor(np.concatenate([_theta(rng, B) for _ in range(T_)]), device=DEV).view(T_, B, 6)
    for dt in (torch.float32, torch.bfloat16):
        one = torch.empty((T_, B, 784), device=DEV, dtype=dt)
        for t in range(T_):
            mops.stn_forward(U, th[t], (28, 28), out=one[t])
        allr = torch.empty_like(one)
        mops.stn_forward(U, th.view(T_ * B, 6), (28, 28), out=allr.view(T_ * B, 784), n=T_ * B)
        torch.cuda.synchronize()
        assert torch.equal(one, allr)

"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: fp32 forward values bit-exact with the C oracle
(every elementwise op and every dense layer's k-ordered fma chain), integer
counts bit-exact, reductions (BCE/MSE/KL sums) within 1e-5 relative; backward
within 2e-3 relative of a float64 torch autograd restatement under a
well-conditioned canvas cotangent.
"""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao
from oracle import air_torch as at

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _cuda(a, dtype=torch.float32):
    return torch.as_tensor(np.asarray(a)).to(DEV, dtype).contiguous()


@pytest.mark.parametrize("M,N,K", [(64, 1024, 2500), (37, 50, 256), (128, 784, 512),
                                   (5, 7, 3), (64, 64, 0)])
def test_gemm_bit_exact_chain(M, N, K):
    from mog_air import ops
    rng = np.random.default_rng(M + N + K)
    x = rng.standard_normal((M, K)).astype(np.float32)
    w = rng.standard_normal((K, N)).astype(np.float32)
    b = rng.standard_normal(N).astype(np.float32)
    ref = ao.dense_chain(x, w, b)
    out = torch.empty((M, N), device=DEV)
    ops.dense(_cuda(x), _cuda(w), _cuda(b), out)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


def test_gemm_kseg_is_one_chain():
    """mog_gemm_f32_kseg: five K-segments (the heads' dh = sum_z dhid_z W1_z^T
    form) equal ONE k-ordered chain over the concatenated K, bit for bit."""
    from mog_air import _lib
    rng = np.random.default_rng(11)
    M, N, ks, S = 300, 256, 64, 5
    A = [rng.standard_normal((M, ks)).astype(np.float32) for _ in range(S)]
    W = [rng.standard_normal((N, ks)).astype(np.float32) for _ in range(S)]  # [N][K] (transB)
    Acat = np.concatenate(A, 1)
    Wcat = np.concatenate(W, 1)
    ref = ao.dense_chain(Acat, np.ascontiguousarray(Wcat.T), np.zeros(N, np.float32))
    dA = [_cuda(a) for a in A]
    dW = [_cuda(w) for w in W]
    out = torch.empty((M, N), device=DEV)
    _lib.call("mog_gemm_f32_kseg", S, _lib.ptr_array([a.data_ptr() for a in dA]),
              _lib.ptr_array([w.data_ptr() for w in dW]), out.data_ptr(), None, None,
              M, N, ks, ks, ks, N, 0, 1, 0, None)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), ref)


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (True, True)])
def test_gemm_transposes(ta, tb):
    from mog_air import ops
    rng = np.random.default_rng(3)
    M, N, K = 70, 90, 130
    A = rng.standard_normal((M, K)).astype(np.float32)
    Bm = rng.standard_normal((K, N)).astype(np.float32)
    As = A.T.copy() if ta else A
    Bs = Bm.T.copy() if tb else Bm
    out = torch.empty((M, N), device=DEV)
    ops.gemm([_cuda(As)], [_cuda(Bs)], [out], M, N, K, As.shape[1], Bs.shape[1], N,
             transA=ta, transB=tb)
    np.testing.assert_allclose(out.cpu().numpy(), A.astype(np.float64) @ Bm, rtol=1e-4,
                               atol=1e-3)


def test_gemm_splitk_atomic():
    from mog_air import ops
    rng = np.random.default_rng(4)
    M, N, K = 100, 60, 5000
    A = rng.standard_normal((K, M)).astype(np.float32)   # stored transposed
    Bm = rng.standard_normal((K, N)).astype(np.float32)
    out = torch.zeros((M, N), device=DEV)
    ops.gemm([_cuda(A)], [_cuda(Bm)], [out], M, N, K, M, N, N, transA=True,
             epi=ops.EPI_ATOMIC, splitk=8)
    np.testing.assert_allclose(out.cpu().numpy(), A.T.astype(np.float64) @ Bm, rtol=1e-4,
                               atol=2e-3)


@pytest.mark.parametrize("M,N,K,lda,ldb,nb", [(256, 50, 24576, 256, 50, 2), (50, 256, 3001, 52, 260, 1),
                                              (64, 1, 24576, 64, 2, 3), (64, 2, 777, 64, 2, 2),
                                              (64, 2, 192, 64, 2, 2), (256, 64, 8192, 256, 320, 5),
                                              (17, 13, 200, 20, 16, 1)])
def test_gemm_narrow_weight_gradients(M, N, K, lda, ldb, nb):
    """The split-K weight gradients of the narrow layers (transA + atomic):
    batched, with strides and column sums, against float64; one K chunk
    (K < 512: split-K 1) is deterministic."""
    from mog_air import ops
    rng = np.random.default_rng(40 + M + N)
    A = [rng.standard_normal((K, lda)).astype(np.float32) for _ in range(nb)]
    Bm = [rng.standard_normal((K, ldb)).astype(np.float32) for _ in range(nb)]
    Ad, Bd = [_cuda(a) for a in A], [_cuda(b) for b in Bm]

    def run():
        out = [torch.full((M, N), 0.5, device=DEV) for _ in range(nb)]
        cs = [torch.full((N,), -1.0, device=DEV) for _ in range(nb)]
        ops.gemm(Ad, Bd, out, M, N, K, lda, ldb, N, transA=True, epi=ops.EPI_ATOMIC,
                 splitk=max(1, min(K // 256, 8)), colsum=cs)
        return [o.cpu().numpy() for o in out], [c.cpu().numpy() for c in cs]

    out, cs = run()
    for i in range(nb):
        ref = A[i][:, :M].astype(np.float64).T @ Bm[i][:, :N] + 0.5
        mag = np.abs(A[i][:, :M]).astype(np.float64).T @ np.abs(Bm[i][:, :N])
        assert (np.abs(out[i] - ref) <= 1e-6 * mag + 1e-6).all()
        csr = Bm[i][:, :N].astype(np.float64).sum(0) - 1.0
        assert (np.abs(cs[i] - csr) <= 1e-6 * np.abs(Bm[i][:, :N]).sum(0) + 1e-6).all()
    if K < 512:
        out2, cs2 = run()
        for i in range(nb):
            np.testing.assert_array_equal(out[i], out2[i])
            np.testing.assert_array_equal(cs[i], cs2[i])


def test_stn_forward_bit_exact():
    from mog_air import ops
    rng = np.random.default_rng(5)
    N = 32
    U = rng.uniform(size=(N, 50, 50)).astype(np.float32)
    s = rng.uniform(0.05, 1.2, N).astype(np.float32)
    t = rng.uniform(-1.5, 1.5, (N, 2)).astype(np.float32)
    th = np.stack([s, 0 * s, t[:, 0], 0 * s, s, t[:, 1]], 1).astype(np.float32)
    ref = ao.stn(U, th, (28, 28)).reshape(N, -1)
    out = ops.stn_forward(_cuda(U.reshape(N, -1)), _cuda(th), (28, 28))
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
    # write direction with theta^-1
    r = rng.uniform(size=(N, 28, 28)).astype(np.float32)
    thb = np.stack([1 / s, 0 * s, -t[:, 0] / s, 0 * s, 1 / s, -t[:, 1] / s], 1).astype(np.float32)
    ref_w = ao.stn(r, thb, (50, 50)).reshape(N, -1)
    out_w = ops.stn_forward(_cuda(r.reshape(N, -1)), _cuda(thb), (50, 50))
    np.testing.assert_array_equal(out_w.cpu().numpy(), ref_w)


def test_stn_accumulate_masked():
    from mog_air import ops
    rng = np.random.default_rng(6)
    N = 8
    r = rng.uniform(size=(N, 784)).astype(np.float32)
    s = rng.uniform(0.2, 0.9, N).astype(np.float32)
    thb = np.stack([1 / s, 0 * s, 0 * s, 0 * s, 1 / s, 0 * s], 1).astype(np.float32)
    canvas0 = rng.uniform(size=(N, 2500)).astype(np.float32)
    z = rng.uniform(size=N).astype(np.float32)
    mask = (np.arange(N) % 2).astype(np.float32)
    w = ao.stn(r.reshape(N, 28, 28), thb, (50, 50)).reshape(N, -1)
    ref = np.where(mask[:, None] != 0, canvas0 + z[:, None] * w, canvas0)
    cv = _cuda(canvas0)
    ops.stn_forward(_cuda(r), _cuda(thb), (50, 50), out=cv, z=_cuda(z), mask=_cuda(mask),
                    accumulate=True)
    np.testing.assert_array_equal(cv.cpu().numpy(), ref)


@pytest.mark.parametrize("sep", [True, False])
@pytest.mark.parametrize("src,dst", [(28, 50), (50, 28), (28, 64)])
def test_stn_backward_vs_autograd(sep, src, dst):
    """axis-aligned transforms take the separable (atomic-free) dU path,
    sheared ones the LDS-atomic path; both against float64 autograd."""
    from mog_air import ops
    rng = np.random.default_rng(7 + src + dst)
    N = 16
    r = rng.uniform(size=(N, src, src))
    s = rng.uniform(0.2, 0.9, N)
    t = rng.uniform(-0.8, 0.8, (N, 2))
    sh = np.zeros(N) if sep else rng.uniform(-0.2, 0.2, N)
    thb = np.stack([1 / s, sh, -t[:, 0] / s, -sh, 1 / s, -t[:, 1] / s], 1)
    G = rng.standard_normal((N, dst * dst))
    gs = rng.uniform(size=N)
    U = torch.tensor(r, requires_grad=True)
    TH = torch.tensor(thb, requires_grad=True)
    out = at.transformer(U, TH, (dst, dst)).reshape(N, -1)
    (out * torch.tensor(G) * torch.tensor(gs)[:, None]).sum().backward()
    dU, dth, dot = ops.stn_backward(_cuda(r.reshape(N, -1)), _cuda(thb), (dst, dst), _cuda(G),
                                    gscale=_cuda(gs), want_dot=True)
    np.testing.assert_allclose(dU.cpu().numpy(), U.grad.numpy().reshape(N, -1), rtol=1e-4,
                               atol=1e-4)
    gt = TH.grad.numpy()
    got = dth.cpu().numpy()
    for k in (0, 2, 4, 5):
        np.testing.assert_allclose(got[:, k], gt[:, k], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(dot.cpu().numpy(), (out.detach().numpy() * G).sum(1), rtol=1e-4,
                               atol=1e-3)


def test_stn_read_backward_dtheta_only():
    """The STN read backward without dU (canvas -> glimpse, dtheta only: the
    train step's form) stages only the window's source rows: dtheta must be
    bit-identical to the form that stages the whole canvas (want_dU), and match
    float64 autograd -- windows partly outside the canvas, flipped axes and
    tiny / large scales included."""
    from mog_air import ops
    rng = np.random.default_rng(17)
    N = 48
    x = rng.uniform(size=(N, 50, 50))
    s = rng.uniform(0.1, 1.3, N) * np.where(np.arange(N) % 5 == 0, -1.0, 1.0)
    t = rng.uniform(-1.3, 1.3, (N, 2))
    th = np.stack([s, 0 * s, t[:, 0], 0 * s, s, t[:, 1]], 1)
    G = rng.standard_normal((N, 784))
    _, dth_only, _ = ops.stn_backward(_cuda(x.reshape(N, -1)), _cuda(th), (28, 28), _cuda(G),
                                      want_dU=False)
    _, dth_full, _ = ops.stn_backward(_cuda(x.reshape(N, -1)), _cuda(th), (28, 28), _cuda(G))
    assert torch.equal(dth_only, dth_full)
    U = torch.tensor(x)
    TH = torch.tensor(th, requires_grad=True)
    out = at.transformer(U, TH, (28, 28)).reshape(N, -1)
    (out * torch.tensor(G)).sum().backward()
    gt, got = TH.grad.numpy(), dth_only.cpu().numpy()
    for k in (0, 2, 4, 5):
        np.testing.assert_allclose(got[:, k], gt[:, k], rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("sep,dt", [(True, torch.bfloat16), (False, torch.bfloat16),
                                    (True, torch.float32), (False, torch.float32)])
def test_stn_backward_sigmoid_bf16_matches_unfused(sep, dt):
    """The write backward with the output-sigmoid gradient folded in (bf16 or
    fp32 dm straight from the kernel) is bit-identical to dU followed by
    mog_sigmoid_backward; dtheta / dot are unchanged."""
    from mog_air import _lib, ops
    from mog_air.ops import dp, stream_ptr
    rng = np.random.default_rng(31)
    N, W, C = 40, 28, 50
    r = rng.uniform(size=(N, W * W)).astype(np.float32)
    s = rng.uniform(0.2, 0.9, N)
    t = rng.uniform(-0.8, 0.8, (N, 2))
    sh = np.zeros(N) if sep else rng.uniform(-0.2, 0.2, N)
    thb = np.stack([1 / s, sh, -t[:, 0] / s, -sh, 1 / s, -t[:, 1] / s], 1)
    G = rng.standard_normal((N // 2, C * C))  # shared cotangent (g_period)
    gs = rng.uniform(size=N)
    gs[3] = 0.0
    dU, dth, dot = ops.stn_backward(_cuda(r), _cuda(thb), (C, C), _cuda(G), gscale=_cuda(gs),
                                    want_dot=True, n=N)
    ref = torch.empty((N, W * W), device=DEV, dtype=dt)
    _lib.call("mog_sigmoid_backward", dp(_cuda(r)), dp(dU), dp(ref), N * W * W,
              int(dt == torch.bfloat16), stream_ptr())
    dm = torch.full((N, W * W), float("nan"), device=DEV, dtype=dt)
    _, dth2, dot2 = ops.stn_backward(_cuda(r), _cuda(thb), (C, C), _cuda(G), gscale=_cuda(gs),
                                     want_dot=True, n=N, dm=dm)
    torch.cuda.synchronize()
    iv = torch.int16 if dt == torch.bfloat16 else torch.int32
    assert torch.equal(dm.view(iv), ref.view(iv))
    assert torch.equal(dth2, dth) and torch.equal(dot2, dot)


def _setup(batch=16, seed=0, train=True, T=3, num_prior=None, bias_scale=0.05):
    cfg = ao.AirConfig(batch=batch, max_steps=T, train=train, num_prior=num_prior,
                       scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01)
    P = ao.init_params(cfg, seed=100 + seed, bias_scale=bias_scale)
    nz = ao.make_noise(cfg, seed=200 + seed)
    x, k = ao.synthetic_canvases(batch, seed=300 + seed)
    return cfg, P, nz, x, k


def _model(cfg, P, train=True, scope="parity"):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=cfg.canvas_size,
                 scale_prior_variance=cfg.scale_prior_variance,
                 z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                 z_pres_temperature=cfg.z_pres_temperature,
                 stopping_threshold=cfg.stopping_threshold, vae_likelihood_std=cfg.vae_likelihood_std,
                 learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=train,
                 num_prior=cfg.num_prior, scope=scope, device=DEV)
    m.params.load_dict(P)
    return m


def _noise(nz):
    return {k: _cuda(v) for k, v in nz.items()}


@pytest.mark.parametrize("train,seed,num_prior", [(True, 0, None), (False, 1, None),
                                                  (True, 2, (1, 3))])
def test_forward_parity(train, seed, num_prior):
    cfg, P, nz, x, k = _setup(seed=seed, train=train, num_prior=num_prior,
                              T=4 if num_prior else 3)
    ro = ao.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, train=train, scope=f"fwd{seed}")
    m.infer(x, k, noise=_noise(nz))
    assert m.executed_steps == ro["T"]
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ro["digits"])
    np.testing.assert_array_equal(m.rec_scales.cpu().numpy()[..., 0], ro["scale"].T)
    np.testing.assert_array_equal(m.rec_shifts.cpu().numpy(), ro["shift"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_windows.cpu().numpy(), ro["window"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_latents.cpu().numpy(), ro["latent"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.z_pres_probs.cpu().numpy(), ro["z_pres_prob"].T)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ro["canvas"])
    np.testing.assert_array_equal(m.reconstruction.cpu().numpy(), ro["recon"])
    for key in ("z_pres_kls", "scale_kls", "shift_kls"):
        np.testing.assert_array_equal(getattr(m, key).cpu().numpy(),
                                      ro[key.replace("kls", "kl")].T, err_msg=key)
    np.testing.assert_array_equal(m.vae_kls.cpu().numpy(), ro["vae_kl"].T)
    np.testing.assert_allclose(m.reconstruction_loss.cpu().numpy(), ro["bce"], rtol=1e-5)
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ro["loss"], rtol=1e-5)
    assert abs(m.loss - ro["loss_mean"]) <= 1e-3
    assert m.accuracy == pytest.approx(ro["accuracy"])


def test_gradient_parity_vs_float64_autograd():
    cfg, P, nz, x, k = _setup(seed=3, batch=8)
    rng = np.random.default_rng(9)
    Gc = (rng.standard_normal((cfg.batch, 2500)) * 0.01).astype(np.float32)
    m = _model(cfg, P, scope="grad")
    grads = m.compute_gradients(x, k, noise=_noise(nz), canvas_cotangent=_cuda(Gc))
    Pt = at.to_torch(P, requires_grad=True)
    out = at.air_forward(cfg, Pt, at.to_torch(nz), torch.tensor(x, dtype=torch.float64),
                         z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                         canvas_cotangent=torch.tensor(Gc, dtype=torch.float64),
                         fixed_steps=True)
    out["loss"].backward()
    for name, p in Pt.items():
        ref = p.grad.numpy() if p.grad is not None else np.zeros(p.shape)
        got = grads[name]
        err = np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-12)
        assert err < 2e-3 or np.linalg.norm(got - ref) < 1e-6, (name, err)


def test_train_step_adam_parity():
    cfg, P, nz, x, k = _setup(seed=4, batch=8)
    rng = np.random.default_rng(10)
    Gc = (rng.standard_normal((cfg.batch, 2500)) * 0.01).astype(np.float32)
    m = _model(cfg, P, scope="adam")
    grads = m.compute_gradients(x, k, noise=_noise(nz), canvas_cotangent=_cuda(Gc))
    m.params.apply_adam(1e-4, 1.0)
    got = m.params.state_dict()
    Pt = at.to_torch(P, dtype=torch.float32)
    gt = {n: torch.tensor(g) for n, g in grads.items()}
    mt = {n: torch.zeros_like(p) for n, p in Pt.items()}
    vt = {n: torch.zeros_like(p) for n, p in Pt.items()}
    at.tf_clip_adam_step(Pt, gt, mt, vt, 1, lr=1e-4, clip=1.0)
    for n in P:
        np.testing.assert_allclose(got[n], Pt[n].numpy(), rtol=1e-5, atol=1e-7, err_msg=n)


def test_train_steps_finite_and_counts():
    cfg, P, nz, x, k = _setup(seed=5, batch=64)
    m = _model(cfg, P, scope="train")
    losses = []
    for i in range(3):
        loss, acc, mse, gs = m.step(x, k)
        losses.append(loss)
        assert np.isfinite(loss) and 0.0 <= acc <= 1.0
    assert gs == 3
    assert np.all(np.isfinite(m.params.flat.cpu().numpy()))

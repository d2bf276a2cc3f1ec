"""The fp32 fused step kernel (vae_step.hip stn_vae_step_f32_kernel: STN read
-> seven v_mfma_f32_16x16x4_f32 layers with their exact epilogues -> sample ->
output layer -> STN write, 32-image tiles) against the unfused fp32 sequence
it replaces (stn_forward, mog_gemm_f32 chains with pre-activations,
vae_sample_forward, the Philox output epilogue, stn_write_parts) and against
the C oracle, bit for bit.  Reference: air/air_model.py:523-588,
air/vae.py:5-48, air/transformer.py:18-175.
"""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

pytestmark = pytest.mark.gpu
DEV = "cuda:0"

SAVED = ("g", "a1", "a2", "mu", "lv", "d1", "d2")
OUTS = ("z", "r", "vkl", "runloss", "zval", "zmask", "loss_b")


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _setup(batch, seed, canvas=50, T=3, num_prior=None):
    cfg = ao.AirConfig(batch=batch, max_steps=T, scale_prior_variance=0.05,
                       z_pres_prior_log_odds=-0.01, canvas_size=canvas, num_prior=num_prior)
    P = ao.init_params(cfg, seed=1500 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=1600 + seed)
    if canvas == 50:
        x, k = ao.synthetic_canvases(batch, seed=1700 + seed)
    else:
        x, k = ao.synthetic_canvases(batch, canvas=canvas, seed=1700 + seed, counts=(2, 4),
                                     side=(22, 30))
    return cfg, P, nz, x, k


def _model(cfg, P, scope, fused, num_prior=None):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=cfg.canvas_size, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=True, scope=scope, device=DEV, precision="fp32",
                 fused_step=fused, batch_vae=True, num_prior=num_prior)
    m.FUSED_F32_MIN_ROWS = 0  # the fused kernel at these test batches too
    m.params.load_dict(P)
    return m


def _bits(a):
    return a.view(torch.int32)


def _compare(mf, mu, names):
    torch.cuda.synchronize()
    bad = []
    for n in names:
        a, b = _bits(getattr(mf._ws, n)), _bits(getattr(mu._ws, n))
        if not torch.equal(a, b):
            d = a != b
            bad.append((n, int(d.sum()), d.numel()))
    assert not bad, bad
    np.testing.assert_array_equal(mf.canvas.cpu().numpy(), mu.canvas.cpu().numpy())
    assert mf.loss == mu.loss


@pytest.mark.parametrize("batch,canvas", [(128, 50), (192, 50), (64, 64)])
def test_fused_f32_matches_unfused_bitwise(batch, canvas):
    """Training form: every saved activation (glimpse, pre- and post-
    activations, mu / lv / z), r, the VAE KL, the canvas and the loss equal
    the unfused sequence's bits; so do the gradients computed from them."""
    cfg, P, nz, x, k = _setup(batch, seed=batch + canvas, canvas=canvas)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    mf = _model(cfg, P, "f32f%d_%d" % (batch, canvas), True)
    mu = _model(cfg, P, "f32u%d_%d" % (batch, canvas), False)
    assert mf.fused_f32 and not mu.fused_f32 and mf._batched_vae(batch)
    G = torch.as_tensor((np.random.default_rng(7).standard_normal((batch, canvas ** 2)) * 0.01)
                        .astype(np.float32)).to(DEV)
    gf = mf.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    gu = mu.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    _compare(mf, mu, SAVED + OUTS)
    assert torch.equal(mf._ws.prows, mu._ws.prows)
    # same bits into the same backward launches (split-K atomics: the weight-
    # gradient sums may differ in order only)
    for n in gu:
        d = np.linalg.norm(gf[n] - gu[n]) / max(np.linalg.norm(gu[n]), 1e-30)
        assert d < 1e-6, (n, d)


def test_fused_f32_inkernel_noise_matches_unfused():
    """Perf mode (no injected noise): eps_x from the Philox counters inside the
    output layer, in both forms."""
    cfg, P, nz, x, k = _setup(256, seed=3)
    mf = _model(cfg, P, "f32nf", True)
    mu = _model(cfg, P, "f32nu", False)
    mf.noise_seed = mu.noise_seed = 4242
    mf.compute_gradients(x, k)
    mu.compute_gradients(x, k)
    assert mf._ws.eps_x_offset is not None
    _compare(mf, mu, SAVED + OUTS)


@pytest.mark.parametrize("num_prior", [None, (1, 3)])
def test_fused_f32_bit_exact_vs_oracle(num_prior):
    """The fused fp32 step inside the model against the C oracle's forward."""
    T = 4 if num_prior else 3
    cfg, P, nz, x, k = _setup(64, seed=9, T=T, num_prior=num_prior)
    ro = ao.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, "f32o%d" % (num_prior is not None), True, num_prior=num_prior)
    assert m.fused_f32 and m._batched_vae(64)
    m.infer(x, k, noise={n: torch.as_tensor(v).to(DEV) for n, v in nz.items()})
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ro["digits"])
    np.testing.assert_array_equal(m.rec_latents.cpu().numpy(), ro["latent"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.vae_kls.cpu().numpy(), ro["vae_kl"].T)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ro["canvas"])
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ro["loss"], rtol=1e-5)


def test_fused_f32_forward_only_leaves_saved_buffers():
    """save=False (infer): same r / z / KL / parts, saved buffers untouched."""
    cfg, P, nz, x, k = _setup(128, seed=4)
    m = _model(cfg, P, "f32fwd", True)
    X = torch.as_tensor(x).to(DEV)
    m.infer(X, torch.as_tensor(k).to(DEV))
    ws = m._ws
    outs = ("cparts", "prows", "vkl", "r", "z")

    def run(save):
        for n in outs:
            getattr(ws, n).zero_()
        for n in SAVED:
            getattr(ws, n).fill_(7.0)
        m._vae_forward_all(X, ws, 0.3, save=save)
        torch.cuda.synchronize()
        return {n: getattr(ws, n).clone() for n in outs + SAVED}

    tr, fw = run(True), run(False)
    for n in outs:
        assert torch.equal(tr[n].view(torch.int32), fw[n].view(torch.int32)), n
    for n in SAVED:
        assert bool((fw[n] == 7.0).all()), n
        assert not bool((tr[n] == 7.0).all()), n


def test_pack_frag_f32_layout():
    """fragment (ks, ct), lane (li, g), slot kk holds W[16 ks + 4 kk + g][16 ct + li]"""
    from mog_air.ops import _ops
    rng = np.random.default_rng(3)
    K, N = 50, 70
    W = rng.standard_normal((K, N)).astype(np.float32)
    KS, NCT = (K + 15) // 16, (N + 15) // 16
    out = torch.empty(KS * NCT * 256, device=DEV)
    _ops.pack_frag_f32_([torch.as_tensor(W).to(DEV)], [K], [N], [out])
    got = out.cpu().numpy().reshape(KS, NCT, 4, 16, 4)  # ks, ct, g, li, kk
    Wp = np.zeros((KS * 16, NCT * 16), np.float32)
    Wp[:K, :N] = W
    ks, ct, g, li, kk = np.meshgrid(*[np.arange(n) for n in got.shape], indexing="ij")
    np.testing.assert_array_equal(got, Wp[16 * ks + 4 * kk + g, 16 * ct + li])

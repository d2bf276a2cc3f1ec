"""The AIR glimpse VAE of all T loop steps run after the recurrent loop over
T*B rows (AIRModel._vae_forward_all: one fused launch, or T-row-tall GEMMs)
against the per-step schedule, bit for bit, and the fp32 result against the C
oracle.  AIR's VAE never feeds the recurrence (air_model.py:454-456: the LSTM
input is the image alone), so only the running loss needs care: it is
replayed from the step records in the loop's order (mog_air_runloss)."""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


def _setup(batch, seed, train=True, num_prior=None, T=3):
    cfg = ao.AirConfig(batch=batch, max_steps=T, train=train, num_prior=num_prior,
                       scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01)
    P = ao.init_params(cfg, seed=800 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=900 + seed)
    x, k = ao.synthetic_canvases(batch, seed=1000 + seed)
    return cfg, P, nz, x, k


def _model(cfg, P, scope, precision, fused, batched, num_prior=None):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                 learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=cfg.train,
                 scope=scope, device=DEV, precision=precision, fused_step=fused,
                 batch_vae=batched, num_prior=num_prior)
    m.params.load_dict(P)
    return m


def _bits(a):
    return a.view(torch.int16) if a.dtype == torch.bfloat16 else a.view(torch.int32)


@pytest.mark.parametrize("precision,fused", [("fp32", False), ("bf16", True), ("bf16", False)])
def test_batched_vae_matches_per_step_bitwise(precision, fused):
    cfg, P, nz, x, k = _setup(batch=128, seed=1)
    noise = {n: torch.as_tensor(v).to(DEV) for n, v in nz.items()}
    tag = "%s%d" % (precision, fused)
    mb = _model(cfg, P, "bv_b" + tag, precision, fused, True)
    ms = _model(cfg, P, "bv_s" + tag, precision, fused, False)
    assert mb._batched_vae(128) and not ms._batched_vae(128)
    G = torch.as_tensor((np.random.default_rng(5).standard_normal((128, 2500)) * 0.01)
                        .astype(np.float32)).to(DEV)
    gb = mb.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    gs = ms.compute_gradients(x, k, noise=noise, canvas_cotangent=G)
    torch.cuda.synchronize()
    names = ["runloss", "vkl", "mu", "lv", "z", "r", "zval", "zmask", "loss_b"]
    names += ["gb", "a1b", "a2b", "zb", "d1b", "d2b"] if precision == "bf16" else \
        ["g", "a1", "a2", "d1", "d2"]
    for n in names:
        assert torch.equal(_bits(getattr(mb._ws, n)), _bits(getattr(ms._ws, n))), n
    if fused:
        assert torch.equal(mb._ws.prows, ms._ws.prows)
    # parts are stored only inside part_rows: the summed canvas is the check
    # (-0 vs +0 allowed: the loss kernel starts from the first part, the
    # running accumulation from +0)
    np.testing.assert_array_equal(mb.canvas.cpu().numpy(), ms.canvas.cpu().numpy())
    assert mb.loss == ms.loss
    for n in gb:
        np.testing.assert_array_equal(gb[n], gs[n], err_msg=n)


@pytest.mark.parametrize("num_prior", [None, (1, 3)])
def test_batched_vae_fp32_bit_exact_vs_oracle(num_prior):
    cfg, P, nz, x, k = _setup(batch=64, seed=2, num_prior=num_prior, T=4 if num_prior else 3)
    ro = ao.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, "bv_o%d" % (num_prior is not None), "fp32", False, True,
               num_prior=num_prior)
    assert m._batched_vae(64)
    m.infer(x, k, noise={n: torch.as_tensor(v).to(DEV) for n, v in nz.items()})
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ro["digits"])
    np.testing.assert_array_equal(m.rec_latents.cpu().numpy(), ro["latent"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_windows.cpu().numpy(), ro["window"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.vae_kls.cpu().numpy(), ro["vae_kl"].T)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ro["canvas"])
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ro["loss"], rtol=1e-5)


def test_fused_forward_only_matches_training_form_bitwise():
    """The fused step kernel without the backward's saved activations (the
    forward-only form infer() runs) writes the same canvas parts, row ranges,
    VAE KL, r and latents as the training form and leaves the saved buffers
    untouched."""
    cfg, P, nz, x, k = _setup(batch=128, seed=4)
    m = _model(cfg, P, "bv_fwd", "bf16", True, True)
    X = torch.as_tensor(x).to(DEV)
    m.infer(X, torch.as_tensor(k).to(DEV))
    ws = m._ws
    outs = ("cparts", "prows", "vkl", "r", "z")
    saved = ("gb", "a1b", "a2b", "mu", "lv", "zb", "d1b", "d2b")

    def run(save):
        for n in outs:
            getattr(ws, n).zero_()
        for n in saved:
            getattr(ws, n).fill_(7.0)
        m._vae_forward_all(X, ws, 0.3, save=save)
        torch.cuda.synchronize()
        return {n: getattr(ws, n).clone() for n in outs + saved}

    tr, fw = run(True), run(False)
    for n in outs:
        assert torch.equal(_bits(tr[n]), _bits(fw[n])), n
    for n in saved:
        assert bool((fw[n] == 7.0).all()), n
        assert not bool((tr[n] == 7.0).all()), n

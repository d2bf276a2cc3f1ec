"""Every AIR loop step's heads and scalars in one launch each
(mog_air_step_forward_steps, the batched-VAE forward) against the per-step
launches (mog_air_step_forward once per step) on the same parameters and
noise: every record, state and output bitwise, the loop predicate included
(a threshold that stops every image after step 0 makes live[1] = 0, so the
z_pres-term records are rewritten by mog_air_runloss), and the C oracle's
forward bit-exact at the reference's batch of 64.  Reference:
air/air_model.py:435-736 (loop body), :428-432 (predicate)."""
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


def _setup(batch, T, train, num_prior, thr, seed):
    cfg = ao.AirConfig(batch=batch, max_steps=T, train=train, num_prior=num_prior,
                       scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                       stopping_threshold=thr)
    P = ao.init_params(cfg, seed=100 + seed, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=200 + seed)
    x, k = ao.synthetic_canvases(batch, seed=300 + seed)
    return cfg, P, nz, x, k


def _model(cfg, P, scope, one_launch):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=cfg.canvas_size,
                 scale_prior_variance=cfg.scale_prior_variance,
                 z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                 z_pres_temperature=cfg.z_pres_temperature,
                 stopping_threshold=cfg.stopping_threshold,
                 vae_likelihood_std=cfg.vae_likelihood_std, learning_rate=1e-4,
                 gradient_clipping_norm=1.0, cnn=False, train=cfg.train, num_prior=cfg.num_prior,
                 scope=scope, device=DEV)
    m.params.load_dict(P)
    m.STEPS_ONE_LAUNCH = one_launch
    return m


def _bits(t):
    return t.contiguous().view(torch.int32)


FIELDS = ("rec", "th_f", "th_b", "scale", "shift", "zprob", "zkl", "skl", "shkl", "zmask",
          "zval", "zc", "stop", "digits", "live", "runloss", "prows", "h", "hid", "canvas", "recon",
          "loss_b")


@pytest.mark.parametrize("B,T,train,num_prior,thr,grads", [
    (64, 3, True, None, 0.99, True),       # the reference's batch (configs[0] shape)
    (128, 3, False, None, 0.99, False),    # test mode, two workgroups of images
    (192, 4, True, (1, 3), 0.99, False),   # per-step marginal prior bias
    (64, 3, True, None, 1e-6, True),       # every image stops after step 0: live[1] = 0
])
def test_steps_one_launch_matches_per_step(B, T, train, num_prior, thr, grads):
    cfg, P, nz, x, k = _setup(B, T, train, num_prior, thr, seed=B + T)
    noise = {n: torch.as_tensor(np.asarray(v)).to(DEV, torch.float32).contiguous()
             for n, v in nz.items()}
    xs = torch.as_tensor(x).to(DEV).contiguous()
    ks = torch.as_tensor(k).to(DEV).contiguous()
    out = {}
    for one in (True, False):
        m = _model(cfg, P, f"steps{B}_{T}_{thr}_{int(one)}", one)
        if grads:
            m.compute_gradients(xs, ks, noise=noise)
        else:
            m.infer(xs, ks, noise=noise)
        torch.cuda.synchronize()
        ws = m._ws
        out[one] = {f: getattr(ws, f).clone() for f in FIELDS if getattr(ws, f, None) is not None}
        out[one]["loss"] = torch.tensor([m.loss])
        if grads:
            out[one]["grad"] = m.params.grad.clone()
    if thr < 0.5:
        assert int(out[True]["live"][1]) == 0, "the threshold did not stop every image"
    for f, a in out[True].items():
        b = out[False][f]
        assert torch.equal(_bits(a), _bits(b)), f


def test_b64_forward_bit_exact_vs_oracle():
    """The batched path at the reference's batch of 64 (one-launch steps)
    against the C oracle: counts, windows, latents, KLs and canvas bitwise."""
    cfg, P, nz, x, k = _setup(64, 3, True, None, 0.99, seed=7)
    ro = ao.forward(cfg, P, nz, x, k)
    m = _model(cfg, P, "steps_oracle", True)
    noise = {n: torch.as_tensor(np.asarray(v)).to(DEV, torch.float32).contiguous()
             for n, v in nz.items()}
    m.infer(x, k, noise=noise)
    assert m.executed_steps == ro["T"]
    np.testing.assert_array_equal(m.rec_num_digits.cpu().numpy(), ro["digits"])
    np.testing.assert_array_equal(m.rec_scales.cpu().numpy()[..., 0], ro["scale"].T)
    np.testing.assert_array_equal(m.rec_shifts.cpu().numpy(), ro["shift"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.rec_windows.cpu().numpy(), ro["window"].transpose(1, 0, 2))
    np.testing.assert_array_equal(m.z_pres_probs.cpu().numpy(), ro["z_pres_prob"].T)
    np.testing.assert_array_equal(m.canvas.cpu().numpy(), ro["canvas"])
    for key in ("z_pres_kls", "scale_kls", "shift_kls"):
        np.testing.assert_array_equal(getattr(m, key).cpu().numpy(),
                                      ro[key.replace("kls", "kl")].T, err_msg=key)
    np.testing.assert_allclose(m.per_image_loss.cpu().numpy(), ro["loss"], rtol=1e-5)

"""The configurations bench.py times, at their own size and with the model's
default dispatch (no threshold lowered, nothing monkeypatched): the
BASELINE.json headline step -- AIR, B = 8192, T = 3, fp32, bench.make_model's
hyper-parameters and bench.synthetic's canvases, one ``train_step_async``
(forward + backward + clip + TF Adam) -- and configs[1] (the same in bf16).

At B = 8192 the model takes paths no smaller test reaches by default: the
fused fp32 STN-read -> VAE -> STN-write kernel over T*B = 24,576 rows
(FUSED_F32_MIN_ROWS), the NT x3 input gradients (X3_DX_MIN_ROWS), the x3
weight gradients, the side-stream forks (SIDE_MIN_BATCH) and split-K weight
gradients.  Checks:
  * forward: two 64-image slices of the step's per-image records (counts,
    scales, shifts, windows, latents, z_pres probabilities, every KL, the
    canvas) are bit-identical to the C oracle (oracle/air_ref.c, the
    restatement of air/air_model.py:426-900) run on those images with the
    same noise slice (the device Philox noise of the step, eps_x regenerated
    from the kernel's counter range); per-image loss within 1e-5 relative;
  * backward: the gradient of the step equals that of the same step with
    one k pass per weight gradient (ONE_PASS_WGRADS: no split-K) within the
    x3 gate of tests/test_gpu_x3.py in the 2-norm (2e-5 per tensor, 2e-4 for
    tensors of <= 64 entries) and elementwise within 2e-4 of the tensor's
    largest entry (test_gpu_x3's 1e-5 is for 3,072-row sums; these are
    24,576-row sums, and the heads' bias gradients are column sums with heavy
    cancellation: measured 1.4e-5 for recognition_1/weights and 7.9e-5 for
    z_pres/log_odds/hidden/biases) -- the two differ only in how the weight
    gradients' partial sums are ordered;
  * bf16 (configs[1]): counts, scales, shifts, z_pres probabilities and the
    z_pres / scale / shift KLs bit-identical to the fp32 step on the same
    images and noise (AIR's count chain never reads the VAE);
    the batch ELBO within 2e-3 relative of the fp32 step's (DESIGN.md §2's
    bf16 gate); gradients against the bf16 one-pass step as above.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
B = 8192


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")


@pytest.fixture(scope="module")
def data():
    import bench
    x, k = bench.synthetic(B, 1234)  # the bench's rank-0 batch
    return torch.from_numpy(x).to(DEV), torch.from_numpy(k).to(DEV)


def _step(precision, X, K, scope, one_pass=False):
    """One bench train step; returns what the checks read."""
    import bench
    from mog_air import ops
    m = bench.make_model(precision, DEV, 1, 0, scope)
    P0 = m.params.state_dict()
    prior_lo = m.hyper("z_pres_prior_log_odds")
    if one_pass:
        m.ONE_PASS_WGRADS = True
    else:  # the default dispatch this test is about
        assert not m.ONE_PASS_WGRADS
    assert B >= m.SIDE_MIN_BATCH and m._batched_vae(B)
    assert 3 * B >= m.X3_DX_MIN_ROWS and 3 * B >= m.X3_MIN_ROWS
    if precision == "fp32":
        assert m.fused_f32 and 3 * B >= m.FUSED_F32_MIN_ROWS
    else:
        assert m.fused_step
    m.train_step_async(X, K)
    torch.cuda.synchronize()
    ws = m._ws
    assert ws.eps_x_offset is not None  # eps_x generated inside the kernels
    eps_x = torch.empty_like(ws.eps_x)
    ops.rng_fill(eps_x, m.noise_seed, ws.eps_x_offset, True)
    noise = {"eps_scale": ws.eps_scale, "eps_shift": ws.eps_shift, "eps_z": ws.eps_z,
             "eps_x": eps_x, "u": ws.u}
    out = {"P0": P0, "prior_lo": prior_lo, "T": m.executed_steps,
           "noise": {n: v.cpu().numpy() for n, v in noise.items()},
           "grad": m.params.grad_dict(), "loss": m.loss,
           "digits": ws.digits.cpu().numpy(), "loss_b": ws.loss_b.cpu().numpy(),
           "canvas": m.canvas.cpu().numpy()}
    for n in ("scale", "shift", "r", "z", "zprob", "zkl", "skl", "shkl", "vkl"):
        out[n] = getattr(ws, n).cpu().numpy()
    del m
    torch.cuda.empty_cache()
    return out


@pytest.fixture(scope="module")
def fp32(data):
    return _step("fp32", *data, "headline_fp32")


@pytest.fixture(scope="module")
def bf16(data):
    return _step("bf16", *data, "headline_bf16")


def _slices():
    rng = np.random.default_rng(8192)
    return [np.arange(64), np.sort(rng.choice(B, 64, replace=False))]


@pytest.mark.parametrize("which", [0, 1])
def test_headline_fp32_forward_slice_bit_exact_vs_oracle(data, fp32, which):
    from oracle import air_oracle as ao
    idx = _slices()[which]
    X, K = data
    x = X.cpu().numpy()[idx]
    k = K.cpu().numpy()[idx]
    nz = {n: np.ascontiguousarray(v[:, idx]) for n, v in fp32["noise"].items()}
    cfg = ao.AirConfig(batch=len(idx), max_steps=3, train=True, scale_prior_variance=0.05)
    ro = ao.forward(cfg, fp32["P0"], nz, x, k, z_pres_prior_log_odds=fp32["prior_lo"])
    T = ro["T"]
    assert T <= fp32["T"]
    np.testing.assert_array_equal(fp32["digits"][idx], ro["digits"])
    sl = lambda a: a[:T][:, idx]  # noqa: E731
    np.testing.assert_array_equal(sl(fp32["scale"]), ro["scale"])
    np.testing.assert_array_equal(sl(fp32["shift"]), ro["shift"])
    np.testing.assert_array_equal(sl(fp32["r"]), ro["window"])
    np.testing.assert_array_equal(sl(fp32["z"]), ro["latent"])
    np.testing.assert_array_equal(sl(fp32["zprob"]), ro["z_pres_prob"])
    for n, o in (("zkl", "z_pres_kl"), ("skl", "scale_kl"), ("shkl", "shift_kl"),
                 ("vkl", "vae_kl")):
        np.testing.assert_array_equal(sl(fp32[n]), ro[o], err_msg=n)
    np.testing.assert_array_equal(fp32["canvas"][idx], ro["canvas"])
    np.testing.assert_allclose(fp32["loss_b"][idx], ro["loss"], rtol=1e-5)


def _grad_gate(got, ref):
    for n in ref:
        a = got[n].astype(np.float64)
        b = ref[n].astype(np.float64)
        nb = np.linalg.norm(b) + 1e-30
        tol = 2e-5 if b.size > 64 else 2e-4
        assert np.isfinite(a).all(), n
        assert np.linalg.norm(a - b) <= tol * nb, (n, np.linalg.norm(a - b) / nb)
        assert np.abs(a - b).max() <= 2e-4 * (np.abs(b).max() + 1e-30), n


def test_headline_fp32_gradients_vs_one_pass(data, fp32):
    one = _step("fp32", *data, "headline_fp32_1p", one_pass=True)
    np.testing.assert_array_equal(one["loss_b"], fp32["loss_b"])  # same forward
    _grad_gate(fp32["grad"], one["grad"])


def test_configs1_bf16_counts_bit_exact_and_elbo(fp32, bf16):
    for n in ("digits", "scale", "shift", "zprob", "zkl", "skl", "shkl"):
        np.testing.assert_array_equal(bf16[n], fp32[n], err_msg=n)
    assert bf16["T"] == fp32["T"]
    rel = abs(bf16["loss"] - fp32["loss"]) / abs(fp32["loss"])
    assert rel <= 2e-3, rel


def test_configs1_bf16_gradients_vs_one_pass(data, bf16):
    one = _step("bf16", *data, "headline_bf16_1p", one_pass=True)
    np.testing.assert_array_equal(one["loss_b"], bf16["loss_b"])
    _grad_gate(bf16["grad"], one["grad"])


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_headline_step_deterministic(data, fp32, bf16, precision):
    """Run to run at the bench's size: a second fresh model's step gives the
    same loss and gradient bits -- every weight-gradient partial is summed in
    a fixed order (grouped x3 / bf16 TN kernels with workspaces, the heads'
    output layers with one writer per element, the x-rows gradient's splits
    reduced in order; DESIGN.md §2 "Deterministic step")."""
    first = fp32 if precision == "fp32" else bf16
    again = _step(precision, *data, f"headline_{precision}_again")
    assert again["loss"] == first["loss"]
    for n, g in first["grad"].items():
        assert np.array_equal(np.ascontiguousarray(g).view(np.int32),
                              np.ascontiguousarray(again["grad"][n]).view(np.int32)), n

"""Pins the CPU oracle before it is trusted as the parity reference.

Reference has no tests / golden vectors, so the oracle is pinned
by (1) known-answer properties of the reference STN, (2) the
accuracy of the elementary-function spec against libm, and (3) agreement with
an independent float64 torch restatement on every non-fragile quantity.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import air_oracle as ao
from oracle import air_torch as at


def _ulp_err(got, ref):
    got = got.astype(np.float32)
    ref64 = ref.astype(np.float64)
    ulp = np.spacing(np.abs(ref64.astype(np.float32))).astype(np.float64)
    return np.abs(got.astype(np.float64) - ref64) / np.maximum(ulp, 1e-45)


@pytest.mark.parametrize("fn,lo,hi,ref,tol", [
    (0, -87.0, 88.0, np.exp, 2.0),
    (1, 1e-30, 1e30, np.log, 2.0),
    (2, -10.0, 10.0, np.expm1, 3.0),
    (3, -10.0, 10.0, np.tanh, 3.0),
    (4, -30.0, 30.0, lambda x: 1.0 / (1.0 + np.exp(-x)), 3.0),
    (6, 0.0, 1.0, np.log1p, 3.0),
])
def test_math_spec_vs_libm(fn, lo, hi, ref, tol):
    lib = ao._load()
    rng = np.random.default_rng(fn)
    if fn == 1:
        x = np.exp(rng.uniform(np.log(lo), np.log(hi), 20000)).astype(np.float32)
    else:
        x = rng.uniform(lo, hi, 20000).astype(np.float32)
    x = np.concatenate([x, np.linspace(-0.5, 0.5, 1001, dtype=np.float32)])
    if fn == 1:
        x = np.abs(x) + np.float32(1e-6)
    y = np.zeros_like(x)
    lib.oracle_math_vec(fn, x.ctypes.data_as(ao._FP), y.ctypes.data_as(ao._FP),
                        ctypes.c_int(x.size))
    r = ref(x.astype(np.float64))
    assert np.max(_ulp_err(y, r)) <= tol


def test_softplus_thresholds():
    lib = ao._load()
    x = np.array([-20, -13.95, -13.94, 0.0, 13.94, 13.95, 20], np.float32)
    y = np.zeros_like(x)
    lib.oracle_math_vec(5, x.ctypes.data_as(ao._FP), y.ctypes.data_as(ao._FP), x.size)
    assert y[-1] == np.float32(20) and y[-2] == np.float32(13.95)
    # TF evaluates log(exp(x) + 1) in fp32 between the thresholds (cancellation
    # near the low threshold is part of the reference semantics)
    f = np.float32
    ex = np.exp(x).astype(f)
    tf_ref = np.where(x > f(13.9423847), x, np.where(x < f(-13.9423847), ex,
                                                     np.log((ex + f(1)).astype(f))))
    np.testing.assert_allclose(y, tf_ref, rtol=1e-6, atol=1e-7)


def test_stn_identity_reproduces_image():
    # theta = identity, equal in/out size: pixel (i,j) samples at (x,y) with
    # x = (xt+1)(W-1.001)/2 = j*(W-1.001)/(W-1): a 1.001 shrink.
    rng = np.random.default_rng(0)
    U = rng.uniform(size=(2, 28, 28)).astype(np.float32)
    th = np.tile(np.array([1, 0, 0, 0, 1, 0], np.float32), (2, 1))
    out = ao.stn(U, th, (28, 28))
    np.testing.assert_allclose(out, U, atol=2e-3)
    assert out[0, 0, 0] == U[0, 0, 0]


def test_stn_out_of_range_read_is_zero():
    # glimpse centred at (-1.3,-1.3) with s = 0.27 reads nothing
    rng = np.random.default_rng(1)
    U = rng.uniform(size=(1, 50, 50)).astype(np.float32)
    th = np.array([[0.27, 0, -1.3, 0, 0.27, -1.3]], np.float32)
    out = ao.stn(U, th, (28, 28))
    assert np.count_nonzero(out) == 0


@pytest.mark.parametrize("s,support", [(0.27, 196), (0.5, 576), (1.0, 2500)])
def test_stn_write_support(s, support):
    # write support = canvas pixels whose sample lands in 0 <= x < W-1 on both
    # axes; SURVEY §8c quotes ~floor(49 s + 1)^2 (196 at s=.27, 2500 at s=1;
    # exactly 24^2 at s=.5 since x_t=-0.5 is not on the 50-point grid).
    r = np.full((1, 28, 28), 0.5, np.float32)
    th = np.array([[1 / s, 0, 0, 0, 1 / s, 0]], np.float32)
    out = ao.stn(r, th, (50, 50))
    xt = np.float32(-1) + np.float32(2 / 49) * np.arange(50, dtype=np.float32)
    xt[-1] = 1
    x = ((np.float32(1 / s) * xt + 1) * np.float32(27 - 0.001)) / 2
    n_in = int(np.count_nonzero((x >= 0) & (x < 27)))
    assert n_in * n_in == support
    assert np.count_nonzero(np.abs(out) > 1e-6) == support


def test_stn_matches_torch_fp32_bitwise():
    rng = np.random.default_rng(2)
    U = rng.uniform(size=(4, 50, 50)).astype(np.float32)
    s = rng.uniform(0.2, 0.9, 4).astype(np.float32)
    t = rng.uniform(-0.8, 0.8, (4, 2)).astype(np.float32)
    th = np.stack([s, 0 * s, t[:, 0], 0 * s, s, t[:, 1]], 1).astype(np.float32)
    a = ao.stn(U, th, (28, 28))
    b = at.transformer(torch.from_numpy(U), torch.from_numpy(th), (28, 28)).numpy()
    np.testing.assert_array_equal(a, b)


def _setup(batch=8, seed=0, train=True, T=3, num_prior=None, bias_scale=0.05):
    cfg = ao.AirConfig(batch=batch, max_steps=T, train=train, num_prior=num_prior)
    P = ao.init_params(cfg, seed=100 + seed, bias_scale=bias_scale)
    nz = ao.make_noise(cfg, seed=200 + seed)
    x, k = ao.synthetic_canvases(batch, seed=300 + seed)
    return cfg, P, nz, x, k


@pytest.mark.parametrize("train", [True, False])
def test_c_oracle_vs_torch_float64(train):
    cfg, P, nz, x, k = _setup(train=train)
    prior = float(ao.annealed_log_odds(0))
    ro = ao.forward(cfg, P, nz, x, k, z_pres_prior_log_odds=prior)
    rt = at.air_forward(cfg, at.to_torch(P), at.to_torch(nz), torch.tensor(x, dtype=torch.float64),
                        torch.tensor(k), z_pres_prior_log_odds=prior)
    assert ro["T"] == rt["T"]
    np.testing.assert_array_equal(ro["digits"], rt["digits"].numpy())
    for key in ("scale", "shift", "z_pres_prob", "z_pres", "latent", "window"):
        np.testing.assert_allclose(ro[key], rt[key].detach().numpy().reshape(ro[key].shape),
                                   rtol=2e-4, atol=2e-5, err_msg=key)
    for key in ("z_pres_kl", "scale_kl", "shift_kl", "vae_kl"):
        np.testing.assert_allclose(ro[key], rt[key].numpy(), rtol=1e-4, atol=1e-4,
                                   err_msg=key)
    np.testing.assert_allclose(ro["canvas"], rt["canvas"].detach().numpy(), atol=2e-5)
    np.testing.assert_allclose(ro["running_loss"], rt["running_loss"].detach().numpy(),
                               rtol=1e-4)


def test_c_oracle_num_prior_and_fixed_steps():
    cfg, P, nz, x, k = _setup(num_prior=(1, 3), T=4)
    ro = ao.forward(cfg, P, nz, x, k, z_pres_prior_log_odds=-0.01)
    rt = at.air_forward(cfg, at.to_torch(P), at.to_torch(nz),
                        torch.tensor(x, dtype=torch.float64), z_pres_prior_log_odds=-0.01,
                        fixed_steps=True)
    np.testing.assert_array_equal(ro["digits"], rt["digits"].numpy())
    np.testing.assert_allclose(ro["running_loss"], rt["running_loss"].detach().numpy(),
                               rtol=1e-4)


def test_annealing_schedule():
    assert abs(float(ao.annealed_log_odds(0)) - np.log(1e4)) < 1e-5
    assert abs(float(ao.annealed_log_odds(3000)) - np.log(1e3)) < 1e-4
    assert abs(float(ao.annealed_log_odds(10 ** 6)) - np.log(2e-9)) < 1e-4


def test_marginal_objective_matches_reference_rule():
    # hand-evaluated air_model.py:86-107 for num_prior=[1,3], max_steps=4:
    # objective [1, .5, 1, 0] -> [100, logit(.5)=0, 100, -100]
    mo = ao.marginal_objective((1, 3), 4)
    np.testing.assert_array_equal(mo, np.array([100, 0, 100, -100], np.float32))

"""Pins the AIR-ASR oracle (oracle/asr_ref.c) before it is trusted: agreement
with the independent float64 torch restatement (oracle/asr_torch.py) on every
non-fragile quantity — executed steps, counts, scales / shifts, per-type KL
sums, the regularisers (entropy, area, bbox out / size / overlap, margin,
element-wise number loss) — for the learned z_pres prior and fix_steps, train
and test models.  The reference ships no ASR fixtures (parity with TF-1.12
unpinned)."""
import numpy as np
import pytest
import torch

from oracle import asr_oracle as so
from oracle import asr_torch as st


def _cfg(**kw):
    base = dict(batch=6, max_steps=4, constrains_num=(1, 3), constrains_num_gamma=0.5,
                constrains_margin_gamma=100.0, constrains_num_element_gamma=10.0,
                constrains_bbox_gamma=1.0, constrains_sharesize_gamma=0.3,
                constrains_area_gamma=0.2, constrains_area_minmax=(17.0, 23.0))
    base.update(kw)
    return so.AsrConfig(**base)


@pytest.mark.parametrize("kw", [dict(), dict(train=False), dict(fix_steps=2),
                                dict(z_pres_temperature=1.0, stopping_threshold=0.99)])
def test_c_oracle_matches_torch_restatement(kw):
    cfg = _cfg(**kw)
    P = so.init_params(cfg, seed=3, bias_scale=0.05)
    nz = so.make_noise(cfg, seed=4)
    from oracle import air_oracle as ao
    x, k = ao.synthetic_canvases(cfg.batch, seed=5)
    ref = so.forward(cfg, P, nz, x, k)
    Pt = {n: torch.tensor(v, dtype=torch.float64) for n, v in P.items()}
    out = st.asr_forward(cfg, Pt, nz, torch.tensor(x, dtype=torch.float64))
    T = ref["T"]
    assert out["T"] == T
    np.testing.assert_array_equal(out["digits"].numpy(), ref["digits"])
    np.testing.assert_allclose(out["scale"].numpy(), ref["scale"].T, rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(out["shift"].numpy(), ref["shift"].transpose(1, 0, 2),
                               rtol=2e-5, atol=1e-6)
    np.testing.assert_allclose(out["z_pres_prob"].numpy(), ref["z_pres_prob"].T, rtol=2e-5,
                               atol=1e-6)
    kl = (ref["z_pres_kl"].sum(0) + ref["scale_kl"].sum(0) + ref["shift_kl"].sum(0) +
          ref["vae_kl"].sum(0))
    np.testing.assert_allclose(out["kl"].detach().numpy(), kl, rtol=2e-4, atol=2e-3)
    for key in ("area", "out", "size", "overlap", "element"):
        np.testing.assert_allclose(out[key].detach().numpy(), ref[key], rtol=1e-4, atol=2e-3,
                                   err_msg=key)
    np.testing.assert_allclose(out["pr"].detach().numpy(), ref["pr_loss"], rtol=1e-4, atol=2e-3)
    assert float(out["margin"]) == pytest.approx(ref["margin"], rel=1e-4, abs=1e-3)


def test_c_oracle_known_answers():
    # fix_steps: the prior forces exactly fix_steps objects in the test model
    # when the posterior agrees; area loss is constant (amax - amin) for scales
    # inside the range; the bbox losses vanish for a single step
    cfg = _cfg(max_steps=1, train=False, constrains_margin_gamma=0.0)
    P = so.init_params(cfg, seed=8, bias_scale=0.05)
    nz = so.make_noise(cfg, seed=9)
    from oracle import air_oracle as ao
    x, k = ao.synthetic_canvases(cfg.batch, seed=10)
    ref = so.forward(cfg, P, nz, x, k)
    assert ref["T"] == 1
    np.testing.assert_array_equal(ref["size"], 0.0)
    np.testing.assert_array_equal(ref["overlap"], 0.0)
    np.testing.assert_array_equal(ref["element"], 0.0)
    assert ref["margin"] == 0.0
    sc = ref["scale"][0] * 50
    inside = (sc >= 17) & (sc <= 23)
    np.testing.assert_allclose(ref["area"][inside], 6.0, rtol=1e-6)

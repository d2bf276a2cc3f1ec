"""Generation loop (air_model.py:1001-1146, vae.py:51-86):
the C oracle's known-answer properties on CPU, and the HIP path
(AIRModel.generate: mog_generation_prior + fp32 decoder GEMMs + STN write
accumulate) bit-exact against the oracle on injected prior noise."""
import numpy as np
import pytest
import torch

from oracle import air_oracle as ao


def _noise(T, G, seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    return {"eps_scale": rng.standard_normal((T, G)).astype(f),
            "eps_shift": rng.standard_normal((T, G, 2)).astype(f),
            "eps_z": rng.standard_normal((T, G, 50)).astype(f),
            "eps_x": rng.standard_normal((T, G, 784)).astype(f)}


def test_oracle_generation_known_answers():
    cfg = ao.AirConfig(batch=3, scale_prior_variance=0.05)
    P = ao.init_params(cfg, seed=5, bias_scale=0.05)
    out0 = ao.generate(cfg, P, _noise(0, 3, 1), 3, 0)
    assert not out0["canvas"].any()
    nz = _noise(2, 3, 2)
    out = ao.generate(cfg, P, nz, 3, 2)
    assert np.all(out["digits"] == 2)
    s = 1.0 / out["st_back"][..., 0]
    ref_s = 1.0 / (1.0 + np.exp(-(-1.0 + nz["eps_scale"] * np.sqrt(0.05))))
    np.testing.assert_allclose(s, ref_s, rtol=1e-5)
    # one step: the canvas equals that step's written window; pixels whose
    # clipped corners coincide on both axes are exactly zero
    one = ao.generate(cfg, P, {k: v[:1] for k, v in nz.items()}, 3, 1)
    # (the half-degenerate border samples keep the reference's ~1e-6 cancellation residue)
    assert one["canvas"].min() >= -1e-5 and one["canvas"].max() <= 1 + 1e-5
    assert (one["canvas"] == 0).sum() > 0 and (one["canvas"] > 0).sum() > 0
    # additivity: two steps = step 0 + step 1 (fp32 add of the two windows)
    two = out["canvas"]
    first = one["canvas"]
    second = ao.generate(cfg, P, {k: v[1:] for k, v in nz.items()}, 3, 1)["canvas"]
    np.testing.assert_array_equal(two, (first + second).astype(np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("T,G", [(1, 5), (3, 64), (4, 17)])
def test_hip_generation_matches_oracle(T, G):
    from mog_air.air_model import AIRModel
    cfg = ao.AirConfig(batch=G, scale_prior_variance=0.05)
    P = ao.init_params(cfg, seed=7 + T, bias_scale=0.05)
    nz = _noise(T, G, 10 + T)
    ref = ao.generate(cfg, P, nz, G, T)
    m = AIRModel(max_steps=6, scale_prior_variance=0.05, cnn=False, train=False,
                 scope=f"gen{T}_{G}", device="cuda:0", generation_batch_size=G)
    m.params.load_dict(P)
    out = m.generate(T, noise={k: torch.as_tensor(v).cuda() for k, v in nz.items()})
    assert tuple(out.shape) == (G, 50, 50, 1)
    np.testing.assert_array_equal(out.reshape(G, -1).cpu().numpy(), ref["canvas"])
    np.testing.assert_array_equal(m.generated_st_back.cpu().numpy(),
                                  ref["st_back"].transpose(1, 0, 2).reshape(G, T, 2, 3))
    assert np.all(m.generated_num_digits.cpu().numpy() == T)


@pytest.mark.gpu
def test_hip_generation_device_noise_runs():
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=3, cnn=False, train=False, scope="gen_dev", device="cuda:0",
                 precision="bf16")
    out = m.generate(2)
    v = out.cpu().numpy()
    assert v.shape == (64, 50, 50, 1) and np.isfinite(v).all() and v.max() > 0

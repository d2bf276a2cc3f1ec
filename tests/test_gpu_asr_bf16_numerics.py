"""SURVEY.md §8 D.5 for AIR-ASR: what the bf16 glimpse-VAE configuration
does to the inferred counts and the ELBO, on the configurations the bench
times -- configs[2] (train_air_pr.py -dn 13 -gm 100 -gne 10: learned z_pres
prior, number regularisers) and configs[4] (-dn 3 -ds bbox20k -gb 1 -gs 10
-ga 20: fix_steps 3, bbox / size / area regularisers), bench.make_asr_model's
hyper-parameters, B = 256, train-mode forward, the SAME weights, canvases and
injected noise in fp32 (bit-exact with the C oracle, tests/test_gpu_asr.py)
and bf16.

Unlike AIR, the ASR loop feeds step t's latent z (a VAE output, bf16 in this
configuration) into step t+1's LSTM inputs and heads
(air_number_bbox_location.py:413-422), so bf16 rounding reaches the z_pres
logits of later steps and can flip a count (rec_num_digits,
air_number_bbox_location.py:715) where the fp32 decision was close.  Recorded
(``MOG_NUMERICS_OUT``, default gpurun_out/r06_asr_bf16_numerics.json; the
committed copy is profiles/r06_asr_bf16_numerics.json): the count mismatch
rate, the executed-step agreement, |dLoss| / |Loss| of the batch training
loss (the negative ELBO plus the regulariser terms,
air_number_bbox_location.py:930-968), the same over the images whose counts
agree, and for every flipped image the fp32 / bf16 z_pres probabilities at its first
differing step.

Gates (measured on MI355X, profiles/r06_asr_bf16_numerics.json: 0 of 256
counts differ in either configuration, |dLoss| / |Loss| 1.1e-4 and 3.8e-5,
z_pres probabilities within 2.8e-4): count mismatch rate <= 2 %, the same
executed steps, |dLoss| / |Loss| <= 1e-3 (SURVEY §8 D.5's ELBO bar); z_pres
probabilities of step 0 (before any VAE output reaches the loop)
bit-identical."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda:0")
B = 256
RESULTS = {}


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    yield
    out = os.environ.get("MOG_NUMERICS_OUT", os.path.join("gpurun_out",
                                                            "r06_asr_bf16_numerics.json"))
    if RESULTS:
        os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
        with open(out, "w") as f:
            json.dump(RESULTS, f, indent=1)


def _noise(T, Bn, seed):
    rng = np.random.default_rng(seed)
    f = np.float32
    return {"eps_scale": rng.standard_normal((T, Bn)).astype(f),
            "eps_shift": rng.standard_normal((T, Bn, 2)).astype(f),
            "eps_z": rng.standard_normal((T, Bn, 50)).astype(f),
            "eps_x": rng.standard_normal((T, Bn, 784)).astype(f),
            "u": rng.uniform(0.0, 1.0, (T, Bn)).astype(f)}


def _forward(precision, name, cfg, data, x, k, nz):
    import bench
    m = bench.make_asr_model(precision, DEV, f"num_{name}_{precision}", cfg=cfg)
    m.infer(x, k, noise={n: torch.as_tensor(v).to(DEV) for n, v in nz.items()})
    out = {"T": m.executed_steps, "digits": m.rec_num_digits.cpu().numpy().copy(),
           "loss": m.loss, "loss_b": m.per_image_loss.cpu().numpy().copy(),
           "zprob": m._ws.zprob.cpu().numpy().copy()}
    return out


@pytest.mark.parametrize("name", ["configs_2_asr", "configs_4_asr_bbox"])
def test_asr_bf16_counts_and_elbo(name):
    import bench
    cfg = bench.ASR_BBOX if name == "configs_4_asr_bbox" else None
    data = bench.ASR_BBOX_DATA if cfg is not None else {}
    x, k = bench.synthetic(B, 777, **data)
    nz = _noise(6, B, 778)
    f32 = _forward("fp32", name, cfg, data, x, k, nz)
    b16 = _forward("bf16", name, cfg, data, x, k, nz)
    flips = np.nonzero(f32["digits"] != b16["digits"])[0]
    rate = float(len(flips)) / B
    rel = abs(b16["loss"] - f32["loss"]) / abs(f32["loss"])
    detail = []
    for i in flips:
        detail.append({"image": int(i), "count_fp32": int(f32["digits"][i]),
                       "count_bf16": int(b16["digits"][i]),
                       "zprob_fp32": [float(v) for v in f32["zprob"][:, i]],
                       "zprob_bf16": [float(v) for v in b16["zprob"][:, i]]})
    same = f32["digits"] == b16["digits"]
    dz = np.abs(f32["zprob"] - b16["zprob"])
    RESULTS[name] = {
        "batch": B, "max_steps": 6, "fix_steps": 3 if cfg is not None else None,
        "executed_steps_fp32": f32["T"], "executed_steps_bf16": b16["T"],
        "count_mismatch_rate": rate, "count_mismatches": int(len(flips)),
        "loss_fp32": f32["loss"], "loss_bf16": b16["loss"], "rel_loss_deviation": rel,
        "rel_loss_deviation_count_agreeing_images": float(
            abs(b16["loss_b"][same].mean() - f32["loss_b"][same].mean())
            / abs(f32["loss_b"][same].mean())),
        "zprob_abs_diff_per_step_mean": [float(v) for v in dz.mean(1)],
        "zprob_abs_diff_per_step_max": [float(v) for v in dz.max(1)],
        "flips": detail[:32]}
    assert f32["T"] == b16["T"]
    np.testing.assert_array_equal(f32["zprob"][0], b16["zprob"][0])
    assert rate <= 0.02, RESULTS[name]
    assert rel <= 1e-3, RESULTS[name]

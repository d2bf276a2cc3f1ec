"""Per-tensor 2-norm differences of the fp32 step's gradients between the
x3 forms and the fp32 chain, and chain against chain (the setting of
tests/test_gpu_x3.py::test_x3_fp32_step_gradients_match_chain); prints the
largest ratios ||a - b|| / ||b||."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mog_air.air_model import AIRModel  # noqa: E402

rng = np.random.default_rng(5)
x = (rng.uniform(size=(1024, 2500)) * (rng.uniform(size=(1024, 2500)) < 0.3)).astype(np.float32)
grads = []
for x3 in (1, 2, 0, 0, 0):
    m = AIRModel(max_steps=3, max_digits=3, canvas_size=50, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, cnn=False, train=True, scope="x3",
                 device="cuda:0", precision="fp32", seed=3, noise_seed=4)
    m.X_GRAD_X3 = x3
    m.VAE_WGRAD_X3 = m.VAE_DX_X3 = x3 != 0
    m.X3_DX_MIN_ROWS = 2048
    grads.append({k: torch.as_tensor(np.asarray(v), dtype=torch.float64)
                  for k, v in m.compute_gradients(x).items()})
for name, g in (("x3=1", grads[0]), ("x3=2", grads[1]), ("chain2", grads[3]), ("chain3", grads[4])):
    r = sorted((((g[k] - grads[2][k]).norm() / (grads[2][k].norm() + 1e-30)).item(), k)
               for k in g if g[k].numel() > 64)
    print(name, " ".join(f"{k.split('/')[-2]}/{k.split('/')[-1]}:{v:.1e}" for v, k in r[-4:]), flush=True)

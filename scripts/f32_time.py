"""fp32 fused step vs the unfused fp32 sequence at B rows (bench.fp32_step_roofline),
then one launch with MOG_VS_TIMING=1 (per-phase times of stn_vae_step_f32_kernel).
usage: python scripts/f32_time.py [B]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    dev = torch.device("cuda:0")
    out = bench.fp32_step_roofline(B, 20, dev)
    print(json.dumps(out), flush=True)
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=1, max_digits=1, canvas_size=50, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=True, scope="f32time", device=dev, precision="fp32")
    x, k = bench.synthetic(B, 4322, 50)
    X = torch.from_numpy(x).to(dev)
    m.infer(X, torch.from_numpy(k).to(dev))
    m._vae_forward_all(X, m._ws, 0.3)
    torch.cuda.synchronize()
    os.environ["MOG_VS_TIMING"] = "1"
    m._vae_forward_all(X, m._ws, 0.3)
    torch.cuda.synchronize()
    sys.stderr.flush()


if __name__ == "__main__":
    main()

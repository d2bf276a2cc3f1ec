"""Run the fused step kernel a few times at one batch (profiling target:
rocprofv3 --pmc / --kernel-trace).  usage: vs_once.py [B] [launches]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from mog_air.air_model import AIRModel  # noqa: E402
import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    m = AIRModel(max_steps=3, cnn=False, train=True, device="cuda:0", precision="bf16",
                 scope="vs1", scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                 seed=77, noise_seed=78)
    x, k = bench.synthetic(B, 4321)
    x = torch.as_tensor(x).to("cuda:0")
    k = torch.as_tensor(k).to("cuda:0")
    m.infer(x, k)
    torch.cuda.synchronize()
    for i in range(n):
        m._step_fused(x, m._ws, i % 3, 0.3)
    torch.cuda.synchronize()
    print("done", B, n)


if __name__ == "__main__":
    main()

"""The north-star fused bf16 step (bench.fused_step_roofline) at B = 65,536,
C = 50 and 64, 30 launches each, three times (A/B of kernel variants across
gpurun calls)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
for _ in range(3):
    for C in (50, 64):
        r = bench.fused_step_roofline(65536, 30, dev, canvas=C)
        print(f"C={C}: {r['avg_launch_us']:.1f} us frac {r['frac']:.3f}", flush=True)

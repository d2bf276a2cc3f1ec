"""Time the north-star fused step launch (bench.fused_step_roofline: 65,536
images, C = 50 / 64, training form) in the lockstep and the pipelined form;
MOG_VS_TIMING=1 adds the per-role phase breakdown on stderr."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", "65536"))
for canvas in (50, 64):
    for form in ("0", "1"):
        os.environ["MOG_VS_PIPE"] = form
        r = bench.fused_step_roofline(B, 20, dev, canvas=canvas)
        print(f"C={canvas} pipe={form}: {r['avg_launch_us']:.1f} us  frac {r['frac']:.3f}", flush=True)

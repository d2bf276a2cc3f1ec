"""A/B timing of the fused step kernels (bf16 north-star form at C = 50,
training and forward-only; the fp32 fused step) for the library MOG_AIR_LIB
points at (default: the in-tree build).  usage: python scripts/ab_fused.py TAG"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
tag = sys.argv[1] if len(sys.argv) > 1 else "in-tree"
for _ in range(2):
    a = bench.fused_step_roofline(65536, 30, dev)
    f = bench.fused_step_roofline(65536, 30, dev, save=False)
    p = bench.fp32_step_roofline(65536, 10, dev)
    print(f"{tag}: bf16 train {a['avg_launch_us']:.1f} us ({a['frac']:.3f}), fwd "
          f"{f['avg_launch_us']:.1f} us, fp32 {p['avg_chain_us']:.1f} us ({p['frac']:.3f})",
          flush=True)

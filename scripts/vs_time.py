"""Average duration of the fused step kernel at batch B over a few launches
(HIP events on the launch stream); MOG_VS_MT picks the tile variant.
usage: python scripts/vs_time.py B [C]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    B = int(sys.argv[1])
    C = int(sys.argv[2]) if len(sys.argv) > 2 else 50
    r = bench.fused_step_roofline(B, 20, torch.device("cuda:0"), canvas=C)
    print(f"MT={os.environ.get('MOG_VS_MT', 'auto')} B={B} C={C}: {r['avg_launch_us']:.1f} us "
          f"frac {r['frac']:.3f}", flush=True)


if __name__ == "__main__":
    main()

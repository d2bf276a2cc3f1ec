"""Fused step kernel at B = 65,536 (the north-star roofline shape): lockstep
vs pipelined form, training and forward-only, C = 50 and 64 (HIP events on
the launch stream, bench.fused_step_roofline), then one MOG_VS_TIMING launch of
the pipelined form (per-tile role spans).
usage: python scripts/vs_pipe_time.py [B]"""
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
    for pipe in ("0", "1"):
        os.environ["MOG_VS_PIPE"] = pipe
        for C, save in ((50, True), (50, False), (64, True)):
            r = bench.fused_step_roofline(B, 20, dev, canvas=C, save=save)
            print(f"pipe={pipe} B={B} C={C} save={save}: {r['avg_launch_us']:.1f} us "
                  f"frac {r['frac']:.3f}", flush=True)
    os.environ["MOG_VS_PIPE"] = "1"
    os.environ["MOG_VS_TIMING"] = "1"
    bench.fused_step_roofline(B, 2, dev, canvas=50, save=True)


if __name__ == "__main__":
    main()

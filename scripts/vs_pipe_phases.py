"""Pipelined fused-step kernel with roles masked out (MOG_VS_PHASES: 1 = STN
read by the samplers, 8 = STN write): per-tile role spans at B = 65,536 for
all / no-read / no-write / neither (profiling aid; outputs not meaningful).
usage: python scripts/vs_pipe_phases.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    os.environ["MOG_VS_PIPE"] = "1"
    for ph in ("31", "30", "23", "22"):
        os.environ["MOG_VS_PHASES"] = ph
        os.environ.pop("MOG_VS_TIMING", None)
        r = bench.fused_step_roofline(65536, 10, dev, canvas=50, save=True)
        print(f"phases={ph}: {r['avg_launch_us']:.1f} us", flush=True)
        os.environ["MOG_VS_TIMING"] = "1"
        bench.fused_step_roofline(65536, 1, dev, canvas=50, save=True)
        sys.stderr.flush()


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def prio_sweep():
    """MOG_VS_PRIO (hex: M W S nibbles) variants of the full kernel."""
    dev = torch.device("cuda:0")
    os.environ["MOG_VS_PIPE"] = "1"
    os.environ["MOG_VS_PHASES"] = "31"
    os.environ.pop("MOG_VS_TIMING", None)
    for pr in ("000", "021", "012", "011", "022", "100", "120", "210"):
        os.environ["MOG_VS_PRIO"] = pr
        r = bench.fused_step_roofline(65536, 10, dev, canvas=50, save=True)
        print(f"prio={pr}: {r['avg_launch_us']:.1f} us", flush=True)
    os.environ["MOG_VS_PRIO"] = "000"


if __name__ == "__main__" and len(sys.argv) > 1:
    prio_sweep()

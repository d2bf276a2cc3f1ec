"""Kernel-trace target: N train steps of the configs[2] ASR model (bench.make_asr_model)
at batch B.  usage: asr_steps.py [precision] [B] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp32"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dev = torch.device("cuda:0")
    el, m = bench.timed_train(prec, B, n, 2, dev, model=bench.make_asr_model(prec, dev, "asrtr"))
    print(f"ASR {prec} B={B}: {el / n * 1e3:.3f} ms/step, executed steps {m.executed_steps}")

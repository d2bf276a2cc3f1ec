"""Profiling target: AIR-ASR configs[2] train steps at B rows (fp32)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
prec = sys.argv[2] if len(sys.argv) > 2 else "fp32"
dev = torch.device("cuda:0")
el, m = bench.timed_train(prec, B, 4, 2, dev, model=bench.make_asr_model(prec, dev, "asrtr"))
print(f"ASR {prec} B={B}: {el / 4 * 1e3:.3f} ms/step", flush=True)

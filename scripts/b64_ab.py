"""A/B of a model class switch on the captured batch-64 AIR step (the bench's
config_1_batch64_fp32 workload): alternating rounds, ms per step.
usage: python scripts/b64_ab.py ATTR[=v1,v2] [rounds] [steps] [B] [asr]  (default values True,False)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

attr, _, vs = sys.argv[1].partition("=")
VALS = [int(v) for v in vs.split(",")] if vs else [True, False]
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 200
B = int(sys.argv[4]) if len(sys.argv) > 4 else 64
ASR = sys.argv[5:6] == ["asr"]  # configs[2]'s AIR-ASR step instead of AIR's
dev = torch.device("cuda:0")
models = {}
for v in VALS:
    m = (bench.make_asr_model("fp32", dev, f"ab{int(v)}") if ASR
         else bench.make_model("fp32", dev, 1, 0, f"ab{int(v)}"))
    setattr(m, attr, v)
    models[v] = m
res = {v: [] for v in VALS}
for r in range(rounds):
    for v in VALS:
        el, _ = bench.timed_train("fp32", B, steps, 20, dev, model=models[v], graph=B <= 512)
        res[v].append(el / steps * 1e3)
        print(f"{attr}={v}: {res[v][-1]:.4f} ms/step", flush=True)
for v in VALS:
    print(f"{attr}={v}: min {min(res[v]):.4f} median {sorted(res[v])[len(res[v]) // 2]:.4f}")

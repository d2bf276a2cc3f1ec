"""A/B of AIR-ASR class flags on the bench's configs[2] step (one process):
python3 scripts/ab_asr.py [fp32|bf16] FLAG=v,FLAG=v ... (each set timed twice, alternating)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mog_air.asr_model import AIRModel  # noqa: E402

dev = torch.device("cuda:0")
prec = sys.argv[1]
sets = [dict(kv.split("=") for kv in a.split(",")) if a != "-" else {} for a in sys.argv[2:]]
base = {k: getattr(AIRModel, k) for s in sets for k in s}
for rep in range(2):
    for s in sets:
        for k, v in base.items():
            setattr(AIRModel, k, v)
        for k, v in s.items():
            setattr(AIRModel, k, type(base[k])(int(v)))
        el, m = bench.timed_train(prec, 8192, 10, 3, dev,
                                  model=bench.make_asr_model(prec, dev, "abasr"))
        print(rep, s or "defaults", f"ASR {prec} {el / 10 * 1e3:.3f} ms", flush=True)
        del m

"""A/B of AIRModel class flags on the bench's sub-workloads (one process):
python3 scripts/ab_flags.py FLAG=v,FLAG=v ... ; times configs[1] bf16, configs[3]
dSprites bf16 and the fp32 headline with each flag set, alternating twice."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from mog_air.air_model import AIRModel  # noqa: E402

dev = "cuda:0"
sets = [dict(kv.split("=") for kv in a.split(",")) if a != "-" else {} for a in sys.argv[1:]]
base = {k: getattr(AIRModel, k) for s in sets for k in s}
loads = [("fp32", 50, None), ("bf16", 50, None), ("bf16", 64, dict(counts=(2, 3, 4)))]
for rep in range(2):
    for s in sets:
        for k, v in base.items():
            setattr(AIRModel, k, v)
        for k, v in s.items():
            setattr(AIRModel, k, type(base[k])(int(v)) if not isinstance(base[k], str) else v)
        res = []
        for prec, canvas, data in loads:
            el, m = bench.timed_train(prec, 8192, 10, 3, dev, scope="ab", canvas=canvas, data=data)
            res.append(f"{prec} C{canvas} {el / 10 * 1e3:.3f}")
            del m
            if os.environ.get("MOG_AB_EMPTY") == "1":
                torch.cuda.empty_cache()
        print(rep, s or "defaults", "; ".join(res), flush=True)

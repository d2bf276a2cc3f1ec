"""Profiling target: captured train steps at the reference's batch of 64."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda:0")
# (second argument "asr": configs[2]'s AIR-ASR step instead of AIR's)
model = bench.make_asr_model("fp32", dev, "b64asr") if sys.argv[2:3] == ["asr"] else None
el, m = bench.timed_train("fp32", B, 10, 5, dev, scope="b64g", graph=True, model=model)
print(f"B={B} graph: {el / 10 * 1e3:.3f} ms/step", flush=True)

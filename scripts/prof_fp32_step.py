"""Kernel-trace target: the fp32 step chain of bench.fp32_step_roofline."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    print(json.dumps(bench.fp32_step_roofline(n, 10, torch.device("cuda:0"))))

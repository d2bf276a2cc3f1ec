"""mog_copy_f4 bandwidth (GB/s of bytes read + written) and torch's copy_."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
print(os.environ.get("MOG_COPY_VARIANT", "0"), "mog_copy_f4 %.0f GB/s" % bench.copy_bandwidth(dev, 1.0),
      flush=True)
if os.environ.get("MOG_COPY_VARIANT", "0") == "0":
    n = (1 << 30) // 4
    a, b = torch.ones(n, device=dev), torch.empty(n, device=dev)
    for _ in range(3):
        b.copy_(a)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    print("torch copy_ %.0f GB/s" % (2.0 * n * 4 * 20 / (e0.elapsed_time(e1) * 1e-3) / 1e9), flush=True)

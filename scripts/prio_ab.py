"""A/B of the main stream's priority: the headline fp32 train step (and the
bf16 one) at B = 8192, run from torch's default-priority stream vs from a
high-priority stream (the model forks its side streams from the current
stream, so the side streams' kernels then yield CUs to the main chain's),
alternating arms, median ms per step over rounds."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda:0")
B = int(os.environ.get("B", "8192"))
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
print("priority range", torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else None, flush=True)
for prec in ("fp32", "bf16"):
    m = bench.make_model(prec, dev, 1, 0, "prio_" + prec)
    x, k = bench.synthetic(B, 1234)
    X, K = torch.from_numpy(x).to(dev), torch.from_numpy(k).to(dev)
    high = torch.cuda.Stream(device=dev, priority=-1)
    res = {"default": [], "high": []}
    for _ in range(3):
        m.train_step_async(X, K)
    torch.cuda.synchronize()
    for rnd in range(6):
        for arm in ("default", "high"):
            s = high if arm == "high" else torch.cuda.current_stream(dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                m.train_step_async(X, K)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(10):
                    m.train_step_async(X, K)
                torch.cuda.synchronize()
                res[arm].append((time.perf_counter() - t0) / 10 * 1e3)
    print(prec, {a: round(statistics.median(v), 4) for a, v in res.items()},
          {a: [round(t, 3) for t in v] for a, v in res.items()}, flush=True)

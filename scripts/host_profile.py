"""Host-side (Python) cost of one train step at a launch-bound batch: cProfile
over N steps of the fp32 headline model (default B = 64, the reference's
batch), sorted by own time.  usage: host_profile.py [B] [steps]"""
import cProfile
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda:0")
    m = bench.make_model("fp32", dev, 1, 0, "hostprof")
    x, k = bench.synthetic(B, 1234)
    X = torch.as_tensor(x).to(dev)
    K = torch.as_tensor(k).to(dev)
    for _ in range(5):
        m.train_step_async(X, K, global_batch=B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        m.train_step_async(X, K, global_batch=B)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"B={B}: host issue {(t1 - t0) / n * 1e3:.3f} ms/step, wall {(t2 - t0) / n * 1e3:.3f} ms/step")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        m.train_step_async(X, K, global_batch=B)
    pr.disable()
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()

"""Per-node cost of a captured hipGraph of dependent tiny kernels on one
stream (the floor under the batch-64 step's ~75 launches)."""
import time

import torch

dev = "cuda:0"
x = torch.zeros(64, device=dev)
big = torch.zeros(64 * 1024, device=dev)
for n, t in ((100, x), (100, big)):
    g = torch.cuda.CUDAGraph()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(n):
            t.add_(1.0)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    b = time.perf_counter()
    print(f"graph of {n} add_ on {t.numel()} floats: {(b - a) / 20 / n * 1e6:.2f} us per node",
          flush=True)
    a = time.perf_counter()
    for _ in range(20):
        for _ in range(n):
            t.add_(1.0)
    torch.cuda.synchronize()
    b = time.perf_counter()
    print(f"eager: {(b - a) / 20 / n * 1e6:.2f} us per launch", flush=True)

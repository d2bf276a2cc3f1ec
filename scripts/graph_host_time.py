"""Host cost of the captured train step at the reference's batch of 64: issue
time per step of each part of AIRModel._train_step_graphed (noise fills, prior
fill, graph replay, Adam) against the wall time per step."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
n = 50
dev = torch.device("cuda:0")
m = bench.make_model("fp32", dev, 1, 0, "ght")
x, k = bench.synthetic(B, 1234)
X, K = torch.as_tensor(x).to(dev), torch.as_tensor(k).to(dev)
for _ in range(5):
    m.train_step_graphed(X, K)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(n):
    m.train_step_graphed(X, K)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"B={B}: host issue {(t1 - t0) / n * 1e3:.3f} ms/step, wall {(t2 - t0) / n * 1e3:.3f} ms/step")
ws = m._graph_ws
parts = {"noise": lambda: m._fill_noise(ws, None),
         "prior": lambda: m._prior_dev.fill_(m.hyper("z_pres_prior_log_odds")),
         "replay": lambda: m._graph.replay(),
         "adam": lambda: m.params.apply_adam(m.hyper("learning_rate"), m.gradient_clipping_norm)}
for name, fn in parts.items():
    torch.cuda.synchronize()
    a = time.perf_counter()
    for _ in range(n):
        fn()
    b = time.perf_counter()
    torch.cuda.synchronize()
    c = time.perf_counter()
    print(f"  {name}: issue {(b - a) / n * 1e3:.3f} ms, wall {(c - a) / n * 1e3:.3f} ms", flush=True)

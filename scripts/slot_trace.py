"""Two identical fp32 headline models timed back to back in one process (the
second is often ~10 % slower): the profiling target of scripts/gpu_slot_trace.sh."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 2):
    el, m = bench.timed_train("fp32", 8192, 10, 5, torch.device("cuda:0"), scope="slot")
    print(f"model {i}: {el / 10 * 1e3:.3f} ms/step", flush=True)
    ws = m._ws
    big = sorted(((t.numel() * t.element_size(), n, t.data_ptr()) for n, t in vars(ws).items()
                  if isinstance(t, torch.Tensor) and t.is_cuda), reverse=True)[:12]
    print("  ", " ".join(f"{n}:{p % (2 << 20):#x}" for _, n, p in big), flush=True)
    del m

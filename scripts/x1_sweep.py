"""bf16 x-rows gradient X^T dGsum [2500 x 1024, K = 8192] on gemm_x3p_tn's
one-piece form: launch time by split-K (HIP events)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

B, M, N = 8192, 2500, 1024
Mp = 2504
dev = "cuda:0"
Xb = (torch.randn(B, Mp, device=dev) * 0.1).to(torch.bfloat16)
G = (torch.randn(B, N, device=dev) * 0.1).to(torch.bfloat16)
C = torch.zeros(M, N, device=dev)
cs = torch.zeros(N, device=dev)
for sk in (1, 2, 3, 4, 6, 8, 16):
    def go():
        ops.gemm_x3p_tn(Xb.view(-1), 0, G, 0, C, M, N, B, Mp, N, N, splitk=sk, colsum=cs, npieces=1)
    for _ in range(3):
        go()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        go()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 20 * 1e3
    print(f"splitk {sk:2d}: {us:7.1f} us  {2.0 * B * M * N / us / 1e6:7.1f} TF", flush=True)

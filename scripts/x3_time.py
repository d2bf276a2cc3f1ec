"""Stand-alone timing of the x-part weight gradient at the bench shape
(X^T dG: M = 2500, N = 1024, K = 8192): x3 GEMM at split-K 4/8/16 against the
fp32 MFMA split-K GEMM, HIP events, 20 launches each."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mog-asr_amd"))
from mog_air import ops  # noqa: E402

dev = "cuda:0"
M, N, K = 2500, 1024, 8192
X = torch.rand(K, M, device=dev)
G = torch.randn(K, N, device=dev)
C = torch.zeros(M, N, device=dev)
cs = torch.zeros(N, device=dev)


def t(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1000


fl = 2.0 * M * N * K
for sk in (4, 8, 16):
    us = t(lambda: ops.gemm_x3_tn(X, G, C, M, N, K, M, N, N, splitk=sk, colsum=cs))
    print(f"x3 stages={os.environ.get('MOG_X3_STAGES', '1')} splitk={sk}: {us:.1f} us "
          f"({fl / us / 1e6:.0f} TF/s fp32-equivalent)")
X3 = torch.empty(3, K, 2504, device=dev, dtype=torch.bfloat16)
G3 = torch.empty(3, K, N, device=dev, dtype=torch.bfloat16)
us = t(lambda: ops.split3_bf16(X, X3, K, M, M, 2504, K * 2504))
print(f"split X: {us:.1f} us")
us = t(lambda: ops.split3_bf16(G, G3, K, N, N, N, K * N))
print(f"split dG: {us:.1f} us")
for sk in (4, 8, 16):
    us = t(lambda: ops.gemm_x3p_tn(X3, K * 2504, G3, K * N, C, M, N, K, 2504, N, N, splitk=sk,
                                   colsum=cs))
    print(f"x3 pre-split splitk={sk}: {us:.1f} us ({fl / us / 1e6:.0f} TF/s fp32-equivalent)")
us = t(lambda: ops.gemm([X], [G], [C], M, N, K, M, N, N, transA=True, epi=ops.EPI_ATOMIC,
                        splitk=4, colsum=[cs]))
print(f"fp32 chain splitk=4: {us:.1f} us ({fl / us / 1e6:.0f} TF/s)")

"""x-rows gradient X^T dGsum [2500 x 1024, K = 8192] on gemm_x3p_tn: launch
time by split-K (HIP events) for the one-piece (bf16 configuration) and the
three-piece (fp32) forms, with a correctness check against an fp64 matmul
of the same operands.  The kernel variant is MOG_X3P_VAR (read once per
process: run one process per variant, scripts/gpu_x1_sweep.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

B, M, N = 8192, 2500, 1024
Mp = 2504
dev = "cuda:0"
var = os.environ.get("MOG_X3P_VAR", "0")
torch.manual_seed(0)
X = torch.rand(B, Mp, device=dev) * (torch.rand(B, Mp, device=dev) > 0.6)
X[:, M:] = 0
G = torch.randn(B, N, device=dev) * 0.01
X3 = torch.empty(3, B, Mp, device=dev, dtype=torch.bfloat16)
G3 = torch.empty(3, B, N, device=dev, dtype=torch.bfloat16)
ops.split3_bf16(X, X3, B, Mp, Mp, Mp, B * Mp)
ops.split3_bf16(G, G3, B, N, N, N, B * N)
Xb, Gb = X.to(torch.bfloat16), G.to(torch.bfloat16)
C = torch.zeros(M, N, device=dev)
cs = torch.zeros(N, device=dev)
ref1 = Xb[:, :M].double().t() @ Gb.double()
ref3 = X[:, :M].double().t() @ G.double()
for npieces, sk, red in [(p, k, r) for p in (1, 3) for k in (1, 2, 3, 4, 6, 8)
                         for r in (True, False) if k > 1 or r]:
        if npieces == 1:
            def go():
                ops.gemm_x3p_tn(Xb.view(-1), 0, Gb, 0, C, M, N, B, Mp, N, N, splitk=sk, colsum=cs,
                                npieces=1, reduce=red)
        else:
            def go():
                ops.gemm_x3p_tn(X3.view(-1), B * Mp, G3, B * N, C, M, N, B, Mp, N, N, splitk=sk,
                                colsum=cs, npieces=3, reduce=red)
        C.zero_()
        cs.zero_()
        go()
        torch.cuda.synchronize()
        ref = ref1 if npieces == 1 else ref3
        err = ((C.double() - ref).abs().max() / ref.abs().max()).item()
        cref = (Gb.double() if npieces == 1 else G.double()).sum(0)
        cerr = ((cs.double() - cref).abs().max() / cref.abs().max()).item()
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
        fl = 2.0 * B * M * N * (1 if npieces == 1 else 6)
        print(f"var {var} npieces {npieces} splitk {sk:2d} {'reduce' if red else 'atomic'}: {us:7.1f} us  {fl / us / 1e6:7.1f} TF"
              f"  relerr {err:.2e} colsum {cerr:.2e}", flush=True)

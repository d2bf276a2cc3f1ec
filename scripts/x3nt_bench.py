"""Stand-alone timing of the NT x3 GEMM (dX = dY W^T, the fp32 VAE input
gradients) at the train step's shapes, HIP events; MOG_AIR_LIB points at
another build for A/B.  Prints the max error against float64 relative to
sum |a||b| as well."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

dev = "cuda:0"


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


def nt(M, N, K, epi):
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    aux = torch.randn(M, N, device=dev) if epi else None
    W3 = torch.empty(3, N, K, device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(W, W3, N, K, K, K, N * K)
    C = torch.empty(M, N, device=dev)
    us = timeit(lambda: ops.gemm_x3_nt(A, W3, N * K, C, M, N, K, K, K, N, aux=aux,
                                       ldaux=N if epi else 0))
    r = slice(0, 2048)
    ref = A[r].double() @ W.double().t()
    mag = A[r].double().abs() @ W.double().abs().t()
    if epi:
        s = torch.sigmoid(aux[r].double())
        ref, mag = ref * s, mag * s
    err = ((C[r].double() - ref).abs() / mag).max().item()
    fl = 2.0 * M * N * K * 6
    print(f"NT M={M} N={N} K={K} epi={epi}: {us:.1f} us "
          f"({fl / us / 1e6:.0f} TF bf16 = {fl / us / 1e6 / 2500:.2f} of peak), err {err:.1e}",
          flush=True)


nt(24576, 512, 784, 1)
nt(24576, 256, 512, 1)
nt(24576, 512, 256, 1)
nt(24576, 784, 512, 0)

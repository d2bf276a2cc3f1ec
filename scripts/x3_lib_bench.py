"""Calibration: the three-piece (x3) fp32-accurate products of the fp32 step
as ONE bf16 GEMM with K' = 6K (pieces concatenated along k, fp32 accumulate
and output) through the vendor library (torch.mm(out_dtype=float32) ->
hipBLASLt), against this repo's x3 kernels on the same shapes.  Not product
code: it decides whether the library GEMM is worth binding."""
import os
import sys
import time

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


def tn(M, N, K):
    """C[M,N] = A^T B over K rows (weight gradient)."""
    A = torch.randn(K, M, device=dev)
    B = torch.randn(K, N, device=dev)
    C = torch.zeros(M, N, device=dev)
    Mp = (M + 7) // 8 * 8
    A3 = torch.empty(3, K, Mp, device=dev, dtype=torch.bfloat16)
    B3 = torch.empty(3, K, N, device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(A, A3, K, M, M, Mp, K * Mp)
    ops.split3_bf16(B, B3, K, N, N, N, K * N)
    t_inkernel = timeit(lambda: ops.gemm_x3_tn(A, B, C, M, N, K, M, N, N,
                                               splitk=max(1, min(K // 256, 8))))
    t_pre = timeit(lambda: ops.gemm_x3p_tn(A3.view(-1), K * Mp, B3, K * N, C, M, N, K, Mp, N, N,
                                           splitk=max(1, min(K // 256, 8))))
    Acat = torch.cat([A3[2], A3[1], A3[0], A3[1], A3[0], A3[0]], 0)[:, :M]  # [6K, M]
    Bcat = torch.cat([B3[0], B3[1], B3[2], B3[0], B3[1], B3[0]], 0)       # [6K, N]
    At = Acat.t()
    t_lib = timeit(lambda: torch.mm(At, Bcat, out_dtype=torch.float32))
    ref = A.double().t() @ B.double()
    got = torch.mm(At, Bcat, out_dtype=torch.float32).double()
    err = ((got - ref).abs() / (A.double().abs().t() @ B.double().abs())).max().item()
    fl = 2.0 * M * N * K
    print(f"TN M={M} N={N} K={K}: x3 in-kernel {t_inkernel:.1f} us, x3 pre-split {t_pre:.1f} us, "
          f"library bf16 K'=6K {t_lib:.1f} us ({6 * fl / t_lib / 1e6:.0f} TF bf16), lib err {err:.1e}",
          flush=True)


def nt(M, N, K):
    """C[M,N] = A B^T (input gradient dY W^T)."""
    A = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev)
    W3 = torch.empty(3, N, K, device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(W, W3, N, K, K, K, N * K)
    C = torch.empty(M, N, device=dev)
    t_nt = timeit(lambda: ops.gemm_x3_nt(A, W3, N * K, C, M, N, K, K, K, N))
    A3 = torch.empty(3, M, K, device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(A, A3, M, K, K, K, M * K)
    Acat = torch.cat([A3[2], A3[1], A3[0], A3[1], A3[0], A3[0]], 1)  # [M, 6K]
    Wcat = torch.cat([W3[0], W3[1], W3[2], W3[0], W3[1], W3[0]], 1)  # [N, 6K]
    t_lib = timeit(lambda: torch.mm(Acat, Wcat.t(), out_dtype=torch.float32))
    t_f32 = timeit(lambda: torch.mm(A, W.t()))
    fl = 2.0 * M * N * K
    print(f"NT M={M} N={N} K={K}: x3 nt {t_nt:.1f} us ({6 * fl / t_nt / 1e6:.0f} TF bf16), library "
          f"bf16 K'=6K {t_lib:.1f} us (+ split of A not counted), torch fp32 {t_f32:.1f} us",
          flush=True)


tn(2500, 1024, 8192)
tn(784, 512, 24576)
tn(512, 784, 24576)
nt(24576, 512, 784)
nt(24576, 784, 512)
nt(24576, 256, 512)

"""Split-K sweep of the fp32 weight-gradient GEMMs (dW = X^T dY, K = T*B rows,
atomic epilogue) of the AIR train step at B = 8192, T = 3.  The tile is the
one MOG_GEMM_TILE forces (read once per process), so run one process per tile:
    MOG_GEMM_TILE=64 python scripts/sweep_dw.py ; MOG_GEMM_TILE=128 python scripts/sweep_dw.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

B, TB = 8192, 3 * 8192
SHAPES = [
    ("dW_x", 2500, 1024, B),
    ("dW_rec1", 784, 512, TB),
    ("dW_genmean", 512, 784, TB),
    ("dW_rec2", 512, 256, TB),
    ("dW_gen2", 256, 512, TB),
    ("dW_Wh", 256, 1024, 2 * B),
]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev = "cuda:0"
    tag = os.environ.get("MOG_GEMM_TILE", "auto")
    splits = [int(s) for s in os.environ.get("SPLITS", "1,2,4,8,16,32").split(",")]
    for name, M, N, K in SHAPES:
        A = torch.randn(K, M, device=dev)
        Bm = torch.randn(K, N, device=dev)
        C = torch.zeros(M, N, device=dev)
        flop = 2.0 * M * N * K
        best = None
        for s in splits:
            if K // s < 64:
                continue
            t = timeit(lambda: ops.gemm([A], [Bm], [C], M, N, K, M, N, N, transA=True,
                                        epi=ops.EPI_ATOMIC, splitk=s))
            tf = flop / t / 1e6
            best = max(best or 0, tf)
            print(f"{name:11s} M={M:5d} N={N:5d} K={K:6d} tile={tag:5s} splitk={s:3d} "
                  f"{t:8.1f}us {tf:6.1f} TF", flush=True)
        print(f"{name:11s} best {best:6.1f} TF", flush=True)


if __name__ == "__main__":
    main()

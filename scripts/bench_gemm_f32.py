"""fp32 GEMM micro-benchmark on the AIR train-step shapes (B = 8192, T = 3):
mog_gemm_f32 (auto tile, or the tile MOG_GEMM_TILE=64|128 forces) next to torch.matmul fp32 (hipBLASLt) as a calibration point (not
used by the product).  usage: python scripts/bench_gemm_f32.py [tile]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

B, TB = 8192, 3 * 8192
# name, M, N, K, transA, transB, epi, splitk
SHAPES = [
    ("xproj", B, 1024, 2500, 0, 0, ops.EPI_STORE, 1),
    ("recur", B, 1024, 256, 0, 0, ops.EPI_STORE, 1),
    ("enc1", B, 512, 784, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("enc2", B, 256, 512, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("dec2", B, 512, 256, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("genmean", B, 784, 512, 0, 0, ops.EPI_SIGMOID_NOISE, 1),
    ("enc1_TB", TB, 512, 784, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("enc2_TB", TB, 256, 512, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("dec2_TB", TB, 512, 256, 0, 0, ops.EPI_SOFTPLUS, 1),
    ("genmean_TB", TB, 784, 512, 0, 0, ops.EPI_SIGMOID_NOISE, 1),
    ("dX_dd2", TB, 512, 784, 0, 1, ops.EPI_SOFTPLUS_BWD, 1),
    ("dX_dg", TB, 784, 512, 0, 1, ops.EPI_STORE, 1),
    ("dX_da1", TB, 512, 256, 0, 1, ops.EPI_SOFTPLUS_BWD, 1),
    ("lstm_dh", B, 256, 1024, 0, 1, ops.EPI_STORE, 1),
    ("dW_x", 2500, 1024, B, 1, 0, ops.EPI_ATOMIC, 0),
    ("dW_rec1", 784, 512, TB, 1, 0, ops.EPI_ATOMIC, 0),
    ("dW_genmean", 512, 784, TB, 1, 0, ops.EPI_ATOMIC, 0),
    ("dW_rec2", 512, 256, TB, 1, 0, ops.EPI_ATOMIC, 0),
    ("dW_Wh", 256, 1024, 2 * B, 1, 0, ops.EPI_ATOMIC, 0),
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
    return e0.elapsed_time(e1) / iters * 1e3  # us


def splitk_for(M, N, K, target=2048):
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    return max(1, min(K // 256, (target + tiles - 1) // tiles))


def main():
    dev = "cuda:0"
    tag = os.environ.get("MOG_GEMM_TILE", "auto")
    only_ref = len(sys.argv) > 1 and sys.argv[1] == "ref"
    only = os.environ.get("GEMM_ONLY")
    for name, M, N, K, ta, tb, epi, sk in SHAPES:
        if only and name not in only.split(","):
            continue
        A = torch.randn((K, M) if ta else (M, K), device=dev)
        Bm = torch.randn((N, K) if tb else (K, N), device=dev)
        C = torch.zeros(M, N, device=dev)
        aux = torch.rand(M, N, device=dev)
        bias = torch.zeros(N, device=dev)
        flop = 2.0 * M * N * K
        if only_ref:
            a = A.t() if ta else A
            b = Bm.t() if tb else Bm
            t = timeit(lambda: torch.matmul(a, b))
            print(f"{name:11s} M={M:6d} N={N:5d} K={K:6d} hipBLASLt fp32 {t:8.1f}us "
                  f"{flop / t / 1e6:6.1f} TF", flush=True)
            continue
        s = splitk_for(M, N, K) if sk == 0 else 1
        kw = dict(transA=bool(ta), transB=bool(tb), epi=epi, splitk=s)
        if epi in (ops.EPI_SOFTPLUS_BWD, ops.EPI_SIGMOID_NOISE):
            kw.update(aux=[aux], ldaux=N)
        if epi in (ops.EPI_SOFTPLUS, ops.EPI_SIGMOID_NOISE):
            kw.update(bias=[bias])
        lda = M if ta else K
        ldb = K if tb else N
        t = timeit(lambda: ops.gemm([A], [Bm], [C], M, N, K, lda, ldb, N, **kw))
        print(f"{name:11s} M={M:6d} N={N:5d} K={K:6d} tile={tag:7s} splitk={s:3d} {t:8.1f}us "
              f"{flop / t / 1e6:6.1f} TF", flush=True)


if __name__ == "__main__":
    main()

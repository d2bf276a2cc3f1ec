"""Weight-gradient GEMM microbenchmark: dW += X^T dY (split-K, atomics) for
the fp32 train step's shapes (B = 8192, T = 3: K = 24576 rows for the VAE,
8192 for the x-projection), timed per shape for a list of split-K targets.

usage: python scripts/dw_bench.py [targets...]   (env MOG_GEMM_TILE / MOG_GEMM_BK
select the tile; MOG_DW32_TARGET is what the model uses)"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "mog-asr_amd"))
import torch  # noqa: E402

from mog_air.ops import EPI_ATOMIC, gemm  # noqa: E402

DEV = "cuda:0"
TB = 24576
SHAPES = [  # name, K rows, M (in), N (out), batch
    ("rec1", TB, 784, 512, 1), ("rec2", TB, 512, 256, 1), ("mulv", TB, 256, 50, 2),
    ("gen1", TB, 50, 256, 1), ("gen2", TB, 256, 512, 1), ("gmean", TB, 512, 784, 1),
    ("xgrad", 8192, 2500, 1024, 1)]


def run(targets):
    torch.manual_seed(0)
    tot = {t: 0.0 for t in targets}
    for name, K, M, N, nb in SHAPES:
        X = [torch.randn(K, M, device=DEV) for _ in range(nb)]
        dY = [torch.randn(K, N, device=DEV) for _ in range(nb)]
        out = [torch.zeros(M, N, device=DEV) for _ in range(nb)]
        bo = [torch.zeros(N, device=DEV) for _ in range(nb)]
        flop = 2.0 * K * M * N * nb
        line = []
        for tgt in targets:
            tiles = ((M + 63) // 64) * ((N + 63) // 64) * nb
            splitk = max(1, min(K // 256, (tgt + tiles - 1) // tiles))
            f = lambda: gemm(X, dY, out, M, N, K, M, N, N, transA=True, epi=EPI_ATOMIC,  # noqa
                             splitk=splitk, colsum=bo)
            for _ in range(3):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                f()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / 20 * 1e3
            tot[tgt] += us
            line.append("t%-5d sk%-3d %7.1f us %5.1f TF" % (tgt, splitk, us, flop / us * 1e-6))
        print("%-6s %s" % (name, " | ".join(line)), flush=True)
    print("total  " + " | ".join("t%d %.1f us" % (t, v) for t, v in tot.items()), flush=True)


if __name__ == "__main__":
    run([int(a) for a in sys.argv[1:]] or [256, 512, 1024, 2048])

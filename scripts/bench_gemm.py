"""Micro-benchmark of the hand-written GEMMs on the train-step shapes, next to
torch.matmul (hipBLASLt) as a calibration point (not used by the product)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import torch  # noqa: E402

from mog_air import ops  # noqa: E402


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


def main():
    dev = "cuda:0"
    B = 8192
    shapes = [("vae1 fwd", B, 512, 784), ("vae6 fwd", B, 784, 512), ("vae2 fwd", B, 256, 512),
              ("vae1 dX", B, 784, 512)]
    for name, M, N, K in shapes:
        A = torch.randn(M, K, device=dev).to(torch.bfloat16)
        Bt = torch.randn(N, K, device=dev).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        Cf = torch.empty(M, N, device=dev)
        bias = torch.zeros(N, device=dev)
        flop = 2.0 * M * N * K
        t_store = timeit(lambda: ops.gemm_bf16([A], [Bt], [Cf], M, N, K, K, K, N))
        t_sp = timeit(lambda: ops.gemm_bf16([A], [Bt], [C], M, N, K, K, K, N,
                                            epi=ops.BF_SOFTPLUS, bias=[bias]))
        t_ref = timeit(lambda: torch.matmul(A, Bt.t()))
        print(f"{name:10s} M={M} N={N} K={K}: store {t_store:7.1f}us ({flop/t_store/1e6:6.0f} TF) "
              f"softplus {t_sp:7.1f}us  hipBLASLt {t_ref:7.1f}us ({flop/t_ref/1e6:6.0f} TF)")
    # TN weight gradient
    if os.environ.get("GEMM_TN_ONLY"):
        shapes_tn = (("dW1", 3 * B, 784, 512), ("dWgo", 3 * B, 512, 784),
                     ("dWx", B, 2504, 1024), ("dW2", 3 * B, 512, 256))
        for name, K, M, N in shapes_tn:
            X = torch.randn(K, M, device=dev).to(torch.bfloat16)
            dY = torch.randn(K, N, device=dev).to(torch.bfloat16)
            out = torch.zeros(M, N, device=dev)
            flop = 2.0 * M * N * K
            for thr in ("512", "1"):
                os.environ["MOG_BF16_BIG_TN"] = thr
                for sk in (1, 2, 4, 8, 16):
                    if K // sk < 512:
                        continue
                    t = timeit(lambda: ops.gemm_bf16([X], [dY], [out], M, N, K, M, N, N,
                                                     tn=True, epi=ops.BF_ATOMIC, splitk=sk))
                    print(f"{name} thr={thr} splitk={sk}: {t:7.1f}us ({flop/t/1e6:6.0f} TF)",
                          flush=True)
            t_ref = timeit(lambda: torch.matmul(X.t(), dY))
            print(f"{name} hipBLASLt {t_ref:7.1f}us ({flop/t_ref/1e6:6.0f} TF)", flush=True)
        return
    for name, K, M, N in (("dW1", 3 * B, 784, 512), ("dWgo", 3 * B, 512, 784)):
        X = torch.randn(K, M, device=dev).to(torch.bfloat16)
        dY = torch.randn(K, N, device=dev).to(torch.bfloat16)
        out = torch.zeros(M, N, device=dev)
        flop = 2.0 * M * N * K
        for sk in (8, 16, 32):
            t = timeit(lambda: ops.gemm_bf16([X], [dY], [out], M, N, K, M, N, N, tn=True,
                                             epi=ops.BF_ATOMIC, splitk=sk))
            print(f"{name} TN splitk={sk}: {t:7.1f}us ({flop/t/1e6:6.0f} TF)")
        t_ref = timeit(lambda: torch.matmul(X.t(), dY))
        print(f"{name} hipBLASLt {t_ref:7.1f}us ({flop/t_ref/1e6:6.0f} TF)")
    # fp32 LSTM x-projection
    M, N, K = B, 1024, 2500
    X = torch.randn(M, K, device=dev)
    W = torch.randn(K, N, device=dev)
    G = torch.empty(M, N, device=dev)
    flop = 2.0 * M * N * K
    t = timeit(lambda: ops.gemm([X], [W], [G], M, N, K, K, N, N), iters=5)
    t_ref = timeit(lambda: torch.matmul(X, W), iters=5)
    print(f"xproj fp32: {t:7.1f}us ({flop/t/1e6:6.0f} TF)  torch fp32 {t_ref:7.1f}us "
          f"({flop/t_ref/1e6:6.0f} TF)")


if __name__ == "__main__":
    main()

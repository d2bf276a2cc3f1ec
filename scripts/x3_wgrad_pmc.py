"""(MODE=nt: the NT input-gradient kernel instead, dX = dY W^T at 24,576 rows.)
One x3 VAE weight-gradient shape (gemm_x3_tn_kernel<false,3>, the fp32 step's
784 x 512 x 24,576 with its split-K 19) launched 10 times, for rocprofv3 --pmc
passes (scripts/gpu_x3_pmc.sh); prints the event-timed launch."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

M, N, K = int(os.environ.get("M", 784)), int(os.environ.get("N", 512)), 24576
dev = "cuda:0"
g = torch.Generator(device=dev).manual_seed(0)
A = torch.rand(K, M, device=dev, generator=g)
B = torch.randn(K, N, device=dev, generator=g) * 1e-3
C = torch.zeros(M, N, device=dev)
cs = torch.zeros(N, device=dev)
if os.environ.get("MODE") == "nt":
    # the VAE input-gradient form: dX [24,576 x N] = dY [24,576 x M] W^T, W [N x M]
    Ad = torch.randn(K, M, device=dev, generator=g) * 1e-3
    W = torch.randn(N, M, device=dev, generator=g) * 0.05
    W3 = torch.empty(3, N, M, device=dev, dtype=torch.bfloat16)
    ops.split3_bf16(W, W3, N, M, M, M, N * M)
    aux = torch.rand(K, N, device=dev, generator=g) + 0.1
    D = torch.empty(K, N, device=dev)

    def nt():
        ops.gemm_x3_nt(Ad, W3, N * M, D, K, N, M, M, M, N, aux=aux, ldaux=N)
    for _ in range(3):
        nt()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        nt()
    e1.record()
    torch.cuda.synchronize()
    print(f"x3 nt {K}x{N}x{M}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us", flush=True)
    sys.exit(0)
tiles = ((M + 127) // 128) * ((N + 127) // 128)
sk = max(1, min(K // 256, (512 + tiles - 1) // tiles))
for _ in range(3):
    ops.gemm_x3_tn(A, B, C, M, N, K, M, N, N, splitk=sk, colsum=cs, reduce=False)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    ops.gemm_x3_tn(A, B, C, M, N, K, M, N, N, splitk=sk, colsum=cs, reduce=False)
e1.record()
torch.cuda.synchronize()
print(f"x3 tn {M}x{N}x{K} splitk {sk}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us", flush=True)

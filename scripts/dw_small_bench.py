"""Stand-alone timing of the fp32 step's small weight-gradient GEMMs (the
side-stream launches AIRModel._dw makes at T*B = 24,576 rows: the VAE's
256 x 50 / 50 x 256 layers, the heads' hidden and output layers, the LSTM
recurrent rows), HIP events, over the split-K targets.  Not product code."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402
from mog_air.air_model import AIRModel  # noqa: E402

dev = "cuda:0"
TB = 24576


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


class _M:
    _dw = AIRModel._dw


def case(name, X, dY, M, N, K, lda, ldb, nout, colsum=True):
    out = [torch.zeros(M, N, device=dev) for _ in range(nout)]
    cs = [torch.zeros(N, device=dev) for _ in range(nout)] if colsum else None
    m = _M()
    for tgt in ("256", "512", "1024", "2048", "4096"):
        os.environ["MOG_DW32_TARGET"] = tgt
        us = timeit(lambda: m._dw(X, dY, out, K, M, N, lda, ldb, cs))
        print(f"  {name} target {tgt}: {us:.1f} us", flush=True)
    os.environ["MOG_DW32_TARGET"] = "2048"
    us = timeit(lambda: m._dw(X, dY, out, K, M, N, lda, ldb, cs))
    ref = [(x[:K].double().t() @ d[:K, :N].double()) if d.shape[1] == N else None
           for x, d in zip(X, dY)]
    fl = 2.0 * M * N * K * nout
    print(f"{name}: M={M} N={N} K={K} x{nout}: {us:.1f} us ({fl / us / 1e6:.1f} TF/s)", flush=True)
    del ref


torch.manual_seed(0)
a2 = torch.randn(TB, 256, device=dev)
dmu, dlv = torch.randn(TB, 50, device=dev), torch.randn(TB, 50, device=dev)
case("rec_mean+lv", [a2, a2], [dmu, dlv], 256, 50, TB, 256, 50, 2)
z, dd1 = torch.randn(TB, 50, device=dev), torch.randn(TB, 256, device=dev)
case("generative_1", [z], [dd1], 50, 256, TB, 50, 256, 1)
h = torch.randn(TB, 256, device=dev)
dhid = torch.randn(TB, 5, 64, device=dev)
case("heads hidden", [h] * 5, [dhid[:, i] for i in range(5)], 256, 64, TB, 256, 320, 5)
hid = torch.randn(5, TB, 64, device=dev)
dout = torch.randn(5, TB, 2, device=dev)
case("heads out k=1", [hid[i] for i in range(3)], [dout[i] for i in range(3)], 64, 1, TB, 64, 2, 3)
case("heads out k=2", [hid[i] for i in range(3, 5)], [dout[i] for i in range(3, 5)], 64, 2, TB,
     64, 2, 2)
dG = torch.randn(2 * 8192, 1024, device=dev)
case("lstm rec rows", [h[:16384]], [dG], 256, 1024, 16384, 256, 1024, 1, colsum=False)

"""Measured answer to "a dense or MFMA STN backward" (DESIGN.md §4.5, round 5):
times the dense fp32-MFMA input gradient dU = W_y^T (s G) W_x of the STN write
backward (scripts/stn_dense_probe.hip, built into scripts/bin/) at the fp32
step's 24,576 images against the product kernel (mog_stn_backward: dU AND
dtheta AND dot in one launch) on the same AIR-like inputs, and checks the
probe's dU against the product's.  Prints one JSON line.

usage: python scripts/stn_dense_probe.py [N] [B]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

from mog_air import ops  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 24576
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
dev = torch.device("cuda:0")
lib = ctypes.CDLL(os.path.join(ROOT, "scripts", "bin", "libstn_dense_probe.so"))
lib.stn_dense_du.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
g = torch.Generator().manual_seed(1)
# AIR's write transform (glimpse 28 -> canvas 50): theta_back = [1/s, 0, -tx/s, 0, 1/s, -ty/s]
s = 0.25 + 0.5 * torch.rand(N, generator=g)
tx, ty = (torch.rand(N, generator=g) * 1.6 - 0.8 for _ in range(2))
th = torch.stack([1 / s, torch.zeros(N), -tx / s, torch.zeros(N), 1 / s, -ty / s], 1).float().to(dev)
r = torch.rand(N, 784, generator=g).to(dev)
dcanvas = (torch.randn(B, 2500, generator=g) * 1e-3).to(dev)
zc = torch.rand(N, generator=g).to(dev)
dU_ref = torch.empty(N, 784, device=dev)
dth = torch.empty(N, 6, device=dev)
dot = torch.empty(N, device=dev)
dU_p = torch.empty(N, 784, device=dev)


def product():
    ops.stn_backward(r, th, (50, 50), dcanvas, gscale=zc, dU=dU_ref, dtheta=dth, dot=dot,
                     want_dot=True, n=N)


def probe():
    rc = lib.stn_dense_du(dcanvas.data_ptr(), B, th.data_ptr(), zc.data_ptr(), dU_p.data_ptr(), N,
                          ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    assert rc == 0, rc


def timeit(f, reps=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


product()
probe()
torch.cuda.synchronize()
err = float((dU_p - dU_ref).abs().max() / (dU_ref.abs().max() + 1e-30))
t_prod, t_probe = timeit(product), timeit(probe)
# algorithmic bytes of the write backward: r 3,136 + cotangent 10,000 / T
# + dU 3,136 + theta / dtheta / dot 52 per image
algo = N * (3136 + 10000 * B / N + 3136 + 52)
print(json.dumps({"images": N, "product_write_bwd_us": t_prod, "dense_mfma_dU_only_us": t_probe,
                  "dense_mfma_count_per_image": 156,
                  "product_frac_hbm": algo / (t_prod * 1e-6) / 8e12,
                  "dU_max_rel_diff_vs_product": err}), flush=True)

"""Micro-benchmark of the STN kernels at the train-step shapes (B images)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from mog_air import ops  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(2):
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    only_wbwd = len(sys.argv) > 2 and sys.argv[2] == "wbwd"
    dev = "cuda:0"
    rng = np.random.default_rng(0)
    s = rng.uniform(0.3, 0.7, B)
    t = rng.uniform(-0.6, 0.6, (B, 2))
    for sep in (True, False):
        sh = np.zeros(B) if sep else np.full(B, 0.05)
        thf = torch.tensor(np.stack([s, sh, t[:, 0], -sh, s, t[:, 1]], 1), dtype=torch.float32,
                           device=dev)
        thb = torch.tensor(np.stack([1 / s, sh, -t[:, 0] / s, -sh, 1 / s, -t[:, 1] / s], 1),
                           dtype=torch.float32, device=dev)
        r = torch.rand(B, 784, device=dev)
        x = torch.rand(B, 2500, device=dev)
        G = torch.randn(B, 2500, device=dev)
        g28 = torch.randn(B, 784, device=dev)
        zs = torch.rand(B, device=dev)
        dU = torch.empty(B, 784, device=dev)
        dth = torch.empty(B, 6, device=dev)
        dot = torch.empty(B, device=dev)
        os.environ["MOG_STN_TIMING"] = "1"
        ops.stn_backward(r, thb, (50, 50), G, gscale=zs, dU=dU, dtheta=dth, dot=dot, want_dot=True)
        ops.stn_backward(x, thf, (28, 28), g28, want_dU=False, dtheta=dth)
        del os.environ["MOG_STN_TIMING"]
        tw = timeit(lambda: ops.stn_backward(r, thb, (50, 50), G, gscale=zs, dU=dU, dtheta=dth,
                                             dot=dot, want_dot=True))
        if only_wbwd:
            print(f"sep={sep}: write-bwd {tw:7.1f} us", flush=True)
            continue
        tr = timeit(lambda: ops.stn_backward(x, thf, (28, 28), g28, want_dU=False, dtheta=dth))
        out = torch.empty(B, 784, device=dev)
        cv = torch.zeros(B, 2500, device=dev)
        m1 = torch.ones(B, device=dev)
        tf = timeit(lambda: ops.stn_forward(x, thf, (28, 28), out=out))
        ta = timeit(lambda: ops.stn_forward(r, thb, (50, 50), out=cv, z=zs, mask=m1,
                                            accumulate=True))
        print(f"sep={sep}: write-bwd {tw:7.1f} us  read-bwd {tr:7.1f} us  read-fwd {tf:7.1f} us  "
              f"write-fwd-acc {ta:7.1f} us", flush=True)


if __name__ == "__main__":
    main()

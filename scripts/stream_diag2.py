"""Repeat one plain forked step on fresh models (ONE_PASS_WGRADS) and list
the workspace buffers and gradient tensors that differ from the first run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_streams as ts  # noqa: E402

model, prec, B, n = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
make = ts._air if model == "air" else ts._asr
data = ts._data(B)
SKIP = {"G", "cparts", "eps_x", "dr", "dz", "dg", "dth_f", "dth_b", "dot", "dr_all", "canvas",
        "recon", "tmp_a2", "dm1"}


KEEP = []
ONE = [None]


def run(i):
    if os.environ.get("DIAG_ONE") == "1" and ONE[0] is not None:
        m = ONE[0]
    else:
        m = make("d2_%d" % i, prec)
        ONE[0] = m
    if os.environ.get("DIAG_KEEP") == "1":
        KEEP.append(m)
    if os.environ.get("DIAG_NOSIDE") == "1":
        m.SIDE_MIN_BATCH = 1 << 30
    m.ONE_PASS_WGRADS = True
    m.compute_gradients(*data[0])
    torch.cuda.synchronize()
    ws = m._ws
    d = {k: v.clone() for k, v in vars(ws).items() if isinstance(v, torch.Tensor) and k not in SKIP}
    g = m.params.grad_dict()
    out = torch.empty_like(ws.dth_f_all)
    W, TB = m.windows_size, B * m.max_steps
    from mog_air import ops
    ops.stn_backward(data[0][0].reshape(B, -1), ws.th_f, (W, W), ws.dg_all, want_dU=False,
                     dtheta=out, n=TB)
    torch.cuda.synchronize()
    bad = (out.view(-1, 6) != ws.dth_f_all.view(-1, 6)).any(dim=1).nonzero().flatten()
    mism.append(int(bad.numel()))
    if bad.numel():
        r = int(bad[0])
        print("   relaunch", out.view(-1, 6)[r].tolist(), "\n   in-model", ws.dth_f_all.view(-1, 6)[r].tolist(), flush=True)
    return d, g


mism = []
ref, gref = run(0)
for i in range(1, n):
    cur, g = run(i)
    bad = [k for k in ref if not torch.equal(ref[k].view(torch.uint8), cur[k].view(torch.uint8))]
    gbad = [k for k in gref if gref[k].tobytes() != g[k].tobytes()]
    print(i, "ws differs:", bad, "| grads differ:", gbad, flush=True)
print("SUMMARY", os.environ.get("DIAG_TAG", ""), "mismatching images per run:", mism, flush=True)

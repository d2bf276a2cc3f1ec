"""Is the STN read backward deterministic on fixed inputs, and does it read
LDS it did not write?  (mog_lds_poison before each launch.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_streams as ts  # noqa: E402
from mog_air import ops  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
data = ts._data(B)
m = ts._air("lds", "fp32")
m.ONE_PASS_WGRADS = True
m.compute_gradients(*data[0])
torch.cuda.synchronize()
ws, W, TB = m._ws, m.windows_size, B * m.max_steps
X = data[0][0].reshape(B, -1).float().contiguous()


def once(poison=None):
    out = torch.empty((TB, 6), device="cuda:0")
    if poison is not None:
        ops.lds_poison(poison)
    ops.stn_backward(X, ws.th_f, (W, W), ws.dg_all, want_dU=False, dtheta=out, n=TB)
    torch.cuda.synchronize()
    return out


ref = once()
print("in-model dth_f_all equal to a plain relaunch:", torch.equal(ref, ws.dth_f_all), flush=True)
for label, p in (("plain", None), ("nan", 0x7FC00000), ("zero", 0), ("big", 0x5F000000)):
    diffs = []
    for _ in range(5):
        o = once(p)
        diffs.append(int((o.view(torch.int32) != ref.view(torch.int32)).any(dim=1).sum()))
    print(label, "images differing per launch:", diffs, flush=True)

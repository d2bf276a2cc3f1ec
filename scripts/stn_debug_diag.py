"""Diagnosis build (-DMOG_STN_DEBUG): per-pixel operands of the STN read
backward alone vs beside a side-stream GEMM; prints the first differing
pixels' operands."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "scripts")]
sys.argv = [sys.argv[0], "none"]
import torch  # noqa: E402

import stn_concurrency as sc  # noqa: E402
from mog_air import _lib  # noqa: E402

lib = _lib.load()
lib.mog_stn_debug_set.argtypes = [ctypes.c_void_p]
TB, Hout, Wout = sc.TB, 28, 28
NAMES = ["g", "Ia", "Ib", "Ic", "Id", "ax", "bx", "ay", "by", "x0", "x1", "y0", "y1", "dx", "dy", "gm"]


def run(side_fn, spin):
    dbg = torch.full((TB * Hout * Wout * 16,), float("nan"), device="cuda:0")
    lib.mog_stn_debug_set(ctypes.c_void_p(dbg.data_ptr()))
    out = torch.empty_like(sc.ref)
    if side_fn is not None:
        ev = torch.cuda.Event()
        ev.record(sc.main)
        sc.side.wait_event(ev)
        with torch.cuda.stream(sc.side):
            for _ in range(3):
                side_fn()
    sc.ops.spin(spin)
    sc.stn(out)
    torch.cuda.synchronize()
    lib.mog_stn_debug_set(ctypes.c_void_p(0))
    return out, dbg.view(TB, Hout, Wout, 16)


o0, d0 = run(None, 0)
found = 0
for r in range(40):
    o1, d1 = run(sc.x3_nt, (r % 8) * 2000)
    badimg = (o1.view(TB, -1) != o0.view(TB, -1)).any(dim=1).nonzero().flatten().tolist()
    if not badimg:
        continue
    for n in badimg[:3]:
        a, b = d0[n].view(torch.int32), d1[n].view(torch.int32)
        diff = (a != b).any(dim=2).nonzero().tolist()
        print(f"rep {r} image {n}: {len(diff)} pixels differ; dtheta {o0.view(TB, -1)[n].tolist()} vs {o1.view(TB, -1)[n].tolist()}", flush=True)
        for (i, j) in diff[:6]:
            fa, fb = d0[n, i, j], d1[n, i, j]
            fields = [k for k in range(16) if fa.view(torch.int32)[k] != fb.view(torch.int32)[k]]
            def show(f):
                return {NAMES[k]: (int(f.view(torch.int32)[k]) if k in (9, 10, 11, 12) else float(f[k])) for k in fields}
            print(f"   pixel ({i},{j}) fields {[NAMES[k] for k in fields]} alone {show(fa)} beside {show(fb)}", flush=True)
    found += 1
    if found >= 4:
        break
print("done", flush=True)

"""Diagnosis: the bf16 captured step against eager at the reference's batch of
64, repeated; reports the first step and the parameters / gradients that
differ (tests/test_gpu_graph.py::test_graph_replay_matches_eager_bitwise)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import test_gpu_graph as tg  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
data = tg._batches(4)
bad = 0
for rep in range(reps):
    me, mg = tg._model("re%d" % rep, prec), tg._model("rg%d" % rep, prec)
    for i, (x, k) in enumerate(data):
        me.train_step_async(x, k)
        mg.train_step_graphed(x, k)
        torch.cuda.synchronize()
        same = torch.equal(me.params.flat.view(torch.int32), mg.params.flat.view(torch.int32))
        gsame = torch.equal(me.params.grad.view(torch.int32), mg.params.grad.view(torch.int32))
        if not (same and gsame):
            diff = []
            for name, shape in me.params.specs:
                o = me.params.offsets[name]
                n = int(np.prod(shape))
                dg = (me.params.grad[o:o + n] - mg.params.grad[o:o + n]).abs().max().item()
                if dg > 0 or not torch.equal(me.params.grad[o:o + n].view(torch.int32),
                                             mg.params.grad[o:o + n].view(torch.int32)):
                    diff.append((name, dg))
            print(f"rep {rep} step {i}: params equal {same}, grads equal {gsame}; grads differ: "
                  f"{diff[:6]}", flush=True)
            bad += 1
            break
print(f"{prec}: {bad} of {reps} runs differ", flush=True)

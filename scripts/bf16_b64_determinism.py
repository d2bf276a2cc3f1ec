"""Determinism probe for the bf16 batch-64 flake (DESIGN §4.8 open items):
the same inputs and noise run repeatedly through (1) the train-mode forward
(fused bf16 step kernel, saved activations) and (2) compute_gradients; counts
the runs whose outputs / gradients differ bitwise from the first run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_graph as tg  # noqa: E402

prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
x, k = tg._batches(1)[0]
m = tg._model("det" + prec, prec)
names = ("r", "gb", "a1b", "a2b", "zb", "d1b", "d2b", "z", "mu", "lv", "cparts", "prows", "means")
ref, gref, bad_f, bad_g = None, None, {}, 0
for i in range(n):
    m._noise_ctr = 0
    g = m.compute_gradients(x, k)
    torch.cuda.synchronize()
    ws = m._ws
    cur = {a: getattr(ws, a).clone() for a in names if isinstance(getattr(ws, a, None), torch.Tensor)}
    gr = m.params.grad.clone()
    if ref is None:
        ref, gref = cur, gr
        continue
    for a in cur:
        if not torch.equal(cur[a].view(torch.uint8) if cur[a].dtype != torch.bool else cur[a],
                           ref[a].view(torch.uint8) if ref[a].dtype != torch.bool else ref[a]):
            bad_f[a] = bad_f.get(a, 0) + 1
    if not torch.equal(gr.view(torch.int32), gref.view(torch.int32)):
        bad_g += 1
print(f"{prec}: {n - 1} repeats; forward buffers differing: {bad_f or 'none'}; "
      f"gradients differing in {bad_g} runs", flush=True)

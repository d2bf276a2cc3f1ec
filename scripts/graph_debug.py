"""Graph-capture probe: does capturing change any state; eager vs replay."""
import sys
import torch
sys.path.insert(0, 'mog-asr_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import test_gpu_graph as tg  # noqa: E402

data = tg._batches(2)
me, mg = tg._model("ea", "fp32"), tg._model("gb", "fp32")
x, k = data[0]
me.train_step_async(x, k)
mg._graph_noise = True
mg._prior_dev = torch.zeros(1, device="cuda:0")
mg._prior_dev.fill_(mg.hyper("z_pres_prior_log_odds"))
mg.train_step_async(x, k)
torch.cuda.synchronize()
print("after eager step 0: params equal", torch.equal(me.params.flat, mg.params.flat),
      "grad equal", torch.equal(me.params.grad, mg.params.grad), flush=True)
snap = {n: getattr(mg._ws, n).clone() for n in ("r", "mu", "Gx", "h", "eps_x")}
p0, g0 = mg.params.flat.clone(), mg.params.grad.clone()
X, K = mg._prep(x, k)
mg._capture(X, K, None)
torch.cuda.synchronize()
print("capture changed params", not torch.equal(p0, mg.params.flat), "grad",
      not torch.equal(g0, mg.params.grad),
      {n: not torch.equal(v, getattr(mg._ws, n)) for n, v in snap.items()}, flush=True)

"""One rank of tests/test_dp_gloo.py (run as a subprocess; gloo on CPU).

Computes the CPU restatement's gradient on this rank's contiguous shard with
the model's data-parallel loss scaling, reduces it with the product helper
mog_air.parallel.allreduce_grads, and rank 0 saves the result."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mog_air import parallel  # noqa: E402
from oracle import air_oracle as ao  # noqa: E402
from oracle import air_torch as at  # noqa: E402

B = 8


def cfg_for(batch):
    return ao.AirConfig(batch=batch, max_steps=3, scale_prior_variance=0.05,
                        z_pres_prior_log_odds=-0.01)


def inputs():
    cfg = cfg_for(B)
    P = ao.init_params(cfg, seed=41, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=42)
    x, k = ao.synthetic_canvases(B, seed=43)
    return P, nz, x, k


def grads(P, nz, x, k, lo, hi, scale):
    cfg = cfg_for(hi - lo)
    Pt = at.to_torch(P, requires_grad=True)
    noise = {n: torch.tensor(v[:, lo:hi], dtype=torch.float64) for n, v in nz.items()}
    out = at.air_forward(cfg, Pt, noise, torch.tensor(x[lo:hi], dtype=torch.float64),
                         torch.tensor(k[lo:hi]), z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                         fixed_steps=True)
    (out["loss"] * scale).backward()
    return torch.cat([Pt[n].grad.reshape(-1) for n in sorted(Pt)])


# ---- AIR-ASR: the loop predicate and the margin's batch mean are global ----
BA = 6


def asr_inputs():
    from oracle import asr_oracle as so
    cfg = so.AsrConfig(batch=BA, max_steps=4, constrains_num=(1, 3), constrains_num_gamma=0.5,
                       constrains_margin_gamma=100.0, constrains_num_element_gamma=10.0,
                       constrains_bbox_gamma=1.0, constrains_sharesize_gamma=0.3,
                       constrains_area_gamma=0.2, constrains_area_minmax=(17.0, 23.0),
                       stopping_threshold=0.5, z_pres_temperature=1.0)  # shards exit at 3 and 2
    P = so.init_params(cfg, seed=51, bias_scale=0.05)
    nz = so.make_noise(cfg, seed=52)
    x, _ = ao.synthetic_canvases(BA, seed=53)
    G = np.random.default_rng(54).standard_normal((BA, cfg.canvas_size ** 2)) * 0.01
    return cfg, P, nz, x, G


def asr_grads(cfg, P, nz, x, G, lo, hi, live_reduce=None, zsum_reduce=None):
    import dataclasses

    from oracle import asr_torch as st
    c = dataclasses.replace(cfg, batch=hi - lo)
    Pt = {n: torch.tensor(v, dtype=torch.float64, requires_grad=True) for n, v in P.items()}
    noise = {n: v[:, lo:hi] for n, v in nz.items()}
    out = st.asr_forward(c, Pt, noise, torch.tensor(x[lo:hi], dtype=torch.float64),
                         canvas_cotangent=torch.tensor(G[lo:hi]), live_reduce=live_reduce,
                         zsum_reduce=zsum_reduce, global_batch=cfg.batch)
    out["loss"].backward()
    g = torch.cat([(Pt[n].grad if Pt[n].grad is not None else torch.zeros_like(Pt[n])).reshape(-1)
                   for n in sorted(Pt)])
    return g, float(out["loss"].detach()), int(out["T"])


class _ShardModel:
    """Stand-in carrying the hook attributes parallel.attach installs on the
    HIP ASR model (same lambdas, here on CPU tensors over gloo)."""
    grad_world = 1
    zsum_hook = None
    live_hook = None


def asr_main(out_path):
    rank, world = dist.get_rank(), dist.get_world_size()
    cfg, P, nz, x, G = asr_inputs()
    lo, hi = parallel.shard(BA, rank, world)
    m = _ShardModel()
    m.grad_world = world
    parallel.attach(m)
    live = torch.zeros(cfg.max_steps + 1, dtype=torch.float64)
    step = [0]

    def live_reduce(flag):  # the model's live[t + 1] slot, reduced by its hook
        t = step[0]
        step[0] += 1
        live[t + 1] = 1.0 if flag else 0.0
        m.live_hook(live, t)
        return live[t + 1].item() > 0

    def zsum_reduce(zs):
        m.zsum_hook(zs)
        return zs

    g, loss, T = asr_grads(cfg, P, nz, x, G, lo, hi, live_reduce, zsum_reduce)
    m.grad_reducer.launch(g)
    m.grad_reducer.wait()
    lt = torch.tensor([loss], dtype=torch.float64)
    dist.all_reduce(lt)  # shard losses add up to the full-batch loss (margin counted per rank)
    if rank == 0:
        np.savez(out_path, g=g.numpy(), loss=lt.numpy(), T=np.array([T]))


def main():
    out_path = sys.argv[1]
    torch.set_num_threads(1)
    dist.init_process_group("gloo")
    try:
        if len(sys.argv) > 2 and sys.argv[2] == "asr":
            asr_main(out_path)
            return
        rank, world = dist.get_rank(), dist.get_world_size()
        P, nz, x, k = inputs()
        lo, hi = parallel.shard(B, rank, world)
        # loss-mean over the local shard x B_local / B_global (grad_world scaling)
        g = grads(P, nz, x, k, lo, hi, (hi - lo) / B)
        parallel.allreduce_grads(g)
        if rank == 0:
            np.save(out_path, g.numpy())
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

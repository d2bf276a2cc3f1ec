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


def main():
    out_path = sys.argv[1]
    torch.set_num_threads(1)
    dist.init_process_group("gloo")
    try:
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

"""One rank of tests/test_gpu_dp.py: the HIP AIR / AIR-ASR model on cuda:0
with a gloo process group (several ranks share the one GPU of a test box;
the RCCL path is the same code with backend "nccl").  Each rank runs its
contiguous shard of the batch through ``compute_gradients`` with
``parallel.attach`` installed (bucketed async all-reduce, global loop
predicate, ASR batch-mean hook) and saves what it saw.

Kinds: air / asr (13 / 11 images: odd shards, the per-step VAE path),
air64 / air64b (128 images, 64-row shards, fp32 / bf16: the batched T*B-row
VAE; below AIRModel.SIDE_MIN_BATCH every launch stays on the main stream)
and air1k / asr1k (2,048 images, 1,024 per rank, AIR without ``-ap`` as
bench.py runs it, and AIR-ASR: from SIDE_MIN_BATCH the VAE weight gradients
fork to the side stream and the main stream joins them (vae_done) before the
glimpse bucket's all-reduce -- air_model.py _vae_weight_grads_async /
_backward_body; the x3 weight gradients and the pre-split x-rows gradient
run at these sizes too).

Kind rccl1: ONE rank over RCCL (backend "nccl" on the HIP device; RCCL
refuses two ranks on one GPU, so a one-GPU box can only run it at world 1),
with the reducer and the global loop-flag hook installed by hand (attach
installs nothing at world 1): the bucketed async all-reduces and the MAX
all-reduce of the live flag go through RCCL on the device exactly as on an
8-GPU node, and the gradient must equal the no-reducer run bit for bit.

usage: gpu_dp_worker.py <out_prefix> air|asr|air64|air64b|air1k|asr1k|rccl1"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from mog_air import parallel  # noqa: E402

DEV = "cuda:0"


BATCH = {"air": 13, "asr": 11, "air64": 128, "air64b": 128, "rccl1": 128, "air1k": 2048,
         "asr1k": 2048}


def air_case(batch=13, num_prior=(1, 3)):
    from oracle import air_oracle as ao
    cfg = ao.AirConfig(batch=batch, max_steps=3, train=True, num_prior=num_prior,
                       scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01)
    P = ao.init_params(cfg, seed=71, bias_scale=0.05)
    nz = ao.make_noise(cfg, seed=72)
    x, k = ao.synthetic_canvases(cfg.batch, seed=73)
    G = (np.random.default_rng(74).standard_normal((cfg.batch, 2500)) * 0.01).astype(np.float32)
    return cfg, P, nz, x, k, G


def air_model(cfg, P, world, scope, precision="fp32"):
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, canvas_size=cfg.canvas_size,
                 scale_prior_variance=cfg.scale_prior_variance,
                 z_pres_prior_log_odds=cfg.z_pres_prior_log_odds,
                 z_pres_temperature=cfg.z_pres_temperature,
                 stopping_threshold=cfg.stopping_threshold,
                 vae_likelihood_std=cfg.vae_likelihood_std, learning_rate=1e-4,
                 gradient_clipping_norm=1.0, cnn=False, train=True, num_prior=cfg.num_prior,
                 scope=scope, device=DEV, grad_world=world, precision=precision)
    m.params.load_dict(P)
    return m


def asr_case(batch=11):
    from oracle import air_oracle as ao
    from oracle import asr_oracle as so
    cfg = so.AsrConfig(batch=batch, max_steps=4, constrains_num=(1, 3), constrains_num_gamma=0.5,
                       constrains_margin_gamma=100.0, constrains_num_element_gamma=10.0,
                       constrains_bbox_gamma=1.0, constrains_sharesize_gamma=0.3,
                       constrains_area_gamma=0.2, constrains_area_minmax=(17.0, 23.0),
                       stopping_threshold=0.5, z_pres_temperature=1.0)
    P = so.init_params(cfg, seed=81, bias_scale=0.05)
    nz = so.make_noise(cfg, seed=82)
    x, k = ao.synthetic_canvases(cfg.batch, seed=83)
    G = (np.random.default_rng(84).standard_normal((cfg.batch, 2500)) * 0.01).astype(np.float32)
    return cfg, P, nz, x, k, G


def asr_model(cfg, P, world, scope):
    from mog_air.asr_model import AIRModel
    m = AIRModel(max_steps=cfg.max_steps, max_digits=cfg.max_steps, canvas_size=cfg.canvas_size,
                 vae_likelihood_std=cfg.vae_likelihood_std, z_pres_prior_log_odds=-0.01,
                 z_pres_temperature=cfg.z_pres_temperature,
                 stopping_threshold=cfg.stopping_threshold, learning_rate=1e-4,
                 gradient_clipping_norm=1.0, cnn=False, train=True, scope=scope,
                 constrains_num=list(cfg.constrains_num),
                 constrains_num_gamma=cfg.constrains_num_gamma,
                 constrains_margin_gamma=cfg.constrains_margin_gamma,
                 constrains_num_element_gamma=cfg.constrains_num_element_gamma,
                 constrains_bbox_gamma=cfg.constrains_bbox_gamma,
                 constrains_sharesize_gamma=cfg.constrains_sharesize_gamma,
                 constrains_area_gamma=cfg.constrains_area_gamma,
                 constrains_area_minmax=list(cfg.constrains_area_minmax),
                 fix_steps=cfg.fix_steps, device=DEV, grad_world=world)
    m.params.load_dict(P)
    return m


def run(kind, lo, hi, world, scope, attach=True):
    """compute_gradients on images [lo, hi) of the case; returns a dict."""
    if kind.startswith("asr"):
        cfg, P, nz, x, k, G = asr_case(BATCH[kind])
        m = asr_model(cfg, P, world, scope)
    else:
        cfg, P, nz, x, k, G = air_case(BATCH[kind], None if kind == "air1k" else (1, 3))
        m = air_model(cfg, P, world, scope, "bf16" if kind == "air64b" else "fp32")
    reducer = None
    if attach and world > 1:
        reducer = parallel.attach(m, global_steps=True)
        reducer.log = []
    if attach and kind == "rccl1":  # world 1 over RCCL: the hooks by hand
        reducer = parallel.GradReducer()
        reducer.log = []
        m.grad_reducer = reducer
        m.live_hook = lambda live, t: dist.all_reduce(live[t + 1:t + 2], op=dist.ReduceOp.MAX)
    noise = {n: torch.as_tensor(np.ascontiguousarray(v[:, lo:hi])).to(DEV) for n, v in nz.items()}
    grads = m.compute_gradients(x[lo:hi], k[lo:hi], noise=noise,
                                canvas_cotangent=torch.as_tensor(G[lo:hi]).to(DEV),
                                global_batch=cfg.batch)
    names = sorted(grads)
    out = {"g": np.concatenate([grads[n].reshape(-1) for n in names]),
           "T": np.array([m.executed_steps]),
           "digits": m.rec_num_digits.cpu().numpy(),
           "loss_b": m.per_image_loss.cpu().numpy(),
           "mean": np.array([m.loss])}
    if reducer is not None:
        out["buckets"] = np.array(reducer.log)
    if kind.startswith("asr"):
        out["margin"] = m._ws.margin.cpu().numpy()
    out["batched"] = np.array([int(getattr(m, "_batched_vae", lambda b: False)(hi - lo))])
    # the side-stream fork of the VAE weight gradients (AIRModel.SIDE_MIN_BATCH)
    out["side"] = np.array([int(hi - lo >= m.SIDE_MIN_BATCH)])
    return out


def main():
    prefix, kind = sys.argv[1], sys.argv[2]
    if kind == "rccl1":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", device_id=torch.device(DEV))
    else:
        dist.init_process_group("gloo")
    try:
        rank, world = dist.get_rank(), dist.get_world_size()
        n = BATCH[kind]
        lo, hi = parallel.shard(n, rank, world)
        res = run(kind, lo, hi, world, scope=f"dp_{kind}_{rank}")
        np.savez(f"{prefix}_{rank}.npz", lo=np.array([lo]), hi=np.array([hi]), **res)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""AIR train-step throughput on MI355X (BASELINE.json metric):
images/sec/node for the AIR train step, Multi-MNIST-like 50x50 synthetic
canvases, max_steps = 3 (all 3 steps always computed), data-parallel over N
GPUs (one process per GPU, RCCL all-reduce of the flat gradient buffer).

A step = forward (LSTM, heads, STN read, glimpse VAE, STN write, canvas) +
backward + gradient all-reduce + per-tensor clip + TF Adam, on one batch of
synthetic input already resident in HBM.  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "mog-asr_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec/node AIR train step, Multi-MNIST 50×50 max_steps=3, 1/2/4/8 GPU"
# peaks from /opt/skills/guides/MI355X_MICROARCH.md (dense, spec)
HBM_PEAK_GBS = 8000.0
FP32_MFMA_PEAK_TFLOPS = 157.3
BF16_MFMA_PEAK_TFLOPS = 2500.0
PMC_SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")
PRECISION = "bf16"  # set from --precision in main()


def kernel_work(name, B, C2=2500, H=256, T=3):
    """Algorithmic work per launch of a tagged kernel: (bound, amount, unit,
    peak).  Per-unit figures in DESIGN.md §Roofline."""
    if name == "lstm_x_projection":          # Gx = X Wx, [B,C2] x [C2,4H], fp32 MFMA
        return "mfma", 2.0 * B * C2 * 4 * H / 1e12, "TFLOP/s", FP32_MFMA_PEAK_TFLOPS
    if name == "lstm_x_projection_grad":     # dWx = X^T dGsum (bf16 MFMA in the bf16 config)
        peak = BF16_MFMA_PEAK_TFLOPS if PRECISION == "bf16" else FP32_MFMA_PEAK_TFLOPS
        return "mfma", 2.0 * B * C2 * 4 * H / 1e12, "TFLOP/s", peak
    if name == "stn_vae_step":               # 30,024 B per image-step
        return "hbm", B * 30024 / 1e9, "GB/s", HBM_PEAK_GBS
    return None


def roofline(events, B):
    """Dominant tagged kernel (largest total time in the timed region)."""
    best = None
    for name, evs in events.items():
        durs = [a.elapsed_time(b) * 1e-3 for a, b in evs]  # seconds
        tot = sum(durs)
        if kernel_work(name, B) is None:
            continue
        if best is None or tot > best[1]:
            best = (name, tot, durs)
    if best is None:
        return None
    name, tot, durs = best
    bound, amount, unit, peak = kernel_work(name, B)
    avg = tot / len(durs)
    achieved = amount / avg
    traffic = None
    try:
        with open(PMC_SUMMARY) as f:
            pmc = json.load(f)
        traffic = pmc.get(name, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    return {"kernel": name, "bound": bound, "achieved": achieved, "peak": peak, "unit": unit,
            "frac": achieved / peak, "traffic": traffic, "launches": len(durs),
            "avg_launch_us": avg * 1e6}


def fused_step_roofline(batch: int, launches: int, dev):
    """North-star measurement (BASELINE.json): the fused STN-read -> glimpse VAE
    -> STN-write step kernel alone at `batch` images on this GPU, inputs
    resident in HBM (theta / masks from one forward pass of a bf16 model on
    the same synthetic canvases).  Timed with HIP events on the stream the
    kernel is launched on; algorithmic bytes per image-step = 30,024
    (SURVEY.md §8 D.3)."""
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=3, cnn=False, train=True, device=dev, precision="bf16",
                 scale_prior_variance=0.05, z_pres_prior_log_odds=-0.01,
                 scope="roofline%d" % batch, seed=77, noise_seed=78)
    x, k = synthetic(batch, 4321)
    X = torch.from_numpy(x).to(dev)
    K = torch.from_numpy(k).to(dev)
    m.infer(X, K)
    ws = m._ws
    for t in range(3):
        m._step_fused(X, ws, t, 0.3)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    evs = []
    for i in range(launches):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        m._step_fused(X, ws, i % 3, 0.3)
        e1.record(s)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    durs = [a.elapsed_time(b) * 1e-3 for a, b in evs]
    avg = sum(durs) / len(durs)
    achieved = batch * 30024 / 1e9 / avg
    traffic = None
    try:
        with open(PMC_SUMMARY) as f:
            traffic = json.load(f).get("stn_vae_step_b%d" % batch, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        pass
    out = {"kernel": "stn_vae_step", "batch": batch, "bound": "hbm", "achieved": achieved,
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
           "traffic": traffic, "launches": launches, "avg_launch_us": avg * 1e6,
           "algorithmic_bytes_per_launch": batch * 30024}
    del m, ws
    torch.cuda.empty_cache()
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch (configs[1])")
    ap.add_argument("--max-steps", type=int, default=3)
    ap.add_argument("--precision", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--roofline-batch", type=int, default=65536,
                    help="batch of the stand-alone fused-step roofline run (0: skip)")
    ap.add_argument("--roofline-launches", type=int, default=30)
    return ap.parse_args()


def synthetic(batch, seed):
    rng = np.random.default_rng(seed)
    imgs = np.zeros((batch, 50, 50), np.float32)
    ks = rng.integers(1, 4, size=batch)
    for b in range(batch):
        for _ in range(ks[b]):
            s = int(rng.integers(17, 24))
            y, x = (int(v) for v in rng.integers(0, 50 - s + 1, 2))
            g = rng.uniform(0, 1, (s, s)).astype(np.float32)
            g = np.where(rng.uniform(size=(s, s)) < 0.35, g, 0.0)
            imgs[b, y:y + s, x:x + s] += np.where(g >= 0.05, g, 0.0)
    return np.clip(imgs, 0, 1).reshape(batch, 2500), ks.astype(np.int32)


def cpu_baseline(seconds: float):
    """CPU restatement (oracle/air_torch.py, fp32), batch 64, T=3, on this host."""
    from oracle import air_oracle as ao
    from oracle import air_torch as at
    cores = min(16, os.cpu_count() or 1)
    torch.set_num_threads(cores)
    cfg = ao.AirConfig(batch=64, max_steps=3, scale_prior_variance=0.05)
    P = at.to_torch(ao.init_params(cfg), dtype=torch.float32, requires_grad=True)
    m = {k: torch.zeros_like(v) for k, v in P.items()}
    v = {k: torch.zeros_like(v_) for k, v_ in P.items()}
    x, k = synthetic(64, 99)
    X, Tg = torch.tensor(x), torch.tensor(k)
    times = []
    t_end = time.perf_counter() + seconds
    it = 0
    while time.perf_counter() < t_end or it < 4:
        nz = at.to_torch(ao.make_noise(cfg, seed=it), dtype=torch.float32)
        t0 = time.perf_counter()
        at.train_step(cfg, P, m, v, it + 1, nz, X, Tg, prior_lo=9.21)
        times.append(time.perf_counter() - t0)
        it += 1
    med = float(np.median(times[2:] if len(times) > 4 else times))
    return {"value": 64.0 / med, "unit": "images/sec", "cores": cores, "kind": "port",
            "sample": f"{len(times)} train steps of batch 64 (T=3) of the fp32 torch CPU "
                      f"restatement (not TF-1.12); median step {med * 1e3:.1f} ms"}


def main():
    args = parse()
    global PRECISION
    PRECISION = args.precision
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)
    from mog_air.air_model import AIRModel

    B, T = args.batch, args.max_steps
    model = AIRModel(max_steps=T, max_digits=T, rnn_units=256, canvas_size=50, windows_size=28,
                     scale_prior_mean=-1.0, scale_prior_variance=0.05,
                     vae_likelihood_std=0.3, z_pres_prior_log_odds=-0.01,
                     z_pres_temperature=1.0, stopping_threshold=0.99, learning_rate=1e-4,
                     gradient_clipping_norm=1.0, cnn=False, train=True, scope="bench",
                     annealing_schedules={"z_pres_prior_log_odds": {
                         "init": 10000.0, "min": 1e-9, "factor": 0.1, "iters": 3000,
                         "staircase": False, "log": True}},
                     device=dev, seed=1235, noise_seed=1235 + rank, grad_world=world,
                     precision=args.precision)
    if world > 1:
        from mog_air import parallel
        parallel.attach(model)  # one RCCL all-reduce of the flat gradient per step
    x, k = synthetic(B, 1234 + rank)
    X = torch.from_numpy(x).to(dev)
    K = torch.from_numpy(k).to(dev)
    for _ in range(args.warmup):
        model.train_step_async(X, K)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    model.kernel_events = {}
    t0 = time.perf_counter()
    for _ in range(args.steps):
        model.train_step_async(X, K)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    roof = roofline(model.kernel_events, B)
    model.kernel_events = None
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    executed = model.executed_steps
    loss = model.loss
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision, "data": "synthetic",
            "config": {"workload": "AIR baseline train step (configs[1] batch)",
                       "model": "AIR (LSTM 256, VAE 784-512-256-50, heads 64)",
                       "global_batch": B * world, "per_gpu_batch": B, "canvas": "50x50",
                       "max_steps": T, "data_dependent_steps_would_be": executed,
                       "parallelism": f"dp{world}", "loss_last": loss},
            "roofline": roof,
        }
        if args.roofline_batch > 0 and world == 1 and args.precision == "bf16":
            out["fused_step_roofline"] = fused_step_roofline(args.roofline_batch,
                                                             args.roofline_launches, dev)
        if args.cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

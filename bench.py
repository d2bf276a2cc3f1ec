"""AIR train-step throughput on MI355X (BASELINE.json metric):
images/sec/node for the AIR train step, Multi-MNIST-like 50x50 synthetic
canvases, max_steps = 3 (all 3 steps always computed), data-parallel over N
GPUs (one process per GPU, RCCL all-reduce of the gradient in buckets
overlapped with the backward).

A step = forward (LSTM, heads, STN read, glimpse VAE, STN write, canvas) +
backward + gradient all-reduce + per-tensor clip + TF Adam, on one batch of
synthetic input already resident in HBM.  Prints ONE JSON line on rank 0.

Headline ``value``: the train step at the REFERENCE's precision (fp32
arithmetic throughout, air/vae.py:5-48, air/air_model.py:533-588), per-GPU
batch 8192 (the batch configs[1] is quoted on).  Extra keys on the same line
(rank 0, N = 1 only): ``configs_1_bf16`` (configs[1] itself: bf16 VAE, fp32
elsewhere), ``config_1_batch64_fp32`` (the reference's own batch of 64),
``fp32_step_roofline`` (the same step at reference precision against the fp32
MFMA roof), ``fused_step_roofline`` / ``fused_step_roofline_c64`` (the north-star fused
STN-read -> VAE -> STN-write kernel at B = 65,536, C = 50 and 64, training form),
``fused_step_roofline_fwd`` (its forward-only form, C = 50),
``configs_4_asr_bbox_{fp32,bf16}`` (configs[4] on one GPU), ``roofline`` (the
dominant kernel group of the headline step: every tagged launch priced, the
largest total time wins) and ``cpu_baseline``.  HBM-bound lines also carry
``frac_of_measured_copy``: achieved bytes over a measured float4 copy
(``copy_bandwidth``).

``python bench.py --gpus N`` without a torch.distributed launcher starts the
N ranks itself (fresh child processes, before anything touches the GPU).
"""
import argparse
import json
import os
import socket
import subprocess
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


def fused_bytes_per_image_step(C2: int, x_bytes: int = 4) -> int:
    """read x, read+write the running canvas (fp32), 24 B of
    per-image scalars: 30,024 B at C = 50, 49,176 B at C = 64."""
    return C2 * x_bytes + 2 * C2 * 4 + 24


# what each tagged kernel group is (the roofline's "kernel" names the group)
KERNEL_NAMES = {
    "lstm_x_projection": "gemm_f32 (LDS-DMA, bit-exact fp32 chain): Gx = X Wx",
    "lstm_x_projection_grad": "gemm_x3p_tn: dWx = X^T dGsum (bf16 cores; fp32: 3-piece split)",
    "stn_vae_step": "stn_vae_step_kernel (fused bf16 STN read + VAE + STN write)",
    "stn_vae_step_all": "stn_vae_step_kernel (fused bf16, all T steps' rows)",
    "stn_vae_step_f32_all": "stn_vae_step_f32_kernel (fused fp32 STN read + VAE + STN write)",
    "vae_wgrad_x3": "gemm_x3_tn_kernel<false,3>: VAE weight gradients, fp32 operands split "
                    "in-kernel (bf16 cores; priced on fp32 flops)",
    "vae_dgrad_x3": "gemm_x3_nt_kernel: VAE input gradients dY W^T (bf16 cores, 3-piece)",
    "vae_dgrad_f32": "gemm_f32 transB: VAE input gradients (fp32 chain)",
    "wgrad_f32": "gemm_f32 transA split-K: heads / small VAE weight gradients",
    "rec_wgrad_x3": "gemm_x3_tn_kernel<false,3>: LSTM recurrent-rows weight gradient (bf16 cores, "
                    "3-piece)",
    "wgrad_bf16": "gemm_bf16 TN: bf16 VAE weight gradients",
    "vae_wgrad_bf16": "wgrad_tn_bf16_kernel (+ its split reduction): the seven bf16 VAE weight "
                      "gradients in one launch",
    "heads_wgrad_x3": "wgrad_tn_x3_kernel: the five heads' hidden-layer weight gradients, grouped "
                      "(bf16 cores, 3-piece, deterministic)",
    "wgrad_group": "wgrad_group_kernel: every fp32-chain weight gradient of a small-batch step, "
                   "one launch",
    "stn_write_bwd": "stn_bwd_kernel: STN write backward (through the output sigmoid)",
    "stn_read_bwd": "stn_bwd_kernel: STN read backward (dtheta only)",
}
PEAKS = {"fp32": FP32_MFMA_PEAK_TFLOPS, "bf16": BF16_MFMA_PEAK_TFLOPS}


def kernel_work(name, B, precision, C2=2500, H=256, T=3):
    """Algorithmic work of one launch of a tag the model records without its
    own work figure: (bound, amount in flops or bytes, peak key).  Per-unit
    figures in DESIGN.md §4.1."""
    if name == "lstm_x_projection":          # Gx = X Wx, [B,C2] x [C2,4H], fp32 MFMA
        return "mfma", 2.0 * B * C2 * 4 * H, "fp32"
    if name == "stn_vae_step":
        return "hbm", B * fused_bytes_per_image_step(C2), None
    if name == "stn_vae_step_all":           # all T steps' rows in one launch
        return "hbm", T * B * fused_bytes_per_image_step(C2), None
    if name == "stn_vae_step_f32_all":       # the fp32 fused step over T*B rows: MFMA-bound
        return "mfma", T * B * vae_chain_flops_per_image(), "fp32"
    return None


def pmc_field(tag, field):
    """A field of profiles/pmc_summary.json's entry for `tag` (the rocprofv3
    kernel-trace / PMC figures of the same kernel in the same workload)."""
    try:
        with open(PMC_SUMMARY) as f:
            return json.load(f).get(tag, {}).get(field)
    except (OSError, ValueError):
        return None


def pmc_traffic(tag):
    return pmc_field(tag, "hbm_bytes_per_launch")


def roofline(events, B, precision):
    """The dominant kernel group of the timed step: every tagged launch
    (AIRModel._timed: one kernel launch each, on the stream it runs on, with
    its algorithmic flops or bytes), grouped by tag.  achieved = the group's
    algorithmic work / its summed launch durations; peak: the fp32 or bf16
    dense MFMA peak, or 8 TB/s of HBM.  The fp32 gradients on the bf16 matrix
    cores (three-piece splits, tag work ending in "x3") are priced on their
    fp32 flops against the fp32 peak, with the six bf16 products they issue
    against the bf16 peak beside it (``x3_bf16_products_frac``).

    Only main-stream groups can be the line's roofline: a side-stream
    launch's HIP events also count the time its first workgroups wait for
    CUs that the main stream's kernel holds, so its event time is not its
    kernel time (rocprofv3's kernel trace ranks the groups by kernel time;
    DESIGN.md §4.9).  The largest main-stream total wins; every group,
    side-stream ones flagged, is listed under ``launches_priced``."""
    rows = []
    for name, evs in events.items():
        durs, amount, bound, peak_key, x3, side = [], 0.0, None, None, False, False
        for e0, e1, work, on_side in evs:
            if work is None:
                work = kernel_work(name, B, precision)
            if work is None:
                continue
            bound, a, peak_key = work[:3]
            x3 = len(work) > 3 and work[3] == "x3"
            side = side or on_side
            durs.append(e0.elapsed_time(e1) * 1e-3)  # seconds
            amount += a
        if not durs:
            continue
        total = sum(durs)
        extra = {}
        if bound == "mfma":
            achieved, unit, peak = amount / total / 1e12, "TFLOP/s", PEAKS[peak_key]
            if x3:
                extra["x3_bf16_products_frac"] = 6.0 * achieved / BF16_MFMA_PEAK_TFLOPS
        else:
            achieved, unit, peak = amount / total / 1e9, "GB/s", HBM_PEAK_GBS
            extra["frac_of_measured_copy"] = achieved / copy_bandwidth(torch.device(
                "cuda", torch.cuda.current_device()))
        rows.append({"kernel": name, "what": KERNEL_NAMES.get(name, name), "bound": bound,
                     "stream": "side" if side else "main",
                     "achieved": achieved, "peak": peak, "unit": unit, "frac": achieved / peak,
                     **extra,
                     "traffic": pmc_traffic(f"{name}_{precision}_b{B}"),
                     "profiled_avg_us": pmc_field(f"{name}_{precision}_b{B}", "profiled_avg_us"),
                     "launches": len(durs), "avg_launch_us": total / len(durs) * 1e6,
                     "total_us": total * 1e6,
                     "algorithmic_per_launch": amount / len(durs),
                     "algorithmic_unit": "flop" if bound == "mfma" else "bytes"})
    if not rows:
        return None
    rows.sort(key=lambda r: -r["total_us"])
    main = [r for r in rows if r["stream"] == "main"] or rows
    out = dict(main[0])
    out["launches_priced"] = [{k: r[k] for k in ("kernel", "stream", "frac", "avg_launch_us",
                                                 "total_us", "launches", "unit", "achieved")}
                              for r in rows]
    return out


def synthetic(batch, seed, canvas=50, counts=None, side=None):
    """Multi-MNIST-like canvases: 1-3 glyphs of side
    U{17..23} (scaled with the canvas), ~35 % inked at U(0,1), < 0.05 -> 0.
    counts: objects per image drawn uniformly from this tuple (default 1..3);
    side: (lo, hi) glyph side, hi exclusive (the bbox datasets: 11..15)."""
    rng = np.random.default_rng(seed)
    imgs = np.zeros((batch, canvas, canvas), np.float32)
    if counts is None:
        ks = rng.integers(1, 4, size=batch)
    else:
        ks = np.asarray(counts)[rng.integers(0, len(counts), size=batch)]
    lo, hi = side if side is not None else ((17, 24) if canvas == 50 else (22, 31))
    for b in range(batch):
        for _ in range(ks[b]):
            s = int(rng.integers(lo, hi))
            y, x = (int(v) for v in rng.integers(0, canvas - s + 1, 2))
            g = rng.uniform(0, 1, (s, s)).astype(np.float32)
            g = np.where(rng.uniform(size=(s, s)) < 0.35, g, 0.0)
            imgs[b, y:y + s, x:x + s] += np.where(g >= 0.05, g, 0.0)
    return np.clip(imgs, 0, 1).reshape(batch, canvas * canvas), ks.astype(np.int32)


def make_model(precision, dev, world, rank, scope, canvas=50):
    from mog_air.air_model import AIRModel
    return AIRModel(max_steps=3, max_digits=3, rnn_units=256, canvas_size=canvas, windows_size=28,
                    scale_prior_mean=-1.0, scale_prior_variance=0.05,
                    vae_likelihood_std=0.3, z_pres_prior_log_odds=-0.01,
                    z_pres_temperature=1.0, stopping_threshold=0.99, learning_rate=1e-4,
                    gradient_clipping_norm=1.0, cnn=False, train=True, scope=scope,
                    annealing_schedules={"z_pres_prior_log_odds": {
                        "init": 10000.0, "min": 1e-9, "factor": 0.1, "iters": 3000,
                        "staircase": False, "log": True}},
                    device=dev, seed=1235, noise_seed=1235 + rank, grad_world=world,
                    precision=precision)


# configs[4] (train_air_pr.py -dn 3 -ds bbox20k -gb 1 -gs 10 -ga 20,
# train_air_pr.py:40-61,77-98): three objects of side 11..15, fix_steps 3,
# bbox / size / area regularisers
ASR_BBOX = dict(constrains_num=[3], constrains_margin_gamma=0.0,
                constrains_num_element_gamma=0.0, constrains_bbox_gamma=1.0,
                constrains_sharesize_gamma=10.0, constrains_area_gamma=20.0,
                constrains_area_minmax=[11, 15], fix_steps=3)
ASR_BBOX_DATA = dict(counts=(3,), side=(11, 16))


def make_asr_model(precision, dev, scope, canvas=50, world=1, rank=0, cfg=None):
    """configs[2]: train_air_pr.py -dn 13 -gm 100 -gne 10 (AIR-ASR with the
    number regularisers: objects {1, 3}, margin gamma 100, element gamma 10,
    z_pres temperature 0.1, MAX_STEPS 6; train_air_pr.py:63-82); cfg=ASR_BBOX
    for configs[4]."""
    from mog_air.asr_model import AIRModel as AsrModel
    kw = dict(constrains_num=[1, 3], constrains_margin_gamma=100.0,
              constrains_num_element_gamma=10.0, constrains_area_minmax=[17, 23])
    kw.update(cfg or {})
    return AsrModel(None, None, max_steps=6, max_digits=6, rnn_units=256, canvas_size=canvas,
                    windows_size=28, vae_latent_dimensions=50, vae_recognition_units=(512, 256),
                    vae_generative_units=(256, 512), fix_scale_distribution=True,
                    vae_prior_mean=0.0, vae_prior_variance=1.0, vae_likelihood_std=0.0,
                    scale_hidden_units=64, shift_hidden_units=64, z_pres_hidden_units=64,
                    z_pres_prior_log_odds=-0.01, z_pres_temperature=0.1, stopping_threshold=0.9,
                    learning_rate=1e-4, gradient_clipping_norm=1.0, cnn=False, train=True,
                    scope=scope, annealing_schedules={}, device=dev, seed=1235,
                    noise_seed=1235 + rank, grad_world=world, precision=precision, **kw)


def timed_train(precision, B, steps, warmup, dev, world=1, rank=0, events=False, scope="bench",
                model=None, canvas=50, data=None, graph=False):
    """Time `steps` train steps of batch B per rank (after `warmup`); returns
    (seconds, model).  Barrier + synchronize on both sides; the caller takes
    the max over ranks.  data: synthetic() keywords (counts, side).  graph:
    the captured train step (AIRModel.train_step_graphed; one device)."""
    if model is None:
        model = make_model(precision, dev, world, rank, scope, canvas=canvas)
    if world > 1:
        from mog_air import parallel
        parallel.attach(model)  # bucketed RCCL all-reduce overlapped with the backward
    x, k = synthetic(B, 1234 + rank, canvas, **(data or {}))
    X = torch.from_numpy(x).to(dev)
    K = torch.from_numpy(k).to(dev)
    step = model.train_step_graphed if graph else model.train_step_async
    for _ in range(warmup):
        step(X, K, global_batch=B * world)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step(X, K, global_batch=B * world)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if events:
        # the roofline's per-launch HIP events over `steps` more steps of the
        # same model and batch (an event pair around each tagged launch costs
        # a few microseconds: the value's steps above run without them)
        model.kernel_events = {}
        for _ in range(steps):
            step(X, K, global_batch=B * world)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
    return el, model


_COPY_GBS = None


def copy_bandwidth(dev, gib: float = 1.0, launches: int = 20) -> float:
    """Measured device copy bandwidth (GB/s of bytes read + written): a
    float4 grid-stride copy (mog_copy_f4) of `gib` GiB, HIP events on the
    launch stream -- the yardstick SURVEY.md §8 D.3 asks for beside the
    8 TB/s spec.  Measured once per process."""
    global _COPY_GBS
    if _COPY_GBS is None:
        from mog_air import ops
        n = int(gib * (1 << 30)) // 4
        src = torch.ones(n, device=dev)
        dst = torch.empty(n, device=dev)
        for _ in range(3):
            ops._ops.copy_f4_(src, dst)
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(launches):
            ops._ops.copy_f4_(src, dst)
        e1.record(s)
        torch.cuda.synchronize()
        _COPY_GBS = 2.0 * n * 4 * launches / (e0.elapsed_time(e1) * 1e-3) / 1e9
        del src, dst
        torch.cuda.empty_cache()
    return _COPY_GBS


def fused_step_roofline(batch: int, launches: int, dev, canvas: int = 50, save: bool = True):
    """North-star measurement (BASELINE.json): the fused STN-read -> glimpse VAE
    -> STN-write step kernel alone at `batch` images on this GPU, inputs
    resident in HBM (theta / masks from one forward pass of a bf16 model on
    the same synthetic canvases).  Timed with HIP events on the stream the
    kernel is launched on; algorithmic bytes per image-step from SURVEY.md §8
    D.3 (30,024 at C = 50, 49,176 at C = 64).  save=True: the training form,
    which also writes the backward's saved activations (SAVED_BYTES per
    image-step on top); save=False: the forward-only form (evaluation)."""
    m = make_model("bf16", dev, 1, 0, "roofline%d_%d_%d" % (batch, canvas, save), canvas=canvas)
    m.noise_seed = 78
    x, k = synthetic(batch, 4321, canvas)
    X = torch.from_numpy(x).to(dev)
    K = torch.from_numpy(k).to(dev)
    m.infer(X, K)
    ws = m._ws
    for t in range(3):
        m._step_fused(X, ws, t, 0.3, save=save)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    evs = []
    for i in range(launches):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        m._step_fused(X, ws, i % 3, 0.3, save=save)
        e1.record(s)
        evs.append((e0, e1))
    torch.cuda.synchronize()
    durs = [a.elapsed_time(b) * 1e-3 for a, b in evs]
    avg = sum(durs) / len(durs)
    per = fused_bytes_per_image_step(canvas * canvas)
    achieved = batch * per / 1e9 / avg
    tag = "stn_vae_step_b%d" % batch + ("" if canvas == 50 else "_c%d" % canvas) + \
        ("" if save else "_fwd")
    copy = copy_bandwidth(dev)
    traffic = pmc_traffic(tag)
    out = {"kernel": "stn_vae_step", "mode": "train" if save else "forward-only",
           "batch": batch, "canvas": canvas, "bound": "hbm",
           "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": achieved / HBM_PEAK_GBS, "measured_copy_GBs": copy,
           "frac_of_measured_copy": achieved / copy,
           "traffic": traffic,
           "actual_traffic_GBs": traffic / avg / 1e9 if traffic else None,
           "launches": launches,
           "avg_launch_us": avg * 1e6, "algorithmic_bytes_per_launch": batch * per,
           "algorithmic_bytes_per_image_step": per}
    if save:
        out["saved_activation_bytes_per_image_step"] = SAVED_BYTES
    if canvas != 50:
        # the kernel stores only the window rows of each canvas part, so the
        # full-canvas read-modify-write of SURVEY §8 D.3 overstates its bytes
        # (at C = 64 the priced rate exceeds a measured copy): priced on the
        # bytes it moves (rocprofv3 FETCH + WRITE), or not at all
        out["algorithmic_frac_not_a_roofline"] = out.pop("frac")
        out.pop("frac_of_measured_copy")
        out["frac"] = traffic / avg / 1e9 / HBM_PEAK_GBS if traffic else None
        out["frac_basis"] = "actual HBM bytes (pmc_summary traffic) / launch time"
    del m, ws
    torch.cuda.empty_cache()
    return out


# bytes per image-step of the backward's saved activations the training form
# also writes: glimpse, a1, a2, d1, d2 (bf16), mu / logvar (fp32), z bf16 copy
SAVED_BYTES = 2 * (784 + 512 + 256 + 256 + 512) + 4 * 2 * 50 + 2 * 56


def vae_chain_flops_per_image(W2=784, R1=512, R2=256, Z=50, G1=256, G2=512) -> float:
    """Dense-layer flops of one glimpse VAE pass (vae.py:5-48): 2.21 MFLOP."""
    return 2.0 * (W2 * R1 + R1 * R2 + 2 * R2 * Z + Z * G1 + G1 * G2 + G2 * W2)


def fp32_step_roofline(batch: int, launches: int, dev):
    """SURVEY §8 D.3's fp32 step (STN read -> glimpse VAE -> STN write at
    reference precision) at `batch` images, priced against the fp32 MFMA roof
    (batch x 2.21 MFLOP; >= 919 us at 65,536): the fused fp32 step kernel
    (stn_vae_step_f32_kernel, bit-identical to the unfused sequence), one step
    over `batch` rows (AIRModel._vae_forward_all); timed with HIP events on the
    launch stream.  The unfused sequence (STN read, seven bit-exact fp32 GEMMs
    with fused epilogues, latent sample, STN write into canvas parts) is timed
    beside it as `unfused_us`."""
    from mog_air.air_model import AIRModel
    m = AIRModel(max_steps=1, max_digits=1, canvas_size=50, scale_prior_variance=0.05,
                 z_pres_prior_log_odds=-0.01, learning_rate=1e-4, gradient_clipping_norm=1.0,
                 cnn=False, train=True, scope="fp32roof%d" % batch, device=dev,
                 precision="fp32", seed=1235, noise_seed=79)
    x, k = synthetic(batch, 4322, 50)
    X = torch.from_numpy(x).to(dev)
    K = torch.from_numpy(k).to(dev)
    m.infer(X, K)
    ws = m._ws
    assert m._batched_vae(batch)
    fused = m.fused_f32

    def timed(n):
        for _ in range(2):
            m._vae_forward_all(X, ws, 0.3)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        evs = []
        for _ in range(n):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            m._vae_forward_all(X, ws, 0.3)
            e1.record(s)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        return sum(a.elapsed_time(b) * 1e-3 for a, b in evs) / len(evs)

    avg = timed(launches)
    unfused = None
    if fused:
        m.fused_f32 = False
        unfused = timed(max(2, launches // 2)) * 1e6
        m.fused_f32 = True
    flop = batch * vae_chain_flops_per_image()
    kern = ("stn_vae_step_f32 (fused fp32 STN read + VAE chain + STN write, bit-exact)" if fused
            else "fp32 STN read + VAE GEMM chain + STN write (unfused, bit-exact)")
    out = {"kernel": kern,
           "batch": batch, "bound": "mfma", "achieved": flop / avg / 1e12,
           "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": flop / avg / 1e12 / FP32_MFMA_PEAK_TFLOPS, "launches": launches,
           "avg_chain_us": avg * 1e6, "roof_us": flop / FP32_MFMA_PEAK_TFLOPS / 1e6,
           "flop_per_image": vae_chain_flops_per_image(), "unfused_us": unfused}
    del m, ws
    torch.cuda.empty_cache()
    return out


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch (configs[1])")
    ap.add_argument("--precision", default="fp32", choices=["bf16", "fp32"],
                    help="headline precision (fp32 = the reference's arithmetic)")
    ap.add_argument("--extras", type=int, default=1,
                    help="N = 1: also time configs[1] (bf16), batch 64, the fused-step rooflines")
    ap.add_argument("--cpu-baseline", type=int, default=1)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--roofline-batch", type=int, default=65536,
                    help="batch of the stand-alone fused-step roofline runs (0: skip)")
    ap.add_argument("--roofline-launches", type=int, default=30)
    ap.add_argument("--workload", default="air", choices=["air", "asr_bbox"],
                    help="air: the BASELINE.json metric (AIR train step); asr_bbox: configs[4] "
                         "(train_air_pr.py -dn 3 -ds bbox20k -gb 1 -gs 10 -ga 20), the data-"
                         "parallel ASR-bbox train step")
    return ap.parse_args()


def physical_cores():
    """(threads to use, physical cores of the node, logical CPUs available):
    one thread per physical core this process may run on, capped by the
    cgroup CPU quota when there is one."""
    cpus = sorted(os.sched_getaffinity(0))
    cores = set()
    for c in cpus:
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "core_id") as f1, open(base + "physical_package_id") as f2:
                cores.add((f2.read().strip(), f1.read().strip()))
        except OSError:
            cores.add(("?", str(c)))
    node = set()
    for c in range(os.cpu_count() or 1):
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            with open(base + "core_id") as f1, open(base + "physical_package_id") as f2:
                node.add((f2.read().strip(), f1.read().strip()))
        except OSError:
            node.add(("?", str(c)))
    use = len(cores)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, p = f.read().split()
        if q != "max":
            use = max(1, min(use, int(int(q) // int(p))))
    except (OSError, ValueError):
        pass
    return use, len(node), len(cpus)


def cpu_baseline(seconds: float):
    """CPU restatement (oracle/air_torch.py, fp32), batch 64, T=3, on this
    host, one torch thread per available physical core."""
    from oracle import air_oracle as ao
    from oracle import air_torch as at
    use, node_cores, logical = physical_cores()
    torch.set_num_threads(use)
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
    return {"value": 64.0 / med, "unit": "images/sec", "cores": use, "kind": "port",
            "node_physical_cores": node_cores, "logical_cpus_available": logical,
            "sample": f"{len(times)} train steps of batch 64 (T=3) of the fp32 torch CPU "
                      f"restatement (not TF-1.12), {use} threads; median step "
                      f"{med * 1e3:.1f} ms"}


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` outside torch.distributed.run: start N ranks as
    fresh processes (this parent never touches the GPU) and return the
    worst exit code.  Rank r drives GPU r."""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    # more ranks than GPUs (a rehearsal of the data-parallel path on a one-GPU
    # box): RCCL refuses two ranks on one device, so those ranks use gloo
    # (device_count() does not initialise the GPU in this parent)
    extra = {} if n <= torch.cuda.device_count() else {"MOG_DP_BACKEND": "gloo"}
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   HSA_ENABLE_IPC_MODE_LEGACY="0", **extra)
        procs.append(subprocess.Popen([sys.executable] + sys.argv, env=env))
    rcs = [p.wait() for p in procs]
    return max(rcs, key=abs)


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        # RCCL (one GPU per rank, as torch.distributed.run starts the ranks);
        # MOG_DP_BACKEND=gloo for ranks sharing a device (spawn_ranks sets it
        # when asked for more ranks than there are GPUs)
        ndev = torch.cuda.device_count()
        backend = os.environ.get("MOG_DP_BACKEND") or "nccl"
        local = local % max(ndev, 1)
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    B, T = args.batch, 3
    asr = args.workload == "asr_bbox"
    if asr:
        T = 6
        el, model = timed_train(args.precision, B, args.steps, args.warmup, dev, world, rank,
                                events=True, data=ASR_BBOX_DATA,
                                model=make_asr_model(args.precision, dev, "bench_asrbb", world=world,
                                                     rank=rank, cfg=ASR_BBOX))
    else:
        el, model = timed_train(args.precision, B, args.steps, args.warmup, dev, world, rank,
                                events=True)
    roof = roofline(model.kernel_events, B, args.precision)
    model.kernel_events = None
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    executed = model.executed_steps
    loss = model.loss
    del model
    torch.cuda.empty_cache()
    ms = el / args.steps * 1e3
    value = B * world * args.steps / el
    if rank == 0:
        workload = ("AIR baseline train step (training_air_original.py AIRModel, "
                    f"{args.precision}), per-GPU batch {B} (configs[1] batch)")
        model_name = "AIR (LSTM 256, VAE 784-512-256-50, heads 64)"
        metric = METRIC
        if asr:
            metric = ("images/sec/node AIR-ASR bbox train step (configs[4]: train_air_pr.py -dn 3 "
                      "-ds bbox20k -gb 1 -gs 10 -ga 20), Multi-MNIST 50x50, 1/2/4/8 GPU")
            workload = ("AIR-ASR train step (air_number_bbox_location.py AIRModel, "
                        f"{args.precision}): 3 objects of side 11-15, fix_steps 3, bbox / size / "
                        f"area regularisers, MAX_STEPS 6, per-GPU batch {B}")
            model_name = "AIR-ASR (inference + generative LSTMCell 256, VAE 784-512-256-50)"
        out = {
            "metric": metric, "value": value, "unit": "images/sec",
            "n_gpus": world if backend in (None, "nccl") else min(world, torch.cuda.device_count()),
            "ranks": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision, "data": "synthetic",
            "config": {"workload": workload, "model": model_name,
                       "global_batch": B * world, "per_gpu_batch": B, "canvas": "50x50",
                       "max_steps": T, "data_dependent_steps_would_be": executed,
                       "parallelism": f"dp{world}", "loss_last": loss,
                       "collective_backend": {"nccl": "rccl"}.get(backend, backend)},
            "roofline": roof,
        }
        if world == 1 and args.extras and not asr:
            if args.precision != "bf16":
                el2, m2 = timed_train("bf16", B, 10, 3, dev, scope="bench_bf16", events=True)
                out["configs_1_bf16"] = {
                    "value": B * 10 / el2, "unit": "images/sec", "ms_per_step": el2 / 10 * 1e3,
                    "dtype": "bf16", "batch": B, "steps": 10,
                    "workload": "configs[1]: bf16 VAE GEMM operands/activations (fp32 "
                                "accumulate), fused STN+VAE step kernel, LSTM/heads/STN/loss "
                                "fp32", "roofline": roofline(m2.kernel_events, B, "bf16")}
                del m2
            for prec in ("fp32", "bf16"):
                el4, m4 = timed_train(prec, B, 10, 3, dev,
                                      model=make_asr_model(prec, dev, "bench_asr_" + prec))
                out["configs_2_asr_" + prec] = {
                    "value": B * 10 / el4, "unit": "images/sec", "ms_per_step": el4 / 10 * 1e3,
                    "dtype": prec, "batch": B, "steps": 10, "max_steps": 6,
                    "executed_steps": m4.executed_steps,
                    "workload": "configs[2]: AIR-ASR train step (train_air_pr.py -dn 13 -gm 100 "
                                "-gne 10: number regularisers, learned z_pres prior, "
                                "MAX_STEPS 6)"}
                del m4
            # configs[4] (train_air_pr.py -dn 3 -ds bbox20k -gb 1 -gs 10 -ga 20) on one
            # GPU; the driver's multi-GPU runs of it use --workload asr_bbox
            for prec in ("fp32", "bf16"):
                el7, m7 = timed_train(prec, B, 10, 3, dev, data=ASR_BBOX_DATA,
                                      model=make_asr_model(prec, dev, "bench_asrbb_" + prec,
                                                           cfg=ASR_BBOX))
                out["configs_4_asr_bbox_" + prec] = {
                    "value": B * 10 / el7, "unit": "images/sec", "ms_per_step": el7 / 10 * 1e3,
                    "dtype": prec, "batch": B, "steps": 10, "max_steps": 6, "fix_steps": 3,
                    "workload": "configs[4]: AIR-ASR bbox train step (train_air_pr.py -dn 3 -ds "
                                "bbox20k -gb 1 -gs 10 -ga 20: 3 objects of side 11-15, fix_steps "
                                "3, bbox / size / area regularisers), one MI355X"}
                del m7
            # configs[2] at the reference's own batch of 64
            el5, m5 = timed_train("fp32", 64, 30, 5, dev, graph=True,
                                  model=make_asr_model("fp32", dev, "bench_asr_b64"))
            el5e, m5e = timed_train("fp32", 64, 30, 5, dev,
                                    model=make_asr_model("fp32", dev, "bench_asr_b64e"))
            out["configs_2_asr_fp32_b64"] = {
                "value": 64 * 30 / el5, "unit": "images/sec", "ms_per_step": el5 / 30 * 1e3,
                "dtype": "fp32", "batch": 64, "steps": 30, "max_steps": 6,
                "eager_ms_per_step": el5e / 30 * 1e3,
                "workload": "configs[2] (train_air_pr.py -dn 13 -gm 100 -gne 10) at the "
                            "reference's batch of 64, the captured train step "
                            "(train_step_graphed); eager_ms_per_step: launched kernel by kernel"}
            del m5, m5e
            # configs[3]: Multi-dSprites 2-4 objects on 64 x 64 canvases
            # (multi_dsprites.py:391-392, training_air_original.py -data sprites -dn 24),
            # bf16 fused step, max_steps 3 as the headline metric
            el6, m6 = timed_train("bf16", B, 10, 3, dev, scope="bench_c64", canvas=64,
                                  data=dict(counts=(2, 3, 4)))
            out["configs_3_dsprites_bf16"] = {
                "value": B * 10 / el6, "unit": "images/sec", "ms_per_step": el6 / 10 * 1e3,
                "dtype": "bf16", "batch": B, "steps": 10, "canvas": 64, "max_steps": 3,
                "workload": "configs[3]: AIR train step on 64x64 Multi-dSprites-like canvases "
                            "(2-4 objects of side 22-30), bf16 fused step kernel"}
            del m6
            torch.cuda.empty_cache()
            el3, m3 = timed_train("fp32", 64, 50, 5, dev, scope="bench_b64", graph=True)
            el3e, m3e = timed_train("fp32", 64, 50, 5, dev, scope="bench_b64e")
            out["config_1_batch64_fp32"] = {
                "value": 64 * 50 / el3, "unit": "images/sec", "ms_per_step": el3 / 50 * 1e3,
                "dtype": "fp32", "batch": 64, "steps": 50,
                "eager_ms_per_step": el3e / 50 * 1e3,
                "workload": "configs[0] shape (the reference's batch of 64) on one MI355X: "
                            "the captured train step (forward + backward replayed from one "
                            "hipGraph; noise fills, annealed prior and TF Adam launched around "
                            "it, AIRModel.train_step_graphed); eager_ms_per_step: the same step "
                            "launched kernel by kernel"}
            del m3, m3e
            torch.cuda.empty_cache()
            if args.roofline_batch > 0:
                out["fused_step_roofline"] = fused_step_roofline(args.roofline_batch,
                                                                 args.roofline_launches, dev)
                out["fused_step_roofline_c64"] = fused_step_roofline(
                    args.roofline_batch, args.roofline_launches, dev, canvas=64)
                out["fused_step_roofline_fwd"] = fused_step_roofline(
                    args.roofline_batch, args.roofline_launches, dev, save=False)
                out["fp32_step_roofline"] = fp32_step_roofline(args.roofline_batch,
                                                               args.roofline_launches, dev)
        if args.cpu_baseline and world == 1 and not asr:
            out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

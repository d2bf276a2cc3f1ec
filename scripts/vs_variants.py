"""Fused step kernel variants at one batch, one model / input set: each
variant is a set of environment overrides read by the launcher on every call
(MOG_VS_PIPE, MOG_VS_PHASES, MOG_VS_PRIO, MOG_VS_LA, ...), timed over 20
launches with HIP events on the launch stream; `timing` variants print the
per-tile role spans / phase times of one launch.
usage: python scripts/vs_variants.py [B] [C] VAR...   (VAR = KEY=VAL,KEY=VAL[:timing])"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mog-asr_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    args = sys.argv[1:]
    B = int(args.pop(0)) if args and args[0].isdigit() else 65536
    C = int(args.pop(0)) if args and args[0].isdigit() else 50
    dev = torch.device("cuda:0")
    m = bench.make_model("bf16", dev, 1, 0, "vsvar", canvas=C)
    m.noise_seed = 78
    x, k = bench.synthetic(B, 4321, C)
    X, K = torch.from_numpy(x).to(dev), torch.from_numpy(k).to(dev)
    m.infer(X, K)
    ws = m._ws
    for i in range(40):  # clocks settle before the first timed variant
        m._step_fused(X, ws, i % 3, 0.3, save=True)
    torch.cuda.synchronize()
    per = bench.fused_bytes_per_image_step(C * C)
    base = dict(os.environ)
    for v in args:
        timing = v.endswith(":timing")
        spec = v[:-7] if timing else v
        env = dict(kv.split("=", 1) for kv in spec.split(",") if kv)
        os.environ.clear()
        os.environ.update(base)
        os.environ.update(env)
        for t in range(3):
            m._step_fused(X, ws, t, 0.3, save=True)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        evs = []
        for i in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            m._step_fused(X, ws, i % 3, 0.3, save=True)
            e1.record(s)
            evs.append((e0, e1))
        torch.cuda.synchronize()
        us = sum(a.elapsed_time(b) for a, b in evs) / len(evs) * 1e3
        print(f"{spec or 'default'}: {us:.1f} us  frac {B * per / (us * 1e-6) / 8e12:.3f}",
              flush=True)
        if timing:
            os.environ["MOG_VS_TIMING"] = "1"
            m._step_fused(X, ws, 0, 0.3, save=True)
            torch.cuda.synchronize()
            sys.stderr.flush()


if __name__ == "__main__":
    main()

"""One workload per process, for rocprofv3 passes whose dispatches must not
be mixed with others' (kernel trace, --pmc FETCH_SIZE / WRITE_SIZE):

  fused_bf16 [B] [C]  the north-star fused step launch (bench.fused_step_roofline:
                      training form, one loop step), 5 launches after 2 warm-ups
  step_fp32 [B]       the headline fp32 train step (bench defaults), 5 steps after 10
                      (the clocks settle over the first steps: the tables keep
                      the last 5 steps' dispatches)
  step_bf16 [B]       configs[1]'s bf16 train step, 5 steps after 10
  fused_f32 [B]       the fp32 fused step over B rows (bench.fp32_step_roofline)
  asr_fp32 / asr_bf16 [B]  configs[2]'s AIR-ASR train step, 3 steps after 2

usage: python scripts/prof_one.py <workload> [B] [C]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "mog-asr_amd")]
import torch  # noqa: E402

import bench  # noqa: E402


STEPS, WARM = 5, 10  # train-step workloads (scripts/pmc_tables.py keeps the last STEPS)


def main():
    w = sys.argv[1]
    dev = torch.device("cuda:0")
    if w == "fused_bf16":
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
        C = int(sys.argv[3]) if len(sys.argv) > 3 else 50
        r = bench.fused_step_roofline(B, 5, dev, canvas=C)
        print(f"fused_bf16 B={B} C={C}: {r['avg_launch_us']:.1f} us frac {r['frac']:.3f}")
    elif w in ("step_fp32", "step_bf16"):
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
        prec = w.split("_")[1]
        el, m = bench.timed_train(prec, B, STEPS, WARM, dev, scope="prof_" + prec)
        print(f"{w} B={B}: {el / STEPS * 1e3:.3f} ms per step")
    elif w in ("asr_fp32", "asr_bf16"):
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
        prec = w.split("_")[1]
        m = bench.make_asr_model(prec, dev, "prof_asr_" + prec)
        el, m = bench.timed_train(prec, B, 3, 2, dev, model=m)
        print(f"{w} B={B}: {el / 3 * 1e3:.3f} ms per step")
    elif w == "fused_f32":
        B = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
        r = bench.fp32_step_roofline(B, 5, dev)
        print(f"fused_f32 B={B}: {r['avg_chain_us']:.1f} us frac {r['frac']:.3f}")
    else:
        raise SystemExit(__doc__)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

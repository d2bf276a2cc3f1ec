"""Copies a round's bench evidence (ROUND, default r06) out of gpurun_out/ (scripts/final_pass.sh,
scripts/prof_evidence.sh) into profiles/: the bench JSON line measured under
rocprofv3 and that run's --stats kernel summary; with --traces also the
per-workload kernel traces (start / duration / queue / grid / name)."""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
R = os.environ.get("ROUND", "r06")
O = os.path.join(ROOT, "gpurun_out", R + "prof")
P = os.path.join(ROOT, "profiles")


def main():
    line = [ln for ln in open(os.path.join(O, "bench.log")) if ln.startswith("{")][-1]
    json.loads(line)
    with open(os.path.join(P, R + "_bench.json"), "w") as f:
        f.write(line)
    stats = glob.glob(os.path.join(O, "bench", "**", "*kernel_stats.csv"), recursive=True)
    shutil.copy(stats[0], os.path.join(P, R + "_bench_kernel_stats.csv"))
    if "--traces" in sys.argv:
        for td in sorted(d for d in glob.glob(os.path.join(O, "t_*")) if os.path.isdir(d)):
            tr = glob.glob(os.path.join(td, "**", "*kernel_trace.csv"), recursive=True)[0]
            rows = list(csv.DictReader(open(tr)))
            t0 = min(int(r["Start_Timestamp"]) for r in rows)
            name = os.path.join(P, R + "_trace_" + os.path.basename(td)[2:] + ".csv")
            with open(name, "w", newline="") as f:
                w = csv.writer(f)
                w.writerow(["start_us", "dur_us", "stream", "grid_x", "kernel"])
                for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
                    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                    w.writerow([round((s - t0) / 1e3, 1), round((e - s) / 1e3, 1), r["Queue_Id"],
                                r["Grid_Size_X"], r["Kernel_Name"].split("(")[0]
                                if r["Kernel_Name"].startswith("void") else r["Kernel_Name"]])
    print("profiles updated:", json.loads(line)["ms_per_step"], "ms/step under rocprofv3")


if __name__ == "__main__":
    main()

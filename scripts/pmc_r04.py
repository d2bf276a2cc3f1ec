"""Per-workload kernel table from rocprofv3 passes of scripts/prof_one.py
(scripts/prof_r04.sh): for every kernel symbol of a workload, dispatches,
average duration (kernel trace) and HBM bytes per dispatch from separate
FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md §HBM: FETCH_SIZE halves a
wide coalesced read on gfx950, so it is doubled; both counters in KiB).  The
workload's target launch (the one bench.py prices) is the LAST `n` dispatches
of its target symbol -- prof_one.py runs the priced launches last.

usage: python scripts/pmc_r04.py <dir with t_*/f_*/w_* pass outputs> [out.json]"""
import csv
import glob
import json
import os
import re
import sys

# workload -> (target symbol substring, priced dispatches run last, work per launch, unit)
TARGETS = {
    "fused_bf16_65536_50": ("stn_vae_step", 5, 65536 * 30024, "bytes"),
    "fused_bf16_65536_64": ("stn_vae_step", 5, 65536 * 49176, "bytes"),
    "fused_f32_24576": ("stn_vae_step_f32_kernel", 5, 24576 * 2206720.0 * 1.0, "flop"),
    "step_fp32_8192": ("stn_vae_step_f32_kernel", 3, 24576 * 2206720.0, "flop"),
}


def short(sym):
    s = sym.replace("(anonymous namespace)::", "")
    s = re.sub(r"\(.*$", "", s)
    return s[:90]


def rows_of(d, pattern):
    out = []
    for fn in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        out += list(csv.DictReader(open(fn)))
    return out


def counter(d, name):
    rows = [r for r in rows_of(d, "*counter_collection.csv") if r.get("Counter_Name") == name]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    by = {}
    for r in rows:
        by.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return by


def trace(d):
    rows = rows_of(d, "*kernel_trace.csv")
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = {}
    for r in rows:
        by.setdefault(short(r["Kernel_Name"]), []).append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return by


def main():
    root = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    res = {"_note": "per workload (scripts/prof_one.py): durations us from --kernel-trace, "
                    "hbm_bytes = (2*FETCH_SIZE + WRITE_SIZE) KiB*1024 per dispatch from separate "
                    "--pmc passes; target = the last n dispatches of the priced kernel"}
    for w, (sym, n, work, unit) in TARGETS.items():
        td, fd, wd = (os.path.join(root, p + w) for p in ("t_", "f_", "w_"))
        if not os.path.isdir(td):
            continue
        tr, fe, wr = trace(td), counter(fd, "FETCH_SIZE"), counter(wd, "WRITE_SIZE")
        kern = {}
        for k, durs in tr.items():
            e = {"dispatches": len(durs), "avg_us": sum(durs) / len(durs), "total_us": sum(durs)}
            if k in fe and k in wr and fe[k] and wr[k]:
                e["hbm_bytes_avg"] = (2 * sum(fe[k]) / len(fe[k]) + sum(wr[k]) / len(wr[k])) * 1024
            kern[k] = e
        tgt = [k for k in tr if sym in k and (sym != "stn_vae_step" or "f32" not in k)]
        entry = {"kernels_by_total_time": dict(sorted(kern.items(), key=lambda kv: -kv[1]["total_us"])[:12])}
        if tgt:
            k = max(tgt, key=lambda k: len(tr[k]))
            durs = tr[k][-n:]
            avg = sum(durs) / len(durs)
            t = {"kernel": k, "launches": len(durs), "avg_us": avg,
                 "work_per_launch": work, "work_unit": unit}
            if k in fe and k in wr:
                f = fe[k][-n:]
                ww = wr[k][-n:]
                t["fetch_bytes"] = 2 * sum(f) / len(f) * 1024
                t["write_bytes"] = sum(ww) / len(ww) * 1024
                t["hbm_bytes_per_launch"] = t["fetch_bytes"] + t["write_bytes"]
            if unit == "bytes":
                t["achieved_GBps"] = work / avg / 1e3
                t["frac_of_8TBps"] = work / avg / 1e3 / 8000
            else:
                t["achieved_TFLOPs"] = work / avg / 1e6
                t["frac_of_fp32_157TF"] = work / avg / 1e6 / 157.3
            entry["target"] = t
        res[w] = entry
    s = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(s)
    print(s)


if __name__ == "__main__":
    main()

"""Per-workload kernel tables and the bench's traffic entries, from
rocprofv3 passes of scripts/prof_one.py (scripts/prof_evidence.sh): per kernel
symbol the dispatches, average duration (kernel trace) and HBM bytes per
dispatch from separate FETCH_SIZE / WRITE_SIZE passes (MI355X_MICROARCH.md
§HBM: FETCH_SIZE halves a wide coalesced read on gfx950, so it is doubled;
both counters in KiB).  Writes the per-workload tables to <out.json> and
merges one entry per bench.py roofline tag -- "<tag>_<precision>_b<B>",
hbm_bytes_per_launch averaged over the tag's dispatches -- into
profiles/pmc_summary.json (stale tags of earlier rounds are dropped).

usage: python scripts/pmc_tables.py <dir with t_*/f_*/w_* pass outputs> <out.json> [round tag]"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SUMMARY = os.path.join(ROOT, "profiles", "pmc_summary.json")

# bench tag -> (workload, symbol predicate, which dispatches: "all" | "even" | "odd" | "last5"
# | "5not4" / "5is4": all but / only every fifth, from the fifth)
TAGS = {
    "stn_vae_step_f32_all_fp32_b8192": ("step_fp32_8192", lambda k: "stn_vae_step_f32_kernel" in k, "all"),
    # wgrad_tn_x3_kernel runs the seven VAE weight gradients (grouped), the
    # five heads' hidden layers, then the LSTM recurrent rows: three per step
    # in that order (each followed by its wgrad_tn_reduce_kernel, not counted)
    "vae_wgrad_x3_fp32_b8192": ("step_fp32_8192", lambda k: k.startswith("wgrad_tn_x3_kernel"), "mod3_0"),
    "heads_wgrad_x3_fp32_b8192": ("step_fp32_8192", lambda k: k.startswith("wgrad_tn_x3_kernel"), "mod3_1"),
    "rec_wgrad_x3_fp32_b8192": ("step_fp32_8192", lambda k: k.startswith("wgrad_tn_x3_kernel"), "mod3_2"),
    "vae_dgrad_x3_fp32_b8192": ("step_fp32_8192", lambda k: "gemm_x3_nt_kernel" in k, "all"),
    "lstm_x_projection_grad_fp32_b8192": ("step_fp32_8192", lambda k: "gemm_x3_tn_kernel<true, 3>" in k, "all"),
    "lstm_x_projection_fp32_b8192": ("step_fp32_8192", lambda k: "gemm_f32_dma_kernel<128, 128, 16, 3, false, false, 0>" in k, "all"),
    # the step runs the STN write backward, then the read backward
    "stn_write_bwd_fp32_b8192": ("step_fp32_8192", lambda k: k.startswith("stn_bwd_kernel"), "even"),
    "stn_read_bwd_fp32_b8192": ("step_fp32_8192", lambda k: k.startswith("stn_bwd_kernel"), "odd"),
    "stn_vae_step_all_bf16_b8192": ("step_bf16_8192", lambda k: k.startswith("void stn_vae_step_kernel"), "all"),
    "vae_wgrad_bf16_bf16_b8192": ("step_bf16_8192", lambda k: "wgrad_tn_bf16_kernel" in k, "all"),
    "lstm_x_projection_grad_bf16_b8192": ("step_bf16_8192", lambda k: "gemm_x3_tn_kernel<true, 1>" in k, "all"),
    "lstm_x_projection_bf16_b8192": ("step_bf16_8192", lambda k: "gemm_f32_dma_kernel<128, 128, 16, 3, false, false, 0>" in k, "all"),
    "stn_vae_step_b65536": ("fused_bf16_65536_50", lambda k: k.startswith("void stn_vae_step_kernel"), "last5"),
    "stn_vae_step_b65536_c64": ("fused_bf16_65536_64", lambda k: k.startswith("void stn_vae_step_kernel"), "last5"),
}


STEP_N, STEP_KEEP = 15, 5  # prof_one.py's train-step workloads: 10 warm-up + 5 steps


def short(sym):
    s = sym.replace("(anonymous namespace)::", "")
    s = re.sub(r"\(.*$", "", s)
    return s[:100]


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


def pick(v, which):
    if which == "even":
        return v[0::2]
    if which == "odd":
        return v[1::2]
    if which == "last5":
        return v[-5:]
    if which == "5not4":
        return [x for i, x in enumerate(v) if i % 5 != 4]
    if which.startswith("mod3_"):
        return v[int(which[-1])::3]
    if which == "5is4":
        return v[4::5]
    return v


def main():
    root, out = sys.argv[1], sys.argv[2]
    rnd = sys.argv[3] if len(sys.argv) > 3 else "r06"
    tables, data = {}, {}
    for td in sorted(glob.glob(os.path.join(root, "t_*"))):
        w = os.path.basename(td)[2:]
        fd, wd = os.path.join(root, "f_" + w), os.path.join(root, "w_" + w)
        tr, fe, wr = trace(td), counter(fd, "FETCH_SIZE"), counter(wd, "WRITE_SIZE")
        data[w] = (tr, fe, wr)
        kern = {}
        for k, durs in tr.items():
            e = {"dispatches": len(durs), "avg_us": sum(durs) / len(durs), "total_us": sum(durs)}
            if fe.get(k) and wr.get(k):
                e["hbm_bytes_avg"] = (2 * sum(fe[k]) / len(fe[k]) + sum(wr[k]) / len(wr[k])) * 1024
            kern[k] = e
        tables[w] = dict(sorted(kern.items(), key=lambda kv: -kv[1]["total_us"]))
    with open(out, "w") as f:
        json.dump(tables, f, indent=1)
    try:
        summary = json.load(open(SUMMARY))
    except (OSError, ValueError):
        summary = {}
    summary = {k: v for k, v in summary.items() if k.startswith("_") or "source" in v and v["source"].endswith(f"({rnd})")}
    summary["_note"] = ("hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE per dispatch (gfx950 "
                        "FETCH_SIZE halving corrected), from separate --pmc passes of "
                        "scripts/prof_one.py workloads (scripts/prof_evidence.sh); key = bench.py "
                        "roofline tag _ precision _ b<batch>, averaged over the tag's dispatches")
    for tag, (w, pred, which) in TAGS.items():
        if w not in data:
            continue
        tr, fe, wr = data[w]
        syms = [k for k in tr if pred(k)]
        durs, fb, wb = [], [], []
        # train-step workloads (prof_one.py: STEP_N steps, of which the last
        # STEP_KEEP are kept -- the clocks settle over the first ones)
        keep = (lambda v: v[len(v) - len(v) // STEP_N * STEP_KEEP:]) if w.startswith("step_") \
            else (lambda v: v)
        for k in syms:
            durs += pick(keep(tr[k]), which)
            fb += pick(keep(fe.get(k, [])), which)
            wb += pick(keep(wr.get(k, [])), which)
        if not durs or not fb or not wb:
            continue
        fetch = 2 * sum(fb) / len(fb) * 1024
        write = sum(wb) / len(wb) * 1024
        summary[tag] = {"kernel_symbols": syms, "workload": w, "dispatches": len(durs),
                        "profiled_avg_us": sum(durs) / len(durs), "fetch_bytes": fetch,
                        "write_bytes": write, "hbm_bytes_per_launch": fetch + write,
                        "source": f"scripts/prof_evidence.sh ({rnd})"}
    with open(SUMMARY, "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: (v.get("profiled_avg_us"), v.get("hbm_bytes_per_launch"))
                      for k, v in summary.items() if not k.startswith("_")}, indent=1))


if __name__ == "__main__":
    main()

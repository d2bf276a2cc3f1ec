"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (run separately, as
MI355X_MICROARCH.md §HBM prescribes) into profiles/pmc_summary.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE
is exact for 16 B/lane stores.  Both counters are in KiB.

Tag -> kernel selection: the tagged launch is the dispatch of the named kernel
symbol with the largest FETCH_SIZE in each train step (the x-projection GEMM
shares its template instantiation with the smaller recurrent GEMMs).

usage: python scripts/pmc_summary.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import sys

TAGS = {
    "lstm_x_projection": "gemm_f32_kernel<128, 128, false, false, 0>",
    "lstm_x_projection_grad": "gemm_f32_kernel<64, 64, true, false, 5>",
    "stn_vae_step": "stn_vae_step",
}


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") == counter:
                rows.append(r)
    return rows


def per_kernel(rows, symbol, grid=None):
    vals = [(int(r["Dispatch_Id"]), float(r["Counter_Value"])) for r in rows
            if symbol in r["Kernel_Name"]
            and (grid is None or int(float(r.get("Grid_Size", -1))) == grid)]
    return sorted(vals)


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_summary.json"
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {"_note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024, "
                    "gfx950 FETCH_SIZE halving corrected; averaged over the largest-fetch "
                    "dispatch of the tagged kernel symbol per train step"}
    jobs = [(tag, sym, None) for tag, sym in TAGS.items()]
    # the fused step kernel runs at the bench batch (8192: 256 workgroups of 32
    # images x 1024 threads) and in the stand-alone north-star roofline run
    # (65,536: 1024 workgroups of 64 images x 1024 threads)
    jobs = [j for j in jobs if j[0] != "stn_vae_step"] + [
        ("stn_vae_step", "stn_vae_step", 8192 // 32 * 1024),
        ("stn_vae_step_b65536", "stn_vae_step", 65536 // 64 * 1024)]
    for tag, sym, grid in jobs:
        fv, wv = per_kernel(fetch, sym, grid), per_kernel(write, sym, grid)
        if not fv or not wv:
            continue
        fmax = max(v for _, v in fv)
        fsel = [v for _, v in fv if v >= 0.5 * fmax]
        wmax = max(v for _, v in wv)
        wsel = [v for _, v in wv if v >= 0.5 * wmax] if tag.endswith("grad") else \
            [v for (i, v) in wv][:len(fsel)]
        # pair write dispatches with the selected fetch dispatches by order
        fids = [i for i, v in fv if v >= 0.5 * fmax]
        wmap = dict(wv)
        wsel = [wmap.get(i) for i in fids if wmap.get(i) is not None] or wsel
        fk = sum(fsel) / len(fsel)
        wk = sum(wsel) / len(wsel)
        res[tag] = {"kernel_symbol": sym, "grid_threads": grid, "fetch_kib": fk, "write_kib": wk,
                    "dispatches": len(fsel),
                    "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0}
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

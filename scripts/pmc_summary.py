"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (run separately, as
MI355X_MICROARCH.md §HBM prescribes) into profiles/pmc_summary.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half
of the bytes of a wide (16 B/lane) coalesced read, so it is doubled; WRITE_SIZE
is exact for 16 B/lane stores and float atomics.  Both counters are in KiB.

Tag -> dispatch selection: the kernel symbol AND the launch grid (total
work-items) of the launch bench.py times, then, among those dispatches, the
ones with the largest FETCH_SIZE (the x-projection shares symbol and grid
with the two smaller recurrent GEMMs of the same step).  The grids below are
those of the bench workloads: per-GPU batch 8192 (fp32 headline, bf16
configs[1]) and the stand-alone fused-step roofline runs at 65,536.

usage: python scripts/pmc_summary.py <fetch_dir> <write_dir> [out.json]
"""
import csv
import glob
import json
import os
import sys

B = 8192


def _ceil(a, b):
    return (a + b - 1) // b


def _x_grad_grid_fp32(B, C2=2500, N=1024, target=2048, BK=32):
    """gemm_f32 transA split-K launch of dWx (air_model._dw, launch_dma with
    32-deep k-tiles for transA)."""
    tiles = _ceil(C2, 64) * _ceil(N, 64)
    splitk = max(1, min(B // 256, _ceil(target, tiles)))
    kchunk = _ceil(_ceil(B, splitk), BK) * BK
    return tiles * _ceil(B, kchunk) * 256


# tag -> (kernel symbol substring, grid work-items)
TAGS = {
    "lstm_x_projection_fp32_b%d" % B: ("gemm_f32_dma_kernel<128, 128, 16, 3, false, false, 0>",
                                       (1024 // 128) * (B // 128) * 256),
    "lstm_x_projection_grad_fp32_b%d" % B: ("gemm_f32_dma_kernel<64, 64, 32, 2, true, false, 5>",
                                            _x_grad_grid_fp32(B)),
    "lstm_x_projection_bf16_b%d" % B: ("gemm_f32_dma_kernel<128, 128, 16, 3, false, false, 0>",
                                       (1024 // 128) * (B // 128) * 256),
    "stn_vae_step_bf16_b%d" % B: ("stn_vae_step", B // 32 * 1024),
    "stn_vae_step_b65536": ("stn_vae_step", 65536 // 64 * 1024),
    "stn_vae_step_b65536_c64": ("stn_vae_step", 65536 // 64 * 1024),
    "stn_vae_step_b65536_fwd": ("stn_vae_step", 65536 // 64 * 1024),
    # bench.fp32_step_roofline: the fp32 fused step, 32-image tiles
    "stn_vae_step_f32_b65536": ("stn_vae_step_f32_kernel", 65536 // 32 * 1024),
}
# bench.py runs the three B = 65,536 fused-step measurements in this order
# (same symbol and grid): training form at C = 50, at C = 64, forward-only at C = 50
FUSED_ORDER = ("stn_vae_step_b65536", "stn_vae_step_b65536_c64", "stn_vae_step_b65536_fwd")


def load(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    rows = []
    for fn in files:
        for r in csv.DictReader(open(fn)):
            if r.get("Counter_Name") == counter:
                rows.append(r)
    return rows


def per_kernel(rows, symbol, grid):
    return sorted((int(r["Dispatch_Id"]), float(r["Counter_Value"]), r) for r in rows
                  if symbol in r["Kernel_Name"] and int(float(r.get("Grid_Size", -1))) == grid)


def main():
    fdir, wdir = sys.argv[1], sys.argv[2]
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_summary.json"
    fetch, write = load(fdir, "FETCH_SIZE"), load(wdir, "WRITE_SIZE")
    res = {"_note": "hbm_bytes_per_launch = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 "
                    "FETCH_SIZE halving corrected), averaged over the dispatches of the tagged "
                    "kernel symbol with the bench launch's grid and >= 0.5x the largest fetch"}
    for tag, (sym, grid) in TAGS.items():
        fv, wv = per_kernel(fetch, sym, grid), per_kernel(write, sym, grid)
        if not fv or not wv:
            continue
        fmax = max(v for _, v, _ in fv)
        fsel = [(i, v) for i, v, _ in fv if v >= 0.5 * fmax]
        # the three fused-step runs share symbol and grid: equal groups of
        # dispatches in FUSED_ORDER (dispatch order)
        if tag in FUSED_ORDER:
            fsel = [(i, v) for i, v, _ in fv]
            third = len(fsel) // 3
            g = FUSED_ORDER.index(tag)
            fsel = fsel[g * third:(g + 1) * third]
            if not fsel:
                continue
        ids = [i for i, _ in fsel]
        wmap = {i: v for i, v, _ in wv}
        wsel = [wmap[i] for i in ids if i in wmap]
        if not wsel:  # separate passes: dispatch ids do not line up, pair by order
            wsel = [v for _, v, _ in wv][:len(fsel)]
        fk = sum(v for _, v in fsel) / len(fsel)
        wk = sum(wsel) / len(wsel)
        res[tag] = {"kernel_symbol": sym, "grid_threads": grid, "fetch_kib": fk,
                    "write_kib": wk, "dispatches": len(fsel),
                    "hbm_bytes_per_launch": (2.0 * fk + wk) * 1024.0}
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()

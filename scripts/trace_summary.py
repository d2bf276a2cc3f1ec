"""Per-form kernel durations of a rocprofv3 --kernel-trace run of bench.py
(scripts/prof_round.sh), selected exactly as scripts/pmc_summary.py selects
the counter dispatches: kernel symbol + launch grid, the three B = 65,536
bf16 fused-step forms (training C = 50, training C = 64, forward-only C = 50)
split by dispatch order.  Every `frac` of the bench line can be recomputed
from these averages and the algorithmic work per launch.

usage: python scripts/trace_summary.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import FUSED_ORDER, TAGS  # noqa: E402


def main():
    path = sys.argv[1]
    out = sys.argv[2] if len(sys.argv) > 2 else None
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    res = {"_note": "durations in us from rocprofv3 --kernel-trace (Start/End timestamps); "
                    "dispatches selected by kernel symbol and grid work-items (pmc_summary.TAGS)"}
    for tag, (sym, grid) in TAGS.items():
        sel = []
        for r in rows:
            g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            if sym in r["Kernel_Name"] and g == grid:
                sel.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        if tag in FUSED_ORDER and sel:
            third = len(sel) // 3
            k = FUSED_ORDER.index(tag)
            sel = sel[k * third:(k + 1) * third]
        if tag.startswith("lstm_x_projection") and sel:
            # the x-projection shares symbol and grid with the smaller GEMMs of
            # the same step: keep the launches >= 0.5x the longest
            top = max(sel)
            sel = [d for d in sel if d >= 0.5 * top]
        if not sel:
            continue
        res[tag] = {"kernel_symbol": sym, "grid_threads": grid, "dispatches": len(sel),
                    "avg_us": sum(sel) / len(sel), "min_us": min(sel), "max_us": max(sel)}
    txt = json.dumps(res, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(txt)
    print(txt)


if __name__ == "__main__":
    main()

"""Per-kernel averages of an SQ --pmc pass (scripts/pmc_gemm_sq.sh): wave
state fractions, MFMA-busy fraction of the SIMD cycles and the effective clock
(GRBM_GUI_ACTIVE / 8 XCDs / dispatch wall time, MI355X_MICROARCH.md DVFS)."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:] or ["gpurun_out/pmc_sq0"]:
    print("==", d)
    rows = []
    for fn in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(fn)))
    disp = defaultdict(dict)
    for r in rows:
        e = disp[r["Dispatch_Id"]]
        e[r["Counter_Name"]] = float(r["Counter_Value"])
        e["name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "")[:64]
        e["grid"] = r["Grid_Size"]
        e["dur"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg = defaultdict(list)
    for e in disp.values():
        if "gemm" in e["name"]:
            agg[(e["name"], e["grid"])].append(e)
    for k, es in agg.items():
        a = {n: sum(e[n] for e in es) / len(es) for n in es[0] if n not in ("name", "grid")}
        wc = a["SQ_WAVE_CYCLES"] or 1
        clk = a["GRBM_GUI_ACTIVE"] / 8 / a["dur"]
        print("%-64s grid %8s %7.1f us clk %.2f GHz mfma %.2f | wait_any %.2f wait_inst %.2f "
              "active %.2f lds %.2f" % (k[0], k[1], a["dur"] / 1e3, clk,
                                        a["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * a["GRBM_GUI_ACTIVE"] / 8),
                                        a["SQ_WAIT_ANY"] / wc, a["SQ_WAIT_INST_ANY"] / wc,
                                        a["SQ_ACTIVE_INST_ANY"] / wc, a["SQ_WAIT_INST_LDS"] / wc))

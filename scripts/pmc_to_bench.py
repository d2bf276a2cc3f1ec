"""Merge the per-workload counter table of scripts/pmc_r04.py into
profiles/pmc_summary.json under the tags bench.py looks up (bench.pmc_traffic:
"<kernel tag>_<precision>_b<batch>" for the train step's dominant launch,
"stn_vae_step_b65536[_c64]" for the fused-step roofline runs).
usage: python scripts/pmc_to_bench.py <pmc_r04.json> [profiles/pmc_summary.json]"""
import json
import sys

MAP = {
    "stn_vae_step_b65536": "fused_bf16_65536_50",
    "stn_vae_step_b65536_c64": "fused_bf16_65536_64",
    "stn_vae_step_f32_all_fp32_b8192": "step_fp32_8192",
    "stn_vae_step_f32_b24576": "fused_f32_24576",
}


def main():
    src = json.load(open(sys.argv[1]))
    out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_summary.json"
    try:
        res = json.load(open(out))
    except (OSError, ValueError):
        res = {}
    for tag, w in MAP.items():
        t = (src.get(w) or {}).get("target")
        if not t or "hbm_bytes_per_launch" not in t:
            continue
        res[tag] = {"kernel_symbol": t["kernel"], "workload": w, "dispatches": t["launches"],
                    "fetch_bytes": t["fetch_bytes"], "write_bytes": t["write_bytes"],
                    "hbm_bytes_per_launch": t["hbm_bytes_per_launch"],
                    "profiled_avg_us": t["avg_us"], "source": "scripts/prof_r04.sh (round 4)"}
    res["_note"] = ("hbm_bytes_per_launch = 2*FETCH_SIZE + WRITE_SIZE per dispatch (gfx950 "
                    "FETCH_SIZE halving corrected), from separate --pmc passes; round-4 entries "
                    "name their workload (scripts/prof_one.py) and source")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k in MAP}, indent=1))


if __name__ == "__main__":
    main()

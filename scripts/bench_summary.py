"""One-screen summary of a bench.py JSON line (the last line starting with '{')."""
import json
import sys

line = [ln for ln in open(sys.argv[1]) if ln.startswith("{")][-1]
d = json.loads(line)
print("headline ms/step %.3f  value %.0f img/s" % (d["ms_per_step"], d["value"]))
for k, v in d.items():
    if isinstance(v, dict) and "ms_per_step" in v:
        print("%-28s %.3f ms%s" % (k, v["ms_per_step"], "  eager %.3f" % v["eager_ms_per_step"]
                                    if v.get("eager_ms_per_step") else ""))
for k in ("fused_step_roofline", "fused_step_roofline_c64", "fused_step_roofline_fwd",
          "fp32_step_roofline"):
    v = d.get(k)
    if v:
        print("%-28s %.1f us  frac %.3f %s" % (k, v.get("avg_launch_us", v.get("avg_chain_us")),
                                               v["frac"], {x: v[x] for x in v if x.startswith("frac_")}))
r = d["roofline"]
print("roofline", r["kernel"], "%.3f" % r["frac"], "%.1f us" % r["avg_launch_us"])
for x in r.get("launches_priced", []):
    print("   ", x)
c = d.get("cpu_baseline")
if c:
    print("cpu", c["value"], c["cores"])

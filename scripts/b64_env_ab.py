"""A/B of a profiling-build environment override on the captured batch-64 AIR
step: each value in its own child process (the library reads the override
once), alternating rounds.  usage: python scripts/b64_env_ab.py VAR v1,v2,.. [rounds] [air|asr]
Runs with MOG_AIR_LIB = the profiling build (make PROFILE=1)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
var, vals = sys.argv[1], sys.argv[2].split(",")
rounds = int(sys.argv[3]) if len(sys.argv) > 3 else 2
which = sys.argv[4] if len(sys.argv) > 4 else "air"  # "asr": configs[2]'s AIR-ASR step
env0 = dict(os.environ, MOG_AIR_LIB=os.path.join(ROOT, "mog-asr_amd", "mog_air", "_lib", "prof",
                                                 "libmog_air.so"))
CHILD = f"""
import sys
sys.path.insert(0, "mog-asr_amd")
import torch, bench
dev = torch.device("cuda:0")
m = bench.make_asr_model("fp32", dev, "ab") if "{which}" == "asr" else None
el, m = bench.timed_train("fp32", 64, 200, 20, dev, graph=True, model=m)
print(f"{{el / 200 * 1e3:.4f}} ms/step")
"""
for r in range(rounds):
    for v in vals:
        env = dict(env0, **{var: v})
        out = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True,
                             text=True, timeout=240, cwd=ROOT)
        line = [ln for ln in out.stdout.splitlines() if "ms/step" in ln]
        print(f"{var}={v}: {line[-1] if line else out.stderr[-300:]}", flush=True)

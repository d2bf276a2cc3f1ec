"""Print the kernels of the last complete train step from a rocprofv3 kernel trace."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "clip_adam" in r["Kernel_Name"]]
a, b = idx[-2] + 1, idx[-1] + 1
agg = {}
tot = 0.0
for r in rows[a:b]:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = n.split("(")[0] if "gemm" not in n else n[:n.find("(")]
    g = f'{int(r["Grid_Size_X"])//int(r["Workgroup_Size_X"])}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}'
    if len(sys.argv) > 2:
        print(f"{d:8.1f} us  {g:>14} vgpr={r['VGPR_Count']} lds={r['LDS_Block_Size']} {n}")
    k = n
    agg.setdefault(k, [0, 0.0])
    agg[k][0] += 1
    agg[k][1] += d
for k, (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} us  n={c:3d}  {k}")
span = (int(rows[b - 1]["End_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3
# GPU busy time = union of the kernels' intervals (both streams); the rest of
# the span is idle (launch / host gaps)
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[a:b])
busy, cur_s, cur_e, gaps = 0, iv[0][0], iv[0][1], []
for s_, e_ in iv[1:]:
    if s_ > cur_e:
        busy += cur_e - cur_s
        gaps.append((s_ - cur_e) / 1e3)
        cur_s, cur_e = s_, e_
    else:
        cur_e = max(cur_e, e_)
busy += cur_e - cur_s
print(f"sum {tot:.1f} us  span {span:.1f} us  busy {busy / 1e3:.1f} us  idle {span - busy / 1e3:.1f} us "
      f"in {len(gaps)} gaps (largest {sorted(gaps)[-5:] if gaps else []})")

"""Summarise a rocprofv3 kernel_trace.csv: per (kernel, grid) average duration."""
import csv
import sys
from collections import defaultdict

rows = defaultdict(list)
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        name = r["Kernel_Name"].split("(")[0][:60]
        key = (name, r["Grid_Size_X"], r["Grid_Size_Y"], r["Workgroup_Size_X"], r["VGPR_Count"], r["LDS_Block_Size"])
        rows[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
    v.sort()
    print(f"{key[0]:60s} grid=({key[1]},{key[2]}) wg={key[3]} vgpr={key[4]} lds={key[5]} n={len(v):5d} "
          f"avg={sum(v)/len(v):8.2f}us med={v[len(v)//2]:8.2f} min={v[0]:8.2f}")

# inter-kernel gaps (graph replays put kernels back to back on one queue)
ev = []
with open(sys.argv[1]) as f:
    for r in csv.DictReader(f):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][:40]))
ev.sort()
gaps = sorted((b[0] - a[1]) / 1e3 for a, b in zip(ev, ev[1:]) if 0 <= b[0] - a[1] < 20000)
if gaps:
    print(f"inter-kernel gaps: n={len(gaps)} median={gaps[len(gaps)//2]:.2f}us p10={gaps[len(gaps)//10]:.2f} p90={gaps[9*len(gaps)//10]:.2f}")

#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace of tools/time_ba.py: per-kernel time of the last single C4
solve and per-kernel totals of the batched solves (grid.y >= 64)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ba = [r for r in rows if "k_ba" in r["Kernel_Name"] or "chol" in r["Kernel_Name"] or "k_cb" in r["Kernel_Name"]]
single = [r for r in ba if int(r["Grid_Size_Y"]) == 1 and "ctl" not in r["Kernel_Name"] or
          ("ctl" in r["Kernel_Name"] and int(r["Grid_Size_X"]) <= 1024)]
# the last single solve: from the last k_ba_ctl_init with grid 1024 (one problem) onwards
inits = [i for i, r in enumerate(ba) if "ctl_init" in r["Kernel_Name"] and int(r["Grid_Size_X"]) == 1024]
for title, seq in (("single C4 solve", ba[inits[-2]:inits[-1]] if len(inits) > 1 else []),):
    agg = collections.defaultdict(lambda: [0, 0.0])
    for r in seq:
        k = r["Kernel_Name"].split("(")[0].replace("orbhip::", "")
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1000 if seq else 0
    print(f"== {title}: span {span:.1f} us, kernel sum {sum(v[1] for v in agg.values()):.1f} us")
    for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
        print(f"  {k:40s} {v[0]:5d} {v[1] / v[0]:9.2f} {v[1]:9.1f}")
agg = collections.defaultdict(lambda: [0, 0.0])
t0 = t1 = None
for r in ba:
    if int(r["Grid_Size_Y"]) >= 64 or (int(r["Grid_Size_X"]) >= 64 * 1024 and "ctl" in r["Kernel_Name"]) or \
            ("chol_reg" in r["Kernel_Name"] and int(r["Grid_Size_X"]) >= 512 * 64):
        k = r["Kernel_Name"].split("(")[0].replace("orbhip::", "")
        agg[k][0] += 1
        agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
print(f"== batched solves: kernel sum {sum(v[1] for v in agg.values()):.1f} us")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {k:40s} {v[0]:5d} {v[1] / v[0]:9.2f} {v[1]:9.1f}")

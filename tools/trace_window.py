#!/usr/bin/env python3
"""Per-kernel time in one window of a rocprofv3 kernel trace: from the k-th last launch whose name
contains MARKER up to the next such launch (or the end). Usage: trace_window.py trace.csv MARKER [k] [--grid]
Prints the window's span, the kernel-time sum and per kernel: launches, mean us, total us."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker, k = sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1
by_grid = "--grid" in sys.argv   # one line per (kernel, grid size)
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
if len(idx) < k:
    raise SystemExit(f"{len(idx)} launches match {marker!r}")
a = idx[-k]
b = idx[-k + 1] if k > 1 else len(rows)
seq = rows[a:b]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in seq:
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("orbhip::", "")
    name = name[5:] if name.startswith("void ") else name
    name = name.split("(")[0]
    if by_grid:
        name += f" [{r['Grid_Size_X']}x{r['Grid_Size_Y']}]"
    agg[name][0] += 1
    agg[name][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1000
print(f"== window {marker!r} #{k} from the end: {len(seq)} launches, span {span:.1f} us, "
      f"kernel sum {sum(v[1] for v in agg.values()):.1f} us")
for name, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"  {name[:60]:60s} {v[0]:5d} {v[1] / v[0]:9.2f} {v[1]:9.1f}")

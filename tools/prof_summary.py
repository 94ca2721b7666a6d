#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into the committed files under profiles/.

  python tools/prof_summary.py stats  <kernel_stats.csv> <out.md> [title]
  python tools/prof_summary.py traffic <fetch counter_collection.csv> <write counter_collection.csv> <out.json>

`traffic` follows MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes (they do not fit one TCC pass), both are in KB, and on gfx950 FETCH_SIZE
reports half the bytes of a wide coalesced read, so it is doubled. Per-launch values are the
mean over every dispatch of a kernel in the pass.
"""
import csv
import json
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    m = re.match(r"(?:void )?(?:[\w:]+::)?(\w+)(?:<.*)?\(", name)
    return m.group(1) if m else name[:60]


def stats(src, dst, title="kernel stats"):
    rows = list(csv.DictReader(open(src)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    with open(dst, "w") as f:
        f.write(f"# {title}\n\nSource: `rocprofv3 --kernel-trace --stats --output-format csv` (`{src.split('/')[-1]}`).\n\n")
        f.write("| kernel | calls | avg us | min us | max us | total ms | % |\n|---|---:|---:|---:|---:|---:|---:|\n")
        for r in rows:
            f.write(f"| {short(r['Name'])} | {r['Calls']} | {float(r['AverageNs'])/1e3:.2f} | {float(r['MinNs'])/1e3:.2f} | "
                    f"{float(r['MaxNs'])/1e3:.2f} | {float(r['TotalDurationNs'])/1e6:.3f} | {100*float(r['TotalDurationNs'])/tot:.2f} |\n")


def per_kernel(src, counter):
    acc = defaultdict(list)
    for r in csv.DictReader(open(src)):
        if r["Counter_Name"] == counter:
            acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return acc


def traffic(fetch_src, write_src, dst):
    fe, wr = per_kernel(fetch_src, "FETCH_SIZE"), per_kernel(write_src, "WRITE_SIZE")
    out = {"source": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes of "
                     "`python3 bench.py --steps 100 --warmup 10 --no-cpu --no-extra`",
           "correction": "FETCH_SIZE (KB) x 2 (gfx950 wide-read undercount) + WRITE_SIZE (KB); x1024 -> bytes",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        out["kernels"][k] = {"dispatches": max(len(fe.get(k, [])), len(wr.get(k, []))),
                             "fetch_kb_raw": round(f, 3), "write_kb": round(w, 3),
                             "hbm_bytes_per_launch": int(round((2 * f + w) * 1024))}
    json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3], *(sys.argv[4:5] or ["kernel stats"]))
    else:
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])

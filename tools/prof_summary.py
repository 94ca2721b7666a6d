#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into the committed files under profiles/.

  python tools/prof_summary.py stats  <kernel_stats.csv> <out.md> [title]
  python tools/prof_summary.py sections <kernel_trace.csv> <out.md> <warmup> <steps>
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
    name = name.replace("(anonymous namespace)::", "")
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


def traffic(fetch_src, write_src, dst, regime="c2"):
    fe, wr = per_kernel(fetch_src, "FETCH_SIZE"), per_kernel(write_src, "WRITE_SIZE")
    out = {"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE, separate passes of "
                     f"`python3 tools/pmc_workload.py {regime}` (tools/gpu_pmc.sh)",
           "correction": "FETCH_SIZE (KB) x 2 (gfx950 wide-read undercount) + WRITE_SIZE (KB); x1024 -> bytes",
           "kernels": {}}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0])) / max(len(wr.get(k, [])), 1)
        out["kernels"][k] = {"dispatches": max(len(fe.get(k, [])), len(wr.get(k, []))),
                             "fetch_kb_raw": round(f, 3), "write_kb": round(w, 3),
                             "hbm_bytes_per_launch": int(round((2 * f + w) * 1024))}
    json.dump(out, open(dst, "w"), indent=1)


def durations(trace_csv):
    acc = defaultdict(list)
    for r in csv.DictReader(open(trace_csv)):
        acc[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
    return acc


def sections(trace_csv, dst, warmup, steps):
    """Append to `dst` the C2 section's per-kernel averages split by bench phase.

    The camera streams are the streams with warmup + 2 * steps launches of a kernel (bench.py
    c2_headline: W warmup frames, K timed frames, K stage-replay frames per camera); their
    launches are split in issue order. Everything else (the one-camera figures) is one row."""
    per = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(trace_csv)):
        per[r["Stream_Id"]][short(r["Kernel_Name"])].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    n_cam = warmup + 2 * steps
    cams = [s for s, ks in per.items() if any(len(v) == n_cam for v in ks.values())]
    acc = defaultdict(lambda: defaultdict(list))
    for s, ks in per.items():
        for k, v in ks.items():
            v.sort()
            d = [(e - b) / 1e3 for b, e in v]
            if s in cams and len(v) >= n_cam - 1:
                acc[k]["timed"] += d[warmup:warmup + steps]
                acc[k]["replay"] += d[warmup + steps:]
            else:
                acc[k]["other"] += d
    with open(dst, "a") as f:
        f.write(f"\n## By bench phase ({len(cams)} camera streams; W = {warmup}, K = {steps} frames per camera)\n\n"
                "From the kernel trace (`*_kernel_trace.csv`, End - Start per dispatch). `timed` = the K frames "
                "of the timed region, `replay` = the K frames of the stage replay whose stage timer gives the "
                "bench's `avg_launch_ms`, `other` = the one-camera figures after the camera streams close.\n\n"
                "| kernel | timed n | timed avg us | replay n | replay avg us | other n | other avg us |\n"
                "|---|---:|---:|---:|---:|---:|---:|\n")
        for k in sorted(acc, key=lambda k: -sum(acc[k]["timed"])):
            cells = []
            for ph in ("timed", "replay", "other"):
                v = acc[k][ph]
                cells += [str(len(v)), f"{sum(v) / len(v):.2f}" if v else "-"]
            f.write(f"| {k} | " + " | ".join(cells) + " |\n")


SIMDS, CUS = 1024, 256
FP64_MFMA_PEAK_TFS = 78.6


def counters(pmc_dir, dst, regimes):
    """VALU / LDS / MFMA activity per launch from the p1 / p2 passes of each regime.

    Units (MI355X_MICROARCH.md, PMC slots and cycle constants): SQ_INSTS_* count wave-instructions;
    SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles summed over waves;
    GRBM_GUI_ACTIVE is the dispatch's GPU-busy cycles summed over the 8 XCDs (so / 8 = cycles).
    Derived, chip-wide over the kernel's busy cycles C = GRBM_GUI_ACTIVE / 8:
      valu_issue_frac = SQ_INSTS_VALU / (1024 SIMDs x C / 2)   a wave64 VALU op holds a SIMD-32 2 cycles
      lds_issue_frac  = SQ_INSTS_LDS / (256 CUs x C)           one LDS instruction per CU per cycle
      f64 MFMA TF/s   = SQ_INSTS_VALU_MFMA_MOPS_F64 x 512 / duration, against the 78.6 TF fp64 peak
      stall split     = SQ_WAIT_ANY, SQ_WAIT_INST_ANY, SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
    """
    import glob
    out = {"source": "rocprofv3 --kernel-trace --pmc, two SQ passes per regime (tools/gpu_pmc.sh); "
                     "per-launch means over every dispatch of the kernel in the pass",
           "definitions": counters.__doc__, "regimes": {}}
    for rg in regimes:
        res = {}
        data = {}
        for ps in ("p1", "p2"):
            src = glob.glob(f"{pmc_dir}/{rg}_{ps}/**/*counter_collection.csv", recursive=True)
            tr = glob.glob(f"{pmc_dir}/{rg}_{ps}/**/*kernel_trace.csv", recursive=True)
            if not src:
                continue
            names = set(r["Counter_Name"] for r in csv.DictReader(open(src[0])))
            for c in names:
                for k, v in per_kernel(src[0], c).items():
                    data.setdefault(k, {})[c] = sum(v) / len(v)
            if tr and ps == "p1":
                for k, v in durations(tr[0]).items():
                    data.setdefault(k, {})["dur_s"] = sum(v) / len(v)
        for k, d in data.items():
            g = d.get("GRBM_GUI_ACTIVE", 0.0)
            cyc = g / 8.0
            e = {"duration_us": round(1e6 * d.get("dur_s", 0.0), 3), "busy_cycles": round(cyc, 1)}
            for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_MFMA",
                      "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS", "SQ_INSTS_VALU_MFMA_MOPS_F64",
                      "SQ_VALU_MFMA_BUSY_CYCLES"):
                if c in d:
                    e[c] = round(d[c], 1)
            if cyc > 0:
                if "SQ_INSTS_VALU" in d:
                    e["valu_issue_frac"] = round(d["SQ_INSTS_VALU"] / (SIMDS * cyc / 2), 5)
                if "SQ_INSTS_LDS" in d:
                    e["lds_issue_frac"] = round(d["SQ_INSTS_LDS"] / (CUS * cyc), 5)
            if d.get("SQ_ACTIVE_INST_LDS"):
                e["lds_bank_conflict_per_active_lds_cycle"] = round(d.get("SQ_LDS_BANK_CONFLICT", 0) /
                                                                     d["SQ_ACTIVE_INST_LDS"], 4)
            if d.get("SQ_WAVE_CYCLES"):
                wc = d["SQ_WAVE_CYCLES"]
                e["wave_time_split"] = {"waiting": round(d.get("SQ_WAIT_ANY", 0) / wc, 4),
                                        "issue_stalled": round(d.get("SQ_WAIT_INST_ANY", 0) / wc, 4),
                                        "issuing": round(d.get("SQ_ACTIVE_INST_ANY", 0) / wc, 4)}
            if d.get("SQ_INSTS_VALU_MFMA_MOPS_F64") and d.get("dur_s"):
                tf = d["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512 / d["dur_s"] / 1e12
                e["f64_mfma_tflops"] = round(tf, 4)
                e["f64_mfma_frac_of_peak"] = round(tf / FP64_MFMA_PEAK_TFS, 6)
            res[k] = e
        out["regimes"][rg] = res
    json.dump(out, open(dst, "w"), indent=1)


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3], *(sys.argv[4:5] or ["kernel stats"]))
    elif sys.argv[1] == "sections":
        sections(sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5]))
    elif sys.argv[1] == "counters":
        counters(sys.argv[2], sys.argv[3], sys.argv[4:])
    else:
        traffic(sys.argv[2], sys.argv[3], sys.argv[4], *(sys.argv[5:6] or ["c2"]))

#!/usr/bin/env python3
"""C4 LBA latency while a C5 GBA runs on another context (two host threads, two streams: the
persistent Cholesky launches of the device are ordered between them, DESIGN.md §4 'concurrent
contexts'), against each alone. ORBHIP_DAG_HANDOFF_TAIL=1 selects r04's hand-off (wait for the
other stream's whole queued tail) for the A/B."""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import Optimizer  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem  # noqa: E402

gba_p, _ = synthetic_ba_problem(n_kf=400, n_pts=20000, layout="loop", window=20, seed=11)
lba_p, _ = synthetic_ba_problem()
gba, lba = Optimizer(), Optimizer()
gba.BundleAdjustment(gba_p, nIterations=10)
lba.LocalBundleAdjustment(lba_p)


def lba_times(n):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        lba.LocalBundleAdjustment(lba_p)
        ts.append(time.perf_counter() - t)
    return np.array(ts) * 1e3


def gba_times(n):
    ts = []
    for _ in range(n):
        t = time.perf_counter()
        gba.BundleAdjustment(gba_p, nIterations=10)
        ts.append(time.perf_counter() - t)
    return np.array(ts) * 1e3


la = lba_times(30)
ga = gba_times(10)
res = {}
done = threading.Event()


def run_gba():
    res["gba"] = gba_times(20)
    done.set()


def run_lba():
    ts = []
    while not done.is_set():
        t = time.perf_counter()
        lba.LocalBundleAdjustment(lba_p)
        ts.append(time.perf_counter() - t)
    res["lba"] = np.array(ts) * 1e3


th = [threading.Thread(target=run_gba), threading.Thread(target=run_lba)]
for t in th:
    t.start()
for t in th:
    t.join()
lc, gc = res["lba"], res["gba"]
mode = "tail" if os.environ.get("ORBHIP_DAG_HANDOFF_TAIL") else "after-launch"
print(f"hand-off {mode}: LBA alone median {np.median(la):.3f} ms p90 {np.percentile(la, 90):.3f} | "
      f"LBA during GBA median {np.median(lc):.3f} ms p90 {np.percentile(lc, 90):.3f} max {lc.max():.3f} ({lc.size} solves) | "
      f"GBA alone {np.median(ga):.2f} ms, with LBAs {np.median(gc):.2f} ms | handoffs {gba.stats()['dag_handoffs']}",
      flush=True)

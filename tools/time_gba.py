#!/usr/bin/env python3
"""Time GlobalBundleAdjustment (C5: 400 KF loop / 20k points / ~80k obs, 20-KF co-visibility
window) on one GPU, and optionally the oracle on one CPU core for a few iterations."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import Optimizer  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem  # noqa: E402

n_kf = int(sys.argv[1]) if len(sys.argv) > 1 else 400
n_pts = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
iters = int(sys.argv[3]) if len(sys.argv) > 3 else 10
t = time.perf_counter()
prob, _ = synthetic_ba_problem(n_kf=n_kf, n_pts=n_pts, layout="loop", window=20, seed=11)
print(f"problem: {n_kf} KF, {n_pts} pts, {prob.edge_pose.shape[0]} obs ({time.perf_counter() - t:.1f}s to build)")
opt = Optimizer()
opt.BundleAdjustment(prob, nIterations=1)
ts = []
for _ in range(5):
    t = time.perf_counter()
    r = opt.BundleAdjustment(prob, nIterations=iters)
    ts.append(time.perf_counter() - t)
print(f"GBA {iters} it: {np.median(ts)*1e3:.2f} ms median of 5 (min {min(ts)*1e3:.2f})  trials={r.lm_trials} "
      f"chi2 {r.initial_chi2:.1f} -> {r.final_chi2:.1f}  ND_K={os.environ.get('ORBHIP_ND_K', 'auto')} "
      f"levels={os.environ.get('ORBHIP_ND_LEVELS', '2')}")

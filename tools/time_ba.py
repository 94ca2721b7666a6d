#!/usr/bin/env python3
"""Time the C4 LocalBundleAdjustment on the GPU (and optionally profile it)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import Optimizer  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B = int(sys.argv[2]) if len(sys.argv) > 2 else 0
prob, _ = synthetic_ba_problem()
opt = Optimizer()
for _ in range(2):
    r = opt.LocalBundleAdjustment(prob)
t = time.perf_counter()
for _ in range(n):
    r = opt.LocalBundleAdjustment(prob)
dt = (time.perf_counter() - t) / n
print(f"LBA C4: {dt*1e3:.3f} ms/solve  {1/dt:.1f} LBA/s  trials={r.lm_trials} chi2 {r.initial_chi2:.1f}->{r.final_chi2:.1f}")
if B > 0:
    probs = [synthetic_ba_problem(seed=7 + i)[0] for i in range(B)]
    batch = opt.prepare_batch(probs)
    opt.run_batch(batch)   # warm-up at full size (pinned staging grows once)
    t = time.perf_counter()
    rs = opt.run_batch(batch)
    dt = time.perf_counter() - t
    print(f"LBA C4 batch of {B}: {dt*1e3:.2f} ms  {B/dt:.1f} LBA/s  trials={[r.lm_trials for r in rs[:4]]}")

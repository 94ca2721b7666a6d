#!/usr/bin/env python3
"""Time Optimizer::PoseOptimization on the GPU (batched, one wavefront per frame) and the oracle."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import Optimizer  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_pose_problem  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
n = int(sys.argv[2]) if len(sys.argv) > 2 else 600
probs = [synthetic_pose_problem(n=n, outlier_frac=0.15, seed=1000 + i)[0] for i in range(B)]
opt = Optimizer()
opt.PoseOptimization(probs[0])
t = time.perf_counter()
for _ in range(20):
    opt.PoseOptimization(probs[0])
dt1 = (time.perf_counter() - t) / 20
rates = {}
for w in ("1", "4"):
    os.environ["ORBHIP_POSE_WAVES"] = w
    opt.PoseOptimization_batch(probs)
    t = time.perf_counter()
    rs = opt.PoseOptimization_batch(probs)
    rates[w] = B / (time.perf_counter() - t)
os.environ.pop("ORBHIP_POSE_WAVES")
t = time.perf_counter()
k = 0
while time.perf_counter() - t < 2.0:
    O.pose_optimization(probs[k % B]); k += 1
dto = (time.perf_counter() - t) / k
print(f"PoseOptimization n={n}: single {dt1*1e3:.3f} ms; batch of {B}: W=1 {rates['1']:.0f}, W=4 {rates['4']:.0f} frames/s; "
      f"oracle 1 core {dto*1e3:.3f} ms/frame; trials mean {sum(r.lm_trials for r in rs)/B:.1f}")

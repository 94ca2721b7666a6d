#!/usr/bin/env python3
"""Short fixed workloads for the rocprofv3 --pmc passes (tools/gpu_pmc.sh), one regime each so a
kernel's counters are not mixed across regimes:

  c2    the bench's C2 stream: 16 cameras (640x480, extract + match to the camera's previous
        frame), 40 steps of one frame per camera, as in the bench's timed region
  c3    the bench's C3 batch (1280x720, B=64, extract + 63 pair matches), 96 batches
        (PMC_C3_STEPS): k_fast_cells averages 368 us over the first 16 batches after start, 348
        over 96, against the bench's warm 345 (profiles/r05_pmc_c3_kernel_stats.md)
  c4    the C4-sized dense reduced camera system (n = 294) solved by k_chol_dag, 2 x 21 solves
  c4lba C4 LocalBundleAdjustment (50 KF / 2000 pts / 8000 obs, 10 LM iterations), 3 solves
  c5    the C5-sized dense reduced camera system (n = 2394) solved by k_chol_dag, 2 x 21 solves
  c5nd  the nested-dissection solve the C5 GBA runs (399 poses, cyclic band 19), 2 x 61 solves
"""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402

mode = sys.argv[1]
if mode == "c2":
    s = bench.FrontendC2(0, 1, 16)
    for _ in range(40):
        s.step()
elif mode == "c3":
    c3 = bench.BatchC3(0, 1)
    for _ in range(int(os.environ.get("PMC_C3_STEPS", "96"))):
        c3.step()
elif mode == "c4":
    for _ in range(2):
        bench.ba_cholesky_roofline(294, "c4")
elif mode == "c4lba":
    from orb_slam3_ros2_amd import Optimizer
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem()
    opt = Optimizer()
    for _ in range(3):
        opt.LocalBundleAdjustment(prob)
elif mode == "c5":
    for _ in range(2):
        bench.ba_cholesky_roofline(2394, "c5")
elif mode == "c5nd":
    for _ in range(2):
        bench.ba_nd_roofline()
else:
    raise SystemExit(f"unknown mode {mode}")
torch.cuda.synchronize()
print("workload", mode, "done")

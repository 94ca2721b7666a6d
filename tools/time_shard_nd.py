#!/usr/bin/env python3
"""Time the sharded C5 GBA by keyframe segments on one GPU: K in-process shards
(orbhip_ba_solve_shards_local; the collectives are k_ba_multi_reduce), the one-GPU nested
dissection for reference, and (r06) K landmark shards whose summed S every shard solves (the
replicated form) by nested dissection or by the plain DAG solve. Run under rocprofv3 --kernel-trace to get the
per-rank pieces (one segment's k_chol_dag_multi, the separator k_chol_dag, the assembly and
back-substitution) for the modelled N-rank trial."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
from orb_slam3_ros2_amd import Optimizer  # noqa: E402
from orb_slam3_ros2_amd.optimizer import BAProblem  # noqa: E402
from orb_slam3_ros2_amd.sharding import shard_problem, shard_problem_nd  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
prob, _ = synthetic_ba_problem(n_kf=400, n_pts=20000, layout="loop", window=20, seed=11)
p = BAProblem(**{**prob.__dict__, "iterations": 10, "huber_delta": float(np.sqrt(5.99))})
opt = Optimizer()
parts = [shard_problem_nd(p, r, K)[0] for r in range(K)]
lparts = [shard_problem(p, r, K)[0] for r in range(K)]


def landmark(nd):
    os.environ["ORBHIP_ND"] = "1" if nd else "0"   # read per call: the replicated form's solver
    try:
        return opt.solve_shards_local(lparts)
    finally:
        os.environ.pop("ORBHIP_ND", None)


for name, fn in (("one GPU, nested dissection", lambda: opt.solve(p)),
                 (f"{K} in-process segment shards", lambda: opt.solve_shards_local(parts)),
                 (f"{K} in-process landmark shards, summed S dissected", lambda: landmark(True)),
                 (f"{K} in-process landmark shards, summed S on the DAG", lambda: landmark(False))):
    fn()
    t = time.perf_counter()
    r = fn()
    dt = time.perf_counter() - t
    r0 = r[0] if isinstance(r, list) else r
    print(f"{name}: {dt * 1e3:.2f} ms  trials={r0.lm_trials} chi2 {r0.initial_chi2:.1f} -> {r0.final_chi2:.1f}",
          flush=True)

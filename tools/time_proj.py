#!/usr/bin/env python3
"""Time the projection matchers (GPU, host-buffer API) against the oracle on one core."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import ORBmatcher  # noqa: E402
from orb_slam3_ros2_amd.matcher import ProjFrame  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_projection_scene  # noqa: E402
from oracle import pyoracle as O  # noqa: E402

s = synthetic_projection_scene(n_kp=1250, n_mp=1000, seed=77)
f = ProjFrame(s["kps"], s["desc"], s["pose_q"], s["pose_t"], s["fx"], s["fy"], s["cx"], s["cy"], claimed=s["claimed"])
mt = ORBmatcher(0.9, True)


def bench(fn, reps=20):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        r = fn()
    return (time.perf_counter() - t) / reps * 1e3, r


g1, r1 = bench(lambda: mt.SearchByProjectionLastFrame(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"]))
o1, _ = bench(lambda: O.search_by_projection_last(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"]))
mt2 = ORBmatcher(0.8, False)
g2, r2 = bench(lambda: mt2.SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                             s["skip"], th=1.0))
o2, _ = bench(lambda: O.search_local_points(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                            s["skip"], th=1.0, nnratio=0.8))
print(f"SearchByProjection(last) 1250 kps x 1000 pts: GPU {g1:.3f} ms ({r1[0]} matches), oracle 1 core {o1:.3f} ms")
print(f"SearchLocalPoints 1250 kps x 1000 pts: GPU {g2:.3f} ms ({r2[0]} matches), oracle 1 core {o2:.3f} ms")

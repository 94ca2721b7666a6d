#!/usr/bin/env python3
"""SearchLocalPoints latency split: the Python call, the bare C call (arguments built once), and
the C call's parts (kernels from a rocprofv3 kernel trace of this script)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import ORBmatcher  # noqa: E402
from orb_slam3_ros2_amd._lib import LocalPointsC, lib, ptr  # noqa: E402
from orb_slam3_ros2_amd.matcher import ProjFrame  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_projection_scene  # noqa: E402

s = synthetic_projection_scene(n_kp=1250, n_mp=1000, seed=77)
f = ProjFrame(s["kps"], s["desc"], s["pose_q"], s["pose_t"], s["fx"], s["fy"], s["cx"], s["cy"], claimed=s["claimed"])
mt = ORBmatcher(0.8, False)


def t(fn, reps=200):
    fn()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    return (time.perf_counter() - t0) / reps * 1e6


py = t(lambda: mt.SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                    s["skip"], th=1.0))
pts = np.ascontiguousarray(s["points"], np.float32)
nrm = np.ascontiguousarray(s["normals"], np.float32)
mn = np.ascontiguousarray(s["min_dist"], np.float32)
mx = np.ascontiguousarray(s["max_dist"], np.float32)
d = np.ascontiguousarray(s["mp_desc"], np.uint8)
sk = np.ascontiguousarray(s["skip"], np.uint8)
m = pts.shape[0]
match = np.full(m, -1, np.int32)
iv = np.zeros(m, np.uint8)
lvl = np.full(m, -1, np.int32)
fc = f.to_c()
lc = LocalPointsC(m, ptr(pts), ptr(nrm), ptr(mn), ptr(mx), ptr(d), ptr(sk))
L = lib()
h = mt.ctx.handle
fcr, lcr = ctypes.byref(fc), ctypes.byref(lc)
a = (ptr(iv), ptr(lvl), ptr(match))
c = t(lambda: L.orbhip_search_local_points(h, fcr, lcr, 0.5, 1.0, 0.8, 0, 0.0, *a))
prep = t(lambda: (f.to_c(), np.full(m, -1, np.int32), np.zeros(m, np.uint8), np.full(m, -1, np.int32)))
print(f"SearchLocalPoints: python call {py:.1f} us, bare C call {c:.1f} us, to_c + output arrays {prep:.1f} us")

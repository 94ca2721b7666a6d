#!/usr/bin/env python3
"""Device timing trace of one SearchLocalPoints call (f8 workload: 1250 keypoints x 1000 map
points): k_proj_lists work-group spread, work-group 0's phases (1 staging, 2 window scan, 3
descriptors + list stores, 4 arrival, 5 the window before the scan, which 2 then excludes) and
the resolving work-group's phases (16 offsets + counts, 17 list entries to LDS, 18 fixed-point
rounds, 20 rotation filter + count, 21 outputs), in cycles."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import ORBmatcher  # noqa: E402
from orb_slam3_ros2_amd._lib import lib  # noqa: E402
from orb_slam3_ros2_amd.matcher import ProjFrame  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_projection_scene  # noqa: E402

STRIDE, NK, KID = 16384, 8, 7
s = synthetic_projection_scene(n_kp=1250, n_mp=1000, seed=77)
f = ProjFrame(s["kps"], s["desc"], s["pose_q"], s["pose_t"], s["fx"], s["fy"], s["cx"], s["cy"], claimed=s["claimed"])
mt = ORBmatcher(0.8, False)
L = lib()
L.orbhip_test_trace.argtypes = [ctypes.c_int, ctypes.c_void_p]


def call():
    return mt.SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"], s["skip"],
                                th=1.0)


for _ in range(50):
    call()
for rep in range(3):
    assert L.orbhip_test_trace(1, None) == 0
    n = call()[0]
    buf = np.zeros(NK * STRIDE, np.uint64)
    assert L.orbhip_test_trace(0, buf.ctypes.data) == 0
    seg = buf[KID * STRIDE: KID * STRIDE + 8192].reshape(-1, 2).astype(np.int64)
    ok = seg[:, 1] > 0
    st, en = seg[ok, 0], seg[ok, 1]
    t0 = st.min()
    dur = (en - st) / 100.0
    last = int(np.argmax(en))
    ph = buf[KID * STRIDE + 8192: KID * STRIDE + 8192 + 32].astype(np.int64)
    print(f"matches {n}: wgs={len(st)} span={(en.max() - t0) / 100:.2f}us start skew={(st.max() - t0) / 100:.2f}us "
          f"wg dur min/med/max={dur.min():.2f}/{np.median(dur):.2f}/{dur.max():.2f}us; resolving wg {last} "
          f"starts {(st[last] - t0) / 100:.2f} ends {(en[last] - t0) / 100:.2f}us; second-latest end "
          f"{(np.sort(en)[-2] - t0) / 100:.2f}us")
    print("   wg0 phases: " + ", ".join(f"{i}:{ph[i]}" for i in range(1, 6)) + " | resolve: " +
          ", ".join(f"{i}:{ph[i]}" for i in range(16, 22)))

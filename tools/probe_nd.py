#!/usr/bin/env python3
"""Time the nested-dissection solve (ba_nd.hip) on a C5-structured system (399 optimised poses,
cyclic band of 19) for several segment counts, against the plain persistent DAG solve."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_nd_gpu import banded_system, nd_solve  # noqa: E402
from orb_slam3_ros2_amd._lib import lib  # noqa: E402

n_pose, w = (int(a) for a in (sys.argv[1:3] if len(sys.argv) > 2 else (399, 19)))
A, b, bi, bj = banded_system(n_pose, w, True, seed=1)
ref = np.linalg.solve(A, b)
L = lib()
x = np.zeros(A.shape[0])
ms = ctypes.c_float(0)
rc = L.orbhip_test_cholesky_dag(A.ctypes.data, b.ctypes.data, x.ctypes.data, A.shape[0], 20, 0, ctypes.byref(ms), None)
print(f"plain DAG n={A.shape[0]}: rc={rc} {ms.value * 1e3:.1f} us err={np.abs(x - ref).max() / np.abs(ref).max():.1e}")
for K in [0, 2, 3, 4, 5, 6, 8, 10, 12, 16]:
    rc, x, t, ku = nd_solve(A, b, n_pose, bi, bj, K, reps=20)
    err = np.abs(x - ref).max() / np.abs(ref).max() if rc == 0 else float("nan")
    print(f"nd K={K} (used {ku}): rc={rc} {t * 1e3:.1f} us err={err:.1e}", flush=True)

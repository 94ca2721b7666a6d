#!/usr/bin/env python3
"""Product-build timing of the persistent DAG solve (k_chol_dag, no debug stamps): device us per
solve at the given sizes (dense SPD), median of 5 calls of `reps` solves each. ORBHIP_LIB selects
an A/B build of the library."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402

L = lib()
f = L.orbhip_test_cholesky_dag
f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
for n in [int(a) for a in (sys.argv[1:] or ["294", "342"])]:
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.normal(size=n)
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    ts = []
    for _ in range(5):
        assert f(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, 20, 0, ctypes.byref(ms), None) == 0
        ts.append(ms.value * 1e3)
    err = np.abs(x - np.linalg.solve(A, b)).max() / np.abs(np.linalg.solve(A, b)).max()
    print(f"n={n}: {np.median(ts):.1f} us per solve (min {min(ts):.1f}) relerr {err:.1e}", flush=True)

#!/usr/bin/env python3
"""Diagnostic: time the single-workgroup Cholesky kernel per phase on random SPD systems."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402

L = lib()
L.orbhip_test_cholesky.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
for n in [int(a) for a in (sys.argv[1:] or ["294", "294", "31", "100", "480"])]:
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.normal(size=n)
    x = np.zeros(n)
    ph = np.zeros(5, np.uint64)
    ms = ctypes.c_float(0)
    rc = L.orbhip_test_cholesky(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, ph.ctypes.data, ctypes.byref(ms))
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    print(f"n={n} rc={rc} {ms.value*1e3:.1f} us relerr={err:.2e} cycles: diag={ph[0]} panel={ph[1]} "
          f"trailing={ph[2]} backsolve={ph[3]}", flush=True)

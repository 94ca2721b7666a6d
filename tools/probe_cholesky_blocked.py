#!/usr/bin/env python3
"""Diagnostic: blocked multi-workgroup Cholesky solve on random SPD systems, dense and banded
(cyclic band + loop-closure corner, the GBA C5 structure)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402

L = lib()
L.orbhip_test_cholesky_blocked.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p]


def run(A, b, tag):
    n = A.shape[0]
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    for _ in range(2):   # second run is warm
        rc = L.orbhip_test_cholesky_blocked(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, ctypes.byref(ms))
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    print(f"{tag} n={n} rc={rc} {ms.value*1e3:.1f} us relerr={err:.2e}", flush=True)
    return err


for n in [int(a) for a in (sys.argv[1:] or ["294", "500", "1000", "2394"])]:
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.normal(size=n)
    run(A, b, "dense ")
    # cyclic band of 20 poses (120 rows) wrapping around: the C5 loop
    bw = 120
    idx = np.arange(n)
    d = np.abs(idx[:, None] - idx[None, :])
    mask = np.minimum(d, n - d) < bw
    Bm = np.where(mask, rng.normal(size=(n, n)), 0.0)
    A2 = Bm @ Bm.T
    A2 = np.where(mask | (np.abs(A2) > 0), A2, 0.0) + n * np.eye(n)
    run(A2, b, "banded")

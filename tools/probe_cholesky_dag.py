#!/usr/bin/env python3
"""Probe the persistent tiled-DAG Cholesky (ba_chol_dag.hip) against numpy: dense, banded and
band + loop-corner SPD systems; device us per solve and the chain workgroup's phase cycles
(s_memtime: prologue, forward, backward, poll waits, diag32 sum)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402


def spd(n, shape, rng):
    if shape == "dense":
        M = rng.normal(size=(n, n))
        return M @ M.T + n * np.eye(n)
    bw = 120
    M = np.zeros((n, n))
    for i in range(n):
        lo = max(0, i - bw)
        M[i, lo:i + 1] = rng.normal(size=i + 1 - lo)
    if shape == "loop":
        M[n - 120:, :120] = rng.normal(size=(120, 120)) * 0.3
    return M @ M.T + n * np.eye(n)


L = lib()
cases = [a.split(":") for a in (sys.argv[1:] or ["31:dense", "100:dense", "294:dense", "600:band", "2394:loop", "2394:dense"])]
for n_s, shape in cases:
    n = int(n_s)
    rng = np.random.default_rng(n)
    A = spd(n, shape, rng)
    A = 0.5 * (A + A.T)
    b = rng.normal(size=n)
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    dbg = np.zeros(8 + 256, np.uint64)
    t0 = time.time()
    rc = L.orbhip_test_cholesky_dag(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, 10, 0, ctypes.byref(ms),
                                    dbg.ctypes.data)
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    nt = (n + 31) // 32
    ks = dbg[8:8 + nt - 1]
    print(f"n={n} {shape}: rc={rc} dag {ms.value * 1e3:.1f} us relerr={err:.2e} | cycles prologue={dbg[0]} "
          f"forward={dbg[1]} backward={dbg[2]} waits={dbg[3]} diag={dbg[4]} total={dbg[5]} | interval "
          f"min/med/max {ks.min() if len(ks) else 0}/{int(np.median(ks)) if len(ks) else 0}/{ks.max() if len(ks) else 0} "
          f"({time.time() - t0:.1f}s)", flush=True)

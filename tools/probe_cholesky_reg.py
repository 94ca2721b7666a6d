#!/usr/bin/env python3
"""Diagnostic: time the register-resident single-workgroup Cholesky (ba_chol_reg.hip) against
numpy on random SPD systems, and the previous LDS-panel solver on the same systems."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402

L = ctypes.CDLL(os.environ["ORBHIP_PROBE_LIB"]) if os.environ.get("ORBHIP_PROBE_LIB") else lib()
L.orbhip_test_cholesky_reg.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
L.orbhip_test_cholesky.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
for n in [int(a) for a in (sys.argv[1:] or ["6", "31", "100", "160", "240", "294", "304"])]:
    rng = np.random.default_rng(n)
    M = rng.normal(size=(n, n))
    A = M @ M.T + n * np.eye(n)
    b = rng.normal(size=n)
    ref = np.linalg.solve(A, b)
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    phr = np.zeros(48, np.uint64)
    rc = L.orbhip_test_cholesky_reg(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, 20, ctypes.byref(ms),
                                    phr.ctypes.data)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    x2 = np.zeros(n)
    ph = np.zeros(5, np.uint64)
    ms2 = ctypes.c_float(0)
    L.orbhip_test_cholesky(A.ctypes.data, b.ctypes.data, x2.ctypes.data, n, ph.ctypes.data, ctypes.byref(ms2))
    print(f"n={n} rc={rc} reg {ms.value*1e3:.1f} us relerr={err:.2e} | lds-panel {ms2.value*1e3:.1f} us | reg cycles: load+diag0={phr[0]} panels={phr[1]} "
          f"trailing={phr[2]} back={phr[3]} diag-sum={phr[4]} [pre={phr[5]} elim={phr[6]} epilogue={phr[7]}]", flush=True)
    pw = phr[8:48].reshape(8, 5)
    print("   per wave [load, panel, trailing(+own diag), back, diag]:", pw.tolist(), flush=True)

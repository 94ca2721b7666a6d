"""Host preparation of the BA problems (ba_solver.hip prepare) at the C4 and C5 sizes: the serial
build into a fresh Prep, into a reused one, and the threaded pair build (orbhip_test_ba_prepare;
host code only)."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem  # noqa: E402

f = lib().orbhip_test_ba_prepare
f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
for name, kw in (("C4", {}), ("C5", dict(n_kf=400, n_pts=20000, layout="loop", window=20, seed=11))):
    prob, _ = synthetic_ba_problem(**kw)
    pn = prob.normalized()
    pc = pn.to_c()
    out = np.zeros(4)
    for t in (1, 4, 8, 16):
        fresh, reused = [], []
        for _ in range(10):
            rc = f(ctypes.addressof(pc), t, out.ctypes.data)
            assert rc == 0, rc
            if t == 1:
                fresh.append(out[2]); reused.append(out[3])
            else:
                reused.append(out[3])
        if t == 1:
            print(f"{name}: serial fresh {np.median(fresh):.3f} ms, serial reused {np.median(reused):.3f} ms", flush=True)
        else:
            print(f"{name}: threaded x{t} {np.median(reused):.3f} ms", flush=True)

"""Nested-dissection solve time at the C5 band (399 poses, cyclic w = 19) per segment count K and
dissection depth (ORBHIP_ND_LEVELS 1 / 2): whole solve, interiors + assembly, separator + back-
substitution (orbhip_test_nd_stages, HIP events over `reps` solves). K = 0: the planner's choice."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402
from orb_slam3_ros2_amd.synthetic import banded_pose_system  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    A, b, bi, bj = banded_pose_system(399, 19, True, seed=1)
    ref = np.linalg.solve(A, b)
    f = lib().orbhip_test_nd_stages
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 3 + \
        [ctypes.c_void_p] * 4
    for levels in ("1", "2"):
        os.environ["ORBHIP_ND_LEVELS"] = levels
        for K in (0, 4, 5, 6, 7, 8, 9, 10):
            x = np.zeros(A.shape[0])
            ms, ku = ctypes.c_float(0), ctypes.c_int(0)
            stage = (ctypes.c_float * 2)()
            seg = (ctypes.c_int * 65)()
            rc = f(A.ctypes.data, b.ctypes.data, x.ctypes.data, 399, bi.ctypes.data, bj.ctypes.data, bi.size, K, reps,
                   ctypes.byref(ms), ctypes.byref(ku), stage, seg)
            err = float(np.abs(x - ref).max() / np.abs(ref).max()) if rc == 0 else -1
            print(f"levels {levels} K {K:2d} (used {ku.value:2d}) rc {rc}: solve {ms.value * 1e3:7.1f} us  "
                  f"interiors+assembly {stage[0] * 1e3:7.1f}  separator+backsolve {stage[1] * 1e3:7.1f}  err {err:.1e}",
                  flush=True)


if __name__ == "__main__":
    main()

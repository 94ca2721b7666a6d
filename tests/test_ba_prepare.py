"""The BA host preparation (ba_solver.hip prepare: landmark / pose CSRs, Schur pair lists grouped by
pose block, envelope, work items) built on host threads for a large problem (the C5 GBA) against
the serial build: every list identical, so the device sums run in the same order either way. Host
code only: runs without a GPU."""
import ctypes

import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem


@pytest.mark.parametrize("n_kf,n_pts,layout,window", [(400, 20000, "loop", 20), (120, 6000, "arc", None),
                                                      (60, 30000, "arc", None)])
def test_threaded_prepare_matches_serial(n_kf, n_pts, layout, window):
    from orb_slam3_ros2_amd._lib import lib
    prob, _ = synthetic_ba_problem(n_kf=n_kf, n_pts=n_pts, layout=layout, window=window, seed=11)
    pn = prob.normalized()   # keeps the arrays the C view points into alive
    pc = pn.to_c()
    f = lib().orbhip_test_ba_prepare
    f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    out = np.zeros(4)
    for threads in (2, 5, 16):
        rc = f(ctypes.addressof(pc), threads, out.ctypes.data)
        assert rc == 0, (threads, rc)
        assert out[0] >= n_kf - 1 and out[1] > 0

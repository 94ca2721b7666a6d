import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.lib()
    return pyoracle

@pytest.fixture(scope="session")
def c5_case(oracle):
    """C5 at its full size (BASELINE configs[4]): 400 KF loop / 20k points / 80k obs, 20-KF
    co-visibility window, n = 2394, BundleAdjustment(nIterations=10, bRobust=true); the oracle
    solve (~20 s on one core) is shared by the tests below."""
    import numpy as np
    from orb_slam3_ros2_amd.optimizer import BAProblem
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem(n_kf=400, n_pts=20000, layout="loop", window=20, seed=11)
    p = BAProblem(**{**prob.__dict__, "iterations": 10, "huber_delta": float(np.sqrt(5.99))})
    return prob, p, oracle.ba_solve(p)



# Load torch's HIP runtime before liborbhip.so (see orb_slam3_ros2_amd/_lib.py).
try:
    import torch  # noqa: F401,E402
except Exception:
    pass

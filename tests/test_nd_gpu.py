"""Nested dissection of the reduced camera system (ba_nd.hip; a20 / a22): K partial
factorizations of the segment interiors in one k_chol_dag_multi launch, the separator system's
assembly and solve, the interiors' back-substitution.

The solver is checked against numpy's fp64 solve on pose-structured SPD systems built the way a
GBA's reduced camera system is (a sum of landmark terms over windows of consecutive keyframes, on
a loop or a line), and through GlobalBundleAdjustment against the oracle LM at the C5 size with the
dissection on (the default for a lone banded GBA), forced to other segment counts, and off. The
solver restates the same LL^T in another elimination order: equal to rounding (north_star: 1e-4 on
the BA; here 1e-9 on the linear solve). Parity unpinned by the reference (oracle/ba_oracle.cpp)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def banded_system(n_pose, w, cyclic, seed, n_land=None):
    from orb_slam3_ros2_amd.synthetic import banded_pose_system
    return banded_pose_system(n_pose, w, cyclic, seed, n_land)


def nd_solve(A, b, n_pose, bi, bj, K=0, reps=1):
    from orb_slam3_ros2_amd._lib import lib
    L = lib()
    f = L.orbhip_test_nd_solve
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] + [ctypes.c_void_p] * 2 + [ctypes.c_int] * 3 + \
        [ctypes.c_void_p] * 2
    x = np.zeros(A.shape[0])
    ms = ctypes.c_float(0)
    ku = ctypes.c_int(0)
    A = np.ascontiguousarray(A)
    rc = f(A.ctypes.data, b.ctypes.data, x.ctypes.data, n_pose, bi.ctypes.data, bj.ctypes.data, bi.size, K, reps,
           ctypes.byref(ms), ctypes.byref(ku))
    return rc, x, ms.value, ku.value


@pytest.mark.parametrize("n_pose,w,cyclic,K", [(120, 7, True, 0), (120, 7, True, 2), (120, 7, True, 5),
                                                (96, 5, False, 3), (96, 5, False, 0), (399, 19, True, 0),
                                                (399, 19, True, 8), (200, 3, True, 16)])
def test_nd_solve_matches_numpy(n_pose, w, cyclic, K):
    A, b, bi, bj = banded_system(n_pose, w, cyclic, seed=n_pose + w + K)
    rc, x, ms, ku = nd_solve(A, b, n_pose, bi, bj, K)
    assert rc == 0, rc
    assert K == 0 or ku == K
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    assert err < 1e-9, (err, ku)


@pytest.mark.parametrize("levels", ["1", "2"])
@pytest.mark.parametrize("K", [6, 7, 8, 10])
def test_nd_two_levels_match_numpy(K, levels, monkeypatch):
    """The second level (a cyclic separator system of >= 6 separators dissected once more: even
    separators eliminated by one more k_chol_dag_multi, the odd ones solved densely; K odd: the last
    inner segment holds three separators) against the one-level solve and numpy, at the C5 band."""
    monkeypatch.setenv("ORBHIP_ND_LEVELS", levels)
    A, b, bi, bj = banded_system(399, 19, True, seed=40 + K)
    rc, x, ms, ku = nd_solve(A, b, 399, bi, bj, K)
    assert rc == 0 and ku == K, (rc, ku)
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    assert err < 1e-9, (err, ku)


def test_nd_not_planned_for_a_dense_system():
    A, b, bi, bj = banded_system(60, 40, False, seed=3)
    rc, _, _, _ = nd_solve(A, b, 60, bi, bj, 0)
    assert rc == -5   # ORBHIP_ERR_UNSUPPORTED: the plain solve is the better one


@pytest.mark.parametrize("env", [{}, {"ORBHIP_ND_K": "2"}, {"ORBHIP_ND_K": "8"}, {"ORBHIP_ND": "0"},
                                 {"ORBHIP_ND_K": "8", "ORBHIP_ND_LEVELS": "1"}, {"ORBHIP_ND_K": "7"}])
def test_gba_c5_dissection_parity(c5_case, env, monkeypatch):
    """GlobalBundleAdjustment at the C5 size (n = 2394) with the dissection's default plan, 2 and 8
    segments, and the plain DAG solve: each equal to the oracle LM (schedule identical, 1e-4)."""
    from orb_slam3_ros2_amd import Optimizer
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    prob, p, o = c5_case
    g = Optimizer().BundleAdjustment(prob, nIterations=10, bRobust=True)
    assert g.iterations_done == o["iterations_done"] and g.lm_trials == o["lm_trials"]
    assert abs(g.final_chi2 - o["final_chi2"]) <= 1e-4 * abs(o["final_chi2"])
    q = lambda a: a.astype(np.float64) * np.where(a[:, 3:4] < 0, -1.0, 1.0)   # noqa: E731
    assert np.abs(q(g.pose_q) - q(o["pose_q"])).max() < 1e-4
    assert np.abs(g.pose_t.astype(np.float64) - o["pose_t"]).max() / max(1.0, np.abs(o["pose_t"]).max()) < 1e-4
    assert np.abs(g.points.astype(np.float64) - o["points"]).max() / max(1.0, np.abs(o["points"]).max()) < 1e-4


def test_nd_plan_respects_backsolve_lds():
    """A wide cyclic band near the solver's n = 4096 limit (680 poses, half-bandwidth 114): with
    K = 2 a segment (226-pose interior + two 114-pose separators: 86 tiles) would exceed the
    back-substitution's 128 KB of LDS (84 tiles), so the forced plan is refused up front
    (ORBHIP_ERR_UNSUPPORTED, no device error); the automatic plan either fits or is not made."""
    A, b, bi, bj = banded_system(680, 114, True, seed=7)
    rc, _, _, _ = nd_solve(A, b, 680, bi, bj, 2)
    assert rc == -5, rc
    rc, x, _, ku = nd_solve(A, b, 680, bi, bj, 0)
    assert rc in (0, -5), rc
    if rc == 0:
        ref = np.linalg.solve(A, b)
        assert np.abs(x - ref).max() / np.abs(ref).max() < 1e-9, ku


def test_gba_forced_k2_on_a_wide_band_falls_back(monkeypatch):
    """The same wide band as a GlobalBundleAdjustment (a 681-keyframe loop with a 115-keyframe
    co-visibility window, n = 4080) with ORBHIP_ND_K=2 forced: the planner refuses the segment
    that would not fit the back-substitution's LDS and the solve runs on the plain DAG solver;
    it equals the solve with the dissection off (same solver, same schedule)."""
    from orb_slam3_ros2_amd import Optimizer
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem(n_kf=681, n_pts=6000, layout="loop", window=115, seed=17)
    monkeypatch.setenv("ORBHIP_ND_K", "2")
    g = Optimizer().BundleAdjustment(prob, nIterations=3, bRobust=True)
    monkeypatch.delenv("ORBHIP_ND_K")
    monkeypatch.setenv("ORBHIP_ND", "0")
    r = Optimizer().BundleAdjustment(prob, nIterations=3, bRobust=True)
    assert g.lm_trials == r.lm_trials and g.final_chi2 < g.initial_chi2
    assert abs(g.final_chi2 - r.final_chi2) <= 1e-9 * abs(r.final_chi2)

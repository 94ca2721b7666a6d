"""Optimizer::PoseOptimization (U:src/Optimizer.cc): oracle KATs on the CPU
and the device path (one wavefront per frame) against the oracle on the GPU.

Parity unpinned by the reference (no fixtures upstream); the oracle is pinned by definitional
KATs: exact observations converge to the ground-truth pose, injected gross mismatches are the
outliers, fewer than 3 correspondences leave the pose untouched and return 0.
"""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import _mat_to_quat, synthetic_pose_problem


def _qdist(a, b):
    return 1.0 - abs(float(np.dot(a / np.linalg.norm(a), b / np.linalg.norm(b))))


def test_oracle_exact_observations_converge(oracle):
    prob, gt = synthetic_pose_problem(n=300, outlier_frac=0.0, seed=11)
    Xc = prob.points.astype(np.float64) @ gt["R"].T + gt["t"]
    prob.uv = np.stack([prob.fx * Xc[:, 0] / Xc[:, 2] + prob.cx, prob.fy * Xc[:, 1] / Xc[:, 2] + prob.cy],
                       1).astype(np.float32)
    r = oracle.pose_optimization(prob)
    assert r["n_inliers"] == 300 and not r["outlier"].any()
    assert _qdist(r["pose_q"], _mat_to_quat(gt["R"])) < 1e-9
    assert np.abs(r["pose_t"] - gt["t"]).max() < 1e-4


def test_oracle_flags_the_gross_mismatches(oracle):
    prob, gt = synthetic_pose_problem(n=600, outlier_frac=0.2, seed=12)
    r = oracle.pose_optimization(prob)
    bad = gt["bad"]
    out = r["outlier"].astype(bool)
    # the gross mismatches are outliers; of the good edges only the chi2(2) > 5.991 tail (5%) is
    assert out[bad].mean() > 0.95
    assert out[~bad].mean() < 0.09
    assert r["n_inliers"] == int((r["outlier"] == 0).sum())
    assert _qdist(r["pose_q"], _mat_to_quat(gt["R"])) < 1e-5


def test_oracle_too_few_correspondences(oracle):
    prob, _ = synthetic_pose_problem(n=2, outlier_frac=0.0, seed=13)
    r = oracle.pose_optimization(prob)
    assert r["n_inliers"] == 0 and r["lm_trials"] == 0
    assert np.array_equal(r["pose_t"], prob.pose_t)


def test_oracle_small_frames_stop_after_one_round(oracle):
    # optimizer.edges().size() < 10: one round of optimize(10) only (<= 100 trials)
    prob, _ = synthetic_pose_problem(n=8, outlier_frac=0.0, seed=14)
    r = oracle.pose_optimization(prob)
    big, _ = synthetic_pose_problem(n=40, outlier_frac=0.0, seed=14)
    rb = oracle.pose_optimization(big)
    assert 0 < r["lm_trials"] <= 100 and rb["lm_trials"] > r["lm_trials"]


def _check(g, o, tol=1e-4):
    assert g.n_inliers == o["n_inliers"]
    assert np.array_equal(g.outlier, o["outlier"])
    assert _qdist(g.pose_q, o["pose_q"]) < tol * tol
    assert np.abs(g.pose_t - o["pose_t"]).max() <= tol * max(1.0, float(np.abs(o["pose_t"]).max()))


@pytest.mark.gpu
@pytest.mark.parametrize("waves", ["1", "4"])
def test_pose_optimization_matches_oracle(oracle, monkeypatch, waves):
    # ORBHIP_POSE_WAVES forces the frame-group width (1 = batched layout, 4 = latency layout)
    monkeypatch.setenv("ORBHIP_POSE_WAVES", waves)
    from orb_slam3_ros2_amd import Optimizer
    opt = Optimizer()
    for seed, n, frac in [(21, 600, 0.15), (22, 1000, 0.3), (23, 150, 0.05), (24, 9, 0.0), (25, 64, 0.5)]:
        prob, _ = synthetic_pose_problem(n=n, outlier_frac=frac, seed=seed)
        _check(opt.PoseOptimization(prob), oracle.pose_optimization(prob))


@pytest.mark.gpu
@pytest.mark.parametrize("waves", ["1", "4"])
def test_pose_optimization_batch_and_edge_cases(oracle, monkeypatch, waves):
    monkeypatch.setenv("ORBHIP_POSE_WAVES", waves)
    from orb_slam3_ros2_amd import Optimizer
    opt = Optimizer()
    probs = [synthetic_pose_problem(n=int(n), outlier_frac=0.2, seed=100 + i)[0]
             for i, n in enumerate([0, 1, 2, 3, 10, 63, 64, 65, 500, 1500])]
    rs = opt.PoseOptimization_batch(probs)
    for p, r in zip(probs, rs):
        _check(r, oracle.pose_optimization(p))
    assert rs[0].n_inliers == 0 and rs[2].n_inliers == 0

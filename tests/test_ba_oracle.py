"""KATs for the BA oracle (LM / Schur restatement of g2o as used by Optimizer::LocalBundleAdjustment)."""
import numpy as np

from orb_slam3_ros2_amd.synthetic import _mat_to_quat, synthetic_ba_problem


def test_noise_free_problem_converges_to_ground_truth(oracle):
    prob, gt = synthetic_ba_problem(n_kf=12, n_pts=300, seed=3, rot_noise=0.002, trans_noise=0.004,
                                    pt_noise=0.01)
    # replace observations by exact projections of the ground truth
    R, t, X = gt["R"], gt["t"], gt["points"]
    Xc = np.einsum("eij,ej->ei", R[prob.edge_pose], X[prob.edge_point]) + t[prob.edge_pose]
    prob.edge_uv = np.stack([prob.fx * Xc[:, 0] / Xc[:, 2] + prob.cx, prob.fy * Xc[:, 1] / Xc[:, 2] + prob.cy],
                            1).astype(np.float32)
    prob.iterations = 30
    r = oracle.ba_solve(prob)
    assert r["final_chi2"] < 1e-3 * r["initial_chi2"]
    assert r["final_chi2"] < 1e-2
    qgt = np.array([_mat_to_quat(Rk) for Rk in R])
    # monocular gauge: KF0 fixed, scale may drift slightly; rotations are gauge-free
    assert np.max(np.abs(np.abs(np.sum(r["pose_q"] * qgt, 1)) - 1)) < 1e-6


def test_chi2_monotone_and_fixed_pose_untouched(oracle):
    prob, _ = synthetic_ba_problem(n_kf=10, n_pts=200, seed=4)
    r = oracle.ba_solve(prob)
    assert r["final_chi2"] < r["initial_chi2"]
    assert np.array_equal(r["pose_q"][0], prob.pose_q[0] / np.linalg.norm(prob.pose_q[0]).astype(np.float32)) or \
        np.allclose(r["pose_q"][0], prob.pose_q[0], atol=1e-7)
    assert np.allclose(r["pose_t"][0], prob.pose_t[0], atol=0)


def test_outlier_flags_follow_chi2(oracle):
    prob, _ = synthetic_ba_problem(n_kf=10, n_pts=200, seed=5)
    prob.edge_uv[::37] += 40.0   # gross outliers
    r = oracle.ba_solve(prob)
    out = (r["edge_chi2"] > 5.991) | (r["edge_depth_ok"] == 0)
    assert out[::37].mean() > 0.9

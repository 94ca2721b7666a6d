"""Golden fixtures (tests/golden/, written by tools/gen_golden.py from the oracle).

CPU: the oracle reproduces every stored vector (regression pin of the restatement; the
reference itself ships no fixtures — parity unpinned by the reference).
GPU: the product reproduces the same stored bytes through the C-ABI, without running the
oracle on the box: bit-exact keypoints/descriptors/order/monoIndex, bit-exact matches,
BA within 1e-4 relative (north_star tolerance).
"""
import glob
import hashlib
import os

import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_frame

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FRAMES = sorted(glob.glob(os.path.join(GOLD, "frame_*.npz")))
REL = 1e-4


def _frame(z):
    if "image" in z.files:
        return z["image"]
    img = synthetic_frame(int(z["seed"]), int(z["w"]), int(z["h"]))
    assert hashlib.md5(img.tobytes()).hexdigest() == str(z["image_md5"]), "synthetic generator drifted"
    return img


def _ba_problem(z):
    from orb_slam3_ros2_amd.optimizer import BAProblem
    fx, fy, cx, cy = (float(v) for v in z["cam"])
    return BAProblem(z["pose_q"], z["pose_t"], z["pose_fixed"], z["points"], z["edge_pose"], z["edge_point"],
                     z["edge_uv"], z["edge_octave"], z["inv_sigma2"], fx, fy, cx, cy, float(z["huber_delta"]),
                     int(z["iterations"]))


def test_fixtures_present():
    assert len(FRAMES) >= 3 and os.path.exists(os.path.join(GOLD, "ba_10kf_200pt_s21.npz"))


@pytest.mark.parametrize("path", FRAMES, ids=os.path.basename)
def test_oracle_reproduces_frame_fixture(oracle, path):
    z = np.load(path)
    mono, kps, desc = oracle.extract(_frame(z), nfeatures=int(z["nfeatures"]), lap=tuple(z["lap"]))
    assert mono == int(z["mono"])
    assert np.array_equal(kps, z["kps"]) and np.array_equal(desc, z["desc"])


def test_oracle_reproduces_match_fixture(oracle):
    z = np.load(os.path.join(GOLD, "match_640x480_s11.npz"))
    n, m, b, s = oracle.match_bf(z["q_desc"], z["q_angle"], z["t_desc"], z["t_angle"], int(z["th_low"]),
                                 float(z["ratio"]), bool(z["check_orientation"]))
    assert n == int(z["n"]) and np.array_equal(m, z["match"])
    assert np.array_equal(b, z["best"]) and np.array_equal(s, z["second"])


def test_oracle_reproduces_ba_fixture(oracle):
    z = np.load(os.path.join(GOLD, "ba_10kf_200pt_s21.npz"))
    r = oracle.ba_solve(_ba_problem(z))
    assert [r["iterations_done"], r["lm_trials"]] == z["out_iters"].tolist()
    np.testing.assert_allclose([r["initial_chi2"], r["final_chi2"]], z["out_chi2"], rtol=1e-9)
    np.testing.assert_allclose(r["pose_t"], z["out_pose_t"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(r["points"], z["out_points"], rtol=1e-6, atol=1e-7)


# ---------------------------------------------------------------- GPU: product vs fixtures
@pytest.mark.gpu
@pytest.mark.parametrize("path", FRAMES, ids=os.path.basename)
def test_gpu_matches_frame_fixture(path):
    from orb_slam3_ros2_amd import ORBextractor
    from tests.helpers import diff_report, oracle_kps_to_struct
    z = np.load(path)
    ext = ORBextractor(int(z["nfeatures"]), 1.2, 8, 20, 7)
    mono, gk, gd = ext(_frame(z), None, tuple(int(v) for v in z["lap"]))
    ok = oracle_kps_to_struct(z["kps"])
    same = (mono == int(z["mono"]) and len(gk) == len(ok) and all(np.array_equal(gk[f], ok[f]) for f in ok.dtype.names)
            and np.array_equal(gd, z["desc"]))
    assert same, diff_report(gk, gd, ok, z["desc"])


@pytest.mark.gpu
def test_gpu_matches_match_fixture():
    from orb_slam3_ros2_amd import ORBmatcher
    z = np.load(os.path.join(GOLD, "match_640x480_s11.npz"))
    mt = ORBmatcher(float(z["ratio"]), bool(z["check_orientation"]))
    n, m, b, s = mt.match_bf(z["q_desc"], z["q_angle"], z["t_desc"], z["t_angle"], int(z["th_low"]))
    assert n == int(z["n"]) and np.array_equal(m, z["match"])
    assert np.array_equal(b, z["best"]) and np.array_equal(s, z["second"])


@pytest.mark.gpu
def test_gpu_matches_ba_fixture():
    from orb_slam3_ros2_amd import Optimizer
    z = np.load(os.path.join(GOLD, "ba_10kf_200pt_s21.npz"))
    g = Optimizer().LocalBundleAdjustment(_ba_problem(z))
    assert [g.iterations_done, g.lm_trials] == z["out_iters"].tolist()
    assert abs(g.final_chi2 - z["out_chi2"][1]) <= REL * z["out_chi2"][1]
    q = np.where(g.pose_q[:, 3:4] < 0, -g.pose_q, g.pose_q)
    qo = np.where(z["out_pose_q"][:, 3:4] < 0, -z["out_pose_q"], z["out_pose_q"])
    assert np.abs(q - qo).max() < REL
    assert np.abs(g.pose_t - z["out_pose_t"]).max() / max(1.0, np.abs(z["out_pose_t"]).max()) < REL
    assert np.abs(g.points - z["out_points"]).max() / max(1.0, np.abs(z["out_points"]).max()) < REL

"""Projection-guided matching: SearchByProjection(CurrentFrame, LastFrame)
and Tracking::SearchLocalPoints (Frame::isInFrustum + SearchByProjection(F, vpMapPoints)).

Oracle KATs on the CPU (definitional: a MapPoint projected exactly onto its own keypoint with its
own descriptor matches it; claimed keypoints are never matched; skipped points are not in view),
and the device path (one wavefront per query + greedy fixed point; the list/resolve form, its
overflow into the round kernels, and the round kernels alone) against the oracle on the GPU, bit-exact (match indices, in-view flags, predicted levels). Parity unpinned by the reference
(no fixtures upstream).
"""
import numpy as np
import pytest

from orb_slam3_ros2_amd.matcher import ProjFrame
from orb_slam3_ros2_amd.synthetic import synthetic_projection_scene


# the device forms: the one-launch list/resolve path (default), the same as two launches, the list
# path overflowing into the round kernels (list capacity 2), and the round kernels alone
PROJ_MODES = {"lists": {}, "two": {"ORBHIP_PROJ_TWO": "1"}, "overflow": {"ORBHIP_PROJ_CAP": "2"},
              "rounds": {"ORBHIP_PROJ_ROUNDS": "1"}}


@pytest.fixture(params=list(PROJ_MODES))
def proj_mode(request, monkeypatch):
    for k, v in PROJ_MODES[request.param].items():
        monkeypatch.setenv(k, v)
    return request.param


def _frame(s, claimed=True):
    return ProjFrame(s["kps"], s["desc"], s["pose_q"], s["pose_t"], s["fx"], s["fy"], s["cx"], s["cy"],
                     claimed=s["claimed"] if claimed else None)


def test_oracle_exact_projection_matches_its_keypoint(oracle):
    s = synthetic_projection_scene(n_kp=400, n_mp=300, seed=1, dup_frac=0.0, distractor_frac=0.0,
                                   claimed_frac=0.0)
    f = _frame(s, claimed=False)
    # descriptors identical to the source keypoint: distance 0 wins unless a duplicate took it
    n, match = oracle.search_by_projection_last(f, s["points"], s["desc"][s["src"]], s["kps"]["octave"][s["src"]],
                                                s["kps"]["angle"][s["src"]], th=15.0, check_orientation=False)
    hit = match >= 0
    assert n == hit.sum() and hit.mean() > 0.8
    assert (match[hit] == s["src"][hit]).mean() > 0.98


def test_oracle_claimed_never_matched_and_skip(oracle):
    s = synthetic_projection_scene(seed=2)
    f = _frame(s)
    _, match = oracle.search_by_projection_last(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"])
    assert not s["claimed"][match[match >= 0]].any()
    assert len(set(match[match >= 0].tolist())) == (match >= 0).sum()      # each keypoint at most once
    _, m2, iv, lvl = oracle.search_local_points(f, s["points"], s["normals"], s["min_dist"], s["max_dist"],
                                                s["mp_desc"], s["skip"], th=1.0, nnratio=0.8)
    assert not iv[s["skip"] == 1].any() and (m2[iv == 0] == -1).all()
    assert ((lvl >= 0) == (iv == 1)).all() and lvl.max() <= 7
    assert not s["claimed"][m2[m2 >= 0]].any()
    assert len(set(m2[m2 >= 0].tolist())) == (m2 >= 0).sum()


@pytest.mark.gpu
def test_search_by_projection_last_matches_oracle(oracle, proj_mode):
    from orb_slam3_ros2_amd import ORBmatcher
    mt = ORBmatcher(0.9, True)
    for seed in range(5):
        s = synthetic_projection_scene(seed=10 + seed)
        f = _frame(s, claimed=seed % 2 == 0)
        for th, ori in [(15.0, True), (7.0, False)]:
            mt.mbCheckOrientation = ori
            n, m = mt.SearchByProjectionLastFrame(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"], th)
            on, om = oracle.search_by_projection_last(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"],
                                                      th, ori)
            assert n == on and np.array_equal(m, om), (seed, th, ori, proj_mode)


@pytest.mark.gpu
def test_search_local_points_matches_oracle(oracle, proj_mode):
    from orb_slam3_ros2_amd import ORBmatcher
    for seed in range(5):
        s = synthetic_projection_scene(seed=20 + seed)
        f = _frame(s)
        for th, ratio, far in [(1.0, 0.8, False), (3.0, 0.8, False), (5.0, 0.6, True)]:
            mt = ORBmatcher(ratio, False)
            r = mt.SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                     s["skip"], th=th, far_points=far, th_far=5.0)
            o = oracle.search_local_points(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                           s["skip"], th=th, nnratio=ratio, far_points=far, th_far=5.0)
            assert r[0] == o[0], (seed, th, proj_mode)
            for a, b in zip(r[1:], o[1:]):
                assert np.array_equal(a, b), (seed, th, proj_mode)


@pytest.mark.gpu
def test_projection_edge_cases(oracle, proj_mode):
    from orb_slam3_ros2_amd import ORBmatcher
    mt = ORBmatcher(0.9, True)
    s = synthetic_projection_scene(n_kp=100, n_mp=50, seed=30)
    s["kps"], s["desc"], s["claimed"] = s["kps"][:0], s["desc"][:0], s["claimed"][:0]
    f = _frame(s)
    n, m = mt.SearchByProjectionLastFrame(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"])
    assert n == 0 and (m == -1).all()
    s = synthetic_projection_scene(n_kp=300, n_mp=0, seed=31)
    n, m = mt.SearchByProjectionLastFrame(_frame(s), s["points"], s["mp_desc"], s["last_octave"], s["last_angle"])
    assert n == 0 and m.size == 0


@pytest.mark.gpu
def test_projection_ragged_sizes(oracle, proj_mode):
    """Frame keypoint counts off the list kernel's 256-key scan step and map-point counts off its
    4-query work-groups (the last work-group part-filled), both searches against the oracle."""
    from orb_slam3_ros2_amd import ORBmatcher
    for n_kp, n_mp, seed in [(777, 333, 40), (257, 5, 41), (1, 3, 42)]:
        s = synthetic_projection_scene(n_kp=n_kp, n_mp=n_mp, seed=seed)
        f = _frame(s)
        mt = ORBmatcher(0.9, True)
        n, m = mt.SearchByProjectionLastFrame(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"], 15.0)
        on, om = oracle.search_by_projection_last(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"],
                                                  15.0, True)
        assert n == on and np.array_equal(m, om), (n_kp, n_mp, proj_mode)
        ml = ORBmatcher(0.8, False)
        r = ml.SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"], s["skip"],
                                 th=3.0)
        o = oracle.search_local_points(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                       s["skip"], th=3.0, nnratio=0.8)
        assert r[0] == o[0], (n_kp, n_mp, proj_mode)
        for a, b in zip(r[1:], o[1:]):
            assert np.array_equal(a, b), (n_kp, n_mp, proj_mode)


def test_proj_frame_view_tracks_pose_and_arrays():
    """ProjFrame.to_c(): the pose / bounds / intrinsics are re-read on every call (Tracking updates
    Tcw in place after PoseOptimization), reassigned arrays get fresh pointers, unchanged arrays
    keep theirs (no conversion per call)."""
    s = synthetic_projection_scene(n_kp=50, n_mp=10, seed=5)
    f = _frame(s)
    c0 = f.to_c()
    kp_ptr, cl_ptr = c0.kps, c0.claimed
    f.pose_q[:] = [0.0, 0.0, 0.0, 1.0]
    f.pose_t[:] = [0.5, -0.25, 2.0]
    c1 = f.to_c()
    assert list(c1.pose_q) == [0.0, 0.0, 0.0, 1.0] and list(c1.pose_t) == [0.5, -0.25, 2.0]
    assert c1.kps == kp_ptr and c1.claimed == cl_ptr
    f.claimed = np.zeros(50, np.uint8)
    f.fx = 123.0
    c2 = f.to_c()
    assert c2.claimed == f.claimed.ctypes.data and c2.claimed != cl_ptr and c2.fx == 123.0
    assert c2.kps == kp_ptr


@pytest.mark.gpu
def test_pose_change_between_searches(oracle):
    """The same ProjFrame searched, its Tcw changed in place (PoseOptimization), searched again:
    the second search uses the new pose (oracle on the same frame)."""
    from orb_slam3_ros2_amd import ORBmatcher
    s = synthetic_projection_scene(seed=50)
    f = _frame(s)
    mt = ORBmatcher(0.9, True)
    for step in range(3):
        n, m = mt.SearchByProjectionLastFrame(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"], 15.0)
        on, om = oracle.search_by_projection_last(f, s["points"], s["mp_desc"], s["last_octave"], s["last_angle"],
                                                  15.0, True)
        assert n == on and np.array_equal(m, om), step
        r = ORBmatcher(0.8, False).SearchLocalPoints(f, s["points"], s["normals"], s["min_dist"], s["max_dist"],
                                                     s["mp_desc"], s["skip"], th=3.0)
        o = oracle.search_local_points(f, s["points"], s["normals"], s["min_dist"], s["max_dist"], s["mp_desc"],
                                       s["skip"], th=3.0, nnratio=0.8)
        assert r[0] == o[0] and all(np.array_equal(a, b) for a, b in zip(r[1:], o[1:])), step
        f.pose_t[:] = f.pose_t + np.float32([0.02, -0.01, 0.03])   # in place, as Tracking does

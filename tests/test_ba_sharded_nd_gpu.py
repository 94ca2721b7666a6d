"""GPU: the sharded GlobalBundleAdjustment by keyframe segments (the §8e distributed step on the
device: each shard factors its segment's interior with the partial DAG Cholesky, the separator
system and the pose update are summed over the shards, every shard solves the separator system;
the LM runs device-driven with the collectives on the stream, no host round trip per trial).

In-process shards (orbhip_ba_solve_shards_local, sums by k_ba_multi_reduce) stand in for the ranks
on one GPU; the RCCL form runs the same slot with ncclAllReduce in those places: a one-rank
communicator holding all K segments (orbhip_ba_solve_sharded_segments: the rank's segments summed on
the device, then the all-reduce) runs every collective of the dissected slot through RCCL. Each against the
oracle LM (schedule identical, 1e-4 on poses / points / chi2) at the full C5 size with 4 and 8
segments, and on 100- and 150-KF loops with 2 and 3. Parity unpinned by the reference."""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem

pytestmark = pytest.mark.gpu
REL = 1e-4


def _close(g, o):
    assert g.iterations_done == o["iterations_done"] and g.lm_trials == o["lm_trials"]
    assert abs(g.final_chi2 - o["final_chi2"]) <= REL * abs(o["final_chi2"])
    q = lambda a: a.astype(np.float64) * np.where(a[:, 3:4] < 0, -1.0, 1.0)   # noqa: E731
    assert np.abs(q(g.pose_q) - q(o["pose_q"])).max() < REL
    assert np.abs(g.pose_t.astype(np.float64) - o["pose_t"]).max() / max(1.0, np.abs(o["pose_t"]).max()) < REL
    assert np.abs(g.points.astype(np.float64) - o["points"]).max() / max(1.0, np.abs(o["points"]).max()) < REL


def _solve_segments(opt, p, K, per2=True, rccl=False):
    from orb_slam3_ros2_amd.sharding import merge_results_nd, shard_problem_nd
    parts = [shard_problem_nd(p, r, K) for r in range(K)]
    l0 = opt.stats()["dag_launches"]
    shards = [q[0] for q in parts]
    res = opt.solve_sharded_segments(shards) if rccl else opt.solve_shards_local(shards)
    # the dissected form launches two persistent solves per shard and trial (its segment's partial
    # factorization, the separator system), so does the replicated form when it dissects the summed
    # S (r06, its union adjacency); on the plain DAG solve (ORBHIP_ND=0) it launches one
    per = (opt.stats()["dag_launches"] - l0) / (K * res[0].lm_trials)
    assert per >= 2 if per2 else per < 2, per
    for r in res[1:]:
        assert np.array_equal(r.pose_t, res[0].pose_t)   # every shard applies the same pose update
    return merge_results_nd(p, res, [q[1] for q in parts], [q[2] for q in parts])


@pytest.mark.parametrize("K", [4, 8])
def test_c5_segment_shards_parity(c5_case, K):
    from orb_slam3_ros2_amd import Optimizer
    _, p, o = c5_case
    _close(_solve_segments(Optimizer(), p, K), o)


@pytest.mark.parametrize("n_kf,K", [(100, 2), (150, 3)])
def test_loop_segment_shards_parity(oracle, n_kf, K, monkeypatch):
    from orb_slam3_ros2_amd import Optimizer
    from orb_slam3_ros2_amd.optimizer import BAProblem
    monkeypatch.setenv("ORBHIP_ND_MIN", "0")   # n = 594 / 894: below the default size for the dissection
    prob, _ = synthetic_ba_problem(n_kf=n_kf, n_pts=30 * n_kf, layout="loop", window=20, seed=35)
    p = BAProblem(**{**prob.__dict__, "iterations": 10, "huber_delta": float(np.sqrt(5.99))})
    _close(_solve_segments(Optimizer(), p, K), oracle.ba_solve(p))


@pytest.mark.parametrize("nd", [1, 0])
def test_segment_shards_replicated_fallback(c5_case, monkeypatch, nd):
    """ORBHIP_SHARD_ND=0: the same shards sum S itself and every shard solves it (replicated), by
    nested dissection of the summed S planned on the shards' union adjacency (nd=1), or on the
    plain DAG solve over the union envelope (ORBHIP_ND=0)."""
    from orb_slam3_ros2_amd import Optimizer
    monkeypatch.setenv("ORBHIP_SHARD_ND", "0")
    if not nd:
        monkeypatch.setenv("ORBHIP_ND", "0")
    _, p, o = c5_case
    _close(_solve_segments(Optimizer(), p, 4, per2=bool(nd)), o)


def _rccl_optimizer():
    from orb_slam3_ros2_amd import Optimizer
    opt = Optimizer()
    opt.comm_init(1, 0, Optimizer.comm_unique_id())
    return opt


@pytest.mark.parametrize("K", [4, 8])
def test_c5_rccl_rank_segments_parity(c5_case, K):
    """One RCCL rank with K local segments: the kNdPack / kNdBz / kNdX all-reduces, the Hpp / chi2
    sums and the plan / stop / timeout consensus all go through ncclAllReduce."""
    _, p, o = c5_case
    _close(_solve_segments(_rccl_optimizer(), p, K, rccl=True), o)


@pytest.mark.parametrize("nd", [1, 0])
def test_c5_rccl_rank_segments_replicated(c5_case, monkeypatch, nd):
    """ORBHIP_SHARD_ND=0 over RCCL with 4 local shards: S summed on the device, all-reduced in full,
    copied to the other shards; every shard solves it by the dissection planned on the union
    adjacency (all-reduced, nd=1) or on the union envelope's DAG plan (ORBHIP_ND=0)."""
    monkeypatch.setenv("ORBHIP_SHARD_ND", "0")
    if not nd:
        monkeypatch.setenv("ORBHIP_ND", "0")
    _, p, o = c5_case
    _close(_solve_segments(_rccl_optimizer(), p, 4, per2=bool(nd), rccl=True), o)


@pytest.mark.parametrize("nd", [1, 0])
def test_c5_rccl_landmark_shard_dissected(c5_case, monkeypatch, nd):
    """The landmark-shard form on one RCCL rank (orbhip_ba_solve_sharded: S all-reduced over its
    union envelope, packed): the summed S solved by the dissection planned on the all-reduced
    union adjacency (two persistent solves per trial), or by the plain DAG solve (ORBHIP_ND=0)."""
    if not nd:
        monkeypatch.setenv("ORBHIP_ND", "0")
    _, p, o = c5_case
    opt = _rccl_optimizer()
    l0 = opt.stats()["dag_launches"]
    g = opt.solve_sharded(p)
    per = (opt.stats()["dag_launches"] - l0) / g.lm_trials
    assert per >= 2 if nd else per < 2, per
    _close(g, o)

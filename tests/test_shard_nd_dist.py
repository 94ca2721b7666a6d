"""Host logic of the sharded solve by keyframe segments (csrc/ba_nd.hip seg_sel mode, the §8e
distributed step of the C5 GlobalBundleAdjustment), on the CPU over gloo (world size 2).

sharding.shard_problem_nd gives rank r the landmarks of segment r. Each rank builds the reduced
camera system of its shard alone (tests/ba_numpy.py: Gauss-Newton, landmarks eliminated), with the
damping of the poses it owns (its interior + own separator, as BaArgs::own adds Hpp + lambda). The
rank's interior rows must then be complete, which is what lets it eliminate its interior locally:
this test runs the device step's arithmetic in numpy — the partial factorization of
[[S_II, S_IZ], [S_ZI, 0]] over (I_r, Z_{r-1}, Z_r), the separator system summed by ONE all-reduce,
the replicated separator solve, the interior back-substitution, the x sum — and compares it with
the solve of the summed full system. Same segmentation formula as nd_plan_band (seg[r] =
floor(r np / K), separators of w poses). Parity here is against numpy's own solve."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _problem():
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem(n_kf=48, n_pts=900, layout="loop", window=5, seed=4)
    return prob


def _owned(plan, r, K):
    return np.arange(plan["seg"][r], plan["seg"][r + 1])


def _segment_vars(plan, r, K):
    """Interior, previous separator and own separator variables of segment r (optimised order)."""
    seg, w, cyc = plan["seg"], plan["w"], plan["cyclic"]
    own = cyc or r < K - 1
    prev = cyc or r > 0
    iend = seg[r + 1] - (w if own else 0)
    v = lambda poses: (np.asarray(poses)[:, None] * 6 + np.arange(6)).reshape(-1)   # noqa: E731
    I = v(np.arange(seg[r], iend))
    t = (r - 1) % K
    Zp = v(np.arange(seg[t + 1] - w, seg[t + 1])) if prev else np.zeros(0, np.int64)
    Zo = v(np.arange(iend, seg[r + 1])) if own else np.zeros(0, np.int64)
    return I, Zp, Zo


def _local_system(prob, r, K, plan):
    from orb_slam3_ros2_amd.sharding import shard_problem_nd
    from ba_numpy import reduced_system
    sh, _, _ = shard_problem_nd(prob, r, K)
    S, b = reduced_system(sh)
    d = np.zeros(S.shape[0])
    d[(_owned(plan, r, K)[:, None] * 6 + np.arange(6)).reshape(-1)] = 1.0   # damping of the owned poses
    return S + np.diag(d), b


def _nd_rank_parts(S, b, plan, r, K):
    """One rank's part of the dissected solve (numpy): its share of the separator system (the
    all-reduce's input) and a function finishing the solve from the summed system (its x share)."""
    I, Zp, Zo = _segment_vars(plan, r, K)
    n = S.shape[0]
    nsep = K if plan["cyclic"] else K - 1
    Zg = np.concatenate([np.arange(plan["seg"][t + 1] - plan["w"], plan["seg"][t + 1]) for t in range(nsep)])
    Zg = (Zg[:, None] * 6 + np.arange(6)).reshape(-1)   # separator system order -> variables
    pos = {int(g): k for k, g in enumerate(Zg)}
    Zl = np.concatenate([Zp, Zo])
    L = np.linalg.cholesky(S[np.ix_(I, I)])
    W = np.linalg.solve(L, S[np.ix_(I, Zl)])
    y = np.linalg.solve(L, b[I])
    SZ = S[np.ix_(Zg, Zg)].copy()
    bZ = b[Zg].copy()
    zi = np.array([pos[int(g)] for g in Zl], np.int64)
    SZ[np.ix_(zi, zi)] -= W.T @ W
    bZ[zi] -= W.T @ y

    def finish(SZs, bZs):
        xZ = np.linalg.solve(SZs, bZs)
        xl = np.zeros(n)
        xl[I] = np.linalg.solve(L.T, y - W @ xZ[zi])
        xl[Zo] = xZ[[pos[int(g)] for g in Zo]]
        return xl
    return SZ, bZ, finish


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import torch
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from orb_slam3_ros2_amd.sharding import nd_segments, pose_blocks
        prob = _problem()
        npo, bi, bj = pose_blocks(prob)
        plan = nd_segments(npo, bi, bj, WORLD)
        S, b = _local_system(prob, rank, WORLD, plan)

        def allreduce(a):
            t = torch.from_numpy(np.ascontiguousarray(a))
            dist.all_reduce(t)
            return t.numpy()

        SZ, bZ, finish = _nd_rank_parts(S, b, plan, rank, WORLD)
        x = allreduce(finish(allreduce(SZ), allreduce(bZ)))
        Sf = allreduce(S)
        bf = allreduce(b)
        xr = np.linalg.solve(Sf, bf)
        q.put((rank, float(np.abs(x - xr).max() / np.abs(xr).max())))
    finally:
        dist.destroy_process_group()


def test_shard_nd_step_gloo_matches_full_solve():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(WORLD)]
    for rank, err in res:
        assert err < 1e-9, (rank, err)


@pytest.mark.parametrize("K", [3, 4, 8])
def test_shard_nd_in_process(K):
    """The same step with K ranks in one process (the sum a plain one), at the C5 pose graph's
    shape scaled down (48-KF loop): equal to the full solve, and every rank's interior rows are
    those of the full system (the landmark assignment is complete)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from orb_slam3_ros2_amd.sharding import nd_segments, pose_blocks
    prob = _problem()
    npo, bi, bj = pose_blocks(prob)
    plan = nd_segments(npo, bi, bj, K)
    if plan is None:
        pytest.skip("band too wide for this many segments")
    loc = [_local_system(prob, r, K, plan) for r in range(K)]
    Sf, bf = sum(s for s, _ in loc), sum(b for _, b in loc)
    for r, (S, b) in enumerate(loc):
        I, _, _ = _segment_vars(plan, r, K)
        assert np.allclose(S[I], Sf[I], rtol=0, atol=1e-9 * np.abs(Sf).max())
    parts = [_nd_rank_parts(S, b, plan, r, K) for r, (S, b) in enumerate(loc)]
    SZ = sum(q[0] for q in parts)
    bZ = sum(q[1] for q in parts)
    x = sum(q[2](SZ, bZ) for q in parts)
    xr = np.linalg.solve(Sf, bf)
    assert np.abs(x - xr).max() / np.abs(xr).max() < 1e-9

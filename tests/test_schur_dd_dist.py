"""The distributed C5 step's arithmetic (tests/schur_dd_model.py, DESIGN.md §C5 sharding):
nested dissection of the reduced camera system by keyframe segments. Each rank eliminates its
interior, one all-reduce sums the separator system, every rank solves it, an all-gather collects
the interiors; the result equals the full solve. gloo world size 2 on the CPU; the C5 shape (400
KF loop, 20-KF window, 8 segments) in one process; and the partition's premise (every landmark's
observations fit one co-visibility window, so it touches at most one interior) on the C5 problem
the bench solves."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from schur_dd_model import Partition, covisibility_system, dd_solve
        part = Partition(40, WORLD, 5)
        Ss, bs = covisibility_system(part, 400, seed=1)   # every rank builds all, keeps its own
        x = dd_solve(torch.from_numpy(Ss[rank]), torch.from_numpy(bs[rank]), part, rank).numpy()
        xr = np.linalg.solve(sum(Ss), sum(bs))
        q.put((rank, float(np.abs(x - xr).max() / np.abs(xr).max())))
    finally:
        dist.destroy_process_group()


def _worker_segments(rank, port, q):
    """Two ranks x two local segments each (K = 4): the orbhip_ba_solve_sharded_segments flow."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from schur_dd_model import Partition, covisibility_system, dd_solve_segments
        part = Partition(48, 2 * WORLD, 5)
        Ss, bs = covisibility_system(part, 500, seed=5)
        mine = [2 * rank, 2 * rank + 1]
        x = dd_solve_segments([Ss[r] for r in mine], [bs[r] for r in mine], part, rank).numpy()
        xr = np.linalg.solve(sum(Ss), sum(bs))
        q.put((rank, float(np.abs(x - xr).max() / np.abs(xr).max())))
    finally:
        dist.destroy_process_group()


def _worker_segments_two_level(rank, port, q):
    """Two ranks x four local segments (K = 8), the separator system dissected once more on every
    rank after the all-reduce (the device's second level)."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        from schur_dd_model import Partition, covisibility_system, dd_solve_segments
        part = Partition(80, 8, 5)
        Ss, bs = covisibility_system(part, 800, seed=6)
        mine = list(range(4 * rank, 4 * rank + 4))
        x = dd_solve_segments([Ss[r] for r in mine], [bs[r] for r in mine], part, rank, levels=2).numpy()
        xr = np.linalg.solve(sum(Ss), sum(bs))
        q.put((rank, float(np.abs(x - xr).max() / np.abs(xr).max())))
    finally:
        dist.destroy_process_group()


def _run_gloo(target):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=target, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [q.get(timeout=5) for _ in range(WORLD)]


def test_dd_solve_segments_gloo_ranks_times_local():
    for rank, err in _run_gloo(_worker_segments):
        assert err < 1e-10, (rank, err)


def test_dd_solve_segments_gloo_two_levels():
    for rank, err in _run_gloo(_worker_segments_two_level):
        assert err < 1e-10, (rank, err)


def test_dd_solve_gloo_matches_full_solve():
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
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    res = [q.get(timeout=5) for _ in range(WORLD)]
    for rank, err in res:
        assert err < 1e-10, (rank, err)


def test_partial_systems_live_on_their_segment():
    from schur_dd_model import Partition, covisibility_system
    part = Partition(48, 4, 6)
    Ss, _ = covisibility_system(part, 600, seed=2)
    for r, S in enumerate(Ss):
        nz = set(np.nonzero(np.abs(S).sum(0))[0].tolist())
        assert nz <= set(np.concatenate([part.interior(r), part.adjacent(r)]).tolist()), r
    for r in range(part.ranks):   # interiors pairwise uncoupled in the summed system
        for t in range(part.ranks):
            if t != r:
                assert not np.any(sum(Ss)[np.ix_(part.interior(r), part.interior(t))])


def test_dd_solve_c5_shape_in_process():
    from schur_dd_model import Partition, covisibility_system, dd_solve_local
    part = Partition(400, 8, 20)
    Ss, bs = covisibility_system(part, 6000, seed=3)
    x = dd_solve_local(Ss, bs, part).numpy()
    xr = np.linalg.solve(sum(Ss), sum(bs))
    assert np.abs(x - xr).max() / np.abs(xr).max() < 1e-10
    assert part.n_sep == 912 and part.interior(0).size == 186


def test_two_level_dissection_of_the_separator_system():
    """The separator system after the all-reduce is cyclic block-tridiagonal (8 separators of
    19 keyframes): a second dissection level (odd separators as interiors, 4 ranks) solves it
    exactly too (the model of DESIGN.md §C5 sharding prices both levels)."""
    import torch
    from schur_dd_model import (Partition, covisibility_system, dd_local, dd_solve_local,
                                             split_assembled)
    part = Partition(400, 8, 20)
    Ss, bs = covisibility_system(part, 6000, seed=4)
    loc = [dd_local(torch.from_numpy(S), torch.from_numpy(b), part, r) for r, (S, b) in enumerate(zip(Ss, bs))]
    Sz = sum(l[1] for l in loc).numpy()
    bz = sum(l[2] for l in loc).numpy()
    p2 = Partition(8, 4, 2, dof=part.sep * part.dof)
    # block-tridiagonal cyclic: separators two apart are uncoupled
    m = part.sep * part.dof
    assert not np.any(Sz[:m, 2 * m:3 * m]) and not np.any(Sz[:m, 4 * m:5 * m])
    S2, b2 = split_assembled(Sz, bz, p2)
    assert np.allclose(sum(S2), Sz, rtol=0, atol=0) and np.allclose(sum(b2), bz, rtol=0, atol=0)
    xz = dd_solve_local(S2, b2, p2).numpy()
    xr = np.linalg.solve(Sz, bz)
    assert np.abs(xz - xr).max() / np.abs(xr).max() < 1e-10


def test_c5_landmarks_fit_one_window():
    """Premise of the partition on the bench's C5 problem: every landmark is observed by keyframes
    within one cyclic 20-keyframe window, so it touches at most one segment interior."""
    from schur_dd_model import Partition
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem(n_kf=400, n_pts=20000, layout="loop", window=20, seed=11)
    part = Partition(400, 8, 20)
    ep, pt = np.asarray(prob.edge_pose), np.asarray(prob.edge_point)
    order = np.argsort(pt, kind="stable")
    ep, pt = ep[order], pt[order]
    starts = np.searchsorted(pt, np.arange(prob.points.shape[0]))
    ends = np.append(starts[1:], len(pt))
    interior_of = np.full(400, -1)
    for r in range(part.ranks):
        interior_of[part.interior_kf(r)] = r
    for m in range(prob.points.shape[0]):
        kfs = np.unique(ep[starts[m]:ends[m]])
        if kfs.size == 0:
            continue
        # cyclic span: the largest gap between consecutive observing keyframes closes the circle
        gaps = np.diff(np.concatenate([kfs, [kfs[0] + 400]]))
        assert 400 - gaps.max() + 1 <= part.window, m
        touched = set(interior_of[kfs].tolist()) - {-1}
        assert len(touched) <= 1, (m, kfs)

"""N > 1 path on the CPU (gloo, world size 2): landmark shards partition the problem, and the
shards' partial reduced camera systems sum (all_reduce) to the full system — the identity the
RCCL all-reduce of orbhip_ba_solve_sharded relies on."""
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
        from orb_slam3_ros2_amd.sharding import shard_bounds, shard_problem
        from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
        from tests.ba_numpy import reduced_system
        prob, _ = synthetic_ba_problem(n_kf=12, n_pts=240, layout="loop", window=5, seed=3)
        sh, lo, hi, sel = shard_problem(prob, rank, WORLD)
        # 1. edge / landmark partition
        counts = torch.tensor([len(sel), hi - lo], dtype=torch.int64)
        allc = [torch.zeros(2, dtype=torch.int64) for _ in range(WORLD)]
        dist.all_gather(allc, counts)
        E, M = prob.edge_pose.shape[0], prob.points.shape[0]
        assert sum(int(c[0]) for c in allc) == E and sum(int(c[1]) for c in allc) == M
        b = shard_bounds(prob, WORLD)
        assert b[0] == 0 and b[-1] == M and np.all(np.diff(b) >= 0)
        assert np.array_equal(sh.pose_q, prob.pose_q) and np.all(sh.edge_point < hi - lo)
        # 2. partial reduced systems add up to the full one
        S, bs = reduced_system(sh)
        St = torch.from_numpy(S.copy())
        bt = torch.from_numpy(bs.copy())
        dist.all_reduce(St)
        dist.all_reduce(bt)
        Sf, bf = reduced_system(prob)
        scale = np.abs(Sf).max()
        q.put((rank, float(np.abs(St.numpy() - Sf).max() / scale), float(np.abs(bt.numpy() - bf).max() / np.abs(bf).max())))
    finally:
        dist.destroy_process_group()


def test_shards_sum_to_full_system_gloo():
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
    for rank, dS, db in res:
        assert dS < 1e-12 and db < 1e-12, (rank, dS, db)


def test_shard_bounds_balance_edges():
    from orb_slam3_ros2_amd.sharding import shard_bounds
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    prob, _ = synthetic_ba_problem(n_kf=20, n_pts=1000, layout="loop", window=6, seed=5)
    for n in (1, 2, 3, 8):
        b = shard_bounds(prob, n)
        cnt = np.bincount(prob.edge_point, minlength=prob.points.shape[0])
        per = [cnt[b[i]:b[i + 1]].sum() for i in range(n)]
        assert sum(per) == prob.edge_pose.shape[0]
        assert max(per) - min(per) <= 2 * cnt.max()

"""N > 1 path on the CPU (gloo, world size 2): landmark shards partition the problem, and the
shards' partial reduced camera systems sum (all_reduce) to the full system — the identity the
RCCL all-reduce of orbhip_ba_solve_sharded relies on — also when only their
union envelope is packed and summed (the blocked-solver sizes)."""
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
        # 3. the envelope-packed all-reduce of orbhip_ba_solve_sharded (k_ba_env_pack): per
        # 32-row tile R the columns [32 rf[R], 32 R + 32) of each shard's S, rf the union (min
        # over the shards) of their envelopes, summed packed and unpacked, equal the full
        # system's lower triangle; outside the union envelope every entry is zero
        n = S.shape[0]
        nt = (n + 31) // 32
        rf = np.arange(nt)
        for r in range(n):
            nz = np.nonzero(S[r, :r + 1])[0]
            if nz.size:
                rf[r // 32] = min(rf[r // 32], nz[0] // 32)
        rft = torch.from_numpy(rf.astype(np.int64))
        dist.all_reduce(rft, op=dist.ReduceOp.MIN)
        rf = rft.numpy()
        spans = [(32 * R, min(32 * R + 32, n), 32 * rf[R], min(32 * R + 32, n)) for R in range(nt)]
        packed = torch.from_numpy(np.concatenate([S[r0:r1, c0:c1].ravel() for r0, r1, c0, c1 in spans]))
        dist.all_reduce(packed)
        Senv = np.zeros_like(S)
        o = 0
        for r0, r1, c0, c1 in spans:
            k = (r1 - r0) * (c1 - c0)
            Senv[r0:r1, c0:c1] = packed.numpy()[o:o + k].reshape(r1 - r0, c1 - c0)
            o += k
        rows, cols = np.indices(S.shape)
        lower = cols <= rows
        env = lower & (cols >= 32 * rf[rows // 32])
        assert not np.any(Sf[lower & ~env]), "a non-zero of the summed S outside the union envelope"
        d_env = float(np.abs(Senv - Sf)[env].max() / scale)
        q.put((rank, max(float(np.abs(St.numpy() - Sf).max() / scale), d_env),
               float(np.abs(bt.numpy() - bf).max() / np.abs(bf).max())))
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

"""N > 1 path on the CPU (gloo, world size 2): landmark shards partition the problem, and the
shards' partial reduced camera systems sum (all_reduce) to the full system — the identity the
RCCL all-reduce of orbhip_ba_solve_sharded relies on — also when only their
union envelope is packed and summed (the blocked-solver sizes) — and (r06) the replicated form's
nested dissection: the shards' pose adjacencies all-reduced (max) give the summed system's block
structure, and the dissection planned on it (interiors eliminated, the separator system solved,
back-substitution) solves the summed system."""
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
        # 4. the replicated form's dissection (ba_solve_batch: union adjacency, nd_plan, nd_setup)
        d_nd = _nd_union_check(rank, dist, torch)
        q.put((rank, max(float(np.abs(St.numpy() - Sf).max() / scale), d_env),
               float(np.abs(bt.numpy() - bf).max() / np.abs(bf).max()), d_nd))
    finally:
        dist.destroy_process_group()


def _nd_union_check(rank, dist, torch):
    """A 24-keyframe loop (window 4) in landmark shards: each rank's pose adjacency as a byte map,
    all-reduced with MAX (the ncclUint8 all-reduce of the replicated form), must equal the summed
    system's block structure; the two-segment cyclic dissection planned on it (nd_plan_band:
    w = the cyclic half-bandwidth, segment r = interior [seg_r, seg_r+1 - w) + separator
    [seg_r+1 - w, seg_r+1)) solves S + lambda I by interior elimination, the separator system and
    back-substitution. Returns the relative difference to the dense solve."""
    from orb_slam3_ros2_amd.sharding import shard_problem
    from orb_slam3_ros2_amd.synthetic import synthetic_ba_problem
    from tests.ba_numpy import reduced_system
    prob, _ = synthetic_ba_problem(n_kf=24, n_pts=480, layout="loop", window=4, seed=4)
    sh = shard_problem(prob, rank, WORLD)[0]
    S, bs = reduced_system(sh)
    n = S.shape[0]
    npz = n // 6
    blk = np.abs(S).reshape(npz, 6, npz, 6).max(axis=(1, 3)) > 0
    adj = torch.from_numpy(np.tril(blk).astype(np.uint8))
    dist.all_reduce(adj, op=dist.ReduceOp.MAX)
    St, bt = torch.from_numpy(S.copy()), torch.from_numpy(bs.copy())
    dist.all_reduce(St)
    dist.all_reduce(bt)
    Sf, bf = St.numpy() + 1e-3 * np.abs(St.numpy()).max() * np.eye(n), bt.numpy()
    full = np.abs(Sf).reshape(npz, 6, npz, 6).max(axis=(1, 3)) > 0
    assert np.array_equal(np.tril(full), adj.numpy().astype(bool)), "union adjacency != summed structure"
    i, j = np.nonzero(adj.numpy())
    d = np.abs(i - j)
    wl, wc = int(d.max()), int(np.minimum(d, npz - d).max())
    assert wl > wc   # cyclic
    K, w = 2, wc
    seg = [r * npz // K for r in range(K + 1)]
    inter = [np.arange(seg[r], seg[r + 1] - w) for r in range(K)]
    seps = [np.arange(seg[r + 1] - w, seg[r + 1]) for r in range(K)]
    var = lambda poses: (6 * poses[:, None] + np.arange(6)).ravel()   # noqa: E731
    I = [var(x) for x in inter]
    Z = np.concatenate([var(x) for x in seps])
    assert not np.any(Sf[np.ix_(I[0], I[1])]), "two interiors couple"
    SZ, bZ = Sf[np.ix_(Z, Z)].copy(), bf[Z].copy()
    for Ir in I:   # each interior eliminated (the partial factorizations), its fill on the separators
        A, C = Sf[np.ix_(Ir, Ir)], Sf[np.ix_(Z, Ir)]
        SZ -= C @ np.linalg.solve(A, C.T)
        bZ -= C @ np.linalg.solve(A, bf[Ir])
    x = np.zeros(n)
    x[Z] = np.linalg.solve(SZ, bZ)
    for Ir in I:   # back-substitution of the interiors
        x[Ir] = np.linalg.solve(Sf[np.ix_(Ir, Ir)], bf[Ir] - Sf[np.ix_(Ir, Z)] @ x[Z])
    xd = np.linalg.solve(Sf, bf)
    return float(np.abs(x - xd).max() / np.abs(xd).max())


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
    for rank, dS, db, dnd in res:
        assert dS < 1e-12 and db < 1e-12 and dnd < 1e-9, (rank, dS, db, dnd)


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

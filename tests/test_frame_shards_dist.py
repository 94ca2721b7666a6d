"""N > 1 path of the batched front-end (C3) on the CPU (gloo, world size 2 and 3): contiguous
B/N frame slices with a one-frame halo. Each rank extracts its slice + halo and
matches its own pairs with the oracle (the CPU stand-in for the device path, which runs the same
partition in bench.py); the gathered per-pair results equal the single-process pass over the whole
batch, and every pair is owned by exactly one rank."""
import os

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from orb_slam3_ros2_amd.sharding import frame_slice_with_halo, frame_slices


def test_frame_slices_partition():
    for B in (0, 1, 2, 5, 63, 64, 65):
        for N in (1, 2, 3, 4, 8):
            sl = frame_slices(B, N)
            assert sl[0][0] == 0 and sl[-1][1] == B
            assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
            assert max(h - l for l, h in sl) - min(h - l for l, h in sl) <= 1
            owned = []
            for r in range(N):
                lo, hx, plo, phi = frame_slice_with_halo(B, r, N)
                assert lo <= plo <= phi and phi <= max(hx - 1, lo) and hx <= B
                owned += list(range(plo, phi))
            assert sorted(owned) == list(range(max(B - 1, 0))), (B, N)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import pyoracle as O
        from orb_slam3_ros2_amd.synthetic import synthetic_stream
        B = 7
        frames = synthetic_stream(B, 320, 240, 8)
        lo, hx, plo, phi = frame_slice_with_halo(B, rank, world)
        ext = {i: O.extract(frames[i], nfeatures=500) for i in range(lo, hx)}
        res = {}
        for i in range(plo, phi):
            _, ka, da = ext[i]
            _, kb, db = ext[i + 1]
            n, m, _, _ = O.match_bf(da, ka[:, 3], db, kb[:, 3], 50, 0.9, True)
            res[i] = (n, m.tolist())
        out = [None] * world
        dist.all_gather_object(out, res)
        if rank == 0:
            merged = {}
            for d in out:
                assert not (set(d) & set(merged))   # each pair owned once
                merged.update(d)
            ref = {}
            full = [O.extract(f, nfeatures=500) for f in frames]
            for i in range(B - 1):
                n, m, _, _ = O.match_bf(full[i][2], full[i][1][:, 3], full[i + 1][2], full[i + 1][1][:, 3], 50, 0.9,
                                        True)
                ref[i] = (n, m.tolist())
            q.put(merged == ref)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_halo_slices_reproduce_whole_batch_gloo(world):
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True

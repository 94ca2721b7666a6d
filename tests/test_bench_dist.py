"""bench.py's N > 1 bookkeeping on the CPU (gloo, world size 2, ORBHIP_BENCH_REHEARSAL=1 so that
the bench's reductions use host tensors): the max / sum over ranks that the timed regions and
the aggregate `value` use, and the C5 sharded-parity verdict AND-ed over the ranks (one rank's
sharded result off by more than 1e-4, or a different LM schedule, fails it on every rank)."""
import os
import socket
from types import SimpleNamespace

import numpy as np
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _res(chi2, q, t, pts, it=10, trials=10):
    return SimpleNamespace(final_chi2=chi2, pose_q=q, pose_t=t, points=pts, iterations_done=it, lm_trials=trials)


def _worker(rank, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ["ORBHIP_BENCH_REHEARSAL"] = "1"
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        import bench
        out = {"max": bench._max_over_ranks(WORLD, 1.0 + rank), "sum": bench._sum_over_ranks(WORLD, 1.0 + rank)}
        rng = np.random.default_rng(5)
        qq, tt, pp = rng.normal(size=(4, 4)), rng.normal(size=(4, 3)), rng.normal(size=(10, 3))
        sel = np.arange(5 * rank, 5 * rank + 5)
        ref = _res(100.0, qq, tt, pp)
        good = _res(100.0 * (1 + 1e-7), qq, tt, pp[sel])
        out["good"] = bench.c5_sharded_parity(WORLD, good, ref, sel)
        # rank 1's points off by 1e-3 of the scale: the verdict fails on both ranks
        bad_pts = pp[sel] + (1e-3 * np.abs(pp).max() if rank == 1 else 0.0)
        out["bad"] = bench.c5_sharded_parity(WORLD, _res(100.0, qq, tt, bad_pts), ref, sel)
        # rank 0 ran one trial more: schedule differs
        out["sched"] = bench.c5_sharded_parity(WORLD, _res(100.0, qq, tt, pp[sel], trials=11 - rank), ref, sel)
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_bench_rank_reductions_and_sharded_verdict_gloo():
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
    for _ in range(WORLD):
        rank, out = q.get(timeout=5)
        assert out["max"] == 2.0 and out["sum"] == 3.0
        assert out["good"]["c5_sharded_parity"] and out["good"]["c5_sharded_schedule_equal"]
        assert not out["bad"]["c5_sharded_parity"] and out["bad"]["c5_sharded_max_rel_err"] > 1e-4
        assert not out["sched"]["c5_sharded_parity"] and not out["sched"]["c5_sharded_schedule_equal"]

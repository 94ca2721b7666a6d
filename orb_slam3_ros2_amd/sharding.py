"""Landmark sharding of a BundleAdjustment problem (SURVEY.md §8e, C5 GlobalBundleAdjustment).

Every shard holds ALL poses and a contiguous range of landmarks with their edges. The ranges are
cut so that every shard carries about the same number of edges. The reduced camera system S is a
sum over landmarks, so the shards' partial systems add up to the full one. The device solver sums
them: in-process with orbhip_ba_solve_shards_local, across GPUs over RCCL with
orbhip_ba_solve_sharded.
"""
from __future__ import annotations

import numpy as np


def shard_bounds(prob, nshards: int) -> np.ndarray:
    """Landmark index boundaries [b_0 = 0, ..., b_n = M] balancing the edge count per shard."""
    M = prob.points.shape[0]
    cnt = np.bincount(np.asarray(prob.edge_point), minlength=M).astype(np.int64)
    cum = np.concatenate([[0], np.cumsum(cnt)])
    E = cum[-1]
    b = [0]
    for s in range(1, nshards):
        b.append(int(np.searchsorted(cum, E * s / nshards, side="left")))
    b.append(M)
    return np.maximum.accumulate(np.array(b, np.int64))


def shard_problem(prob, rank: int, nshards: int):
    """The rank's shard: all poses, landmarks [lo, hi) re-indexed from 0, their edges (in the
    problem's edge order). Returns (shard BAProblem, lo, hi, edge indices into the full problem)."""
    from .optimizer import BAProblem
    p = prob.normalized()
    b = shard_bounds(p, nshards)
    lo, hi = int(b[rank]), int(b[rank + 1])
    sel = np.nonzero((p.edge_point >= lo) & (p.edge_point < hi))[0]
    sh = BAProblem(p.pose_q, p.pose_t, p.pose_fixed, p.points[lo:hi].copy(), p.edge_pose[sel].copy(),
                   (p.edge_point[sel] - lo).astype(np.int32), p.edge_uv[sel].copy(), p.edge_octave[sel].copy(),
                   p.inv_sigma2, p.fx, p.fy, p.cx, p.cy, p.huber_delta, p.iterations, p.early_stop)
    return sh, lo, hi, sel


def merge_results(prob, shard_results, bounds, edge_sets):
    """Full-problem BAResult from the shards' results (poses from shard 0: all are identical)."""
    from .optimizer import BAResult
    M, E = prob.points.shape[0], prob.edge_pose.shape[0]
    pts = np.zeros((M, 3), np.float32)
    chi2 = np.zeros(E, np.float32)
    dok = np.zeros(E, np.uint8)
    for r, (res, sel) in enumerate(zip(shard_results, edge_sets)):
        pts[bounds[r]:bounds[r + 1]] = res.points
        chi2[sel] = res.edge_chi2
        dok[sel] = res.edge_depth_ok
    r0 = shard_results[0]
    return BAResult(r0.pose_q, r0.pose_t, pts, chi2, dok, r0.initial_chi2, r0.final_chi2, r0.iterations_done,
                    r0.lm_trials)

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


# ---------------------------------------------------------------------------------------------
# Sharding by keyframe segments (the distributed nested dissection, csrc/ba_nd.hip): shard r holds
# the landmarks of segment r, so its partial reduced camera system has complete interior rows and
# the ranks exchange only the separator system and the pose update.
# ---------------------------------------------------------------------------------------------
def pose_blocks(prob):
    """The coupled pose pairs (i <= j, optimised-pose order) of a problem: poses that observe a
    common landmark (the 6x6 blocks of its reduced camera system). Returns (np, bi, bj)."""
    p = prob.normalized()
    opt = np.cumsum(1 - p.pose_fixed.astype(np.int64)) - 1
    opt[p.pose_fixed == 1] = -1
    npo = int((p.pose_fixed == 0).sum())
    oe = opt[p.edge_pose]
    keep = oe >= 0
    pts, po = p.edge_point[keep], oe[keep]
    order = np.lexsort((po, pts))
    pts, po = pts[order], po[order]
    pairs = set()
    start = 0
    for k in range(1, len(pts) + 1):
        if k == len(pts) or pts[k] != pts[start]:
            q = np.unique(po[start:k])
            for a in range(len(q)):
                for b in range(a, len(q)):
                    pairs.add((int(q[a]), int(q[b])))
            start = k
    for i in range(npo):
        pairs.add((i, i))
    pr = sorted(pairs)
    return npo, np.array([a for a, _ in pr], np.int32), np.array([b for _, b in pr], np.int32)


def nd_segments(npo: int, bi, bj, nshards: int):
    """The dissection ba_nd.hip plans for nshards segments (nd_bandwidth + nd_plan_band): returns
    dict(w, cyclic, seg) or None when an interior would be narrower than the band."""
    d = np.abs(np.asarray(bj, np.int64) - np.asarray(bi, np.int64))
    wl = int(d.max()) if d.size else 0
    wc = int(np.minimum(d, npo - d).max()) if d.size else 0
    cyc = wl > wc
    w = max(1, wc if cyc else wl)
    if nshards < 2:
        return None
    seg = [r * npo // nshards for r in range(nshards + 1)]
    for r in range(nshards):
        own = cyc or r < nshards - 1
        if seg[r + 1] - seg[r] - (w if own else 0) < w:
            return None
    return dict(w=w, cyclic=cyc, seg=seg)


def segment_of_landmarks(prob, nshards: int):
    """The shard (segment) of every landmark: the segment whose interior it is seen from, else the
    segment owning the separator it is seen from (landmarks seen by fixed poses only: shard 0)."""
    p = prob.normalized()
    npo, bi, bj = pose_blocks(p)
    plan = nd_segments(npo, bi, bj, nshards)
    if plan is None:
        raise ValueError("the pose graph is not a band narrow enough for this many segments")
    seg, w, K = plan["seg"], plan["w"], nshards
    opt = np.cumsum(1 - p.pose_fixed.astype(np.int64)) - 1
    opt[p.pose_fixed == 1] = -1
    interior_of = np.full(npo, -1, np.int64)
    sep_of = np.full(npo, -1, np.int64)
    for r in range(K):
        own = plan["cyclic"] or r < K - 1
        end = seg[r + 1] - (w if own else 0)
        interior_of[seg[r]:end] = r
        if own:
            sep_of[end:seg[r + 1]] = r
    M = p.points.shape[0]
    shard = np.zeros(M, np.int64)
    best_int = np.full(M, -1, np.int64)
    best_sep = np.full(M, -1, np.int64)
    oe = opt[p.edge_pose]
    for e in np.nonzero(oe >= 0)[0]:
        m, q = int(p.edge_point[e]), int(oe[e])
        if interior_of[q] >= 0:
            best_int[m] = interior_of[q]
        elif best_sep[m] < 0:
            best_sep[m] = sep_of[q]
    shard = np.where(best_int >= 0, best_int, np.where(best_sep >= 0, best_sep, 0))
    return shard, plan


def shard_problem_nd(prob, rank: int, nshards: int):
    """The rank's shard for a sharded solve by segments: all poses, the landmarks of segment `rank`
    (re-indexed from 0, in landmark order) and their edges (in the problem's edge order).
    Returns (shard BAProblem, landmark indices, edge indices into the full problem)."""
    from .optimizer import BAProblem
    p = prob.normalized()
    shard, _ = segment_of_landmarks(p, nshards)
    pts = np.nonzero(shard == rank)[0]
    remap = np.full(p.points.shape[0], -1, np.int64)
    remap[pts] = np.arange(pts.size)
    sel = np.nonzero(remap[p.edge_point] >= 0)[0]
    sh = BAProblem(p.pose_q, p.pose_t, p.pose_fixed, p.points[pts].copy(), p.edge_pose[sel].copy(),
                   remap[p.edge_point[sel]].astype(np.int32), p.edge_uv[sel].copy(), p.edge_octave[sel].copy(),
                   p.inv_sigma2, p.fx, p.fy, p.cx, p.cy, p.huber_delta, p.iterations, p.early_stop)
    return sh, pts, sel


def merge_results_nd(prob, shard_results, point_sets, edge_sets):
    """Full-problem BAResult from the shards of shard_problem_nd (poses from shard 0)."""
    from .optimizer import BAResult
    M, E = prob.points.shape[0], prob.edge_pose.shape[0]
    pts = np.zeros((M, 3), np.float32)
    chi2 = np.zeros(E, np.float32)
    dok = np.zeros(E, np.uint8)
    for res, ps, sel in zip(shard_results, point_sets, edge_sets):
        pts[ps] = res.points
        chi2[sel] = res.edge_chi2
        dok[sel] = res.edge_depth_ok
    r0 = shard_results[0]
    return BAResult(r0.pose_q, r0.pose_t, pts, chi2, dok, r0.initial_chi2, r0.final_chi2, r0.iterations_done,
                    r0.lm_trials)


# ---------------------------------------------------------------------------------------------
# Batched front-end (C3) over ranks: SURVEY.md §8e "Extract: contiguous batch slices, B/N per GPU;
# Match: frame pairs (i, i+1) partitioned, each GPU also loads the first frame of the next slice".
# ---------------------------------------------------------------------------------------------
def frame_slices(B: int, nranks: int):
    """Contiguous frame ranges [lo_r, hi_r) covering 0..B-1, sizes differing by at most one."""
    if B < 0 or nranks < 1:
        raise ValueError("frame_slices: B >= 0 and nranks >= 1")
    base, extra = divmod(B, nranks)
    lo, out = 0, []
    for r in range(nranks):
        hi = lo + base + (1 if r < extra else 0)
        out.append((lo, hi))
        lo = hi
    return out


def frame_slice_with_halo(B: int, rank: int, nranks: int):
    """The rank's work for a B-frame extract + consecutive-pair match batch.

    Returns (lo, hi_ext, pair_lo, pair_hi): the rank extracts frames [lo, hi_ext) — its own slice
    plus a one-frame halo (the first frame of the next non-empty slice) — and owns the match pairs
    (i, i+1) for i in [pair_lo, pair_hi). Every pair 0..B-2 is owned by exactly one rank and every
    frame is extracted by its owner (halo frames a second time, by the previous rank). No
    collective is needed: pairs never cross a slice boundary without the halo frame at hand.
    """
    lo, hi = frame_slices(B, nranks)[rank]
    if hi <= lo:
        return lo, lo, lo, lo
    hi_ext = min(hi + 1, B)
    return lo, hi_ext, lo, hi_ext - 1

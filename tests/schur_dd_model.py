"""Test-side model (moved out of the product package in r05): the r03 torch restatement of the
distributed C5 step, superseded on the device by csrc/ba_nd.hip (segment-dissected, device-driven).
Kept as the arithmetic reference of tests/test_schur_dd_dist.py and tools/model_c5_dd.py.

Domain decomposition of the C5 reduced camera system over ranks (SURVEY.md §8e, row "GBA
sharded"): the distributed LM step's linear solve.

Why: with landmark shards (sharding.py) every rank builds a partial reduced camera system S and an
all-reduce sums it, but every rank then factors the whole n = 2394 system, the 0.68 ms that is 70%
of a C5 LM iteration: more GPUs cannot shorten it. The poses of a GlobalBundleAdjustment loop are
coupled only inside a co-visibility window (Optimizer::GlobalBundleAdjustemnt over the map's
keyframes, SURVEY.md C5: 400 KF loop, 20-KF window), so S is a cyclic block band and a nested
dissection by keyframe segments splits its factorization:

  segment r = keyframes [r*seg, (r+1)*seg): interior I_r = its first seg - sep keyframes, separator
  Z_r = its last sep = window - 1 keyframes. Two interiors are never coupled (a window of `window`
  keyframes cannot reach across a separator), interior I_r touches only Z_{r-1} and Z_r.
  Landmarks go to the rank of the interior their window touches (a window touches at most one),
  separator-only landmarks to the separator's rank, so rank r's partial S lives on
  Z_{r-1} + I_r + Z_r and its interior rows are complete without any exchange.

The step, per rank (`dd_solve`: dd_local, one all-reduce, dd_finish, one all-gather):
  1. local:  L = chol(S_II), W = L^-1 S_IZ, y = L^-1 b_I; the separator contribution
             C_r = S_ZZ^(r) - W^T W and c_r = b_Z^(r) - W^T y (Z = Z_{r-1} + Z_r)
  2. one all-reduce of the separator system  S_Z = sum_r C_r,  b_Z = sum_r c_r
     (block-tridiagonal cyclic, n_Z = P * sep * 6; replicated solve, no broadcast)
  3. x_Z = S_Z^-1 b_Z  (every rank)
  4. x_I = L^-T (y - W x_Z), then an all-gather of the interiors (every rank updates all poses)

The result is the full solve x = S^-1 b exactly (up to rounding): S_Z is the Schur complement of
the interiors. This module states the arithmetic with torch tensors (float64) over
torch.distributed (gloo on CPU in the tests; tests/test_schur_dd_dist.py); the modelled 8-rank
C5 time from measured kernel times is in DESIGN.md §C5 sharding.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Partition:
    """Nested dissection of n_kf keyframes (6 variables each) into `ranks` cyclic segments."""
    n_kf: int
    ranks: int
    window: int
    dof: int = 6

    def __post_init__(self):
        if self.ranks < 2:
            raise ValueError("a partition needs >= 2 segments")
        if self.n_kf % self.ranks:
            raise ValueError("n_kf must be a multiple of the segment count")
        self.seg = self.n_kf // self.ranks
        self.sep = self.window - 1
        if self.seg - self.sep < 1:
            raise ValueError("segments shorter than a co-visibility window")

    def interior_kf(self, r: int) -> np.ndarray:
        return np.arange(r * self.seg, r * self.seg + self.seg - self.sep)

    def separator_kf(self, r: int) -> np.ndarray:
        return np.arange((r + 1) * self.seg - self.sep, (r + 1) * self.seg)

    def vars_of(self, kfs: np.ndarray) -> np.ndarray:
        return (kfs[:, None] * self.dof + np.arange(self.dof)[None, :]).reshape(-1)

    def interior(self, r: int) -> np.ndarray:
        return self.vars_of(self.interior_kf(r))

    def adjacent(self, r: int) -> np.ndarray:
        """Z_{r-1} then Z_r (global variable indices)."""
        return np.concatenate([self.vars_of(self.separator_kf((r - 1) % self.ranks)),
                               self.vars_of(self.separator_kf(r))])

    def separator_index(self, r: int) -> np.ndarray:
        """Positions of Z_{r-1} + Z_r inside the separator system (Z_0, Z_1, ... in rank order)."""
        m = self.sep * self.dof
        prev = (r - 1) % self.ranks
        return np.concatenate([np.arange(prev * m, prev * m + m), np.arange(r * m, r * m + m)])

    @property
    def n_sep(self) -> int:
        return self.ranks * self.sep * self.dof


def landmark_rank(part: Partition, first_kf: int) -> int:
    """Rank of a landmark whose window starts at keyframe `first_kf` (cyclic): the interior it
    touches, else the separator's owner."""
    last = first_kf + part.window - 1
    for k in range(first_kf, last + 1):
        r, off = divmod(k % part.n_kf, part.seg)
        if off < part.seg - part.sep:
            return r
    return (first_kf % part.n_kf) // part.seg


def covisibility_system(part: Partition, n_landmarks: int, seed: int = 0, damping: float = 1.0):
    """A reduced camera system with C5's structure, as the per-rank partial systems the landmark
    shards produce: each landmark adds a rank-3 term on its window's poses (the -W V^-1 W^T of its
    elimination, here + B B^T, SPD), each pose a damped diagonal block (the LM-damped pose
    Hessian). Returns (list of per-rank dense partial S, list of per-rank partial b)."""
    rng = np.random.default_rng(seed)
    n = part.n_kf * part.dof
    Ss = [np.zeros((n, n)) for _ in range(part.ranks)]
    bs = [np.zeros(n) for _ in range(part.ranks)]
    for _ in range(n_landmarks):
        s = int(rng.integers(part.n_kf))
        kfs = (s + np.arange(part.window)) % part.n_kf
        idx = part.vars_of(kfs)
        B = rng.standard_normal((idx.size, 3)) / np.sqrt(part.window)
        r = landmark_rank(part, s)
        Ss[r][np.ix_(idx, idx)] += B @ B.T
        bs[r][idx] += B @ rng.standard_normal(3)
    for k in range(part.n_kf):   # pose blocks: to the rank owning the keyframe
        r = k // part.seg
        idx = part.vars_of(np.array([k]))
        A = rng.standard_normal((part.dof, part.dof))
        Ss[r][np.ix_(idx, idx)] += A @ A.T / part.dof + damping * np.eye(part.dof)
    return Ss, bs


def split_assembled(S, b, part: Partition):
    """Per-rank partial systems of an ASSEMBLED system with the partition's structure (every
    rank holds the sum, e.g. the separator system after the all-reduce): rank r keeps its
    interior's rows and columns and the diagonal block of its own separator Z_r, so the ranks'
    parts sum to S again. Used for a second dissection level on the separator system
    (Partition(ranks, ranks // 2, 2, dof = sep * 6): odd separators become the interiors)."""
    n = S.shape[0]
    Ss, bs = [], []
    for r in range(part.ranks):
        I, Zr = part.interior(r), part.vars_of(part.separator_kf(r))
        A = np.zeros((n, n))
        A[I, :] = S[I, :]
        A[:, I] = S[:, I]
        A[np.ix_(Zr, Zr)] = S[np.ix_(Zr, Zr)]
        bb = np.zeros(n)
        bb[I] = b[I]
        bb[Zr] = b[Zr]
        Ss.append(A)
        bs.append(bb)
    return Ss, bs


def dd_local(S_r, b_r, part: Partition, rank: int):
    """Step 1 on rank `rank` (torch float64): factor the interior, eliminate it. Returns
    (state, Sz, bz): this rank's contribution to the separator system, scattered to its size."""
    import torch
    I = torch.as_tensor(part.interior(rank))
    Zv = torch.as_tensor(part.adjacent(rank))
    S_II = S_r[I][:, I]
    S_IZ = S_r[I][:, Zv]
    S_ZZ = S_r[Zv][:, Zv]
    L = torch.linalg.cholesky(S_II)
    W = torch.linalg.solve_triangular(L, S_IZ, upper=False)
    y = torch.linalg.solve_triangular(L, b_r[I].unsqueeze(1), upper=False)
    zi = torch.as_tensor(part.separator_index(rank))
    Sz = torch.zeros((part.n_sep, part.n_sep), dtype=torch.float64)
    bz = torch.zeros(part.n_sep, dtype=torch.float64)
    Sz[zi.unsqueeze(1), zi.unsqueeze(0)] += S_ZZ - W.T @ W
    bz[zi] += b_r[Zv] - (W.T @ y).squeeze(1)
    return (L, W, y, zi), Sz, bz


def dd_finish(state, Sz, bz):
    """Steps 3-4 after the all-reduce: the separator solve (replicated) and this rank's
    interior. Returns (x_interior, x_separators)."""
    import torch
    L, W, y, zi = state
    xz = torch.cholesky_solve(bz.unsqueeze(1), torch.linalg.cholesky(Sz)).squeeze(1)
    xi = torch.linalg.solve_triangular(L.T, y - W @ xz[zi].unsqueeze(1), upper=True).squeeze(1)
    return xi, xz


def dd_finish_given(state, xz):
    """dd_finish with the separator solution already known (the second level solved it)."""
    import torch
    L, W, y, zi = state
    xi = torch.linalg.solve_triangular(L.T, y - W @ xz[zi].unsqueeze(1), upper=True).squeeze(1)
    return xi, xz


def dd_assemble(xis, xz, part: Partition):
    """The full x from every rank's interior (the all-gather) and the separators."""
    import torch
    x = torch.zeros(part.n_kf * part.dof, dtype=torch.float64)
    m = part.sep * part.dof
    for r in range(part.ranks):
        x[torch.as_tensor(part.interior(r))] = xis[r]
        x[torch.as_tensor(part.vars_of(part.separator_kf(r)))] = xz[r * m:(r + 1) * m]
    return x


def dd_solve(S_r, b_r, part: Partition, rank: int, group=None):
    """The distributed solve on this rank over torch.distributed (one all-reduce of the separator
    system, one all-gather of the interiors). S_r, b_r: this rank's partial system (torch
    float64; only Z_{r-1} + I_r + Z_r are read). Returns the full x on every rank."""
    import torch
    import torch.distributed as dist
    state, Sz, bz = dd_local(S_r, b_r, part, rank)
    flat = torch.cat([Sz.reshape(-1), bz])
    dist.all_reduce(flat, group=group)
    nz = part.n_sep
    xi, xz = dd_finish(state, flat[:nz * nz].reshape(nz, nz), flat[nz * nz:])
    xis = [torch.empty_like(xi) for _ in range(part.ranks)]
    dist.all_gather(xis, xi, group=group)
    return dd_assemble(xis, xz, part)


def dd_solve_local(Ss, bs, part: Partition):
    """Every rank in one process (the all-reduce a sum): dd_solve's arithmetic at any shape
    without a process group."""
    import torch
    loc = [dd_local(torch.as_tensor(S), torch.as_tensor(b), part, r) for r, (S, b) in enumerate(zip(Ss, bs))]
    Sz = sum(l[1] for l in loc)
    bz = sum(l[2] for l in loc)
    fin = [dd_finish(l[0], Sz, bz) for l in loc]
    return dd_assemble([f[0] for f in fin], fin[0][1], part)


def dd_solve_separator_two_level(Sz, bz, part: Partition):
    """The separator system's second dissection level (ba_nd.hip nd_inner_plan, replicated on every
    rank after the all-reduce): the even separators eliminated as interiors, the odd ones solved
    densely (Partition(K, K // 2, 2, dof = sep * 6); K even here)."""
    import torch
    p2 = Partition(part.ranks, part.ranks // 2, 2, dof=part.sep * part.dof)
    S2, b2 = split_assembled(Sz.numpy(), bz.numpy(), p2)
    return dd_solve_local(S2, b2, p2).to(torch.float64)


def dd_solve_segments(Ss_loc, bs_loc, part: Partition, rank: int, group=None, levels: int = 1):
    """Ranks x local segments (the device's orbhip_ba_solve_sharded_segments): this rank holds
    segments rank*L .. rank*L+L-1 of part.ranks = world*L (Ss_loc / bs_loc: their partial systems).
    The local separator contributions are summed in-process first, then one all-reduce; every
    segment finishes its interior, and the pose update is summed over the ranks (each interior once,
    the separators from rank 0) like the device's kNdX all-reduce. Returns the full x."""
    import torch
    import torch.distributed as dist
    L = len(Ss_loc)
    loc = [dd_local(torch.as_tensor(S), torch.as_tensor(b), part, rank * L + j) for j, (S, b) in
           enumerate(zip(Ss_loc, bs_loc))]
    nz = part.n_sep
    flat = torch.cat([sum(l[1] for l in loc).reshape(-1), sum(l[2] for l in loc)])
    dist.all_reduce(flat, group=group)
    Sz, bz = flat[:nz * nz].reshape(nz, nz), flat[nz * nz:]
    x = torch.zeros(part.n_kf * part.dof, dtype=torch.float64)
    m = part.sep * part.dof
    xz2 = dd_solve_separator_two_level(Sz, bz, part) if levels > 1 else None
    for j, l in enumerate(loc):
        r = rank * L + j
        xi, xz = dd_finish(l[0], Sz, bz) if xz2 is None else dd_finish_given(l[0], xz2)
        x[torch.as_tensor(part.interior(r))] = xi
        if rank == 0 and j == 0:
            for t in range(part.ranks):
                x[torch.as_tensor(part.vars_of(part.separator_kf(t)))] = xz[t * m:(t + 1) * m]
    dist.all_reduce(x, group=group)
    return x

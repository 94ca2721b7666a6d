"""Optimizer mirror (U:src/Optimizer.cc) over liborbhip.so.

``Optimizer.LocalBundleAdjustment(problem)`` runs the g2o problem LocalBundleAdjustment
builds (VertexSE3Expmap poses, marginalised VertexSBAPointXYZ points, EdgeSE3ProjectXYZ
mono edges with Huber sqrt(5.991), BlockSolver_6_3 + Levenberg, optimize(10)) on the GPU
and returns the optimised poses/points and the per-edge chi2 / depth flags that the
reference uses to erase outlier observations (chi2 > 5.991 or depth <= 0).
``Optimizer.BundleAdjustment`` is the same solver with the GBA defaults.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import BAProblemC, BAResultC, Context, PoseProblemC, PoseResultC, check, lib, ptr

TH_HUBER_MONO = float(np.sqrt(np.float32(5.991)))


@dataclass
class BAProblem:
    pose_q: np.ndarray          # [P,4] float32 (x,y,z,w), Tcw rotation
    pose_t: np.ndarray          # [P,3] float32
    pose_fixed: np.ndarray      # [P] uint8
    points: np.ndarray          # [M,3] float32 world
    edge_pose: np.ndarray       # [E] int32
    edge_point: np.ndarray      # [E] int32
    edge_uv: np.ndarray         # [E,2] float32
    edge_octave: np.ndarray     # [E] int32
    inv_sigma2: np.ndarray      # [L] float32
    fx: float
    fy: float
    cx: float
    cy: float
    huber_delta: float = TH_HUBER_MONO
    iterations: int = 10
    early_stop: int = 0

    def normalized(self) -> "BAProblem":
        c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
        return BAProblem(c(self.pose_q, np.float32), c(self.pose_t, np.float32), c(self.pose_fixed, np.uint8),
                         c(self.points, np.float32), c(self.edge_pose, np.int32), c(self.edge_point, np.int32),
                         c(self.edge_uv, np.float32), c(self.edge_octave, np.int32), c(self.inv_sigma2, np.float32),
                         float(self.fx), float(self.fy), float(self.cx), float(self.cy), float(self.huber_delta),
                         int(self.iterations), int(self.early_stop))

    def to_c(self) -> BAProblemC:
        return BAProblemC(self.pose_q.shape[0], self.points.shape[0], self.edge_pose.shape[0], ptr(self.pose_q),
                          ptr(self.pose_t), ptr(self.pose_fixed), ptr(self.points), ptr(self.edge_pose),
                          ptr(self.edge_point), ptr(self.edge_uv), ptr(self.edge_octave), ptr(self.inv_sigma2),
                          self.inv_sigma2.shape[0], self.fx, self.fy, self.cx, self.cy, self.huber_delta,
                          self.iterations, self.early_stop)


@dataclass
class BAResult:
    pose_q: np.ndarray
    pose_t: np.ndarray
    points: np.ndarray
    edge_chi2: np.ndarray
    edge_depth_ok: np.ndarray
    initial_chi2: float
    final_chi2: float
    iterations_done: int
    lm_trials: int

    def outlier_edges(self, th: float = 5.991) -> np.ndarray:
        """Edges LocalBundleAdjustment erases: chi2 > 5.991 || !isDepthPositive()."""
        return np.nonzero((self.edge_chi2 > th) | (self.edge_depth_ok == 0))[0]


@dataclass
class PoseProblem:
    """The g2o problem Optimizer::PoseOptimization(Frame*) builds for one monocular Frame: the
    initial Tcw and, per matched MapPoint, its world position and the undistorted keypoint."""
    pose_q: np.ndarray          # [4] float32 (x,y,z,w), pFrame->GetPose() rotation
    pose_t: np.ndarray          # [3] float32
    points: np.ndarray          # [N,3] float32 MapPoint::GetWorldPos
    uv: np.ndarray              # [N,2] float32 mvKeysUn[i].pt
    octave: np.ndarray          # [N] int32 mvKeysUn[i].octave
    inv_sigma2: np.ndarray      # [L] float32 mvInvLevelSigma2
    fx: float
    fy: float
    cx: float
    cy: float

    def normalized(self) -> "PoseProblem":
        c = lambda a, dt: np.ascontiguousarray(a, dtype=dt)  # noqa: E731
        return PoseProblem(c(self.pose_q, np.float32).reshape(4), c(self.pose_t, np.float32).reshape(3),
                           c(self.points, np.float32).reshape(-1, 3), c(self.uv, np.float32).reshape(-1, 2),
                           c(self.octave, np.int32).reshape(-1), c(self.inv_sigma2, np.float32),
                           float(self.fx), float(self.fy), float(self.cx), float(self.cy))

    def to_c(self) -> PoseProblemC:
        return PoseProblemC(self.points.shape[0], ptr(self.pose_q), ptr(self.pose_t), ptr(self.points), ptr(self.uv),
                            ptr(self.octave), ptr(self.inv_sigma2), self.inv_sigma2.shape[0], self.fx, self.fy,
                            self.cx, self.cy)


@dataclass
class PoseResult:
    pose_q: np.ndarray          # optimised Tcw
    pose_t: np.ndarray
    outlier: np.ndarray         # [N] uint8: mvbOutlier
    n_inliers: int              # PoseOptimization return value
    lm_trials: int


@dataclass
class BABatch:
    """A batch of problems in C-ABI form (Optimizer.prepare_batch); run_batch solves it in place."""
    problems: list
    outs: list
    cprobs: object
    cres: object


class Optimizer:
    def __init__(self, device: int = -1, ctx: Context | None = None):
        self.ctx = ctx or Context(device)

    def solve(self, prob: BAProblem, stop_flag: ctypes.c_int | None = None) -> BAResult:
        p = prob.normalized()
        P, M, E = p.pose_q.shape[0], p.points.shape[0], p.edge_pose.shape[0]
        # (every output word is written by the solve: no zero fill)
        out = BAResult(np.empty((P, 4), np.float32), np.empty((P, 3), np.float32), np.empty((M, 3), np.float32),
                       np.empty(E, np.float32), np.empty(E, np.uint8), 0.0, 0.0, 0, 0)
        rc = BAResultC(ptr(out.pose_q), ptr(out.pose_t), ptr(out.points), ptr(out.edge_chi2),
                       ptr(out.edge_depth_ok), 0.0, 0.0, 0, 0)
        pc = p.to_c()
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve(self.ctx.handle, ctypes.byref(pc), ctypes.byref(rc), sf), "orbhip_ba_solve")
        out.initial_chi2, out.final_chi2 = rc.initial_chi2, rc.final_chi2
        out.iterations_done, out.lm_trials = rc.iterations_done, rc.lm_trials
        return out

    def prepare_single(self, prob: BAProblem) -> "BABatch":
        """The C-ABI view of one problem (orbhip_ba_problem / orbhip_ba_result over the problem's
        own arrays and fresh outputs), as LocalMapping's C++ adapter holds it:
        run_single is the orbhip_ba_solve call alone, without solve()'s per-call marshalling."""
        p = prob.normalized()
        outs, cres = self._results_for([p])
        return BABatch([p], outs, p.to_c(), cres)

    def run_single(self, single: "BABatch", stop_flag: ctypes.c_int | None = None) -> BAResult:
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve(self.ctx.handle, ctypes.byref(single.cprobs), single.cres, sf), "orbhip_ba_solve")
        return self._fill(single.outs, single.cres)[0]

    def solve_batch(self, probs, stop_flag: ctypes.c_int | None = None):
        """B independent problems in one batched solve (replicas); returns a list of BAResult."""
        return self.run_batch(self.prepare_batch(probs), stop_flag)

    def prepare_batch(self, probs) -> "BABatch":
        """The C-ABI view of a batch (orbhip_ba_problem / orbhip_ba_result arrays over the
        problems' own arrays and freshly allocated outputs), as a C++ host adapter holds it: the
        Python marshalling is done once here, run_batch is the orbhip_ba_solve_batch call alone."""
        ps = [p.normalized() for p in probs]
        outs, cres = self._results_for(ps)
        cprobs = (BAProblemC * len(ps))(*[p.to_c() for p in ps])
        return BABatch(ps, outs, cprobs, cres)

    def run_batch(self, batch: "BABatch", stop_flag: ctypes.c_int | None = None):
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve_batch(self.ctx.handle, batch.cprobs, len(batch.problems), batch.cres, sf),
              "orbhip_ba_solve_batch")
        return self._fill(batch.outs, batch.cres)

    # ---- sharded BundleAdjustment ----
    def _results_for(self, ps):
        outs, cres = [], (BAResultC * len(ps))()
        for i, p in enumerate(ps):
            P, M, E = p.pose_q.shape[0], p.points.shape[0], p.edge_pose.shape[0]
            o = BAResult(np.zeros((P, 4), np.float32), np.zeros((P, 3), np.float32), np.zeros((M, 3), np.float32),
                         np.zeros(E, np.float32), np.zeros(E, np.uint8), 0.0, 0.0, 0, 0)
            outs.append(o)
            cres[i] = BAResultC(ptr(o.pose_q), ptr(o.pose_t), ptr(o.points), ptr(o.edge_chi2), ptr(o.edge_depth_ok),
                                0.0, 0.0, 0, 0)
        return outs, cres

    @staticmethod
    def _fill(outs, cres):
        for o, r in zip(outs, cres):
            o.initial_chi2, o.final_chi2, o.iterations_done, o.lm_trials = (r.initial_chi2, r.final_chi2,
                                                                              r.iterations_done, r.lm_trials)
        return outs

    def solve_shards_local(self, shards, stop_flag: ctypes.c_int | None = None):
        """All shards of one problem in this process, summed on the device (orbhip_ba_solve_shards_local)."""
        ps = [p.normalized() for p in shards]
        outs, cres = self._results_for(ps)
        cprobs = (BAProblemC * len(ps))(*[p.to_c() for p in ps])
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve_shards_local(self.ctx.handle, cprobs, len(ps), cres, sf),
              "orbhip_ba_solve_shards_local")
        return self._fill(outs, cres)

    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib().orbhip_comm_unique_id(buf), "orbhip_comm_unique_id")
        return bytes(buf)

    def comm_init(self, nranks: int, rank: int, unique_id: bytes):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().orbhip_comm_init(self.ctx.handle, int(nranks), int(rank), buf), "orbhip_comm_init")

    def solve_sharded(self, shard: BAProblem, stop_flag: ctypes.c_int | None = None) -> BAResult:
        """This rank's shard of a problem solved jointly over RCCL (after comm_init)."""
        p = shard.normalized()
        outs, cres = self._results_for([p])
        pc = p.to_c()
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve_sharded(self.ctx.handle, ctypes.byref(pc), cres, sf), "orbhip_ba_solve_sharded")
        return self._fill(outs, cres)[0]

    def solve_sharded_segments(self, shards, stop_flag: ctypes.c_int | None = None):
        """This rank's consecutive shards (segments rank*len .. of nranks*len, sharding.shard_problem_nd)
        solved jointly over RCCL (after comm_init): summed on the device, then all-reduced."""
        ps = [p.normalized() for p in shards]
        outs, cres = self._results_for(ps)
        cprobs = (BAProblemC * len(ps))(*[p.to_c() for p in ps])
        sf = ctypes.addressof(stop_flag) if stop_flag is not None else None
        check(lib().orbhip_ba_solve_sharded_segments(self.ctx.handle, cprobs, len(ps), cres, sf),
              "orbhip_ba_solve_sharded_segments")
        return self._fill(outs, cres)

    def stats(self) -> dict:
        """orbhip_ba_stats: persistent-Cholesky launches on this device (all contexts), those that
        first waited for another stream's solve, the hand-off timeouts this context saw and the
        solves it re-ran on the non-persistent solvers."""
        out = (ctypes.c_int64 * 4)()
        check(lib().orbhip_ba_stats(self.ctx.handle, out), "orbhip_ba_stats")
        return dict(dag_launches=out[0], dag_handoffs=out[1], dag_timeouts=out[2], dag_reruns=out[3])

    def LocalBundleAdjustment(self, prob: BAProblem, stop_flag=None) -> BAResult:
        return self.solve(prob, stop_flag)

    def BundleAdjustment(self, prob: BAProblem, nIterations: int = 20, bRobust: bool = True,
                         stop_flag=None) -> BAResult:
        p = BAProblem(**{**prob.__dict__, "iterations": nIterations,
                         "huber_delta": float(np.sqrt(5.99)) if bRobust else 0.0})
        return self.solve(p, stop_flag)

    # ---- motion-only BA ----
    def PoseOptimization(self, prob: PoseProblem) -> PoseResult:
        """U:src/Optimizer.cc::Optimizer::PoseOptimization(Frame*) for one frame."""
        return self.PoseOptimization_batch([prob])[0]

    def PoseOptimization_batch(self, probs) -> list:
        """Several frames in one launch (one wavefront per frame)."""
        ps = [p.normalized() for p in probs]
        outl = [np.zeros(p.points.shape[0], np.uint8) for p in ps]
        cprobs = (PoseProblemC * len(ps))(*[p.to_c() for p in ps])
        cres = (PoseResultC * len(ps))()
        for i, o in enumerate(outl):
            cres[i].outlier = ptr(o)
        check(lib().orbhip_pose_optimization_batch(self.ctx.handle, cprobs, len(ps), cres),
              "orbhip_pose_optimization_batch")
        return [PoseResult(np.array(r.pose_q[:], np.float32), np.array(r.pose_t[:], np.float32), o, r.n_inliers,
                           r.lm_trials) for r, o in zip(cres, outl)]

"""ORBmatcher mirror (U:src/ORBmatcher.cc) over liborbhip.so.

``DescriptorDistance`` is the SWAR popcount of the reference. ``match_bf`` applies the
acceptance rule shared by SearchByBoW / SearchForInitialization — best/second over the
train set, ``best <= TH_LOW`` and ``best < mfNNratio * second``, then the 30-bin rotation
histogram (ComputeThreeMaxima) when ``mbCheckOrientation`` — order-free over the whole
train set (the C3 brute-force matcher). ``SearchForInitialization`` is the reference function
itself, with its windowed, greedy (stealing) one-to-one semantics.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import (KP_DTYPE, FrameC, InitFrameC, LocalPointsC, ProjLastC, torch_stream, Context, check, lib, ptr)


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = -1, ctx: Context | None = None):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.ctx = ctx or Context(device)
        self._lp_cache = None   # SearchLocalPoints: the C view of the last call's map-point arrays

    @staticmethod
    def DescriptorDistance(a, b) -> int:
        a = np.ascontiguousarray(a, np.uint8).reshape(32)
        b = np.ascontiguousarray(b, np.uint8).reshape(32)
        return check(lib().orbhip_descriptor_distance(ptr(a), ptr(b)), "DescriptorDistance")

    def match_bf(self, q_desc, q_angle, t_desc, t_angle, th_low: int | None = None):
        """Returns (nmatches, match[nq] (train idx or -1), best[nq], second[nq])."""
        q = np.ascontiguousarray(q_desc, np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(t_desc, np.uint8).reshape(-1, 32)
        qa = np.ascontiguousarray(q_angle, np.float32).reshape(-1)
        ta = np.ascontiguousarray(t_angle, np.float32).reshape(-1)
        nq, nt = q.shape[0], t.shape[0]
        m = np.full(nq, -1, np.int32); b = np.zeros(nq, np.int32); s = np.zeros(nq, np.int32)
        th = self.TH_LOW if th_low is None else int(th_low)
        n = lib().orbhip_match_bf(self.ctx.handle, ptr(q), ptr(qa), nq, ptr(t), ptr(ta), nt, th,
                                  ctypes.c_float(self.mfNNratio), int(self.mbCheckOrientation),
                                  ptr(m), ptr(b), ptr(s))
        return check(n, "orbhip_match_bf"), m, b, s

    def match_pairs_device(self, kps, desc, n, match, best, second, nmatch, th_low=None, stream=None):
        """Device tensors from ORBextractor.extract_batch_device: match frame p -> p+1."""
        B, cap = desc.shape[0], desc.shape[1]
        th = self.TH_LOW if th_low is None else int(th_low)
        st = torch_stream(stream)
        check(lib().orbhip_match_pairs_device(self.ctx.handle, ptr(kps), ptr(desc), ptr(n), B, cap, th,
                                              ctypes.c_float(self.mfNNratio), int(self.mbCheckOrientation),
                                              ptr(match), ptr(best), ptr(second), ptr(nmatch), st),
              "orbhip_match_pairs_device")

    def SearchByBoW(self, kf_desc, kf_angle, kf_node, kf_weight, kf_valid, f_desc, f_angle, f_node, f_weight,
                    th_low: int | None = None):
        """U:src/ORBmatcher.cc::SearchByBoW(KeyFrame*, Frame&, vpMapPointMatches) on the GPU.
        node / weight come from ORBVocabulary.transform_features (FeatureVector = weight > 0);
        kf_valid[i]: the KF feature has a good map point. Returns (nmatches, match[nf]) with
        match[f] = KF feature index (its MapPoint in the reference) or -1."""
        c = np.ascontiguousarray
        kd, fd = c(kf_desc, np.uint8).reshape(-1, 32), c(f_desc, np.uint8).reshape(-1, 32)
        ka, fa = c(kf_angle, np.float32), c(f_angle, np.float32)
        kn, fn = c(kf_node, np.int32), c(f_node, np.int32)
        kw, fw = c(kf_weight, np.float64), c(f_weight, np.float64)
        kv = c(kf_valid, np.uint8)
        nkf, nf = kd.shape[0], fd.shape[0]
        m = np.full(nf, -1, np.int32)
        th = self.TH_LOW if th_low is None else int(th_low)
        n = check(lib().orbhip_search_bow(self.ctx.handle, ptr(kd), ptr(ka), ptr(kn), ptr(kw), ptr(kv), nkf, ptr(fd),
                                          ptr(fa), ptr(fn), ptr(fw), nf, ctypes.c_float(self.mfNNratio),
                                          int(self.mbCheckOrientation), th, ptr(m)), "orbhip_search_bow")
        return n, m

    def SearchForInitialization(self, kps1, desc1, kps2, desc2, vbPrevMatched, windowSize: int = 10,
                                bounds2=(0.0, 640.0, 0.0, 480.0)):
        """U:src/ORBmatcher.cc::SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize)
        with the exact greedy semantics (Tracking::MonocularInitialization uses ORBmatcher(0.9, true)
        and windowSize 100). kps: orbhip_kp records; bounds2 = F2's (mnMinX, mnMaxX, mnMinY, mnMaxY).
        Returns (nmatches, vnMatches12, vbPrevMatched updated for the matches)."""
        k1 = np.ascontiguousarray(kps1, KP_DTYPE); k2 = np.ascontiguousarray(kps2, KP_DTYPE)
        d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
        prev = np.ascontiguousarray(vbPrevMatched, np.float32).reshape(-1, 2).copy()
        m = np.full(k1.shape[0], -1, np.int32)
        f1 = InitFrameC(k1.shape[0], ptr(k1), ptr(d1), 0.0, 1.0, 0.0, 1.0)
        f2 = InitFrameC(k2.shape[0], ptr(k2), ptr(d2), *[float(b) for b in bounds2])
        n = check(lib().orbhip_search_for_initialization(self.ctx.handle, ctypes.byref(f1), ctypes.byref(f2),
                                                         ptr(prev), int(windowSize), ctypes.c_float(self.mfNNratio),
                                                         int(self.mbCheckOrientation), ptr(m)),
                  "orbhip_search_for_initialization")
        return n, m, prev

    # ---- projection-guided matching ----
    def SearchByProjectionLastFrame(self, frame: "ProjFrame", points, mp_desc, last_octave, last_angle,
                                    th: float = 15.0):
        """U:src/ORBmatcher.cc::SearchByProjection(CurrentFrame, LastFrame, th, bMono=true).
        Queries = LastFrame entries with a non-outlier MapPoint (index order). Returns
        (nmatches, match[q] = CurrentFrame keypoint or -1)."""
        pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
        d = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        oc = np.ascontiguousarray(last_octave, np.int32)
        an = np.ascontiguousarray(last_angle, np.float32)
        match = np.empty(pts.shape[0], np.int32)   # written in full by the call
        fc = frame.to_c()
        lc = ProjLastC(pts.shape[0], ptr(pts), ptr(d), ptr(oc), ptr(an))
        n = check(lib().orbhip_search_by_projection_last(self.ctx.handle, ctypes.byref(fc), ctypes.byref(lc),
                                                         float(th), int(self.mbCheckOrientation), ptr(match)),
                  "orbhip_search_by_projection_last")
        return n, match

    def SearchLocalPoints(self, frame: "ProjFrame", points, normals, min_dist, max_dist, mp_desc, skip=None,
                          th: float = 1.0, view_cos_limit: float = 0.5, far_points: bool = False,
                          th_far: float = 0.0):
        """Tracking::SearchLocalPoints: Frame::isInFrustum + SearchByProjection(F, vpMapPoints, th,
        bFarPoints, thFarPoints) with this matcher's nnratio. Returns (nmatches, match, in_view, level)."""
        key = (id(points), id(normals), id(min_dist), id(max_dist), id(mp_desc), id(skip))
        hit = self._lp_cache
        if hit is not None and hit[0] == key and all(a is b for a, b in zip(hit[1], (points, normals, min_dist,
                                                                                      max_dist, mp_desc, skip))):
            lc, m = hit[2], hit[3]   # the same arrays as the last call: their C view is still valid
        else:
            pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
            nrm = np.ascontiguousarray(normals, np.float32).reshape(-1, 3)
            mn = np.ascontiguousarray(min_dist, np.float32)
            mx = np.ascontiguousarray(max_dist, np.float32)
            d = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
            sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
            m = pts.shape[0]
            lc = LocalPointsC(m, ptr(pts), ptr(nrm), ptr(mn), ptr(mx), ptr(d), ptr(sk))
            # cached only when no conversion copied an input (the view then reads the caller's
            # memory, so in-place updates are seen); the inputs live with it, so their ids stay theirs
            srcs = (points, normals, min_dist, max_dist, mp_desc, skip)
            views = (pts, nrm, mn, mx, d, sk)
            zero_copy = all(v is o or (v is not None and v.base is o) for v, o in zip(views, srcs))
            self._lp_cache = (key, srcs, lc, m, views) if zero_copy else None
        match = np.empty(m, np.int32)      # written in full by the call (m > 0)
        in_view = np.empty(m, np.uint8)
        level = np.empty(m, np.int32)
        fc = frame.to_c()
        n = check(lib().orbhip_search_local_points(self.ctx.handle, ctypes.byref(fc), ctypes.byref(lc),
                                                   float(view_cos_limit), float(th), float(self.mfNNratio),
                                                   int(far_points), float(th_far), ptr(in_view), ptr(level),
                                                   ptr(match)), "orbhip_search_local_points")
        return n, match, in_view, level


class ProjFrame:
    """The current Frame for projection matching (U:src/Frame.cc): keypoints (orbhip_kp records:
    mvKeysUn — PinholeCamera.UndistortKeyPoints for a distorted camera, mvKeys otherwise),
    descriptors, claimed mask, image bounds (Frame::ComputeImageBounds: PinholeCamera
    .ComputeImageBounds, or [0, width] x [0, height] without distortion), scale tables,
    intrinsics and Tcw."""

    def __init__(self, kps, desc, pose_q, pose_t, fx, fy, cx, cy, width=640, height=480, scale_factor=1.2,
                 n_levels=8, claimed=None, bounds=None):
        self.kps = np.ascontiguousarray(kps, KP_DTYPE)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        self.claimed = None if claimed is None else np.ascontiguousarray(claimed, np.uint8)
        self.pose_q = np.asarray(pose_q, np.float32).reshape(4)
        self.pose_t = np.asarray(pose_t, np.float32).reshape(3)
        self.fx, self.fy, self.cx, self.cy = float(fx), float(fy), float(cx), float(cy)
        self.bounds = (0.0, float(width), 0.0, float(height)) if bounds is None else tuple(float(b) for b in bounds)
        sf = np.ones(n_levels, np.float32)
        for i in range(1, n_levels):
            sf[i] = np.float32(np.float64(sf[i - 1]) * np.float64(np.float32(scale_factor)))
        self.scale_factors = sf
        self.log_scale_factor = float(np.log(np.float32(scale_factor)).astype(np.float32))
        self._c = None

    def to_c(self) -> FrameC:
        """The C view. The pointer fields are cached while kps / desc / claimed / scale_factors are
        the same array objects (Tracking keeps them between SearchByProjection and
        SearchLocalPoints); a reassigned array is converted again and its pointer refreshed. The
        scalars (pose, bounds, intrinsics) are re-filled on every call: Tcw changes in place after
        PoseOptimization."""
        arrs = (self.kps, self.desc, self.claimed, self.scale_factors)
        hit = self._c
        if hit is None or any(a is not b for a, b in zip(hit[0], arrs)):
            self.kps = np.ascontiguousarray(self.kps, KP_DTYPE)
            self.desc = np.ascontiguousarray(self.desc, np.uint8).reshape(-1, 32)
            if self.claimed is not None:
                self.claimed = np.ascontiguousarray(self.claimed, np.uint8)
            self.scale_factors = np.ascontiguousarray(self.scale_factors, np.float32)
            c = FrameC()
            c.n = self.kps.shape[0]
            c.kps, c.desc, c.claimed = ptr(self.kps), ptr(self.desc), ptr(self.claimed)
            c.scale_factors, c.n_levels = ptr(self.scale_factors), len(self.scale_factors)
            # the view keeps the arrays it points into alive
            self._c = hit = ((self.kps, self.desc, self.claimed, self.scale_factors), c)
        c = hit[1]
        if self.claimed is not None and self.claimed.shape[0] < c.n:
            raise ValueError("ProjFrame.claimed shorter than kps")
        c.min_x, c.max_x, c.min_y, c.max_y = (float(b) for b in self.bounds)
        c.log_scale_factor = float(self.log_scale_factor)
        c.fx, c.fy, c.cx, c.cy = float(self.fx), float(self.fy), float(self.cx), float(self.cy)
        c.pose_q[:] = [float(v) for v in np.asarray(self.pose_q, np.float32).reshape(4)]
        c.pose_t[:] = [float(v) for v in np.asarray(self.pose_t, np.float32).reshape(3)]
        return c

"""ORBmatcher mirror (U:src/ORBmatcher.cc) over liborbhip.so.

``DescriptorDistance`` is the SWAR popcount of the reference. ``match_bf`` applies the
acceptance rule shared by SearchByBoW / SearchForInitialization — best/second over the
train set, ``best <= TH_LOW`` and ``best < mfNNratio * second``, then the 30-bin rotation
histogram (ComputeThreeMaxima) when ``mbCheckOrientation`` — order-free over the whole
train set (the greedy one-to-one pass of those functions is not applied).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import torch_stream, Context, check, lib, ptr


class ORBmatcher:
    TH_HIGH = 100
    TH_LOW = 50
    HISTO_LENGTH = 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, device: int = 0, ctx: Context | None = None):
        self.mfNNratio = float(nnratio)
        self.mbCheckOrientation = bool(checkOri)
        self.ctx = ctx or Context(device)

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


"""KeyFrameDatabase mirror (U:src/KeyFrameDatabase.cc) over liborbhip.so: add / erase with a
KeyFrame's BowVector, DetectRelocalizationCandidates and DetectNBestCandidates on the device.
KeyFrames are slots 0..max_kf-1 (the adapter's KeyFrame index); BowVectors are (words ascending,
values) pairs as ORBVocabulary.transform returns them."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import Context, KfdbQueryC, check, lib, ptr


def _bow(bow):
    w, v = bow
    return np.ascontiguousarray(w, np.int32), np.ascontiguousarray(v, np.float64)


class KeyFrameDatabase:
    COVIS = 10

    def __init__(self, max_kf: int, device: int = -1, ctx: Context | None = None):
        self.ctx = ctx or Context(device)
        self.max_kf = int(max_kf)
        self._h = ctypes.c_void_p()
        check(lib().orbhip_kfdb_create(self.ctx.handle, self.max_kf, ctypes.byref(self._h)), "orbhip_kfdb_create")

    def add(self, kf: int, bow):
        w, v = _bow(bow)
        check(lib().orbhip_kfdb_add(self._h, int(kf), ptr(w), ptr(v), w.shape[0]), "orbhip_kfdb_add")

    def erase(self, kf: int):
        check(lib().orbhip_kfdb_erase(self._h, int(kf)), "orbhip_kfdb_erase")

    def _query(self, query_id, bow, covis, kf_map, query_map, flags):
        w, v = _bow(bow)
        cv = np.ascontiguousarray(covis, np.int32).reshape(self.max_kf, self.COVIS)
        km = None if kf_map is None else np.ascontiguousarray(kf_map, np.int32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint8)
        keep = (w, v, cv, km, fl)
        q = KfdbQueryC(int(query_id), ptr(w), ptr(v), w.shape[0], ptr(cv), ptr(km), int(query_map), ptr(fl))
        return q, keep

    def DetectRelocalizationCandidates(self, query_id: int, bow, covis, kf_map=None, query_map: int = 0):
        """Frame F (mnId = query_id, mBowVec = bow) against the database; covis[k] = the 10 best
        covisible KF slots of KF k (-1 padded). Returns the candidate slots in upstream order."""
        q, _keep = self._query(query_id, bow, covis, kf_map, query_map, None)
        out = np.zeros(self.max_kf, np.int32)
        n = check(lib().orbhip_kfdb_detect_relocalization(self._h, ctypes.byref(q), ptr(out), self.max_kf),
                  "orbhip_kfdb_detect_relocalization")
        return out[:n].copy()

    def DetectNBestCandidates(self, query_id: int, bow, covis, connected=None, n: int = 3, kf_map=None,
                              query_map: int = 0, flags=None):
        """KeyFrame pKF (mnId = query_id) -> (loop candidate slots, merge candidate slots)."""
        q, _keep = self._query(query_id, bow, covis, kf_map, query_map, flags)
        con = None if connected is None else np.ascontiguousarray(connected, np.uint8)
        lo = np.zeros(max(n, 1), np.int32); me = np.zeros(max(n, 1), np.int32)
        nl, nm = ctypes.c_int32(), ctypes.c_int32()
        check(lib().orbhip_kfdb_detect_nbest(self._h, ctypes.byref(q), ptr(con), int(n), ptr(lo), ctypes.byref(nl),
                                             ptr(me), ctypes.byref(nm)), "orbhip_kfdb_detect_nbest")
        return lo[:nl.value].copy(), me[:nm.value].copy()

    def close(self):
        if self._h:
            lib().orbhip_kfdb_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

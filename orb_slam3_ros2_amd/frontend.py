"""Camera front-end stream: include/orbhip.h orbhip_frontend_* (see there and DESIGN.md).

One camera's frames as Tracking receives them — U:src/Frame.cc Frame(mono) -> ExtractORB ->
U:src/ORBextractor.cc::operator(), then a Hamming match against the last frame — pipelined on
the device over ``frames_in_flight`` contexts (one HIP stream / hardware queue each). ``push``
never blocks; slot outputs are device tensors valid until the slot is reused.
"""
from __future__ import annotations

import ctypes

from ._lib import OrbParams, check, lib


class FrontendSlotC(ctypes.Structure):
    _fields_ = [("frame", ctypes.c_int64), ("cap", ctypes.c_int32), ("slots", ctypes.c_int32),
                ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("n", ctypes.c_void_p),
                ("mono", ctypes.c_void_p), ("match", ctypes.c_void_p), ("best", ctypes.c_void_p),
                ("second", ctypes.c_void_p), ("nmatch", ctypes.c_void_p)]


class _DevArray:
    """Zero-copy view of library-owned device memory for torch (``__cuda_array_interface__``)."""

    def __init__(self, p, shape, typestr):
        self.__cuda_array_interface__ = {"shape": tuple(shape), "typestr": typestr, "data": (int(p), False),
                                         "version": 2, "strides": None}


class _CtxRef:
    """The ``.handle`` of one of the stream's contexts (for orbhip_profile_stage)."""

    def __init__(self, h):
        self.handle = h


class FrameStream:
    def __init__(self, w: int, h: int, frames_in_flight: int = 8, nfeatures=1000, scaleFactor=1.2, nlevels=8,
                 iniThFAST=20, minThFAST=7, th_low: int = 50, nnratio: float = 0.9, checkOri: bool = True,
                 device: int = -1):
        self.w, self.h, self.S = int(w), int(h), int(frames_in_flight)
        self._h = ctypes.c_void_p()
        prm = OrbParams(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST), int(minThFAST))
        check(lib().orbhip_frontend_create(ctypes.byref(self._h), int(device), ctypes.byref(prm), self.w, self.h,
                                           self.S, int(th_low), ctypes.c_float(nnratio), int(bool(checkOri))),
              "orbhip_frontend_create")
        self._push = lib().orbhip_frontend_push
        v = self._view_c(0)
        self.cap, self.slots = v.cap, v.slots

    @property
    def handle(self):
        return self._h

    def context(self, j: int = 0):
        c = ctypes.c_void_p()
        check(lib().orbhip_frontend_context(self._h, int(j), ctypes.byref(c)), "orbhip_frontend_context")
        return _CtxRef(c)

    def push(self, frame, vLappingArea=(0, 1000)) -> int:
        """frame: uint8 CUDA tensor (H, W), rows stride(0) bytes apart. Returns the slot."""
        rc = self._push(self._h, frame.data_ptr(), frame.stride(0), int(vLappingArea[0]), int(vLappingArea[1]))
        return check(rc, "orbhip_frontend_push")

    def push_ptr(self, d_img: int, stride: int, lap0: int = 0, lap1: int = 1000) -> int:
        """Raw form of push (a device address): the per-frame host work is this one C call."""
        return self._push(self._h, d_img, stride, lap0, lap1)

    def _view_c(self, slot: int) -> FrontendSlotC:
        v = FrontendSlotC()
        check(lib().orbhip_frontend_view(self._h, int(slot), ctypes.byref(v)), "orbhip_frontend_view")
        return v

    def view(self, slot: int) -> dict:
        """Device tensors of a slot (zero-copy; valid until the slot is reused)."""
        import torch
        v = self._view_c(slot)
        cap = v.cap

        def t(p, shape, typestr):
            return torch.as_tensor(_DevArray(p, shape, typestr), device="cuda")
        return {"frame": int(v.frame), "kps": t(v.kps, (cap, 6), "<f4"), "desc": t(v.desc, (cap, 32), "|u1"),
                "n": t(v.n, (1,), "<i4"), "mono": t(v.mono, (1,), "<i4"), "match": t(v.match, (cap,), "<i4"),
                "best": t(v.best, (cap,), "<i4"), "second": t(v.second, (cap,), "<i4"),
                "nmatch": t(v.nmatch, (1,), "<i4")}

    def wait(self, slot: int, stream=None):
        """The frame in `slot` complete: blocks the host (stream None) or orders `stream`."""
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else None
        check(lib().orbhip_frontend_wait(self._h, int(slot), st), "orbhip_frontend_wait")

    def close(self):
        if self._h:
            lib().orbhip_frontend_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

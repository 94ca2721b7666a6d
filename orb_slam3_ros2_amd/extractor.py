"""ORBextractor mirror (U:src/ORBextractor.cc) over liborbhip.so.

Same constructor arguments and call semantics as the reference:

    ext = ORBextractor(nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7)
    monoIndex, keypoints, descriptors = ext(image, None, [0, 1000])

``image`` is a 2-D uint8 array (CV_8UC1); an empty image returns (-1, [], None) like
operator(). Keypoints are returned as a structured numpy array with cv::KeyPoint fields
(x, y, size, angle, response, octave); ``KeyPoint`` objects are available via
``to_keypoints``. Batched, device-resident extraction for torch-ROCm tensors is
``extract_batch_device``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np

from ._lib import torch_stream, KP_DTYPE, Context, OrbHipError, check, lib, ptr


@dataclass
class KeyPoint:
    x: float
    y: float
    size: float
    angle: float
    response: float
    octave: int
    class_id: int = -1

    @property
    def pt(self):
        return (self.x, self.y)


def to_keypoints(arr: np.ndarray):
    return [KeyPoint(float(r["x"]), float(r["y"]), float(r["size"]), float(r["angle"]), float(r["response"]),
                     int(r["octave"])) for r in arr]


class ORBextractor:
    """U:src/ORBextractor.cc::ORBextractor — the constructor builds the per-level tables,
    ``__call__`` is ``operator()``."""

    def __init__(self, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7, device=-1):
        self.nfeatures, self.scaleFactor, self.nlevels = int(nfeatures), float(scaleFactor), int(nlevels)
        self.iniThFAST, self.minThFAST = int(iniThFAST), int(minThFAST)
        self.ctx = Context(device, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)
        self._lvl = {}

    # ---- ctor tables (GetScaleFactors / GetLevels ...) ----
    def level_info(self, w: int, h: int):
        L = self.nlevels
        lw = np.zeros(L, np.int32); lh = np.zeros(L, np.int32)
        nf = np.zeros(L, np.int32); sc = np.zeros(L, np.float32)
        check(lib().orbhip_level_info(self.ctx.handle, w, h, ptr(lw), ptr(lh), ptr(nf), ptr(sc)), "level_info")
        return dict(w=lw, h=lh, feats=nf, scales=sc)

    def GetScaleFactors(self):
        return self.level_info(640, 480)["scales"]

    def GetInverseScaleFactors(self):
        return (np.float32(1.0) / self.GetScaleFactors()).astype(np.float32)

    def GetScaleSigmaSquares(self):
        s = self.GetScaleFactors()
        return (s * s).astype(np.float32)

    def GetInverseScaleSigmaSquares(self):
        return (np.float32(1.0) / self.GetScaleSigmaSquares()).astype(np.float32)

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        return self.scaleFactor

    def max_keypoints(self, w: int, h: int) -> int:
        return check(lib().orbhip_max_keypoints(self.ctx.handle, int(w), int(h)), "max_keypoints")

    # ---- operator() ----
    def __call__(self, image, mask=None, vLappingArea=(0, 1000)):
        if image is None or getattr(image, "size", 0) == 0:
            return -1, np.zeros(0, KP_DTYPE), None
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.ndim != 2:
            raise OrbHipError(-1, "ORBextractor expects CV_8UC1")
        h, w = img.shape
        cap = self.max_keypoints(w, h)
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_int(0)
        mono = ctypes.c_int(0)
        rc = lib().orbhip_extract(self.ctx.handle, ptr(img), w, h, w, int(vLappingArea[0]), int(vLappingArea[1]),
                                  ptr(kps), ptr(desc), cap, ctypes.byref(n), ctypes.byref(mono))
        if rc == -6:
            return -1, np.zeros(0, KP_DTYPE), None
        check(rc, "orbhip_extract")
        nk = n.value
        return mono.value, kps[:nk].copy(), (desc[:nk].copy() if nk else None)

    # ---- batched, device-resident (torch-ROCm ingest / benchmarks) ----
    def extract_batch_device(self, frames, kps_out, desc_out, n_out, mono_out, vLappingArea=(0, 1000),
                             stream=None):
        """frames: uint8 CUDA tensor [B, H, W] (rows may be padded: stride(1) bytes per row).
        kps_out: int32/float32 CUDA tensor with >= B*cap*6 elements; desc_out uint8 [B, cap, 32];
        n_out / mono_out int32 [B]. Asynchronous on ``stream`` (torch stream or None)."""
        B, H, W = frames.shape
        cap = desc_out.shape[1]
        st = torch_stream(stream)
        rc = lib().orbhip_extract_batch_device(self.ctx.handle, ptr(frames), B, W, H, frames.stride(1),
                                               frames.stride(0), int(vLappingArea[0]), int(vLappingArea[1]),
                                               ptr(kps_out), ptr(desc_out), cap, ptr(n_out), ptr(mono_out), st)
        check(rc, "orbhip_extract_batch_device")

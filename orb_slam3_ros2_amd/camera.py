"""Distorted pinhole camera mirror (U:src/CameraModels/Pinhole + U:src/Frame.cc mDistCoef) over
liborbhip.so: Frame::UndistortKeyPoints and Frame::ComputeImageBounds on the GPU (include/orbhip.h
orbhip_undistort_keypoints*, orbhip_image_bounds). The node's camera file is
R:config/Monocular/MilkV.yaml (640 x 360, fx = fy = 342.67, cx 203.0, cy 132.67, k1 -0.35952,
k2 0.080321, p1 0.001794, p2 -0.001439)."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import KP_DTYPE, Context, PinholeC, check, lib, ptr, torch_stream

MILKV = dict(fx=342.67, fy=342.67, cx=203.0, cy=132.67, k1=-0.35952, k2=0.080321, p1=0.001794, p2=-0.001439,
             width=640, height=360)


class PinholeCamera:
    def __init__(self, fx, fy, cx, cy, k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0, width=640, height=480,
                 device: int = -1, ctx: Context | None = None):
        self.c = PinholeC(fx, fy, cx, cy, k1, k2, p1, p2, k3)
        self.width, self.height = int(width), int(height)
        self.ctx = ctx or Context(device)

    @classmethod
    def milkv(cls, ctx: Context | None = None):
        return cls(**MILKV, ctx=ctx)

    def params(self):
        """(fx, fy, cx, cy, k1, k2, p1, p2, k3) as the oracle takes them."""
        c = self.c
        return (c.fx, c.fy, c.cx, c.cy, c.k1, c.k2, c.p1, c.p2, c.k3)

    def UndistortKeyPoints(self, kps) -> np.ndarray:
        """mvKeys (orbhip_kp records) -> mvKeysUn."""
        k = np.ascontiguousarray(kps, KP_DTYPE)
        out = np.empty_like(k)
        check(lib().orbhip_undistort_keypoints(self.ctx.handle, ctypes.byref(self.c), ptr(k), k.shape[0], ptr(out)),
              "orbhip_undistort_keypoints")
        return out

    def undistort_device(self, kps, n, out=None, stream=None):
        """Extraction batch on the device: kps (B, cap, 6) float32 tensor, n (B,) int32 -> out."""
        out = kps if out is None else out
        B, cap = kps.shape[0], kps.shape[1]
        check(lib().orbhip_undistort_keypoints_device(self.ctx.handle, ctypes.byref(self.c), ptr(kps), ptr(n), B, cap,
                                                      ptr(out), torch_stream(stream)),
              "orbhip_undistort_keypoints_device")
        return out

    def ComputeImageBounds(self, cols=None, rows=None):
        """(mnMinX, mnMaxX, mnMinY, mnMaxY)."""
        b = np.zeros(4, np.float32)
        check(lib().orbhip_image_bounds(self.ctx.handle, ctypes.byref(self.c), int(cols or self.width),
                                        int(rows or self.height), ptr(b)), "orbhip_image_bounds")
        return tuple(float(v) for v in b)

"""Camera ingest on the device.

The reference path: ``cam_node.py`` publishes bgr8 frames (R:cam_node.py:55-84). The mono
node converts them with ``cv_bridge::toCvShare(msg, MONO8)`` = cvtColor(BGR2GRAY) and clones
them on the host (R:src/imu_mono_realsense.cpp:294-309). Then TrackMonocular runs ORB
extraction (:337).

Here the bgr8 frame goes to HBM once, as a torch-ROCm uint8 tensor. From there the gray
conversion (bit-exact OpenCV fixed point) and the extraction run on the device with no host
clone.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import torch_stream, check, lib, ptr
from .extractor import ORBextractor


def bgr_to_gray_device(ctx, bgr, gray=None, stream=None):
    """bgr: uint8 CUDA tensor [H, W, 3] or [B, H, W, 3] (rows may be padded). Returns (or
    fills) a uint8 CUDA tensor [H, W] / [B, H, W]. Asynchronous on ``stream``."""
    import torch
    batched = bgr.dim() == 4
    b4 = bgr if batched else bgr[None]
    B, H, W, C = b4.shape
    if C != 3 or b4.dtype != torch.uint8 or b4.stride(2) != 3 or b4.stride(3) != 1:
        raise ValueError("expected a uint8 [.., H, W, 3] tensor with packed pixels")
    if gray is None:
        gray = torch.empty((B, H, W), dtype=torch.uint8, device=b4.device)
    g3 = gray if gray.dim() == 3 else gray[None]
    st = torch_stream(stream)
    check(lib().orbhip_bgr_to_gray_device(ctx.handle, ptr(b4), B, W, H, b4.stride(1), b4.stride(0), ptr(g3),
                                          g3.stride(1), g3.stride(0), st), "orbhip_bgr_to_gray_device")
    return gray if batched or gray.dim() == 2 else gray[0]


class MonoIngest:
    """bgr8 frames -> device gray -> ORBextractor::operator() outputs on the device.

    One call = what the mono node does per image message up to the ORB features of
    Frame::ExtractORB (R:src/imu_mono_realsense.cpp:330-337). Outputs stay in HBM
    (kps [cap, 6] float32, desc [cap, 32] uint8, n, monoIndex), ready for the matcher."""

    def __init__(self, width, height, nfeatures=1000, scaleFactor=1.2, nlevels=8, iniThFAST=20, minThFAST=7,
                 device=-1):
        import torch
        self.torch = torch
        self.ext = ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST, device)
        self.w, self.h = int(width), int(height)
        dev = torch.device("cuda", device) if device >= 0 else torch.device("cuda", torch.cuda.current_device())
        self.cap = self.ext.max_keypoints(self.w, self.h)
        self.bgr = torch.empty((self.h, self.w, 3), dtype=torch.uint8, device=dev)
        self.gray = torch.empty((1, self.h, self.w), dtype=torch.uint8, device=dev)
        self.kps = torch.empty((1, self.cap, 6), dtype=torch.float32, device=dev)
        self.desc = torch.empty((1, self.cap, 32), dtype=torch.uint8, device=dev)
        self.n = torch.zeros(1, dtype=torch.int32, device=dev)
        self.mono = torch.zeros(1, dtype=torch.int32, device=dev)

    def __call__(self, frame_bgr8, vLappingArea=(0, 1000), stream=None):
        t = self.torch
        src = frame_bgr8 if isinstance(frame_bgr8, t.Tensor) else t.from_numpy(np.ascontiguousarray(frame_bgr8))
        if tuple(src.shape) != (self.h, self.w, 3):
            raise ValueError(f"frame shape {tuple(src.shape)} != {(self.h, self.w, 3)}")
        self.bgr.copy_(src, non_blocking=False)
        bgr_to_gray_device(self.ext.ctx, self.bgr, self.gray[0], stream)
        self.ext.extract_batch_device(self.gray, self.kps, self.desc, self.n, self.mono, vLappingArea, stream)
        return self.kps[0], self.desc[0], self.n, self.mono

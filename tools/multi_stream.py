#!/usr/bin/env python3
"""C2 as N independent camera streams (the CPU baseline's layout: one frame stream per thread):
N FrameStream(frames_in_flight=1) objects, frames pushed round-robin from one host thread, no
cross-stream events. Prints total frames/s and host submit time per frame."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402
from orb_slam3_ros2_amd.frontend import FrameStream  # noqa: E402

K = 2000
NF = 32
for N in [int(a) for a in (sys.argv[1:] or ["1", "4", "8", "12", "16"])]:
    cams = [FrameStream(640, 480, 1) for _ in range(N)]
    frames = [torch.from_numpy(bench.make_stream_frames(NF, 640, 480, 1000 * i + 1)).to("cuda") for i in range(N)]
    ptrs = [[f[i].data_ptr() for i in range(NF)] for f in frames]
    pushes = [c.push_ptr for c in cams]
    for k in range(64):
        for i in range(N):
            pushes[i](ptrs[i][k % NF], 640)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(K // N):
        for i in range(N):
            pushes[i](ptrs[i][k % NF], 640)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = (K // N) * N
    print(f"streams={N}: {n / dt:9.1f} frames/s, host submit {1e6 * (t1 - t0) / n:.1f} us/frame", flush=True)
    del cams

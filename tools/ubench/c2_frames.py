#!/usr/bin/env python3
"""Write the bench's 32-frame C2 stream (rank 0) as raw u8 for tools/ubench/c2_native."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402

f = bench.make_stream_frames(32, 640, 480, 1)
os.makedirs("gpurun_out", exist_ok=True)
f.tofile(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c2_frames.u8")

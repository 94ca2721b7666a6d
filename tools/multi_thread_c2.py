#!/usr/bin/env python3
"""Experiment: the C2 headline layout (C cameras, each a FrameStream taking one frame at a time)
pushed from T host threads, each owning C/T cameras (ctypes releases the GIL inside the C-ABI
push). Prints total frames/s per (C, T)."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 400
for C in (16, 32):
    for T in (1, 2, 4, 8):
        c2 = bench.FrontendC2(0, 1, C)
        for _ in range(20):
            c2.step()
        torch.cuda.synchronize()

        def run(t):
            cams = range(t, C, T)
            for k in range(K):
                for c in cams:
                    c2.pushes[c](c2.p_frames[c][k % c2.NF], c2.W)

        th = [threading.Thread(target=run, args=(t,)) for t in range(T)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"cameras={C} host_threads={T}: {C * K / dt:9.1f} frames/s", flush=True)
        del c2

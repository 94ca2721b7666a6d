#!/usr/bin/env python3
"""Experiment: T independent camera streams (bench.StreamC2, S frames in flight each), one host
thread per camera (ctypes releases the GIL inside the C-ABI calls). Prints total frames/s."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

K = 1000
for T in (1, 2, 3, 4):
    for S in (2, 4):
        cams = [bench.StreamC2(t, S) for t in range(T)]
        for c in cams:
            for _ in range(40):
                c.step()
        torch.cuda.synchronize()

        def run(c):
            for _ in range(K):
                c.step()

        th = [threading.Thread(target=run, args=(c,)) for c in cams]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"cameras={T} inflight={S}: {T * K / dt:9.1f} frames/s", flush=True)
        del cams

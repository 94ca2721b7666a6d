#!/usr/bin/env python3
"""Host-side cost of one C2 frame submission, piece by piece (GPU box): the ctypes extract and
match calls, the torch event record / wait, and a no-op C-ABI call with the same argument count."""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import torch  # noqa: E402

c2 = bench.StreamC2(0, 4)
for _ in range(50):
    c2.step()
torch.cuda.synchronize()


def per_call(fn, n=150):
    t = time.perf_counter()
    for _ in range(n):
        fn()
    dt = time.perf_counter() - t
    torch.cuda.synchronize()
    return 1e6 * dt / n


L, j, cur, prev = c2.L, 0, 1, 0
c, sp = c2.handles[j], c2.sts[j]
ex = lambda: c2.extract(c, c2.p_frames[0], 1, 640, 480, 640, 640 * 480, 0, 1000, c2.p_kps[cur], c2.p_desc[cur],
                        c2.cap, c2.p_n[cur], c2.p_mono[cur], sp)
mm = c2.p_mm[cur]
ma = lambda: c2.match(c, c2.p_kps[prev], c2.p_desc[prev], c2.p_n[prev], c2.p_kps[cur], c2.p_desc[cur], c2.p_n[cur],
                      c2.cap, 50, c2.ratio, 1, mm[0], mm[1], mm[2], c2.p_nm[cur], sp)
bad = lambda: c2.extract(None, 0, 1, 640, 480, 640, 640 * 480, 0, 1000, c2.p_kps[cur], c2.p_desc[cur],
                         c2.cap, c2.p_n[cur], c2.p_mono[cur], sp)   # returns at the argument check
ev = c2.ev_x[0]
rec = lambda: ev.record(c2.streams[1])
wt = lambda: c2.streams[2].wait_event(ev)
for _ in range(2):
  print(f"extract call {per_call(ex):.1f} us, match call {per_call(ma):.1f} us, "
        f"ctypes no-op (15 args) {per_call(bad):.1f} us, event record {per_call(rec):.1f} us, "
        f"wait_event {per_call(wt):.1f} us, full step {per_call(c2.step):.1f} us")

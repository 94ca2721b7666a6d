#!/usr/bin/env python3
"""Device timing trace of one C2 step (640x480 extract + match to the previous frame), or one
C3 batch with --c3. Prints, per kernel: workgroups, kernel span, workgroup duration spread,
start skew, and the phase cycles of workgroup 0 (orbhip_device.h TR_* macros)."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401

from orb_slam3_ros2_amd._lib import lib  # noqa: E402
import bench  # noqa: E402

STRIDE, NK = 16384, 8
NAMES = {0: "k_pyr_cone|k_resize(l=1)", 1: "k_fast_cells", 2: "k_octree", 3: "k_desc", 4: "k_match_top2", 5: "k_match_finish",
         6: "k_resize_bands", 7: "k_pyr_flow"}


def main():
    L = lib()
    L.orbhip_test_trace.argtypes = [ctypes.c_int, ctypes.c_void_p]
    c3 = "--c3" in sys.argv
    wl = bench.BatchC3(0) if c3 else bench.StreamC2(0)
    for _ in range(20):
        wl.step()
    torch.cuda.synchronize()
    assert L.orbhip_test_trace(1, None) == 0
    wl.step()
    torch.cuda.synchronize()
    buf = np.zeros(NK * STRIDE, np.uint64)
    assert L.orbhip_test_trace(0, buf.ctypes.data) == 0
    t_min = None
    rows = []
    for k in range(8):
        seg = buf[k * STRIDE: k * STRIDE + 8192].reshape(-1, 2).astype(np.int64)
        ok = seg[:, 1] > 0
        if not ok.any():
            continue
        st, en = seg[ok, 0], seg[ok, 1]
        t_min = st.min() if t_min is None else min(t_min, st.min())
        rows.append((k, st, en))
    for k, st, en in rows:
        dur = (en - st) * 10 / 1000.0   # s_memrealtime = 100 MHz -> us
        print(f"{NAMES[k]:14s} wgs={len(st):5d} span={(en.max() - st.min()) / 100:8.2f}us "
              f"start@{(st.min() - t_min) / 100:8.2f}us  wg dur min/med/max={dur.min():.2f}/{np.median(dur):.2f}/"
              f"{dur.max():.2f}us  start skew={(st.max() - st.min()) / 100:.2f}us")
        if len(st) <= 16:
            print("     per-wg start/dur (us): " + ", ".join(f"{(a - t_min) / 100:.1f}/{(b - a) / 100:.1f}"
                                                    for a, b in zip(st, en)))
        ph = buf[k * STRIDE + 8192: k * STRIDE + 8192 + 64].astype(np.int64)
        nz = np.nonzero(ph)[0]
        if len(nz):
            print("     wg0 phases (cycles): " + ", ".join(f"{i}:{ph[i]}" for i in nz))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Time SearchForInitialization (GPU, host-buffer API) against the oracle on one core, on the
5x initialisation extractor's keypoints (5000 features) of two frames of the synthetic stream."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import ORBextractor, ORBmatcher  # noqa: E402
from orb_slam3_ros2_amd._lib import KP_DTYPE  # noqa: E402
from orb_slam3_ros2_amd.synthetic import shifted_frame, synthetic_frame, synthetic_init_pair  # noqa: E402
from oracle import pyoracle as O  # noqa: E402


def bench(fn, reps=20):
    fn()
    t = time.perf_counter()
    for _ in range(reps):
        r = fn()
    return (time.perf_counter() - t) / reps * 1e3, r


ext = ORBextractor(5000, 1.2, 8, 20, 7)
a = synthetic_frame(3)
ks, ds = [], []
for f in (a, shifted_frame(a, 6, -3, 1)):
    _, kp, d = ext(f)
    k = np.zeros(len(kp), KP_DTYPE)
    for name in ("x", "y", "size", "angle", "response", "octave"):
        k[name] = kp[name]
    ks.append(k); ds.append(d)
prev = np.stack([ks[0]["x"], ks[0]["y"]], 1).astype(np.float32)
mt = ORBmatcher(0.9, True, ctx=ext.ctx)
g, r = bench(lambda: mt.SearchForInitialization(ks[0], ds[0], ks[1], ds[1], prev, 100))
o, _ = bench(lambda: O.search_for_initialization(ks[0], ds[0], ks[1], ds[1], prev, 100, 0.9, True))
nq = int((ks[0]["octave"] == 0).sum())
print(f"SearchForInitialization 5000-feature frames ({nq} octave-0 queries): GPU {g:.3f} ms ({r[0]} matches), "
      f"oracle 1 core {o:.3f} ms")
k1, d1, k2, d2, p = synthetic_init_pair(n1=4000, seed=1)
g, r = bench(lambda: mt.SearchForInitialization(k1, d1, k2, d2, p, 100))
o, _ = bench(lambda: O.search_for_initialization(k1, d1, k2, d2, p, 100, 0.9, True))
print(f"SearchForInitialization synthetic {int((k1['octave'] == 0).sum())} queries x {len(k2)}: GPU {g:.3f} ms "
      f"({r[0]} matches), oracle 1 core {o:.3f} ms")

"""Per-level k_octree work-group durations / start times in one C3 batch (device trace)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
import torch
from orb_slam3_ros2_amd._lib import lib
import bench
L = lib()
L.orbhip_test_trace.argtypes = [ctypes.c_int, ctypes.c_void_p]
wl = bench.BatchC3(0)
for _ in range(3): wl.step()
torch.cuda.synchronize()
L.orbhip_test_trace(1, None); wl.step(); torch.cuda.synchronize()
buf = np.zeros(8 * 16384, np.uint64); L.orbhip_test_trace(0, buf.ctypes.data)
seg = buf[2 * 16384: 2 * 16384 + 8192].reshape(-1, 2).astype(np.int64)[:512]
dur = (seg[:, 1] - seg[:, 0]) / 100.0
st = (seg[:, 0] - seg[:, 0].min()) / 100.0
for l in range(8):
    d = dur[64 * l: 64 * (l + 1)]; s = st[64 * l: 64 * (l + 1)]   # grid (frame, level)
    print(l, "dur min/med/max %.1f %.1f %.1f" % (d.min(), np.median(d), d.max()), "start med %.1f max %.1f" % (np.median(s), s.max()))
d0 = dur[:64]
print("level0 slowest frames", np.argsort(-d0)[:4].tolist(), np.sort(d0)[::-1][:4].tolist(), "fastest", int(np.argmin(d0)), float(d0.min()))
print("level0 by frame", np.round(d0[::4]).astype(int).tolist())
print("level1 by frame", np.round(dur[64:128][::4]).astype(int).tolist())

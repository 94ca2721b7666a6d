#!/usr/bin/env python3
"""Run the GPU extractor on seeded frames and dump every intermediate to an .npz so a
parity mismatch can be localised offline against the oracle (tools/compare_extract_debug.py).

Usage (GPU box): python tools/dump_extract_debug.py gpurun_out/extract_debug.npz
"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd import ORBextractor  # noqa: E402
from orb_slam3_ros2_amd._lib import lib  # noqa: E402
from orb_slam3_ros2_amd.synthetic import synthetic_frame  # noqa: E402

CASES = [(0, 640, 480, 1000), (10, 1280, 720, 1000), (12, 641, 479, 1000)]


def main(out):
    L = lib()
    L.orbhip_test_extract_debug.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 7
    L.orbhip_test_cells.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    res = {}
    for seed, w, h, nf in CASES:
        ext = ORBextractor(nf, 1.2, 8, 20, 7)
        img = synthetic_frame(seed, w, h)
        info = ext.level_info(w, h)
        sizes = np.zeros(4, np.int32)
        rc = L.orbhip_test_extract_debug(ext.ctx.handle, img.ctypes.data, w, h, 0, 1000, None, None, None, None,
                                         None, None, sizes.ctypes.data)
        assert rc == 0, rc
        npyr = int(np.sum(info["w"][1:].astype(np.int64) * info["h"][1:]))
        pyr = np.zeros(npyr, np.uint8)
        cand = np.zeros(sizes[0], np.uint32)
        ccnt = np.zeros(sizes[1], np.int32)
        lvl = np.zeros(sizes[2] * 2, np.uint32)
        lcnt = np.zeros(8, np.int32)
        lnlap = np.zeros(8, np.int32)
        rc = L.orbhip_test_extract_debug(ext.ctx.handle, img.ctypes.data, w, h, 0, 1000, pyr.ctypes.data,
                                         cand.ctypes.data, ccnt.ctypes.data, lvl.ctypes.data, lcnt.ctypes.data,
                                         lnlap.ctypes.data, sizes.ctypes.data)
        assert rc == 0, rc
        cells = np.zeros((sizes[1], 6), np.int32)
        L.orbhip_test_cells(ext.ctx.handle, w, h, cells.ctypes.data, sizes[1])
        mono, k, d = ext(img)
        tag = f"s{seed}_{w}x{h}"
        res.update({f"{tag}_pyr": pyr, f"{tag}_cand": cand, f"{tag}_ccnt": ccnt, f"{tag}_lvl": lvl,
                    f"{tag}_lcnt": lcnt, f"{tag}_lnlap": lnlap, f"{tag}_sizes": sizes, f"{tag}_cells": cells,
                    f"{tag}_kps": k, f"{tag}_desc": d if d is not None else np.zeros((0, 32), np.uint8),
                    f"{tag}_mono": np.array([mono])})
        print(tag, "n", len(k), "mono", mono, "lcnt", lcnt.tolist(), "err", sizes[3], flush=True)
    os.makedirs(os.path.dirname(out) or ".", exist_ok=True)
    np.savez_compressed(out, **res)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/extract_debug.npz")

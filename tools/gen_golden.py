#!/usr/bin/env python3
"""Regenerate tests/golden/*.npz from the oracle (CPU restatement, oracle/).

The reference ships no fixtures: these vectors are the restatement's
outputs on seeded synthetic inputs, committed so that (1) the oracle is regression-pinned
(tests/test_golden.py, CPU) and (2) the GPU path is checked against stored bytes without
running the oracle on the box (tests/test_golden.py, -m gpu).

    python tools/gen_golden.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as O  # noqa: E402
from orb_slam3_ros2_amd.synthetic import shifted_frame, synthetic_ba_problem, synthetic_frame  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")

# (name, seed, w, h, nfeatures, lap)
FRAMES = [("frame_640x480_s1", 1, 640, 480, 1000, (0, 1000)),
          ("frame_320x240_s5", 5, 320, 240, 500, (0, 1000)),
          ("frame_1280x720_s3_lap", 3, 1280, 720, 1000, (0, 1000))]


def gen_frames():
    for name, seed, w, h, nf, lap in FRAMES:
        img = synthetic_frame(seed, w, h)
        mono, kps, desc = O.extract(img, nfeatures=nf, lap=lap)
        extra = {"image": img} if w * h <= 320 * 240 else {}   # larger frames: seed + md5 only
        np.savez_compressed(os.path.join(OUT, name + ".npz"), seed=seed, w=w, h=h, nfeatures=nf,
                            lap=np.array(lap, np.int32), image_md5=hashlib.md5(img.tobytes()).hexdigest(),
                            mono=mono, kps=kps, desc=desc, **extra)
        print(name, "kps", len(kps), "mono", mono)


def gen_match():
    a = synthetic_frame(11, 640, 480)
    b = shifted_frame(a, 3, 1, 12)   # only the descriptors/angles are stored
    _, ka, da = O.extract(a)
    _, kb, db = O.extract(b)
    n, m, bd, sd = O.match_bf(db, kb[:, 3], da, ka[:, 3], 50, 0.9, True)
    np.savez_compressed(os.path.join(OUT, "match_640x480_s11.npz"), q_desc=db, q_angle=kb[:, 3].copy(),
                        t_desc=da, t_angle=ka[:, 3].copy(), th_low=50, ratio=np.float32(0.9), check_orientation=1,
                        n=n, match=m, best=bd, second=sd)
    print("match", n)


def gen_ba():
    prob, _ = synthetic_ba_problem(n_kf=10, n_pts=200, obs_per_pt=4, seed=21)
    r = O.ba_solve(prob)
    p = prob.normalized()
    np.savez_compressed(os.path.join(OUT, "ba_10kf_200pt_s21.npz"),
                        pose_q=p.pose_q, pose_t=p.pose_t, pose_fixed=p.pose_fixed, points=p.points,
                        edge_pose=p.edge_pose, edge_point=p.edge_point, edge_uv=p.edge_uv,
                        edge_octave=p.edge_octave, inv_sigma2=p.inv_sigma2,
                        cam=np.array([p.fx, p.fy, p.cx, p.cy], np.float32), huber_delta=np.float32(p.huber_delta),
                        iterations=p.iterations,
                        out_pose_q=r["pose_q"], out_pose_t=r["pose_t"], out_points=r["points"],
                        out_edge_chi2=r["edge_chi2"], out_edge_depth_ok=r["edge_depth_ok"],
                        out_chi2=np.array([r["initial_chi2"], r["final_chi2"]]),
                        out_iters=np.array([r["iterations_done"], r["lm_trials"]], np.int32))
    print("ba", r["initial_chi2"], "->", r["final_chi2"], "trials", r["lm_trials"])


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    gen_frames()
    gen_match()
    gen_ba()

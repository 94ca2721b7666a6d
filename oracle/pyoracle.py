"""ctypes view of oracle/build/liborb_oracle.so — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
The product (orb_slam3_ros2_amd / liborbhip.so) never does.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "liborb_oracle.so")
_lib = None

_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")


def build() -> None:
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_int, c_float, c_double = ctypes.c_int, ctypes.c_float, ctypes.c_double
        L.orc_level_info.argtypes = [c_int, c_int, c_int, c_float, c_int, _i32p, _i32p, _i32p, _f32p, _i32p]
        L.orc_extract.argtypes = [_u8p, c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_int, c_int, c_int,
                                  _f32p, _u8p, c_int, ctypes.POINTER(c_int)]
        L.orc_pyramid.argtypes = [_u8p, c_int, c_int, c_int, c_float, c_int, _u8p]
        L.orc_extract_levels.argtypes = [_u8p, c_int, c_int, c_int, c_int, c_float, c_int, c_int, c_int,
                                         _f32p, c_int, _f32p, c_int, _i32p]
        L.orc_blur.argtypes = [_u8p, c_int, c_int, _u8p]
        L.orc_gaussian_kernel.argtypes = [c_int, c_double, _i32p]
        L.orc_fast_atan2.argtypes = [c_float, c_float]
        L.orc_fast_atan2.restype = c_float
        L.orc_corner_score.argtypes = [_u8p, c_int]
        L.orc_fast_window.argtypes = [_u8p, c_int, c_int, c_int, c_int, _f32p, c_int]
        L.orc_descriptor_distance.argtypes = [_u8p, _u8p]
        L.orc_match_bf.argtypes = [_u8p, _f32p, c_int, _u8p, _f32p, c_int, c_int, c_float, c_int,
                                   _i32p, _i32p, _i32p]
        L.orc_ba_solve.argtypes = [c_int, c_int, c_int, _f32p, _f32p, _u8p, _f32p, _i32p, _i32p, _f32p, _i32p,
                                   _f32p, c_float, c_float, c_float, c_float, c_float, c_int, c_int, _f32p, _f32p,
                                   _f32p, _f32p, _u8p, _f64p]
        _f64 = _f64p
        L.orc_bow_transform.argtypes = [_u8p, _i32p, _i32p, _i32p, _i32p, _f64, c_int, _u8p, c_int, c_int, _i32p,
                                        _i32p, _f64]
        L.orc_bow_vector.argtypes = [_i32p, _f64, c_int, _i32p, _f64]
        L.orc_search_bow.argtypes = [_u8p, _f32p, _i32p, _u8p, c_int, _u8p, _f32p, _i32p, c_int, c_float, c_int,
                                     c_int, _i32p]
        L.orc_pose_optimization.argtypes = [c_int, _f32p, _f32p, _f32p, _f32p, _i32p, _f32p, c_float, c_float,
                                            c_float, c_float, c_float, _f32p, _f32p, _u8p, _f64]
        vp = ctypes.c_void_p
        L.orc_search_by_projection_last.argtypes = [c_int, vp, _u8p, vp, c_float, c_float, c_float, c_float, _f32p,
                                                    _f32p, _f32p, c_float, c_float, c_float, c_float, c_int, _f32p,
                                                    _u8p, _i32p, _f32p, c_float, c_int, _i32p]
        L.orc_search_local_points.argtypes = [c_int, vp, _u8p, vp, c_float, c_float, c_float, c_float, _f32p, c_int,
                                              c_float, _f32p, _f32p, c_float, c_float, c_float, c_float, c_int,
                                              _f32p, _f32p, _f32p, _f32p, _u8p, vp, c_float, c_float, c_float, c_int,
                                              c_float, _u8p, _i32p, _i32p]
        L.orc_search_for_initialization.argtypes = [c_int, vp, _u8p, c_int, vp, _u8p, c_float, c_float, c_float,
                                                    c_float, _f32p, c_int, c_float, c_int, _i32p]
        L.orc_undistort_keypoints.argtypes = [vp, c_int, _f32p, _f32p, vp]
        L.orc_image_bounds.argtypes = [c_int, c_int, _f32p, _f32p, _f32p]
        L.orc_kfdb_create.argtypes = [c_int, c_int]
        L.orc_kfdb_create.restype = vp
        L.orc_kfdb_destroy.argtypes = [vp]
        L.orc_kfdb_add.argtypes = [vp, c_int, _i32p, _f64p, c_int]
        L.orc_kfdb_erase.argtypes = [vp, c_int]
        L.orc_kfdb_detect_relocalization.argtypes = [vp, ctypes.c_longlong, _i32p, _f64p, c_int, _i32p, vp, c_int,
                                                     _i32p]
        L.orc_kfdb_detect_nbest.argtypes = [vp, ctypes.c_longlong, _i32p, _f64p, c_int, _i32p, vp, vp, c_int, vp,
                                            c_int, _i32p, _i32p, _i32p, _i32p]
        L.orc_bgr2gray.argtypes = [_u8p, c_int, c_int, c_int, _u8p, c_int]
        L.orc_glibc_sincosf_range.argtypes = [ctypes.c_uint32, ctypes.c_uint32, _f32p, _f32p]
        _lib = L
    return _lib


def level_info(w, h, nfeatures=1000, scale_factor=1.2, nlevels=8):
    lw = np.zeros(nlevels, np.int32); lh = np.zeros(nlevels, np.int32)
    feats = np.zeros(nlevels, np.int32); scales = np.zeros(nlevels, np.float32)
    umax = np.zeros(16, np.int32)
    lib().orc_level_info(w, h, nfeatures, scale_factor, nlevels, lw, lh, feats, scales, umax)
    return dict(w=lw, h=lh, feats=feats, scales=scales, umax=umax)


def extract(img: np.ndarray, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7,
            lap=(0, 1000), cap=None):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cap = cap or max(4 * nfeatures, 64)
    kps = np.zeros((cap, 6), np.float32)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int(0)
    mono = lib().orc_extract(img, w, h, w, nfeatures, scale_factor, nlevels, ini_th, min_th, lap[0], lap[1],
                             kps, desc, cap, ctypes.byref(n))
    return mono, kps[: n.value].copy(), desc[: n.value].copy()


def pyramid(img: np.ndarray, scale_factor=1.2, nlevels=8):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    info = level_info(w, h, 1000, scale_factor, nlevels)
    total = int(np.sum(info["w"].astype(np.int64) * info["h"]))
    out = np.zeros(total, np.uint8)
    rc = lib().orc_pyramid(img, w, h, w, scale_factor, nlevels, out)
    assert rc == 0
    levels, off = [], 0
    for l in range(nlevels):
        n = int(info["w"][l]) * int(info["h"][l])
        levels.append(out[off: off + n].reshape(int(info["h"][l]), int(info["w"][l])))
        off += n
    return levels


def extract_levels(img, nfeatures=1000, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7, cap=400000):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    h, w = img.shape
    cand = np.zeros((cap, 6), np.float32)
    kept = np.zeros((max(8 * nfeatures, 64), 6), np.float32)
    counts = np.zeros(2 * nlevels, np.int32)
    rc = lib().orc_extract_levels(img, w, h, w, nfeatures, scale_factor, nlevels, ini_th, min_th,
                                  cand, cap, kept, kept.shape[0], counts)
    assert rc == 0, rc
    c, k, oc, ok = [], [], 0, 0
    for l in range(nlevels):
        nc, nk = int(counts[2 * l]), int(counts[2 * l + 1])
        c.append(cand[oc: oc + nc].copy()); k.append(kept[ok: ok + nk].copy())
        oc += nc; ok += nk
    return c, k


def blur(img):
    img = np.ascontiguousarray(img, dtype=np.uint8)
    out = np.zeros_like(img)
    lib().orc_blur(img, img.shape[1], img.shape[0], out)
    return out


def gaussian_kernel(n=7, sigma=2.0):
    out = np.zeros(n, np.int32)
    lib().orc_gaussian_kernel(n, sigma, out)
    return out


def fast_atan2(y, x):
    return lib().orc_fast_atan2(float(y), float(x))


def match_bf(q, qa, t, ta, th_low=50, ratio=0.9, check_orientation=True):
    q = np.ascontiguousarray(q, np.uint8); t = np.ascontiguousarray(t, np.uint8)
    qa = np.ascontiguousarray(qa, np.float32); ta = np.ascontiguousarray(ta, np.float32)
    nq, nt = q.shape[0], t.shape[0]
    m = np.zeros(nq, np.int32); b = np.zeros(nq, np.int32); s = np.zeros(nq, np.int32)
    n = lib().orc_match_bf(q, qa, nq, t, ta, nt, th_low, ratio, int(check_orientation), m, b, s)
    return n, m, b, s


def bgr2gray(bgr: np.ndarray) -> np.ndarray:
    bgr = np.ascontiguousarray(bgr, np.uint8)
    h, w, _ = bgr.shape
    out = np.empty((h, w), np.uint8)
    lib().orc_bgr2gray(bgr, w, h, 3 * w, out, w)
    return out


def bow_transform(vocab, feats, levelsup=4):
    """Per-feature DBoW2 transform: (word ids, node ids at L - levelsup, weights)."""
    first, nch, children, word = vocab.csr()
    f = np.ascontiguousarray(feats, np.uint8).reshape(-1, 32)
    n = f.shape[0]
    ow = np.zeros(n, np.int32); on = np.zeros(n, np.int32); ov = np.zeros(n, np.float64)
    lib().orc_bow_transform(np.ascontiguousarray(vocab.desc), first, nch, children, word,
                            np.ascontiguousarray(vocab.weight, np.float64), vocab.L, f, n, levelsup, ow, on, ov)
    return ow, on, ov


def bow_vector(word, weight):
    word = np.ascontiguousarray(word, np.int32); weight = np.ascontiguousarray(weight, np.float64)
    ow = np.zeros(len(word), np.int32); ov = np.zeros(len(word), np.float64)
    k = lib().orc_bow_vector(word, weight, len(word), ow, ov)
    return ow[:k].copy(), ov[:k].copy()


def search_bow(kf_desc, kf_angle, kf_node, kf_valid, f_desc, f_angle, f_node, ratio=0.7, check_orientation=True,
               th_low=50):
    c = np.ascontiguousarray
    nkf, nf = len(kf_node), len(f_node)
    m = np.zeros(nf, np.int32)
    n = lib().orc_search_bow(c(kf_desc, np.uint8), c(kf_angle, np.float32), c(kf_node, np.int32),
                             c(kf_valid, np.uint8), nkf, c(f_desc, np.uint8), c(f_angle, np.float32),
                             c(f_node, np.int32), nf, ratio, int(check_orientation), th_low, m)
    return n, m


def glibc_sincosf_range(lo_bits: int, hi_bits: int):
    n = hi_bits - lo_bits + 1
    c = np.empty(n, np.float32); s = np.empty(n, np.float32)
    lib().orc_glibc_sincosf_range(lo_bits, hi_bits, c, s)
    return c, s


def ba_solve(prob):
    """Oracle LM/Schur solve of an orb_slam3_ros2_amd.optimizer.BAProblem. Returns a dict."""
    p = prob.normalized()
    P, M, E = p.pose_q.shape[0], p.points.shape[0], p.edge_pose.shape[0]
    oq = np.zeros((P, 4), np.float32); ot = np.zeros((P, 3), np.float32); op = np.zeros((M, 3), np.float32)
    oc = np.zeros(E, np.float32); od = np.zeros(E, np.uint8); st = np.zeros(4, np.float64)
    lib().orc_ba_solve(P, M, E, p.pose_q, p.pose_t, p.pose_fixed, p.points, p.edge_pose, p.edge_point, p.edge_uv,
                       p.edge_octave, p.inv_sigma2, p.fx, p.fy, p.cx, p.cy, p.huber_delta, p.iterations,
                       p.early_stop, oq, ot, op, oc, od, st)
    return dict(pose_q=oq, pose_t=ot, points=op, edge_chi2=oc, edge_depth_ok=od, initial_chi2=st[0],
                final_chi2=st[1], iterations_done=int(st[2]), lm_trials=int(st[3]))


def pose_optimization(prob):
    """Oracle Optimizer::PoseOptimization of an orb_slam3_ros2_amd.optimizer.PoseProblem."""
    p = prob.normalized()
    n = p.points.shape[0]
    oq = np.zeros(4, np.float32); ot = np.zeros(3, np.float32); ol = np.zeros(n, np.uint8)
    st = np.zeros(1, np.float64)
    nin = lib().orc_pose_optimization(n, p.pose_q, p.pose_t, p.points, p.uv, p.octave, p.inv_sigma2, p.fx, p.fy,
                                      p.cx, p.cy, float(np.float32(np.sqrt(5.991))), oq, ot, ol, st)
    return dict(pose_q=oq, pose_t=ot, outlier=ol, n_inliers=int(nin), lm_trials=int(st[0]))


def _vp(a):
    return None if a is None else a.ctypes.data


def search_by_projection_last(frame, points, mp_desc, last_octave, last_angle, th=15.0, check_orientation=True):
    """Oracle SearchByProjection(CurrentFrame, LastFrame, th, bMono) on a matcher.ProjFrame."""
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
    match = np.full(pts.shape[0], -1, np.int32)
    n = lib().orc_search_by_projection_last(
        frame.kps.shape[0], _vp(frame.kps), frame.desc, _vp(frame.claimed), *frame.bounds, frame.scale_factors,
        frame.pose_q, frame.pose_t, frame.fx, frame.fy, frame.cx, frame.cy, pts.shape[0], pts,
        np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32), np.ascontiguousarray(last_octave, np.int32),
        np.ascontiguousarray(last_angle, np.float32), th, int(check_orientation), match)
    return n, match


def search_local_points(frame, points, normals, min_dist, max_dist, mp_desc, skip=None, th=1.0, nnratio=0.8,
                        view_cos_limit=0.5, far_points=False, th_far=0.0):
    """Oracle isInFrustum + SearchByProjection(F, vpMapPoints, th, bFarPoints, thFarPoints)."""
    pts = np.ascontiguousarray(points, np.float32).reshape(-1, 3)
    m = pts.shape[0]
    match = np.full(m, -1, np.int32); in_view = np.zeros(m, np.uint8); level = np.full(m, -1, np.int32)
    sk = None if skip is None else np.ascontiguousarray(skip, np.uint8)
    n = lib().orc_search_local_points(
        frame.kps.shape[0], _vp(frame.kps), frame.desc, _vp(frame.claimed), *frame.bounds, frame.scale_factors,
        len(frame.scale_factors), frame.log_scale_factor, frame.pose_q, frame.pose_t, frame.fx, frame.fy, frame.cx,
        frame.cy, m, pts, np.ascontiguousarray(normals, np.float32).reshape(-1, 3),
        np.ascontiguousarray(min_dist, np.float32), np.ascontiguousarray(max_dist, np.float32),
        np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32), _vp(sk), view_cos_limit, th, nnratio,
        int(far_points), th_far, in_view, level, match)
    return n, match, in_view, level


def search_for_initialization(kps1, desc1, kps2, desc2, prev_matched, window=100, nnratio=0.9,
                              check_orientation=True, bounds=(0.0, 640.0, 0.0, 480.0)):
    """Oracle SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize).
    kps: orbhip_kp records (matcher.KP_DTYPE). Returns (nmatches, matches12, prev_matched')."""
    from orb_slam3_ros2_amd._lib import KP_DTYPE
    k1 = np.ascontiguousarray(kps1, KP_DTYPE); k2 = np.ascontiguousarray(kps2, KP_DTYPE)
    prev = np.ascontiguousarray(prev_matched, np.float32).reshape(-1, 2).copy()
    m = np.full(k1.shape[0], -1, np.int32)
    n = lib().orc_search_for_initialization(
        k1.shape[0], _vp(k1), np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32), k2.shape[0], _vp(k2),
        np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32), *[float(b) for b in bounds], prev, int(window),
        float(nnratio), int(check_orientation), m)
    return n, m, prev


def _cam(camera):
    """(fx, fy, cx, cy, k1, k2, p1, p2[, k3]) -> float32 cam[4], dist[5]."""
    c = [float(v) for v in camera] + [0.0] * (9 - len(camera))
    return np.array(c[:4], np.float32), np.array(c[4:9], np.float32)


def undistort_keypoints(kps, camera):
    """Frame::UndistortKeyPoints (cv::undistortPoints, 5 iterations): orbhip_kp records -> mvKeysUn."""
    k = np.ascontiguousarray(kps).copy()
    cam, dist = _cam(camera)
    out = k.copy()
    lib().orc_undistort_keypoints(_vp(k), k.shape[0], cam, dist, _vp(out))
    return out


def image_bounds(cols, rows, camera):
    """Frame::ComputeImageBounds -> (mnMinX, mnMaxX, mnMinY, mnMaxY)."""
    cam, dist = _cam(camera)
    b = np.zeros(4, np.float32)
    lib().orc_image_bounds(int(cols), int(rows), cam, dist, b)
    return tuple(float(v) for v in b)


class KeyFrameDatabase:
    """Oracle KeyFrameDatabase (persistent KeyFrame members, inverted file in insertion order)."""

    def __init__(self, max_kf, n_words):
        self.max_kf = max_kf
        self._h = lib().orc_kfdb_create(int(max_kf), int(n_words))

    def add(self, kf, bow):
        w = np.ascontiguousarray(bow[0], np.int32); v = np.ascontiguousarray(bow[1], np.float64)
        lib().orc_kfdb_add(self._h, int(kf), w, v, w.shape[0])

    def erase(self, kf):
        lib().orc_kfdb_erase(self._h, int(kf))

    def DetectRelocalizationCandidates(self, query_id, bow, covis, kf_map=None, query_map=0):
        w = np.ascontiguousarray(bow[0], np.int32); v = np.ascontiguousarray(bow[1], np.float64)
        cv = np.ascontiguousarray(covis, np.int32).reshape(-1)
        km = None if kf_map is None else np.ascontiguousarray(kf_map, np.int32)
        out = np.zeros(self.max_kf, np.int32)
        n = lib().orc_kfdb_detect_relocalization(self._h, int(query_id), w, v, w.shape[0], cv, _vp(km),
                                                 int(query_map), out)
        return out[:n].copy()

    def DetectNBestCandidates(self, query_id, bow, covis, connected=None, n=3, kf_map=None, query_map=0,
                              flags=None):
        w = np.ascontiguousarray(bow[0], np.int32); v = np.ascontiguousarray(bow[1], np.float64)
        cv = np.ascontiguousarray(covis, np.int32).reshape(-1)
        con = None if connected is None else np.ascontiguousarray(connected, np.uint8)
        km = None if kf_map is None else np.ascontiguousarray(kf_map, np.int32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint8)
        lo = np.zeros(max(n, 1), np.int32); me = np.zeros(max(n, 1), np.int32)
        nl = np.zeros(1, np.int32); nm = np.zeros(1, np.int32)
        lib().orc_kfdb_detect_nbest(self._h, int(query_id), w, v, w.shape[0], cv, _vp(con), _vp(km), int(query_map),
                                    _vp(fl), int(n), lo, nl, me, nm)
        return lo[: nl[0]].copy(), me[: nm[0]].copy()

    def __del__(self):
        try:
            lib().orc_kfdb_destroy(self._h)
        except Exception:
            pass

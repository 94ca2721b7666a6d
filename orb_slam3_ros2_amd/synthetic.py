"""Seeded synthetic inputs — no datasets exist offline.

Images: background 128, 300 axis-aligned rectangles (side U[8,96] px, intensity
U[0,255]) drawn in order, then Gaussian noise sigma=4, rounded and clipped to u8.
numpy PCG64 seeded with the frame index. This gives FAST corners in every 35-px
cell, like a textured indoor scene.
"""
from __future__ import annotations

import numpy as np


def synthetic_frame(seed: int, width: int = 640, height: int = 480, n_rect: int = 300,
                    noise_sigma: float = 4.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.full((height, width), 128.0, dtype=np.float64)
    for _ in range(n_rect):
        sw, sh = rng.integers(8, 97, size=2)
        x0 = int(rng.integers(-int(sw) + 1, width))
        y0 = int(rng.integers(-int(sh) + 1, height))
        val = float(rng.integers(0, 256))
        img[max(y0, 0):max(min(y0 + sh, height), 0), max(x0, 0):max(min(x0 + sw, width), 0)] = val
    if noise_sigma > 0:
        img += rng.normal(0.0, noise_sigma, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synthetic_batch(first_seed: int, batch: int, width: int, height: int) -> np.ndarray:
    return np.stack([synthetic_frame(first_seed + i, width, height) for i in range(batch)])


def shifted_frame(base: np.ndarray, dx: int, dy: int, seed: int, noise_sigma: float = 2.0) -> np.ndarray:
    """A second view of ``base``: integer translation (edge-replicated) plus fresh noise,
    so consecutive frames share most corners (matcher workloads)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    h, w = base.shape
    ys = np.clip(np.arange(h) - dy, 0, h - 1)
    xs = np.clip(np.arange(w) - dx, 0, w - 1)
    img = base[ys][:, xs].astype(np.float64)
    img += rng.normal(0.0, noise_sigma, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synthetic_stream(n: int, width: int, height: int, seed0: int, noise_sigma: float = 4.0,
                     margin=(256, 128)) -> np.ndarray:
    """A camera panning over one static scene (SURVEY.md 8d image spec at every frame): the scene
    is a (width + mx) x (height + my) image with the 640x480 rectangle density (300 per 640x480),
    frame i the crop at a smooth offset (2-4 px right, 0-1 px down per frame, bouncing inside the
    margin) plus fresh N(0, noise_sigma) noise. Consecutive frames share most corners, and every
    frame has the same statistics (noise does not accumulate along the stream)."""
    mx, my = margin
    W, H = width + mx, height + my
    n_rect = int(round(300 * (W * H) / (640 * 480)))
    world = synthetic_frame(seed0, W, H, n_rect=n_rect, noise_sigma=0.0).astype(np.float64)
    rng = np.random.Generator(np.random.PCG64(seed0 + 1))
    out = np.empty((n, height, width), np.uint8)
    ox = oy = 0
    for i in range(n):
        img = world[oy:oy + height, ox:ox + width] + rng.normal(0.0, noise_sigma, size=(height, width))
        out[i] = np.clip(np.rint(img), 0, 255).astype(np.uint8)
        ox += 2 + (i % 3)
        oy += i % 2
        if ox > mx:
            ox = ox % (mx + 1)
        if oy > my:
            oy = oy % (my + 1)
    return out


# ---------------------------------------------------------------------------
# Bundle-adjustment problems
# ---------------------------------------------------------------------------
D435I = dict(fx=614.67, fy=617.63, cx=326.22, cy=245.58, w=640, h=480)   # R:config/Monocular/RealSense_D435i.yaml:16-29


def _rodrigues(w):
    th = np.linalg.norm(w)
    if th < 1e-12:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * (K @ K)


def _mat_to_quat(R):
    """(x, y, z, w), w >= 0."""
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        w, x, y, z = 0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s
    else:
        i = int(np.argmax(np.diag(R)))
        j, k = (i + 1) % 3, (i + 2) % 3
        s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0) * 2
        q = np.zeros(3)
        q[i] = 0.25 * s
        w = (R[k, j] - R[j, k]) / s
        q[j] = (R[j, i] + R[i, j]) / s
        q[k] = (R[k, i] + R[i, k]) / s
        x, y, z = q
    q = np.array([x, y, z, w])
    if q[3] < 0:
        q = -q
    return q / np.linalg.norm(q)


def _look_at(c, target=np.zeros(3)):
    """Rcw for a camera at c looking at target (camera z forward, y down)."""
    z = target - c
    z /= np.linalg.norm(z)
    up = np.array([0.0, -1.0, 0.0])
    x = np.cross(up, z)
    x /= np.linalg.norm(x)
    y = np.cross(z, x)
    return np.stack([x, y, z])   # rows: camera axes in world


def synthetic_ba_problem(n_kf=50, n_pts=2000, obs_per_pt=4, seed=7, layout="arc", window=None,
                         rot_noise=0.01, trans_noise=0.02, pt_noise=0.05, n_levels=8, scale_factor=1.2):
    """C4 (layout='arc'): KFs on a 2 m-radius arc looking inward, points uniform in a 1 m cube at
    the centre, each point seen by `obs_per_pt` distinct KFs. C5 (layout='loop'): KFs around a full
    circle, each point observed from a `window`-KF sliding window (co-visibility band).
    Returns (BAProblem with perturbed initial state, ground-truth dict)."""
    from .optimizer import BAProblem, TH_HUBER_MONO
    rng = np.random.Generator(np.random.PCG64(seed))
    cam = D435I
    if layout == "arc":
        ang = np.linspace(-np.pi / 3, np.pi / 3, n_kf)
        radius = 2.0
    else:
        ang = np.linspace(0, 2 * np.pi, n_kf, endpoint=False)
        radius = 4.0
    Rs, ts = [], []
    for a in ang:
        c = np.array([radius * np.sin(a), 0.3 * np.sin(3 * a), -radius * np.cos(a)])
        R = _look_at(c)
        Rs.append(R)
        ts.append(-R @ c)
    Rs, ts = np.array(Rs), np.array(ts)
    pts = rng.uniform(-0.5, 0.5, size=(n_pts, 3))
    edges_pose, edges_pt = [], []
    for m in range(n_pts):
        if window is None:
            kfs = rng.choice(n_kf, obs_per_pt, replace=False)
        else:
            start = int(rng.integers(0, n_kf))
            kfs = (start + rng.choice(window, obs_per_pt, replace=False)) % n_kf
            # place the point where that window looks (in front of its middle keyframe)
            mid = (start + window // 2) % n_kf
            cmid = -Rs[mid].T @ ts[mid]
            pts[m] = cmid * 0.55 + rng.uniform(-0.4, 0.4, size=3)
        for k in sorted(kfs.tolist()):
            edges_pose.append(k)
            edges_pt.append(m)
    edges_pose = np.array(edges_pose, np.int32)
    edges_pt = np.array(edges_pt, np.int32)
    E = len(edges_pose)
    octave = rng.integers(0, n_levels, size=E).astype(np.int32)
    scales = np.ones(n_levels, np.float32)
    for i in range(1, n_levels):
        scales[i] = np.float32(np.float64(scales[i - 1]) * np.float64(np.float32(scale_factor)))
    inv_sigma2 = (np.float32(1.0) / (scales * scales)).astype(np.float32)
    Xc = np.einsum("eij,ej->ei", Rs[edges_pose], pts[edges_pt]) + ts[edges_pose]
    uv = np.stack([cam["fx"] * Xc[:, 0] / Xc[:, 2] + cam["cx"], cam["fy"] * Xc[:, 1] / Xc[:, 2] + cam["cy"]], 1)
    sig = np.power(np.float64(scale_factor), octave)
    uv += rng.normal(size=uv.shape) * sig[:, None]
    # perturbed initial state (KF0 stays at ground truth and is fixed)
    q0, t0 = [], []
    for k in range(n_kf):
        if k == 0:
            R, t = Rs[k], ts[k]
        else:
            R = _rodrigues(rng.normal(size=3) * rot_noise) @ Rs[k]
            t = ts[k] + rng.normal(size=3) * trans_noise
        q0.append(_mat_to_quat(R))
        t0.append(t)
    fixed = np.zeros(n_kf, np.uint8)
    fixed[0] = 1
    p0 = pts + rng.normal(size=pts.shape) * pt_noise
    prob = BAProblem(np.array(q0, np.float32), np.array(t0, np.float32), fixed, p0.astype(np.float32), edges_pose,
                     edges_pt, uv.astype(np.float32), octave, inv_sigma2, np.float32(cam["fx"]),
                     np.float32(cam["fy"]), np.float32(cam["cx"]), np.float32(cam["cy"]), TH_HUBER_MONO, 10, 0)
    gt = dict(R=Rs, t=ts, points=pts)
    return prob, gt


def synthetic_pose_problem(n=600, outlier_frac=0.15, seed=3, rot_noise=0.02, trans_noise=0.05, n_levels=8,
                           scale_factor=1.2):
    """A tracked monocular Frame for PoseOptimization: a camera looking at map points 2-6 m away,
    keypoints = projections + 1.2^octave px noise, a fraction replaced by gross mismatches
    (uniform in the image), initial pose perturbed like a constant-velocity prediction.
    Returns (PoseProblem, ground truth dict)."""
    from .optimizer import PoseProblem
    rng = np.random.Generator(np.random.PCG64(seed))
    cam = D435I
    R = _rodrigues(rng.normal(size=3) * 0.3)
    t = rng.normal(size=3) * 0.5
    # points in front of the camera, inside the image
    z = rng.uniform(2.0, 6.0, size=n)
    u = rng.uniform(20, 620, size=n)
    v = rng.uniform(20, 460, size=n)
    Xc = np.stack([(u - cam["cx"]) / cam["fx"] * z, (v - cam["cy"]) / cam["fy"] * z, z], 1)
    Xw = (Xc - t) @ R          # R^T (Xc - t)
    octave = rng.integers(0, n_levels, size=n).astype(np.int32)
    scales = np.ones(n_levels, np.float32)
    for i in range(1, n_levels):
        scales[i] = np.float32(np.float64(scales[i - 1]) * np.float64(np.float32(scale_factor)))
    inv_sigma2 = (np.float32(1.0) / (scales * scales)).astype(np.float32)
    uv = np.stack([u, v], 1) + rng.normal(size=(n, 2)) * np.power(np.float64(scale_factor), octave)[:, None]
    bad = rng.random(n) < outlier_frac
    uv[bad] = np.stack([rng.uniform(0, 640, bad.sum()), rng.uniform(0, 480, bad.sum())], 1)
    R0 = _rodrigues(rng.normal(size=3) * rot_noise) @ R
    t0 = t + rng.normal(size=3) * trans_noise
    prob = PoseProblem(_mat_to_quat(R0).astype(np.float32), t0.astype(np.float32), Xw.astype(np.float32),
                       uv.astype(np.float32), octave, inv_sigma2, cam["fx"], cam["fy"], cam["cx"], cam["cy"])
    return prob, dict(R=R, t=t, bad=bad)


def synthetic_projection_scene(n_kp=1000, n_mp=900, seed=5, dup_frac=0.15, distractor_frac=0.15,
                               claimed_frac=0.05, width=640, height=480, n_levels=8):
    """A tracked Frame plus MapPoints for the projection matchers.
    Keypoints uniform over the image (some on the far right / bottom edge, outside PosInGrid),
    random descriptors; MapPoints back-projected from keypoints at 1-8 m (pixel jitter ~ the
    keypoint scale, 0-40 flipped descriptor bits, rotation +12 deg), near-duplicates of the same
    keypoint (greedy conflicts) and random distractors. Returns a dict of arrays."""
    from ._lib import KP_DTYPE
    rng = np.random.Generator(np.random.PCG64(seed))
    cam = D435I
    kps = np.zeros(n_kp, KP_DTYPE)
    kps["x"] = rng.uniform(0, width, n_kp).astype(np.float32)
    kps["y"] = rng.uniform(0, height, n_kp).astype(np.float32)
    edge = rng.random(n_kp) < 0.03
    kps["x"][edge] = rng.uniform(width - 6, width, edge.sum()).astype(np.float32)
    kps["octave"] = rng.integers(0, n_levels, n_kp)
    kps["angle"] = rng.uniform(0, 360, n_kp).astype(np.float32)
    kps["size"] = 31.0
    kps["response"] = rng.uniform(20, 80, n_kp).astype(np.float32)
    desc = rng.integers(0, 256, (n_kp, 32), dtype=np.uint8)
    R = _rodrigues(rng.normal(size=3) * 0.4)
    t = rng.normal(size=3)
    q = _mat_to_quat(R).astype(np.float32)
    Rf = R.astype(np.float32)
    Ow = (-Rf.T @ t.astype(np.float32)).astype(np.float64)
    src = rng.choice(n_kp, n_mp, replace=False) if (dup_frac == 0 and n_mp <= n_kp) else \
        rng.integers(0, max(n_kp, 1), n_mp)
    ndup = int(dup_frac * n_mp)
    src[:ndup] = rng.integers(0, max(1, n_kp // 20), ndup)          # many points on few keypoints
    rng.shuffle(src)
    sc = np.power(1.2, kps["octave"][src])
    z = rng.uniform(1.0, 8.0, n_mp)
    u = kps["x"][src] + rng.normal(size=n_mp) * sc
    v = kps["y"][src] + rng.normal(size=n_mp) * sc
    Xc = np.stack([(u - cam["cx"]) / cam["fx"] * z, (v - cam["cy"]) / cam["fy"] * z, z], 1)
    pts = (Xc - t) @ R
    mdesc = desc[src].copy()
    for m in range(n_mp):
        nb = int(rng.integers(0, 41))
        bits = rng.choice(256, nb, replace=False)
        for b in bits:
            mdesc[m, b >> 3] ^= np.uint8(1 << (b & 7))
    dis = rng.random(n_mp) < distractor_frac
    mdesc[dis] = rng.integers(0, 256, (dis.sum(), 32), dtype=np.uint8)
    octave = np.clip(kps["octave"][src] + rng.integers(-1, 2, n_mp), 0, n_levels - 1).astype(np.int32)
    angle = ((kps["angle"][src] + 12.0 + rng.normal(size=n_mp) * 3.0) % 360.0).astype(np.float32)
    # MapPoint geometry for isInFrustum
    PO = pts - Ow
    dist = np.linalg.norm(PO, axis=1)
    normals = PO / dist[:, None] + rng.normal(size=(n_mp, 3)) * 0.05
    normals /= np.linalg.norm(normals, axis=1)[:, None]
    back = rng.random(n_mp) < 0.05
    normals[back] *= -1
    max_dist = dist * rng.uniform(0.75, 1.4, n_mp)
    min_dist = max_dist / np.float64(1.2) ** (n_levels - 1)
    claimed = (rng.random(n_kp) < claimed_frac).astype(np.uint8)
    skip = (rng.random(n_mp) < 0.05).astype(np.uint8)
    return dict(kps=kps, desc=desc, pose_q=q, pose_t=t.astype(np.float32), fx=cam["fx"], fy=cam["fy"], cx=cam["cx"],
                cy=cam["cy"], points=pts.astype(np.float32), mp_desc=mdesc, last_octave=octave, last_angle=angle,
                normals=normals.astype(np.float32), min_dist=min_dist.astype(np.float32),
                max_dist=max_dist.astype(np.float32), claimed=claimed, skip=skip, src=src)


def _flip_bits(rng, d, nb):
    d = d.copy()
    for b in rng.choice(256, nb, replace=False):
        d[b >> 3] ^= np.uint8(1 << (b & 7))
    return d


def synthetic_init_pair(n1=1500, seed=9, width=640, height=480, n_levels=8, level0_frac=0.6, steal_frac=0.15,
                        distractor_frac=0.3, rot_deg=10.0, shift=(14.0, -6.0)):
    """Two frames for monocular initialisation (U:src/ORBmatcher.cc::SearchForInitialization):
    F1 keypoints (level0_frac on octave 0), F2 = F1 moved by `shift` px + jitter with 0-30
    flipped descriptor bits and a rotation of ~rot_deg (some random, for the histogram filter),
    some on octave 1 (level filter), plus distractors; `steal_frac` of the F1 level-0 keypoints get
    a later F1 twin near them whose descriptor is closer to the same F2 keypoint (the greedy
    steal path). F2 is shuffled. Returns (kps1, desc1, kps2, desc2, prev_matched)."""
    from ._lib import KP_DTYPE
    rng = np.random.Generator(np.random.PCG64(seed))
    k1 = np.zeros(n1, KP_DTYPE)
    k1["x"] = rng.uniform(0, width, n1).astype(np.float32)
    k1["y"] = rng.uniform(0, height, n1).astype(np.float32)
    k1["octave"] = np.where(rng.random(n1) < level0_frac, 0, rng.integers(1, n_levels, n1))
    k1["angle"] = rng.uniform(0, 360, n1).astype(np.float32)
    k1["size"] = 31.0
    k1["response"] = rng.uniform(20, 80, n1).astype(np.float32)
    d1 = rng.integers(0, 256, (n1, 32), dtype=np.uint8)
    k2, d2 = [], []
    for i in range(n1):
        if k1["octave"][i] != 0 or rng.random() < 0.2:
            continue
        r = np.zeros(1, KP_DTYPE)[0]
        r["x"] = np.float32(k1["x"][i] + shift[0] + rng.normal() * 3)
        r["y"] = np.float32(k1["y"][i] + shift[1] + rng.normal() * 3)
        r["octave"] = 0 if rng.random() > 0.05 else 1
        rot = rot_deg + rng.normal() * 2 if rng.random() > 0.1 else rng.uniform(0, 360)
        r["angle"] = np.float32((k1["angle"][i] - rot) % 360.0)
        r["size"] = 31.0
        r["response"] = np.float32(50)
        k2.append(r)
        d2.append(_flip_bits(rng, d1[i], int(rng.integers(0, 31))))
    # steals: a later F1 keypoint near i whose descriptor is closer to i's F2 partner
    n2m = len(k2)
    for j in rng.choice(n2m, int(steal_frac * n2m), replace=False):
        t = rng.integers(0, n1)
        k1["octave"][t] = 0
        k1["x"][t] = np.float32(k2[j]["x"] - shift[0] + rng.normal() * 5)
        k1["y"][t] = np.float32(k2[j]["y"] - shift[1] + rng.normal() * 5)
        k1["angle"][t] = np.float32((k2[j]["angle"] + rot_deg) % 360.0)
        d1[t] = _flip_bits(rng, d2[j], int(rng.integers(0, 12)))
    nd = int(distractor_frac * n2m)
    for _ in range(nd):
        r = np.zeros(1, KP_DTYPE)[0]
        r["x"] = np.float32(rng.uniform(0, width)); r["y"] = np.float32(rng.uniform(0, height))
        r["octave"] = 0; r["angle"] = np.float32(rng.uniform(0, 360)); r["size"] = 31.0; r["response"] = 40.0
        k2.append(r)
        # near-copies of a random F1 descriptor: second-best competition for the ratio test
        d2.append(_flip_bits(rng, d1[rng.integers(0, n1)], int(rng.integers(5, 40))))
    k2 = np.array(k2, KP_DTYPE)
    d2 = np.stack(d2).astype(np.uint8)
    perm = rng.permutation(k2.shape[0])
    k2, d2 = k2[perm], d2[perm]
    prev = np.stack([k1["x"], k1["y"]], 1).astype(np.float32)
    return k1, d1, k2, d2, prev


def synthetic_kfdb_scene(n_kf=200, n_words=20000, words_per_place=400, seed=13, n_maps=2, common_pool=0,
                         common_frac=0.3):
    """A keyframe trajectory for KeyFrameDatabase queries. KF i sees the
    words of places i-2..i+2 (a sliding window, so neighbours share many words) plus random
    words; values positive, L1-normalised (DBoW2 BowVector). covis[i] = the 10 nearest KFs by
    index (GetBestCovisibilityKeyFrames order: most shared first), maps split the trajectory.
    A few KFs revisit an early place (loop closures). common_pool > 0 adds a pool of words every KF
    sees a fraction of (repetitive texture: many KFs pass the 0.8 x max common-words cut and the
    scores crowd). Returns dict(bows, covis, kf_map, place)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    n_places = n_kf + 4
    place_words = [rng.choice(n_words, words_per_place, replace=False) for _ in range(n_places)]
    place = np.arange(n_kf)
    loops = rng.choice(np.arange(n_kf // 2, n_kf), max(1, n_kf // 20), replace=False)
    place[loops] = rng.integers(0, n_kf // 4, loops.shape[0])
    pool = rng.choice(n_words, common_pool, replace=False) if common_pool else None
    bows = []
    for i in range(n_kf):
        ws = [] if pool is None else [pool[rng.random(common_pool) < common_frac]]
        for d in range(-2, 3):
            p = min(max(place[i] + d, 0), n_places - 1)
            pw = place_words[p]
            ws.append(pw[rng.random(pw.shape[0]) < 0.35])
        ws.append(rng.choice(n_words, 60, replace=False))
        w = np.unique(np.concatenate(ws)).astype(np.int32)
        v = rng.gamma(2.0, 1.0, w.shape[0])
        bows.append((w, v / v.sum()))
    covis = np.full((n_kf, 10), -1, np.int32)
    for i in range(n_kf):
        nb = sorted((j for j in range(max(0, i - 8), min(n_kf, i + 9)) if j != i), key=lambda j: (abs(i - j), j))
        covis[i, : min(10, len(nb))] = nb[:10]
    kf_map = (np.arange(n_kf) * n_maps // n_kf).astype(np.int32)
    return dict(bows=bows, covis=covis, kf_map=kf_map, place=place)


def synthetic_query_bow(scene, kf, seed, n_words=20000, keep=0.6, noise=80):
    """A frame near keyframe `kf` (or seeing several places: a list of KFs): a subset of their
    words plus noise words, L1-normalised."""
    rng = np.random.Generator(np.random.PCG64(seed))
    kfs = [kf] if np.isscalar(kf) else list(kf)
    parts = []
    for k in kfs:
        w0, _ = scene["bows"][int(k)]
        parts.append(w0[rng.random(w0.shape[0]) < keep])
    w = np.unique(np.concatenate(parts + [rng.choice(n_words, noise, replace=False)])).astype(np.int32)
    v = rng.gamma(2.0, 1.0, w.shape[0])
    return w, v / v.sum()


def banded_pose_system(n_pose, w, cyclic, seed, n_land=None):
    """A reduced-camera-system-shaped SPD matrix: S = sum of landmark terms v v^T, each over the
    6-vectors of a window of <= w + 1 consecutive poses (cyclic: windows wrap around, a keyframe
    loop), + 0.5 I; and the pose blocks (i <= j) of its structure. (399 poses, w = 19, cyclic: the
    C5 GBA's system) Returns (S, b, block_i, block_j)."""
    rng = np.random.default_rng(seed)
    n = 6 * n_pose
    A = np.zeros((n, n))
    blocks = set()
    for _ in range(n_land or 6 * n_pose):
        s = int(rng.integers(0, n_pose if cyclic else n_pose - w))
        ln = int(rng.integers(2, w + 2))
        poses = [(s + k) % n_pose for k in range(ln) if cyclic or s + k < n_pose]
        idx = np.concatenate([np.arange(6 * p, 6 * p + 6) for p in poses])
        v = rng.normal(size=idx.size)
        A[np.ix_(idx, idx)] += np.outer(v, v)
        for a in poses:
            for b in poses:
                blocks.add((min(a, b), max(a, b)))
    for p in range(n_pose):
        blocks.add((p, p))
    A += np.eye(n) * 0.5
    bi = np.array([b[0] for b in sorted(blocks)], np.int32)
    bj = np.array([b[1] for b in sorted(blocks)], np.int32)
    return A, rng.normal(size=n), bi, bj

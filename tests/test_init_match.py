"""Monocular initialisation matching: U:src/ORBmatcher.cc::SearchForInitialization(F1, F2,
vbPrevMatched, vnMatches12, windowSize) (the greedy pass).

CPU: the C++ oracle against an independent pure-Python restatement of the same loop (also
counting how often the steal path runs, so the fixtures exercise it), definitional KATs
(identical frames match themselves; an empty F2 gives nothing). GPU: the device path (ranked
grid, wave-per-query candidate lists, one-wave greedy chain in LDS) through the C-ABI against
the oracle, bit-exact (matches12, nmatches, the updated vbPrevMatched). Parity unpinned by the
reference (no fixtures upstream).
"""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_init_pair

POP = np.array([bin(i).count("1") for i in range(256)], np.int32)


def py_search_for_initialization(k1, d1, k2, d2, prev, window, ratio, ori, bounds=(0.0, 640.0, 0.0, 480.0)):
    """Pure-Python restatement (walk order: cells ix outer, iy inner, index order in a cell)."""
    minx, maxx, miny, maxy = [np.float32(b) for b in bounds]
    invw = np.float32(64) / (maxx - minx)
    invh = np.float32(48) / (maxy - miny)
    grid = {}
    for k in range(len(k2)):
        px = int(np.round(np.float32(k2["x"][k] - minx) * invw))
        py = int(np.round(np.float32(k2["y"][k] - miny) * invh))
        if 0 <= px < 64 and 0 <= py < 48:
            grid.setdefault((px, py), []).append(k)
    n1 = len(k1)
    m12 = np.full(n1, -1, np.int64)
    md = np.full(len(k2), 2**31 - 1, np.int64)
    m21 = np.full(len(k2), -1, np.int64)
    hist = [[] for _ in range(30)]
    steals = 0
    prev = prev.copy()
    r = np.float32(window)
    for i in range(n1):
        if k1["octave"][i] > 0:
            continue
        x, y = np.float32(prev[i, 0]), np.float32(prev[i, 1])
        x0 = max(0, int(np.floor(np.float32(x - minx - r) * invw)))
        x1 = min(63, int(np.ceil(np.float32(x - minx + r) * invw)))
        y0 = max(0, int(np.floor(np.float32(y - miny - r) * invh)))
        y1 = min(47, int(np.ceil(np.float32(y - miny + r) * invh)))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        cand = []
        for ix in range(x0, x1 + 1):
            for iy in range(y0, y1 + 1):
                for k in grid.get((ix, iy), []):
                    if k2["octave"][k] != 0:
                        continue
                    if abs(np.float32(k2["x"][k] - x)) < r and abs(np.float32(k2["y"][k] - y)) < r:
                        cand.append(k)
        if not cand:
            continue
        dist = POP[np.bitwise_xor(d1[i][None, :], d2[cand])].sum(1)
        best, best2, bi = 2**31 - 1, 2**31 - 1, -1
        for k, d in zip(cand, dist):
            if md[k] <= d:
                continue
            if d < best:
                best2, best, bi = best, int(d), k
            elif d < best2:
                best2 = int(d)
        if best <= 50 and np.float32(best) < np.float32(best2) * np.float32(ratio):
            if m21[bi] >= 0:
                m12[m21[bi]] = -1
                steals += 1
            m12[i] = bi
            m21[bi] = i
            md[bi] = best
            if ori:
                rot = np.float32(k1["angle"][i] - k2["angle"][bi])
                if rot < 0:
                    rot = np.float32(rot + np.float32(360))
                b = int(np.round(np.float32(rot * np.float32(1.0 / 30))))
                hist[0 if b == 30 else b].append(i)
    if ori:
        sizes = [len(h) for h in hist]
        m1 = m2 = m3 = 0
        i1 = i2 = i3 = -1
        for b, s in enumerate(sizes):
            if s > m1:
                m3, m2, m1, i3, i2, i1 = m2, m1, s, i2, i1, b
            elif s > m2:
                m3, m2, i3, i2 = m2, s, i2, b
            elif s > m3:
                m3, i3 = s, b
        if m2 < 0.1 * m1:
            i2 = i3 = -1
        elif m3 < 0.1 * m1:
            i3 = -1
        for b in range(30):
            if b in (i1, i2, i3):
                continue
            for i in hist[b]:
                m12[i] = -1
    for i in np.nonzero(m12 >= 0)[0]:
        prev[i] = (k2["x"][m12[i]], k2["y"][m12[i]])
    return int((m12 >= 0).sum()), m12.astype(np.int32), prev, steals


@pytest.mark.parametrize("seed,window,ratio,ori", [(1, 100, 0.9, True), (2, 100, 0.9, False), (3, 40, 0.7, True)])
def test_oracle_matches_python_restatement(oracle, seed, window, ratio, ori):
    k1, d1, k2, d2, prev = synthetic_init_pair(n1=700, seed=seed)
    n, m, p = oracle.search_for_initialization(k1, d1, k2, d2, prev, window, ratio, ori)
    pn, pm, pp, steals = py_search_for_initialization(k1, d1, k2, d2, prev, window, ratio, ori)
    assert n == pn and np.array_equal(m, pm) and np.array_equal(p, pp)
    assert n > 50
    if window == 100:
        assert steals > 0          # the fixture exercises the steal path


def test_oracle_identical_frames_match_themselves(oracle):
    k1, d1, _, _, prev = synthetic_init_pair(n1=600, seed=4)
    lvl0 = k1["octave"] == 0
    n, m, p = oracle.search_for_initialization(k1, d1, k1, d1, prev, 100, 0.9, False)
    hit = m >= 0
    assert n == hit.sum() and not hit[~lvl0].any()
    assert (m[hit] == np.nonzero(hit)[0]).all()      # distance 0 to itself
    assert hit[lvl0].mean() > 0.9
    assert np.array_equal(p, prev)                   # matched onto itself: positions unchanged
    n0, m0, _ = oracle.search_for_initialization(k1, d1, k1[:0], d1[:0], prev, 100, 0.9, True)
    assert n0 == 0 and (m0 == -1).all()


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["rounds", "chain"])
def test_search_for_initialization_matches_oracle(oracle, monkeypatch, path):
    """Both device formulations: the parallel fixed-point rounds (default) and the one-wave chain
    (ORBHIP_INIT_CHAIN, also the fallback when a rank overflows its claim slots)."""
    from orb_slam3_ros2_amd import ORBmatcher
    if path == "chain":
        monkeypatch.setenv("ORBHIP_INIT_CHAIN", "1")
    for seed in range(6):
        k1, d1, k2, d2, prev = synthetic_init_pair(n1=1500 + 500 * seed, seed=20 + seed)
        for window, ratio, ori in [(100, 0.9, True), (100, 0.9, False), (50, 0.7, True), (200, 0.9, True)]:
            mt = ORBmatcher(ratio, ori)
            n, m, p = mt.SearchForInitialization(k1, d1, k2, d2, prev, window)
            on, om, op = oracle.search_for_initialization(k1, d1, k2, d2, prev, window, ratio, ori)
            assert n == on and np.array_equal(m, om) and np.array_equal(p, op), (seed, window, ratio, ori)


@pytest.mark.gpu
def test_search_for_initialization_extracted_frames(oracle):
    """Real ORB keypoints: the 5x initialisation extractor (5000 features) on two frames of the
    synthetic stream, as Tracking::MonocularInitialization calls it (0.9, true, window 100),
    then a second call on the updated vbPrevMatched."""
    from orb_slam3_ros2_amd import ORBextractor, ORBmatcher
    from orb_slam3_ros2_amd._lib import KP_DTYPE
    from orb_slam3_ros2_amd.synthetic import shifted_frame, synthetic_frame
    ext = ORBextractor(5000, 1.2, 8, 20, 7)
    a = synthetic_frame(3)
    frames = [a, shifted_frame(a, 6, -3, 1), shifted_frame(a, 11, -5, 2)]
    ks, ds = [], []
    for f in frames:
        _, kp, d = ext(f)
        k = np.zeros(len(kp), KP_DTYPE)
        for name in ("x", "y", "size", "angle", "response", "octave"):
            k[name] = kp[name]
        ks.append(k); ds.append(d)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    prev = np.stack([ks[0]["x"], ks[0]["y"]], 1).astype(np.float32)
    oprev = prev.copy()
    for j in (1, 2):
        n, m, prev = mt.SearchForInitialization(ks[0], ds[0], ks[j], ds[j], prev, 100)
        on, om, oprev = oracle.search_for_initialization(ks[0], ds[0], ks[j], ds[j], oprev, 100, 0.9, True)
        assert n == on and np.array_equal(m, om) and np.array_equal(prev, oprev), j
        assert n > 100


@pytest.mark.gpu
def test_search_for_initialization_crowded_rank(oracle):
    """Many queries around one F2 keypoint: round 0 puts them all on one rank (more claimants
    than the claim slots, so the chain decides), with equal distances (no steal: only the first
    keeps it) and with strictly decreasing distances (every query steals from the previous)."""
    from orb_slam3_ros2_amd import ORBmatcher
    k1, d1, k2, d2, prev = synthetic_init_pair(n1=300, seed=6)
    k2 = k2[k2["octave"] == 0][:1].copy()
    d2 = np.zeros((1, 32), np.uint8) + 0x5A
    assert len(k2) == 1
    q = np.repeat(k2, 24)
    q["angle"] = np.linspace(0, 40, 24, dtype=np.float32)
    p = np.stack([q["x"], q["y"]], 1).astype(np.float32) + 3.0
    for steal in (False, True):
        dq = np.repeat(d2, 24, 0)
        if steal:
            for i in range(24):      # 30 - i differing bits: each later query is strictly closer
                bits = np.unpackbits(dq[i])
                bits[: 30 - i] ^= 1
                dq[i] = np.packbits(bits)
        else:
            dq[:, 0] ^= 0x0F          # distance 4 for everybody
        mt = ORBmatcher(0.9, True)
        n, m, pp = mt.SearchForInitialization(q, dq, k2, d2, p, 100)
        on, om, op = oracle.search_for_initialization(q, dq, k2, d2, p, 100, 0.9, True)
        assert n == on and np.array_equal(m, om) and np.array_equal(pp, op), steal
        assert on == 1 and om[-1 if steal else 0] == 0


@pytest.mark.gpu
def test_search_for_initialization_edges(oracle):
    from orb_slam3_ros2_amd import ORBmatcher
    from orb_slam3_ros2_amd._lib import OrbHipError
    mt = ORBmatcher(0.9, True)
    k1, d1, k2, d2, prev = synthetic_init_pair(n1=300, seed=5)
    # empty F2, empty F1, no octave-0 queries
    assert mt.SearchForInitialization(k1, d1, k2[:0], d2[:0], prev)[0] == 0
    n, m, _ = mt.SearchForInitialization(k1[:0], d1[:0], k2, d2, prev[:0])
    assert n == 0 and m.shape == (0,)
    k1b = k1.copy()
    k1b["octave"] = 3
    n, m, _ = mt.SearchForInitialization(k1b, d1, k2, d2, prev, 100)
    assert n == 0 and (m == -1).all()
    # queries far outside the image: no cells
    far = prev + 5000.0
    n, m, p = mt.SearchForInitialization(k1, d1, k2, d2, far, 100)
    on, om, op = oracle.search_for_initialization(k1, d1, k2, d2, far, 100, 0.9, True)
    assert n == on == 0 and np.array_equal(p, op)
    k1c = k1.copy()
    k1c["octave"][0] = -1
    with pytest.raises(OrbHipError):
        mt.SearchForInitialization(k1c, d1, k2, d2, prev)

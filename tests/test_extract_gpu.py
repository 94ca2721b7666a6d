"""GPU parity: ORBextractor::operator() on gfx950 vs the CPU restatement (oracle/).

Bit-exact on every keypoint field (x, y, size, angle, response, octave), the descriptor
bits, the output order and monoIndex. Inputs: the seeded synthetic frames of SURVEY.md
§8(d) plus edge cases (constant frame, pure noise, small/odd sizes, lapping variants).
Parity is against the restatement; the reference itself is unbuildable here.
"""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_frame
from tests.helpers import diff_report, oracle_kps_to_struct

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ext1000():
    from orb_slam3_ros2_amd import ORBextractor
    return ORBextractor(1000, 1.2, 8, 20, 7)


def _check(ext, oracle, img, nfeatures=1000, lap=(0, 1000), scale=1.2, nlevels=8, ini=20, mn=7):
    mono, gk, gd = ext(img, None, lap)
    omono, ok6, od = oracle.extract(img, nfeatures, scale, nlevels, ini, mn, lap)
    ok = oracle_kps_to_struct(ok6)
    same = (mono == omono and len(gk) == len(ok) and all(np.array_equal(gk[f], ok[f]) for f in ok.dtype.names)
            and (len(ok) == 0 or np.array_equal(gd, od)))
    assert same, f"monoIndex gpu={mono} oracle={omono}\n" + diff_report(gk, gd, ok, od)
    return len(gk)


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_c2_640x480_bit_exact(ext1000, oracle, seed):
    n = _check(ext1000, oracle, synthetic_frame(seed, 640, 480))
    assert n > 900


@pytest.mark.parametrize("w,h,seed", [(1280, 720, 10), (752, 480, 11), (641, 479, 12), (320, 240, 13)])
def test_sizes_bit_exact(ext1000, oracle, w, h, seed):
    _check(ext1000, oracle, synthetic_frame(seed, w, h))


@pytest.mark.parametrize("w,h,scale,nlev,seed", [(1280, 720, 1.2, 8, 30), (641, 479, 1.2, 8, 31),
                                                 (641, 481, 1.5, 5, 32), (801, 601, 1.9, 4, 33),
                                                 (1001, 751, 2.5, 3, 34)])
@pytest.mark.parametrize("hi", ["bands", "bands5", "resize", "cone", "flow"])
def test_resize_cascade_bit_exact(oracle, monkeypatch, w, h, scale, nlev, seed, hi):
    """The batch engine forced on single frames: k_resize for every level (the default), the
    one-launch dataflow pyramid (ORBHIP_RZ_FLOW=1, k_pyr_flow), or
    k_resize for levels 1-2 and then levels 3.. by the opt-in k_resize_bands (ORBHIP_RZ_BANDS=16
    or 5 row bands per frame) or the opt-in batch cone (ORBHIP_CONE_HI=1). Odd sizes take the edge
    lanes, scale factors above 1.2 k_resize's per-row path (a 4-row group reads more than 6
    source rows), all bit-exact against the oracle's cv::resize restatement."""
    from orb_slam3_ros2_amd import ORBextractor
    monkeypatch.setenv("ORBHIP_NO_CONE", "1")
    if hi == "cone":
        monkeypatch.setenv("ORBHIP_CONE_HI", "1")
    elif hi == "bands":
        monkeypatch.setenv("ORBHIP_RZ_BANDS", "16")
    elif hi == "bands5":
        monkeypatch.setenv("ORBHIP_RZ_BANDS", "5")
    elif hi == "flow":
        monkeypatch.setenv("ORBHIP_RZ_FLOW", "1")
    ext = ORBextractor(1000, scale, nlev, 20, 7)
    _check(ext, oracle, synthetic_frame(seed, w, h), scale=scale, nlevels=nlev)


@pytest.mark.parametrize("pack", ["1", "0"])
def test_packed_candidates_bit_exact(oracle, monkeypatch, pack):
    """FAST's packed candidate layout (one atomic per cell into its level's region, the octree
    reading each cell's run through the offset table; opt-in, ORBHIP_CAND_PACK=1) and the fixed
    slot ranges: the keypoints and descriptors are the oracle's either way (the octree's key order
    is cell-major through the table in both)."""
    from orb_slam3_ros2_amd import ORBextractor
    monkeypatch.setenv("ORBHIP_CAND_PACK", pack)
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    _check(ext, oracle, synthetic_frame(81, 640, 480))
    _check(ext, oracle, synthetic_frame(82, 1280, 720))
    _check(ext, oracle, synthetic_frame(83, 641, 479))


@pytest.mark.parametrize("tile", [5, 17, 48])
def test_batch_cone_tiles_bit_exact(oracle, monkeypatch, tile):
    """The opt-in batch cone (levels 3.. from level 2, ORBHIP_CONE_HI_TILE per plan lookup) at
    tile edges other than its default 32: every tiling writes the same pyramid."""
    from orb_slam3_ros2_amd import ORBextractor
    monkeypatch.setenv("ORBHIP_NO_CONE", "1")
    monkeypatch.setenv("ORBHIP_CONE_HI", "1")
    monkeypatch.setenv("ORBHIP_CONE_HI_TILE", str(tile))
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    _check(ext, oracle, synthetic_frame(70 + tile, 1280, 720))
    _check(ext, oracle, synthetic_frame(71 + tile, 641, 479))


@pytest.mark.parametrize("tile", [12, 14, 16, 20])
def test_cone_tiles_bit_exact(oracle, monkeypatch, tile):
    """k_pyr_cone at the tile edges the front-end picks by camera count (10 / 14 / 16) and
    others (ORBHIP_CONE_TILE, read per plan lookup): every tiling writes the same pyramid."""
    from orb_slam3_ros2_amd import ORBextractor
    monkeypatch.setenv("ORBHIP_CONE_TILE", str(tile))
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    _check(ext, oracle, synthetic_frame(40 + tile, 640, 480))
    _check(ext, oracle, synthetic_frame(41 + tile, 752, 480))


def test_milkv_1250_features(oracle):
    """R:config/Monocular/MilkV.yaml:42-55 (1250 features) at its 640x360 camera size."""
    from orb_slam3_ros2_amd import ORBextractor
    ext = ORBextractor(1250, 1.2, 8, 20, 7)
    _check(ext, oracle, synthetic_frame(21, 640, 360), nfeatures=1250)


def test_initializer_5x_features(oracle):
    """Tracking's mpIniORBextractor uses 5*nFeatures (U:src/Tracking.cc)."""
    from orb_slam3_ros2_amd import ORBextractor
    ext = ORBextractor(5000, 1.2, 8, 20, 7)
    _check(ext, oracle, synthetic_frame(22, 640, 480), nfeatures=5000)


@pytest.mark.parametrize("lap", [(0, 1000), (0, 0), (-1, -1), (200, 400), (0, 100000)])
def test_lapping_area_order(ext1000, oracle, lap):
    _check(ext1000, oracle, synthetic_frame(30, 1280, 720), lap=lap)


def test_constant_frame_has_no_keypoints(ext1000, oracle):
    img = np.full((480, 640), 77, np.uint8)
    mono, k, d = ext1000(img)
    assert mono == 0 and len(k) == 0
    _check(ext1000, oracle, img)


def test_uniform_noise(ext1000, oracle):
    rng = np.random.default_rng(5)
    _check(ext1000, oracle, rng.integers(0, 256, size=(480, 640), dtype=np.uint8))


@pytest.mark.parametrize("cap", [0, 64])
def test_fast_dense_pass(oracle, monkeypatch, cap):
    """k_fast_cells keeps at most kClistCap pair-test survivors per cell in LDS; a cell with more
    walks every pixel instead. A lowered cap (0: every cell, 64: the textured ones) forces that
    dense pass on frames whose survivors fit the default list."""
    monkeypatch.setenv("ORBHIP_FAST_CLIST_CAP", str(cap))
    from orb_slam3_ros2_amd import ORBextractor
    ext = ORBextractor(1000, 1.2, 8, 20, 7)   # a fresh context: the plan reads the cap
    rng = np.random.default_rng(9)
    for img in (synthetic_frame(3, 640, 480), rng.integers(0, 256, size=(480, 640), dtype=np.uint8),
                (128 + rng.integers(-9, 10, size=(480, 640))).astype(np.uint8)):
        assert _check(ext, oracle, img) > 0


@pytest.mark.parametrize("nt", [128, 256, 512, 1024])
@pytest.mark.parametrize("cap", [0, 2048])
@pytest.mark.parametrize("size", [(640, 480), (320, 240)])
def test_fast_threads_per_cell_batched(oracle, monkeypatch, nt, cap, size):
    """Every k_fast_cells variant (threads per cell pinned per plan by ORBHIP_FAST_NT) on a batch
    of 3 frames through the device path, with the survivor list (cap 2048, the default; the
    compact LDS variant lists 768) and the dense pass forced (cap 0): each frame equals the
    oracle. 640x480 cells fit the compact LDS variant (128 / 256 threads); 320x240 has one-row
    levels whose cells (up to 75 rows) take the full one."""
    import torch
    monkeypatch.setenv("ORBHIP_FAST_NT", str(nt))
    monkeypatch.setenv("ORBHIP_FAST_CLIST_CAP", str(cap))
    from orb_slam3_ros2_amd import ORBextractor
    ext = ORBextractor(1000, 1.2, 8, 20, 7)   # a fresh context: the plan reads both variables
    rng = np.random.default_rng(nt + cap)
    B, (W, H) = 3, size
    frames = np.stack([synthetic_frame(70 + nt % 7, W, H), rng.integers(0, 256, size=(H, W), dtype=np.uint8),
                       (128 + rng.integers(-9, 10, size=(H, W))).astype(np.uint8)])
    kcap = ext.max_keypoints(W, H)
    dev = torch.device("cuda:0")
    kps = torch.zeros((B, kcap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, kcap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    ext.extract_batch_device(torch.from_numpy(frames).to(dev), kps, desc, n, mono)
    torch.cuda.synchronize()
    for i in range(B):
        omono, ok6, od = oracle.extract(frames[i], 1000, 1.2, 8, 20, 7, (0, 1000))
        ok = oracle_kps_to_struct(ok6)
        assert int(n[i]) == len(ok) and int(mono[i]) == omono
        kk = kps[i, : len(ok)].cpu().numpy()
        assert np.array_equal(kk[:, 0], ok["x"]) and np.array_equal(kk[:, 1], ok["y"])
        assert np.array_equal(kk[:, 3], ok["angle"]) and np.array_equal(kk[:, 5].view(np.int32), ok["octave"])
        assert np.array_equal(desc[i, : len(ok)].cpu().numpy(), od)


def test_low_contrast_uses_min_threshold(ext1000, oracle):
    """Cells with no corner at iniThFAST=20 fall back to minThFAST=7."""
    rng = np.random.default_rng(6)
    img = (128 + rng.integers(-9, 10, size=(480, 640))).astype(np.uint8)
    _check(ext1000, oracle, img)


def test_empty_image_returns_minus_one(ext1000):
    mono, k, d = ext1000(np.zeros((0, 0), np.uint8))
    assert mono == -1 and len(k) == 0 and d is None


def test_batch_device_matches_single(ext1000):
    import torch
    B, H, W = 4, 480, 640
    frames = np.stack([synthetic_frame(40 + i, W, H) for i in range(B)])
    cap = ext1000.max_keypoints(W, H)
    dev = torch.device("cuda:0")
    tf = torch.from_numpy(frames).to(dev)
    kps = torch.zeros((B, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    ext1000.extract_batch_device(tf, kps, desc, n, mono)
    torch.cuda.synchronize()
    for i in range(B):
        m1, k1, d1 = ext1000(frames[i])
        assert int(n[i]) == len(k1) and int(mono[i]) == m1
        kk = kps[i, : len(k1)].cpu().numpy()
        assert np.array_equal(kk[:, 0], k1["x"]) and np.array_equal(kk[:, 3], k1["angle"])
        assert np.array_equal(kk[:, 5].view(np.int32), k1["octave"])
        assert np.array_equal(desc[i, : len(k1)].cpu().numpy(), d1)


def test_device_sincosf_matches_glibc_exhaustive(oracle):
    """Every float in [0, 6.2832]: device glibc_sinf/cosf restatement == host glibc."""
    from orb_slam3_ros2_amd._lib import lib
    lo = np.float32(0.0).view(np.uint32).item()
    hi = np.float32(6.2832).view(np.uint32).item()
    chunk = 1 << 27
    total_bad = 0
    for a in range(lo, hi + 1, chunk):
        b = min(a + chunk - 1, hi)
        c, s = oracle.glibc_sincosf_range(a, b)
        bad = lib().orbhip_test_sincosf_sweep(a, b, c.ctypes.data, s.ctypes.data)
        assert bad >= 0
        total_bad += bad
    assert total_bad == 0


def test_large_batch_paths_match_oracle(ext1000, oracle):
    """B = 16: the batch launch shapes (per-level k_resize cascade, 256-thread FAST cells, a
    keypoint per wave in k_desc) against the oracle, frame by frame."""
    import torch
    B, H, W = 16, 480, 640
    frames = np.stack([synthetic_frame(60 + i, W, H) for i in range(B)])
    cap = ext1000.max_keypoints(W, H)
    dev = torch.device("cuda:0")
    tf = torch.from_numpy(frames).to(dev)
    kps = torch.zeros((B, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    ext1000.extract_batch_device(tf, kps, desc, n, mono)
    torch.cuda.synchronize()
    for i in range(B):
        om, ok, od = oracle.extract(frames[i])
        assert int(n[i]) == len(ok) and int(mono[i]) == om, i
        kk = kps[i, : len(ok)].cpu().numpy()
        assert np.array_equal(kk[:, :5], ok[:, :5]), i
        assert np.array_equal(kk[:, 5].view(np.int32), ok[:, 5].astype(np.int32)), i
        assert np.array_equal(desc[i, : len(ok)].cpu().numpy(), od), i


def test_graph_replay_recomputes_from_current_inputs(monkeypatch):
    """With ORBHIP_GRAPH=1, repeated device calls with identical arguments on a stream replay a
    captured launch graph (graph_cache.h). A replay must read the buffers' CURRENT contents: the same input
    buffer is refilled with different frames between calls, and every extraction and match must
    equal the direct launches on the HIP null stream."""
    import torch
    from orb_slam3_ros2_amd import ORBextractor, ORBmatcher
    from orb_slam3_ros2_amd._lib import lib
    monkeypatch.setenv("ORBHIP_GRAPH", "1")
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    H, W = 480, 640
    cap = ext.max_keypoints(W, H)
    dev = torch.device("cuda:0")
    imgs = [torch.from_numpy(synthetic_frame(60 + i, W, H)).to(dev) for i in range(5)]

    def bufs():
        return (torch.zeros((2, cap, 6), dtype=torch.float32, device=dev),
                torch.zeros((2, cap, 32), dtype=torch.uint8, device=dev),
                torch.zeros(2, dtype=torch.int32, device=dev), torch.zeros(2, dtype=torch.int32, device=dev),
                torch.zeros((3, cap), dtype=torch.int32, device=dev), torch.zeros(1, dtype=torch.int32, device=dev))

    def run(frame_buf, b, stream):
        kps, desc, n, mono, mm, nm = b
        ext.extract_batch_device(frame_buf, kps, desc, n, mono, stream=stream)
        mt.match_pairs_device(kps, desc, n, mm[0:1], mm[1:2], mm[2:3], nm, stream=stream)

    st = torch.cuda.Stream()
    fb = torch.empty((2, H, W), dtype=torch.uint8, device=dev)
    got, ref = bufs(), bufs()
    for i in range(4):
        pair = torch.stack([imgs[i], imgs[i + 1]])
        fb.copy_(pair)
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            run(fb, got, st)
        st.synchronize()
        run(pair.contiguous(), ref, None)   # null stream: direct
        torch.cuda.synchronize()
        kps, desc, n, mono, mm, nm = got
        rk, rd, rn, rmono, rmm, rnm = ref
        assert torch.equal(n, rn) and torch.equal(mono, rmono) and torch.equal(nm, rnm), i
        for f in range(2):
            c = int(rn[f])
            assert torch.equal(kps[f, :c], rk[f, :c]) and torch.equal(desc[f, :c], rd[f, :c]), (i, f)
        assert torch.equal(mm[:, : int(rn[0])], rmm[:, : int(rn[0])]), i
    assert lib().orbhip_launch_graphs(ext.ctx.handle) >= 2   # extract + match replayed


def _clustered_frame(seed, w=640, h=480):
    """A flat frame with one small, dense, high-contrast patch: thousands of FAST candidates in
    a few cells, so DistributeOctTree divides deep (far below the pyramid depth) around it."""
    rng = np.random.default_rng(seed)
    img = np.full((h, w), 128, np.uint8)
    y0, x0 = h // 3, w // 2
    img[y0:y0 + 40, x0:x0 + 48] = rng.integers(0, 256, size=(40, 48), dtype=np.uint8)
    return img


@pytest.mark.parametrize("engine", ["pyramid", "sweep", "dh1", "dh2", "dh3"])
def test_octree_engines(oracle, monkeypatch, engine):
    """k_octree divides with the pyramid (counts of every depth-d cell, no key sweeps) and falls
    back to the key-sweep path when a node to divide sits at the pyramid's deepest level. Each
    engine, and the fallback forced by shallow pyramids (ORBHIP_OCTREE_DH), bit-exact against the
    oracle on C2 / C3-sized frames, 5000 features, noise and clustered keys."""
    from orb_slam3_ros2_amd import ORBextractor
    if engine == "sweep":
        monkeypatch.setenv("ORBHIP_OCTREE_SWEEP", "1")
    elif engine != "pyramid":
        monkeypatch.setenv("ORBHIP_OCTREE_DH", engine[2:])
    rng = np.random.default_rng(17)
    e1000 = ORBextractor(1000, 1.2, 8, 20, 7)
    for img in (synthetic_frame(40, 640, 480), synthetic_frame(41, 1280, 720), _clustered_frame(42),
                rng.integers(0, 256, size=(480, 640), dtype=np.uint8), _clustered_frame(43, 1280, 720)):
        _check(e1000, oracle, img)
    e5000 = ORBextractor(5000, 1.2, 8, 20, 7)
    for img in (synthetic_frame(44, 640, 480), _clustered_frame(45)):
        _check(e5000, oracle, img, nfeatures=5000)

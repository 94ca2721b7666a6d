"""GPU parity: Hamming brute-force matcher (DescriptorDistance, best/second, TH_LOW, ratio,
rotation histogram) vs the oracle, on extractor outputs and on the SURVEY §8(d) microbench,
through both device formulations (one launch with a last-workgroup filter; top-2 partials +
finish kernel)."""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import shifted_frame, synthetic_frame

pytestmark = pytest.mark.gpu


@pytest.fixture(params=["fused", "two-kernel"], autouse=True)
def match_path(request, monkeypatch):
    """Every test runs on both device matchers: the one-launch k_match_fused (<= 4 pairs, the
    default) and the k_match_top2 + k_match_finish pair (larger batches; forced here)."""
    if request.param == "two-kernel":
        monkeypatch.setenv("ORBHIP_MATCH_UNFUSED", "1")
    return request.param


@pytest.fixture(scope="module")
def matcher():
    from orb_slam3_ros2_amd import ORBmatcher
    return ORBmatcher(0.9, True)


def _cmp(matcher, oracle, q, qa, t, ta, th=50, ratio=0.9, ori=True):
    matcher.mfNNratio, matcher.mbCheckOrientation = ratio, ori
    n, m, b, s = matcher.match_bf(q, qa, t, ta, th)
    on, om, ob, os_ = oracle.match_bf(q, qa, t, ta, th, ratio, ori)
    assert np.array_equal(b, ob) and np.array_equal(s, os_)
    assert np.array_equal(m, om) and n == on
    return n


def test_microbench_flips(matcher, oracle):
    rng = np.random.default_rng(1234)
    q = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
    t = q.copy()
    for i in range(1000):
        for bit in rng.choice(256, int(rng.integers(0, 41)), replace=False):
            t[i, bit // 8] ^= np.uint8(1 << (bit % 8))
    t = np.concatenate([t, rng.integers(0, 256, (1000, 32), dtype=np.uint8)])[rng.permutation(2000)]
    qa = rng.uniform(0, 360, 1000).astype(np.float32)
    ta = rng.uniform(0, 360, 2000).astype(np.float32)
    for ori in (False, True):
        _cmp(matcher, oracle, q, qa, t, ta, ori=ori)


def test_extracted_frame_pair(matcher, oracle):
    from orb_slam3_ros2_amd import ORBextractor
    ext = ORBextractor(1000)
    a = synthetic_frame(100)
    b = shifted_frame(a, 3, -2, 101)
    _, ka, da = ext(a)
    _, kb, db = ext(b)
    n = _cmp(matcher, oracle, da, ka["angle"], db, kb["angle"])
    assert n > 300
    _cmp(matcher, oracle, da, ka["angle"], db, kb["angle"], th=100, ratio=0.6)


def test_ties_and_tiles(matcher, oracle):
    """duplicate train descriptors (first index wins), > 1024 trains (multiple LDS tiles)."""
    rng = np.random.default_rng(7)
    base = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    t = np.concatenate([base, base, base])          # every query has 3 exact ties
    q = base[rng.permutation(700)[:300]]
    a = np.zeros(300, np.float32)
    ta = np.zeros(2100, np.float32)
    _cmp(matcher, oracle, q, a, t, ta, ratio=1.01)   # ratio > 1 so ties (d < r*d) can be accepted


def test_empty_sets(matcher, oracle):
    q = np.zeros((5, 32), np.uint8)
    n, m, b, s = matcher.match_bf(q, np.zeros(5, np.float32), np.zeros((0, 32), np.uint8), np.zeros(0, np.float32))
    assert n == 0 and np.all(m == -1)


def test_pairs_device(oracle):
    import torch
    from orb_slam3_ros2_amd import ORBextractor, ORBmatcher
    ext = ORBextractor(1000)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    B, H, W = 4, 480, 640
    frames = [synthetic_frame(200)]
    for i in range(1, B):
        frames.append(shifted_frame(frames[-1], 2, 1, 200 + i))
    frames = np.stack(frames)
    cap = ext.max_keypoints(W, H)
    dev = torch.device("cuda:0")
    kps = torch.zeros((B, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    ext.extract_batch_device(torch.from_numpy(frames).to(dev), kps, desc, n, mono)
    mm = torch.zeros((B - 1, cap), dtype=torch.int32, device=dev)
    bb = torch.zeros_like(mm); ss = torch.zeros_like(mm)
    nm = torch.zeros(B - 1, dtype=torch.int32, device=dev)
    mt.match_pairs_device(kps, desc, n, mm, bb, ss, nm)
    torch.cuda.synchronize()
    for p in range(B - 1):
        nq, nt = int(n[p]), int(n[p + 1])
        q = desc[p, :nq].cpu().numpy(); t = desc[p + 1, :nt].cpu().numpy()
        qa = kps[p, :nq, 3].cpu().numpy(); ta = kps[p + 1, :nt, 3].cpu().numpy()
        on, om, ob, os_ = oracle.match_bf(q, qa, t, ta, 50, 0.9, True)
        assert int(nm[p]) == on and np.array_equal(mm[p, :nq].cpu().numpy(), om)


def _extract_stream(B, seed):
    import torch
    from orb_slam3_ros2_amd import ORBextractor
    from orb_slam3_ros2_amd.synthetic import synthetic_stream
    ext = ORBextractor(1000)
    frames = torch.from_numpy(synthetic_stream(B, 640, 480, seed)).to("cuda:0")
    cap = ext.max_keypoints(640, 480)
    dev = frames.device
    kps = torch.zeros((B, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    mono = torch.zeros(B, dtype=torch.int32, device=dev)
    ext.extract_batch_device(frames, kps, desc, n, mono)
    torch.cuda.synchronize()
    return ext, kps, desc, n, cap


@pytest.mark.parametrize("fill", ["zeros", "bin0_indices", "previous_results", "word_ids"])
def test_stale_output_buffers_vs_oracle(oracle, fill):
    """Adversarial stale contents in the match/best/second outputs: the one-launch
    matcher's last workgroup reads match[] back, so anything a plain store left behind in another
    XCD's L2 would surface here as a bin-0 tentative match. Every pair is checked against the
    oracle, never against another device path."""
    import torch
    from orb_slam3_ros2_amd import ORBmatcher
    B = 6
    ext, kps, desc, n, cap = _extract_stream(B, 4242)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    dev = kps.device
    refs = []
    for p in range(B - 1):
        nq, nt = int(n[p]), int(n[p + 1])
        q = desc[p, :nq].cpu().numpy(); t = desc[p + 1, :nt].cpu().numpy()
        qa = kps[p, :nq, 3].cpu().numpy(); ta = kps[p + 1, :nt, 3].cpu().numpy()
        refs.append(oracle.match_bf(q, qa, t, ta, 50, 0.9, True))
    rng = np.random.default_rng(5)
    for rep in range(3):
        if fill == "zeros":
            mm = torch.zeros((B - 1, cap), dtype=torch.int32, device=dev)
        elif fill == "bin0_indices":   # non-negative indices with bits 24+ clear = bin-0 tentative matches
            mm = torch.arange(cap, dtype=torch.int32, device=dev).repeat(B - 1, 1)
        elif fill == "previous_results":   # the oracle's answer for a DIFFERENT pair
            prev = np.full((B - 1, cap), -1, np.int32)
            for p in range(B - 1):
                om = refs[(p + 1 + rep) % (B - 1)][1]
                prev[p, :len(om)] = om
            mm = torch.from_numpy(prev).to(dev)
        else:                          # random word ids (what bow_transform leaves in the ctx scratch)
            mm = torch.from_numpy(rng.integers(0, 1 << 20, (B - 1, cap), dtype=np.int32)).to(dev)
        bb = torch.full_like(mm, 7); ss = torch.full_like(mm, 3)
        nm = torch.full((B - 1,), 12345, dtype=torch.int32, device=dev)
        # one pair per launch (the C2 fused shape) and all pairs in one launch
        for p in range(B - 1):
            mt.match_pairs_device(kps[p:p + 2], desc[p:p + 2], n[p:p + 2], mm[p:p + 1], bb[p:p + 1], ss[p:p + 1],
                                  nm[p:p + 1])
        torch.cuda.synchronize()
        for p in range(B - 1):
            on, om, ob, os_ = refs[p]
            nq = len(om)
            assert int(nm[p]) == on, (fill, rep, p)
            assert np.array_equal(mm[p, :nq].cpu().numpy(), om), (fill, rep, p)
            assert np.array_equal(bb[p, :nq].cpu().numpy(), ob) and np.array_equal(ss[p, :nq].cpu().numpy(), os_)


def test_match_bf_sequence_vs_oracle(oracle):
    """The host match_bf reuses the context's device scratch for its outputs: a sequence of calls
    over different pairs (each leaving its results behind for the next) and a DBoW2 transform in
    between, every call against the oracle."""
    from orb_slam3_ros2_amd import ORBextractor, ORBmatcher
    from orb_slam3_ros2_amd.synthetic import synthetic_stream
    ext = ORBextractor(1000)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    frames = synthetic_stream(8, 640, 480, 99)
    out = [ext(f) for f in frames]
    for k in range(1, len(out)):
        _, ka, da = out[k - 1]
        _, kb, db = out[k]
        for ori in (True, False):
            mt.mbCheckOrientation = ori
            n, m, b, s = mt.match_bf(da, ka["angle"], db, kb["angle"])
            on, om, ob, os_ = oracle.match_bf(da, ka["angle"], db, kb["angle"], 50, 0.9, ori)
            assert n == on and np.array_equal(m, om) and np.array_equal(b, ob), (k, ori)

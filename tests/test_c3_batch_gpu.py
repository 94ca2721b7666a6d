"""C3 at its full size (BASELINE configs[2]): 1280 x 720, a batch of 64 consecutive frames
extracted in one batched call and the 63 consecutive pairs brute-force matched (TH_LOW 50, ratio
0.9, rotation check), every frame and every pair against the oracle (keypoints, descriptors and
monoIndex bit-exact; match indices and counts bit-exact). Then the multi-GPU partition of the same
batch (contiguous slices + a one-frame halo, bench.BatchC3 on rank r of N) run
slice by slice on this device: the union of the ranks' pair results is the whole batch's."""
import numpy as np
import pytest

from orb_slam3_ros2_amd._lib import KP_DTYPE
from orb_slam3_ros2_amd.sharding import frame_slice_with_halo
from tests.helpers import diff_report, oracle_kps_to_struct

pytestmark = pytest.mark.gpu
W, H, B = 1280, 720, 64


def _run(frames_np, reps=1):
    import torch
    from orb_slam3_ros2_amd import ORBextractor, ORBmatcher
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    dev = torch.device("cuda:0")
    nb = len(frames_np)
    cap = ext.max_keypoints(W, H)
    kps = torch.zeros((nb, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((nb, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(nb, dtype=torch.int32, device=dev)
    mono = torch.zeros(nb, dtype=torch.int32, device=dev)
    fr = torch.from_numpy(np.ascontiguousarray(frames_np)).to(dev)
    for _ in range(reps):   # reps > 1: the same context's launches back to back (k_pyr_flow generations)
        ext.extract_batch_device(fr, kps, desc, n, mono)
    mm = torch.full((3, max(nb - 1, 1), cap), -7, dtype=torch.int32, device=dev)
    nm = torch.zeros(max(nb - 1, 1), dtype=torch.int32, device=dev)
    if nb > 1:
        mt.match_pairs_device(kps, desc, n, mm[0], mm[1], mm[2], nm)
    torch.cuda.synchronize()
    return kps.cpu().numpy(), desc.cpu().numpy(), n.cpu().numpy(), mono.cpu().numpy(), mm.cpu().numpy(), \
        nm.cpu().numpy()


@pytest.fixture(scope="module")
def c3():
    from orb_slam3_ros2_amd.synthetic import synthetic_stream
    frames = synthetic_stream(B, W, H, 5000)          # the bench's C3 batch
    return frames, _run(frames)


def test_c3_batch_vs_oracle(c3, oracle):
    frames, (kps, desc, n, mono, mm, nm) = c3
    ok = {}
    for f in range(B):
        omono, k6, od = oracle.extract(frames[f])
        gk = np.frombuffer(kps[f, :n[f]].tobytes(), KP_DTYPE)
        ref = oracle_kps_to_struct(k6)
        assert mono[f] == omono and np.array_equal(gk, ref) and np.array_equal(desc[f, :n[f]], od), \
            (f, diff_report(gk, desc[f, :n[f]], ref, od))
        ok[f] = (k6, od)
    for p in range(B - 1):
        (k1, d1), (k2, d2) = ok[p], ok[p + 1]
        on, om, _, _ = oracle.match_bf(d1, k1[:, 3].astype(np.float32), d2, k2[:, 3].astype(np.float32), 50, 0.9,
                                       True)
        assert nm[p] == on and np.array_equal(mm[0, p, :n[p]], om), p
        assert on > 200


def test_c3_flow_pyramid_reproduces_batch(c3, monkeypatch):
    """The batch pyramid as one dataflow launch (ORBHIP_RZ_FLOW=1, k_pyr_flow: 16-row band tasks
    from a ticket counter, each waiting on the flags of the bands its source rows lie in) gives the
    oracle-checked batch bit for bit, over three launches on one context (the band flags carry the
    launch generation, nothing is reset between launches)."""
    monkeypatch.setenv("ORBHIP_RZ_FLOW", "1")
    frames, ref = c3
    got = _run(frames, reps=3)
    for a, b in zip(got, ref):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("N", [2, 3, 8])
def test_c3_halo_slices_reproduce_batch(c3, N):
    frames, (kps, desc, n, mono, mm, nm) = c3
    seen = []
    for r in range(N):
        lo, hx, plo, phi = frame_slice_with_halo(B, r, N)
        k2, d2, n2, m2, mm2, nm2 = _run(frames[lo:hx])
        assert np.array_equal(n2, n[lo:hx]) and np.array_equal(m2, mono[lo:hx])
        for f in range(hx - lo):
            assert np.array_equal(k2[f, :n2[f]], kps[lo + f, :n2[f]])
        for p in range(plo, phi):
            j = p - lo
            assert nm2[j] == nm[p] and np.array_equal(mm2[:, j, :n[p]], mm[:, p, :n[p]]), (N, r, p)
        seen += list(range(plo, phi))
    assert sorted(seen) == list(range(B - 1))


def test_c3_pipelined_batches_match_single(c3):
    """bench.PipelinedC3 (two 64-frame batches in flight, each slot its own context and stream):
    after several alternating batches, every slot holds exactly the one-batch results (the
    oracle-checked ones above)."""
    import torch
    import bench
    frames, (kps, desc, n, mono, mm, nm) = c3
    pc = bench.PipelinedC3(0, 1, 2)
    for _ in range(5):
        pc.step()
    torch.cuda.synchronize()
    for sl in pc.slots:
        assert np.array_equal(sl.n.cpu().numpy(), n) and np.array_equal(sl.mono.cpu().numpy(), mono)
        for f in range(B):
            assert np.array_equal(sl.kps[f, :n[f]].cpu().numpy(), kps[f, :n[f]])
            assert np.array_equal(sl.desc[f, :n[f]].cpu().numpy(), desc[f, :n[f]])
        assert np.array_equal(sl.nm.cpu().numpy(), nm)
        for p in range(B - 1):
            c = nm[p]
            assert np.array_equal(sl.mm[0, p].cpu().numpy()[: n[p]], mm[0, p][: n[p]]), p

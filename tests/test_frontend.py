"""The camera front-end stream (include/orbhip.h orbhip_frontend_*, FrameStream): frames pushed
through the pipelined device stream give exactly the oracle's per-frame results (extraction of
the frame, brute-force match against the previous frame), and the same as the one-frame device
calls, for 1, 3 and 8 frames in flight; frame 0 has no match; misuse is rejected."""
import numpy as np
import pytest

from tests.helpers import diff_report, oracle_kps_to_struct
from orb_slam3_ros2_amd._lib import KP_DTYPE

pytestmark = pytest.mark.gpu


def _direct(ext, mt, frames, k, cap):
    import torch
    dev = frames.device
    kps = torch.zeros((2, cap, 6), dtype=torch.float32, device=dev)
    desc = torch.zeros((2, cap, 32), dtype=torch.uint8, device=dev)
    n = torch.zeros(2, dtype=torch.int32, device=dev)
    mono = torch.zeros(2, dtype=torch.int32, device=dev)
    ext.extract_batch_device(frames[k - 1:k + 1].contiguous(), kps, desc, n, mono)
    mm = torch.zeros((3, cap), dtype=torch.int32, device=dev)
    nm = torch.zeros(1, dtype=torch.int32, device=dev)
    mt.match_pairs_device(kps, desc, n, mm[0:1], mm[1:2], mm[2:3], nm)
    torch.cuda.synchronize()
    return kps, desc, n, mono, mm, nm


@pytest.mark.parametrize("S", [1, 3, 8])
def test_frontend_matches_oracle_and_one_frame_calls(S, oracle):
    import torch
    from orb_slam3_ros2_amd import FrameStream, ORBextractor, ORBmatcher
    from orb_slam3_ros2_amd.synthetic import synthetic_stream
    K = 45
    frames = torch.from_numpy(synthetic_stream(K, 640, 480, 77)).to("cuda")
    fs = FrameStream(640, 480, S)
    assert fs.slots == (2 if S == 1 else 2 * S)
    slots = [fs.push(frames[k]) for k in range(K)]
    assert slots == [k % fs.slots for k in range(K)]
    fs.wait(slots[-1])
    torch.cuda.synchronize()
    ext = ORBextractor(1000, 1.2, 8, 20, 7)
    mt = ORBmatcher(0.9, True, ctx=ext.ctx)
    cap = fs.cap
    host = frames.cpu().numpy()
    okp = {}
    for k in range(K - fs.slots - 1, K):
        okp[k] = oracle.extract(host[k])
    for k in range(K - fs.slots, K):
        v = fs.view(slots[k])
        assert v["frame"] == k
        kps, desc, n, mono, mm, nm = _direct(ext, mt, frames, k, cap)
        c, cq = int(n[1]), int(n[0])
        assert int(v["n"][0]) == c and int(v["mono"][0]) == int(mono[1]), k
        assert torch.equal(v["kps"][:c], kps[1, :c]) and torch.equal(v["desc"][:c], desc[1, :c]), k
        assert int(v["nmatch"][0]) == int(nm[0]) and int(nm[0]) > 100, k
        for j, name in enumerate(("match", "best", "second")):
            assert torch.equal(v[name][:cq], mm[j, :cq]), (k, name)
        # the oracle: this frame's extraction and its match against the previous frame
        omono, ok6, od = okp[k]
        gk = np.frombuffer(v["kps"][:c].cpu().numpy().tobytes(), KP_DTYPE)
        gd = v["desc"][:c].cpu().numpy()
        ok = oracle_kps_to_struct(ok6)
        assert int(v["mono"][0]) == omono and np.array_equal(gk, ok) and np.array_equal(gd, od), \
            (k, diff_report(gk, gd, ok, od))
        _, pk6, pd = okp[k - 1]
        on, om, ob, os_ = oracle.match_bf(pd, pk6[:, 3].astype(np.float32), od, ok6[:, 3].astype(np.float32),
                                          50, 0.9, True)
        assert int(v["nmatch"][0]) == on, k
        assert np.array_equal(v["match"][:cq].cpu().numpy(), om), k


def test_frontend_first_frame_and_misuse():
    import torch
    from orb_slam3_ros2_amd import FrameStream, OrbHipError
    from orb_slam3_ros2_amd.synthetic import synthetic_stream
    frames = torch.from_numpy(synthetic_stream(2, 640, 480, 3)).to("cuda")
    fs = FrameStream(640, 480, 2)
    with pytest.raises(OrbHipError):
        fs.wait(0)                      # nothing pushed yet
    s0 = fs.push(frames[0])
    fs.wait(s0)
    v = fs.view(s0)
    assert v["frame"] == 0 and int(v["nmatch"][0]) == -1 and int(v["n"][0]) > 500
    with pytest.raises(OrbHipError):
        fs.view(fs.slots)
    from orb_slam3_ros2_amd._lib import lib
    assert lib().orbhip_frontend_push(fs.handle, frames[1].data_ptr(), 639, 0, 1000) < 0   # stride < w
    st = torch.cuda.Stream()
    s1 = fs.push(frames[1])
    fs.wait(s1, stream=st)              # stream-ordered form
    st.synchronize()
    assert int(fs.view(s1)["nmatch"][0]) > 100
    fs.close()

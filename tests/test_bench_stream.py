"""The bench's pipelined C2 stream (frames of one camera stream in flight on several contexts /
streams with event hand-offs) produces exactly the sequential per-frame results. The stream
cycles through 32 frames, so from frame 32 on every call repeats an earlier one and, with
ORBHIP_GRAPH=1, runs as a launch-graph replay; the reference runs on the HIP null stream with
every kernel launched directly."""
import numpy as np
import pytest

from tests.helpers import oracle_kps_to_struct
from orb_slam3_ros2_amd._lib import KP_DTYPE


@pytest.mark.gpu
@pytest.mark.parametrize("graphs", [False, True])
def test_pipelined_stream_matches_sequential(monkeypatch, graphs, oracle):
    import torch
    import bench
    K = 75
    seq = bench.StreamC2(0, 1, null_stream=True)   # built before the switch: direct launches
    ref = []
    for _ in range(K):
        seq.step()
        torch.cuda.synchronize()
        cur = (seq.s - 1) % seq.ns
        ref.append((int(seq.n[cur]), seq.kps[cur].clone(), seq.desc[cur].clone(), int(seq.nm[cur]),
                    seq.mm[cur].clone()))
    # the sequential reference itself against the oracle (every stream frame of the last cycle)
    okp = {}
    for k in range(K - 9, K):
        okp[k] = oracle.extract(seq.frames_np[k % seq.NF])
    for k in range(K - 8, K):
        n, kps, desc, nm, mm = ref[k]
        _, ok6, od = okp[k]
        gk = np.frombuffer(kps[:n].cpu().numpy().tobytes(), KP_DTYPE)
        assert np.array_equal(gk, oracle_kps_to_struct(ok6)) and np.array_equal(desc[:n].cpu().numpy(), od), k
        _, pk6, pd = okp[k - 1]
        on, om, ob, os_ = oracle.match_bf(pd, pk6[:, 3].astype(np.float32), od, ok6[:, 3].astype(np.float32),
                                          50, 0.9, True)
        assert nm == on and np.array_equal(mm[0, :len(om)].cpu().numpy(), om), k
    if graphs:
        monkeypatch.setenv("ORBHIP_GRAPH", "1")
    for S in (1, 2, 4):
        pip = bench.StreamC2(0, S)
        for _ in range(K):
            pip.step()
        torch.cuda.synchronize()
        assert all((pip.L.orbhip_launch_graphs(h) > 0) == graphs for h in pip.handles), S
        for k in range(K - pip.ns, K):   # the frames still held in the slots
            slot = k % pip.ns
            n, kps, desc, nm, mm = ref[k]
            assert int(pip.n[slot]) == n and int(pip.nm[slot]) == nm, (S, k)
            assert torch.equal(pip.kps[slot, :n], kps[:n]) and torch.equal(pip.desc[slot, :n], desc[:n]), (S, k)
            nq = ref[k - 1][0]   # the match's queries are the previous frame's keypoints
            assert torch.equal(pip.mm[slot, :, :nq], mm[:, :nq]), (S, k)

"""The bench's pipelined C2 stream (frames of one camera stream in flight on several contexts /
streams with event hand-offs) produces exactly the sequential per-frame results."""
import numpy as np
import pytest


@pytest.mark.gpu
def test_pipelined_stream_matches_sequential():
    import torch
    import bench
    K = 23
    seq = bench.StreamC2(0, 1)
    ref = []
    for _ in range(K):
        seq.step()
        torch.cuda.synchronize()
        cur = (seq.s - 1) % seq.ns
        ref.append((int(seq.n[cur]), seq.kps[cur].clone(), seq.desc[cur].clone(), int(seq.nm[cur]),
                    seq.mm[cur].clone()))
    for S in (2, 4):
        pip = bench.StreamC2(0, S)
        for _ in range(K):
            pip.step()
        torch.cuda.synchronize()
        for k in range(K - pip.ns, K):   # the frames still held in the slots
            slot = k % pip.ns
            n, kps, desc, nm, mm = ref[k]
            assert int(pip.n[slot]) == n and int(pip.nm[slot]) == nm, (S, k)
            assert torch.equal(pip.kps[slot, :n], kps[:n]) and torch.equal(pip.desc[slot, :n], desc[:n]), (S, k)
            nq = ref[k - 1][0]   # the match's queries are the previous frame's keypoints
            assert torch.equal(pip.mm[slot, :, :nq], mm[:, :nq]), (S, k)

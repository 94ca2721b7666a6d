"""a23 ingest: bgr8 -> gray (cv_bridge MONO8 = cvtColor BGR2GRAY, bit-exact) on the device,
then ORB extraction, against the oracle restatement of the same two steps."""
import numpy as np
import pytest

from orb_slam3_ros2_amd.synthetic import synthetic_frame


def _bgr(seed, w, h):
    rng = np.random.Generator(np.random.PCG64(seed))
    g = synthetic_frame(seed, w, h).astype(np.int32)
    tint = rng.integers(-40, 41, size=3)
    noise = rng.integers(-6, 7, size=(h, w, 3))
    return np.clip(g[:, :, None] + tint[None, None, :] + noise, 0, 255).astype(np.uint8)


def test_oracle_bgr2gray_known_answers(oracle):
    px = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [10, 20, 30]]], np.uint8)
    g = oracle.bgr2gray(px)[0]
    exp = [(b * 1868 + gg * 9617 + r * 4899 + 8192) >> 14 for b, gg, r in px[0].astype(int)]
    assert g.tolist() == exp == [29, 150, 76, 255, 0, 22]


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(640, 480), (1920, 1080), (641, 479), (17, 5)])
def test_gpu_bgr2gray_bit_exact(oracle, w, h):
    import torch
    from orb_slam3_ros2_amd import ORBextractor
    from orb_slam3_ros2_amd.ingest import bgr_to_gray_device
    ext = ORBextractor()
    bgr = _bgr(3, w, h)
    g = bgr_to_gray_device(ext.ctx, torch.from_numpy(bgr).cuda())
    torch.cuda.synchronize()
    assert np.array_equal(g.cpu().numpy(), oracle.bgr2gray(bgr))


@pytest.mark.gpu
def test_gpu_bgr2gray_batched_padded(oracle):
    import torch
    from orb_slam3_ros2_amd import ORBextractor
    from orb_slam3_ros2_amd.ingest import bgr_to_gray_device
    ext = ORBextractor()
    frames = np.stack([_bgr(s, 320, 240) for s in range(3)])
    big = torch.zeros((3, 240, 336, 3), dtype=torch.uint8, device="cuda")   # padded rows
    big[:, :, :320] = torch.from_numpy(frames).cuda()
    g = bgr_to_gray_device(ext.ctx, big[:, :, :320])
    torch.cuda.synchronize()
    for i in range(3):
        assert np.array_equal(g[i].cpu().numpy(), oracle.bgr2gray(frames[i]))


@pytest.mark.gpu
def test_mono_ingest_end_to_end(oracle):
    from orb_slam3_ros2_amd.ingest import MonoIngest
    from tests.helpers import oracle_kps_to_struct
    bgr = _bgr(8, 640, 480)
    ing = MonoIngest(640, 480)
    kps, desc, n, mono = ing(bgr)
    nk = int(n.item())          # no device-wide synchronize: stream ordering must suffice
    omono, ok6, od = oracle.extract(oracle.bgr2gray(bgr))
    ok = oracle_kps_to_struct(ok6)
    gk = kps[:nk].cpu().numpy().view(np.float32)
    assert int(mono.item()) == omono and nk == len(ok)
    assert np.array_equal(gk[:, 0], ok["x"]) and np.array_equal(gk[:, 3], ok["angle"])
    assert np.array_equal(desc[:nk].cpu().numpy(), od)

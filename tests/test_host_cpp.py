"""The C++ host mirror (include/orbhip.hpp) driven by a compiled program, as the reference's
C++ host would call it: golden frame -> ORBextractor::operator() bit-exact; golden BA problem
-> Optimizer::LocalBundleAdjustment within 1e-4. The program is built by build() /
tests/cpp/Makefile; the CPU test only checks that it compiles and links against the C-ABI."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CPP = os.path.join(ROOT, "tests", "cpp")
EXE = os.path.join(CPP, "build", "host_adapter_check")
GOLD = os.path.join(ROOT, "tests", "golden")


def _build():
    subprocess.check_call(["make", "-s", "-C", CPP])
    assert os.path.exists(EXE)


def test_host_adapter_compiles_and_links():
    _build()


def _unpack(d):
    z = np.load(os.path.join(GOLD, "frame_320x240_s5.npz"))
    z["image"].astype(np.uint8).tofile(os.path.join(d, "image.u8"))
    np.array([z["w"], z["h"], z["nfeatures"], z["lap"][0], z["lap"][1], z["mono"], len(z["kps"])],
             np.int32).tofile(os.path.join(d, "meta.i32"))
    z["kps"].astype(np.float32).tofile(os.path.join(d, "kps.f32"))
    z["desc"].astype(np.uint8).tofile(os.path.join(d, "desc.u8"))
    b = np.load(os.path.join(GOLD, "ba_10kf_200pt_s21.npz"))
    np.array(list(b["cam"]) + [float(b["huber_delta"]), float(b["iterations"])], np.float32).tofile(
        os.path.join(d, "ba_meta.f32"))
    for k, ext, dt in [("pose_q", "f32", np.float32), ("pose_t", "f32", np.float32), ("pose_fixed", "u8", np.uint8),
                       ("points", "f32", np.float32), ("edge_pose", "i32", np.int32), ("edge_point", "i32", np.int32),
                       ("edge_uv", "f32", np.float32), ("edge_octave", "i32", np.int32),
                       ("inv_sigma2", "f32", np.float32)]:
        np.ascontiguousarray(b[k], dt).tofile(os.path.join(d, f"ba_{k}.{ext}"))
    b["out_pose_t"].astype(np.float32).tofile(os.path.join(d, "ba_out_pose_t.f32"))
    b["out_points"].astype(np.float32).tofile(os.path.join(d, "ba_out_points.f32"))
    b["out_chi2"].astype(np.float64).tofile(os.path.join(d, "ba_out_meta.f64"))


@pytest.mark.gpu
def test_host_adapter_on_gpu(tmp_path):
    if not os.path.exists(EXE):
        _build()
    _unpack(str(tmp_path))
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.join(ROOT, "orb_slam3_ros2_amd") + ":" +
               os.environ.get("LD_LIBRARY_PATH", ""))
    r = subprocess.run([EXE, str(tmp_path)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host adapter OK" in r.stdout

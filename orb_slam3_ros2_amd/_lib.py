"""ctypes binding of liborbhip.so (include/orbhip.h). Fails loudly when the library is absent."""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_NAME = "liborbhip.so"
_lib = None


class OrbHipError(RuntimeError):
    CODES = {-1: "ORBHIP_ERR_ARG", -2: "ORBHIP_ERR_CAPACITY", -3: "ORBHIP_ERR_DEVICE", -4: "ORBHIP_ERR_NOT_PD",
             -5: "ORBHIP_ERR_UNSUPPORTED", -6: "ORBHIP_ERR_EMPTY", -7: "ORBHIP_ERR_TIMEOUT"}

    def __init__(self, code: int, what: str = ""):
        self.code = code
        super().__init__(f"{what}: {self.CODES.get(code, code)}")


def library_path() -> str:
    # ORBHIP_LIB: an A/B build of the same library (tools/build_ab.sh); default the in-tree build
    return os.environ.get("ORBHIP_LIB") or os.path.join(_HERE, _LIB_NAME)


class KP(ctypes.Structure):
    _fields_ = [("x", ctypes.c_float), ("y", ctypes.c_float), ("size", ctypes.c_float), ("angle", ctypes.c_float),
                ("response", ctypes.c_float), ("octave", ctypes.c_int32)]


KP_DTYPE = np.dtype([("x", np.float32), ("y", np.float32), ("size", np.float32), ("angle", np.float32),
                     ("response", np.float32), ("octave", np.int32)])


class OrbParams(ctypes.Structure):
    _fields_ = [("n_features", ctypes.c_int32), ("scale_factor", ctypes.c_float), ("n_levels", ctypes.c_int32),
                ("ini_th_fast", ctypes.c_int32), ("min_th_fast", ctypes.c_int32)]


class BAProblemC(ctypes.Structure):
    _fields_ = [("n_poses", ctypes.c_int32), ("n_points", ctypes.c_int32), ("n_edges", ctypes.c_int32),
                ("pose_q", ctypes.c_void_p), ("pose_t", ctypes.c_void_p), ("pose_fixed", ctypes.c_void_p),
                ("points", ctypes.c_void_p), ("edge_pose", ctypes.c_void_p), ("edge_point", ctypes.c_void_p),
                ("edge_uv", ctypes.c_void_p), ("edge_octave", ctypes.c_void_p), ("inv_sigma2", ctypes.c_void_p),
                ("n_octaves", ctypes.c_int32), ("fx", ctypes.c_float), ("fy", ctypes.c_float),
                ("cx", ctypes.c_float), ("cy", ctypes.c_float), ("huber_delta", ctypes.c_float),
                ("iterations", ctypes.c_int32), ("early_stop", ctypes.c_int32)]


class BAResultC(ctypes.Structure):
    _fields_ = [("pose_q", ctypes.c_void_p), ("pose_t", ctypes.c_void_p), ("points", ctypes.c_void_p),
                ("edge_chi2", ctypes.c_void_p), ("edge_depth_ok", ctypes.c_void_p),
                ("initial_chi2", ctypes.c_double), ("final_chi2", ctypes.c_double),
                ("iterations_done", ctypes.c_int32), ("lm_trials", ctypes.c_int32)]


class PoseProblemC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("pose_q", ctypes.c_void_p), ("pose_t", ctypes.c_void_p),
                ("points", ctypes.c_void_p), ("uv", ctypes.c_void_p), ("octave", ctypes.c_void_p),
                ("inv_sigma2", ctypes.c_void_p), ("n_octaves", ctypes.c_int32), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float)]


class PoseResultC(ctypes.Structure):
    _fields_ = [("pose_q", ctypes.c_float * 4), ("pose_t", ctypes.c_float * 3), ("outlier", ctypes.c_void_p),
                ("n_inliers", ctypes.c_int32), ("lm_trials", ctypes.c_int32)]


class PinholeC(ctypes.Structure):
    _fields_ = [("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("k1", ctypes.c_float), ("k2", ctypes.c_float), ("p1", ctypes.c_float), ("p2", ctypes.c_float),
                ("k3", ctypes.c_float)]


class FrameC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("claimed", ctypes.c_void_p),
                ("min_x", ctypes.c_float), ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float),
                ("scale_factors", ctypes.c_void_p), ("n_levels", ctypes.c_int32), ("log_scale_factor", ctypes.c_float),
                ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("pose_q", ctypes.c_float * 4), ("pose_t", ctypes.c_float * 3)]


class ProjLastC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("points", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("octave", ctypes.c_void_p), ("angle", ctypes.c_void_p)]


class InitFrameC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("kps", ctypes.c_void_p), ("desc", ctypes.c_void_p), ("min_x", ctypes.c_float),
                ("max_x", ctypes.c_float), ("min_y", ctypes.c_float), ("max_y", ctypes.c_float)]


class KfdbQueryC(ctypes.Structure):
    _fields_ = [("query_id", ctypes.c_int64), ("words", ctypes.c_void_p), ("values", ctypes.c_void_p),
                ("n", ctypes.c_int32), ("covis", ctypes.c_void_p), ("kf_map", ctypes.c_void_p),
                ("query_map", ctypes.c_int32), ("kf_flags", ctypes.c_void_p)]


class LocalPointsC(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("points", ctypes.c_void_p), ("normals", ctypes.c_void_p),
                ("min_dist", ctypes.c_void_p), ("max_dist", ctypes.c_void_p), ("desc", ctypes.c_void_p),
                ("skip", ctypes.c_void_p)]


# every symbol include/orbhip.h declares (tests check the export table against this list)
EXPORTED = ["orbhip_abi_version", "orbhip_create", "orbhip_destroy", "orbhip_level_info", "orbhip_max_keypoints",
            "orbhip_extract", "orbhip_extract_batch_device", "orbhip_descriptor_distance", "orbhip_match_bf",
            "orbhip_match_pairs_device", "orbhip_match_frames_device", "orbhip_profile_stage",
            "orbhip_profile_collect", "orbhip_launch_graphs", "orbhip_ba_solve", "orbhip_ba_solve_batch", "orbhip_ba_stats", "orbhip_bgr_to_gray_device",
            "orbhip_comm_unique_id", "orbhip_comm_init", "orbhip_ba_solve_sharded", "orbhip_ba_solve_sharded_segments",
            "orbhip_ba_solve_shards_local",
            "orbhip_vocab_create", "orbhip_vocab_load_text", "orbhip_vocab_destroy", "orbhip_vocab_info",
            "orbhip_bow_transform", "orbhip_bow_transform_device", "orbhip_search_bow",
            "orbhip_pose_optimization", "orbhip_pose_optimization_batch", "orbhip_search_by_projection_last",
            "orbhip_search_local_points", "orbhip_search_for_initialization",
            "orbhip_kfdb_create", "orbhip_kfdb_destroy", "orbhip_kfdb_add", "orbhip_kfdb_erase",
            "orbhip_kfdb_detect_relocalization", "orbhip_kfdb_detect_nbest",
            "orbhip_frontend_create", "orbhip_frontend_destroy", "orbhip_frontend_push", "orbhip_frontend_view",
            "orbhip_frontend_wait", "orbhip_frontend_context", "orbhip_undistort_keypoints",
            "orbhip_undistort_keypoints_device", "orbhip_image_bounds"]


def lib():
    """Load liborbhip.so (raises if it was not built — there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    path = library_path()
    # torch-ROCm bundles its own libamdhip64.so.7 (same SONAME as /opt/rocm's). Load it first
    # so liborbhip binds to the SAME HIP runtime: device pointers from torch tensors are then
    # valid in our kernels, and torch does not fail to initialise a second runtime.
    try:
        import torch  # noqa: F401
    except Exception:
        pass
    if not os.path.exists(path):
        raise OrbHipError(-3, f"{path} missing — run __graft_entry__.build()")
    L = ctypes.CDLL(path)
    vp, i32, f32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    L.orbhip_abi_version.restype = i32
    L.orbhip_create.argtypes = [ctypes.POINTER(vp), i32, ctypes.POINTER(OrbParams)]
    L.orbhip_destroy.argtypes = [vp]
    L.orbhip_level_info.argtypes = [vp, i32, i32, vp, vp, vp, vp]
    L.orbhip_max_keypoints.argtypes = [vp, i32, i32]
    L.orbhip_extract.argtypes = [vp, vp, i32, i32, i32, i32, i32, vp, vp, i32, ctypes.POINTER(i32),
                                 ctypes.POINTER(i32)]
    L.orbhip_extract_batch_device.argtypes = [vp, vp, i32, i32, i32, i32, ctypes.c_int64, i32, i32, vp, vp, i32,
                                              vp, vp, vp]
    L.orbhip_descriptor_distance.argtypes = [vp, vp]
    L.orbhip_match_bf.argtypes = [vp, vp, vp, i32, vp, vp, i32, i32, f32, i32, vp, vp, vp]
    L.orbhip_match_pairs_device.argtypes = [vp, vp, vp, vp, i32, i32, i32, f32, i32, vp, vp, vp, vp, vp]
    L.orbhip_match_frames_device.argtypes = [vp, vp, vp, vp, vp, vp, vp, i32, i32, f32, i32, vp, vp, vp, vp, vp]
    L.orbhip_vocab_create.argtypes = [vp, i32, i32, i32, i32, i32, vp, vp, vp, vp, ctypes.POINTER(vp)]
    L.orbhip_vocab_load_text.argtypes = [vp, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.orbhip_vocab_destroy.argtypes = [vp]
    L.orbhip_vocab_info.argtypes = [vp, vp, vp, vp, vp]
    L.orbhip_bow_transform.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp]
    L.orbhip_bow_transform_device.argtypes = [vp, vp, vp, vp, i32, i32, i32, vp, vp, vp, vp]
    L.orbhip_search_bow.argtypes = [vp, vp, vp, vp, vp, vp, i32, vp, vp, vp, vp, i32, f32, i32, i32, vp]
    L.orbhip_comm_unique_id.argtypes = [vp]
    L.orbhip_comm_init.argtypes = [vp, i32, i32, vp]
    L.orbhip_ba_solve_sharded.argtypes = [vp, ctypes.POINTER(BAProblemC), ctypes.POINTER(BAResultC), vp]
    L.orbhip_ba_solve_sharded_segments.argtypes = [vp, ctypes.POINTER(BAProblemC), i32, ctypes.POINTER(BAResultC), vp]
    L.orbhip_ba_solve_shards_local.argtypes = [vp, ctypes.POINTER(BAProblemC), i32, ctypes.POINTER(BAResultC), vp]
    L.orbhip_bgr_to_gray_device.argtypes = [vp, vp, i32, i32, i32, i32, ctypes.c_int64, vp, i32, ctypes.c_int64, vp]
    L.orbhip_profile_stage.argtypes = [vp, i32]
    L.orbhip_profile_collect.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int32)]
    L.orbhip_launch_graphs.argtypes = [vp]
    L.orbhip_ba_solve.argtypes = [vp, ctypes.POINTER(BAProblemC), ctypes.POINTER(BAResultC), vp]
    L.orbhip_ba_solve_batch.argtypes = [vp, ctypes.POINTER(BAProblemC), i32, ctypes.POINTER(BAResultC), vp]
    L.orbhip_ba_stats.argtypes = [vp, vp]
    L.orbhip_pose_optimization.argtypes = [vp, ctypes.POINTER(PoseProblemC), ctypes.POINTER(PoseResultC)]
    L.orbhip_pose_optimization_batch.argtypes = [vp, ctypes.POINTER(PoseProblemC), i32, ctypes.POINTER(PoseResultC)]
    L.orbhip_search_by_projection_last.argtypes = [vp, ctypes.POINTER(FrameC), ctypes.POINTER(ProjLastC), f32, i32,
                                                   vp]
    L.orbhip_search_local_points.argtypes = [vp, ctypes.POINTER(FrameC), ctypes.POINTER(LocalPointsC), f32, f32, f32,
                                             i32, f32, vp, vp, vp]
    L.orbhip_search_for_initialization.argtypes = [vp, ctypes.POINTER(InitFrameC), ctypes.POINTER(InitFrameC), vp,
                                                   i32, f32, i32, vp]
    L.orbhip_kfdb_create.argtypes = [vp, i32, ctypes.POINTER(vp)]
    L.orbhip_kfdb_destroy.argtypes = [vp]
    L.orbhip_kfdb_add.argtypes = [vp, i32, vp, vp, i32]
    L.orbhip_kfdb_erase.argtypes = [vp, i32]
    L.orbhip_kfdb_detect_relocalization.argtypes = [vp, ctypes.POINTER(KfdbQueryC), vp, i32]
    L.orbhip_kfdb_detect_nbest.argtypes = [vp, ctypes.POINTER(KfdbQueryC), vp, i32, vp, vp, vp, vp]
    L.orbhip_frontend_create.argtypes = [ctypes.POINTER(vp), i32, ctypes.POINTER(OrbParams), i32, i32, i32, i32, f32,
                                         i32]
    L.orbhip_frontend_destroy.argtypes = [vp]
    L.orbhip_frontend_push.argtypes = [vp, vp, i32, i32, i32]
    L.orbhip_frontend_view.argtypes = [vp, i32, vp]
    L.orbhip_frontend_wait.argtypes = [vp, i32, vp]
    L.orbhip_frontend_context.argtypes = [vp, i32, ctypes.POINTER(vp)]
    L.orbhip_undistort_keypoints.argtypes = [vp, ctypes.POINTER(PinholeC), vp, i32, vp]
    L.orbhip_undistort_keypoints_device.argtypes = [vp, ctypes.POINTER(PinholeC), vp, vp, i32, i32, vp, vp]
    L.orbhip_image_bounds.argtypes = [vp, ctypes.POINTER(PinholeC), i32, i32, vp]
    L.orbhip_test_sincosf.argtypes = [vp, vp, vp, ctypes.c_int64]
    L.orbhip_test_sincosf_sweep.argtypes = [ctypes.c_uint32, ctypes.c_uint32, vp, vp]
    L.orbhip_test_sincosf_sweep.restype = ctypes.c_int64
    # measurement hooks of the dense Cholesky (HIP events around back-to-back launches)
    L.orbhip_test_cholesky_reg.argtypes = [vp, vp, vp, i32, i32, ctypes.POINTER(f32), vp]
    L.orbhip_test_cholesky_blocked.argtypes = [vp, vp, vp, i32, ctypes.POINTER(f32)]
    L.orbhip_test_cholesky_dag.argtypes = [vp, vp, vp, i32, i32, i32, ctypes.POINTER(f32), vp]
    _lib = L
    return L


def torch_stream(stream=None):
    """hipStream_t for a device call on torch tensors: the given torch stream, else torch's
    CURRENT stream (handle 0 = the HIP null stream, which the ABI takes as such) — so the call
    is ordered after the torch work that produced its inputs and before torch reads its
    outputs."""
    import torch
    s = stream if stream is not None else torch.cuda.current_stream()
    return ctypes.c_void_p(s.cuda_stream)


def check(rc: int, what: str) -> int:
    if rc < 0:
        raise OrbHipError(rc, what)
    return rc


def ptr(a) -> int | None:
    """Data pointer of a numpy array or a torch tensor (host or device)."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        # (the array interface, not a.ctypes: building that object cost ~3 us per pointer, ~14 per
        # BA call)
        return a.__array_interface__["data"][0]
    return a.data_ptr()


class Context:
    """Owns one orbhip_ctx (device memory, pinned staging, one HIP stream). device < 0 (the default):
    the calling thread's current HIP device, i.e. the rank's GPU after torch.cuda.set_device."""

    def __init__(self, device: int = -1, n_features=1000, scale_factor=1.2, n_levels=8, ini_th_fast=20,
                 min_th_fast=7):
        self._h = ctypes.c_void_p()
        prm = OrbParams(int(n_features), float(scale_factor), int(n_levels), int(ini_th_fast), int(min_th_fast))
        check(lib().orbhip_create(ctypes.byref(self._h), int(device), ctypes.byref(prm)), "orbhip_create")

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().orbhip_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

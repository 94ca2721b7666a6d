"""C-ABI contract on the CPU (no GPU here): liborbhip.so exists, loads, exports every entry
point include/orbhip.h declares, and fails loudly (ORBHIP_ERR_DEVICE) when no device is
present — there is no CPU fallback behind the boundary. No compute calls are made."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "orbhip.h")).read()
    return sorted(set(re.findall(r"^\s*int\s+(orbhip_\w+)\s*\(", src, re.M)))


def test_header_declares_the_boundary():
    names = _declared()
    for n in ["orbhip_create", "orbhip_destroy", "orbhip_extract", "orbhip_extract_batch_device",
              "orbhip_descriptor_distance", "orbhip_match_bf", "orbhip_ba_solve", "orbhip_ba_solve_batch"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from orb_slam3_ros2_amd import _lib
    L = _lib.lib()
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    assert sorted(_lib.EXPORTED) == _declared()
    assert L.orbhip_abi_version() == 1


def test_no_oracle_linkage():
    """The product library never links or names the oracle."""
    so = open(os.path.join(ROOT, "orb_slam3_ros2_amd", "liborbhip.so"), "rb").read()
    assert b"orb_oracle" not in so and b"orc_extract" not in so


def test_gfx950_code_object_embedded():
    so = open(os.path.join(ROOT, "orb_slam3_ros2_amd", "liborbhip.so"), "rb").read()
    assert b"gfx950" in so


def test_descriptor_distance_host_helper():
    from orb_slam3_ros2_amd import _lib
    L = _lib.lib()
    a = (ctypes.c_uint8 * 32)(*([0xFF] * 32))
    b = (ctypes.c_uint8 * 32)(*([0x0F] * 32))
    assert L.orbhip_descriptor_distance(a, b) == 128


def test_create_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from orb_slam3_ros2_amd import _lib
    h = ctypes.c_void_p()
    rc = _lib.lib().orbhip_create(ctypes.byref(h), 0, None)
    assert rc == -3 and not h.value
    with pytest.raises(_lib.OrbHipError):
        _lib.Context(0)
    with pytest.raises(_lib.OrbHipError):
        _lib.Context()   # device < 0: the current device, none here either


@pytest.mark.gpu
def test_context_on_the_current_device():
    """device < 0 (the Python default) resolves to the calling thread's current HIP device, so a
    rank of a one-process-per-GPU job (torch.cuda.set_device(LOCAL_RANK)) computes on its own GPU;
    an ordinal past the last device fails loudly."""
    import torch
    from orb_slam3_ros2_amd import _lib
    torch.cuda.set_device(torch.cuda.device_count() - 1)
    h = ctypes.c_void_p()
    assert _lib.lib().orbhip_create(ctypes.byref(h), -1, None) == 0 and h.value
    assert _lib.lib().orbhip_destroy(h) == 0
    assert _lib.lib().orbhip_create(ctypes.byref(h), torch.cuda.device_count(), None) == -3
    torch.cuda.set_device(0)

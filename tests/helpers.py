"""Shared test helpers: compare product keypoints/descriptors with the oracle's."""
import numpy as np

from orb_slam3_ros2_amd._lib import KP_DTYPE


def oracle_kps_to_struct(k6: np.ndarray) -> np.ndarray:
    out = np.zeros(k6.shape[0], KP_DTYPE)
    for i, f in enumerate(["x", "y", "size", "angle", "response"]):
        out[f] = k6[:, i]
    out["octave"] = k6[:, 5].astype(np.int32)
    return out


def diff_report(gk, gd, ok, od, max_lines=10) -> str:
    lines = [f"n gpu={len(gk)} oracle={len(ok)}"]
    n = min(len(gk), len(ok))
    for f in KP_DTYPE.names:
        bad = np.nonzero(gk[f][:n] != ok[f][:n])[0]
        if len(bad):
            lines.append(f"field {f}: {len(bad)} mismatches, first idx {bad[:5].tolist()}")
    if gd is not None and od is not None:
        bad = np.nonzero(np.any(gd[:n] != od[:n], axis=1))[0]
        if len(bad):
            lines.append(f"desc: {len(bad)} rows differ, first {bad[:5].tolist()}")
    for i in range(min(n, max_lines)):
        if any(gk[f][i] != ok[f][i] for f in KP_DTYPE.names):
            lines.append(f"  [{i}] gpu={gk[i]} oracle={ok[i]}")
    return "\n".join(lines)

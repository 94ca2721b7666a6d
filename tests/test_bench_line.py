"""The bench's printed line (CPU only): the driver keeps the last ~4 KB of stdout, so the line
must carry every figure (C2 headline, C3, C4, C5, 8f, CPU baseline) in well under that; the
headline roofline's bytes follow SURVEY.md §8(d); the sharded-C5 parity check flags a mismatch."""
import json
from types import SimpleNamespace

import numpy as np

import bench


def _full_record():
    counters = {f"SQ_{i}": float(i) for i in range(40)}
    return {
        "metric": "m", "value": 40000.0, "unit": "frames/s", "n_gpus": 1, "steps": 20, "warmup": 5,
        "ms_per_step": 0.39, "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": "synthetic", "batch1_frames_per_s": 17000.0, "batch1_latency_ms": 0.058,
        "config": {"workload": "C2", "step": "s", "frames_per_step": 16, "parallelism": "p", "cameras": 16,
                   "host_submit_ms_per_frame": 0.01, "keypoints_per_frame": 1000.0},
        "roofline": {"kernel": "k_pyr_cone", "bound": "latency", "achieved": 76.6, "peak": 8000.0, "unit": "GB/s",
                     "frac": 0.0096, "traffic": 2443062, "counters": counters,
                     "algorithmic_bytes_per_launch": 1649864, "avg_launch_ms": 0.0215,
                     "stage_avg_ms": {str(i): 0.01 for i in range(6)}},
        "extra": {"c5_gba_ms": 5.5, "c5_problem": "x" * 200, "c3_1280x720_b64_extract_match_frames_per_s": 96000.0,
                  "c3_roofline": {"kernel": "k_fast_cells", "bound": "valu issue", "frac": 0.46,
                                  "avg_launch_ms": 0.35, "counters": counters},
                  "c4_lba_ms": 1.5, "c4_roofline": {"kernel": "k_chol_dag", "frac": 0.0014, "counters": counters},
                  "c5_nd_roofline": {"frac": 0.006, "avg_solve_ms": 0.3, "counters": {"k": counters}},
                  "f8_inputs": "y" * 300},
        "cpu_baseline": {"value": 1180.0, "unit": "frames/s", "cores": 16, "kind": "port", "sample": "z" * 300,
                         "host": {"model": "EPYC", "nproc": 256}, "c4_lba_kf_per_s": 770.0,
                         "c4_lba_sample": "w" * 100},
    }


def test_compact_line_keeps_figures_and_fits_the_tail():
    full = _full_record()
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) < 3000
    assert "counters" not in s
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in line
    ex = line["extra"]
    assert ex["c5_gba_ms"] == 5.5 and ex["c4_lba_ms"] == 1.5
    assert ex["c3_1280x720_b64_extract_match_frames_per_s"] == 96000.0
    assert ex["c3_roofline"]["frac"] == 0.46 and ex["c5_nd_roofline"]["avg_solve_ms"] == 0.3
    rf = line["roofline"]
    assert rf["frac"] == 0.0096 and rf["traffic"] == 2443062
    cb = line["cpu_baseline"]
    assert cb["value"] == 1180.0 and cb["cores"] == 16 and cb["kind"] == "port" and cb["c4_lba_kf_per_s"] == 770.0


def test_survey_frame_bytes_c2():
    """1,649,864 B per 640x480 frame at N = 1000 (the level areas of the
    ORBextractor ctor tables, checked against the oracle's own level geometry)."""
    from oracle import pyoracle as O

    class Ext:
        def level_info(self, w, h):
            return O.level_info(w, h)

    assert bench.survey_frame_bytes(Ext(), 640, 480, 1000) == 1649864


def test_c5_sharded_parity_flags():
    def res(scale=1.0, trials=10):
        return SimpleNamespace(final_chi2=100.0 * scale, pose_q=np.ones((4, 4)) * scale, pose_t=np.ones((4, 3)),
                               points=np.ones((5, 3)), iterations_done=10, lm_trials=trials)
    sel = np.arange(5)
    full = res()
    full.points = np.ones((9, 3))
    assert bench.c5_sharded_parity(1, res(), full, sel)["c5_sharded_parity"]
    assert not bench.c5_sharded_parity(1, res(1.001), full, sel)["c5_sharded_parity"]
    bad = bench.c5_sharded_parity(1, res(trials=11), full, sel)
    assert not bad["c5_sharded_parity"] and not bad["c5_sharded_schedule_equal"]

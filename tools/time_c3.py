#!/usr/bin/env python3
"""C3 alone (bench.c3_batch: 1280x720 B=64 extract + 63 pair matches, 8 batches in flight and one at
a time), for A/B of extractor builds (ORBHIP_LIB=tools/ubench/ab/liborbhip_<name>.so)."""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

args = types.SimpleNamespace(c3_steps=int(sys.argv[1]) if len(sys.argv) > 1 else 10, c3_inflight=8)
out = bench.c3_batch(args, 1, 0)
print(json.dumps({k: out[k] for k in ("c3_1280x720_b64_extract_match_frames_per_s",
                                       "c3_one_batch_at_a_time_frames_per_s")} |
                 {"fast_ms": out["c3_roofline"]["stage_avg_ms"].get("k_fast_cells"),
                  "lib": os.environ.get("ORBHIP_LIB", "main")}), flush=True)

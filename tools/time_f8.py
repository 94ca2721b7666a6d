#!/usr/bin/env python3
"""The bench's SURVEY 8f per-call latencies alone (bench.f8_tracking, each call's own context), for
A/B runs of the tracking-path host plumbing."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

out = bench.f8_tracking(None)
out.pop("f8_inputs", None)
print(json.dumps(out))

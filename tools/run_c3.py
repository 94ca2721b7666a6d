#!/usr/bin/env python3
"""Run N steps of the C3 workload (1280x720, B=64, extract + 63-pair match) for PMC passes."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5
c3 = bench.BatchC3(0)
for _ in range(n):
    c3.step()
torch.cuda.synchronize()
print("c3 steps", n)

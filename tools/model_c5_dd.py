#!/usr/bin/env python3
"""Measured pieces of the modelled 8-rank C5 step (DESIGN.md §C5 sharding, tests/schur_dd_model.py): the
persistent DAG Cholesky (k_chol_dag, the kernel the LM loop launches) on
  - the full C5-structured system (n = 2400, cyclic 20-KF band: the 1-GPU solve),
  - one rank's local system Z_{r-1} + I_r + Z_r (n = 414, interior first: an upper bound of the
    interior elimination, which stops after the 186 interior columns),
  - the separator system (n = 912, block-tridiagonal cyclic) after the all-reduce.
  - the interior alone (n = 186: the elimination's chain, without the Schur update),
  - the second level on the separator system: a rank's local system (n = 342), its interior
    (n = 114) and the level-2 separator system (n = 456).
Prints one JSON line."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402,F401

from orb_slam3_ros2_amd._lib import lib  # noqa: E402
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from schur_dd_model import Partition, covisibility_system, dd_local, split_assembled  # noqa: E402


def dag_ms(S, reps=20):
    n = S.shape[0]
    b = np.ones(n)
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    rc = lib().orbhip_test_cholesky_dag(np.ascontiguousarray(S).ctypes.data, b.ctypes.data, x.ctypes.data, n, reps,
                                        0, ctypes.byref(ms), None)
    err = float(np.abs(S @ x - b).max())
    return rc, round(ms.value, 4), err


part = Partition(400, 8, 20)
Ss, bs = covisibility_system(part, 20000, seed=3)
S = sum(Ss)
out = {"full_n2400": dag_ms(S)}
r = 3
idx = np.concatenate([part.interior(r), part.adjacent(r)])
out["local_n%d" % idx.size] = dag_ms(S[np.ix_(idx, idx)])
Sz = sum(dd_local(torch.from_numpy(Ss[k]), torch.from_numpy(bs[k]), part, k)[1] for k in range(part.ranks)).numpy()
out["separator_n%d" % Sz.shape[0]] = dag_ms(Sz)
out["interior_n%d" % part.interior(r).size] = dag_ms(S[np.ix_(part.interior(r), part.interior(r))])
# second level: the separator system dissected (odd separators as interiors, 4 ranks)
p2 = Partition(8, 4, 2, dof=part.sep * part.dof)
bz = sum(dd_local(torch.from_numpy(Ss[k]), torch.from_numpy(bs[k]), part, k)[2] for k in range(part.ranks)).numpy()
S2, b2 = split_assembled(Sz, bz, p2)
i2 = np.concatenate([p2.interior(1), p2.adjacent(1)])
out["l2_local_n%d" % i2.size] = dag_ms(Sz[np.ix_(i2, i2)])
out["l2_interior_n%d" % p2.interior(1).size] = dag_ms(Sz[np.ix_(p2.interior(1), p2.interior(1))])
Sz2 = sum(dd_local(torch.from_numpy(S2[k]), torch.from_numpy(b2[k]), p2, k)[1] for k in range(p2.ranks)).numpy()
out["l2_separator_n%d" % Sz2.shape[0]] = dag_ms(Sz2)
out["separator_bytes_dense"] = int(Sz.nbytes)
m = part.sep * part.dof
out["separator_bytes_block_tridiagonal"] = int(part.ranks * 3 * m * m * 8)
print(json.dumps(out))

#!/usr/bin/env python3
"""Probe the persistent tiled-DAG Cholesky (ba_chol_dag.hip) against numpy: dense, banded and
band + loop-corner SPD systems; device us per solve and the chain workgroup's phase cycles
(s_memtime: prologue, forward, backward, poll waits, diag32 sum)."""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from orb_slam3_ros2_amd._lib import lib  # noqa: E402


def spd(n, shape, rng):
    if shape == "dense":
        M = rng.normal(size=(n, n))
        return M @ M.T + n * np.eye(n)
    bw = 120
    M = np.zeros((n, n))
    for i in range(n):
        lo = max(0, i - bw)
        M[i, lo:i + 1] = rng.normal(size=i + 1 - lo)
    if shape == "loop":
        M[n - 120:, :120] = rng.normal(size=(120, 120)) * 0.3
    return M @ M.T + n * np.eye(n)


L = lib()
if os.environ.get("ORBHIP_PROBE_LIB", ""):   # an alternative build of the library (A/B of a compile-time switch)
    L = ctypes.CDLL(os.environ["ORBHIP_PROBE_LIB"])
    L.orbhip_test_cholesky_dag.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3 + [ctypes.c_void_p] * 2
cases = [a.split(":") for a in (sys.argv[1:] or ["31:dense", "100:dense", "294:dense", "600:band", "2394:loop", "2394:dense"])]
for n_s, shape in cases:
    n = int(n_s)
    rng = np.random.default_rng(n)
    A = spd(n, shape, rng)
    A = 0.5 * (A + A.T)
    b = rng.normal(size=n)
    x = np.zeros(n)
    ms = ctypes.c_float(0)
    dbg = np.zeros(8 + 6 * 200 + 16 * 100 + 3 * 128, np.uint64)   # kDbgWords (ba_chol_dag.h)
    t0 = time.time()
    rc = L.orbhip_test_cholesky_dag(A.ctypes.data, b.ctypes.data, x.ctypes.data, n, 10, int(os.environ.get('ORBHIP_DAG_HELPERS', '0')), ctypes.byref(ms),
                                    dbg.ctypes.data)
    ref = np.linalg.solve(A, b)
    err = np.abs(x - ref).max() / np.abs(ref).max()
    nt = (n + 31) // 32
    ki = max(0, min(nt - 1, 200))
    ph = dbg[8:8 + 6 * ki].reshape(ki, 6).astype(np.int64) if ki else np.zeros((1, 6), np.int64)
    med = np.median(ph, axis=0).astype(int) if ki else [0] * 6
    if os.environ.get("ORBHIP_PROBE_SAVE"):   # raw per-interval words for offline analysis
        np.save(os.path.join(os.environ["ORBHIP_PROBE_SAVE"], f"dag_{n}_{shape}.npy"), dbg)
    print(f"n={n} {shape}: rc={rc} dag {ms.value * 1e3:.1f} us relerr={err:.2e} | cycles prologue={dbg[0]} "
          f"forward={dbg[1]} backward={dbg[2]} diag={dbg[4]} total={dbg[5]} (prologue: barrier {dbg[6]}, part A {dbg[7]}) | interval medians: total {med[0]} "
          f"| wave ends {med[0 + 1]} {int(np.median(ph[:, 2] & 0xFFFFFFFF)) if ki else 0} {med[3]} {med[4]} "
          f"w3 flags in {int(np.median(ph[:, 2] >> 32)) if ki else 0} w0 start {int(np.median(ph[:, 5] & 0xFFFFFFFF)) if ki else 0} "
          f"pre-diag {int(np.median(ph[:, 5] >> 32)) if ki else 0} ({time.time() - t0:.1f}s)", flush=True)
    if ki and n <= 600:   # per interval: total cycles and wave 3's wait for the helpers' flags
        print("    intervals (total/flags-in): " + " ".join(f"{int(r[0])}/{int(r[2]) >> 32}" for r in ph), flush=True)
    ks = min(ki, 100)
    if ks:
        sub = dbg[8 + 6 * 200:8 + 6 * 200 + 16 * ks].reshape(ks, 16).astype(np.int64)
        m = np.median(sub, axis=0).astype(int)
        print(f"    sub-phases (median cycles from the interval start): w0 diagA {m[0]} D(1,*) in {m[1]} diagB {m[2]} | "
              f"w2 loads {m[4]} L(k+2,k) {m[5]} T/D' {m[6]} L(k+1,k) in {m[7]} | "
              f"w3 loads {m[8]} L(k+2,k) {m[9]} T/D' {m[10]} L(k+1,k) in {m[11]} | w0 y {m[3]} "
              f"| W23 form: w2 T {m[12]} D' {m[13]} w3 T {m[14]} D' {m[15]}", flush=True)
    nb = min(nt, 128)
    bk = dbg[8 + 6 * 200 + 16 * 100:].reshape(128, 3).astype(np.int64)[:nb]
    if nb > 1 and bk[1:nb, 0].any():
        st = bk[1:nb]
        print("    backward steps t (start, x_{t-1} formed, s_{t-1} complete; cycles from the backward start): " +
              " ".join(f"{R}:{a}/{b}/{c}" for R, (a, b, c) in zip(range(nb - 1, 0, -1), st[::-1][:12])), flush=True)

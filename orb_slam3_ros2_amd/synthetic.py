"""Seeded synthetic inputs — no datasets exist offline.

Images: background 128, 300 axis-aligned rectangles (side U[8,96] px, intensity
U[0,255]) drawn in order, then Gaussian noise sigma=4, rounded and clipped to u8.
numpy PCG64 seeded with the frame index. This gives FAST corners in every 35-px
cell, like a textured indoor scene.
"""
from __future__ import annotations

import numpy as np


def synthetic_frame(seed: int, width: int = 640, height: int = 480, n_rect: int = 300,
                    noise_sigma: float = 4.0) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.full((height, width), 128.0, dtype=np.float64)
    for _ in range(n_rect):
        sw, sh = rng.integers(8, 97, size=2)
        x0 = int(rng.integers(-int(sw) + 1, width))
        y0 = int(rng.integers(-int(sh) + 1, height))
        val = float(rng.integers(0, 256))
        img[max(y0, 0):max(min(y0 + sh, height), 0), max(x0, 0):max(min(x0 + sw, width), 0)] = val
    if noise_sigma > 0:
        img += rng.normal(0.0, noise_sigma, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def synthetic_batch(first_seed: int, batch: int, width: int, height: int) -> np.ndarray:
    return np.stack([synthetic_frame(first_seed + i, width, height) for i in range(batch)])


def shifted_frame(base: np.ndarray, dx: int, dy: int, seed: int, noise_sigma: float = 2.0) -> np.ndarray:
    """A second view of ``base``: integer translation (edge-replicated) plus fresh noise,
    so consecutive frames share most corners (matcher workloads)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    h, w = base.shape
    ys = np.clip(np.arange(h) - dy, 0, h - 1)
    xs = np.clip(np.arange(w) - dx, 0, w - 1)
    img = base[ys][:, xs].astype(np.float64)
    img += rng.normal(0.0, noise_sigma, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)

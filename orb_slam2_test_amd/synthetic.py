"""Seeded synthetic grayscale sequences (SURVEY.md 8d "Synthetic inputs").

There is no network and no dataset in this environment, so benches and tests use
KITTI/TUM-shaped synthetic frames: value-noise texture (4 octaves of bilinearly
up-sampled uniform noise) plus random rectangles and line edges, so FAST finds
corners in every 30-px cell.  Frame t+1 is the same canvas panned by a seeded
(dx, dy) of at most 8 px plus +-2 intensity noise, so frame-to-frame matching has
true correspondences.  Everything is numpy with ``np.random.Generator(PCG64)``.
"""
import numpy as np

DEFAULT_SEED = 20261015


def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float32)
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    return (g00 * (1 - fx) + g01 * fx) * (1 - fy) + (g10 * (1 - fx) + g11 * fx) * fy


def canvas(h, w, seed=DEFAULT_SEED, n_rects=None, n_lines=None):
    """A textured float32 canvas in [0, 255]."""
    rng = np.random.Generator(np.random.PCG64(seed))
    img = np.zeros((h, w), np.float32)
    for cell, amp in ((32, 0.35), (12, 0.25), (5, 0.2), (2, 0.2)):
        img += amp * _value_noise(rng, h, w, cell)
    img = img * 255.0
    area = h * w
    n_rects = n_rects if n_rects is not None else max(8, area // 6000)
    for _ in range(n_rects):
        rh, rw = rng.integers(6, 60, size=2)
        y, x = rng.integers(0, max(1, h - rh)), rng.integers(0, max(1, w - rw))
        img[y:y + rh, x:x + rw] = img[y:y + rh, x:x + rw] * 0.3 + rng.uniform(0, 255) * 0.7
    n_lines = n_lines if n_lines is not None else max(4, area // 20000)
    for _ in range(n_lines):
        if rng.random() < 0.5:
            y = rng.integers(0, h)
            x0, x1 = sorted(rng.integers(0, w, size=2))
            img[y:y + 2, x0:x1] = rng.uniform(0, 255)
        else:
            x = rng.integers(0, w)
            y0, y1 = sorted(rng.integers(0, h, size=2))
            img[y0:y1, x:x + 2] = rng.uniform(0, 255)
    return np.clip(img, 0, 255)


def frame(h, w, seed=DEFAULT_SEED):
    """A single synthetic u8 frame."""
    return np.rint(canvas(h, w, seed)).astype(np.uint8)


def sequence(n, h, w, seed=DEFAULT_SEED, max_step=8, noise=2):
    """n frames (n, h, w) u8 panning over one canvas with seeded (dx, dy) <= max_step."""
    rng = np.random.Generator(np.random.PCG64(seed + 1))
    steps = rng.integers(-max_step, max_step + 1, size=(n, 2))
    steps[0] = 0
    pos = np.cumsum(steps, axis=0)
    pos -= pos.min(axis=0)
    ch = h + int(pos[:, 0].max()) + 1
    cw = w + int(pos[:, 1].max()) + 1
    base = canvas(ch, cw, seed)
    out = np.empty((n, h, w), np.uint8)
    for t in range(n):
        y, x = pos[t]
        crop = base[y:y + h, x:x + w]
        jitter = rng.integers(-noise, noise + 1, size=(h, w)).astype(np.float32)
        out[t] = np.clip(np.rint(crop + jitter), 0, 255).astype(np.uint8)
    return out


def constant(h, w, value=128):
    return np.full((h, w), value, np.uint8)


def pure_noise(h, w, seed=DEFAULT_SEED):
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    return rng.integers(0, 256, size=(h, w), dtype=np.uint8)

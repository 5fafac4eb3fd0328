"""Seeded synthetic inputs (no dataset images exist offline).

Images are u8 planes built from value noise at three octaves, random axis-aligned rectangles and
checker patches (strong FAST corners) and Gaussian noise (sigma ~3), clipped to [0, 255]. A stereo
right image is the left one warped by a smooth per-pixel disparity in [0, 48] px plus independent
noise, so L/R matching (Frame::ComputeStereoMatches, Frame.cc:811-981) finds real correspondences.
Everything is numpy + an explicit seed, so the same call yields the same bytes on every box.
"""
from __future__ import annotations

import numpy as np


def _value_noise(rng: np.random.Generator, h: int, w: int, cell: int) -> np.ndarray:
    gh, gw = h // cell + 2, w // cell + 2
    grid = rng.random((gh, gw), dtype=np.float64)
    ys = np.arange(h) / cell
    xs = np.arange(w) / cell
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    fy = (ys - y0)[:, None]
    fx = (xs - x0)[None, :]
    fy = fy * fy * (3 - 2 * fy)
    fx = fx * fx * (3 - 2 * fx)
    g00 = grid[y0][:, x0]
    g01 = grid[y0][:, x0 + 1]
    g10 = grid[y0 + 1][:, x0]
    g11 = grid[y0 + 1][:, x0 + 1]
    top = g00 * (1 - fx) + g01 * fx
    bot = g10 * (1 - fx) + g11 * fx
    return top * (1 - fy) + bot * fy


def _scene(rng: np.random.Generator, h: int, w: int) -> np.ndarray:
    img = (0.55 * _value_noise(rng, h, w, 64) + 0.3 * _value_noise(rng, h, w, 16)
           + 0.15 * _value_noise(rng, h, w, 4)) * 200.0 + 20.0
    n_rect = max(8, (h * w) // 2500)
    for _ in range(n_rect):
        rh = int(rng.integers(6, 60))
        rw = int(rng.integers(6, 60))
        y = int(rng.integers(0, max(1, h - rh)))
        x = int(rng.integers(0, max(1, w - rw)))
        if rng.random() < 0.3:
            c = int(rng.integers(3, 9))
            yy, xx = np.mgrid[0:rh, 0:rw]
            chk = ((yy // c + xx // c) % 2).astype(np.float64)
            a, b = rng.uniform(0, 255, 2)
            img[y:y + rh, x:x + rw] = a + (b - a) * chk
        else:
            img[y:y + rh, x:x + rw] = rng.uniform(0, 255)
    return img


def synth_image(seed: int, w: int = 752, h: int = 480, noise: float = 3.0) -> np.ndarray:
    """One seeded u8 image of shape (h, w)."""
    rng = np.random.default_rng(seed)
    img = _scene(rng, h, w) + rng.normal(0.0, noise, (h, w))
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))


def synth_stereo(seed: int, w: int = 752, h: int = 480, max_disp: float = 48.0,
                 noise: float = 3.0) -> tuple[np.ndarray, np.ndarray]:
    """A seeded rectified stereo pair (left, right), right = left warped by a smooth disparity."""
    rng = np.random.default_rng(seed)
    pad = int(max_disp) + 2
    scene = _scene(rng, h, w + pad)
    disp = max_disp * _value_noise(rng, h, w, 96)
    left = scene[:, pad:pad + w]
    # left(u) = scene(u + pad); a point at left column u appears at u - d on the right, so
    # right(u) = scene(u + d(u) + pad) (bilinear in x).
    src = np.clip(np.arange(w)[None, :] + disp + pad, 0, w + pad - 1.001)
    x0 = np.floor(src).astype(np.int64)
    fx = src - x0
    rows = np.arange(h)[:, None]
    right = scene[rows, x0] * (1 - fx) + scene[rows, x0 + 1] * fx
    left = left + rng.normal(0.0, noise, (h, w))
    right = right + rng.normal(0.0, noise, (h, w))
    to_u8 = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)
    return to_u8(left), to_u8(right)


def synth_batch(seed: int, n: int, w: int = 752, h: int = 480) -> np.ndarray:
    """n independent images, shape (n, h, w)."""
    return np.stack([synth_image(seed + i, w, h) for i in range(n)])


# The stereo sequence's geometry: a fronto-parallel textured plane at depth Z = bf / SEQ_DISP seen by
# a rectified pinhole stereo rig translating along +x by SEQ_SHIFT * Z / fx per frame, so the image
# content moves SEQ_SHIFT px left per frame and every scene point has disparity SEQ_DISP: the frames,
# their stereo depths and a constant-velocity motion model agree exactly (Tracking's
# TrackWithMotionModel / SearchLocalPoints find their points where the projection puts them).
SEQ_DISP = 16
SEQ_SHIFT = 2


def synth_stereo_sequence(seed: int, n: int, w: int = 752, h: int = 480, shift: int = SEQ_SHIFT,
                          disp: int = SEQ_DISP, noise: float = 3.0) -> list[tuple[np.ndarray, np.ndarray]]:
    """n seeded rectified stereo pairs of a camera moving along x over one planar scene: frame k's
    left image is scene columns [k * shift, k * shift + w), its right image columns [k * shift +
    disp, ...) (disparity `disp` everywhere), each with its own sensor noise."""
    rng = np.random.default_rng(seed)
    scene = _scene(rng, h, w + (n - 1) * shift + disp)
    to_u8 = lambda a: np.clip(np.rint(a), 0, 255).astype(np.uint8)   # noqa: E731
    out = []
    for k in range(n):
        c = k * shift
        left = scene[:, c:c + w] + rng.normal(0.0, noise, (h, w))
        right = scene[:, c + disp:c + disp + w] + rng.normal(0.0, noise, (h, w))
        out.append((np.ascontiguousarray(to_u8(left)), np.ascontiguousarray(to_u8(right))))
    return out

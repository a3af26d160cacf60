"""Synthetic sample streams for the bench and the parity tests.

There is no audio data in this pipeline (no network, the reference's test
files are private: Makefile:45-49), so inputs are generated:

    x = clamp(round(2^(b-1) * (0.02 + 0.4*sin(2*pi*997*t + 0.3*ch) + 0.1*u))) / 2^(b-1)

with u ~ U[-1, 1) from a seeded splitmix64 stream, seed = 20260206 + 1000*file + ch,
t = i / fs.  b = 24 gives int24-valued samples (every value exact in f32),
b = 16 int16, and bits=None skips the integer rounding (float32 sources).
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 20260206
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def splitmix64(seed: int, count: int) -> np.ndarray:
    """count successive splitmix64 outputs (uint64) for the given seed."""
    idx = np.arange(1, count + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def uniform_pm1(seed: int, count: int) -> np.ndarray:
    """U[-1, 1) doubles from the top 53 bits of splitmix64."""
    return _u_slice(seed, 0, count)


def channel(n: int, fs: float, ch: int = 0, file: int = 0, bits=24, chunk: int = 1 << 22) -> np.ndarray:
    """One deinterleaved channel of n float32 samples."""
    out = np.empty(n, dtype=np.float32)
    seed = SEED_BASE + 1000 * file + ch
    scale = float(2 ** (bits - 1)) if bits else 1.0
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        i = np.arange(s, e, dtype=np.float64)
        u = _u_slice(seed, s, e)
        v = 0.02 + 0.4 * np.sin(2.0 * np.pi * 997.0 * i / fs + 0.3 * ch) + 0.1 * u
        if bits:
            q = np.clip(np.rint(v * scale), -scale, scale - 1.0)
            out[s:e] = (q / scale).astype(np.float32)
        else:
            out[s:e] = v.astype(np.float32)
    return out


def _u_slice(seed: int, s: int, e: int) -> np.ndarray:
    idx = np.arange(s + 1, e + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + idx * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 / 9007199254740992.0) - 1.0


def file_buffer(nch: int, n: int, fs: float, file: int = 0, bits=24) -> np.ndarray:
    """[nch][n] float32 deinterleaved buffer (the reference's AudioBuffer)."""
    return np.stack([channel(n, fs, ch, file, bits) for ch in range(nch)])

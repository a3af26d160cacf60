"""Python handle on the CPU oracle (liblowcut_oracle.so) + an exact restatement.

TEST INFRASTRUCTURE ONLY: imported by tests/, bench.py's cpu_baseline leg and
__graft_entry__.smoke() as the checker, never by the product.

PARITY STATUS ("parity unpinned" for c_lib): see lowcut_oracle.c's header.
The reference (diskerror/audio-fir-filter) ships no tests or golden vectors
and cannot be compiled here (c_lib and Boost are absent), so this oracle is a
restatement of FilterCore.h:20-79 / ProcessFile.cp:47-101, pinned against the
independent exact-rational restatement `exact_filter_range` below.
"""
from __future__ import annotations

import ctypes
import os
from fractions import Fraction

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liblowcut_oracle.so")

MODE_LD, MODE_FMA, MODE_MULADD = 0, 1, 2

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        lib = ctypes.CDLL(LIB_PATH)
        vp, i64, c_int, dbl = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double
        lib.oracle_lowcut_ntaps.argtypes = [dbl]
        lib.oracle_lowcut_ntaps.restype = c_int
        lib.oracle_design_lowcut.argtypes = [dbl, c_int, vp]
        lib.oracle_design_lowcut.restype = c_int
        lib.oracle_apply_filter_range.argtypes = [vp, i64, vp, c_int, vp, vp, i64, i64, c_int]
        lib.oracle_apply_filter_range.restype = None
        lib.oracle_apply_filter_range_ld1.argtypes = [vp, i64, vp, c_int, vp, vp, i64, i64]
        lib.oracle_apply_filter_range_ld1.restype = None
        lib.oracle_filter_channel_mt.argtypes = [vp, i64, vp, c_int, vp, c_int, c_int]
        lib.oracle_filter_channel_mt.restype = c_int
        lib.oracle_max_mag.argtypes = [vp, i64]
        lib.oracle_max_mag.restype = ctypes.c_float
        lib.oracle_scale.argtypes = [vp, i64, dbl]
        lib.oracle_scale.restype = None
        lib.oracle_process_buffer.argtypes = [vp, c_int, i64, vp, c_int, c_int, c_int, c_int, vp]
        lib.oracle_process_buffer.restype = ctypes.c_float
        lib.oracle_filter_points.argtypes = [vp, i64, vp, c_int, vp, i64, vp, vp, c_int]
        lib.oracle_filter_points.restype = None
        _lib = lib
    return _lib


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def lowcut_ntaps(slope_hz: float, fs: float) -> int:
    return load().oracle_lowcut_ntaps(slope_hz / fs)


def design_lowcut(freq_hz: float, fs: float, ntaps: int) -> np.ndarray:
    """dspguide Blackman windowed-sinc low-pass -> spectral inversion (ProcessFile.cp:47-50)."""
    taps = np.zeros(ntaps, dtype=np.float64)
    rc = load().oracle_design_lowcut(freq_hz / fs, ntaps, taps.ctypes.data)
    if rc != 0:
        raise ValueError(f"design_lowcut rc={rc}")
    return taps


def apply_filter_range(x, taps, y, start, end, mode=MODE_LD, y64=None):
    """FilterCore.h:20-79 restated; writes y[start:end] (and y64 if given)."""
    x, taps = _f32(x), _f64(taps)
    assert y.dtype == np.float32 and y.flags.c_contiguous and y.size >= x.size
    if y64 is not None:
        assert y64.dtype == np.float64 and y64.size >= x.size
    lib = load()
    if mode == MODE_LD:
        lib.oracle_apply_filter_range_ld1(x.ctypes.data, x.size, taps.ctypes.data, taps.size,
                                          y.ctypes.data, None if y64 is None else y64.ctypes.data,
                                          start, end)
    else:
        lib.oracle_apply_filter_range(x.ctypes.data, x.size, taps.ctypes.data, taps.size,
                                      y.ctypes.data, None if y64 is None else y64.ctypes.data,
                                      start, end, mode)


def filter_channel(x, taps, mode=MODE_LD, with_f64=False):
    x = _f32(x)
    y = np.zeros(x.size, dtype=np.float32)
    y64 = np.zeros(x.size, dtype=np.float64) if with_f64 else None
    apply_filter_range(x, taps, y, 0, x.size, mode, y64)
    return (y, y64) if with_f64 else y


def filter_points(x, taps, idx, mode=MODE_LD):
    """(y32, y64) at positions idx of the filtered channel x."""
    x, taps = _f32(x), _f64(taps)
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    assert idx.size == 0 or (idx.min() >= 0 and idx.max() < x.size)
    out = np.zeros(idx.size, np.float32)
    out64 = np.zeros(idx.size, np.float64)
    load().oracle_filter_points(x.ctypes.data, x.size, taps.ctypes.data, taps.size,
                                idx.ctypes.data, idx.size, out.ctypes.data, out64.ctypes.data, mode)
    return out, out64


def filter_channel_mt(x, taps, nthreads, mode=MODE_FMA):
    """ProcessFile.cp:57-87 chunk hand-off with pthreads (the CPU baseline)."""
    x, taps = _f32(x), _f64(taps)
    y = np.zeros(x.size, dtype=np.float32)
    rc = load().oracle_filter_channel_mt(x.ctypes.data, x.size, taps.ctypes.data, taps.size,
                                         y.ctypes.data, nthreads, mode)
    if rc != 0:
        raise RuntimeError(f"oracle_filter_channel_mt rc={rc}")
    return y


def max_mag(y) -> float:
    y = _f32(y)
    return float(load().oracle_max_mag(y.ctypes.data, y.size))


def process_buffer(buf, taps, nthreads=1, normalize=False, mode=MODE_FMA):
    """ProcessFile.cp:57-101 on a [nch][n] float32 buffer (in place). Returns the peak."""
    assert buf.dtype == np.float32 and buf.flags.c_contiguous and buf.ndim == 2
    taps = _f64(taps)
    tmp = np.zeros(buf.shape[1], dtype=np.float32)
    return float(load().oracle_process_buffer(buf.ctypes.data, buf.shape[0], buf.shape[1],
                                              taps.ctypes.data, taps.size, nthreads,
                                              1 if normalize else 0, mode, tmp.ctypes.data))


# ---------------------------------------------------------------------------
# Independent exact restatement (pure Python, small sizes only).
# ---------------------------------------------------------------------------
def _fms_exact(h, p, count=None):
    """WindowedSinc::fms conventions in exact rationals."""
    T = len(h)
    if count is None:
        return sum((h[i] * p[i] for i in range(T)), Fraction(0))
    if count < 0:
        c = -count
        return sum((h[T - c + i] * p[i] for i in range(c)), Fraction(0))
    return sum((h[i] * p[i] for i in range(count)), Fraction(0))


def exact_filter_range(x, taps, start, end):
    """The three loops of FilterCore.h:56-76, literally, in exact rationals.

    Out-of-range reads of loop 1 when N <= M (UB in the reference) read 0.
    Returns a list of Fractions for n in [start, end)."""
    xs = [Fraction(float(v)) for v in np.asarray(x, dtype=np.float32)]
    h = [Fraction(float(v)) for v in np.asarray(taps, dtype=np.float64)]
    N = len(xs)
    half = (len(h) - 1) // 2
    padded = xs + [Fraction(0)] * (len(h) + 1)
    out = []
    n = start
    while n < end and n < half:
        out.append(_fms_exact(h, padded, -(n + half + 1)))
        n += 1
    safe = min(end, N - half)
    while n < safe:
        out.append(_fms_exact(h, padded[n - half:]))
        n += 1
    while n < end:
        out.append(_fms_exact(h, padded[n - half:], N - n + half))
        n += 1
    return out


def fraction_to_f32(q: Fraction) -> np.float32:
    """Correctly rounded (RNE) Fraction -> float32."""
    f = np.float32(float(q))  # float(q) is correctly rounded to f64; f64->f32 may double-round
    # fix double rounding: compare exact distances to the neighbours
    cands = [f, np.nextafter(f, np.float32(np.inf)), np.nextafter(f, np.float32(-np.inf))]
    best = min(cands, key=lambda c: (abs(Fraction(float(c)) - q),
                                     int(np.frombuffer(np.float32(c).tobytes(), np.uint32)[0]) & 1))
    return np.float32(best)

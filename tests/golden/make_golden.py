"""Generate the golden vectors in tests/golden/*.npz.

The reference (diskerror/audio-fir-filter) publishes no tests, fixtures or
known-answer vectors and cannot be compiled here (c_lib + Boost absent), so
these vectors come from the long-double CPU restatement in oracle/ and, for
every case small enough, are cross-checked against the exact-rational
restatement (oracle.exact_filter_range) before being written.  Run:

    make -C oracle && python tests/golden/make_golden.py

Each .npz holds (allow_pickle=False):
    x [nch][n] float32 input, taps float64, y [nch][n] float32 expected
    (long double accumulate, one RNE to f32), y64 [nch][n] float64 (the
    un-narrowed long-double value rounded to f64), exact flag.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "audio-fir-filter_amd"))

import oracle  # noqa: E402
import synth  # noqa: E402

EXACT_LIMIT = 400_000  # N*T budget for the pure-Python exact cross-check


def case_impulse():
    taps = oracle.design_lowcut(1000.0, 48000.0, 41)
    x = np.zeros((1, 257), np.float32)
    x[0, 128] = 1.0
    return x, taps


def case_dc():
    taps = oracle.design_lowcut(500.0, 48000.0, 201)
    x = np.full((1, 2000), 0.5, np.float32)
    return x, taps


def case_sine():
    # 5 kHz tone at 48 kHz through a 20 Hz low-cut of 801 taps: passband, gain ~1
    taps = oracle.design_lowcut(20.0, 48000.0, 801)
    i = np.arange(4000)
    x = (0.5 * np.sin(2 * np.pi * 5000.0 * i / 48000.0)).astype(np.float32)[None, :]
    return x, taps


def case_random_int24():
    taps = oracle.design_lowcut(20.0, 48000.0, 401)
    return synth.file_buffer(2, 5000, 48000.0, file=7, bits=24), taps


def case_short_n_lt_t():
    # N < M+1: the reference's loop 1 reads past the end (UB); defined as zero padding
    rng = np.random.default_rng(11)
    taps = rng.standard_normal(101)
    x = rng.uniform(-1, 1, (1, 50)).astype(np.float32)
    return x, taps


def case_tiny():
    rng = np.random.default_rng(12)
    return rng.uniform(-1, 1, (1, 1)).astype(np.float32), rng.standard_normal(3)


def case_single_tap():
    rng = np.random.default_rng(13)
    return rng.uniform(-1, 1, (1, 777)).astype(np.float32), np.array([0.75])


def case_float_source():
    # config-3-like float32 source (no integer rounding), 8 channels, long kernel
    taps = oracle.design_lowcut(20.0, 96000.0, 1601)
    return synth.file_buffer(8, 3000, 96000.0, file=3, bits=None), taps


def case_config1():
    # config 1: 1 s mono 48 kHz int16, -f 20 -s 10 -> M = 4/BW = 19200 (19 201 taps)
    fs = 48000.0
    ntaps = oracle.lowcut_ntaps(10.0, fs)
    taps = oracle.design_lowcut(20.0, fs, ntaps)
    return synth.file_buffer(1, 48000, fs, file=0, bits=16), taps


def case_ragged_taps():
    # tap count that is not a multiple of any kernel tile (2R = 32, stage 256)
    rng = np.random.default_rng(14)
    taps = rng.standard_normal(4001 - 32 * 3 + 6) * 1e-2
    return rng.uniform(-1, 1, (1, 9000)).astype(np.float32), taps


CASES = {
    "impulse": case_impulse,
    "dc": case_dc,
    "sine": case_sine,
    "random_int24": case_random_int24,
    "short_n_lt_t": case_short_n_lt_t,
    "tiny": case_tiny,
    "single_tap": case_single_tap,
    "float_source": case_float_source,
    "config1": case_config1,
    "ragged_taps": case_ragged_taps,
}


def build(name):
    x, taps = CASES[name]()
    y = np.zeros_like(x)
    y64 = np.zeros(x.shape, np.float64)
    for c in range(x.shape[0]):
        yc, y64c = oracle.filter_channel(x[c], taps, oracle.MODE_LD, with_f64=True)
        y[c], y64[c] = yc, y64c
    exact = x.shape[1] * taps.size * x.shape[0] <= EXACT_LIMIT
    if exact:
        for c in range(x.shape[0]):
            ex = oracle.exact_filter_range(x[c], taps, 0, x.shape[1])
            ex32 = np.array([oracle.fraction_to_f32(q) for q in ex], np.float32)
            if not np.array_equal(ex32, y[c]):
                raise SystemExit(f"{name}: long-double oracle disagrees with exact restatement")
    return dict(x=x, taps=taps, y=y, y64=y64, exact=np.array(exact))


def main(names=None):
    for name in names or CASES:
        d = build(name)
        path = os.path.join(HERE, f"{name}.npz")
        np.savez_compressed(path, **d)
        print(f"{name}: x{d['x'].shape} taps={d['taps'].size} exact={bool(d['exact'])} "
              f"-> {os.path.getsize(path)} B")


if __name__ == "__main__":
    main(sys.argv[1:])

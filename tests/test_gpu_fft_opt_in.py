"""GPU parity of the opt-in FFT kernels: 16 waves per workgroup
(csrc/fir_fft16.hpp, LCFIR_FFT_WAVES=16, zero-phase form) and 4 waves per
workgroup (csrc/fir_fft4.hpp, LCFIR_FFT_WAVES=4, every form).  DESIGN.md s4.2
has the measurements that keep the 8-wave kernel the default.

Each kernel runs in a child process (the switch is read once per process),
which also proves through lcfir_ctx_fft_waves that it was the one that ran.
Its outputs are checked against the long-double oracle at
every edge sample plus random positions, against the default 8-wave kernel
(<= 1 f32 ulp everywhere), and its windowed calls (odd starts, windows
shorter than one segment, straddling the range edges) against its own
whole-channel outputs, bit for bit (input windows from lcfir_ctx_window)."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from test_gpu_parity import RMS_TOL, _sample_positions, gpu_filter_channels, lc, max_ulps, rms  # noqa: F401

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = """
import json, sys, numpy as np
sys.path[:0] = [{pkg!r}, {oracle!r}]
import lcfir, synth
cases = json.load(open({cases!r}))
out = {{}}
for i, c in enumerate(cases):
    x = synth.file_buffer(c["nch"], c["n"], 48000.0, file=c["file"], bits=24)
    flt = lcfir.Filter(np.load(c["taps"]), method="fft")
    assert flt.fft_waves == {waves}, flt.fft_waves
    n, nch = c["n"], c["nch"]
    dx = lcfir.DeviceBuffer.from_array(x); dy = lcfir.DeviceBuffer(x.nbytes)
    dpk = lcfir.DeviceBuffer(4 * nch); lcfir.peak_reset_dev(dpk, nch)
    flt.filter_channels_dev(dx, n, nch, n, dy, n, dpk)
    lcfir.sync()
    out[f"y{{i}}"] = dy.download((nch, n))
    out[f"pk{{i}}"] = dpk.download(nch)
    for k, (s, e) in enumerate(c["windows"]):
        lo, hi = flt.window(n, s, e)  # the whole segments: bit for bit
        xw = np.ascontiguousarray(x[:, lo:hi], np.float32)
        dxw = lcfir.DeviceBuffer.from_array(xw); dyw = lcfir.DeviceBuffer(4 * nch * (e - s))
        flt.filter_window_dev(dxw, lo, hi, hi - lo, n, nch, dyw, s, e - s, s, e)
        lcfir.sync()
        out[f"w{{i}}_{{k}}"] = dyw.download((nch, e - s))
np.savez({out!r}, **out)
"""

CASES = [
    # (ntaps, perturb, n, nch, windows); perturb > 0: an asymmetric filter (general pair table)
    (4001, 0.0, 200_003, 2, [(1, 200_002), (1999, 14_385), (77_777, 77_778), (187_000, 200_003)]),
    (801, 0.0, 50_001, 3, [(3, 49_999), (0, 1)]),
    (8001, 0.0, 120_000, 2, [(4000, 24_001)]),
    (4001, 0.0, 3_000, 1, [(0, 3_000), (1_500, 1_501)]),  # shorter than one segment
]
CASES_ALL_FORMS = [
    (4003, 0.0, 100_001, 2, [(5, 99_000)]),     # odd half: general table
    (4001, 1e-9, 60_000, 2, [(2001, 30_000)]),  # asymmetric: general table
    (19_201, 0.0, 150_000, 1, [(9_600, 140_000)]),  # 2 partitions (config 1's kernel)
]


@pytest.mark.parametrize("waves", [16, 4])
def test_opt_in_fft_kernel_parity(lc, oracle_mod, tmp_path, waves):
    import synth
    cases = []
    for i, (ntaps, perturb, n, nch, windows) in enumerate(CASES + (CASES_ALL_FORMS if waves == 4 else [])):
        taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
        if perturb:
            taps = taps + perturb * np.linspace(-1.0, 1.0, ntaps)
        tp = str(tmp_path / f"taps{i}.npy")
        np.save(tp, taps)
        cases.append({"taps": tp, "n": n, "nch": nch, "file": 11 + i, "windows": windows})
    cj = str(tmp_path / "cases.json")
    json.dump(cases, open(cj, "w"))
    out = str(tmp_path / "y.npz")
    code = _CHILD.format(pkg=os.path.join(ROOT, "audio-fir-filter_amd"), oracle=os.path.join(ROOT, "oracle"),
                         cases=cj, out=out, waves=waves)
    subprocess.run([sys.executable, "-c", code], check=True, timeout=300,
                   env=dict(os.environ, LCFIR_FFT_WAVES=str(waves)))
    got = np.load(out)
    for i, c in enumerate(cases):
        taps = np.load(c["taps"])
        half = (len(taps) - 1) // 2
        x = synth.file_buffer(c["nch"], c["n"], 48000.0, file=c["file"], bits=24)
        y16, pk16 = got[f"y{i}"], got[f"pk{i}"]  # the opt-in kernel's outputs
        flt = lc.Filter(taps, method="fft")
        assert flt.fft_waves == 8  # this process runs the default kernel
        y8, _ = gpu_filter_channels(lc, flt, x)
        assert max_ulps(y16, y8) <= 1, i
        assert rms(y16, y8) <= RMS_TOL, i
        for ch in range(c["nch"]):
            idx = _sample_positions(c["n"], half, 2048, 900 + 10 * i + ch)
            ref, _ = oracle_mod.filter_points(x[ch], taps, idx, oracle_mod.MODE_LD)
            assert rms(y16[ch][idx], ref) <= RMS_TOL, (i, ch)
            assert max_ulps(y16[ch][idx], ref) <= 1, (i, ch)
            assert pk16[ch] == np.abs(y16[ch]).max(), (i, ch)
        for k, (s, e) in enumerate(c["windows"]):
            assert np.array_equal(got[f"w{i}_{k}"], y16[:, s:e]), (i, s, e)

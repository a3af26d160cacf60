"""GPU parity of fir_fft16r_kernel (csrc/fir_fft16r.hpp): the L = 16 384
zero-phase unit held in the registers of a 256-thread workgroup, two
workgroups per CU (lcfir_ctx_set_fft_family "register" at seg_len 16384).

Bars as tests/test_gpu_parity.py: RMS vs the long-double oracle <= 1e-9 and
<= 1 f32 ulp per output; windowed calls from lcfir_ctx_window's window and the
reference's thread hand-off bit-identical to the whole channel; fused peaks
equal max |y|; within 1 ulp of the LDS-column kernel of the same segment
length.  The index flow is modelled in scripts/fft16r_model.py (CPU test
tests/test_fft32_tables.py ran it on the host's tables while the kernel was in
the product).  Out of the product since round 6: run it against the variant
library (scripts/variants/r16/README.md).  "l16_reg" is kernel code 4 there."""
import numpy as np
import pytest

from test_gpu_parity import (RMS_TOL, _sample_positions, check_window, gpu_filter_channels, gpu_filter_window,
                             max_ulps, rms)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lc():
    import lcfir
    assert lcfir.device_count() >= 1, "no GPU visible"
    lcfir.FFT_KERNELS.setdefault(4, "l16_reg")  # the variant library's LCFIR_FFT_KERNEL_L16_REG
    return lcfir


def r16_filter(lc, taps, **tuning):
    flt = lc.Filter(taps, method="fft")
    flt.set_fft_tuning(seg_len=16384, **tuning)
    # family 2 exists only in the variant library (scripts/variants/r16/r16_kernel.patch)
    lc._check(lc.load().lcfir_ctx_set_fft_family(flt._ctx, 2))
    u = flt.fft_units
    assert u["kernel"] == "l16_reg" and u["outputs"] == 16384 - len(taps) + 1, u
    assert u["nrm_floats"] == 16 * 1024  # kNrmK16 blocks of 1 024 floats per unit
    return flt


@pytest.mark.parametrize("ntaps", [4001, 4005, 4003, 8001, 1601, 401, 3])
def test_fft16r_against_oracle(lc, oracle_mod, ntaps):
    """Designed low-cuts (even and odd half: the pair-store and the per-output
    store paths; 3 taps: units of 16 382 outputs) on a stereo channel of
    300 001 samples: every edge output and random positions against the
    long-double oracle, fused peaks, within 1 ulp of the LDS-column kernel,
    windowed calls and the thread hand-off bit-identical."""
    import synth
    fs, n = 48000.0, 300_001
    taps = oracle_mod.design_lowcut(20.0, fs, ntaps)
    x = synth.file_buffer(2, n, fs, file=21, bits=24)
    flt = r16_filter(lc, taps)
    y, pk = gpu_filter_channels(lc, flt, x)
    half = (ntaps - 1) // 2
    for c in range(2):
        idx = _sample_positions(n, half, 2048, 1600 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL, c
        assert max_ulps(y[c][idx], ref_ld) <= 1, c
        assert pk[c] == np.abs(y[c]).max()
    lds = lc.Filter(taps, method="fft")
    lds.set_fft_tuning(seg_len=16384)
    lds.set_fft_family("lds")
    assert lds.fft_units["kernel"] == "l16"
    y16, _ = gpu_filter_channels(lc, lds, x)
    assert max_ulps(y, y16) <= 1 and rms(y, y16) <= RMS_TOL
    for start, end in [(1, n - 1), (half + 3, half + 40_000), (123_457, 123_458), (n - 33_000, n)]:
        check_window(lc, flt, x, y, start, end)
    for threads in (3, 7):
        assert np.array_equal(lc.filter_channel(x[0], flt, threads), y[0]), threads


def test_fft16r_config2_every_sample(lc, oracle_mod):
    """Config 2's file (10 min stereo 48 kHz int24, 4 001 taps) on the
    register kernel at L = 16 384: every one of the 57.6 M outputs within
    1 ulp of the default kernel (fir_fft32r), RMS between them <= 1e-9, and
    the long-double oracle at the edges and 4 096 random positions."""
    import synth
    fs, n, nch = 48000.0, 28_800_000, 2
    taps = oracle_mod.design_lowcut(20.0, fs, 4001)
    x = synth.file_buffer(nch, n, fs, file=0, bits=24)
    y, pk = gpu_filter_channels(lc, r16_filter(lc, taps), x)
    dflt = lc.Filter(taps, method="fft")
    assert dflt.fft_units["kernel"] == "l32_reg"
    y32, _ = gpu_filter_channels(lc, dflt, x)
    for c in range(nch):
        assert max_ulps(y[c], y32[c]) <= 1 and rms(y[c], y32[c]) <= RMS_TOL, c
        assert pk[c] == np.abs(y[c]).max()
        idx = _sample_positions(n, 2000, 4096, 1700 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL and max_ulps(y[c][idx], ref_ld) <= 1, c


def test_fft16r_chunks_groups_and_short_channels(lc, oracle_mod):
    """Launch chunks of whole segments and channel groups (bytes and peaks
    identical to one launch); 8 channels of 96 kHz float32; a channel shorter
    than one segment and a one-sample channel against the oracle."""
    import synth
    taps = oracle_mod.design_lowcut(20.0, 96000.0, 4001)
    x = synth.file_buffer(8, 200_003, 96000.0, file=22, bits=None)
    one = r16_filter(lc, taps)
    y0, pk0 = gpu_filter_channels(lc, one, x)
    for chunk, mu in [(70_000, 0), (0, 9), (50_000, 4)]:
        f = r16_filter(lc, taps, chunk=chunk, max_units=mu)
        y1, pk1 = gpu_filter_channels(lc, f, x)
        assert np.array_equal(y0, y1) and np.array_equal(pk0, pk1), (chunk, mu)
    for n in (20_000, 1):
        xs = np.ascontiguousarray(x[:2, :n])
        ys, _ = gpu_filter_channels(lc, one, xs)
        for c in range(2):
            ref = oracle_mod.filter_channel(xs[c], taps, oracle_mod.MODE_LD)
            assert max_ulps(ys[c], ref) <= 1 and rms(ys[c], ref) <= RMS_TOL, (n, c)


@pytest.mark.parametrize("ntaps", [4001, 4003])
def test_fft16r_edge_outputs_every_window_alignment(lc, oracle_mod, ntaps):
    """Outputs next to a window edge (tests/test_gpu_parity.py's
    test_edge_outputs_every_window_alignment) on the register kernel: windows
    starting d = 0..3 samples before the first sample the outputs need."""
    n = 120_001
    rng = np.random.default_rng(ntaps + 7)
    x = (rng.integers(-2**23, 2**23, size=(2, n)) / 2.0**23).astype(np.float32)
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    half = (ntaps - 1) // 2
    flt = r16_filter(lc, taps)
    span = ntaps + 256
    cases = [(0, span, 0, n), (n - span, n, 0, n)]
    for d in range(4):
        s0 = 30_000 + 7 * d
        cases.append((s0, s0 + span, s0 - half - d, s0 + span + half + d))
    for start, end, x_lo, x_hi in cases:
        yw = gpu_filter_window(lc, flt, x, start, end, x_lo, x_hi)
        idx = np.arange(start, end)
        for c in range(2):
            ref, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
            assert max_ulps(yw[c], ref) <= 1 and rms(yw[c], ref) <= RMS_TOL, (c, start, x_lo)


@pytest.mark.parametrize("count,offset,peak,force", [(50_000, 0, 2.5, False), (50_000, 1, 2.5, False),
                                                    (16 * 1024 * 18, 0, 0.5, True), (16 * 1024 * 18 + 1, 0, 3.0, False),
                                                    (7, 0, 0.75, False)])
def test_fft16r_family_switch_and_normalize(lc, oracle_mod, count, offset, peak, force):
    """lcfir_ctx_set_fft_family moves a ctx between kernels (the default
    family keeps the LDS-column kernel at 16 384); a previous file's
    normalize carried by the register kernel's launch (every unit rescales
    its slice before its stage 1) gives the same bytes as the separate calls:
    fused up to 16 Ki floats per unit (the 18-unit launch's limit, and one
    float past it: its own pass), an unaligned buffer its own pass, peaks
    below 1 without force a no-op."""
    import torch
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    flt = lc.Filter(taps, method="fft")
    flt.set_fft_tuning(seg_len=16384)
    assert flt.fft_units["kernel"] == "l16"
    flt.set_fft_family("register")
    assert flt.fft_units["kernel"] == "l16_reg"
    flt.set_fft_family("lds")
    assert flt.fft_units["kernel"] == "l16"
    flt.set_fft_family("register")
    rng = np.random.default_rng(3)
    n, nch = 100_000, 2
    x = np.ascontiguousarray(np.rint(rng.uniform(-0.9, 0.9, (nch, n)) * 2 ** 23) / 2 ** 23, np.float32)
    prev = (rng.standard_normal(count + offset) * 0.5).astype(np.float32)
    units = -(-n // flt.fft_units["outputs"]) * nch
    assert units == 18
    dx = torch.from_numpy(x).cuda()
    res = []
    for fused in (False, True):
        dy = torch.empty((nch, n), dtype=torch.float32, device="cuda")
        dpk = torch.zeros(1, dtype=torch.float32, device="cuda")
        dprev = torch.from_numpy(prev.copy()).cuda()
        dppk = torch.tensor([peak], dtype=torch.float32, device="cuda")
        view = dprev[offset:]
        if fused:
            flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, 0, view, count, dppk, 1, force)
        else:
            flt.filter_window_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, peak_stride=0)
            lc.normalize_dev(view, count, 1, count, dppk, 1, force)
        torch.cuda.synchronize()
        res.append((dy.cpu().numpy(), dpk.cpu().numpy(), dprev.cpu().numpy()))
    assert all(np.array_equal(a, b) for a, b in zip(res[0], res[1]))
    want_fused = offset % 4 == 0 and count <= units * 16 * 1024
    assert flt.nrm_stats == ({"fused": 1, "separate": 0} if want_fused else {"fused": 0, "separate": 1})
    body = prev[offset:]
    if peak > 1.0 or force:
        body = (body.astype(np.float64) * (1.0 / np.float64(np.float32(peak)))).astype(np.float32)
    assert np.array_equal(res[1][2][offset:], body) and np.array_equal(res[1][2][:offset], prev[:offset])

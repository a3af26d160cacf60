"""Seeded randomized GPU parity: random tap counts (odd, 1 .. 40 001; designed
low-cuts, which run the FFT's zero-phase form (odd and even halves), and random
taps, which run its general form), random channel counts and lengths (shorter
than the filter included), random sub-ranges through the windowed entry point,
both methods.  Every case against the oracle at sampled positions:

  * RMS(y - y_longdouble) <= 1e-9 and <= 1 f32 ulp per sample (every method);
  * the direct method bit-exact against ORACLE_FMA;
  * sub-ranges computed from lcfir_ctx_window's input window equal to the
    same outputs of the whole-channel call (bit for bit, same method); from
    the narrowest window [start - half, end + half): bit for bit for the
    direct method, within 1 f32 ulp for the FFT (whose edge segments then
    read zeros where the whole channel has samples);
  * the fused per-channel peak equal to max |y| of the whole channel;
  * channel 0 as ragged device ranges equal to the whole-channel call, bit
    for bit (partition invariance).

A second set fuzzes lcfir_filter_window_norm_dev (a previous file's normalize
carried by the filter call) against the separate filter + normalize calls.
About a third of the FFT cases of both sets force the L = 32 768 segment
(_seg32): linear-phase filters then run the register kernel (fir_fft32r.hpp,
whose launch carries the normalize in two halves of up to kNrmK32 blocks per
unit), the others the park-slab kernel (never fused).  The fused / separate
switch is sized from the plan itself (lcfir_ctx_fft_units), and every case
checks which of the two the library took (lcfir_ctx_nrm_stats).

LCFIR_FUZZ_CASES / LCFIR_FUZZ_NORM_CASES / LCFIR_FUZZ_SEED0 widen or shift the
seed range for a longer campaign (scripts/gpu_run.sh fuzz:SEED0,CASES,NORM[,FAMILY]); the defaults are the
round-end suite's.  LCFIR_FUZZ_FAMILY (lcfir_ctx_set_fft_family: default or
lds) runs the FFT cases on another kernel family: "lds" puts the L = 32 768
zero-phase cases on the park-slab kernel.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-9
SEED0 = int(os.environ.get("LCFIR_FUZZ_SEED0", "0"))
N_CASES = int(os.environ.get("LCFIR_FUZZ_CASES", "120"))
N_NORM_CASES = int(os.environ.get("LCFIR_FUZZ_NORM_CASES", "40"))
FAMILY = os.environ.get("LCFIR_FUZZ_FAMILY", "default")


def _max_ulps(a, b, floor=1e-12):
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    close = np.abs(a.astype(np.float64) - b.astype(np.float64)) <= floor
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return int(np.where(close, 0, np.abs(ia - ib)).max()) if a.size else 0


def _seg32(seed):
    """About a third of the FFT cases run the L = 32 768 segment (fir_fft32.hpp),
    drawn from a stream of its own so the cases themselves stay as they were."""
    return np.random.default_rng(90_000 + seed).random() < 0.35


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    ntaps = int(rng.choice([1, 3, 5, 95, 97, 401, 1601, 4001, 4003, 8001, 10925, 19201, 40001]))
    ntaps = max(1, ntaps + 2 * int(rng.integers(-3, 4)) * (ntaps > 9))
    nch = int(rng.integers(1, 4))
    n = int(rng.choice([1, 7, ntaps // 2 + 1, ntaps + 3, 20_000, 123_457, 300_001]))
    # the FFT is exact only to ~1e-16, so taps with few significant bits can
    # land outputs on f32 rounding ties (test_gpu_parity.TIE_PRONE); AUTO runs
    # such short filters with the direct method, and so does this test
    method = "direct" if ntaps < 64 or (ntaps <= 2001 and rng.random() < 0.4) else "fft"
    designed = rng.random() < 0.6
    return rng, ntaps, nch, max(1, n), method, designed


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + N_CASES))
def test_random_case(oracle_mod, seed):
    import lcfir as lc
    rng, ntaps, nch, n, method, designed = _case(seed)
    if designed:
        taps = oracle_mod.design_lowcut(float(rng.uniform(5.0, 300.0)), 48000.0, ntaps)
    else:
        taps = rng.standard_normal(ntaps) / np.sqrt(ntaps)
    bits = int(rng.choice([16, 24, 0]))
    x = rng.uniform(-0.9, 0.9, (nch, n))
    if bits:
        x = np.rint(x * 2 ** (bits - 1)) / 2 ** (bits - 1)
    x = np.ascontiguousarray(x, np.float32)
    flt = lc.Filter(taps, method=method)
    if method == "fft" and _seg32(seed):
        flt.set_fft_tuning(seg_len=32768)
    if method == "fft" and FAMILY != "default":
        flt.set_fft_family(FAMILY)

    dx = lc.DeviceBuffer.from_array(x)
    dy = lc.DeviceBuffer(x.nbytes)
    dpk = lc.DeviceBuffer(4 * nch)
    lc.peak_reset_dev(dpk, nch)
    flt.filter_channels_dev(dx, n, nch, n, dy, n, dpk)
    lc.sync()
    y = dy.download((nch, n))
    pk = dpk.download(nch)
    for b in (dx, dy, dpk):
        b.free()

    half = (ntaps - 1) // 2
    for c in range(nch):
        idx = np.unique(np.r_[np.arange(min(n, 40)), np.arange(max(0, n - 40), n),
                              rng.integers(0, n, 600)])
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        d = y[c][idx].astype(np.float64) - ref_ld
        assert float(np.sqrt(np.mean(d * d))) <= RMS_TOL, (seed, c)
        assert _max_ulps(y[c][idx], ref_ld) <= 1, (seed, c)
        if method == "direct":
            ref_fma, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_FMA)
            assert np.array_equal(y[c][idx], ref_fma), (seed, c)
        assert pk[c] == np.abs(y[c]).max(), (seed, c)

    # partition invariance: channel 0 as ragged device ranges (each call reads
    # the whole channel) gives the whole-channel bytes
    cuts = np.unique(np.r_[0, rng.integers(0, n + 1, int(rng.integers(1, 6))), n])
    dx0 = lc.DeviceBuffer.from_array(np.ascontiguousarray(x[0]))
    dy0 = lc.DeviceBuffer.from_array(np.zeros(n, np.float32))
    for s_, e_ in zip(cuts[:-1], cuts[1:]):
        flt.apply_range_dev(dx0, n, dy0, int(s_), int(e_))
    lc.sync()
    y0 = dy0.download(n)
    dx0.free()
    dy0.free()
    assert np.array_equal(y0, y[0]), (seed, cuts.tolist())

    # sub-ranges from only their input window (a file sharded by sample range)
    for _ in range(3):
        start = int(rng.integers(0, n))
        end = int(rng.integers(start, n + 1))
        if end == start:
            continue
        for exact, (lo, hi) in ((True, flt.window(n, start, end)),
                                (False, (max(0, start - half), min(n, end + half)))):
            xw = np.ascontiguousarray(x[:, lo:hi])
            dxw = lc.DeviceBuffer.from_array(xw)
            dyw = lc.DeviceBuffer(4 * nch * (end - start))
            flt.filter_window_dev(dxw, lo, hi, hi - lo, n, nch, dyw, start, end - start, start, end)
            lc.sync()
            yw = dyw.download((nch, end - start))
            dxw.free()
            dyw.free()
            if exact or method == "direct":
                assert np.array_equal(yw, y[:, start:end]), (seed, start, end, lo, hi)
            else:
                assert _max_ulps(yw, y[:, start:end]) <= 1, (seed, start, end)


def _norm_case(seed):
    rng = np.random.default_rng(5000 + seed)
    ntaps = int(rng.choice([401, 1601, 4001, 4001, 4003, 8001, 10925, 19201]))
    method = "direct" if ntaps <= 1601 and rng.random() < 0.3 else "fft"
    nch = int(rng.integers(1, 4))
    n = int(rng.choice([1, 7, ntaps // 2 + 1, 20_000, 123_457, 300_001]))
    designed = rng.random() < 0.6
    return rng, ntaps, method, nch, n, designed


def _norm_params(rng, n, nch, units):
    """count, offset, peaks, force of a case.  units: the filter's
    fft_units.  A one-partition FFT launch of U = ceil(n / B) x nch units
    carries the normalize iff count <= U x nrm_floats (a 16-B aligned buffer):
    the counts straddle that switch (the limit itself, +-1 float, +-1 block)."""
    B, cap = max(1, units["outputs"]), units["nrm_floats"]
    blk = 2048 if units["kernel"] == "l32_reg" else 1024
    boundary = -(-n // B) * nch * cap if cap else -(-n // B) * nch * 1024
    count = int(rng.choice([
        1, 3, int(rng.integers(1, 5_000)), int(rng.integers(1, boundary + 1)),
        int(rng.integers(1, boundary + 1)), boundary, boundary + 1, max(1, boundary - blk), boundary + blk,
        boundary + int(rng.integers(-8, 9)), int(rng.integers(boundary, 2 * boundary + 1))]))
    if rng.random() < 0.05:
        count = 0  # a plain filter call
    offset = int(rng.choice([0, 0, 0, 0, 0, 1, 2, 3, 4]))  # floats: 16-B aligned when offset % 4 == 0
    npeak = int(rng.integers(1, 4))
    peaks = rng.choice([0.0, 0.25, 0.999, 1.0, 1.0000001, 1.5, 3.0], npeak).astype(np.float32)
    if rng.random() < 0.5:
        peaks[int(rng.integers(npeak))] = np.float32(rng.uniform(0.01, 4.0))
    force = bool(rng.random() < 0.4)
    fused = bool(cap and count and count <= boundary and offset % 4 == 0)
    return max(0, count), offset, peaks, force, fused


@pytest.mark.parametrize("seed", range(SEED0, SEED0 + N_NORM_CASES))
def test_random_norm_case(oracle_mod, seed):
    """filter + previous-buffer rescale in one call (fused into the FFT launch
    where fft_nrm_fusable, else its own pass) equals the two separate calls
    byte for byte: the filter's outputs and peak, and the rescaled buffer,
    which also equals (float)((double)v * (1 / max(peaks))) under the
    ProcessFile.cp:98-101 decision."""
    import torch  # before lcfir: one HIP runtime in the process
    import lcfir as lc
    rng, ntaps, method, nch, n, designed = _norm_case(seed)
    if designed:
        taps = oracle_mod.design_lowcut(float(rng.uniform(5.0, 300.0)), 48000.0, ntaps)
    else:
        taps = rng.standard_normal(ntaps) / np.sqrt(ntaps)
    flt = lc.Filter(taps, method=method)
    if method == "fft" and _seg32(seed):
        flt.set_fft_tuning(seg_len=32768)
    if method == "fft" and FAMILY != "default":
        flt.set_fft_family(FAMILY)
    units = flt.fft_units
    if method == "fft" and designed and ntaps >= 4001 and FAMILY != "lds":
        # linear-phase filters from ~4 000 taps run the register kernel
        assert units["kernel"] == "l32_reg", (seed, units)
    count, offset, peaks, force, want_fused = _norm_params(rng, n, nch, units)
    if method != "fft":
        want_fused = False
    x = np.ascontiguousarray(np.rint(rng.uniform(-0.9, 0.9, (nch, n)) * 2 ** 23) / 2 ** 23, np.float32)
    prev = (rng.standard_normal(count + offset) * 0.5).astype(np.float32)
    dx = torch.from_numpy(x).cuda()
    res = []
    for fused in (False, True):
        dy = torch.empty((nch, n), dtype=torch.float32, device="cuda")
        dpk = torch.zeros(1, dtype=torch.float32, device="cuda")
        dprev = torch.from_numpy(prev.copy()).cuda()
        dppk = torch.from_numpy(peaks.copy()).cuda()
        view = dprev[offset:]
        if fused:
            flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, 0, view, count,
                                       dppk, peaks.size, force)
        else:
            flt.filter_window_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, peak_stride=0)
            if count:
                lc.normalize_dev(view, count, 1, count, dppk, peaks.size, force)
        torch.cuda.synchronize()
        res.append((dy.cpu().numpy(), dpk.cpu().numpy(), dprev.cpu().numpy()))
    (y0, p0, r0), (y1, p1, r1) = res
    case = (seed, ntaps, method, nch, n, count, offset, peaks.tolist(), force, units)
    st = flt.nrm_stats
    assert (st["fused"], st["separate"]) == ((1, 0) if want_fused else (0, 1 if count else 0)), (case, st)
    assert np.array_equal(y0, y1) and np.array_equal(p0, p1), case
    assert np.array_equal(r0, r1), case
    pk = np.float32(peaks.max())
    body = prev[offset:]
    if (pk > 1.0 or force) and pk > 0.0:
        body = (body.astype(np.float64) * (1.0 / np.float64(pk))).astype(np.float32)
    assert np.array_equal(r1[offset:], body) and np.array_equal(r1[:offset], prev[:offset]), case
    assert p1[0] == np.abs(y1).max(), case

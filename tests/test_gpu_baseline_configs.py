"""BASELINE.json's headline configs under GPU parity, at full size:

  * config 2 (10 min stereo 48 kHz int24, 4001 taps): EVERY one of the 57.6 M
    outputs against the oracle's strict-order f64 FMA restatement of
    FilterCore.h:56-76, run multithreaded on the box's cores (~12 s).
    Config 3 (8-ch 96 kHz f32, 8001 taps) the same way, all 46.1 M outputs.  Bars:
    direct method bit-exact; FFT within 1 f32 ulp of it everywhere, RMS vs the
    long-double oracle <= 1e-9, and every FFT/FMA difference an output whose
    long-double value is within 1 ulp too (f32 rounding of values the two f64
    sums place on either side of a tie);
  * configs 4 and 5 (8 x 60-min stereo int24 files, one GPU, the bench's batch
    driver): per-file outputs at the edges + random positions against the
    long-double oracle; the per-file peak = max|y| over that file's channels
    (ProcessFile.cp:92-96, checked on every sample on the device); with
    --normalize every sample equals (float)((double)y * (1 / peak_file)) of the
    un-normalized result (ProcessFile.cp:98-101; peak_scale.hpp's rule).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-9


def _cores():
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))  # the box's CPU share for one GPU


def _ulps(a, b):
    ia = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


@pytest.fixture(scope="module")
def tt():
    import torch  # before lcfir: one HIP runtime in the process
    assert torch.cuda.is_available()
    import lcfir
    lcfir.load()
    return torch, lcfir


@pytest.fixture(scope="module")
def config2(oracle_mod):
    import synth
    fs, n, nch = 48000.0, 28_800_000, 2
    taps = oracle_mod.design_lowcut(20.0, fs, oracle_mod.lowcut_ntaps(48.0, fs))
    assert taps.size == 4001
    x = synth.file_buffer(nch, n, fs, file=0, bits=24)
    ref = np.stack([oracle_mod.filter_channel_mt(x[c], taps, _cores(), oracle_mod.MODE_FMA)
                    for c in range(nch)])
    return x, taps, ref


@pytest.mark.slow
@pytest.mark.parametrize("method", ["direct", "fft"])
def test_config2_every_sample(tt, oracle_mod, config2, method):
    torch, lc = tt
    x, taps, ref = config2
    nch, n = x.shape
    flt = lc.Filter(taps, method=method)
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty_like(xd)
    pk = torch.zeros(nch, dtype=torch.float32, device="cuda")
    flt.filter_channels_dev(xd, n, nch, n, yd, n, pk)
    torch.cuda.synchronize()
    y = yd.cpu().numpy()
    peaks = pk.cpu().numpy()
    del xd, yd
    for c in range(nch):
        assert np.isfinite(y[c]).all()
        assert peaks[c] == np.abs(y[c]).max()
        if method == "direct":
            assert np.array_equal(y[c], ref[c])
            continue
        u = _ulps(y[c], ref[c])
        assert u.max() <= 1
        diff = np.nonzero(u)[0]
        # every output where the FFT and the FMA chain round differently:
        # within 1 ulp of the long-double value as well
        if diff.size:
            ld, _ = oracle_mod.filter_points(x[c], taps, diff[:20000], oracle_mod.MODE_LD)
            assert _ulps(y[c][diff[:20000]], ld).max() <= 1
        # RMS vs the long-double oracle: the FMA chain stands in for it except
        # at the differing outputs, where the long-double values are used
        d = y[c].astype(np.float64) - ref[c].astype(np.float64)
        if diff.size:
            ld_all, _ = oracle_mod.filter_points(x[c], taps, diff, oracle_mod.MODE_LD)
            d[diff] = y[c][diff].astype(np.float64) - ld_all.astype(np.float64)
        assert np.sqrt(np.mean(d * d)) <= RMS_TOL


@pytest.fixture(scope="module")
def config3(oracle_mod):
    import synth
    fs, n, nch = 96000.0, 5_760_000, 8
    taps = oracle_mod.design_lowcut(20.0, fs, 8001)
    x = synth.file_buffer(nch, n, fs, file=3, bits=None)  # float32 source
    ref = np.stack([oracle_mod.filter_channel_mt(x[c], taps, _cores(), oracle_mod.MODE_FMA)
                    for c in range(nch)])
    return x, taps, ref


@pytest.mark.slow
@pytest.mark.parametrize("method", ["direct", "fft"])
def test_config3_every_sample(tt, oracle_mod, config3, method):
    """Config 3 (60 s of 8-channel 96 kHz float32, 8001 taps): every one of
    the 46.1 M outputs, with config 2's bars (direct bit-exact against the
    FMA chain; FFT within 1 ulp of it, every difference within 1 ulp of the
    long-double value, RMS <= 1e-9) and the fused per-channel peaks."""
    torch, lc = tt
    x, taps, ref = config3
    nch, n = x.shape
    flt = lc.Filter(taps, method=method)
    xd = torch.from_numpy(x).cuda()
    yd = torch.empty_like(xd)
    pk = torch.zeros(nch, dtype=torch.float32, device="cuda")
    flt.filter_channels_dev(xd, n, nch, n, yd, n, pk)
    torch.cuda.synchronize()
    y = yd.cpu().numpy()
    peaks = pk.cpu().numpy()
    del xd, yd
    for c in range(nch):
        assert np.isfinite(y[c]).all()
        assert peaks[c] == np.abs(y[c]).max()
        if method == "direct":
            assert np.array_equal(y[c], ref[c])
            continue
        u = _ulps(y[c], ref[c])
        assert u.max() <= 1
        diff = np.nonzero(u)[0]
        d = y[c].astype(np.float64) - ref[c].astype(np.float64)
        if diff.size:
            ld, _ = oracle_mod.filter_points(x[c], taps, diff, oracle_mod.MODE_LD)
            assert _ulps(y[c][diff], ld).max() <= 1
            d[diff] = y[c][diff].astype(np.float64) - ld.astype(np.float64)
        assert np.sqrt(np.mean(d * d)) <= RMS_TOL


def _positions(n, half, k, seed):
    rng = np.random.default_rng(seed)
    edges = np.r_[np.arange(0, half + 64), np.arange(n - half - 64, n)]
    return np.unique(np.r_[edges, rng.integers(0, n, k)])


@pytest.mark.slow
def test_configs_4_and_5_batch(tt, oracle_mod):
    """One GPU, the bench's batch driver over 8 x 60-min stereo int24 files
    (two generated files reused, as bench.py does), without and with
    --normalize; every file has its own input and output buffers."""
    torch, lc = tt
    import batch
    import synth
    fs, n, nch, nfiles = 48000.0, 172_800_000, 2, 8
    taps = oracle_mod.design_lowcut(20.0, fs, oracle_mod.lowcut_ntaps(48.0, fs))
    half = (taps.size - 1) // 2
    src = [synth.file_buffer(nch, n, fs, file=k, bits=24) for k in range(2)]
    # file 1 is made loud (peak > 1 after filtering): ProcessFile.cp:98 rescales
    # it even without --normalize
    src[1] = (src[1] * np.float32(3.0)).astype(np.float32)
    dev = torch.device("cuda", 0)
    flt = lc.Filter(taps)
    assert flt.method == "fft"
    refs = {}
    for k in range(2):
        for c in range(nch):
            idx = _positions(n, half, 2048, 50 + 10 * k + c)
            refs[(k, c)] = (idx, oracle_mod.filter_points(src[k][c], taps, idx, oracle_mod.MODE_LD)[0])

    def run(normalize):
        be = batch.DeviceBackend(flt, dev)
        r = batch.BatchRunner(be, 0, 1, [n] * nfiles, nch, half, normalize, "file")
        r.prepare(lambda f, lo, hi: src[f % 2][:, lo:hi])
        r.step()
        return r

    r4 = run(False)
    res4 = r4.results()
    peaks4 = r4.peaks.cpu().numpy()
    assert [sh.file for sh, _ in res4] == list(range(nfiles))
    pre = {}  # un-normalized outputs of the quiet files, the loud ones' peaks
    for sh, y in res4:
        k = sh.file % 2
        yh = y.cpu().numpy()
        if k == 0:
            # quiet: peak <= 1, the output is the filter's; its peak over both channels
            assert peaks4[sh.file] == float(y.abs().max()) <= 1.0
            for c in range(nch):
                idx, ref = refs[(k, c)]
                d = yh[c][idx].astype(np.float64) - ref
                assert np.sqrt(np.mean(d * d)) <= RMS_TOL
                assert _ulps(yh[c][idx], ref).max() <= 1
            pre[sh.file] = y
        else:
            # loud: rescaled by 1/peak even without --normalize (peak > 1)
            assert peaks4[sh.file] > 1.0
            gain = 1.0 / float(np.float32(peaks4[sh.file]))
            for c in range(nch):
                idx, ref = refs[(k, c)]
                want = (ref.astype(np.float32).astype(np.float64) * gain).astype(np.float32)
                assert _ulps(yh[c][idx], want).max() <= 1
            assert float(y.abs().max()) <= 1.0
        del yh
    # all four copies of each source file are the same bits (no cross-file state)
    for f in range(2, nfiles):
        assert torch.equal(res4[f][1], res4[f % 2][1])
    del res4

    s0 = flt.nrm_stats
    r5 = run(True)
    peaks5 = r5.peaks.cpu().numpy()
    assert np.array_equal(peaks5, peaks4)  # the per-file peak, pre-normalize
    for sh, y in r5.results():
        if sh.file % 2 == 0:
            # every sample: (float)((double)y * (1 / peak_file)) of the config-4 output
            gain = 1.0 / float(np.float32(peaks5[sh.file]))
            want = (pre[sh.file].double() * gain).float()
            assert torch.equal(y, want)
        else:
            # loud files: config 4 rescaled them already; --normalize gives the same
            assert torch.equal(y, r4.results()[sh.file][1])
    # every file's normalize but the last rode in the next file's filter launch
    # (a 60-min file's slice fits the fused form on both FFT kernels)
    s1 = flt.nrm_stats
    assert s1["fused"] - s0["fused"] >= nfiles - 1 and s1["separate"] == s0["separate"], (s0, s1)
    del r5
    # config 5's per-rank shape at N = 8: one file per rank with the peak
    # exchange in every step (force_exchange; the all-reduce is the identity at
    # world 1, test_gpu_batch.py runs it through RCCL), each step's normalize
    # carried by the next step's filter launch (BatchRunner defer); results()
    # runs the last one.  Every sample as the per-file rule gives it.
    be = batch.DeviceBackend(flt, dev)
    r = batch.BatchRunner(be, 0, 1, [n], nch, half, True, "file", allreduce_max=lambda t: None,
                          force_exchange=True)
    assert r.defer
    r.prepare(lambda f, lo, hi: src[0][:, lo:hi])
    s0 = flt.nrm_stats
    for _ in range(3):
        r.step()
    (sh, y), = r.results()
    s1 = flt.nrm_stats
    assert s1["fused"] - s0["fused"] >= 2 and s1["separate"] == s0["separate"], (s0, s1)
    assert float(r.peaks[0].item()) == peaks4[0]
    gain = 1.0 / float(np.float32(peaks4[0]))
    assert torch.equal(y, (pre[0].double() * gain).float())
    r.close()

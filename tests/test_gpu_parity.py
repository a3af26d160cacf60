"""GPU parity: the HIP path, called through the C ABI, against the oracle.

Bars (written here, used below):
  * METHOD direct: bit-exact against the oracle's strict-order f64 FMA chain
    (ORACLE_FMA) -- same accumulation order and rounding, so any difference is
    a bug;
  * every method: RMS(y_gpu - y_longdouble) <= 1e-9 in full-scale units
    (BASELINE.json north_star), and at most 1 ulp(f32) per sample (samples
    within 1e-12 of the reference are exempt from the ulp count).
"""
import threading

import numpy as np
import pytest

from conftest import golden_names, load_golden

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-9
METHODS = ["direct", "fft"]
# Golden cases whose exact outputs sit ON f32 rounding ties (taps with few
# significant bits: 0.75 * x needs 26 bits).  Any method that is not exact in
# f64 (the FFT: error ~1e-16) may round those ties either way; AUTO uses the
# direct method for such filters (short tap counts).
TIE_PRONE = {"single_tap"}


def is_f32_tie(v):
    """True if the f64 value v lies exactly half-way between two f32 values."""
    a = np.float32(v)
    if float(a) == v:
        return False
    b = np.nextafter(a, np.float32(np.inf) if v > float(a) else np.float32(-np.inf))
    return 2.0 * v == float(a) + float(b)


@pytest.fixture(scope="module")
def lc():
    import lcfir
    assert lcfir.device_count() >= 1, "no GPU visible"
    return lcfir


def rms(a, b):
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    return float(np.sqrt(np.mean(d * d))) if d.size else 0.0


def max_ulps(a, b, floor=1e-12):
    """Largest f32 ulp distance between a and b, ignoring pairs that agree to
    `floor` in absolute value (ulps are meaningless around 0, e.g. the DC case)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    close = np.abs(a.astype(np.float64) - b.astype(np.float64)) <= floor
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    d = np.where(close, 0, np.abs(ia - ib))
    return int(d.max()) if a.size else 0


def make_filter(lc, taps, method):
    """Filter with the requested method; skip if the method cannot take this tap count."""
    try:
        return lc.Filter(taps, method=method)
    except lc.LcfirError as e:
        if method != "direct" and e.code == lc.EINVAL:
            pytest.skip(f"{method} does not support {len(taps)} taps")
        raise


def gpu_filter_channels(lc, flt, x):
    """Run lcfir_filter_channels_dev on a [nch][n] host array; returns (y, peaks)."""
    x = np.ascontiguousarray(x, np.float32)
    nch, n = x.shape
    dx = lc.DeviceBuffer.from_array(x)
    dy = lc.DeviceBuffer(max(1, x.nbytes))
    dpk = lc.DeviceBuffer(4 * nch)
    lc.peak_reset_dev(dpk, nch)
    flt.filter_channels_dev(dx, n, nch, n, dy, n, dpk)
    lc.sync()
    y = dy.download((nch, n))
    pk = dpk.download(nch)
    for b in (dx, dy, dpk):
        b.free()
    return y, pk


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("name", golden_names())
def test_golden_vectors(lc, oracle_mod, name, method):
    g = load_golden(name)
    flt = make_filter(lc, g["taps"], method)
    y, pk = gpu_filter_channels(lc, flt, g["x"])
    for c in range(g["x"].shape[0]):
        assert max_ulps(y[c], g["y"][c]) <= 1
        if method == "fft" and name in TIE_PRONE:
            # every mismatch must be an exact f32 rounding tie of the exact sum
            bad = np.nonzero(y[c] != g["y"][c])[0]
            assert all(is_f32_tie(g["y64"][c][i]) for i in bad)
        else:
            assert rms(y[c], g["y"][c]) <= RMS_TOL
        if method == "direct":
            ref = oracle_mod.filter_channel(g["x"][c], g["taps"], oracle_mod.MODE_FMA)
            assert np.array_equal(y[c], ref), f"channel {c}: direct kernel not bit-exact"
        assert pk[c] == np.abs(y[c]).max()


@pytest.mark.parametrize("method", METHODS)
@pytest.mark.parametrize("threads", [1, 2, 3, 8])
def test_chunk_handoff_threads(lc, oracle_mod, method, threads):
    """ProcessFile.cp:60-83: N host threads, disjoint [start,end), one channel."""
    g = load_golden("random_int24")
    flt = make_filter(lc, g["taps"], method)
    prog = lc.ThreadSafeProgress(g["x"].shape[1])
    y = lc.filter_channel(g["x"][0], flt, threads, prog)
    assert prog.count == g["x"].shape[1]
    ref = oracle_mod.filter_channel(g["x"][0], g["taps"], oracle_mod.MODE_FMA)
    if method == "direct":
        assert np.array_equal(y, ref)
    assert rms(y, g["y"][0]) <= RMS_TOL


@pytest.mark.parametrize("method", METHODS)
def test_apply_range_writes_only_its_range(lc, oracle_mod, method):
    g = load_golden("ragged_taps")
    x, taps = g["x"][0], g["taps"]
    flt = make_filter(lc, taps, method)
    n = x.size
    for (s, e) in [(0, 1), (0, 1955), (1954, 1957), (3000, 7000), (n - 5, n), (n, n), (17, 18)]:
        y = np.full(n, np.float32(7.0))
        lc.apply_filter_range(x, flt, y, s, e)
        assert np.all(y[:s] == 7.0) and np.all(y[e:] == 7.0)
        ref = oracle_mod.filter_channel(x, taps, oracle_mod.MODE_FMA)
        if method == "direct":
            assert np.array_equal(y[s:e], ref[s:e])
        assert rms(y[s:e], g["y"][0][s:e]) <= RMS_TOL


@pytest.mark.parametrize("method", METHODS)
def test_apply_range_dev(lc, oracle_mod, method):
    g = load_golden("float_source")
    x, taps = g["x"][3], g["taps"]
    flt = make_filter(lc, taps, method)
    n = x.size
    dx = lc.DeviceBuffer.from_array(x)
    dy = lc.DeviceBuffer.from_array(np.zeros(n, np.float32))
    for (s, e) in [(0, 700), (700, 2999), (2999, 3000)]:
        flt.apply_range_dev(dx, n, dy, s, e)
    lc.sync()
    y = dy.download(n)
    assert rms(y, g["y"][3]) <= RMS_TOL
    if method == "direct":
        assert np.array_equal(y, oracle_mod.filter_channel(x, taps, oracle_mod.MODE_FMA))


@pytest.mark.parametrize("kind", ["direct", "sym", "general", "parts"])
def test_partition_invariance(lc, oracle_mod, kind):
    """SURVEY.md s4's partition invariance (ProcessFile.cp:60-83): the output
    does not depend on how a channel is split into ranges.  The reference's
    per-thread chunk hand-off at 1-64 threads (host-pointer ranges, each a
    concurrent lcfir_apply_range), ragged device ranges (lcfir_apply_range_dev)
    and the whole-channel launch give the same bytes: the direct method by its
    fixed FMA order, the FFT by its segment grid anchored at output 0 of the
    channel (fir_fft.hpp fft_grid_start)."""
    import synth
    n = 150_001
    ntaps = {"direct": 801, "sym": 4001, "general": 4003, "parts": 19201}[kind]
    taps = oracle_mod.design_lowcut(30.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method="direct" if kind == "direct" else "fft")
    x = synth.file_buffer(1, n, 48000.0, file=9, bits=24)
    y, _ = gpu_filter_channels(lc, flt, x)
    for threads in (1, 2, 3, 7, 64):
        assert np.array_equal(lc.filter_channel(x[0], flt, threads), y[0]), threads
    rng = np.random.default_rng(ntaps)
    cuts = np.unique(np.r_[0, rng.integers(1, n, 9), 12_384, 12_385, n])
    dx = lc.DeviceBuffer.from_array(x[0])
    dy = lc.DeviceBuffer.from_array(np.zeros(n, np.float32))
    for s_, e_ in zip(cuts[:-1], cuts[1:]):
        flt.apply_range_dev(dx, n, dy, int(s_), int(e_))
    lc.sync()
    assert np.array_equal(dy.download(n), y[0])
    dx.free()
    dy.free()
    idx = _sample_positions(n, ntaps // 2, 1024, 77)
    ref, _ = oracle_mod.filter_points(x[0], taps, idx, oracle_mod.MODE_LD)
    assert rms(y[0][idx], ref) <= RMS_TOL and max_ulps(y[0][idx], ref) <= 1


@pytest.mark.parametrize("ntaps", [4001, 4003, 19201])
def test_adversarial_inputs(lc, oracle_mod, ntaps):
    """Full-scale inputs that stress the FFT's dynamic range, against the
    long-double oracle at every edge sample plus random positions (RMS <= 1e-9,
    <= 1 f32 ulp with the 1e-12 floor for outputs that cancel to ~0):
    Nyquist (+-1 alternating: passes the low-cut at full gain), full-scale DC
    (cancels to ~0 in the interior), the sign-matched input that drives one
    output to sum|h| (the largest any +-1 input can reach), a full-scale square
    wave at the cutoff, and isolated full-scale impulses at both edges."""
    n = 60_001
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    half = (ntaps - 1) // 2
    k = np.arange(n)
    matched = np.ones(n)
    n0 = n // 2
    matched[n0 - half:n0 - half + ntaps] = np.where(taps >= 0, 1.0, -1.0)
    square = np.where((k // 1200) % 2 == 0, 1.0, -1.0)  # 20 Hz at 48 kHz
    edges = np.zeros(n)
    edges[[0, 1, n - 2, n - 1]] = [1.0, -1.0, -1.0, 1.0]
    x = np.stack([(-1.0) ** k, np.full(n, 1.0 - 2.0 ** -23), matched, square, edges]).astype(np.float32)
    flt = lc.Filter(taps, method="fft")
    y, pk = gpu_filter_channels(lc, flt, x)
    for c in range(x.shape[0]):
        idx = _sample_positions(n, half, 1024, 40 + c)
        if c == 2:
            idx = np.unique(np.r_[idx, n0 - 2:n0 + 3])
        ref, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref) <= RMS_TOL, c
        assert max_ulps(y[c][idx], ref) <= 1, c
        assert pk[c] == np.abs(y[c]).max(), c
    assert abs(float(y[2][n0]) - float(np.abs(taps).sum())) <= 1e-6 * float(np.abs(taps).sum())


def test_concurrent_contexts_and_threads(lc, oracle_mod):
    """Several filters used from several threads at once (re-entrancy)."""
    g1, g2 = load_golden("random_int24"), load_golden("sine")
    f1, f2 = lc.Filter(g1["taps"]), lc.Filter(g2["taps"])
    out = {}

    def job(key, flt, x):
        out[key] = lc.filter_channel(x, flt, 3)

    ts = [threading.Thread(target=job, args=(i, f, gg["x"][0]))
          for i, (f, gg) in enumerate([(f1, g1), (f2, g2), (f1, g1), (f2, g2)])]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for i, gg in enumerate([g1, g2, g1, g2]):
        assert rms(out[i], gg["y"][0]) <= RMS_TOL


def test_errors_are_reported(lc):
    flt = lc.Filter(np.ones(3))
    x = np.zeros(10, np.float32)
    y = np.zeros(10, np.float32)
    with pytest.raises(lc.LcfirError) as e:
        flt.apply_range(x, y, 5, 11)
    assert e.value.code == lc.EINVAL
    with pytest.raises(lc.LcfirError):
        flt.apply_range(x, y, 6, 5)
    d = lc.DeviceBuffer.from_array(np.zeros(100, np.float32))
    with pytest.raises(lc.LcfirError) as e:  # in-place (aliasing) is rejected
        flt.apply_range_dev(d, 100, d, 0, 100)
    assert "alias" in str(e.value)
    with pytest.raises(lc.LcfirError):
        lc.Filter(np.ones(3), device=99)


def test_empty_and_degenerate(lc):
    flt = lc.Filter(np.array([2.0]))
    y, pk = gpu_filter_channels(lc, flt, np.zeros((1, 0), np.float32))
    assert y.size == 0
    x = np.array([[0.25, -0.5, 1.0]], np.float32)
    y, pk = gpu_filter_channels(lc, flt, x)
    assert np.array_equal(y, 2 * x) and pk[0] == 2.0


def test_peak_and_normalize_match_processfile(lc, oracle_mod):
    """ProcessFile.cp:91-101 post-pass on the device vs the oracle."""
    g = load_golden("random_int24")
    flt = lc.Filter(g["taps"], method="direct")
    for gain, force in [(1.0, False), (1.0, True), (3.0, False)]:
        x = np.ascontiguousarray(g["x"] * np.float32(gain))
        nch, n = x.shape
        dx = lc.DeviceBuffer.from_array(x)
        dy = lc.DeviceBuffer(x.nbytes)
        dpk = lc.DeviceBuffer(4 * nch)
        lc.peak_reset_dev(dpk, nch)
        flt.filter_channels_dev(dx, n, nch, n, dy, n, dpk)
        lc.normalize_dev(dy, n, nch, n, dpk, nch, force)
        lc.sync()
        y = dy.download((nch, n))
        ref = x.copy()
        peak = oracle_mod.process_buffer(ref, g["taps"], nthreads=2, normalize=force)
        assert np.array_equal(y, ref), (gain, force)
        assert np.isclose(dpk.download(nch).max(), peak, rtol=0, atol=0)
        # standalone peak kernel agrees with the fused one
        dpk2 = lc.DeviceBuffer(4 * nch)
        lc.peak_reset_dev(dpk2, nch)
        flt.filter_channels_dev(dx, n, nch, n, dy, n, None)
        lc.peak_dev(dy, n, nch, n, dpk2)
        lc.sync()
        assert np.array_equal(dpk2.download(nch), dpk.download(nch))
    assert lc.channel_peak(g["y"][0]) == np.abs(g["y"][0]).max()


def _sample_positions(n, half, k, seed):
    rng = np.random.default_rng(seed)
    edges = np.r_[np.arange(0, min(n, half + 64)), np.arange(max(0, n - half - 64), n)]
    rand = rng.integers(0, n, k)
    blocks = np.r_[[4095, 4096, 4097, 8191, 8192]]
    return np.unique(np.r_[edges, rand, blocks[blocks < n]])


@pytest.mark.slow
@pytest.mark.parametrize("method", METHODS)
def test_config2_full_size(lc, oracle_mod, method):
    """Config 2 at full size (10 min stereo 48 kHz int24, 4001 taps) through
    filter_channels_dev; checked at every edge sample plus 4096 random positions
    per channel against the oracle, and the fused peak against the output."""
    import synth
    fs, n, nch = 48000.0, 28_800_000, 2
    taps = oracle_mod.design_lowcut(20.0, fs, oracle_mod.lowcut_ntaps(48.0, fs))
    assert taps.size == 4001
    x = synth.file_buffer(nch, n, fs, file=0, bits=24)
    flt = make_filter(lc, taps, method)
    y, pk = gpu_filter_channels(lc, flt, x)
    for c in range(nch):
        idx = _sample_positions(n, 2000, 4096, 100 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL
        assert max_ulps(y[c][idx], ref_ld) <= 1
        if method == "direct":
            ref_fma, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_FMA)
            assert np.array_equal(y[c][idx], ref_fma)
        assert pk[c] == np.abs(y[c]).max()
        assert np.isfinite(y[c]).all()


@pytest.mark.slow
@pytest.mark.parametrize("method", METHODS)
def test_config3_full_size(lc, oracle_mod, method):
    """Config 3: 8 channels x 96 kHz float32 (60 s), 8001 taps (LDS / long-kernel stress)."""
    import synth
    fs, n, nch = 96000.0, 5_760_000, 8
    taps = oracle_mod.design_lowcut(20.0, fs, 8001)
    x = synth.file_buffer(nch, n, fs, file=1, bits=None)
    flt = make_filter(lc, taps, method)
    y, pk = gpu_filter_channels(lc, flt, x)
    for c in range(nch):
        idx = _sample_positions(n, 4000, 1024, 200 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL
        assert max_ulps(y[c][idx], ref_ld) <= 1
        if method == "direct":
            ref_fma, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_FMA)
            assert np.array_equal(y[c][idx], ref_fma)
        assert pk[c] == np.abs(y[c]).max()


@pytest.mark.slow
@pytest.mark.parametrize("method,ntaps", [("fft", 4001), ("direct", 31)])
def test_channel_beyond_2gib(lc, oracle_mod, method, ntaps):
    """One channel of 2^29 + 4097 samples (2.15 GB of f32): past the 32-bit
    byte range of buffer offsets.  The FFT splits the launch (fir_fft.hpp
    fft_chunk, 2^28 outputs); the direct kernel rebases its load resource at
    every stage and walks 64-bit tile indices.  Checked against the oracle at
    both edges, around both 2^28 / 2^29 seams and at random positions (long
    double for the FFT, bit for bit against the strict fma chain for the
    direct form); the fused peak against the full output."""
    n = (1 << 29) + 4097
    rng = np.random.default_rng(29)
    x = (rng.standard_normal(n, dtype=np.float32) * np.float32(0.2))[None, :]
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method=method)
    y, pk = gpu_filter_channels(lc, flt, x)
    seams = np.r_[[(1 << 28) + d for d in range(-40, 40)], [(1 << 29) + d for d in range(-40, 40)]]
    idx = np.unique(np.r_[_sample_positions(n, ntaps // 2, 2048, 29), seams])
    if method == "direct":
        ref, _ = oracle_mod.filter_points(x[0], taps, idx, oracle_mod.MODE_FMA)
        assert np.array_equal(y[0][idx], ref)
    else:
        ref_ld, _ = oracle_mod.filter_points(x[0], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[0][idx], ref_ld) <= RMS_TOL
        assert max_ulps(y[0][idx], ref_ld) <= 1
    assert pk[0] == np.abs(y[0]).max()
    assert np.isfinite(y[0]).all()


# ---- long filters: the FFT method in partitions (fir_fft.hpp fft_partition_count)
@pytest.mark.parametrize("ntaps", [10925, 19201, 38401, 100001])
def test_fft_partitioned_long_filters(lc, oracle_mod, ntaps):
    """Filters longer than one overlap-save segment favours run as P equal
    partitions summed in f64 (10 925: 2 partitions just past the cost
    crossover; 19 201: config 1's kernel; 38 401, 100 001: more partitions).
    Whole channels through filter_channels_dev and a sub-range through
    filter_window, against the long-double oracle at every edge sample and
    random positions; the fused peak against the output."""
    import synth
    fs, n, nch = 48000.0, 300_000, 2
    taps = oracle_mod.design_lowcut(20.0, fs, ntaps)
    x = synth.file_buffer(nch, n, fs, file=5, bits=24)
    flt = lc.Filter(taps, method="fft")
    y, pk = gpu_filter_channels(lc, flt, x)
    for c in range(nch):
        idx = _sample_positions(n, ntaps // 2, 2048, 300 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL
        assert max_ulps(y[c][idx], ref_ld) <= 1
        assert pk[c] == np.abs(y[c]).max()
    # a sub-range from only the input window it needs (a file sharded by sample
    # range): every partition's shifted reads must stay inside that window
    half = (ntaps - 1) // 2
    for start, end in [(12_345, n - 23_456), (half + 7, half + 70_007), (n - 5_000, n)]:
        check_window(lc, flt, x, y, start, end)


def check_window(lc, flt, x, y, start, end):
    """Outputs [start, end) of a windowed call against the whole-channel
    outputs y: bit for bit from lcfir_ctx_window's window (the FFT's whole
    segments), within 1 f32 ulp from the narrowest window the outputs need
    (its edge segments read zeros where the whole channel has samples)."""
    n = x.shape[1]
    half = (flt.ntaps - 1) // 2
    lo, hi = flt.window(n, start, end)
    assert lo <= max(0, start - half) and hi >= min(n, end + half)
    yw = gpu_filter_window(lc, flt, x, start, end, lo, hi)
    assert np.array_equal(yw, y[:, start:end]), (start, end, lo, hi)
    yn = gpu_filter_window(lc, flt, x, start, end, max(0, start - half), min(n, end + half))
    assert max_ulps(yn, y[:, start:end]) <= 1 and rms(yn, y[:, start:end]) <= RMS_TOL, (start, end)


def gpu_filter_window(lc, flt, x, start, end, x_lo, x_hi):
    """Outputs [start, end) of every channel through lcfir_filter_window_dev,
    given only the samples [x_lo, x_hi) of each channel."""
    nch, n = x.shape
    xw = np.ascontiguousarray(x[:, x_lo:x_hi], np.float32)
    dx = lc.DeviceBuffer.from_array(xw)
    dy = lc.DeviceBuffer(4 * nch * (end - start))
    flt.filter_window_dev(dx, x_lo, x_hi, x_hi - x_lo, n, nch, dy, start, end - start, start, end)
    lc.sync()
    y = dy.download((nch, end - start))
    dx.free()
    dy.free()
    return y


def test_fft_partitioned_chunk_seams(lc, oracle_mod):
    """A partitioned filter with launches split into 65 536-output chunks
    (lcfir_ctx_set_fft_tuning chunk): the f64 partial-sum scratch restarts at
    every seam.  Bit-identical to the unchunked launch, and checked around each
    seam against the long-double oracle."""
    import synth
    n, chunk = 400_000, 65_536
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 19201)
    x = synth.file_buffer(1, n, 48000.0, file=6, bits=24)
    y_one, pk_one = gpu_filter_channels(lc, lc.Filter(taps, method="fft"), x)
    flt = lc.Filter(taps, method="fft")
    flt.set_fft_tuning(chunk=chunk)
    y, pk = gpu_filter_channels(lc, flt, x)
    y, pk, x = y[0], pk[0], x[0]
    # chunks are whole segments of the channel's grid: the unchunked launch
    # gives the same bytes
    assert np.array_equal(y, y_one[0]) and pk == pk_one[0]
    seams = np.r_[[s + o for s in range(chunk, n, chunk) for o in range(-3, 3)]]
    idx = np.unique(np.r_[_sample_positions(n, 9600, 512, 61), seams])
    ref_ld, _ = oracle_mod.filter_points(x, taps, idx, oracle_mod.MODE_LD)
    assert rms(y[idx], ref_ld) <= RMS_TOL
    assert max_ulps(y[idx], ref_ld) <= 1
    assert pk == np.abs(y).max()


@pytest.mark.parametrize("max_units", [7, 20])
def test_fft_channel_groups(lc, max_units):
    """The kernels index units in 32 bits, so fft_launch splits a launch into
    channel groups of at most 2^31 - 1 units (fir_fft.hpp FftGrid).  The
    max_units tuning forces the split at small sizes -- one channel per launch
    (7) and groups of two (20, 9 segments per channel) -- for a zero-phase and
    a partitioned filter, with per-channel peaks: every output and peak
    bit-identical to one launch."""
    import synth
    nch, n = 5, 100_000
    x = synth.file_buffer(nch, n, 48000.0, file=8, bits=24)
    for taps in (lc.design_lowcut(20.0, 4.0, 48000.0), lc.design_lowcut(20.0, 10.0, 48000.0)):
        y0, pk0 = gpu_filter_channels(lc, lc.Filter(taps, method="fft"), x)
        flt = lc.Filter(taps, method="fft")
        flt.set_fft_tuning(max_units=max_units)
        y1, pk1 = gpu_filter_channels(lc, flt, x)
        assert np.array_equal(y0, y1) and np.array_equal(pk0, pk1)
        assert np.all(pk0 > 0)


# ---- linear-phase filters: the zero-phase form (fir_fft.hpp fft_sym_eligible)
@pytest.mark.parametrize("ntaps,perturb", [(4001, 0.0), (4001, 1e-9), (4003, 0.0), (801, 0.0)])
def test_fft_zero_phase_form(lc, oracle_mod, ntaps, perturb):
    """Symmetric taps run in zero-phase form (real pair table, outputs c in
    [half, L - half); an odd half, 4 003 taps, makes the range's ends odd and
    takes the per-output store path); taps with a visible antisymmetric part
    run the general table.  Every form against the
    long-double oracle, sub-ranges against whole channels (the shifted output
    window), and the zero-phase form against the general one on the same
    filter (lcfir_ctx_set_fft_tuning zero_phase 0)."""
    import synth
    fs, n = 48000.0, 200_003
    taps = oracle_mod.design_lowcut(20.0, fs, ntaps)
    if perturb:
        taps = taps + perturb * np.linspace(-1.0, 1.0, ntaps)  # antisymmetric part >> 2^-50 |h|_1
    x = synth.file_buffer(2, n, fs, file=7, bits=24)
    flt = lc.Filter(taps, method="fft")
    y, _ = gpu_filter_channels(lc, flt, x)
    half = (ntaps - 1) // 2
    for c in range(2):
        idx = _sample_positions(n, half, 2048, 500 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL
        assert max_ulps(y[c][idx], ref_ld) <= 1
    for start, end in [(1, n - 1), (half - 1, half + 12_385), (77_777, 77_778), (n - 13_000, n)]:
        check_window(lc, flt, x, y, start, end)
    # the general pair table on the same filter (zero-phase form off)
    assert flt.fft_info["zero_phase"] == (perturb == 0.0)
    flt_g = lc.Filter(taps, method="fft")
    flt_g.set_fft_tuning(zero_phase=False)
    y_general, _ = gpu_filter_channels(lc, flt_g, x)
    assert not flt_g.fft_info["zero_phase"]
    assert max_ulps(y, y_general) <= 1
    assert rms(y, y_general) <= RMS_TOL


def test_staging_pool_cap_release_and_ctx_destroy(lc, oracle_mod):
    """lcfir_apply_range's staging pool: 40 concurrent range calls on one
    channel share at most 16 slots (the rest wait for one), the result is the
    one-range bytes; lcfir_staging_release frees every idle slot and its
    stream, later calls make new ones, and destroying the ctx afterwards does
    not touch the released streams (apply_range never registers them with the
    ctx).  A partitioned filter, so the ctx also kept per-stream scratch."""
    g = load_golden("random_int24")
    x = np.ascontiguousarray(g["x"][0], np.float32)
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 19201)
    flt = lc.Filter(taps, method="fft")
    whole = np.zeros_like(x)
    flt.apply_range(x, whole, 0, x.size)
    y = lc.filter_channel(x, flt, 40)
    assert np.array_equal(y, whole)
    live, idle = lc.staging_count(0)
    assert 1 <= live <= 16 and idle == live
    lc.staging_release(0)
    assert lc.staging_count(0) == (0, 0)
    assert np.array_equal(lc.filter_channel(x, flt, 5), whole)
    lc.staging_release(-1)
    flt.close()
    ref = oracle_mod.filter_channel(x, taps, oracle_mod.MODE_LD)
    assert rms(whole, ref) <= RMS_TOL and max_ulps(whole, ref) <= 1


# ---- the L = 32 768 segment (fir_fft32.hpp): both halves, every output form
@pytest.mark.parametrize("ntaps,perturb", [(4001, 0.0), (4003, 0.0), (8001, 0.0), (8001, 1e-9), (19201, 0.0),
                                           (38401, 0.0), (100001, 0.0)])
def test_fft_seg32_forms(lc, oracle_mod, ntaps, perturb):
    """The 32 768-sample segment (two 8192-point halves split by bin parity,
    park slab, radix-2 merge) forced by lcfir_ctx_set_fft_tuning, for the
    zero-phase (4001, 8001, 19201 taps: one partition; 4003: odd half, the
    per-output store path), general (8001 with a visible antisymmetric part)
    and partitioned (38401, 100001) forms: against the long-double oracle at every edge sample and
    random positions, within 1 ulp of the 16 384-sample segment, windowed calls
    bit-identical to the whole channel, the reference's thread hand-off
    bit-identical, peaks fused."""
    import synth
    fs, n = 48000.0, 300_001
    taps = oracle_mod.design_lowcut(20.0, fs, ntaps)
    if perturb:
        taps = taps + perturb * np.linspace(-1.0, 1.0, ntaps)
    x = synth.file_buffer(2, n, fs, file=11, bits=24)
    flt = lc.Filter(taps, method="fft")
    flt.set_fft_tuning(seg_len=32768)
    info = flt.fft_info
    assert info["seg_len"] == 32768
    assert info["zero_phase"] == (perturb == 0.0 and ntaps in (4001, 4003, 8001, 19201))
    y, pk = gpu_filter_channels(lc, flt, x)
    half = (ntaps - 1) // 2
    for c in range(2):
        idx = _sample_positions(n, half, 2048, 900 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL, c
        assert max_ulps(y[c][idx], ref_ld) <= 1, c
        assert pk[c] == np.abs(y[c]).max()
    f16 = lc.Filter(taps, method="fft")
    f16.set_fft_tuning(seg_len=16384)
    y16, _ = gpu_filter_channels(lc, f16, x)
    assert max_ulps(y, y16) <= 1 and rms(y, y16) <= RMS_TOL
    for start, end in [(1, n - 1), (half + 3, half + 40_000), (123_457, 123_458), (n - 33_000, n)]:
        check_window(lc, flt, x, y, start, end)
    for threads in (3, 7):
        assert np.array_equal(lc.filter_channel(x[0], flt, threads), y[0]), threads


def test_fft_seg32_chunks_and_groups(lc, oracle_mod):
    """The 32 768-sample segment under launch chunks of whole segments and
    channel groups (lcfir_ctx_set_fft_tuning chunk / max_units): bytes and
    peaks identical to one launch; a channel shorter than one segment and a
    one-sample channel."""
    import synth
    taps = oracle_mod.design_lowcut(20.0, 96000.0, 8001)
    x = synth.file_buffer(5, 200_003, 96000.0, file=12, bits=None)
    one = lc.Filter(taps, method="fft")
    one.set_fft_tuning(seg_len=32768)
    y0, pk0 = gpu_filter_channels(lc, one, x)
    for chunk, mu in [(70_000, 0), (0, 9), (50_000, 4)]:
        f = lc.Filter(taps, method="fft")
        f.set_fft_tuning(seg_len=32768, chunk=chunk, max_units=mu)
        y1, pk1 = gpu_filter_channels(lc, f, x)
        assert np.array_equal(y0, y1) and np.array_equal(pk0, pk1), (chunk, mu)
    for n in (20_000, 1):
        xs = np.ascontiguousarray(x[:2, :n])
        ys, _ = gpu_filter_channels(lc, one, xs)
        for c in range(2):
            ref = oracle_mod.filter_channel(xs[c], taps, oracle_mod.MODE_LD)
            assert max_ulps(ys[c], ref) <= 1 and rms(ys[c], ref) <= RMS_TOL, (n, c)


@pytest.mark.parametrize("ntaps,n,nch,want_L", [(12001, 3_000_000, 2, 32768), (19201, 48_000, 1, 32768),
                                                (8001, 600_000, 8, 32768), (4001, 600_000, 2, 32768),
                                                (3001, 600_000, 2, 16384)])
def test_fft_auto_seg_len(lc, oracle_mod, ntaps, n, nch, want_L):
    """The automatic segment length (fir_fft.hpp fft_choose_seg_len), a
    function of the taps: linear-phase filters from ~4 000 taps take the
    L = 32 768 segment on the register kernel (config 2's 4 001, config 3's
    8 001; 12 001 taps: one partition instead of two; config 1's 19 201 taps
    on its short channel too), 3 001 taps stay at 16 384.  The product path as
    it runs by default, against the long-double oracle at every edge sample
    and random positions, fused peaks."""
    import synth
    fs = 48000.0
    taps = oracle_mod.design_lowcut(20.0, fs, ntaps)
    x = synth.file_buffer(nch, n, fs, file=13, bits=24)
    flt = lc.Filter(taps, method="fft")
    y, pk = gpu_filter_channels(lc, flt, x)
    assert flt.fft_info["seg_len"] == want_L
    half = (ntaps - 1) // 2
    for c in range(min(nch, 2)):
        idx = _sample_positions(n, half, 1024, 1300 + c)
        ref_ld, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y[c][idx], ref_ld) <= RMS_TOL, c
        assert max_ulps(y[c][idx], ref_ld) <= 1, c
    assert np.array_equal(pk, np.abs(y).max(axis=1))


def test_fft_auto_seg_len_follows_the_channel(lc, oracle_mod):
    """The automatic choice is a function of the taps alone, not of the
    channel or of the first call's range: a ctx whose first call is a
    50 000-output range of a 3 M-sample channel (the reference's per-thread
    chunk, a rank's share of a split file) picks the same segment length as one
    whose first call is the whole channel, so the range's bytes equal the
    whole-channel call's."""
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 12001)
    n = 3_000_000
    x = np.ascontiguousarray(synth.file_buffer(1, n, 48000.0, file=14, bits=24)[0])
    whole = lc.Filter(taps, method="fft")
    y, _ = gpu_filter_channels(lc, whole, x[None, :])
    part = lc.Filter(taps, method="fft")
    dx = lc.DeviceBuffer.from_array(x)
    dy = lc.DeviceBuffer.from_array(np.zeros(n, np.float32))
    start, end = 1_234_567, 1_284_567
    part.apply_range_dev(dx, n, dy, start, end)
    lc.sync()
    yr = dy.download(n)
    dx.free()
    dy.free()
    assert whole.fft_info["seg_len"] == part.fft_info["seg_len"] == 32768
    assert np.array_equal(yr[start:end], y[0][start:end])


@pytest.mark.parametrize("ntaps", [8001, 10001, 19201])
def test_fft_plan_independent_of_first_call(lc, oracle_mod, ntaps):
    """the plan (segment length, partitions) is a function of the
    taps, so a ctx whose first call is lcfir_ctx_window (one channel assumed
    before), one whose first call is a 2-channel filter_channels launch of a
    short file and one asked fft_info first all run the same plan, and the
    window-first ctx's bytes equal the channels-first ctx's."""
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    n = 60_000  # short: the old shape model flipped 19 201 taps between lengths here
    x = synth.file_buffer(2, n, 48000.0, file=15, bits=24)
    chans = lc.Filter(taps, method="fft")
    y_ch, _ = gpu_filter_channels(lc, chans, x)
    win = lc.Filter(taps, method="fft")
    lo, hi = win.window(n, 0, n)
    info = lc.Filter(taps, method="fft")
    assert win.fft_info == chans.fft_info == info.fft_info
    y_win, _ = gpu_filter_channels(lc, win, x)
    assert np.array_equal(y_ch, y_win)
    assert (lo, hi) == (0, n)


# ---- the loads' zero padding at every window alignment
@pytest.mark.parametrize("method,ntaps,seg_len,zero_phase", [
    ("direct", 15, 0, True), ("direct", 97, 0, True), ("direct", 801, 0, True), ("direct", 4003, 0, True),
    ("fft", 4001, 16384, True), ("fft", 4003, 16384, True), ("fft", 4003, 16384, False),
    ("fft", 4005, 32768, True), ("fft", 4003, 32768, True), ("fft", 4003, 32768, False),
    ("fft", 19203, 16384, True)])
def test_edge_outputs_every_window_alignment(lc, oracle_mod, method, ntaps, seg_len, zero_phase):
    """Outputs next to a window edge: the whole channel's first and last T + 256
    outputs, and windowed calls whose window [x_lo, x_hi) starts d = 0..3
    samples before the first sample the outputs need (and ends d after the
    last).  Samples outside a window read as zeros through the loads'
    range-checked buffer resources ("negative" offsets are out of range), so
    every alignment of the window against the kernels' load offsets -- the
    sample pair straddling the window start, lanes whose first loads fall
    before it and later ones after -- is checked against the oracle: bit for
    bit (direct, strict fma order) or <= 1 ulp (FFT)."""
    n = 120_001
    rng = np.random.default_rng(ntaps + seg_len)
    # two channels: a tile or unit that stored past its range would land in
    # the next channel's outputs
    x = (rng.integers(-2**23, 2**23, size=(2, n)) / 2.0**23).astype(np.float32)
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    half = (ntaps - 1) // 2
    flt = lc.Filter(taps, method=method)
    if method == "fft":
        flt.set_fft_tuning(seg_len=seg_len, zero_phase=zero_phase)
    span = ntaps + 256  # every output whose taps reach past a window edge, and more
    cases = [(0, span, 0, n), (n - span, n, 0, n)]
    for d in range(4):
        s0 = 30_000 + 7 * d
        cases.append((s0, s0 + span, s0 - half - d, s0 + span + half + d))
    for start, end, x_lo, x_hi in cases:
        yw = gpu_filter_window(lc, flt, x, start, end, x_lo, x_hi)
        idx = np.arange(start, end)
        for c in range(2):
            if method == "direct":
                ref, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_FMA)
                assert np.array_equal(yw[c], ref), (c, start, x_lo)
            else:
                ref, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
                assert max_ulps(yw[c], ref) <= 1 and rms(yw[c], ref) <= RMS_TOL, (c, start, x_lo)


@pytest.mark.parametrize("method,ntaps", [("direct", 31), ("direct", 801), ("fft", 4001)])
def test_many_channels(lc, oracle_mod, method, ntaps):
    """300 channels in one call: more channels than the direct kernel's grid
    holds workgroups per channel (launch_direct caps it at 3 per CU split over
    the channels, so each channel gets one or two), and the FFT's channel x
    segment unit grid.  A sample of channels against the oracle (bit for bit
    for the direct form), every channel's fused peak against its output, and
    the channels' independence: a channel of zeros stays zeros."""
    nch, n = 300, 9_001
    rng = np.random.default_rng(300 + ntaps)
    x = (rng.integers(-2**23, 2**23, size=(nch, n)) / 2.0**23).astype(np.float32)
    x[17] = 0.0
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method=method)
    y, pk = gpu_filter_channels(lc, flt, x)
    assert not y[17].any() and pk[17] == 0.0
    for c in [0, 1, 150, 298, 299]:
        if method == "direct":
            ref = oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_FMA)
            assert np.array_equal(y[c], ref), c
        else:
            ref = oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_LD)
            assert max_ulps(y[c], ref) <= 1 and rms(y[c], ref) <= RMS_TOL, c
    assert np.array_equal(pk, np.abs(y).max(axis=1))


@pytest.mark.parametrize("method,ntaps,seg_len", [("direct", 31, 0), ("direct", 801, 0), ("fft", 4001, 16384),
                                                 ("fft", 4003, 16384), ("fft", 8001, 32768)])
def test_padded_channel_strides(lc, oracle_mod, method, ntaps, seg_len):
    """lcfir_filter_window_dev with channel strides wider than the window and
    the outputs (x_stride = window + 13, y_stride = count + 7, odd on
    purpose): the outputs byte-identical to the packed layout's, the padding
    of y never written (a sentinel survives), per-channel peaks equal."""
    nch, n = 3, 70_001
    rng = np.random.default_rng(ntaps + 7)
    x = (rng.integers(-2**23, 2**23, size=(nch, n)) / 2.0**23).astype(np.float32)
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    flt = lc.Filter(taps, method=method)
    if method == "fft":
        flt.set_fft_tuning(seg_len=seg_len)
    start, end = 12_345, 61_000
    lo, hi = flt.window(n, start, end)
    count = end - start
    y_ref, pk_ref = None, None
    for xs_pad, ys_pad in ((0, 0), (13, 7)):
        xs, ys = (hi - lo) + xs_pad, count + ys_pad
        xp = np.zeros((nch, xs), np.float32)
        xp[:, :hi - lo] = x[:, lo:hi]
        xp[:, hi - lo:] = 1e30  # never read
        dx = lc.DeviceBuffer.from_array(xp)
        dy = lc.DeviceBuffer.from_array(np.full((nch, ys), -7.0, np.float32))
        dpk = lc.DeviceBuffer(4 * nch)
        lc.peak_reset_dev(dpk, nch)
        flt.filter_window_dev(dx, lo, hi, xs, n, nch, dy, start, ys, start, end, dpk)
        lc.sync()
        y = dy.download((nch, ys))
        pk = dpk.download(nch)
        for b in (dx, dy, dpk):
            b.free()
        assert np.all(y[:, count:] == -7.0)
        if y_ref is None:
            y_ref, pk_ref = y[:, :count].copy(), pk
        else:
            assert np.array_equal(y[:, :count], y_ref) and np.array_equal(pk, pk_ref)
    ref, _ = oracle_mod.filter_points(x[1], taps, np.arange(start, end), oracle_mod.MODE_LD)
    assert max_ulps(y_ref[1], ref) <= 1 and rms(y_ref[1], ref) <= RMS_TOL


def test_fft_kernel_families(lc, oracle_mod):
    """lcfir_ctx_set_fft_family: the default runs config 2's 4 001 taps on
    the register kernel (fir_fft32r), LDS the park-slab kernel at the same
    L = 32 768, outputs within 1 ulp of each other and of the long-double
    oracle; round 5's experimental family 2 (fir_fft16r, now
    scripts/variants/r16/) and unknown families fail with LCFIR_EINVAL."""
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    x = synth.file_buffer(2, 200_003, 48000.0, file=41, bits=24)
    ys = {}
    for fam, kernel in (("default", "l32_reg"), ("lds", "l32_park")):
        flt = lc.Filter(taps, method="fft")
        if fam == "lds":  # its unit costs alone would pick L = 16 384 at 4 001 taps
            flt.set_fft_tuning(seg_len=32768)
        flt.set_fft_family(fam)
        assert flt.fft_info["seg_len"] == 32768 and flt.fft_units["kernel"] == kernel, fam
        ys[fam], _ = gpu_filter_channels(lc, flt, x)
    assert max_ulps(ys["default"], ys["lds"]) <= 1 and rms(ys["default"], ys["lds"]) <= RMS_TOL
    idx = _sample_positions(x.shape[1], 2000, 1024, 41)
    ref, _ = oracle_mod.filter_points(x[0], taps, idx, oracle_mod.MODE_LD)
    assert rms(ys["default"][0][idx], ref) <= RMS_TOL and max_ulps(ys["default"][0][idx], ref) <= 1
    flt = lc.Filter(taps, method="fft")
    for bad in (2, 3, -1):
        with pytest.raises(lc.LcfirError) as e:
            lc._check(lc.load().lcfir_ctx_set_fft_family(flt._ctx, bad))
        assert e.value.code == 1 and "family" in str(e.value)
    assert flt.fft_units["kernel"] == "l32_reg"  # a refused family leaves the plan alone

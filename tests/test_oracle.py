"""CPU tests of the oracle (the checker) against the golden vectors and an
independent exact-rational restatement of FilterCore.h:56-76.

The reference publishes no tests; these are the known-answer
tests s4 asks for: impulse -> taps, DC -> ~0 interior, passband sine ->
unity gain, zero-padded edges, partition invariance, N < M+1."""
import numpy as np
import pytest

from conftest import golden_names, load_golden


@pytest.mark.parametrize("name", golden_names())
def test_oracle_reproduces_golden(oracle_mod, name):
    g = load_golden(name)
    for c in range(g["x"].shape[0]):
        y, y64 = oracle_mod.filter_channel(g["x"][c], g["taps"], oracle_mod.MODE_LD, with_f64=True)
        assert np.array_equal(y, g["y"][c])
        assert np.array_equal(y64, g["y64"][c])


@pytest.mark.parametrize("name", ["impulse", "short_n_lt_t", "tiny", "single_tap"])
def test_golden_matches_exact_rationals(oracle_mod, name):
    g = load_golden(name)
    assert bool(g["exact"])
    x, taps = g["x"][0], g["taps"]
    ex = oracle_mod.exact_filter_range(x, taps, 0, x.size)
    ex32 = np.array([oracle_mod.fraction_to_f32(q) for q in ex], np.float32)
    assert np.array_equal(ex32, g["y"][0])


@pytest.mark.parametrize("N,T,start,end", [(300, 41, 0, 300), (300, 41, 17, 290),
                                           (60, 101, 5, 55), (1000, 201, 900, 1000)])
def test_three_loop_fma_chain_equals_exact(oracle_mod, N, T, start, end):
    rng = np.random.default_rng(N * 7 + T)
    x = rng.uniform(-1, 1, N).astype(np.float32)
    taps = rng.standard_normal(T)
    y = np.zeros(N, np.float32)
    oracle_mod.apply_filter_range(x, taps, y, start, end, oracle_mod.MODE_FMA)
    ex = oracle_mod.exact_filter_range(x, taps, start, end)
    ex32 = np.array([oracle_mod.fraction_to_f32(q) for q in ex], np.float32)
    assert np.array_equal(y[start:end], ex32)
    assert not y[:start].any() and not y[end:].any()  # only [start, end) written


def test_impulse_gives_centred_taps(oracle_mod):
    g = load_golden("impulse")
    taps, y = g["taps"], g["y"][0]
    half = (taps.size - 1) // 2
    # y[n] = h[128 + half - n]; the low-cut kernel is symmetric
    np.testing.assert_array_equal(y[128 - half:128 + half + 1], taps[::-1].astype(np.float32))
    assert not y[:128 - half].any() and not y[128 + half + 1:].any()


def test_dc_is_removed_in_the_interior(oracle_mod):
    g = load_golden("dc")
    half = (g["taps"].size - 1) // 2
    interior = g["y64"][0][half:-half]
    assert np.abs(interior).max() < 1e-12
    assert np.abs(g["y64"][0][:half]).max() > 1e-3  # zero-padded edge sees a step


def test_passband_sine_has_unity_gain(oracle_mod):
    g = load_golden("sine")
    half = (g["taps"].size - 1) // 2
    x, y = g["x"][0][half:-half], g["y64"][0][half:-half]
    assert np.abs(y - x).max() < 1e-3


@pytest.mark.parametrize("threads", [1, 2, 3, 7, 16])
def test_partition_invariance(oracle_mod, threads):
    """ProcessFile.cp:64-69 chunking cannot change any output."""
    g = load_golden("random_int24")
    for mode in (oracle_mod.MODE_FMA, oracle_mod.MODE_LD):
        y = oracle_mod.filter_channel_mt(g["x"][0], g["taps"], threads, mode)
        ref = oracle_mod.filter_channel(g["x"][0], g["taps"], mode)
        assert np.array_equal(y, ref)


def test_fma_chain_close_to_long_double(oracle_mod):
    g = load_golden("config1")
    y = oracle_mod.filter_channel_mt(g["x"][0], g["taps"], 8, oracle_mod.MODE_FMA)
    d = y.astype(np.float64) - g["y"][0]
    assert np.sqrt(np.mean(d * d)) <= 1e-9
    assert np.mean(y != g["y"][0]) < 1e-3


def test_tap_design(oracle_mod):
    fs = 48000.0
    assert oracle_mod.lowcut_ntaps(48.0, fs) == 4001   # configs 2 and 4
    assert oracle_mod.lowcut_ntaps(10.0, fs) == 19201  # config 1
    assert oracle_mod.lowcut_ntaps(96.0, 96000.0) == 4001
    taps = oracle_mod.design_lowcut(20.0, fs, 4001)
    assert abs(taps.sum()) < 1e-12                      # zero DC gain (low-cut)
    np.testing.assert_allclose(taps, taps[::-1], rtol=0, atol=1e-15)  # linear phase
    assert 0.99 < taps[2000] < 1.0


def test_process_buffer_normalize_rule(oracle_mod):
    """ProcessFile.cp:92-101: rescale iff peak > 1 or --normalize."""
    g = load_golden("random_int24")
    buf = g["x"].copy()
    peak = oracle_mod.process_buffer(buf, g["taps"], nthreads=2, normalize=False)
    assert peak < 1.0
    np.testing.assert_array_equal(buf[0], oracle_mod.filter_channel(g["x"][0], g["taps"],
                                                                     oracle_mod.MODE_FMA))
    buf2 = g["x"].copy()
    peak2 = oracle_mod.process_buffer(buf2, g["taps"], nthreads=2, normalize=True)
    assert peak2 == peak
    assert abs(max(np.abs(buf2).max(), 0) - 1.0) < 1e-6
    loud = (g["x"] * 3.0).astype(np.float32)
    oracle_mod.process_buffer(loud, g["taps"], nthreads=1, normalize=False)
    assert np.abs(loud).max() <= 1.0 + 1e-6

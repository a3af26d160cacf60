"""GPU test of the C++ drop-in (include/lcfir/FilterCore.hpp + ProcessBuffer.hpp):
the reference's ProcessFile.cp:57-101 structure (std::thread per chunk calling
apply_filter_range with the FilterCore.h signature) and the device-resident
variant, built by tests/cpp/Makefile, against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, load_golden

pytestmark = pytest.mark.gpu

DRIVER = os.path.join(ROOT, "tests", "cpp", "filtercore_driver")


@pytest.fixture(scope="module")
def driver():
    subprocess.run(["make", "-C", os.path.dirname(DRIVER)], check=True, capture_output=True)
    return DRIVER


def run(driver, tmp_path, x, taps, threads, mode, normalize):
    xi, ti, yo = tmp_path / "x.f32", tmp_path / "t.f64", tmp_path / "y.f32"
    np.ascontiguousarray(x, np.float32).tofile(xi)
    np.ascontiguousarray(taps, np.float64).tofile(ti)
    r = subprocess.run([driver, str(xi), str(ti), str(yo), str(x.shape[0]), str(x.shape[1]),
                        str(threads), str(mode), str(int(normalize))],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    peak = float(r.stdout.split()[1])
    return np.fromfile(yo, np.float32).reshape(x.shape), peak


@pytest.mark.parametrize("threads,mode,normalize", [(1, 0, False), (4, 0, False), (7, 0, True),
                                                    (1, 1, False), (1, 1, True), (3, 2, False),
                                                    (3, 3, False), (4, 4, False), (4, 5, True)])
def test_cpp_process_buffer(driver, tmp_path, oracle_mod, threads, mode, normalize):
    """Modes 2 and 3: a sinc whose data()/size() are not the fms() kernel
    (padded / reversed; the random_int24 taps are asymmetric) -- the drop-in
    must fall back to recovering the taps through fms().  Modes 4 and 5: the
    sinc object is rewritten in place between two files (same address, same
    data() pointer, other taps), through the direct and the fms() path -- the
    second file must use the new taps."""
    g = load_golden("random_int24")
    taps = g["taps"]
    if mode == 3:  # visibly asymmetric, so reversed taps filter differently
        taps = taps + 1e-3 * np.linspace(-1.0, 1.0, taps.size)
    y, peak = run(driver, tmp_path, g["x"], taps, threads, mode, normalize)
    ref = g["x"].copy()
    ref_peak = oracle_mod.process_buffer(ref, taps, nthreads=2, normalize=normalize,
                                         mode=oracle_mod.MODE_LD)
    d = y.astype(np.float64) - ref
    assert np.sqrt(np.mean(d * d)) <= 1e-9
    assert abs(peak - ref_peak) <= 1e-7 * ref_peak


DROPIN = os.path.join(ROOT, "tests", "cpp", "dropin_processfile")


@pytest.fixture(scope="module")
def dropin():
    subprocess.run(["make", "-C", os.path.dirname(DROPIN)], check=True, capture_output=True)
    return DROPIN


@pytest.mark.parametrize("golden", ["random_int24", "impulse"])
@pytest.mark.parametrize("threads", [1, 3, 8, 64])
def test_reference_call_shape(dropin, tmp_path, oracle_mod, threads, golden):
    """ProcessFile.cp:57-87 with apply_filter_range passed by name to std::thread
    (Diskerror::apply_filter_range of include/lcfir/FilterCore.h, reference
    parameter types), a WindowedSinc stand-in with only getMo2()/fms(): taps
    recovered through fms, every chunk a concurrent lcfir_apply_range call.
    random_int24 (401 taps) runs the FFT under AUTO, impulse (41 taps) the
    direct kernel, which must also match the strict fma chain bit for bit."""
    g = load_golden(golden)
    x, taps = g["x"], g["taps"]
    xi, ti, yo = tmp_path / "x.f32", tmp_path / "t.f64", tmp_path / "y.f32"
    np.ascontiguousarray(x, np.float32).tofile(xi)
    np.ascontiguousarray(taps, np.float64).tofile(ti)
    r = subprocess.run([dropin, str(xi), str(ti), str(yo), str(x.shape[0]), str(x.shape[1]),
                        str(threads)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = dict(line.split() for line in r.stdout.strip().splitlines())
    assert int(out["progress"]) == x.size  # every sample reported exactly once
    y = np.fromfile(yo, np.float32).reshape(x.shape)
    import lcfir
    flt = lcfir.Filter(taps)  # the drop-in's method choice (AUTO)
    for c in range(x.shape[0]):
        # partition invariance: any thread count gives the one-range bytes
        whole = np.zeros(x.shape[1], np.float32)
        flt.apply_range(np.ascontiguousarray(x[c], np.float32), whole, 0, x.shape[1])
        assert np.array_equal(y[c], whole), (threads, c)
        if flt.method == "direct":
            assert np.array_equal(y[c], oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_FMA)), c
        ref = oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_LD)
        d = y[c].astype(np.float64) - ref
        assert np.sqrt(np.mean(d * d)) <= 1e-9
        assert np.all(np.abs(d) <= np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64))


BENCH = os.path.join(ROOT, "tests", "cpp", "dropin_bench")


def test_dropin_bench_short(dropin):
    """tests/cpp/dropin_bench (the drop-in's timing tool, profiles/) on a 4-s
    stereo file: both staging modes and pinned caller buffers, 1 and 5
    threads, every file bit-identical to the one-launch device call, the stats
    and the per-call split filled."""
    import json
    r = subprocess.run([BENCH, "--seconds", "4", "--threads", "1,5", "--reps", "1"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert [(d["mode"], d["threads"]) for d in lines] == [(m, t) for m in ("auto", "pageable", "bounce", "pinned")
                                                          for t in (1, 5)]
    for d in lines:
        assert d["bit_identical"] is True and d["msamples_per_s"] > 0 and d["ntaps"] == 4001
        assert d["calls_per_file"] == 2 * d["threads"]
        assert d["staged_calls_frac"] == (1.0 if d["mode"] == "bounce" else 0.0)
        assert d["fanout_msamples_per_s"] >= d["msamples_per_s"] and d["alloc_ms_per_file"] >= 0
        sp = d["split_per_call_ms"]
        assert sp["kernel"] > 0 and sp["h2d"] > 0 and sp["d2h"] > 0 and sp["wall"] > 0


@pytest.mark.parametrize("mode,ntaps", [("bounce", 4001), ("pageable", 4001), ("pageable", 41), ("auto", 4001)])
def test_apply_range_staging_modes(oracle_mod, mode, ntaps):
    """lcfir_apply_range through each staging mode and from pinned host
    memory (copied directly): ranges that span several 4 MiB bounce chunks,
    odd sizes and one-sample ranges, all equal to the device call's bytes
    (FFT at 4 001 taps, the direct form at 41)."""
    import lcfir
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    n = 3_000_001
    x = np.ascontiguousarray(synth.file_buffer(1, n, 48000.0, file=31, bits=24)[0])
    flt = lcfir.Filter(taps)
    dx = lcfir.DeviceBuffer.from_array(x)
    dy = lcfir.DeviceBuffer(4 * n)
    flt.apply_range_dev(dx, n, dy, 0, n)
    lcfir.sync()
    want = dy.download(n)
    lcfir.staging_set_mode(mode)
    try:
        lcfir.range_stats(reset=True)
        y = np.full(n, 7.0, np.float32)
        for start, end in [(0, 1_500_000), (1_500_000, 1_500_001), (1_500_001, n)]:
            flt.apply_range(x, y, start, end)
        assert np.array_equal(y, want)
        st = lcfir.range_stats(reset=True)
        assert st["calls"] == 3 and st["samples"] == n
        # bounce: every call; auto: the two 6 MB windows (the whole-window
        # bounce), not the one-sample call (the runtime's path)
        assert st["staged_calls"] == {"bounce": 3, "pageable": 0, "auto": 2}[mode]
        # pinned caller buffers: DMA straight from / to them
        import ctypes
        lib = lcfir.load()
        px, py = ctypes.c_void_p(), ctypes.c_void_p()
        assert lib.lcfir_host_malloc(4 * n, ctypes.byref(px)) == 0
        assert lib.lcfir_host_malloc(4 * n, ctypes.byref(py)) == 0
        try:
            hx = np.ctypeslib.as_array((ctypes.c_float * n).from_address(px.value))
            hy = np.ctypeslib.as_array((ctypes.c_float * n).from_address(py.value))
            hx[:] = x
            hy[:] = 7.0
            flt.apply_range(hx, hy, 0, n)
            assert np.array_equal(hy, want)
            assert lcfir.range_stats(reset=True)["staged_calls"] == 0
        finally:
            lib.lcfir_host_free(px)
            lib.lcfir_host_free(py)
        if mode == "bounce":
            # a caller range that starts in one pinned registration and ends in
            # another, pageable in between: not one page-locked allocation, so
            # it is staged (both ends pinned is not enough)
            import torch
            rt = torch.cuda.cudart()
            page = 1 << 16
            raw = np.zeros(n + 3 * page, np.float32)
            a0 = (-raw.ctypes.data) % page // 4
            hx = raw[a0:a0 + n]
            hx[:] = x
            lo_len = (page * 4) & ~(page - 1)
            hi_off = (4 * n - lo_len) & ~(page - 1)
            hi_len = (4 * n - hi_off + page - 1) & ~(page - 1)  # into raw's padding: whole pages
            regs = [(hx.ctypes.data, lo_len), (hx.ctypes.data + hi_off, hi_len)]
            done = []
            try:
                for ptr, ln in regs:
                    assert int(rt.cudaHostRegister(ptr, ln, 0)) == 0
                    done.append(ptr)
                y = np.full(n, 7.0, np.float32)
                flt.apply_range(hx, y, 0, n)
                assert np.array_equal(y, want)
                assert lcfir.range_stats(reset=True)["staged_calls"] == 1
            finally:
                for ptr in done:
                    rt.cudaHostUnregister(ptr)
    finally:
        lcfir.staging_set_mode("auto")  # the library's default
    idx = np.r_[np.arange(0, 20), np.arange(n - 20, n), np.arange(1000, n, 100_003)]
    ref, _ = oracle_mod.filter_points(x, taps, idx, oracle_mod.MODE_LD)
    d = want[idx].astype(np.float64) - ref
    assert np.sqrt(np.mean(d * d)) <= 1e-9


def test_apply_range_pinned_link_queues(oracle_mod):
    """Page-locked caller buffers go through the device's two link queues
    (lcfir.hip `Link`): H2D by the copy engine, D2H by pcie_copy_kernel
    through the output's device mapping when both ends are 16-byte aligned
    (else the copy engine); calls under 2 MiB keep their slot stream.  16
    threads calling at once over ranges of every alignment and tail (0..3
    floats past a float4), into a hipHostMalloc'd output (the link queues)
    and a hipHostRegister'd one (the runtime's own path: ROCm 7.2 reports no
    base for a registration, so host_pinned does not claim it), equal the
    device call's bytes; a 7-sample call leaves its neighbours untouched."""
    import ctypes
    import threading
    import lcfir
    import synth
    import torch
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    n = 9_600_017  # 16 ranges of >= 2.4 MB: above lcfir.hip's kLinkMinBytes (2 MiB)
    x = np.ascontiguousarray(synth.file_buffer(1, n, 48000.0, file=32, bits=24)[0])
    flt = lcfir.Filter(taps)
    dx = lcfir.DeviceBuffer.from_array(x)
    dy = lcfir.DeviceBuffer(4 * n)
    flt.apply_range_dev(dx, n, dy, 0, n)
    lcfir.sync()
    want = dy.download(n)
    lib = lcfir.load()
    px, py = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.lcfir_host_malloc(4 * n, ctypes.byref(px)) == 0
    assert lib.lcfir_host_malloc(4 * n, ctypes.byref(py)) == 0
    rt = torch.cuda.cudart()
    page = 1 << 16
    raw = np.zeros(n + 2 * page, np.float32)
    a0 = (-raw.ctypes.data) % page // 4
    reg = raw[a0:a0 + n]
    reg_len = (4 * n + page - 1) & ~(page - 1)
    registered = False
    try:
        hx = np.ctypeslib.as_array((ctypes.c_float * n).from_address(px.value))
        hy = np.ctypeslib.as_array((ctypes.c_float * n).from_address(py.value))
        hx[:] = x
        assert int(rt.cudaHostRegister(reg.ctypes.data, reg_len, 0)) == 0
        registered = True
        # 16 ranges: starts on and off a float4, lengths with every tail
        cuts = [0]
        rng = np.random.default_rng(5)
        while len(cuts) < 16:
            cuts.append(cuts[-1] + 600_000 + int(rng.integers(0, 8)))
        cuts.append(n)
        ranges = list(zip(cuts[:-1], cuts[1:]))
        assert {(e - s) % 4 for s, e in ranges} == {0, 1, 2, 3} and {s % 4 for s, _ in ranges} >= {0, 1, 2, 3}
        for out in (hy, reg):
            out[:] = 7.0
            errs = []

            def call(s, e):
                try:
                    flt.apply_range(hx, out, s, e)
                except Exception as ex:  # surfaced below
                    errs.append(ex)
            threads = [threading.Thread(target=call, args=r) for r in ranges]
            for t in threads:
                t.start()
            for t in threads:
                t.join()
            assert not errs, errs
            assert np.array_equal(out, want)
        # a range inside the buffer: its neighbours keep their bytes
        hy[:] = 7.0
        flt.apply_range(hx, hy, 1_000_003, 1_000_010)
        assert np.array_equal(hy[1_000_003:1_000_010], want[1_000_003:1_000_010])
        assert np.all(hy[:1_000_003] == 7.0) and np.all(hy[1_000_010:] == 7.0)
        # releasing every slot releases the device's link queues too; the
        # next pinned call builds them again
        lcfir.staging_release(0)
        assert lcfir.staging_count(0) == (0, 0)
        hy[:] = 7.0
        flt.apply_range(hx, hy, 0, n)
        assert np.array_equal(hy, want)
    finally:
        if registered:
            rt.cudaHostUnregister(reg.ctypes.data)
        lib.lcfir_host_free(px)
        lib.lcfir_host_free(py)

"""CPU tests of the C ABI boundary: the library loads, exports every symbol
include/lcfir.h declares, and rejects bad arguments before touching a device.
No compute call is made here (no GPU in this container)."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import lcfir


def test_library_exports_every_header_symbol():
    lib = lcfir.load()
    declared = lcfir.header_symbols()
    assert len(declared) >= 20
    out = subprocess.run(["nm", "-D", "--defined-only", lcfir.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = [s for s in declared if s not in exported]
    assert not missing, f"declared in lcfir.h but not exported: {missing}"
    for s in declared:
        assert hasattr(lib, s)
    # every declared symbol has a ctypes signature in the binding
    assert set(declared) <= set(lcfir._SIGNATURES)


def test_library_is_gfx950_code_object():
    blob = open(lcfir.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"fir_direct_f64_kernel" in blob


def test_abi_version():
    assert lcfir.load().lcfir_abi_version() == 1


def test_build_id_is_the_sources_hash():
    """lcfir_build_id() (what PMC sidecars and A/B variants are matched on)
    is the hash audio-fir-filter_amd/src_hash.sh computes over the sources the
    in-tree library was built from: the Makefile compiled this tree's sources,
    not a stale one."""
    want = subprocess.run(["bash", os.path.join(os.path.dirname(lcfir.LIB_PATH), "src_hash.sh")],
                          capture_output=True, text=True, check=True).stdout.strip()
    assert len(want) == 16 and lcfir.build_id() == want


def test_even_tap_count_rejected_without_device():
    lib = lcfir.load()
    taps = np.ones(4, np.float64)
    ctx = ctypes.c_void_p()
    rc = lib.lcfir_ctx_create(0, taps.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), 4,
                              ctypes.byref(ctx))
    assert rc == lcfir.EINVAL
    assert b"odd" in lib.lcfir_last_error()
    assert not ctx.value


def test_null_arguments_rejected():
    lib = lcfir.load()
    assert lib.lcfir_ctx_create(0, None, 3, None) == lcfir.EINVAL
    assert lib.lcfir_apply_range(None, None, 0, None, 0, 0, lcfir.PROGRESS_FN(0), None) == lcfir.EINVAL
    assert lib.lcfir_apply_range_dev(None, None, 0, None, 0, 0, None) == lcfir.EINVAL
    assert lib.lcfir_filter_channels_dev(None, None, 0, 1, 1, None, 0, None, None) == lcfir.EINVAL
    assert lib.lcfir_peak_dev(None, 0, 1, 1, None, None) == lcfir.EINVAL
    assert lib.lcfir_normalize_dev(None, 0, 1, 1, None, 1, 0, None) == lcfir.EINVAL
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    assert lib.lcfir_ctx_window(None, 10, 0, 10, ctypes.byref(lo), ctypes.byref(hi)) == lcfir.EINVAL
    assert lib.lcfir_ctx_destroy(None) == lcfir.OK


def test_python_binding_fails_loudly_without_library(tmp_path):
    with pytest.raises(lcfir.LcfirError):
        lcfir._lib_saved = lcfir._lib
        try:
            lcfir._lib = None
            lcfir.load(str(tmp_path / "nope.so"))
        finally:
            lcfir._lib = lcfir._lib_saved


@pytest.mark.parametrize("freq,slope,fs", [(20, 48, 48000), (20, 10, 48000), (20, 96, 96000),
                                           (15, 10, 44100), (440, 80, 48000)])
def test_design_lowcut_matches_oracle(oracle_mod, freq, slope, fs):
    """Host tap design (ProcessFile.cp:47-50) vs the oracle's restatement."""
    taps = lcfir.design_lowcut(freq, slope, fs)
    assert taps.size == oracle_mod.lowcut_ntaps(slope, fs)
    ref = oracle_mod.design_lowcut(freq, fs, taps.size)
    # same long-double formula compiled by two compilers: agreement to a few
    # ulps of the largest tap (tiny taps near the window's zeros are noise-level)
    assert np.abs(taps - ref).max() <= 4 * np.spacing(np.abs(ref).max())
    assert abs(taps.sum()) < 1e-12 and 0.9 < taps[taps.size // 2] < 1.0


def test_design_lowcut_rejects_bad_args():
    with pytest.raises(lcfir.LcfirError):
        lcfir.design_lowcut(20, 0, 48000)
    with pytest.raises(lcfir.LcfirError):
        lcfir.design_lowcut(30000, 10, 48000)
    # -f 0: every low-pass tap is 0 and the unity-gain normalisation 0/0 --
    # rejected instead of NaN taps (a silently all-zero output file)
    with pytest.raises(lcfir.LcfirError, match="freq"):
        lcfir.design_lowcut(0, 10, 48000)
    with pytest.raises(lcfir.LcfirError):
        lcfir.design_lowcut(-5, 10, 48000)


def test_header_declares_reference_citations():
    text = open(lcfir.HEADER_PATH).read()
    for cite in ("FilterCore.h:20-27", "FilterCore.h:20-79", "ProcessFile.cp:91-101",
                 "ProcessFile.cp:47-50", "ProgressBar.h"):
        assert cite in text

"""CPU check of the FFT plans' host tables (lcfir::fft_plan_tables in
csrc/fir_fft.hpp, dumped by tests/cpp/fft_tables_dump) for both segment
lengths: scripts/fft32_model.py emulates one overlap-save segment with the
kernels' pair step read from those tables lane by lane (task words, special
lane, zero-phase and general layouts) and the L = 32 768 kernel's radix-2
split and merge, and the valid outputs must equal the direct convolution of
the segment to f64 rounding.  Also the header constants against the model."""
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import fft32_model as fm  # noqa: E402
import fft32r_model as rm  # noqa: E402

DUMP = os.path.join(ROOT, "tests", "cpp", "fft_tables_dump")


@pytest.fixture(scope="module")
def dump():
    subprocess.run(["make", "-C", os.path.dirname(DUMP), "fft_tables_dump"], check=True, capture_output=True)
    return DUMP


def test_model_against_convolution():
    fm.main()


def test_register_kernel_model_against_convolution():
    """scripts/fft32r_model.py: fir_fft32r_kernel's data flow (every register
    index, LDS slot of both exchanges and their rounds, the special lane's
    permutation) with its own tables, against direct convolution; no LDS read
    bank conflicts."""
    rm.main(8001)


# family: FftTuning::family (0 default, 1 the LDS-column kernels)
@pytest.mark.parametrize("seg_len,ntaps,sym,family", [
    (32768, 8001, True, 0), (32768, 4001, True, 0), (32768, 4003, False, 0), (32768, 8001, False, 0),
    (32768, 19201, True, 0), (16384, 4001, True, 0), (16384, 4003, False, 0), (32768, 4001, True, 1),
    (16384, 8001, True, 1), (16384, 4005, True, 0)])
def test_tables_emulated_segment(dump, tmp_path, seg_len, ntaps, sym, family):
    import oracle
    taps = oracle.design_lowcut(20.0, 48000.0, ntaps)
    if not sym:  # an asymmetric filter: the general (complex) pair table
        taps = taps + 1e-3 * np.linspace(-1.0, 1.0, ntaps)
    taps.astype(np.float64).tofile(tmp_path / "t.f64")
    subprocess.run([dump, str(tmp_path / "t.f64"), str(seg_len), "1", str(tmp_path / "tb"), str(family)],
                   check=True)
    tb = fm.load_tables(str(tmp_path / "tb"))
    assert tb["L"] == seg_len and tb["parts"] == 1 and tb["sym"] == sym
    # zero-phase single-partition plans: the register kernel of the segment
    # length, as the family allows
    assert tb["reg32"] == (seg_len == 32768 and sym and family != 1)
    rng = np.random.default_rng(ntaps)
    x = rng.uniform(-1, 1, seg_len)
    if tb["reg32"]:  # the register kernel's flow on the host's task words and pair table
        c, conflicts = rm.run(taps, x, tables=tb)
        assert not conflicts
    else:
        c = fm.emulate(x, tb)
    half = (ntaps - 1) // 2
    if tb["sym"]:
        ms = np.arange(half, seg_len - half, 509)  # c[m] = sum_k h[k] x[m - half + k]
        want = np.array([np.dot(taps, x[m - half:m - half + ntaps]) for m in ms])
    else:
        ms = np.arange(ntaps - 1, seg_len, 509)    # c[m] = sum_k h[k] x[m - (T-1) + k]
        want = np.array([np.dot(taps, x[m - (ntaps - 1):m + 1]) for m in ms])
    err = np.abs(c[ms] - want).max()
    assert err < 1e-12 * np.abs(taps).sum(), err


def test_seg_len_choice(dump, tmp_path):
    """fft_choose_seg_len (measured unit costs: CHANGELOG.md s4.2): a function of
    the taps alone, the per-output cost decides.  Linear-phase filters: the
    register kernel's L = 32 768 unit costs 2.2 L = 16 384 units, so 16 384 up
    to ~4 000 taps and 32 768 from config 2's 4 001 (7.65e-5 against 8.07e-5
    per output); 38 401 taps take two L = 32 768 partitions (the park-slab
    kernel, 4.0) instead of five.  Other filters (the general table): the
    park-slab kernel (3.1), 16 384 up to 8 001 taps, 32 768 from 10 001."""
    import oracle
    cases = [(401, True, 16384, 1), (3001, True, 16384, 1), (4001, True, 32768, 1), (8001, True, 32768, 1),
             (19201, True, 32768, 1), (38401, True, 32768, 2),
             (4001, False, 16384, 1), (8001, False, 16384, 1), (10001, False, 32768, 1), (19201, False, 32768, 1)]
    for ntaps, sym, L, parts in cases:
        taps = oracle.design_lowcut(20.0, 48000.0, ntaps)
        if not sym:
            taps = taps + 1e-3 * np.linspace(-1.0, 1.0, ntaps)
        taps.tofile(tmp_path / "t.f64")
        subprocess.run([dump, str(tmp_path / "t.f64"), "0", "1", str(tmp_path / "tb")], check=True)
        tb = fm.load_tables(str(tmp_path / "tb"))
        assert (tb["L"], tb["parts"], tb["sym"]) == (L, parts, sym and parts == 1), ntaps
        assert tb["reg32"] == (L == 32768 and parts == 1 and sym), ntaps


def test_header_constants_match_model():
    s = open(os.path.join(ROOT, "audio-fir-filter_amd", "csrc", "fir_fft32.hpp")).read()
    assert int(re.search(r"kFft32L = (\d+);", s).group(1)) == fm.L
    body = re.search(r"kW32\[16\]\[2\] = \{(.*?)\};", s, re.S).group(1)
    vals = [float(v) for v in re.findall(r"-?\d+\.\d+(?:e-?\d+)?", body)]
    want = fm.W(32, np.arange(16))
    assert np.allclose(np.array(vals[0::2]) + 1j * np.array(vals[1::2]), want, atol=1e-18)


def test_structural_changes_priced_below_the_bar():
    """scripts/fft32r_model.py price(): every candidate
    that moves the register kernel's staging traffic out of its final phase is
    capped by the measured no-DMA ceiling (timing-only variant, 8.9 %) and
    none clears the 8 % build bar once its barriers and rounds are charged;
    the LDS twiddle table does not fit.  DESIGN.md declares fir_fft32r final
    on these numbers."""
    out = rm.price(verbose=False)
    assert 0.08 < out["all_dma_early"][2] < 0.10  # the measured ceiling
    for name, (feasible, net, best) in out.items():
        assert net < rm.BUILD_BAR, name
    assert out["half_dma_early"][2] < rm.BUILD_BAR  # even for free
    assert not out["final_twiddles_lds"][0]
    # no DMA and no stores at all (the unit touches no HBM after its samples):
    # the stores add only 1-2 % once the DMA is gone, whole phase < 12 %
    dma3, mem3 = rm.memory_phase_ceiling()
    assert 0.08 < dma3 < mem3 < 0.12 and mem3 - dma3 < 0.03

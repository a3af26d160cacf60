"""CPU checks of the v3 FFT kernel's index plumbing (csrc/fir_fft.hpp):
the wave-0 lane table and special lane in the header equal the ones
scripts/fft_lds_sim.py derives, every LDS exchange is bank-conflict free under
the gfx950 lane-group rules, and the kernel's full forward/inverse index flow
(numpy) reproduces the 8192-point DFT with bins k and M-k in one lane."""
import os
import re
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import fft_lds_sim as sim  # noqa: E402

HDR = os.path.join(ROOT, "audio-fir-filter_amd", "csrc", "fir_fft.hpp")


def _header():
    return open(HDR).read()


def test_header_tables_match_simulator():
    s = _header()
    body = re.search(r"kFftWave0C0\[32\] = \{([^}]*)\}", s).group(1)
    words = [int(v, 16) for v in body.replace("\n", " ").split(",") if v.strip()]
    want = []
    for lane in range(32, 64):
        (_, da, ea), (_, db, eb) = sim.WAVE0[lane]
        want.append(da | ea << 3 | db << 6 | eb << 9)
    assert words == want
    special = int(re.search(r"kFftSpecialLane = (\d+);", s).group(1))
    assert special == sim.SPECIAL_LANE


def test_header_layouts_match_simulator():
    s = _header()
    # the C index functions, transcribed by regex into Python and compared
    for name, f, n in [("fx1", lambda a, b: sim.x1(a, b), 2), ("fx2", sim.x2, 3),
                       ("fx3", sim.x3, 3), ("fx4", sim.x4, 3)]:
        m = re.search(name + r"\(([^)]*)\) \{\s*return ([^;]*);", s)
        args = [a.split()[-1] for a in m.group(1).split(",")]
        expr = m.group(2).replace("\n", " ")
        g = eval("lambda " + ",".join(args) + ": " + expr)  # noqa: S307 - our own header
        rng = range(64) if n == 2 else range(8)
        for a in (range(64) if n == 2 else range(8)):
            for b in range(8):
                if n == 2:
                    assert g(a, b) == f(a, b)
                else:
                    for c in range(8):
                        assert g(a, b, c) == f(a, b, c)
        del rng


def test_exchanges_conflict_free():
    rep = sim.check_banks()
    assert all(v == 0 for v in rep.values()), rep


def test_index_flow_is_the_dft():
    rng = np.random.default_rng(7)
    z = rng.standard_normal(sim.M) + 1j * rng.standard_normal(sim.M)
    X, lanes = sim.forward_sim(z)
    ref = np.fft.fft(z)
    assert np.max(np.abs(X - ref)) <= 1e-12 * np.max(np.abs(ref))
    for k in range(sim.M):
        assert lanes[k][:2] == lanes[(sim.M - k) % sim.M][:2]
    v = sim.inverse_sim(X)
    assert np.max(np.abs(np.conj(v) - sim.M * np.conj(np.conj(z)))) <= 1e-9 * sim.M


def test_v5_two_workgroup_schedule():
    """The 64 KiB / 4-barrier schedule: correct transform both ways and no
    cross-wave LDS hazard inside any barrier phase."""
    err_f, err_i, hazards = sim.check_v5()
    assert err_f < 1e-12 and err_i < 1e-12
    assert hazards == 0


def test_v5_hazard_detector_is_live():
    """Negative control: the same schedule without barriers must show hazards."""
    class NoBarrier(sim.LDS):
        def barrier(self):
            pass

    lds = NoBarrier()
    sim.v5_forward(np.random.default_rng(1).standard_normal(sim.M) + 0j, lds)
    assert lds.hazards > 0


def test_fft_unit_is_a_bijection_per_round(tmp_path):
    """fft_unit (the persistent grid's unit order) and fft_div compiled host-only from the
    header and run here: one-to-one per round, XCD-aware full rounds, identity
    on the last partial round, the 32-bit map equal to the 64-bit one, and the
    multiply-shift u / nseg exact for u < 2^31 (tests/cpp/fft_unit_check.hip)."""
    import shutil
    import subprocess
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        import pytest
        pytest.skip("hipcc not available")
    exe = tmp_path / "fft_unit_check"
    src = os.path.join(ROOT, "tests", "cpp", "fft_unit_check.hip")
    subprocess.run([hipcc, "--offload-host-only", "-std=c++17", "-O1",
                    "-I" + os.path.join(ROOT, "include"),
                    "-I" + os.path.join(ROOT, "audio-fir-filter_amd", "csrc"), "-o", str(exe), src],
                   check=True, capture_output=True, timeout=300)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.strip().endswith("errors 0")

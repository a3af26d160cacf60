"""CPU tests of the build's kernel-resource gate (audio-fir-filter_amd/check_resources.py).

fir_fft32r_kernel's explicit vmcnt(kR32PairStores) wait at the top of a unit
is correct only while no vector-memory instruction other than the pair stores
follows the split LDS-DMA (csrc/fir_fft32r.hpp); a scratch spill or reload
would be one.  The Makefile fails the build when any instance of the kernel
uses scratch; these tests pin that gate and the built library's remarks.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "audio-fir-filter_amd")
sys.path.insert(0, PKG)
import check_resources  # noqa: E402

REMARK = """csrc/x.hpp:1:1: remark: Function Name: {name} [-Rpass-analysis=kernel-resource-usage]
csrc/x.hpp:1:1: remark:     VGPRs: 256 [-Rpass-analysis=kernel-resource-usage]
csrc/x.hpp:1:1: remark:     ScratchSize [bytes/lane]: {scratch} [-Rpass-analysis=kernel-resource-usage]
csrc/x.hpp:1:1: remark:     VGPRs Spill: {spill} [-Rpass-analysis=kernel-resource-usage]
"""


def test_parser_flags_scratch_in_the_register_kernel():
    ok = REMARK.format(name="_ZN5lcfir17fir_fft32r_kernelILi4ELb0EEEv", scratch=0, spill=0)
    bad = REMARK.format(name="_ZN5lcfir17fir_fft32r_kernelILi4ELb1EEEv", scratch=8, spill=1)
    other = REMARK.format(name="_ZN5lcfir20fir_fft32_f64_kernelILi0EEEv", scratch=160, spill=40)
    k = check_resources.parse(ok + bad + other)
    assert len(k) == 3
    assert k["_ZN5lcfir17fir_fft32r_kernelILi4ELb1EEEv"]["ScratchSize"] == 8
    v = check_resources.violations(k)
    assert len(v) == 1 and "Lb1" in v[0]
    # only the register kernel is gated: the park-slab kernel's waits are compiler-tracked
    assert check_resources.violations(check_resources.parse(ok + other)) == []


def test_gate_exit_status(tmp_path):
    f = tmp_path / "r.txt"
    f.write_text(REMARK.format(name="fir_fft32r_kernel_x", scratch=4, spill=1))
    assert check_resources.main(str(f)) == 1
    f.write_text(REMARK.format(name="fir_fft32r_kernel_x", scratch=0, spill=0))
    assert check_resources.main(str(f)) == 0
    f.write_text(REMARK.format(name="some_other_kernel", scratch=0, spill=0))
    assert check_resources.main(str(f)) == 1  # the gated kernel must be present


def test_built_library_register_kernel_has_no_scratch():
    """The remarks of the last `make` (every instance of fir_fft32r_kernel:
    plain and fused-normalize) show no scratch."""
    remarks = os.path.join(PKG, "liblcfir.remarks")
    if not os.path.exists(remarks):
        subprocess.run(["make", "-C", PKG, "liblcfir.so"], check=True, capture_output=True)
    k = check_resources.parse(open(remarks).read())
    r32 = {n: f for n, f in k.items() if "fir_fft32r_kernel" in n}
    assert len(r32) >= 2, sorted(k)
    assert check_resources.violations(k) == []
    for f in r32.values():
        assert f.get("ScratchSize") == 0 and f.get("VGPRs Spill") == 0

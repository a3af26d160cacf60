"""CPU test of scripts/copy_overlap.py (the drop-in's copy-overlap analysis of
a rocprofv3 kernel + memory-copy + HIP API trace): interval
unions, the H2D/D2H overlap, burst splitting and the API summary on a
synthetic trace with known answers."""
import csv
import os
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import copy_overlap  # noqa: E402


def test_union_and_both():
    assert copy_overlap.union([(0, 10), (5, 15), (20, 25)]) == 20
    assert copy_overlap.union([]) == 0
    # h2d busy [0, 10) and [20, 30); d2h [5, 25): overlap 5 + 5
    assert copy_overlap.both([(0, 10), (20, 30)], [(5, 25)]) == 10
    assert copy_overlap.both([(0, 10)], [(10, 20)]) == 0


def test_trace_dir(tmp_path, capsys):
    d = tmp_path / "t"
    d.mkdir()
    with open(d / "x_memory_copy_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kind", "Direction", "Start_Timestamp", "End_Timestamp"])
        for i in range(4):  # one burst: H2D i, D2H i overlapping H2D i + 1
            s = i * 1_000_000
            w.writerow(["MEMORY_COPY", "MEMORY_COPY_HOST_TO_DEVICE", s, s + 1_000_000])
            w.writerow(["MEMORY_COPY", "MEMORY_COPY_DEVICE_TO_HOST", s + 1_000_000, s + 2_000_000])
        # a second burst far away
        w.writerow(["MEMORY_COPY", "MEMORY_COPY_HOST_TO_DEVICE", 100_000_000, 100_500_000])
    with open(d / "x_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for i in range(4):
            w.writerow(["void lcfir::fir_fft32r_kernel<4, false>", i * 1_000_000 + 900_000, i * 1_000_000 + 950_000])
        w.writerow(["lcfir::(anonymous namespace)::pcie_copy_kernel", 100_600_000, 100_700_000])
    with open(d / "x_hip_api_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Domain", "Function", "Thread_Id", "Start_Timestamp", "End_Timestamp"])
        w.writerow(["HIP_RUNTIME_API", "hipMemcpyAsync", 7, 0, 8_000_000])
        w.writerow(["HIP_RUNTIME_API", "hipMemcpyAsync", 8, 0, 1_000])
    ev = copy_overlap.load(str(d))
    assert len(ev) == 4 * 3 + 2
    bursts = copy_overlap.bursts(ev, 3_000_000)
    assert [len(b) for b in bursts] == [12, 2]
    sys.argv = ["copy_overlap.py", str(d), "--gap", "3"]
    copy_overlap.main()
    out = capsys.readouterr().out
    assert "burst 0: span 5.000 ms, 12 events" in out
    assert "h2d and d2h at once: 3.000 ms (60.0% of span)" in out
    assert "hipMemcpyAsync" in out and "8.000" in out  # total 8.001 ms, max 8.000 ms

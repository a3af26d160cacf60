"""CPU test of the PMC sidecar chain bench.py's roofline.traffic comes from
(scripts/pmc_summary.py -> scripts/make_traffic_json.py, scripts/gpu_run.sh
`traffic` step): per-kernel averages over separate --pmc passes, the gfx950
FETCH_SIZE doubling (MI355X_MICROARCH.md, HBM section), the f64 flop count
(FMA = 2), on synthetic rocprofv3 counter CSVs with known answers."""
import csv
import json
import os
import subprocess
import sys

from conftest import ROOT

SCRIPTS = os.path.join(ROOT, "scripts")
KERNEL = "void lcfir::fir_fft32r_kernel<4, false, lcfir::R32NoProbe>(lcfir::DirectParams, int)"


def _pass(d, name, rows):
    p = d / name
    p.mkdir(parents=True)
    with open(p / "pmc_counter_collection.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"])
        for r in rows:
            w.writerow(r)


def test_summary_and_sidecar(tmp_path):
    d = tmp_path / "traffic1"
    # two dispatches per pass; FETCH_SIZE / WRITE_SIZE in KB per dispatch
    _pass(d, "p_1", [(KERNEL, "FETCH_SIZE", 100000.0, 0, 180000), (KERNEL, "FETCH_SIZE", 102000.0, 0, 182000),
                     ("other_kernel(int)", "FETCH_SIZE", 5.0, 0, 1000)])
    _pass(d, "p_2", [(KERNEL, "WRITE_SIZE", 225000.0, 0, 180000), (KERNEL, "WRITE_SIZE", 225000.0, 0, 180000)])
    _pass(d, "p_3", [(KERNEL, c, v, 0, 180000) for c, v in
                     [("SQ_INSTS_VALU", 61e6), ("SQ_INSTS_VALU_ADD_F64", 10e6), ("SQ_INSTS_VALU_MUL_F64", 2e6),
                      ("SQ_INSTS_VALU_FMA_F64", 20e6)]])
    summ = tmp_path / "s.json"
    subprocess.run([sys.executable, os.path.join(SCRIPTS, "pmc_summary.py"), str(d), "--json", str(summ)],
                   check=True, capture_output=True)
    s = json.load(open(summ))
    k = s[KERNEL.split("(")[0]]
    assert k["FETCH_SIZE"] == 101000.0 and k["WRITE_SIZE"] == 225000.0
    assert k["hbm_read_bytes_corrected"] == 2.0 * 101000.0 * 1024.0
    assert k["dispatches_seen"] == 2
    out = tmp_path / "traffic.json"
    subprocess.run([sys.executable, os.path.join(SCRIPTS, "make_traffic_json.py"), str(summ), str(out),
                    "--method", "fft", "--ntaps", "4001", "--samples-per-launch", "57600000",
                    "--kernel", "fir_fft32r_kernel", "--seg-len", "32768"], check=True, capture_output=True)
    t = json.load(open(out))
    read, write = 2.0 * 101000.0 * 1024.0, 225000.0 * 1024.0
    assert t["hbm_bytes_per_launch"] == read + write
    assert abs(t["traffic_over_algorithmic"] - (read + write) / (8.0 * 57600000)) < 1e-12
    assert t["f64_flops_per_launch"] == 64.0 * (10e6 + 2e6 + 2.0 * 20e6)
    assert t["valu_insts_per_launch"] == 61e6
    # the keys bench.py matches a sidecar on (bench.py, roofline.traffic)
    assert (t["method"], t["ntaps"], t["samples_per_launch"], t["seg_len"], t["kernel"]) == \
        ("fft", 4001, 57600000.0, 32768, "fir_fft32r_kernel")
    # ... and the build it was measured on: by default the in-tree library's id
    import lcfir
    assert t["build_id"] == lcfir.build_id() != "unknown"


def test_bench_refuses_a_sidecar_from_another_build(tmp_path):
    """bench.select_sidecar attaches PMC counters only when the sidecar names
    the loaded library's build id (lcfir_build_id) and the launch shape; the
    line's roofline.traffic_source names the file and the id, or is null."""
    sys.path.insert(0, ROOT)
    import bench
    import lcfir
    me = lcfir.build_id()
    base = {"method": "fft", "ntaps": 4001, "samples_per_launch": 57600000.0, "seg_len": 32768,
            "kernel": "fir_fft32r_kernel", "hbm_bytes_per_launch": 1.0}
    stale = tmp_path / "traffic_stale.json"      # another build of the same kernel name
    json.dump(dict(base, build_id="0123456789abcdef", hbm_bytes_per_launch=2.0), open(stale, "w"))
    legacy = tmp_path / "traffic_legacy.json"    # round 5's sidecars: no build id at all
    json.dump(base, open(legacy, "w"))
    good = tmp_path / "traffic_good.json"
    json.dump(dict(base, build_id=me), open(good, "w"))
    args = ("fft", 4001, 57600000.0, 32768, "fir_fft32r_kernel")
    tj, src = bench.select_sidecar([str(stale), str(legacy)], me, *args)
    assert tj is None and src is None
    tj, src = bench.select_sidecar([str(stale), str(legacy), str(good)], me, *args)
    assert tj["hbm_bytes_per_launch"] == 1.0 and src["build_id"] == me and src["path"].endswith("traffic_good.json")
    # a matching build but another launch shape, or a library without an id
    assert bench.select_sidecar([str(good)], me, "fft", 8001, 57600000.0, 32768, "fir_fft32r_kernel") == (None, None)
    json.dump(dict(base, build_id="unknown"), open(good, "w"))
    assert bench.select_sidecar([str(good)], "unknown", *args) == (None, None)

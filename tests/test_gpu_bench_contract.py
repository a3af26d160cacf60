"""bench.py's one-line JSON contract on a short config-2 run (MI355X): the
keys the driver reads, the roofline and cpu_baseline objects, the parity
probe within tolerance, for serial and pipelined steps (--lanes 1 / 2)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("lanes", [1, 2])
def test_bench_json_line(lanes):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup", "2",
           "--seconds", "10", "--cpu-seconds", "1", "--lanes", str(lanes), "--preroll-s", "0.2",
           "--kernel-launches", "5"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline", "parity"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 4 and d["warmup"] == 2
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["config"]["workload"].startswith("config2") and d["config"]["lanes"] == lanes
    samples = d["config"]["channels"] * d["config"]["samples_per_channel"]
    assert abs(d["value"] - samples / (d["ms_per_step"] / 1e3) / 1e6) / d["value"] < 0.01
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-5
    # config 2's 4 001 linear-phase taps: the L = 32 768 register-resident kernel
    assert r["kernel"] == "fir_fft32r_kernel" and r["launches_timed"] == 5
    # achieved = algorithmic read bytes of one launch / its exclusive duration
    assert abs(r["achieved"] - 4 * samples / (r["kernel_ms"] / 1e3) / 1e9) / r["achieved"] < 1e-3
    assert d["preroll"]["steps"] > 0
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["kind"] == "port" and cb["cores"] >= 1 and cb["sample"]
    assert d["parity"]["rms_vs_longdouble"] <= d["parity"]["tol"] == 1e-9
    assert d["parity"]["max_ulp"] <= 1.0
    ing = d["ingest"]  # PCIe ingest probe: reported beside `value`, never in it
    assert ing["format"] == "s24le" and ing["decode_exact"] is True
    assert ing["bytes"] == 3 * ing["frames"] * ing["channels"] and 0 < ing["h2d_GBps"] < 200


def test_bench_gpus2_spawns_two_ranks():
    """`bench.py --gpus 2` started bare (no WORLD_SIZE) runs two ranks itself
    (torch.distributed.run, one process per rank); on the one-GPU box they
    share the device (LCFIR_BENCH_SHARE_DEVICE=1, gloo).  Config 5 with 2
    files: one file per rank and the peak exchange of --normalize."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env["LCFIR_BENCH_SHARE_DEVICE"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "5", "--files", "2",
           "--seconds", "20", "--steps", "3", "--warmup", "1", "--preroll-s", "0.2", "--kernel-launches", "3",
           "--no-ingest"]
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=110, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["files"] == 2
    assert d["config"]["peak_exchange"] is True and d["config"]["normalize"] is True
    assert d["parity"]["rms_vs_longdouble"] <= 1e-9
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only

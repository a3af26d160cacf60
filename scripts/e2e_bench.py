"""End-to-end rate of the lowcut tool: WAVE files on disk -> pinned host ->
PCIe -> decode/filter/normalize/encode on the GPU -> PCIe -> disk, pipelined
across files (read / 2 GPU streams / write).  This is the PCIe- and disk-
inclusive number DESIGN.md quotes beside bench.py's HBM-resident `value`.

usage: python scripts/e2e_bench.py [--files 4] [--minutes 10] [--out gpurun_out/e2e.json]
Inputs are config-2-shaped synthetic files (stereo 48 kHz int24, SURVEY.md s8d
generator), written to $TMPDIR.
"""
import argparse
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-fir-filter_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import synth  # noqa: E402
import pcm_ref  # noqa: E402


def run_tool(a, exe, paths, work, nch, n):
    """One lowcut run over the generated files into a fresh output directory."""
    out_dir = os.path.join(work, "out")
    shutil.rmtree(out_dir, ignore_errors=True)
    t0 = time.time()
    extra = ["--readers", str(a.readers)] if a.readers else []
    extra += ["--devices", a.devices] if a.devices else []
    r = subprocess.run([exe, "--timing", "-f", "20", "-s", "48", *extra, *paths, out_dir],
                       capture_output=True, text=True, timeout=1200)
    wall = time.time() - t0
    if r.returncode != 0:
        sys.exit(f"lowcut failed: {r.stderr}")
    m = re.search(r"timing total: (\d+) file\(s\), .*?, ([\d.]+) s, ([\d.]+) Msamples/s", r.stdout)
    per_file = re.findall(r"timing (\S+): read ([\d.]+) s, gpu ([\d.]+) s .*write ([\d.]+) s",
                          r.stdout)
    res = {
        "what": "lowcut end to end (disk + pinned host + PCIe + GPU), pipelined across files",
        "files": a.files, "minutes_per_file": a.minutes, "format": "stereo 48 kHz s24le WAVE",
        "readers": a.readers, "devices": a.devices,
        "summary_line": next((l for l in r.stdout.splitlines() if l.startswith("timing total")), None),
        "ntaps": 4001, "samples": a.files * nch * n,
        "tool_seconds": float(m.group(2)), "msamples_per_s": float(m.group(3)),
        "process_wall_seconds": wall,
        "per_file": [{"file": f, "read_s": float(rd), "gpu_s": float(g), "write_s": float(w)}
                     for f, rd, g, w in per_file],
    }
    # steady state: the pipeline's slowest stage per file, after the first
    # file (which also pays the ctx, FFT plan and buffer set-up)
    later = sorted(max(float(rd), float(g), float(w)) for _, rd, g, w in per_file[1:])
    if later:
        res["steady_stage_s"] = later[len(later) // 2]
        res["steady_msamples_per_s"] = nch * n / res["steady_stage_s"] / 1e6
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--files", type=int, default=4)
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "e2e.json"))
    ap.add_argument("--readers", type=int, default=0, help="lowcut --readers (0: the tool's default)")
    ap.add_argument("--devices", default=None, help="lowcut --devices")
    ap.add_argument("--exe", action="append", help="lowcut binary (repeat to alternate several; default: the built one)")
    ap.add_argument("--reps", type=int, default=1, help="runs per binary, alternating")
    a = ap.parse_args()
    rate, nch = 48000, 2
    n = int(a.minutes * 60 * rate)
    work = tempfile.mkdtemp(prefix="lcfir_e2e_")
    try:
        paths = []
        t0 = time.time()
        for i in range(a.files):
            x = synth.file_buffer(nch, n, float(rate), file=i, bits=24)
            p = os.path.join(work, f"f{i}.wav")
            pcm_ref.write_wave(p, x, rate, "s24le")
            paths.append(p)
            del x
        gen_s = time.time() - t0
        exes = a.exe or [os.path.join(ROOT, "audio-fir-filter_amd", "lowcut")]
        runs = []
        for rep in range(a.reps):
            for exe in exes:
                res = run_tool(a, exe, paths, work, nch, n)
                res["input_generation_seconds"] = gen_s
                res["exe"], res["rep"] = os.path.relpath(exe, ROOT), rep
                runs.append(res)
                print(json.dumps({k: res[k] for k in ("exe", "rep", "tool_seconds", "msamples_per_s")}),
                      flush=True)
        out = runs[0] if len(runs) == 1 else {"runs": runs}
        os.makedirs(os.path.dirname(a.out), exist_ok=True)
        with open(a.out, "w") as fh:
            json.dump(out, fh, indent=1)
        if len(runs) == 1:
            print(json.dumps(out))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()

"""bench.py -- filtered Msamples/s of the low-cut FIR hot path on MI355X.

Workload (BASELINE.json configs[1], "config 2"): one 10-minute stereo 48 kHz
int24 file per GPU = 2 channels x 28 800 000 samples, 4001-tap low-cut
(-f 20, M = 4000), synthetic samples (SURVEY.md s8d generator; no audio data
exists in this pipeline), already resident in HBM when timing starts.

One step = the whole per-file compute path of ProcessFile.cp:57-101 on the
device: filter every channel (apply_filter_range over [0, N), fused max|y|),
then the device-side normalize decision/rescale (a no-op unless the peak
exceeds 1 or --normalize).  N GPUs = N ranks, one file each (weak scaling, no
data-path collective; --normalize with --peak-scope global adds the RCCL MAX
all-reduce of the per-file peaks).

Prints ONE JSON line on rank 0 (contract: see README/DESIGN.md).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-fir-filter_amd"))

HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md:36 (spec)
FP64_PEAK_TFLOPS = 78.6     # FP64 vector (spec; half the 157.3 TF FP32 vector rate)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--method", default="auto", choices=["auto", "direct", "fft"])
    ap.add_argument("--seconds", type=float, default=600.0, help="file length (config 2: 600)")
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--fs", type=float, default=48000.0)
    ap.add_argument("--ntaps", type=int, default=4001)
    ap.add_argument("--bits", type=int, default=24, help="0 = float32 source")
    ap.add_argument("--normalize", action="store_true")
    ap.add_argument("--peak-scope", default="file", choices=["file", "global"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    return ap.parse_args()


def design_taps(ntaps, fs):
    """Low-cut taps for the bench (dspguide Blackman windowed-sinc, spectral
    inversion).  Computed here in numpy so the product path never touches the
    oracle; the oracle's identical design is used only by the checks."""
    import numpy as np
    M = ntaps - 1
    half = M // 2
    fc = 20.0 / fs
    i = np.arange(ntaps, dtype=np.float64)
    d = i - half
    with np.errstate(invalid="ignore", divide="ignore"):
        h = np.where(d == 0, 2 * np.pi * fc, np.sin(2 * np.pi * fc * d) / np.where(d == 0, 1, d))
    w = 0.42 - 0.5 * np.cos(2 * np.pi * i / M) + 0.08 * np.cos(4 * np.pi * i / M)
    h = h * w
    h = -(h / h.sum())
    h[half] += 1.0
    return h


def cpu_baseline(x0, taps, budget_s):
    """Oracle restatement of the reference threaded CPU path (FilterCore.h +
    ProcessFile.cp:57-87, strict-order double FMA), on a bounded prefix."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:
        cores = os.cpu_count() or 1
    cores = max(1, min(cores, 16))  # the box's CPU share for one GPU
    n_cal = min(x0.size, 16384 * cores)
    t = time.perf_counter()
    oracle.filter_channel_mt(x0[:n_cal], taps, cores, oracle.MODE_FMA)
    rate = n_cal / max(1e-6, time.perf_counter() - t)
    n = int(min(x0.size, max(n_cal, rate * budget_s)))
    t = time.perf_counter()
    oracle.filter_channel_mt(x0[:n], taps, cores, oracle.MODE_FMA)
    dt = time.perf_counter() - t
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": cores,
            "kind": "port",
            "sample": f"first {n} samples of channel 0 of the bench file, {taps.size} taps, "
                      f"oracle ORACLE_FMA three-loop restatement, {cores} pthreads, "
                      f"{dt:.1f} s"}


def parity_probe(x, y, taps, k=512):
    """RMS vs the long-double oracle at k sampled positions per channel (rank 0)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    rng = np.random.default_rng(5)
    half = (taps.size - 1) // 2
    sq, cnt = 0.0, 0
    for c in range(x.shape[0]):
        n = x.shape[1]
        idx = np.unique(np.r_[np.arange(0, 64), np.arange(n - 64, n), rng.integers(0, n, k),
                              np.arange(half - 8, half + 8)])
        ref, _ = oracle.filter_points(x[c], taps, idx, oracle.MODE_LD)
        d = y[c][idx].astype(np.float64) - ref
        sq += float((d * d).sum())
        cnt += idx.size
    return (sq / cnt) ** 0.5, cnt


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    import lcfir   # after torch: shares torch's HIP runtime (same SONAME)
    import synth
    lcfir.load()
    runtimes = lcfir.hip_runtimes()
    if len(runtimes) != 1:
        raise RuntimeError(f"expected one HIP runtime in the process, found {runtimes}")

    nch, fs = args.channels, args.fs
    n = int(round(args.seconds * fs))
    taps = design_taps(args.ntaps, fs)
    bits = args.bits or None
    # one file per rank: seed offset by the rank (file index)
    x_host = synth.file_buffer(nch, n, fs, file=rank, bits=bits)
    x = torch.from_numpy(x_host).to(dev)
    y = torch.empty_like(x)
    # per-(file, channel) peak slots: file r owns [r*nch, (r+1)*nch); the file's
    # peak is the max over its channels (ProcessFile.cp:92-96)
    peaks = torch.zeros(world * nch, dtype=torch.float32, device=dev)
    flt = lcfir.Filter(taps, device=local, method=args.method)
    method = flt.method
    stream = torch.cuda.current_stream(dev)
    sp = stream.cuda_stream
    my_peaks = peaks[rank * nch:(rank + 1) * nch]

    def step_full(ev=None):
        lcfir.peak_reset_dev(peaks, peaks.numel(), sp)
        if ev is not None:
            ev[0].record(stream)
        flt.filter_channels_dev(x, n, nch, n, y, n, my_peaks, sp)
        if ev is not None:
            ev[1].record(stream)
        if args.normalize and args.peak_scope == "global" and world > 1:
            # batch-global peak (north-star config 5 variant; a deviation from the
            # reference's per-file rule): RCCL MAX all-reduce over xGMI
            dist.all_reduce(peaks, op=dist.ReduceOp.MAX)
            lcfir.normalize_dev(y, n, nch, n, peaks, peaks.numel(), True, sp)
        else:
            lcfir.normalize_dev(y, n, nch, n, my_peaks, nch, args.normalize, sp)

    for _ in range(args.warmup):
        step_full()
    torch.cuda.synchronize(dev)

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        step_full(evs[i])
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in evs) / max(1, args.steps)

    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    samples_per_step = nch * n
    total = samples_per_step * args.steps * world
    value = total / elapsed / 1e6
    ms_per_step = elapsed / args.steps * 1e3
    kern_s = kern_ms / 1e3
    achieved = 4.0 * samples_per_step / kern_s / 1e9
    fp64_tflops = 2.0 * args.ntaps * samples_per_step / kern_s / 1e12

    if rank == 0:
        y_host = y.cpu().numpy()
        rms, npos = parity_probe(x_host, y_host, taps)
        traffic = None
        try:
            with open(args.traffic_json) as f:
                tj = json.load(f)
            if tj.get("method") == method and tj.get("ntaps") == args.ntaps and \
                    tj.get("samples_per_launch") == samples_per_step:
                traffic = tj.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            pass
        line = {
            "metric": "filtered Msamples/sec @4001 taps; achieved HBM GB/s vs roofline",
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md s8d int24 generator), resident in HBM",
            "config": {
                "workload": f"config2: {args.seconds / 60:g} min {nch}-ch {fs / 1000:g} kHz "
                            f"{'int%d' % bits if bits else 'float32'} file per GPU, "
                            f"{args.ntaps}-tap low-cut",
                "channels": nch, "samples_per_channel": n, "ntaps": args.ntaps,
                "method": method, "files_per_gpu": 1,
                "parallelism": f"one file per GPU x{world}",
                "normalize": bool(args.normalize), "peak_scope": args.peak_scope,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 6),
                "traffic": traffic,
                "kernel": "fir_direct_f64_kernel" if method == "direct" else "fir_fft_f64_kernel",
                "kernel_ms": round(kern_ms, 4),
                "bytes_per_unit": 4,
                "binding": "fp64-valu",
                "fp64_tflops": round(fp64_tflops, 3),
                "fp64_frac": round(fp64_tflops / FP64_PEAK_TFLOPS, 4),
            },
            "parity": {"rms_vs_longdouble": rms, "positions": npos, "tol": 1e-9},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(x_host[0], taps, args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

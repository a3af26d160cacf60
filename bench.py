"""bench.py -- filtered Msamples/s of the low-cut FIR hot path on MI355X.

Default workload (BASELINE.json configs[1], "config 2"): one 10-minute stereo
48 kHz int24 file per GPU = 2 channels x 28 800 000 samples, 4001-tap
low-cut (-f 20, M = 4000).  Samples are synthetic (SURVEY.md s8d generator;
no audio data exists in this pipeline) and already resident in HBM when
timing starts.

One step = the per-file compute of ProcessFile.cp:57-101 for every file the
rank owns, through the batch driver (audio-fir-filter_amd/batch.py): filter
every channel (fused max|y| into the file's peak slot), exchange peaks only if
a file is split across ranks (or --peak-scope global), then the device-side
normalize decision and rescale (a no-op unless the peak exceeds 1 or
--normalize).

  --config 1  1 s mono 48 kHz int16, 19 201 taps (-f 20 -s 10): the reference's
              CPU-runnable plumbing case; cpu_baseline runs single-threaded, as
              BASELINE.json states it
  --config 2  (default) one 10-min file per GPU: weak scaling, no collective
  --config 3  one 60-s 8-channel 96 kHz float32 file per GPU, 8001 taps (the
              long-filter stress case; BASELINE.json names no duration, SURVEY.md
              s8a proposes 60 s)
  --config 4  8 x 60-min files over the ranks (one per GPU at N = 8)
  --config 5  config 4 + --normalize (per-file peaks; --peak-scope global adds
              the RCCL MAX all-reduce of the north-star variant)

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-fir-filter_amd"))

HBM_PEAK_GBPS = 8000.0      # MI355X_MICROARCH.md:36 (spec)
HBM_COPY_GBPS = 6290.0      # measured device-to-device copy rate on the box
FP64_PEAK_TFLOPS = 78.6     # FP64 vector (spec; half the 157.3 TF FP32 vector rate)
# f64 VALU ceiling per SIMD for the FFT kernel's own instruction mix: 1.71 ns per wave-instruction
# (tools/valu_mix.hip, 4 waves/SIMD at the 2.4 GHz max clock; profiles/r02_valu_mix.txt)
VALU_NS_PER_INST = 1.71
METRIC = "filtered Msamples/sec @4001 taps; achieved HBM GB/s vs roofline"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--method", default="auto", choices=["auto", "direct", "fft"])
    ap.add_argument("--files", type=int, default=None, help="files in the batch (configs 4/5)")
    ap.add_argument("--seconds", type=float, default=None, help="file length in seconds")
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--fs", type=float, default=48000.0)
    ap.add_argument("--ntaps", type=int, default=4001)
    ap.add_argument("--seg-len", type=int, default=0, choices=[0, 16384, 32768],
                    help="FFT segment length (0 = the library's choice)")
    ap.add_argument("--fft-family", default="default", choices=["default", "lds"],
                    help="FFT kernel family for zero-phase single-partition plans (lcfir_ctx_set_fft_family): "
                         "lds = the LDS-column kernels at L = 32 768 too")
    ap.add_argument("--general-form", action="store_true",
                    help="FFT: the general pair table even for linear-phase taps (zero-phase form off)")
    ap.add_argument("--bits", type=int, default=24, help="0 = float32 source")
    ap.add_argument("--normalize", action="store_true")
    ap.add_argument("--peak-scope", default="file", choices=["file", "global"])
    ap.add_argument("--no-fuse-normalize", action="store_true",
                    help="run every file's normalize as its own pass (A/B of BatchRunner's fused form)")
    ap.add_argument("--lanes", type=int, default=None,
                    help="pipeline consecutive steps over this many streams (BatchRunner lanes): "
                         "a step's first segments fill the CUs the previous step's last round "
                         "leaves idle; 1 = strictly serial steps.  Default: 2 for the one-file "
                         "configs 1-3 (+4-5 %% on configs 2/3), 1 for the 8-file configs 4/5 "
                         "(their 1.3-ms launches gain nothing and two lanes measured -2 %%)")
    ap.add_argument("--preroll-s", type=float, default=2.0,
                    help="untimed steps for this many seconds before the --warmup steps: the "
                         "shader clock ramps over the first few hundred ms of back-to-back "
                         "launches (CHANGELOG.md s5), and a 20-step timed region would otherwise "
                         "sit in that ramp.  0 = off")
    ap.add_argument("--kernel-launches", type=int, default=20,
                    help="launches of the filter alone, one stream, right after the pre-roll: "
                         "the exclusive kernel time roofline.kernel_ms is measured on")
    ap.add_argument("--force-exchange", action="store_true",
                    help="run the peak all-reduce every step even where the plan needs none (at --gpus 1: "
                         "a world-1 RCCL group; config 5 --files 1 is then the N = 8 per-rank step)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--graph", choices=["auto", "on", "off"], default="auto",
                    help="replay the steps from a captured HIP graph (batch.GraphedSteps: 2 x lanes "
                         "steps per replay); auto = on for config 1, whose 48 000-sample steps are "
                         "bound by host-side launch issue")
    ap.add_argument("--graph-per-lane", action="store_true",
                    help="one graph per lane replayed on its own stream instead of one graph for all "
                         "lanes (GraphedSteps(per_lane=True); measured slower for config 1)")
    ap.add_argument("--no-ingest", action="store_true",
                    help="skip the PCIe ingest probe (pinned PCM bytes -> HBM + on-device decode)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline budget")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"))
    a = ap.parse_args()
    if a.config == 1:
        a.seconds = 1.0 if a.seconds is None else a.seconds
        a.channels, a.fs, a.ntaps, a.bits = 1, 48000.0, 19201, 16
    elif a.config == 2:
        a.seconds = 600.0 if a.seconds is None else a.seconds
    elif a.config == 3:
        a.seconds = 60.0 if a.seconds is None else a.seconds
        a.channels, a.fs, a.ntaps, a.bits = 8, 96000.0, 8001, 0
    else:
        a.files = 8 if a.files is None else a.files
        a.seconds = 3600.0 if a.seconds is None else a.seconds
        a.normalize = a.normalize or a.config == 5
    if a.graph == "auto":
        a.graph = "on" if a.config == 1 else "off"
    if a.lanes is None:
        a.lanes = (10 if a.graph == "on" else 2) if a.config in (1, 2, 3) else 1
    return a


def launch_plan(gpus, env):
    """How this invocation runs `--gpus` ranks (one process per GPU):
    'rank' -- it IS a rank: WORLD_SIZE is set (torch.distributed.run, the
    driver's N > 1 launch) and equals --gpus, or neither is set and --gpus is 1;
    'spawn' -- --gpus N > 1 without WORLD_SIZE: start N rank processes with
    torch.distributed.run and wait for them (the parent never touches the GPU).
    A WORLD_SIZE that disagrees with --gpus is an error, never a silent
    single-GPU number recorded as the N-GPU point."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {gpus}: launch {gpus} ranks "
                             f"(torch.distributed.run --nproc-per-node {gpus}) or drop WORLD_SIZE")
        return "rank"
    return "rank" if gpus == 1 else "spawn"


def spawn_ranks(gpus, argv):
    """Run this script as `gpus` ranks under torch.distributed.run on 127.0.0.1
    (a free port), as a CHILD process; returns its exit code.  Called before
    anything initialises the GPU in this process (no exec: the children get
    fresh processes)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    return subprocess.run(cmd, env=env).returncode


def design_taps(ntaps, fs):
    """Low-cut taps (dspguide Blackman windowed-sinc + spectral inversion),
    computed here in numpy so the product path never touches the oracle."""
    import numpy as np
    M = ntaps - 1
    half = M // 2
    fc = 20.0 / fs
    i = np.arange(ntaps, dtype=np.float64)
    d = i - half
    with np.errstate(invalid="ignore", divide="ignore"):
        h = np.where(d == 0, 2 * np.pi * fc, np.sin(2 * np.pi * fc * d) / np.where(d == 0, 1, d))
    w = 0.42 - 0.5 * np.cos(2 * np.pi * i / M) + 0.08 * np.cos(4 * np.pi * i / M) if M else 1.0
    h = h * w
    h = -(h / h.sum())
    h[half] += 1.0
    return h


def host_cores():
    """CPUs this process may run on (nproc: the affinity mask)."""
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cgroup_cpu_quota(root="/sys/fs/cgroup"):
    """The CPU bandwidth limit of this process's cgroup, in CPUs (quota /
    period, rounded up), or None when unlimited or unreadable.  cgroup v2
    `cpu.max` ("<quota> <period>" or "max <period>"), else v1
    `cpu.cfs_quota_us` / `cpu.cfs_period_us`."""
    import math
    try:
        with open(os.path.join(root, "cpu.max")) as f:
            q, p = f.read().split()[:2]
        if q == "max":
            return None
        return max(1, math.ceil(int(q) / int(p)))
    except (OSError, ValueError):
        pass
    try:
        with open(os.path.join(root, "cpu", "cpu.cfs_quota_us")) as f:
            q = int(f.read().strip())
        with open(os.path.join(root, "cpu", "cpu.cfs_period_us")) as f:
            p = int(f.read().strip())
        return None if q <= 0 or p <= 0 else max(1, math.ceil(q / p))
    except (OSError, ValueError):
        return None


def usable_cpus(root="/sys/fs/cgroup"):
    """(usable, affinity, quota): the CPUs this process can really keep busy
    = min(affinity mask, cgroup quota).  On the GPU box the affinity mask
    lists 256 CPUs while the job's share is 16, and 256 threads there run
    slower than 16 (What's weak 5)."""
    aff = host_cores()
    quota = cgroup_cpu_quota(root)
    return (min(aff, quota) if quota else aff), aff, quota


def cpu_rate(oracle, x0, taps, threads, budget_s):
    """Msamples/s of the oracle's threaded restatement on a bounded prefix of
    x0 sized (by a short calibration run) to take about budget_s."""
    n_cal = min(x0.size, 16384 * threads)
    t = time.perf_counter()
    oracle.filter_channel_mt(x0[:n_cal], taps, threads, oracle.MODE_FMA)
    rate = n_cal / max(1e-6, time.perf_counter() - t)
    n = int(min(x0.size, max(n_cal, rate * budget_s)))
    t = time.perf_counter()
    oracle.filter_channel_mt(x0[:n], taps, threads, oracle.MODE_FMA)
    dt = time.perf_counter() - t
    return n / dt / 1e6, n, dt


def cpu_baseline(x0, taps, budget_s, single_thread=False):
    """Oracle restatement of the reference threaded CPU path (FilterCore.h +
    ProcessFile.cp:57-87, strict-order double FMA), on a bounded prefix, with
    one thread per usable CPU (min of the affinity mask and the cgroup CPU
    quota); beside it the reference's own default thread count,
    floor(0.7 x hardware_concurrency) (main.cp:75-76), hardware_concurrency
    being the affinity count the reference would see."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    usable, nproc, quota = usable_cpus()
    cores = 1 if single_thread else usable
    value, n, dt = cpu_rate(oracle, x0, taps, cores, budget_s)
    out = {"value": round(value, 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
           "nproc": nproc, "cgroup_cpu_quota": quota,
           "cores_note": "cores = threads used = min(affinity mask, cgroup CPU quota) "
                         "(1 for config 1, single-threaded as BASELINE.json states)",
           "sample": f"first {n} samples of file 0 (channels laid end to end), {taps.size} "
                     f"taps, oracle ORACLE_FMA three-loop restatement, {cores} pthreads, "
                     f"{dt:.1f} s"}
    if not single_thread:
        ref_threads = max(1, int(0.7 * nproc))  # main.cp:75: floor(0.7 * hw_concurrency)
        v7, n7, dt7 = cpu_rate(oracle, x0, taps, ref_threads, budget_s / 2)
        out["reference_default_threads"] = {
            "value": round(v7, 4), "threads": ref_threads,
            "sample": f"first {n7} samples, {dt7:.1f} s (the reference's -t 0 default, main.cp:75-76)"}
    return out


def ingest_probe(torch, lcfir, x, bits, dev, reps=5, max_frames=28_800_000):
    """What the resident-input `value` leaves out (PCIe H2D
    reported separately): one file's samples as interleaved PCM bytes in
    pinned host memory, copied to HBM and decoded to planar f32 on the device
    (lcfir_decode_pcm_dev) -- the lowcut tool's ingest.  Up to max_frames
    frames of x ([nch][frames] f32), HIP events on a side stream, median of
    reps; the decoded samples are checked against x."""
    import numpy as np
    nch, frames = x.shape
    frames = min(frames, max_frames)
    fmt = {16: "s16le", 24: "s24le"}.get(bits or 0, "f32le")
    xi = np.ascontiguousarray(x[:, :frames].T)  # interleaved [frames][nch]
    if fmt == "f32le":
        pcm = xi.astype("<f4").view(np.uint8).reshape(-1)
    else:
        v = np.rint(xi.astype(np.float64) * 2.0 ** (bits - 1)).astype("<i4")
        pcm = np.ascontiguousarray(v.view(np.uint8).reshape(-1, 4)[:, :bits // 8]).reshape(-1)
    host = torch.empty(pcm.size, dtype=torch.uint8, pin_memory=True)
    host.numpy()[:] = pcm
    d_pcm = torch.empty(pcm.size, dtype=torch.uint8, device=dev)
    d_out = torch.empty((nch, frames), dtype=torch.float32, device=dev)
    s = torch.cuda.Stream(dev)
    h2d, dec = [], []
    with torch.cuda.stream(s):
        for _ in range(reps + 1):
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(s)
            d_pcm.copy_(host, non_blocking=True)
            e[1].record(s)
            lcfir.decode_pcm_dev(d_pcm, fmt, nch, frames, d_out, frames, stream=s.cuda_stream)
            e[2].record(s)
            s.synchronize()
            h2d.append(e[0].elapsed_time(e[1]))
            dec.append(e[1].elapsed_time(e[2]))
    h2d, dec = sorted(h2d[1:])[reps // 2], sorted(dec[1:])[reps // 2]
    ok = bool(torch.equal(d_out.cpu(), torch.from_numpy(np.ascontiguousarray(x[:, :frames]))))
    return {"format": fmt, "frames": frames, "channels": nch, "bytes": int(pcm.size),
            "h2d_ms": round(h2d, 4), "h2d_GBps": round(pcm.size / h2d / 1e6, 2),
            "decode_ms": round(dec, 4), "decode_exact": ok,
            "msamples_per_s": round(nch * frames / (h2d + dec) / 1e3, 1),
            "note": "pinned interleaved PCM -> HBM -> planar f32 on one stream, median of "
                    f"{reps}; outside the timed region and never `value`"}


def parity_probe(x, y, taps, start, gain=None, k=512):
    """RMS and max |error| in f32 ulps vs the long-double oracle at sampled
    positions of one shard's outputs y = outputs [start, start + y.shape[1]) of
    the file x (rank 0).  gain: the normalize factor the step applied (None =
    not rescaled); the oracle value then gets the same f64 rescale and
    rounding (peak_scale.hpp)."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    rng = np.random.default_rng(5)
    half = (taps.size - 1) // 2
    n = x.shape[1]
    count = y.shape[1]
    sq, cnt, worst = 0.0, 0, 0.0
    for c in range(x.shape[0]):
        idx = np.unique(np.r_[np.arange(0, 64), np.arange(count - 64, count), rng.integers(0, count, k),
                              np.arange(half - 8, half + 8)])
        idx = idx[(idx >= 0) & (idx < count)]
        ref, _ = oracle.filter_points(x[c], taps, idx + start, oracle.MODE_LD)
        ref32 = ref.astype(np.float32)
        if gain is not None:
            ref32 = (ref32.astype(np.float64) * gain).astype(np.float32)
            ref = ref32.astype(np.float64)
        got = y[c][idx]
        d = got.astype(np.float64) - ref
        sq += float((d * d).sum())
        cnt += idx.size
        ulp = np.spacing(np.maximum(np.abs(ref32), np.float32(np.finfo(np.float32).tiny)))
        worst = max(worst, float((np.abs(d) / ulp.astype(np.float64)).max()))
    return (sq / cnt) ** 0.5, cnt, worst


class TimedBackend:
    """batch.DeviceBackend with each filter launch bracketed by HIP events
    recorded on the launch stream (the dominant kernel's live duration)."""

    def __init__(self, inner, torch):
        self.inner, self.torch = inner, torch
        self.events = []
        self.record = False

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def _timed(self, fn, *a, **k):
        if not self.record:
            return fn(*a, **k)
        e0 = self.torch.cuda.Event(enable_timing=True)
        e1 = self.torch.cuda.Event(enable_timing=True)
        e0.record(self.inner.stream)
        fn(*a, **k)
        e1.record(self.inner.stream)
        self.events.append((e0, e1))

    def filter(self, *a, **k):
        return self._timed(self.inner.filter, *a, **k)

    def filter_normalize_prev(self, *a, **k):
        # a filter launch that also rescales the previous file (config 5)
        return self._timed(self.inner.filter_normalize_prev, *a, **k)


class TimedCollective:
    """The runner's peak all-reduce with HIP events on the stream it is issued
    from (the lane's current stream): the span from the step's filter work
    being done to the reduced peaks being visible there, i.e. the collective
    plus any wait for the slowest rank."""

    def __init__(self, inner, torch):
        self.inner, self.torch = inner, torch
        self.events = []
        self.record = False

    def __call__(self, peaks):
        if not self.record:
            return self.inner(peaks)
        s = self.torch.cuda.current_stream()
        e0 = self.torch.cuda.Event(enable_timing=True)
        e1 = self.torch.cuda.Event(enable_timing=True)
        e0.record(s)
        self.inner(peaks)
        e1.record(s)
        self.events.append((e0, e1))

    def mean_ms(self):
        if not self.events:
            return None
        return sum(a.elapsed_time(b) for a, b in self.events) / len(self.events)


def rank_spread(records):
    """Per-rank figures of an N-rank line (records: one dict per rank, in rank
    order, from all_gather_object): each numeric field as a list plus its min
    and max, so an under-scaling SCALE point shows which rank (and which GPU,
    by PCI bus id) was slow and what the collective cost."""
    out = {"rank": [r["rank"] for r in records],
           "device": [r.get("device") for r in records]}
    for k in ("ms_per_step", "kernel_ms", "allreduce_ms_per_step", "samples"):
        vals = [r.get(k) for r in records]
        out[k] = vals
        num = [v for v in vals if v is not None]
        out[k + "_min"] = min(num) if num else None
        out[k + "_max"] = max(num) if num else None
    return out


def preroll(step, seconds, sync, agree=None, batch=8):
    """Untimed steps, in batches, until `seconds` have passed.  Every rank
    must run the same number of steps (a step with a peak exchange is a
    collective), so with `agree` (a MIN all-reduce of the continue flag) the
    ranks decide together after each batch and stop as soon as any rank's
    clock has run out.  Returns the step count."""
    steps, t0 = 0, time.perf_counter()
    more = seconds > 0
    while more:
        for _ in range(batch):
            step()
        steps += batch
        sync()
        more = time.perf_counter() - t0 < seconds
        if agree is not None:
            more = agree(more)
    return steps



KERNEL_NAMES = {"l16": "fir_fft_f64_kernel", "l32_park": "fir_fft32_f64_kernel", "l32_reg": "fir_fft32r_kernel"}


def select_sidecar(paths, build_id, method, ntaps, samples_per_launch, seg_len, kernel):
    """The first PMC sidecar (scripts/make_traffic_json.py) measured on this
    launch shape AND on the loaded library (its build_id, lcfir_build_id()):
    (sidecar dict, {"path", "build_id"}), or (None, None).  A sidecar without
    a build id, or from another build, is refused -- its counters may belong
    to a different kernel of the same name (What's weak 6)."""
    for path in paths:
        try:
            with open(path) as f:
                tj = json.load(f)
        except (OSError, ValueError):
            continue
        if not isinstance(tj, dict) or build_id in (None, "", "unknown") or tj.get("build_id") != build_id:
            continue
        if tj.get("method") == method and tj.get("ntaps") == ntaps and \
                tj.get("samples_per_launch") == samples_per_launch and \
                tj.get("seg_len", 16384 if method == "fft" else None) == seg_len and \
                tj.get("kernel", kernel) == kernel:
            return tj, {"path": os.path.relpath(path, ROOT), "build_id": build_id}
    return None, None


def fft_kernel_name(units):
    """The FFT kernel a plan runs, from lcfir_ctx_fft_units."""
    return KERNEL_NAMES[units["kernel"]]

def main():
    args = parse()
    if launch_plan(args.gpus, os.environ) == "spawn":
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("LCFIR_BENCH_SHARE_DEVICE") == "1":
        # rehearsal of the multi-rank path on a box with fewer GPUs than ranks
        local %= max(1, torch.cuda.device_count())
    elif local >= torch.cuda.device_count():
        raise SystemExit(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible "
                         f"(--gpus {args.gpus}; LCFIR_BENCH_SHARE_DEVICE=1 rehearses ranks on fewer GPUs)")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("LCFIR_BENCH_SHARE_DEVICE") == "1":
            # RCCL refuses two ranks on one GPU: the rehearsal runs gloo
            dist.init_process_group("gloo", rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    elif args.force_exchange:
        import socket
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            port = so.getsockname()[1]
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                                device_id=dev)

    import lcfir   # after torch: shares torch's HIP runtime (same SONAME)
    import synth
    import batch
    lcfir.load()
    runtimes = lcfir.hip_runtimes()
    if len(runtimes) != 1:
        raise RuntimeError(f"expected one HIP runtime in the process, found {runtimes}")

    nch, fs = args.channels, args.fs
    n = int(round(args.seconds * fs))
    per_gpu = args.config in (1, 2, 3)  # one file per rank (weak scaling)
    nfiles = world if per_gpu else args.files
    taps = design_taps(args.ntaps, fs)
    half = (args.ntaps - 1) // 2
    bits = args.bits or None
    flt = lcfir.Filter(taps, device=local, method=args.method)
    if args.seg_len or args.general_form:
        flt.set_fft_tuning(seg_len=args.seg_len, zero_phase=not args.general_form)
    if args.fft_family != "default":
        flt.set_fft_family(args.fft_family)
    method = flt.method

    backend = TimedBackend(batch.DeviceBackend(flt, dev, lanes=args.lanes, own_streams=args.graph == "on"),
                           torch)
    collective = TimedCollective(batch.torch_allreduce_max(), torch)
    runner = batch.BatchRunner(backend, rank, world, [n] * nfiles, nch, half, args.normalize,
                               args.peak_scope, collective, lanes=args.lanes,
                               fuse_normalize=not args.no_fuse_normalize, force_exchange=args.force_exchange)
    # synthetic samples; configs 4/5 reuse two generated files to bound host time
    cache = {}

    def file_samples(f):
        key = f if per_gpu else f % 2
        if key not in cache:
            cache[key] = synth.file_buffer(nch, n, fs, file=key, bits=bits)
        return cache[key]

    runner.prepare(lambda f, lo, hi: file_samples(f)[:, lo:hi])
    my_samples = sum(nch * (sh.end - sh.start) for sh in runner.shards)

    # Pre-roll: untimed steps until the shader clock has settled.  Back-to-back
    # launches ramp it over the first few hundred ms (CHANGELOG.md s5: a 20-step
    # region right after 5 warmup steps measured 8-20 % below steady state).
    def agree(more):
        flag = torch.tensor([1 if more else 0], dtype=torch.int32, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    t_pre = time.perf_counter()
    preroll_steps = preroll(runner.step, args.preroll_s, lambda: torch.cuda.synchronize(dev),
                            agree if world > 1 else None)
    preroll_s = time.perf_counter() - t_pre
    # The dominant kernel's exclusive time: the same filter launches, one
    # stream, nothing else in flight (HIP events on that stream), right after
    # the pre-roll so the clock is the timed steps' clock (measured after the
    # timed region instead, behind the host-side parity copy, it read ~20 %
    # long: the clock falls as soon as the GPU idles).  Under two lanes the
    # timed steps' launches overlap by a tail round, so their start-to-end
    # events (overlapped_ms) are not one launch's duration.
    backend.set_lane(0)
    backend.events = []
    peaks_scratch = backend.new_peaks(len(runner.nframes))
    for i in range(2 * args.kernel_launches):
        backend.record = i >= args.kernel_launches  # the first half: untimed lead-in
        sh = runner.shards[i % len(runner.shards)] if runner.shards else None
        if sh is None:
            break
        xw, lo, hi = runner.inputs[i % len(runner.shards)]
        yw = runner.output_buffer(0, i % len(runner.shards))
        backend.filter(xw, lo, hi, runner.nframes[sh.file], nch, yw, sh.start, sh.end,
                       peaks_scratch, sh.file)
    torch.cuda.synchronize(dev)
    backend.record = False
    kern_launches = len(backend.events)
    kern_ms = sum(a.elapsed_time(b) for a, b in backend.events) / max(1, kern_launches)
    backend.events = []
    for _ in range(args.warmup):
        runner.step()
    graphed = None
    if args.graph == "on" and not runner.exchange:
        # captured after the eager warmup (plans, scratch and kernel
        # attributes exist by now); replays run the same steps
        graphed = batch.GraphedSteps(runner, backend.inner, per_lane=args.graph_per_lane)
        graphed.replay()  # untimed: the first replay uploads the graph
    n_replay, n_eager = divmod(args.steps, graphed.per_replay) if graphed else (0, args.steps)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    backend.record = True
    collective.record = True
    t0 = time.perf_counter()
    for _ in range(n_replay):
        graphed.replay()
    for _ in range(n_eager):
        runner.step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    backend.record = False
    collective.record = False
    backend.set_lane(0)
    launches = len(backend.events)
    overlapped_ms = sum(a.elapsed_time(b) for a, b in backend.events) / max(1, launches)
    samples_per_launch = my_samples / max(1, len(runner.shards))
    # parity of the LAST timed step's outputs (rank 0's first shard), copied
    # out before anything else runs on the device
    probe = None
    if rank == 0 and not args.no_parity and runner.shards:
        sh0, y0 = runner.results()[0]
        probe = (sh0, y0.cpu().numpy(), float(runner.peaks[sh0.file].item()))

    ingest = None
    if not args.no_ingest and runner.shards:
        ingest = ingest_probe(torch, lcfir, file_samples(runner.shards[0].file), bits, dev)

    props = torch.cuda.get_device_properties(dev)
    mine = {"rank": rank, "device": f"{props.pci_domain_id:04x}:{props.pci_bus_id:02x}:{props.pci_device_id:02x}"
                                    f" (cuda:{local})",
            "ms_per_step": round(elapsed / args.steps * 1e3, 4), "kernel_ms": round(kern_ms, 6),
            "allreduce_ms_per_step": (round(collective.mean_ms(), 4) if collective.events else None),
            "samples": my_samples}
    records = [mine]
    if world > 1:
        records = [None] * world
        dist.all_gather_object(records, mine)
    total_samples = torch.tensor([float(my_samples)], dtype=torch.float64, device=dev)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        dist.all_reduce(total_samples, op=dist.ReduceOp.SUM)
    total = float(total_samples[0]) * args.steps
    value = total / elapsed / 1e6
    kern_s = kern_ms / 1e3
    achieved = 4.0 * samples_per_launch / kern_s / 1e9
    ms_per_step = elapsed / args.steps * 1e3
    # the whole step against the same roofline: per GPU, 4 B x samples per
    # step / ms_per_step (includes launch gaps, the collective and any
    # normalize pass; with lanes > 1 consecutive steps overlap)
    achieved_step = 4.0 * total / world / elapsed / 1e9
    launches_per_step = max(1, len(runner.shards))
    direct_tflops = 2.0 * args.ntaps * samples_per_launch / kern_s / 1e12

    if rank == 0:
        rms, npos, worst_ulp = None, 0, None
        if probe is not None:
            sh0, y0, peak0 = probe
            x = np.ascontiguousarray(file_samples(sh0.file))
            gain = None
            if args.normalize or peak0 > 1.0:
                gain = 1.0 / float(np.float32(peak0))  # the pass's f64 factor (peak_scale.hpp)
            rms, npos, worst_ulp = parity_probe(x, y0, taps, sh0.start, gain)
        # the PMC sidecar of this exact launch shape AND this library build
        # (--traffic-json, else any profiles/traffic_*.json; select_sidecar)
        plan = flt.fft_info if method == "fft" else {}
        kname = fft_kernel_name(flt.fft_units) if method == "fft" else "fir_direct_f64_kernel"
        sidecars = [args.traffic_json] + sorted(glob.glob(os.path.join(ROOT, "profiles", "traffic_*.json")))
        tj, traffic_source = select_sidecar(sidecars, lcfir.build_id(), method, args.ntaps, samples_per_launch,
                                            plan.get("seg_len"), kname)
        traffic = tj.get("hbm_bytes_per_launch") if tj else None
        f64_flops = tj.get("f64_flops_per_launch") if tj else None
        valu_insts = tj.get("valu_insts_per_launch") if tj else None
        # The f64 kernels are bound by VALU issue, not HBM: the launch's PMC
        # instruction counts (profiles/traffic_latest.json) over the live kernel time.
        # The resource whose floor is higher for this launch.  The direct form
        # issues one fma per tap rounded up to 16 (fir_direct.hpp) against 8 B
        # of HBM read + write per sample: below ~40 taps HBM is the floor.  The
        # FFT is bound by its f64 issue and LDS-exchange latency (DESIGN s4.2).
        if method == "direct":
            t16 = (args.ntaps + 15) // 16 * 16
            binding = "hbm" if 8.0 / (HBM_PEAK_GBPS * 1e9) > 2.0 * t16 / (FP64_PEAK_TFLOPS * 1e12) else "fp64-valu"
        else:
            binding = "fp64-valu"
        simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
        fp64_tflops = f64_flops / kern_s / 1e12 if f64_flops else None
        valu_frac = valu_insts * VALU_NS_PER_INST * 1e-9 / (simds * kern_s) if valu_insts else None
        wl = {1: "config1: 1 s mono 48 kHz int16 file per GPU (-f 20 -s 10)",
              2: "config2: 10 min stereo 48 kHz int24 file per GPU",
              3: f"config3: {args.seconds:g} s 8-channel 96 kHz float32 file per GPU",
              4: f"config4: {nfiles} x {args.seconds / 60:g} min stereo 48 kHz int24 files",
              5: f"config5: {nfiles} x {args.seconds / 60:g} min stereo 48 kHz int24 files, "
                 f"--normalize"}
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak" if per_gpu else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": f"synthetic (SURVEY.md s8d {'int%d' % bits if bits else 'float32'} generator), "
                    f"resident in HBM",
            "config": {
                "workload": wl[args.config] + f", {args.ntaps}-tap low-cut",
                "files": nfiles, "channels": nch, "samples_per_channel": n,
                "ntaps": args.ntaps, "method": method,
                "fft_plan": dict(flt.fft_info, kernel=fft_kernel_name(flt.fft_units)) if method == "fft" else None,
                "parallelism": f"{world} rank(s), files sharded by batch.plan_shards",
                "normalize": bool(args.normalize), "peak_scope": args.peak_scope,
                "peak_exchange": runner.exchange,
                "fused_normalize": runner.fuse and len(runner.shards) > 1,
                # whole run (pre-roll included): normalizes carried inside a
                # filter launch vs run as their own pass (lcfir_ctx_nrm_stats)
                "normalize_launches": flt.nrm_stats if args.normalize else None,
                "lanes": args.lanes,
                "hip_graph": {"replays": n_replay, "steps_per_replay": graphed.per_replay,
                              "graphs": len(graphed.graphs), "eager_steps": n_eager} if graphed else None,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 3),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 6),
                "frac_vs_copy": round(achieved / HBM_COPY_GBPS, 6),
                "frac_vs_copy_note": "achieved / the 6.29 TB/s device copy rate measured on the box "
                                     "(SURVEY.md s8d asks for both; peak stays the 8 TB/s spec)",
                "frac_step": round(achieved_step / HBM_PEAK_GBPS, 6),
                "frac_step_note": "4 B x samples per step per GPU / ms_per_step / 8 TB/s (whole step: "
                                  "launch gaps, collective, normalize passes, lane overlap included)",
                "traffic": traffic,
                # where traffic / fp64_tflops_pmc / valu_issue_frac come from: the
                # sidecar's path and the build id it was measured on (= the loaded
                # library's), null when no sidecar matches this build and shape
                "traffic_source": traffic_source,
                "kernel": "fir_direct_f64_kernel" if method == "direct" else fft_kernel_name(flt.fft_units),
                "kernel_ms": round(kern_ms, 6),
                "kernel_ms_note": f"exclusive: {kern_launches} launches of the filter alone on one "
                                  f"stream right after the pre-roll (HIP events on that stream)",
                "launches_timed": kern_launches,
                "lane_overlap": (f"kernel_ms x {launches_per_step} launch(es) per step = "
                                 f"{kern_ms * launches_per_step:.4f} ms > ms_per_step {ms_per_step:.4f}: "
                                 f"with {args.lanes} lanes consecutive steps overlap one launch's last, "
                                 f"partial round of segments with the next launch, so the step rate beats "
                                 f"a lone launch; frac (exclusive launch) never credits that overlap, "
                                 f"frac_step does") if kern_ms * launches_per_step > ms_per_step else None,
                # None when the timed steps were graph replays (no per-launch events)
                "overlapped_kernel_ms": round(overlapped_ms, 6) if launches else None,
                "bytes_per_unit": 4,
                "binding": binding,
                "direct_equiv_fp64_tflops": round(direct_tflops, 3),
                "fp64_frac": round(direct_tflops / FP64_PEAK_TFLOPS, 4) if method == "direct"
                else (round(fp64_tflops / FP64_PEAK_TFLOPS, 4) if fp64_tflops else None),
                "fp64_tflops_pmc": round(fp64_tflops, 3) if fp64_tflops else None,
                "valu_issue_frac": round(valu_frac, 4) if valu_frac else None,
                "valu_issue_note": "PMC VALU wave-instructions per launch x 1.71 ns / (SIMDs x kernel time); "
                                   "1.71 ns = the f64 pipe's measured ceiling for the kernel's own "
                                   "instruction mix (tools/valu_mix.hip, max clock)",
            },
            "parity": {"rms_vs_longdouble": rms, "max_ulp": worst_ulp, "positions": npos,
                       "tol": 1e-9, "of": "outputs of the last timed step (rank 0, first shard)"},
            "preroll": {"seconds": round(preroll_s, 3), "steps": preroll_steps},
            # per-rank spread (value and ms_per_step above are max-based); the
            # all-reduce time is the peak exchange's HIP-event span per step
            "ranks": rank_spread(records),
        }
        if ingest is not None:
            line["ingest"] = ingest  # rank 0's
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(file_samples(0).reshape(-1), taps,
                                                args.cpu_seconds, single_thread=args.config == 1)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

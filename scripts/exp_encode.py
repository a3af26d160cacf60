"""GPU time of the lowcut tool's post-filter passes on one config-2-shaped file
(stereo 10 min 48 kHz, f32 planes resident in HBM): normalize + encode (round 1)
against the fused lcfir_encode_pcm_scaled_dev (round 2), forced --normalize,
int24 output; both byte-identical (tests/test_gpu_codec.py).  HIP events on
torch's current stream, median of 20 repetitions each, alternating.

usage: python scripts/exp_encode.py [--minutes 10] [--format s24le]
"""
import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-fir-filter_amd"))
import lcfir  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--minutes", type=float, default=10.0)
    ap.add_argument("--format", default="s24le")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    nch, n = 2, int(a.minutes * 60 * 48000)
    nb = lcfir.pcm_bytes(a.format)
    dev = torch.device("cuda", 0)
    y0 = (torch.rand(nch, n, device=dev) * 1.6 - 0.8).contiguous()
    y = torch.empty_like(y0)
    raw = torch.empty(nb * nch * n, dtype=torch.uint8, device=dev)
    peak = torch.full((nch,), 0.8, dtype=torch.float32, device=dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    t_two, t_one = [], []
    for _ in range(a.reps + 2):
        y.copy_(y0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        lcfir.normalize_dev(y, n, nch, n, peak, nch, True, stream=s)
        lcfir.encode_pcm_dev(y, n, nch, n, a.format, raw, stream=s)
        e1.record()
        y.copy_(y0)
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record()
        lcfir.encode_pcm_scaled_dev(y, n, nch, n, a.format, peak, nch, True, raw, stream=s)
        f1.record()
        torch.cuda.synchronize()
        t_two.append(e0.elapsed_time(e1))
        t_one.append(f0.elapsed_time(f1))
    t_two, t_one = t_two[2:], t_one[2:]
    res = {"what": "lowcut post-filter passes per file, forced --normalize",
           "file": f"{nch} ch x {n} frames f32 planes -> {a.format}",
           "normalize_then_encode_ms": round(statistics.median(t_two), 4),
           "fused_encode_ms": round(statistics.median(t_one), 4)}
    res["saved_ms"] = round(res["normalize_then_encode_ms"] - res["fused_encode_ms"], 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()

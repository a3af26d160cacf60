"""Turn a PMC summary (scripts/pmc_summary.py output) into profiles/traffic_latest.json,
the per-launch HBM traffic bench.py reports as roofline.traffic.

usage: python scripts/make_traffic_json.py <pmc_summary.json> <out.json> --method fft \
           --ntaps 4001 --samples-per-launch 57600000 --kernel fir_fft_f64_kernel \
           [--build-id ID]

The sidecar carries the build id (lcfir_build_id(): the library sources' hash)
of the library the counters were measured on -- by default the one
audio-fir-filter_amd/liblcfir.so reports -- and bench.py attaches it only to a
line from that same build.

Also carries the launch's VALU instruction count and f64 flops (SQ_INSTS_VALU*,
when the summary has them) for bench.py's fp64 figures.

HBM bytes per launch = 2 * FETCH_SIZE * 1024 (gfx950 FETCH_SIZE counts half the
bytes of wide streaming reads: MI355X_MICROARCH.md, HBM section) + WRITE_SIZE * 1024.
"""
import argparse
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summary")
    ap.add_argument("out")
    ap.add_argument("--method", required=True)
    ap.add_argument("--ntaps", type=int, required=True)
    ap.add_argument("--samples-per-launch", type=float, required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--seg-len", type=int, default=16384, help="FFT segment length of the launch (0: direct)")
    ap.add_argument("--build-id", default=None,
                    help="lcfir_build_id() of the profiled library (default: ask the in-tree liblcfir.so)")
    a = ap.parse_args()
    if a.build_id is None:
        import os
        import sys
        sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "audio-fir-filter_amd"))
        import lcfir
        a.build_id = lcfir.build_id()
    s = json.load(open(a.summary))
    k = next(v for name, v in s.items() if a.kernel in name)
    read = 2.0 * k["FETCH_SIZE"] * 1024.0
    write = k["WRITE_SIZE"] * 1024.0
    alg = 8.0 * a.samples_per_launch
    out = {
        "method": a.method, "ntaps": a.ntaps, "samples_per_launch": a.samples_per_launch,
        "kernel": a.kernel, "seg_len": a.seg_len if a.method == "fft" else None,
        "build_id": a.build_id,
        "hbm_bytes_per_launch": read + write,
        "hbm_read_bytes_per_launch": read, "hbm_write_bytes_per_launch": write,
        "algorithmic_rw_bytes_per_launch": alg,
        "traffic_over_algorithmic": (read + write) / alg,
        "avg_duration_ns_profiled": k.get("avg_duration_ns"),
        # f64 VALU work of one launch (wave instructions x 64 lanes; FMA = 2 flops)
        "valu_insts_per_launch": k.get("SQ_INSTS_VALU"),
        "f64_flops_per_launch": (64.0 * (k["SQ_INSTS_VALU_ADD_F64"] + k["SQ_INSTS_VALU_MUL_F64"]
                                         + 2.0 * k["SQ_INSTS_VALU_FMA_F64"])
                                 if "SQ_INSTS_VALU_FMA_F64" in k else None),
        "note": "FETCH_SIZE doubled per the gfx950 calibration; separate rocprofv3 --pmc passes",
    }
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

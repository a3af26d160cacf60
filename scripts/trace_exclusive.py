"""Average duration of bench.py's exclusive filter launches, read from a
rocprofv3 --kernel-trace csv of the bench command itself.

bench.py times roofline.kernel_ms on 2 x --kernel-launches back-to-back
filter launches on one stream right after the pre-roll (the first half an
untimed lead-in).  In the trace they are the only long run of consecutive,
non-overlapping launches on one queue (the pre-roll and timed steps
alternate two queues and overlap).  Prints the run's length and the average
duration of its second half -- the launches kernel_ms averages.

usage: python scripts/trace_exclusive.py <kernel_trace.csv> [--kernel fir_fft] [--launches 20]
"""
import argparse
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="fir_fft")
    ap.add_argument("--launches", type=int, default=20)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.kernel in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    best, cur = (0, 0), 0
    for i in range(1, len(rows) + 1):
        ok = (i < len(rows) and rows[i]["Queue_Id"] == rows[i - 1]["Queue_Id"]
              and int(rows[i]["Start_Timestamp"]) >= int(rows[i - 1]["End_Timestamp"]))
        if ok:
            continue
        if i - cur > best[1] - best[0]:
            best = (cur, i)
        cur = i
    run = rows[best[0]:best[1]]
    timed = run[-a.launches:]
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in timed]
    print(json.dumps({"kernel": a.kernel, "run_length": len(run), "launches": len(d),
                      "avg_ns": sum(d) / max(1, len(d)), "min_ns": min(d) if d else None,
                      "max_ns": max(d) if d else None, "all_launches_in_trace": len(rows)}))


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Where the drop-in's PCIe time goes: reads a rocprofv3 --kernel-trace
--memory-copy-trace CSV directory (scripts/gpu_run.sh dropintrace) and, per
burst of device activity (events closer than --gap ms), reports the union busy
time of H2D copies, D2H copies, filter kernels and copy kernels, the time H2D
and D2H run at the same moment, and the copies' mean concurrency.  A burst is
one file's fan-out (ProcessFile.cp:57-87's threads, tests/cpp/dropin_bench).

usage: python3 scripts/copy_overlap.py DIR [--gap MS]"""
import argparse
import csv
import glob
import os


def _rows(d, pattern):
    out = []
    for f in sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True)):
        with open(f, newline="") as fh:
            out.extend(csv.DictReader(fh))
    return out


def _col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def load(d):
    ev = []  # (start_ns, end_ns, class, bytes)
    for r in _rows(d, "*memory_copy_trace.csv"):
        kind = " ".join(str(v) for k, v in r.items() if k and ("Direction" in k or k == "Kind" or "Operation" in k))
        cls = "h2d" if "HOST_TO_DEVICE" in kind else "d2h" if "DEVICE_TO_HOST" in kind else "d2d"
        size = r.get("Size") or r.get("Bytes") or 0
        ev.append((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp")), cls, int(size or 0)))
    for r in _rows(d, "*kernel_trace.csv"):
        name = _col(r, "Kernel_Name")
        cls = "fir" if "fir_" in name else "copyk" if "copy" in name else "other"
        ev.append((int(_col(r, "Start_Timestamp")), int(_col(r, "End_Timestamp")), cls, 0))
    return sorted(ev)


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def both(a, b):
    """time during which some interval of a and some interval of b are active"""
    pts = sorted([(s, 1, 0) for s, _ in a] + [(e, -1, 0) for _, e in a] +
                 [(s, 1, 1) for s, _ in b] + [(e, -1, 1) for _, e in b])
    na = nb = 0
    last, tot = None, 0
    for t, dlt, w in pts:
        if last is not None and na > 0 and nb > 0:
            tot += t - last
        if w == 0:
            na += dlt
        else:
            nb += dlt
        last = t
    return tot


def bursts(ev, gap_ns):
    out, cur, end = [], [], -1
    for e in ev:
        if cur and e[0] > end + gap_ns:
            out.append(cur)
            cur, end = [], -1
        cur.append(e)
        end = max(end, e[1])
    if cur:
        out.append(cur)
    return out


def api_summary(d, top=12):
    """HIP API calls (rocprofv3 --hip-trace): per function, count, total and
    max duration, and the threads that made them -- where the host side of
    the fan-out waits"""
    rows = _rows(d, "*hip_api_trace.csv")
    if not rows:
        return
    agg = {}
    for r in rows:
        f = _col(r, "Function")
        t = int(_col(r, "End_Timestamp")) - int(_col(r, "Start_Timestamp"))
        a = agg.setdefault(f, [0, 0, 0, set()])
        a[0] += 1
        a[1] += t
        a[2] = max(a[2], t)
        a[3].add(r.get("Thread_Id", ""))
    print("HIP API (whole run): function, calls, total ms, max ms, threads")
    for f, (n, tot, mx, th) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"  {f:32s} {n:7d} {tot / 1e6:10.3f} {mx / 1e6:9.3f} {len(th):4d}")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--gap", type=float, default=3.0)
    a = ap.parse_args()
    ev = load(a.dir)
    if not ev:
        raise SystemExit("no trace rows under " + a.dir)
    for i, b in enumerate(bursts(ev, int(a.gap * 1e6))):
        if len(b) < 8:
            continue
        t0, t1 = b[0][0], max(e[1] for e in b)
        span = t1 - t0
        iv = {c: [(s, e) for s, e, k, _ in b if k == c] for c in ("h2d", "d2h", "fir", "copyk", "d2d")}
        busy = {c: union(v) for c, v in iv.items()}
        summed = {c: sum(e - s for s, e in v) for c, v in iv.items()}
        nbytes = {c: sum(n for _, _, k, n in b if k == c) for c in ("h2d", "d2h")}
        line = [f"burst {i}: span {span / 1e6:.3f} ms, {len(b)} events"]
        for c in ("h2d", "d2h", "fir", "copyk"):
            if iv[c]:
                conc = summed[c] / busy[c] if busy[c] else 0.0
                gbs = f", {nbytes[c] / busy[c]:.1f} GB/s while busy" if nbytes.get(c) else ""
                line.append(f"  {c:5s} n={len(iv[c]):4d} busy {busy[c] / 1e6:7.3f} ms ({busy[c] / span:5.1%} of span), "
                            f"mean concurrency {conc:.2f}{gbs}")
        if iv["h2d"] and iv["d2h"]:
            ov = both(iv["h2d"], iv["d2h"])
            line.append(f"  h2d and d2h at once: {ov / 1e6:.3f} ms ({ov / span:.1%} of span)")
        cp = iv["h2d"] + iv["d2h"] + iv["copyk"]
        if cp:
            line.append(f"  any copy busy {union(cp) / 1e6:.3f} ms ({union(cp) / span:.1%}); copy or filter busy "
                        f"{union(cp + iv['fir']) / 1e6:.3f} ms ({union(cp + iv['fir']) / span:.1%})")
        print("\n".join(line))
    api_summary(a.dir)


if __name__ == "__main__":
    main()

"""Multi-process (gloo, CPU) tests of the batch driver's sharding and peak
exchange, up to world 8 (the driver's N = 8 shapes of configs
4 and 5).  The compute is the oracle (tests only), so these
check the host logic: shard plans, windows, the MAX all-reduce of the
per-file peak vector and the per-file / batch-global normalize rule, against
a single-process run of the reference path (ProcessFile.cp:57-101)."""
import os
import sys

import numpy as np
import pytest

import batch
import gloo_ranks

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

HALF = 100  # 201 taps


def make_files(nfiles, nch, n, loud):
    import synth
    files = []
    for f in range(nfiles):
        x = synth.file_buffer(nch, n + 37 * f, 48000.0, file=f, bits=24)
        if loud and f % 2 == 0:
            x = (x * np.float32(3.0)).astype(np.float32)  # peak > 1 after filtering
        files.append(np.ascontiguousarray(x))
    return files


def make_taps():
    import oracle
    return oracle.design_lowcut(300.0, 48000.0, 2 * HALF + 1)


class OracleBackend(batch.Backend):
    """CPU stand-in for DeviceBackend built on the oracle (tests only)."""

    def __init__(self, taps):
        import oracle
        self.o, self.taps = oracle, taps

    def new_peaks(self, nfiles):
        return np.zeros(max(1, nfiles), np.float32)

    def upload(self, file, xw, x_lo, x_hi):
        return np.ascontiguousarray(xw, np.float32)

    def alloc_out(self, nch, count):
        return np.zeros((nch, count), np.float32)

    def zero_peaks(self, peaks):
        peaks[:] = 0

    def filter(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot):
        for c in range(nch):
            xf = np.zeros(n, np.float32)
            xf[x_lo:x_hi] = xw[c]
            y = np.zeros(n, np.float32)
            self.o.apply_filter_range(xf, self.taps, y, start, end, self.o.MODE_FMA)
            yw[c] = y[start:end]
        peaks[slot] = max(peaks[slot], np.abs(yw).max() if yw.size else 0.0)

    def normalize(self, yw, nch, count, peaks, slot, force):
        p = float(peaks.max() if slot is None else peaks[slot])
        if (p > 1.0 or force) and p > 0.0:
            yw[:] = (yw.astype(np.float64) * (1.0 / p)).astype(np.float32)


def _worker(rank, world, nfiles, nch, n, normalize, scope, loud):
    import torch
    import torch.distributed as dist
    files = make_files(nfiles, nch, n, loud)
    taps = make_taps()

    def allreduce(peaks):
        t = torch.from_numpy(peaks)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)

    r = batch.BatchRunner(OracleBackend(taps), rank, world, [f.shape[1] for f in files], nch,
                          HALF, normalize, scope, allreduce)
    r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
    # three steps: with an exchange each step's normalize rides in the next
    # step's filter launches (BatchRunner defer); results() runs the last
    # step's pending ones
    for _ in range(3):
        r.step()
    return rank, r.exchange, [(sh, y.copy()) for sh, y in r.results()], r.peaks.copy()


def run_dist(world, nfiles, nch, n, normalize, scope, loud):
    """The ranks' (rank, exchange, results, peaks), one gloo group (tests/gloo_ranks.py)."""
    return gloo_ranks.run(_worker, world, (nfiles, nch, n, normalize, scope, loud))


def reference(nfiles, nch, n, normalize, scope, loud):
    import oracle
    files = make_files(nfiles, nch, n, loud)
    taps = make_taps()
    if scope == "file":
        out = []
        for x in files:
            buf = x.copy()
            oracle.process_buffer(buf, taps, nthreads=1, normalize=normalize, mode=oracle.MODE_FMA)
            out.append(buf)
        return out
    ys = [np.stack([oracle.filter_channel(x[c], taps, oracle.MODE_FMA) for c in range(nch)])
          for x in files]
    peak = max(float(np.abs(y).max()) for y in ys)
    if (peak > 1.0 or normalize) and peak > 0:
        ys = [(y.astype(np.float64) * (1.0 / peak)).astype(np.float32) for y in ys]
    return ys


@pytest.mark.parametrize("world,nfiles,normalize,scope,loud,exchange", [
    (2, 2, False, "file", True, False),   # one file per rank: no collective
    (2, 2, True, "file", False, True),    # whole files + --normalize: per-file peak exchange
    (2, 2, True, "file", True, True),
    (2, 3, False, "file", True, False),   # 3 files over 2 ranks
    (2, 3, True, "file", True, True),
    (2, 1, False, "file", True, True),    # one file split over 2 ranks: peak exchange
    (2, 1, True, "file", False, True),
    (3, 2, True, "file", True, True),     # 2 files over 3 ranks (one split)
    (2, 2, True, "global", False, True),  # batch-global variant
    # the 8-GPU shapes of configs 4 and 5 (one file per rank), rehearsed on gloo
    (8, 8, False, "file", True, False),   # config 4: 8 files over 8 ranks, no collective
    (8, 8, True, "file", True, True),     # config 5: --normalize, per-file peaks exchanged
    (8, 8, True, "file", False, True),    # config 5 with every file quiet (peak < 1: forced rescale)
    (8, 8, False, "global", True, True),  # batch-global peak (loud files rescale every file)
    (8, 8, True, "global", False, True),
    (8, 1, False, "file", True, True),    # one file split over 8 ranks: windows + peak exchange
    (8, 1, True, "file", False, True),
])
def test_batch_matches_serial_reference(world, nfiles, normalize, scope, loud, exchange):
    nch, n = 2, 3000
    got = run_dist(world, nfiles, nch, n, normalize, scope, loud)
    ref = reference(nfiles, nch, n, normalize, scope, loud)
    assembled = [np.full_like(r, np.nan) for r in ref]
    peaks = []
    for rank, ex, shards, pk in got:
        assert ex == exchange
        for sh, y in shards:
            assembled[sh.file][:, sh.start:sh.end] = y
        peaks.append(pk)
    for a, r in zip(assembled, ref):
        assert np.array_equal(a, r)
    if exchange and scope == "file":
        # after the exchange every rank holds every file's own (pre-normalize) peak
        files = make_files(nfiles, nch, n, loud)
        import oracle
        taps = make_taps()
        want = np.array([max(float(np.abs(oracle.filter_channel(x[c], taps, oracle.MODE_FMA)).max())
                             for c in range(nch)) for x in files], np.float32)
        for pk in peaks:
            assert np.array_equal(pk, want)


def test_plan_shards_rules():
    p = batch.plan_shards([100, 200, 300, 400, 500, 600, 700, 800], 8)
    assert all(len(s) == 1 and s[0].start == 0 for s in p)  # one file per GPU
    assert not batch.file_is_split(p)
    p = batch.plan_shards([1000], 4)
    assert [(s[0].start, s[0].end) for s in p] == [(0, 250), (250, 500), (500, 750), (750, 1000)]
    assert batch.file_is_split(p)
    p = batch.plan_shards([10, 11, 12], 2)
    assert [[sh.file for sh in s] for s in p] == [[0, 2], [1]]
    p = batch.plan_shards([1001, 10], 3)  # file 0 over ranks 0-1, file 1 on rank 2
    assert [(s[0].file, s[0].start, s[0].end) for s in p] == [(0, 0, 500), (0, 500, 1001), (1, 0, 10)]
    assert batch.window(batch.Shard(0, 500, 1001), 1001, 100) == (400, 1001)


class LaneRecorder(OracleBackend):
    """OracleBackend that records the lane each call is issued on."""

    def __init__(self, taps):
        super().__init__(taps)
        self.lane, self.log = 0, []

    def set_lane(self, lane):
        self.lane = lane

    def filter(self, xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot):
        self.log.append(("filter", self.lane, id(yw), id(peaks)))
        super().filter(xw, x_lo, x_hi, n, nch, yw, start, end, peaks, slot)


@pytest.mark.parametrize("lanes,normalize", [(2, True), (3, False)])
def test_batch_lanes_pipeline(lanes, normalize):
    """BatchRunner(lanes > 1): step k on lane k mod lanes with that lane's own
    outputs and peak vectors; every step's results equal the serial reference."""
    nfiles, nch, n = 2, 2, 3000
    files = make_files(nfiles, nch, n, True)
    taps = make_taps()
    be = LaneRecorder(taps)
    r = batch.BatchRunner(be, 0, 1, [f.shape[1] for f in files], nch, HALF, normalize, "file",
                          lanes=lanes)
    r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
    ref = reference(nfiles, nch, n, normalize, "file", True)
    outs_by_lane = {}
    for k in range(2 * lanes + 1):
        r.step()
        res = r.results()
        for sh, y in res:
            assert np.array_equal(y, ref[sh.file][:, sh.start:sh.end])
        step_log = be.log[-nfiles:]
        assert {lane for _, lane, _, _ in step_log} == {k % lanes}
        assert be.lane == 0  # step() leaves lane 0 (the caller's stream) current
        outs_by_lane.setdefault(k % lanes, set()).update(o for _, _, o, _ in step_log)
    # a lane reuses its own output buffers; lanes never share one
    assert all(len(v) == nfiles for v in outs_by_lane.values())
    assert len(set().union(*outs_by_lane.values())) == nfiles * lanes
    with pytest.raises(ValueError):
        batch.BatchRunner(be, 0, 1, [n], nch, HALF, lanes=0)


@pytest.mark.parametrize("lanes,normalize,scope,nfiles", [(1, True, "file", 1), (1, False, "file", 3),
                                                          (2, True, "file", 2), (3, True, "global", 2)])
def test_force_exchange_defers_normalize(lanes, normalize, scope, nfiles):
    """force_exchange at world 1: the all-reduce runs every step (identity
    here), so BatchRunner defers each shard's normalize into the same shard's
    filter launch of the lane's next step (two output sets per lane, three peak
    vectors).  After any number of steps, results() (which runs the pending
    normalizes) equals the serial reference, and the peaks are each file's."""
    nch, n = 2, 3000
    files = make_files(nfiles, nch, n, True)
    taps = make_taps()
    calls = []

    class Rec(OracleBackend):
        inside = False

        def filter_normalize_prev(self, *a, **k):
            calls.append("fused")
            self.inside = True  # the CPU stand-in fuses nothing: its own normalize call is not a pass
            try:
                return super().filter_normalize_prev(*a, **k)
            finally:
                self.inside = False

        def normalize(self, *a, **k):
            if not self.inside:
                calls.append("norm")
            return super().normalize(*a, **k)

    ex = []
    r = batch.BatchRunner(Rec(taps), 0, 1, [f.shape[1] for f in files], nch, HALF, normalize, scope,
                          allreduce_max=lambda pk: ex.append(pk.copy()), lanes=lanes, force_exchange=True)
    assert r.exchange and r.defer and not r.fuse
    r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
    ref = reference(nfiles, nch, n, normalize, scope, True)
    for k in range(2 * lanes + 1):
        calls.clear()
        r.step()
        # a lane's first step has nothing pending; later steps carry one normalize per shard
        assert calls.count("fused") == (nfiles if k >= lanes else 0) and "norm" not in calls
        assert len(ex) == k + 1
    calls.clear()
    res = r.results()  # flushes the pending normalizes of every lane
    assert calls.count("norm") == lanes * nfiles
    for sh, y in res:
        assert np.array_equal(y, ref[sh.file][:, sh.start:sh.end]), sh.file
    for k in range(lanes + 1):  # results() after every step: flushed each time
        r.step()
        for sh, y in r.results():
            assert np.array_equal(y, ref[sh.file][:, sh.start:sh.end]), (k, sh.file)
    r.close()


def _preroll_worker(rank, world):
    import time
    import torch
    import sys
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    def step():  # a step with a peak exchange: a collective, slower on rank 1
        t = torch.zeros(1)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        time.sleep(0.002 * (1 + 3 * rank))

    def agree(more):
        flag = torch.tensor([1 if more else 0], dtype=torch.int32)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())

    t0 = time.perf_counter()
    # rank 1's clock runs out first (a shorter budget): without the agreement
    # rank 0 would go on stepping into a collective rank 1 never joins
    n = bench.preroll(step, 0.25 if rank == 0 else 0.1, lambda: None, agree)
    dist.barrier()
    return rank, n, time.perf_counter() - t0


def test_bench_preroll_agrees_across_ranks():
    """bench.py's pre-roll is time-based; with a peak exchange every step is a
    collective, so the ranks must run the same number of steps.  preroll()
    lets them agree after every batch (gloo, world 2, different budgets and
    step times): same count on both ranks, no deadlock."""
    got = gloo_ranks.run(_preroll_worker, 2)
    assert got[0][1] == got[1][1] and got[0][1] % 8 == 0 and got[0][1] >= 8


def _spread_worker(rank, world):
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench  # noqa: F811 (spawned process)
    # the record bench.py's rank builds (main(): `mine`), with rank-specific values
    mine = {"rank": rank, "device": f"0000:{0x11 + rank:02x}:00 (cuda:{rank})",
            "ms_per_step": 1.0 + 0.01 * rank, "kernel_ms": 0.9 + 0.02 * ((rank * 5) % world),
            "allreduce_ms_per_step": None if world == 1 else 0.1 + 0.001 * rank,
            "samples": 345_600_000 + rank}
    records = [None] * world
    dist.all_gather_object(records, mine)
    return rank, bench.rank_spread(records)


def test_rank_spread_over_8_ranks():
    """bench.rank_spread over the 8 records an N = 8 run gathers (gloo,
    world 8): every rank sees the same spread, in rank order, with the right
    min / max per field -- the diagnosable N > 1 line of SCALE runs."""
    world = 8
    got = gloo_ranks.run(_spread_worker, world)
    spreads = [sp for _, sp in got]
    assert all(sp == spreads[0] for sp in spreads)
    sp = spreads[0]
    assert sp["rank"] == list(range(world))
    assert sp["device"] == [f"0000:{0x11 + r:02x}:00 (cuda:{r})" for r in range(world)]
    assert sp["ms_per_step"] == [1.0 + 0.01 * r for r in range(world)]
    assert sp["ms_per_step_min"] == 1.0 and sp["ms_per_step_max"] == 1.0 + 0.01 * 7
    assert sp["kernel_ms_min"] == 0.9 and abs(sp["kernel_ms_max"] - (0.9 + 0.02 * 7)) < 1e-12
    assert sp["allreduce_ms_per_step_max"] == 0.1 + 0.001 * 7
    assert sp["samples"] == [345_600_000 + r for r in range(world)]
    assert sp["samples_min"] == 345_600_000 and sp["samples_max"] == 345_600_007
    # a world-1 record has no collective: the field's min / max are null
    one = bench.rank_spread([{"rank": 0, "device": "x", "ms_per_step": 1.0, "kernel_ms": 0.9,
                               "allreduce_ms_per_step": None, "samples": 1}])
    assert one["allreduce_ms_per_step_min"] is None and one["allreduce_ms_per_step_max"] is None

"""GPU tests of the sharded-file entry point (lcfir_filter_window_dev) and of
the batch driver's DeviceBackend (single rank), against the oracle."""
import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu

RMS_TOL = 1e-9


@pytest.fixture(scope="module")
def tt():
    import torch  # before lcfir: one HIP runtime in the process
    assert torch.cuda.is_available()
    import lcfir
    lcfir.load()
    assert len(lcfir.hip_runtimes()) == 1, lcfir.hip_runtimes()
    return torch, lcfir


def rms(a, b):
    d = np.asarray(a, np.float64) - np.asarray(b, np.float64)
    return float(np.sqrt(np.mean(d * d))) if d.size else 0.0


@pytest.mark.parametrize("method", ["direct", "fft"])
def test_filter_window_matches_oracle(tt, oracle_mod, method):
    torch, lc = tt
    g = load_golden("float_source")
    x, taps = g["x"][:3], g["taps"]        # 3 channels x 3000, 1601 taps
    nch, n = x.shape
    half = (taps.size - 1) // 2
    flt = lc.Filter(taps, method=method)
    ref = np.stack([oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_FMA) for c in range(nch)])
    # odd and even window edges, ranges touching both ends, a 1-sample range
    for start, end in [(0, n), (1, 2999), (777, 1501), (2998, 2999), (0, 5), (1333, 3000)]:
        lo, hi = max(0, start - half), min(n, end + half)
        for extra_lo, extra_hi in [(0, 0), (min(lo, 3), min(n - hi, 5))]:
            wlo, whi = lo - extra_lo, hi + extra_hi
            xw = torch.from_numpy(np.ascontiguousarray(x[:, wlo:whi])).cuda()
            yw = torch.full((nch, end - start), 7.0, dtype=torch.float32, device="cuda")
            pk = torch.zeros(1, dtype=torch.float32, device="cuda")
            flt.filter_window_dev(xw, wlo, whi, whi - wlo, n, nch, yw, start, end - start, start,
                                  end, pk, 0, peak_stride=0)
            torch.cuda.synchronize()
            y = yw.cpu().numpy()
            if method == "direct":
                assert np.array_equal(y, ref[:, start:end]), (start, end)
            for c in range(nch):
                assert rms(y[c], g["y"][c][start:end]) <= RMS_TOL
            assert pk.item() == np.abs(y).max()


def test_filter_window_rejects_short_window(tt):
    torch, lc = tt
    flt = lc.Filter(np.ones(101))
    xw = torch.zeros((1, 100), device="cuda")
    yw = torch.zeros((1, 10), device="cuda")
    with pytest.raises(lc.LcfirError) as e:
        flt.filter_window_dev(xw, 500, 600, 100, 1000, 1, yw, 540, 10, 540, 550)
    assert "does not cover" in str(e.value)


@pytest.mark.parametrize("normalize,loud,lanes", [(False, False, 1), (True, False, 1), (False, True, 1),
                                                  (True, True, 2), (False, True, 3)])
def test_device_batch_runner(tt, oracle_mod, normalize, loud, lanes):
    """One rank, three files: BatchRunner + DeviceBackend vs ProcessFile.cp:57-101
    (lanes > 1: consecutive steps pipelined over streams; every step's outputs checked)."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 801)
    files = [synth.file_buffer(2, 20000 + 1001 * f, 48000.0, file=f, bits=24) for f in range(3)]
    if loud:
        files[1] = (files[1] * np.float32(3.0)).astype(np.float32)
    flt = lc.Filter(taps, method="direct")
    _run_batch_checks(torch, oracle_mod, flt, files, taps, normalize, lanes)


def _ulps(a, b):
    ia = np.asarray(a, np.float32).view(np.int32).astype(np.int64)
    ib = np.asarray(b, np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return np.abs(ia - ib)


@pytest.mark.parametrize("ntaps,lanes,normalize", [(4001, 2, False), (4001, 2, True), (12001, 2, False),
                                                   (4001, 3, True)])
def test_device_batch_runner_fft_pipelined(tt, oracle_mod, ntaps, lanes, normalize):
    """The headline path exactly as bench.py runs it: the FFT kernel (4001 taps;
    12 001 = two partitions), consecutive steps pipelined over lanes -- every
    step's outputs, read through results() with NO device synchronisation
    (results() orders the caller's stream behind the step's lane), against the
    long-double oracle (<= 1 ulp, RMS <= 1e-9)."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, ntaps)
    files = [synth.file_buffer(2, 40000 + 3001 * f, 48000.0, file=f, bits=24) for f in range(3)]
    files[2] = (files[2] * np.float32(3.0)).astype(np.float32)  # loud: rescaled by 1/peak
    flt = lc.Filter(taps, method="fft")
    half = (taps.size - 1) // 2
    refs = {}
    for f in range(3):
        y = np.stack([oracle_mod.filter_channel(files[f][c], taps, oracle_mod.MODE_LD) for c in range(2)])
        peak = float(np.abs(y).max())
        if normalize or peak > 1.0:
            y = (y.astype(np.float64) * (1.0 / peak)).astype(np.float32)
        refs[f] = y
    be = batch.DeviceBackend(flt, torch.device("cuda", 0), lanes=lanes)
    r = batch.BatchRunner(be, 0, 1, [f.shape[1] for f in files], 2, half, normalize, "file", lanes=lanes)
    r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
    for k in range(2 * lanes + 1):  # an odd number of steps: the last one on lane 0 ... lanes-1
        r.step()
        for sh, y in r.results():
            got = y.cpu().numpy()  # on the caller's stream, no synchronize()
            want = refs[sh.file]
            assert _ulps(got, want).max() <= 1, (k, sh.file)
            d = got.astype(np.float64) - want
            assert np.sqrt(np.mean(d * d)) <= RMS_TOL
    r.close()


@pytest.mark.parametrize("ntaps,world", [(4001, 2), (4003, 3), (19201, 4)])
def test_split_file_ranks_bit_identical(tt, oracle_mod, ntaps, world):
    """A file split by sample range over `world` ranks (plan_shards, one GPU
    standing in for all of them): each rank reads lcfir_ctx_window's input
    window (DeviceBackend.window, the FFT's whole segments), so the ranks'
    outputs put together equal the unsplit run's bit for bit -- the result
    does not depend on the GPU count."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(25.0, 48000.0, ntaps)
    half = (ntaps - 1) // 2
    n = 250_001
    x = synth.file_buffer(2, n, 48000.0, file=4, bits=24)
    flt = lc.Filter(taps, method="fft")

    def run(rank, w):
        be = batch.DeviceBackend(flt, torch.device("cuda", 0))
        r = batch.BatchRunner(be, rank, w, [n], 2, half, False, "file",
                              allreduce_max=lambda t: None)  # the peak exchange is not under test
        r.prepare(lambda f, lo, hi: x[:, lo:hi])
        r.step()
        out = [(sh.start, sh.end, y.cpu().numpy()) for sh, y in r.results()]
        r.close()
        return out

    (s0, e0, whole), = run(0, 1)
    assert (s0, e0) == (0, n)
    got = np.zeros_like(whole)
    covered = 0
    for rank in range(world):
        for s, e, y in run(rank, world):
            got[:, s:e] = y
            covered += e - s
    assert covered == n
    assert np.array_equal(got, whole)


@pytest.mark.parametrize("lanes,normalize,per_lane", [(1, False, True), (3, True, True), (3, True, False)])
def test_graphed_steps_equal_eager(tt, oracle_mod, lanes, normalize, per_lane):
    """batch.GraphedSteps (the steps captured into one HIP graph, 2 x lanes
    steps per replay, lanes forked from lane 0's stream) gives the eager
    steps' bytes: config 1's kernel (19 201 taps, two partitions, its
    partial-sum scratch) over two 48 000-sample files, one loud.  The output
    buffers are poisoned before the replay, so they come from the graph."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 19201)
    half = (taps.size - 1) // 2
    files = [synth.file_buffer(1, 48_000, 48000.0, file=f, bits=16) for f in range(2)]
    files[1] = (files[1] * np.float32(2.0)).astype(np.float32)
    flt = lc.Filter(taps, method="fft")
    dev = torch.device("cuda", 0)

    def runner():
        be = batch.DeviceBackend(flt, dev, lanes=lanes, own_streams=True)
        r = batch.BatchRunner(be, 0, 1, [48_000, 48_000], 1, half, normalize, "file", lanes=lanes)
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        for _ in range(2 * lanes):
            r.step()
        return be, r

    be, r = runner()
    want = [(sh.file, y.cpu().numpy()) for sh, y in r.results()]
    want_pk = r.peaks.cpu().numpy()
    r.close()
    be, r = runner()
    g = batch.GraphedSteps(r, be, per_lane=per_lane)
    assert g.per_replay == 2 * lanes and len(g.graphs) == (lanes if per_lane else 1)
    for sets in r._outs:
        for outs in sets:
            for y in outs:
                y.fill_(float("nan"))
    g.replay()
    torch.cuda.synchronize(dev)
    got = [(sh.file, y.cpu().numpy()) for sh, y in r.results()]
    assert np.array_equal(r.peaks.cpu().numpy(), want_pk)
    for (fa, ya), (fb, yb) in zip(want, got):
        assert fa == fb and np.array_equal(ya, yb), fa
    g.replay()  # again: the same bytes (each lane's peak vectors alternate inside the graph)
    torch.cuda.synchronize(dev)
    assert all(np.array_equal(y.cpu().numpy(), w) for (_, y), (_, w) in zip(r.results(), want))
    r.close()
    for f, y in want:
        ref = files[f].copy()
        oracle_mod.process_buffer(ref, taps, nthreads=1, normalize=normalize, mode=oracle_mod.MODE_LD)
        assert _ulps(y, ref).max() <= 1, f
    torch.cuda.set_stream(torch.cuda.default_stream(dev))  # the steps left lane 0's stream current
    be = batch.DeviceBackend(flt, dev)  # lane 0 = the default stream: not capturable
    with pytest.raises(ValueError):
        batch.GraphedSteps(batch.BatchRunner(be, 0, 1, [48_000], 1, half), be)


def _run_batch_checks(torch, oracle_mod, flt, files, taps, normalize, lanes):
    import batch
    be = batch.DeviceBackend(flt, torch.device("cuda", 0), lanes=lanes)
    r = batch.BatchRunner(be, 0, 1, [f.shape[1] for f in files], 2, (taps.size - 1) // 2, normalize,
                          "file", lanes=lanes)
    r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
    refs = {}
    for f in range(3):
        refs[f] = files[f].copy()
        oracle_mod.process_buffer(refs[f], taps, nthreads=1, normalize=normalize,
                                  mode=oracle_mod.MODE_FMA)
    assert not r.exchange
    steps = []
    for _ in range(2 * lanes):  # steps are repeatable (peaks reset each step, per lane)
        r.step()
        steps.append(r.results())
    torch.cuda.synchronize()
    be.set_lane(0)
    assert len({id(y) for res in steps for _, y in res}) == 3 * lanes  # one output set per lane
    for res in steps:
        for sh, y in res:
            assert np.array_equal(y.cpu().numpy(), refs[sh.file][:, sh.start:sh.end])
    if lanes > 1:
        # re-prepare straight behind steps still in flight on every lane
        for _ in range(lanes):
            r.step()
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        r.step()
        r.step()
        torch.cuda.synchronize()
        for sh, y in r.results():
            assert np.array_equal(y.cpu().numpy(), refs[sh.file][:, sh.start:sh.end])


def test_normalize_clear_dev(tt):
    """lcfir_normalize_clear_dev = lcfir_normalize_dev + zeroing a separate
    peak vector in the same launch (the batch driver's next-step slots)."""
    torch, lc = tt
    rng = np.random.default_rng(3)
    y0 = (rng.standard_normal((2, 5003)) * 1.5).astype(np.float32)
    pk = float(np.abs(y0).max())
    dev = torch.device("cuda", 0)
    peaks = torch.tensor([0.25, pk, 0.5], dtype=torch.float32, device=dev)
    for force in (False, True):
        ya = torch.from_numpy(y0).to(dev)
        yb = ya.clone()
        clear = torch.full((5,), 7.0, dtype=torch.float32, device=dev)
        lc.normalize_dev(ya, 5003, 2, 5003, peaks, 3, force)
        lc.normalize_clear_dev(yb, 5003, 2, 5003, peaks, 3, force, clear, 4)
        torch.cuda.synchronize()
        assert torch.equal(ya, yb)
        assert clear.cpu().tolist() == [0.0, 0.0, 0.0, 0.0, 7.0]
        assert peaks.cpu().tolist()[1] == pk  # the slots read are left alone
    ref = (y0.astype(np.float64) * (1.0 / pk)).astype(np.float32)
    assert np.array_equal(yb.cpu().numpy(), ref)
    # nothing to rescale (nch = 0): the slots are still cleared
    clear = torch.full((3,), 7.0, dtype=torch.float32, device=dev)
    lc.normalize_clear_dev(yb, 5003, 0, 5003, peaks, 3, False, clear, 3)
    torch.cuda.synchronize()
    assert clear.cpu().tolist() == [0.0, 0.0, 0.0]
    # the slots to clear must not overlap the slots read
    with pytest.raises(lc.LcfirError) as e:
        lc.normalize_clear_dev(yb, 5003, 2, 5003, peaks, 3, False, peaks[2:], 1)
    assert "overlap" in str(e.value)


def test_normalize_large_buffer(tt):
    """The rescale loop at full-file sizes (4 loads in flight per thread plus
    the remainder loop): bit-identical to (float)((double)y * (1 / peak)) on
    every sample, ragged lengths, a non-16-byte-aligned channel (scalar path)."""
    torch, lc = tt
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    for n, offset in [(3_000_001, 0), (1_048_576 + 5, 0), (2_500_003, 1)]:
        y0 = (rng.standard_normal((2, n)) * 1.7).astype(np.float32)
        pk = float(np.abs(y0).max())
        buf = torch.zeros(2 * n + 8, dtype=torch.float32, device=dev)
        view = buf[offset:offset + 2 * n].view(2, n)  # offset 1: channel bases 4-byte aligned only
        view.copy_(torch.from_numpy(y0))
        peaks = torch.tensor([pk], dtype=torch.float32, device=dev)
        lc.normalize_dev(view, n, 2, n, peaks, 1, False)
        torch.cuda.synchronize()
        ref = (y0.astype(np.float64) * (1.0 / pk)).astype(np.float32)
        assert np.array_equal(view.cpu().numpy(), ref), (n, offset)


@pytest.mark.parametrize("kind", ["sym", "general", "parts", "direct"])
def test_filter_window_norm_matches_separate_passes(tt, oracle_mod, kind):
    """lcfir_filter_window_norm_dev (a previous file's normalize carried by the
    filter call; fused into the FFT launch for single-partition filters) is
    bit-identical to lcfir_filter_window_dev + lcfir_normalize_dev: the call's
    own outputs and peak, and the rescaled buffer -- for counts of every
    residue mod 4 (the float4 body and the 1..3-float tail), a peak above 1,
    a quiet peak with and without force, and a quiet peak left unscaled."""
    torch, lc = tt
    import synth
    rng = np.random.default_rng(11)
    if kind == "direct":
        taps, method = oracle_mod.design_lowcut(20.0, 48000.0, 801), "direct"
    elif kind == "parts":
        taps, method = oracle_mod.design_lowcut(20.0, 48000.0, 19201), "fft"
    else:
        taps, method = oracle_mod.design_lowcut(20.0, 48000.0, 4001), "fft"
        if kind == "general":
            taps = taps.copy()
            taps[7] += 1e-3  # asymmetric: the general (complex) pair table
    flt = lc.Filter(taps, method=method)
    n, nch = 150_003, 2
    x = synth.file_buffer(nch, n, 48000.0, file=3, bits=24)
    dx = torch.from_numpy(x).cuda()
    for count, peak_val, force in [(200_000, 1.7, False), (100_001, 0.6, True), (99_998, 0.6, False),
                                   (77_779, 2.5, True), (4_099, 3.0, False), (3, 1.25, False)]:
        prev = (rng.standard_normal(count) * 0.3).astype(np.float32)
        res = []
        for fused in (False, True):
            dy = torch.empty((nch, n), dtype=torch.float32, device="cuda")
            dpk = torch.zeros(1, dtype=torch.float32, device="cuda")
            dprev = torch.from_numpy(prev.copy()).cuda()
            dppk = torch.tensor([peak_val], dtype=torch.float32, device="cuda")
            if fused:
                flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, 0, dprev, count,
                                           dppk, 1, force)
            else:
                flt.filter_window_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, peak_stride=0)
                lc.normalize_dev(dprev, count, 1, count, dppk, 1, force)
            torch.cuda.synchronize()
            res.append((dy.cpu().numpy(), dpk.cpu().numpy(), dprev.cpu().numpy()))
        (y0, p0, r0), (y1, p1, r1) = res
        assert np.array_equal(y0, y1) and np.array_equal(p0, p1), (kind, count)
        assert np.array_equal(r0, r1), (kind, count)
        scaled = peak_val > 1.0 or force
        want = (prev.astype(np.float64) * (1.0 / np.float64(np.float32(peak_val)))).astype(np.float32) \
            if scaled else prev
        assert np.array_equal(r1, want), (kind, count)


@pytest.mark.parametrize("lanes,normalize", [(1, True), (1, False), (2, True)])
def test_batch_runner_fused_normalize_identical(tt, oracle_mod, lanes, normalize):
    """BatchRunner's fused per-file normalize (each file's rescale carried by
    the next file's filter launch, the last file's as its own pass) gives the
    same bytes as the unfused step, over 4 files of ragged lengths with one
    loud file, every step of a pipelined run."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    half = (taps.size - 1) // 2
    files = [synth.file_buffer(2, 60_001 + 7_777 * f, 48000.0, file=f, bits=24) for f in range(4)]
    files[1] = (files[1] * np.float32(2.5)).astype(np.float32)
    flt = lc.Filter(taps, method="fft")
    outs = []
    for fuse in (False, True):
        be = batch.DeviceBackend(flt, torch.device("cuda", 0), lanes=lanes)
        r = batch.BatchRunner(be, 0, 1, [f.shape[1] for f in files], 2, half, normalize, "file",
                              lanes=lanes, fuse_normalize=fuse)
        assert r.fuse == fuse
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        got = []
        for _ in range(2 * lanes + 1):
            r.step()
            got.append([(sh.file, y.cpu().numpy(), float(r.peaks[sh.file].item())) for sh, y in r.results()])
        r.close()
        outs.append(got)
    for a, b in zip(*outs):
        for (fa, ya, pa), (fb, yb, pb) in zip(a, b):
            assert fa == fb and pa == pb and np.array_equal(ya, yb), fa


def test_filter_window_norm_fallbacks(tt, oracle_mod):
    """The cases lcfir_filter_window_norm_dev does not fuse still give
    normalize_dev's bytes: a buffer that is not 16-B aligned, several peak
    slots (the max is the peak), ncount = 0 (a plain filter call), and a
    slice too large for one launch's units (a short current file carrying a
    long previous one).  Bad arguments are rejected."""
    torch, lc = tt
    import synth
    rng = np.random.default_rng(5)
    flt = lc.Filter(oracle_mod.design_lowcut(20.0, 48000.0, 4001), method="fft")
    n, nch = 30_001, 1
    x = synth.file_buffer(nch, n, 48000.0, file=2, bits=24)
    dx = torch.from_numpy(x).cuda()
    cases = [(50_001, 1, [1.5]), (40_000, 0, [0.5, 2.25, 1.75]), (0, 0, [3.0]), (3_000_000, 0, [1.5])]
    for count, offset, peaks in cases:
        prev = (rng.standard_normal(count + offset) * 0.4).astype(np.float32)
        res = []
        for fused in (False, True):
            dy = torch.empty((nch, n), dtype=torch.float32, device="cuda")
            dpk = torch.zeros(1, dtype=torch.float32, device="cuda")
            dprev = torch.from_numpy(prev.copy()).cuda()
            dppk = torch.tensor(peaks, dtype=torch.float32, device="cuda")
            view = dprev[offset:]  # offset 1: 4-byte aligned only
            if fused:
                flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, 0, view, count,
                                           dppk, len(peaks), False)
            else:
                flt.filter_window_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, dpk, peak_stride=0)
                if count:
                    lc.normalize_dev(view, count, 1, count, dppk, len(peaks), False)
            torch.cuda.synchronize()
            res.append((dy.cpu().numpy(), dpk.cpu().numpy(), dprev.cpu().numpy()))
        (y0, p0, r0), (y1, p1, r1) = res
        assert np.array_equal(y0, y1) and np.array_equal(p0, p1), count
        assert np.array_equal(r0, r1), count
    dy = torch.empty((nch, n), dtype=torch.float32, device="cuda")
    with pytest.raises(lc.LcfirError):  # the rescaled buffer may not overlap the outputs
        flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, None, 0, dy, n,
                                   torch.ones(1, device="cuda"), 1, True)
    with pytest.raises(lc.LcfirError):  # at least one peak slot
        flt.filter_window_norm_dev(dx, 0, n, n, n, nch, dy, 0, n, 0, n, None, 0, dx, n,
                                   torch.ones(1, device="cuda"), 0, True)


@pytest.mark.parametrize("lanes", [1, 3])
def test_graph_replay_then_eager_steps(tt, oracle_mod, lanes):
    """GraphedSteps.replay() followed by a number of eager steps that is not a
    multiple of the replay's step count, with --normalize (every step rescales
    and clears peak vectors): the lanes' eager steps must queue behind the
    graph's work on their buffers and the graph behind earlier eager work
    (one-graph mode launches on lane 0's stream only).  Every output and peak
    equals an all-eager run of the same step count."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    half = (taps.size - 1) // 2
    files = [synth.file_buffer(1, 200_000 + 1_001 * f, 48000.0, file=f, bits=16) for f in range(2)]
    files[1] = (files[1] * np.float32(2.0)).astype(np.float32)
    flt = lc.Filter(taps, method="fft")
    dev = torch.device("cuda", 0)
    nf = [f.shape[1] for f in files]

    def fresh():
        be = batch.DeviceBackend(flt, dev, lanes=lanes, own_streams=True)
        r = batch.BatchRunner(be, 0, 1, nf, 1, half, True, "file", lanes=lanes)
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        return be, r

    be, r = fresh()
    g = batch.GraphedSteps(r, be)  # one graph for every lane
    g.replay()
    extra = g.per_replay // 2 + 1
    for _ in range(extra):
        r.step()
    got = [(sh.file, y.cpu().numpy()) for sh, y in r.results()]
    got_pk = r.peaks.cpu().numpy()
    r.close()
    total = sum(r._steps)  # eager steps the graph stood for are counted at capture
    be, r = fresh()
    for _ in range(total):
        r.step()
    want = [(sh.file, y.cpu().numpy()) for sh, y in r.results()]
    assert np.array_equal(r.peaks.cpu().numpy(), got_pk)
    for (fa, ya), (fb, yb) in zip(want, got):
        assert fa == fb and np.array_equal(ya, yb), fa
    r.close()
    torch.cuda.set_stream(torch.cuda.default_stream(dev))


@pytest.mark.parametrize("lanes", [2, 3])
def test_graph_replay_results_on_allocation_stream(tt, oracle_mod, lanes):
    """results() straight after a one-graph replay, read on the stream the
    runner's buffers were allocated on (not lane 0's, where the graph ran):
    publish() must order that stream behind the graph, which ran every lane's
    steps on lane 0's stream (the lazy lane waits, DeviceBackend._after_graph).
    The latest lane's outputs are poisoned and lane 0's stream spins before the
    replay, so a read that does not wait for the graph sees NaN -- where the
    two streams sit on different hardware queues: HIP multiplexes streams onto
    GPU_MAX_HW_QUEUES (4 here), and two streams on one queue are ordered anyway
    (on the one-GPU box the unfixed publish() passed this test for that reason).
    Correct by construction; kept as the regression check for boxes that map
    the streams apart."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    half = (taps.size - 1) // 2
    files = [synth.file_buffer(2, 4_000_000, 48000.0, file=20 + f, bits=24) for f in range(2)]
    flt = lc.Filter(taps, method="fft")
    dev = torch.device("cuda", 0)
    # a stream of its own: the legacy default stream would order itself
    # behind every other stream and hide a missing wait
    alloc = torch.cuda.Stream(dev)
    nf = [f.shape[1] for f in files]

    def fresh():
        torch.cuda.set_stream(alloc)
        be = batch.DeviceBackend(flt, dev, lanes=lanes, own_streams=True)
        r = batch.BatchRunner(be, 0, 1, nf, 2, half, False, "file", lanes=lanes)
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        return be, r

    be, r = fresh()
    g = batch.GraphedSteps(r, be)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(be.streams[0]):
        for y in r.output_buffer_set(lanes - 1):
            y.fill_(float("nan"))
        torch.cuda._sleep(40_000_000)  # ~20 ms of spinning ahead of the replay on lane 0's stream
    g.replay()
    res = r.results()
    with torch.cuda.stream(alloc):
        # a device-side read on that stream (a copy to host memory could be
        # ordered by the copy engine instead)
        snap = [y.clone() for _, y in res]
    torch.cuda.synchronize(dev)
    got = [z.cpu().numpy() for z in snap]
    r.close()
    torch.cuda.set_stream(alloc)
    total = sum(r._steps)
    be, r = fresh()
    for _ in range(total):
        r.step()
    want = [y.cpu().numpy() for _, y in r.results()]
    r.close()
    torch.cuda.set_stream(alloc)
    torch.cuda.set_stream(torch.cuda.default_stream(dev))
    for a, b in zip(want, got):
        assert not np.isnan(b).any()
        assert np.array_equal(a, b)


@pytest.fixture(scope="module")
def nccl_world1(tt):
    """A world-size-1 RCCL process group on this GPU (torch.distributed
    backend "nccl" is RCCL on ROCm): BatchRunner(force_exchange=True) then
    runs the config-5 peak all-reduce through RCCL on the lane streams."""
    torch, _ = tt
    import socket
    import torch.distributed as dist
    if dist.is_initialized():
        pytest.skip("a process group already exists")
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    yield dist
    dist.destroy_process_group()


@pytest.mark.parametrize("lanes,normalize", [(1, True), (2, True), (1, False)])
def test_rccl_peak_exchange_world1(tt, oracle_mod, nccl_world1, lanes, normalize):
    """The RCCL leg on the device: torch_allreduce_max (ncclAllReduce MAX of
    the [num_files] peak vector) on the lane streams every step, with each
    file's normalize deferred into the next step's filter launch (BatchRunner
    defer).  Outputs and peaks are bit-identical to the no-exchange run
    (normalize fused within the step), over several steps, and the output
    matches ProcessFile.cp:91-101 against the oracle."""
    torch, lc = tt
    import batch
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, 4001)
    half = (taps.size - 1) // 2
    files = [synth.file_buffer(2, 150_001 + 9_999 * f, 48000.0, file=f, bits=24) for f in range(3)]
    files[2] = (files[2] * np.float32(3.0)).astype(np.float32)
    flt = lc.Filter(taps, method="fft")
    dev = torch.device("cuda", 0)
    res = []
    for exchange in (False, True):
        be = batch.DeviceBackend(flt, dev, lanes=lanes)
        r = batch.BatchRunner(be, 0, 1, [f.shape[1] for f in files], 2, half, normalize, "file",
                              batch.torch_allreduce_max(), lanes=lanes, force_exchange=exchange)
        assert r.exchange == exchange and r.defer == exchange
        r.prepare(lambda f, lo, hi: files[f][:, lo:hi])
        for _ in range(2 * lanes + 1):
            r.step()
        res.append(([(sh.file, y.cpu().numpy()) for sh, y in r.results()], r.peaks.cpu().numpy()))
        r.close()
    (ya, pa), (yb, pb) = res
    assert np.array_equal(pa, pb)
    for (fa, a), (fb, b) in zip(ya, yb):
        assert fa == fb and np.array_equal(a, b), fa
    for f, y in ya:
        ref = files[f].copy()
        oracle_mod.process_buffer(ref, taps, nthreads=1, normalize=normalize, mode=oracle_mod.MODE_LD)
        assert _ulps(y, ref).max() <= 1, f


@pytest.mark.parametrize("parts_taps", [4001, 19201])
def test_graph_replay_after_fft_retuning(tt, oracle_mod, parts_taps):
    """lcfir_ctx_set_fft_tuning drops the ctx's plan, but a HIP
    graph captured earlier passes that plan's tables (pair table, twiddles,
    task words) to its kernels: they are retired until lcfir_ctx_destroy, not
    freed, so the graph still replays the captured bytes after a retune and
    after eager calls that build and use the new plan.  19 201 taps at L =
    16 384 forced: two partitions, so the per-stream scratch is captured too."""
    torch, lc = tt
    import synth
    taps = oracle_mod.design_lowcut(20.0, 48000.0, parts_taps)
    n = 120_000
    x = synth.file_buffer(2, n, 48000.0, file=21, bits=24)
    flt = lc.Filter(taps, method="fft")
    flt.set_fft_tuning(seg_len=16384)
    dx = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    dy = torch.zeros((2, n), dtype=torch.float32, device="cuda")
    s = torch.cuda.Stream()
    flt.filter_channels_dev(dx, n, 2, n, dy, n, None, stream=s.cuda_stream)  # eager: plan + scratch
    torch.cuda.synchronize()
    y0 = dy.cpu().numpy().copy()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        flt.filter_channels_dev(dx, n, 2, n, dy, n, None, stream=s.cuda_stream)
    torch.cuda.synchronize()
    flt.set_fft_tuning(seg_len=32768)  # the captured plan is dropped from the ctx
    dy2 = torch.zeros((2, n), dtype=torch.float32, device="cuda")
    flt.filter_channels_dev(dx, n, 2, n, dy2, n, None, stream=s.cuda_stream)  # the new plan
    torch.cuda.synchronize()
    assert flt.fft_info["seg_len"] == 32768
    dy.zero_()
    torch.cuda.synchronize()
    with torch.cuda.stream(s):
        g.replay()
    torch.cuda.synchronize()
    assert np.array_equal(dy.cpu().numpy(), y0)
    y2 = dy2.cpu().numpy()
    for c in range(2):
        idx = np.r_[np.arange(0, 50), np.arange(n - 50, n), np.arange(5000, n, 997)]
        ref, _ = oracle_mod.filter_points(x[c], taps, idx, oracle_mod.MODE_LD)
        assert rms(y2[c][idx], ref) <= RMS_TOL
    del g
    flt.close()

"""End-to-end: the lowcut tool on real WAVE/AIFF files, on the GPU, against the
oracle's ProcessFile.cp:27-120 (decode -> long-double filter -> per-file
peak/normalize rule -> encode).  Every byte outside the sample payload must be
identical to the input (chunk copy, ProcessFile.cp:103-112); samples must
match the oracle to 1 LSB, with 1-LSB differences allowed only where the f32
filter output sits on a quantiser boundary (rare)."""
import os
import subprocess

import numpy as np
import pytest

import pcm_ref
from conftest import ROOT

pytestmark = pytest.mark.gpu

LOWCUT = os.path.join(ROOT, "audio-fir-filter_amd", "lowcut")


def lowcut(*args):
    r = subprocess.run([LOWCUT, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    return r.stdout


def info(path):
    r = subprocess.run([LOWCUT, "--info", str(path)], capture_output=True, text=True, timeout=60)
    line = r.stdout.split(" chunks=", 1)[0]
    return dict(kv.split("=", 1) for kv in line.split()[3:])


def expected(oracle_mod, x, rate, fmt, freq, slope, normalize):
    """Oracle restatement of process_file's compute on decoded samples."""
    nt = oracle_mod.lowcut_ntaps(slope, rate)
    taps = oracle_mod.design_lowcut(freq, rate, nt)
    y = np.stack([oracle_mod.filter_channel(x[c], taps, oracle_mod.MODE_LD) for c in range(x.shape[0])])
    peak = float(np.abs(y).max())
    if (peak > 1.0 or normalize) and peak > 0:
        y = (y.astype(np.float64) * (1.0 / peak)).astype(np.float32)
    return y


def check_file(oracle_mod, src, dst, x_in, rate, fmt, freq, slope, normalize):
    a, b = open(src, "rb").read(), open(dst, "rb").read()
    d = info(src)
    off, nbytes = int(d["data_offset"]), int(d["data_bytes"])
    assert len(a) == len(b)
    assert a[:off] == b[:off] and a[off + nbytes:] == b[off + nbytes:]  # every other byte kept
    nch = x_in.shape[0]
    got = pcm_ref.np_decode(b[off:off + nbytes], fmt, nch)
    want_f = expected(oracle_mod, x_in, rate, fmt, freq, slope, normalize)
    want = pcm_ref.np_decode(pcm_ref.np_encode(want_f, fmt), fmt, nch)
    if fmt.startswith("f32"):
        dd = got.astype(np.float64) - want_f
        assert np.sqrt(np.mean(dd * dd)) <= 1e-9
    else:
        lsb = 1.0 / (1 << (8 * pcm_ref.NB[fmt[:3]] - 1))
        diff = np.abs(got.astype(np.float64) - want.astype(np.float64))
        assert diff.max() <= lsb * 1.000001
        assert np.mean(diff > 0) <= 1e-4


def tone(nch, n, rate, amp=0.4, bits=24):
    import synth
    return synth.file_buffer(nch, n, float(rate), file=3, bits=bits) * np.float32(amp / 0.5)


def test_config1_mono_int16_wav(tmp_path, oracle_mod):
    """BASELINE config 1: 1 s mono 48 kHz int16 WAV, -f 20 -s 10 (19 201 taps)."""
    import synth
    x = synth.file_buffer(1, 48000, 48000.0, file=0, bits=16)
    src, dst = tmp_path / "c1.wav", tmp_path / "c1_out.wav"
    pcm_ref.write_wave(src, x, 48000, "s16le", extra_chunks=[(b"LIST", b"INFOICMT\x04\x00\x00\x00cfg1")])
    xq = pcm_ref.np_decode(pcm_ref.np_encode(x, "s16le"), "s16le", 1)
    out = lowcut("-v", "-f", 20, "-s", 10, src, dst)
    assert "19201 taps (fft)" in out  # two partitions of 9601 taps (fir_fft.hpp)
    check_file(oracle_mod, src, dst, xq, 48000, "s16le", 20, 10, False)


@pytest.mark.parametrize("container,fmt,comp", [("wav", "s24le", None), ("aif", "s24be", None),
                                                ("aif", "s16le", b"sowt"), ("wav", "f32le", None),
                                                ("aif", "f32be", b"fl32")])
def test_formats_fft_path(tmp_path, oracle_mod, container, fmt, comp):
    x = tone(2, 96000, 48000)
    src, dst = tmp_path / f"in.{container}", tmp_path / f"out.{container}"
    if container == "wav":
        pcm_ref.write_wave(src, x, 48000, fmt)
    else:
        pcm_ref.write_aiff(src, x, 48000, fmt, aifc_comp=comp, extra_chunks=[(b"ANNO", b"lcfir!")])
    xq = pcm_ref.np_decode(pcm_ref.np_encode(x, fmt), fmt, 2)
    out = lowcut("-v", "-f", 20, "-s", 48, src, dst)
    assert "4001 taps (fft)" in out
    check_file(oracle_mod, src, dst, xq, 48000, fmt, 20, 48, False)


@pytest.mark.parametrize("slope,method,ntaps", [(4000, "direct", 49), (2000, "fft", 97)])
def test_short_filter_method_choice(tmp_path, oracle_mod, slope, method, ntaps):
    """A wide slope gives a short kernel: AUTO runs the direct kernel below
    64 taps (-s 4000 at 48 kHz: 49 taps) and the FFT from 64 (-s 2000: 97).
    Same file contract and oracle as every other case."""
    x = tone(2, 50_001, 48000)
    src, dst = tmp_path / "in.wav", tmp_path / "out.wav"
    pcm_ref.write_wave(src, x, 48000, "s24le")
    xq = pcm_ref.np_decode(pcm_ref.np_encode(x, "s24le"), "s24le", 2)
    out = lowcut("-v", "-f", 1000, "-s", slope, src, dst)
    assert f"{ntaps} taps ({method})" in out
    check_file(oracle_mod, src, dst, xq, 48000, "s24le", 1000, slope, False)


@pytest.mark.parametrize("normalize,loud", [(True, False), (False, True)])
def test_normalize_rule(tmp_path, oracle_mod, normalize, loud):
    """ProcessFile.cp:92-101: rescale iff the file's peak > 1 or -n."""
    x = tone(2, 48000, 48000, amp=0.3)
    if loud:  # float source that clips after filtering -> forced normalize
        x = (x * np.float32(4.0)).astype(np.float32)
    fmt = "f32le" if loud else "s24le"
    src, dst = tmp_path / "n.wav", tmp_path / "n_out.wav"
    pcm_ref.write_wave(src, x, 48000, fmt)
    xq = pcm_ref.np_decode(pcm_ref.np_encode(x, fmt), fmt, 2)
    args = ["-n"] if normalize else []
    lowcut(*args, "-f", 20, "-s", 48, src, dst)
    check_file(oracle_mod, src, dst, xq, 48000, fmt, 20, 48, normalize)
    got = pcm_ref.np_decode(open(dst, "rb").read()[int(info(dst)["data_offset"]):], fmt, 2)
    assert np.abs(got).max() <= 1.0


def test_batch_scenario_and_overwrite(tmp_path, oracle_mod):
    """main.cp:112-147: several inputs into a new directory; -O overwrites."""
    srcs = []
    for i, rate in enumerate([44100, 48000, 96000]):
        x = tone(1 + i % 2, 30000, rate)
        p = tmp_path / f"f{i}.wav"
        pcm_ref.write_wave(p, x, rate, "s24le")
        srcs.append((p, pcm_ref.np_decode(pcm_ref.np_encode(x, "s24le"), "s24le", x.shape[0]), rate))
    outdir = tmp_path / "out"
    lowcut("-f", 30, "-s", 60, *[s for s, _, _ in srcs], outdir)
    for p, xq, rate in srcs:
        check_file(oracle_mod, p, outdir / p.name, xq, rate, "s24le", 30, 60, False)
    r = subprocess.run([LOWCUT, *map(str, ["-f", 30, "-s", 60, srcs[0][0], srcs[1][0], outdir])],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "exists" in r.stderr
    lowcut("-O", "-f", 30, "-s", 60, srcs[0][0], srcs[1][0], outdir)


def test_pipeline_mixed_batch(tmp_path, oracle_mod):
    """Six files through the read -> GPU (2 streams) -> write pipeline: mixed
    rates, channel counts, containers and an empty data chunk; each output
    must equal the one-file-at-a-time result."""
    specs = [(44100, 1, "s16le", "wav", 20000), (48000, 2, "s24be", "aif", 50000),
             (48000, 3, "f32le", "wav", 0), (96000, 2, "s24le", "wav", 70000),
             (48000, 1, "s32le", "wav", 12345), (44100, 2, "s16be", "aif", 33333)]
    srcs = []
    for i, (rate, nch, fmt, ext, n) in enumerate(specs):
        x = tone(nch, max(n, 1), rate)[:, :n]
        p = tmp_path / f"m{i}.{ext}"
        (pcm_ref.write_wave if ext == "wav" else pcm_ref.write_aiff)(p, x, rate, fmt)
        srcs.append((p, x, rate, fmt))
    outdir = tmp_path / "batch"
    out = lowcut("--timing", "-f", 25, "-s", 50, *[s[0] for s in srcs], outdir)
    assert out.count("Processing file:") == len(specs) and "timing total: 6 file(s)" in out
    for p, x, rate, fmt in srcs:
        if x.shape[1] == 0:
            assert open(outdir / p.name, "rb").read() == open(p, "rb").read()
            continue
        xq = pcm_ref.np_decode(pcm_ref.np_encode(x, fmt), fmt, x.shape[0])
        check_file(oracle_mod, p, outdir / p.name, xq, rate, fmt, 25, 50, False)
    # the same file alone gives the same bytes (no cross-file state in the slots)
    single = tmp_path / "single.wav"
    lowcut("-f", 25, "-s", 50, srcs[3][0], single)
    assert open(single, "rb").read() == open(outdir / srcs[3][0].name, "rb").read()


def test_pipeline_stops_at_first_failure(tmp_path):
    """main.cp:131-146 processes inputs in order and stops at the first error:
    files before it are written, files after it are not."""
    good = []
    for i in range(3):
        p = tmp_path / f"g{i}.wav"
        pcm_ref.write_wave(p, tone(1, 9000, 48000), 48000, "s16le")
        good.append(p)
    outdir = tmp_path / "o"
    args = ["-f", 20, "-s", 48, good[0], good[1], tmp_path / "missing.wav", good[2], outdir]
    r = subprocess.run([LOWCUT, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "not found" in r.stderr
    assert (outdir / "g0.wav").exists() and (outdir / "g1.wav").exists()
    assert not (outdir / "g2.wav").exists()


def test_pipeline_gpu_stage_failure_keeps_earlier_files(tmp_path, oracle_mod):
    """a failure inside the GPU stage (here the filter design for
    file 2: -f 5000 is above its 8 kHz rate's Nyquist frequency) stops the
    batch at that file, and the earlier file still in the stage's other slot
    (file 1, enqueued before file 2) is finished and written.  Files 0 and 1
    are written and correct, files 2 and 3 are not."""
    specs = [48000, 48000, 8000, 48000]
    srcs = []
    for i, rate in enumerate(specs):
        x = tone(1, 20000, rate)
        p = tmp_path / f"s{i}.wav"
        pcm_ref.write_wave(p, x, rate, "s24le")
        srcs.append((p, pcm_ref.np_decode(pcm_ref.np_encode(x, "s24le"), "s24le", 1), rate))
    outdir = tmp_path / "o"
    args = ["-f", 5000, "-s", 2000, *[p for p, _, _ in srcs], outdir]
    r = subprocess.run([LOWCUT, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "design" in r.stderr, r.stderr + r.stdout
    for p, xq, rate in srcs[:2]:
        check_file(oracle_mod, p, outdir / p.name, xq, rate, "s24le", 5000, 2000, False)
    assert not (outdir / "s2.wav").exists() and not (outdir / "s3.wav").exists()


def test_large_file(tmp_path):
    """A 42 MB WAVE: every non-payload byte kept, and the payload equal to the
    same decode -> filter -> encode through the Python binding of the C ABI."""
    import lcfir as lc
    rate, nch, n = 48000, 2, 7_000_003
    x = tone(nch, n, rate)
    src, dst = tmp_path / "big.wav", tmp_path / "big_out.wav"
    pcm_ref.write_wave(src, x, rate, "s24le", extra_chunks=[(b"LIST", b"INFOICMT\x04\x00\x00\x00big!")])
    assert os.path.getsize(src) > (40 << 20)
    lowcut("-f", 20, "-s", 48, src, dst)
    a, b = open(src, "rb").read(), open(dst, "rb").read()
    d = info(src)
    off, nbytes = int(d["data_offset"]), int(d["data_bytes"])
    assert len(a) == len(b) and a[:off] == b[:off] and a[off + nbytes:] == b[off + nbytes:]
    xq = np.ascontiguousarray(pcm_ref.np_decode(a[off:off + nbytes], "s24le", nch), np.float32)
    flt = lc.Filter(lc.design_lowcut(20.0, 48.0, float(rate)))
    dx = lc.DeviceBuffer.from_array(xq)
    dy = lc.DeviceBuffer(xq.nbytes)
    flt.filter_channels_dev(dx, n, nch, n, dy, n, None)
    lc.sync()
    y = dy.download((nch, n))
    assert np.abs(y).max() <= 1.0  # no normalize in this case
    assert pcm_ref.np_encode(y, "s24le") == b[off:off + nbytes]


def test_batch_duplicate_destination(tmp_path):
    """Two inputs with one file name (dirA/x.wav dirB/x.wav out/): the
    reference's sequential loop (main.cp:131-146) has written out/x.wav when it
    reaches the second, so without -O that is "File exists"; with -O the second
    file's result is the one left."""
    xs = []
    for d, seed in (("A", 1), ("B", 2)):
        (tmp_path / d).mkdir()
        x = tone(1, 9000 + seed, 48000)
        pcm_ref.write_wave(tmp_path / d / "x.wav", x, 48000, "s16le")
        xs.append(tmp_path / d / "x.wav")
    outdir = tmp_path / "out"
    args = ["-f", 20, "-s", 48, xs[0], xs[1], outdir]
    r = subprocess.run([LOWCUT, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "exists" in r.stderr
    assert (outdir / "x.wav").exists()
    first = open(outdir / "x.wav", "rb").read()
    lowcut("-O", *args)
    solo = tmp_path / "solo.wav"
    lowcut("-f", 20, "-s", 48, xs[1], solo)
    assert open(outdir / "x.wav", "rb").read() == open(solo, "rb").read() != first


def _random_file(rng, tmp_path, i):
    rate = int(rng.choice([22050, 44100, 48000, 96000]))
    nch = int(rng.integers(1, 7))
    n = int(rng.choice([1, 7, 100, 5000, 30001]))
    kind = str(rng.choice(["wav", "wavx", "aif", "aifc"]))
    if kind.startswith("wav"):
        fmt, comp = str(rng.choice(["s16le", "s24le", "s32le", "f32le"])), None
    elif kind == "aif":
        fmt, comp = str(rng.choice(["s16be", "s24be", "s32be"])), None
    else:
        fmt, comp = [("s16le", b"sowt"), ("f32be", b"fl32"), ("s24be", b"NONE")][int(rng.integers(3))]
    amp = float(rng.choice([0.3, 0.9]))
    x = tone(nch, n, rate, amp=amp)
    if fmt.startswith("f32") and rng.random() < 0.5:
        x = (x * np.float32(3.0)).astype(np.float32)  # float source above full scale: the >1 rule
    extra = [(b"LIST", b"INFOICMT" + bytes([int(rng.integers(1, 9))]) + b"\x00\x00\x00odd")] \
        if rng.random() < 0.5 else []
    p = tmp_path / f"r{i}.{'wav' if kind.startswith('wav') else 'aif'}"
    if kind.startswith("wav"):
        pcm_ref.write_wave(p, x, rate, fmt, extensible=kind == "wavx", extra_chunks=extra)
    else:
        pcm_ref.write_aiff(p, x, rate, fmt, aifc_comp=comp, extra_chunks=extra)
    return p, x, rate, fmt


@pytest.mark.parametrize("seed", range(int(os.environ.get("LCFIR_CLI_SEED0", "0")),
                                  int(os.environ.get("LCFIR_CLI_SEED0", "0"))
                                  + int(os.environ.get("LCFIR_CLI_SEEDS", "3"))))
def test_cli_random_batch(tmp_path, oracle_mod, seed):
    """Seeded batches of six random files through the tool's pipeline:
    WAVE / WAVE_FORMAT_EXTENSIBLE / AIFF / AIFF-C, 16/24/32-bit and float
    samples, 1-6 channels, 1 .. 30 001 frames (shorter than the filter
    included), four rates, odd-length extra chunks, random -f / -s / -n.
    Every output against the oracle's process_file (check_file); at most a
    couple of 1-LSB quantiser-boundary differences per file."""
    rng = np.random.default_rng(700 + seed)
    freq, slope = float(rng.uniform(10, 200)), float(rng.uniform(30, 200))
    normalize = bool(rng.random() < 0.5)
    srcs = [_random_file(rng, tmp_path, i) for i in range(6)]
    outdir = tmp_path / "out"
    lowcut(*(["-n"] if normalize else []), "-f", f"{freq:.3f}", "-s", f"{slope:.3f}",
           *[s[0] for s in srcs], outdir)
    for p, x, rate, fmt in srcs:
        a, b = open(p, "rb").read(), open(outdir / p.name, "rb").read()
        d = info(p)
        off, nbytes = int(d["data_offset"]), int(d["data_bytes"])
        assert len(a) == len(b) and a[:off] == b[:off] and a[off + nbytes:] == b[off + nbytes:], p.name
        nch = x.shape[0]
        xq = pcm_ref.np_decode(pcm_ref.np_encode(x, fmt), fmt, nch)
        got = pcm_ref.np_decode(b[off:off + nbytes], fmt, nch)
        want_f = expected(oracle_mod, xq, rate, fmt, float(f"{freq:.3f}"), float(f"{slope:.3f}"), normalize)
        if fmt.startswith("f32"):
            dd = got.astype(np.float64) - want_f
            assert np.sqrt(np.mean(dd * dd)) <= 1e-9, p.name
            assert np.abs(got).max() <= 1.0 or not normalize, p.name
        else:
            want = pcm_ref.np_decode(pcm_ref.np_encode(want_f, fmt), fmt, nch)
            lsb = 1.0 / (1 << (8 * pcm_ref.NB[fmt[:3]] - 1))
            diff = np.abs(got.astype(np.float64) - want.astype(np.float64))
            # one quantiser step, or (32-bit samples, finer than f32) one f32 ulp of the filter output
            tol = lsb * 1.000001 + np.spacing(np.abs(want_f).astype(np.float32)).astype(np.float64)
            assert np.all(diff <= tol), p.name
            assert np.sum(diff > 0) <= max(2, 1e-4 * diff.size), p.name


def test_batch_over_device_stages(tmp_path, oracle_mod):
    """--devices: a batch dealt round-robin over GPU stages (north_star: one
    file per GPU).  On the one-GPU box the stages share device 0 ("0,0,0":
    three stages, each with its own contexts, streams and slots): every output
    byte-identical to the single-stage run, written in input order, checked
    against the oracle; the same with files read by parallel reader threads
    (--readers); with a missing input in the middle (four readers) the files
    before it are written and the ones after it are not (main.cp:131-146)."""
    specs = [(48000, 2, "s24le", "wav", 60000), (44100, 1, "s16le", "wav", 20001),
             (96000, 2, "f32le", "wav", 40000), (48000, 1, "s24be", "aif", 33333),
             (48000, 3, "s32le", "wav", 25000), (44100, 2, "s16be", "aif", 12345),
             (48000, 2, "s24le", "wav", 50001)]
    srcs = []
    for i, (rate, nch, fmt, ext, n) in enumerate(specs):
        x = tone(nch, n, rate, amp=0.9 if i == 4 else 0.4)
        p = tmp_path / f"d{i}.{ext}"
        (pcm_ref.write_wave if ext == "wav" else pcm_ref.write_aiff)(p, x, rate, fmt)
        srcs.append((p, x, rate, fmt))
    one, three = tmp_path / "one", tmp_path / "three"
    lowcut("-n", "-f", 25, "-s", 50, "--devices", "0", *[s[0] for s in srcs], one)
    out = lowcut("-n", "-f", 25, "-s", 50, "--devices", "0,0,0", "--timing", *[s[0] for s in srcs], three)
    names = [line.split(": ", 1)[1] for line in out.splitlines() if line.startswith("Processing file:")]
    assert names == [s[0].name for s in srcs]
    assert "3 GPU stage(s)" in out
    # files read by three threads in parallel: same bytes, same order
    par = tmp_path / "par"
    out = lowcut("-n", "-f", 25, "-s", 50, "--devices", "0,0", "--readers", "3", "--timing",
                 *[s[0] for s in srcs], par)
    names = [line.split(": ", 1)[1] for line in out.splitlines() if line.startswith("Processing file:")]
    assert names == [s[0].name for s in srcs]
    assert "3 reader(s)" in out
    for p, x, rate, fmt in srcs:
        assert open(one / p.name, "rb").read() == open(three / p.name, "rb").read(), p.name
        assert open(one / p.name, "rb").read() == open(par / p.name, "rb").read(), p.name
        xq = pcm_ref.np_decode(pcm_ref.np_encode(x, fmt), fmt, x.shape[0])
        check_file(oracle_mod, p, three / p.name, xq, rate, fmt, 25, 50, True)
    stop = tmp_path / "stop"
    args = ["-f", 20, "-s", 48, "--devices", "0,0", "--readers", "4", *[s[0] for s in srcs[:3]],
            tmp_path / "missing.wav", *[s[0] for s in srcs[3:]], stop]
    r = subprocess.run([LOWCUT, *map(str, args)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 1 and "not found" in r.stderr
    assert all((stop / s[0].name).exists() for s in srcs[:3])
    assert not any((stop / s[0].name).exists() for s in srcs[3:])

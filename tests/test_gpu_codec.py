"""GPU tests of the on-device sample codec (lcfir_decode_pcm_dev /
lcfir_encode_pcm_dev) against a numpy restatement of the same conventions.
Byte-exact: decode of every format, encode round trips, clamping and
round-half-even at the quantiser's ties."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FORMATS = ["s16le", "s24le", "s32le", "f32le", "s16be", "s24be", "s32be", "f32be"]


def np_decode(raw: bytes, fmt: str, nch: int) -> np.ndarray:
    nb = {"s16": 2, "s24": 3, "s32": 4, "f32": 4}[fmt[:3]]
    be = fmt.endswith("be")
    b = np.frombuffer(raw, np.uint8).reshape(-1, nb).astype(np.uint32)
    if be:
        b = b[:, ::-1]
    v = np.zeros(b.shape[0], np.uint32)
    for i in range(nb):
        v |= b[:, i] << np.uint32(8 * i)
    if fmt.startswith("f32"):
        out = v.view(np.float32)
    else:
        bits = 8 * nb
        s = (v.astype(np.int64) << (64 - bits)).astype(np.int64) >> (64 - bits)
        out = (s.astype(np.float64) / float(1 << (bits - 1))).astype(np.float32)
    return np.ascontiguousarray(out.reshape(-1, nch).T)


def np_encode(x: np.ndarray, fmt: str) -> bytes:
    nb = {"s16": 2, "s24": 3, "s32": 4, "f32": 4}[fmt[:3]]
    be = fmt.endswith("be")
    inter = np.ascontiguousarray(x.T).reshape(-1)
    if fmt.startswith("f32"):
        v = inter.astype(np.float32).view(np.uint32)
    else:
        scale = float(1 << (8 * nb - 1))
        q = np.rint(inter.astype(np.float64) * scale)
        q = np.nan_to_num(np.clip(q, -scale, scale - 1), nan=0.0)
        v = q.astype(np.int64).astype(np.uint32)
    b = np.stack([(v >> np.uint32(8 * i)) & np.uint32(0xFF) for i in range(nb)], 1).astype(np.uint8)
    if be:
        b = b[:, ::-1]
    return b.tobytes()


@pytest.fixture(scope="module")
def lc():
    import lcfir
    assert lcfir.device_count() >= 1
    return lcfir


@pytest.mark.parametrize("fmt", FORMATS)
@pytest.mark.parametrize("nch,frames", [(1, 1), (2, 100003), (8, 4099)])
def test_decode_matches_numpy(lc, fmt, nch, frames):
    rng = np.random.default_rng(hash((fmt, nch, frames)) & 0xFFFF)
    nb = lc.pcm_bytes(fmt)
    raw = rng.integers(0, 256, nb * nch * frames, dtype=np.uint8)
    if fmt.startswith("f32"):  # avoid NaN payload comparisons
        f = rng.uniform(-2, 2, nch * frames).astype(np.float32)
        raw = np.frombuffer(np_encode(f.reshape(frames, nch).T, fmt), np.uint8).copy()
    d_in = lc.DeviceBuffer.from_array(raw)
    stride = frames + 5
    d_out = lc.DeviceBuffer(4 * nch * stride)
    lc.decode_pcm_dev(d_in, fmt, nch, frames, d_out, stride)
    lc.sync()
    got = d_out.download((nch, stride))[:, :frames]
    want = np_decode(raw.tobytes(), fmt, nch)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("fmt", FORMATS)
def test_encode_roundtrip_and_clamp(lc, fmt):
    rng = np.random.default_rng(7)
    nch, frames = 3, 50001
    nb = lc.pcm_bytes(fmt)
    x = rng.uniform(-1.3, 1.3, (nch, frames)).astype(np.float32)
    if not fmt.startswith("f32"):
        bits = 8 * nb
        # exact quantiser ties (k + 0.5) / 2^(bits-1), representable in f32 for bits <= 16
        if bits <= 16:
            k = rng.integers(-1000, 1000, frames)
            x[0] = ((k + 0.5) / float(1 << (bits - 1))).astype(np.float32)
        x[1, :4] = [np.nan, np.inf, -np.inf, 0.0]
    d_x = lc.DeviceBuffer.from_array(x)
    d_b = lc.DeviceBuffer(nb * nch * frames)
    lc.encode_pcm_dev(d_x, frames, nch, frames, fmt, d_b)
    lc.sync()
    got = d_b.download(nb * nch * frames, np.uint8).tobytes()
    assert got == np_encode(x, fmt)
    # decode(encode(x)) is the quantised signal; encode(decode(bytes)) == bytes
    d_y = lc.DeviceBuffer(4 * nch * frames)
    lc.decode_pcm_dev(d_b, fmt, nch, frames, d_y, frames)
    d_b2 = lc.DeviceBuffer(nb * nch * frames)
    lc.encode_pcm_dev(d_y, frames, nch, frames, fmt, d_b2)
    lc.sync()
    assert d_b2.download(nb * nch * frames, np.uint8).tobytes() == got


def test_codec_rejects_bad_format(lc):
    d = lc.DeviceBuffer(64)
    assert lc.load().lcfir_decode_pcm_dev(d.ptr, 99, 1, 4, d.ptr, 4, None) == lc.EINVAL
    assert lc.load().lcfir_encode_pcm_dev(d.ptr, 4, 1, 4, 0, d.ptr, None) == lc.EINVAL
    assert lc.pcm_bytes("s24le") == 3 and lc.load().lcfir_pcm_bytes(0) == 0


@pytest.mark.parametrize("fmt", ["s16le", "s24le", "s24be", "f32le"])
@pytest.mark.parametrize("peak,force", [(0.5, False), (0.5, True), (1.7, False), (0.0, True)])
def test_encode_scaled_equals_normalize_then_encode(lc, fmt, peak, force):
    """lcfir_encode_pcm_scaled_dev (the lowcut tool's fused pass) is byte-identical
    to lcfir_normalize_dev followed by lcfir_encode_pcm_dev (ProcessFile.cp:91-101,
    :115-117), leaves its input unscaled, and takes the decision from the device."""
    rng = np.random.default_rng(11)
    nch, frames = 2, 40003
    nb = lc.pcm_bytes(fmt)
    x = (rng.uniform(-1.0, 1.0, (nch, frames)) * max(peak, 1e-3)).astype(np.float32)
    pk = np.array([peak * 0.75, peak], np.float32)  # per-channel slots, max = peak
    d_pk = lc.DeviceBuffer.from_array(pk)
    d_x = lc.DeviceBuffer.from_array(x)
    d_fused = lc.DeviceBuffer(nb * nch * frames)
    lc.encode_pcm_scaled_dev(d_x, frames, nch, frames, fmt, d_pk, nch, force, d_fused)
    d_y = lc.DeviceBuffer.from_array(x)
    lc.normalize_dev(d_y, frames, nch, frames, d_pk, nch, force)
    d_ref = lc.DeviceBuffer(nb * nch * frames)
    lc.encode_pcm_dev(d_y, frames, nch, frames, fmt, d_ref)
    lc.sync()
    assert d_fused.download(nb * nch * frames, np.uint8).tobytes() == \
        d_ref.download(nb * nch * frames, np.uint8).tobytes()
    assert np.array_equal(d_x.download((nch, frames)), x)

"""numpy restatement of the PCM codec conventions and WAVE/AIFF writers
(test infrastructure: generates inputs and expected outputs for the codec and
the lowcut tool)."""
import struct

import numpy as np

NB = {"s16": 2, "s24": 3, "s32": 4, "f32": 4}


def np_decode(raw: bytes, fmt: str, nch: int) -> np.ndarray:
    nb = NB[fmt[:3]]
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
    nb = NB[fmt[:3]]
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


def _chunk(cid: bytes, body: bytes, be=False) -> bytes:
    hdr = cid + struct.pack(">I" if be else "<I", len(body))
    return hdr + body + (b"\0" if len(body) & 1 else b"")


def write_wave(path, x: np.ndarray, rate: int, fmt: str, extensible=False, extra_chunks=()):
    """x: [nch][frames] float32 in [-1, 1); fmt s16le/s24le/s32le/f32le."""
    nch = x.shape[0]
    nb = NB[fmt[:3]]
    tag = 3 if fmt.startswith("f32") else 1
    body = struct.pack("<HHIIHH", 0xFFFE if extensible else tag, nch, rate, rate * nch * nb,
                       nch * nb, 8 * nb)
    if extensible:
        guid = struct.pack("<H", tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
        body += struct.pack("<HHI", 22, 8 * nb, 0) + guid
    data = np_encode(x, fmt)
    chunks = _chunk(b"fmt ", body) + b"".join(_chunk(c, d) for c, d in extra_chunks) + \
        _chunk(b"data", data)
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 4 + len(chunks)) + b"WAVE" + chunks)
    return data


def _extended(v: float) -> bytes:
    import math
    if v == 0:
        return b"\0" * 10
    m, e = math.frexp(v)  # v = m * 2^e, 0.5 <= m < 1
    e += 16382
    mant = int(m * (1 << 64))
    return struct.pack(">HQ", e, mant)


def write_aiff(path, x: np.ndarray, rate: int, fmt: str, aifc_comp=None, extra_chunks=()):
    """AIFF (big-endian PCM) or AIFF-C with compression NONE/sowt/fl32."""
    nch, frames = x.shape
    nb = NB[fmt[:3]]
    comm = struct.pack(">hIh", nch, frames, 8 * nb) + _extended(float(rate))
    if aifc_comp is not None:
        comm += aifc_comp + b"\x00\x00"  # empty pascal string, padded
    data = np_encode(x, fmt)
    ssnd = struct.pack(">II", 0, 0) + data
    chunks = (_chunk(b"FVER", struct.pack(">I", 0xA2805140), True) if aifc_comp else b"") + \
        _chunk(b"COMM", comm, True) + b"".join(_chunk(c, d, True) for c, d in extra_chunks) + \
        _chunk(b"SSND", ssnd, True)
    kind = b"AIFC" if aifc_comp is not None else b"AIFF"
    with open(path, "wb") as f:
        f.write(b"FORM" + struct.pack(">I", 4 + len(chunks)) + kind + chunks)
    return data

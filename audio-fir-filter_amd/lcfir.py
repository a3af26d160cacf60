"""ctypes binding of the C ABI in include/lcfir.h (liblcfir.so).

The product is the C ABI and its HIP kernels; this module is the thin
Python-side binding used by bench.py, the tests and smoke().  It never
computes a filtered sample itself and has no CPU fallback: if liblcfir.so is
missing, or the device cannot run it, every call raises LcfirError.

Reference interface mirrored (diskerror/audio-fir-filter):
  Filter(...)                  ~ WindowedSinc<float64_t> as seen by the hot path
                                 (ProcessFile.cp:47-50, FilterCore.h:29 getMo2)
  apply_filter_range(...)      ~ FilterCore.h:20-79, same argument meaning
  filter_channel(...)          ~ the per-channel chunk hand-off, ProcessFile.cp:57-87
"""
from __future__ import annotations

import ctypes
import os
import re
import threading
from typing import Callable, Optional

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
REPO_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(_HERE, "liblcfir.so")
HEADER_PATH = os.path.join(REPO_ROOT, "include", "lcfir.h")

METHOD_AUTO, METHOD_DIRECT, METHOD_FFT = 0, 1, 2
METHODS = {"auto": METHOD_AUTO, "direct": METHOD_DIRECT, "fft": METHOD_FFT}

OK, EINVAL, EDEVICE, ENOMEM, EINTERNAL = 0, 1, 2, 3, 4


class LcfirError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"lcfir error {code}: {msg}")
        self.code = code


PROGRESS_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint64)

STAGING_BOUNCE, STAGING_PAGEABLE, STAGING_AUTO = 0, 1, 2
# lcfir_ctx_fft_units' kernel codes (LCFIR_FFT_KERNEL_*)
FFT_KERNELS = {0: None, 1: "l16", 2: "l32_park", 3: "l32_reg"}
FFT_FAMILIES = {"default": 0, "lds": 1}


class RangeStats(ctypes.Structure):
    """lcfir_range_stats (include/lcfir.h): accounting of lcfir_apply_range."""
    _fields_ = [("calls", ctypes.c_uint64), ("samples", ctypes.c_uint64), ("h2d_bytes", ctypes.c_uint64),
                ("d2h_bytes", ctypes.c_uint64), ("staged_calls", ctypes.c_uint64),
                ("profiled_calls", ctypes.c_uint64), ("wall_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double),
                ("kernel_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}

_c_int, _c_i32, _c_i64 = ctypes.c_int, ctypes.c_int32, ctypes.c_int64
_vp, _fp, _dp = ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_double)
_ctxp = ctypes.c_void_p

_SIGNATURES = {
    "lcfir_abi_version": ([], _c_int),
    "lcfir_last_error": ([], ctypes.c_char_p),
    "lcfir_build_id": ([], ctypes.c_char_p),
    "lcfir_device_count": ([ctypes.POINTER(_c_int)], _c_int),
    "lcfir_ctx_create": ([_c_int, _dp, _c_i32, ctypes.POINTER(_ctxp)], _c_int),
    "lcfir_ctx_destroy": ([_ctxp], _c_int),
    "lcfir_ctx_set_method": ([_ctxp, _c_int], _c_int),
    "lcfir_ctx_get_method": ([_ctxp, ctypes.POINTER(_c_int)], _c_int),
    "lcfir_ctx_half": ([_ctxp, ctypes.POINTER(_c_i32)], _c_int),
    "lcfir_ctx_fft_info": ([_ctxp, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32)],
                           _c_int),
    "lcfir_ctx_fft_units": ([_ctxp, ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32), ctypes.POINTER(_c_i32)],
                            _c_int),
    "lcfir_ctx_nrm_stats": ([_ctxp, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)], _c_int),
    "lcfir_ctx_set_fft_tuning": ([_ctxp, _c_i32, _c_i32, _c_i64, _c_i64], _c_int),
    "lcfir_ctx_set_fft_family": ([_ctxp, _c_int], _c_int),
    "lcfir_ctx_ntaps": ([_ctxp, ctypes.POINTER(_c_i32)], _c_int),
    "lcfir_ctx_window": ([_ctxp, _c_i64, _c_i64, _c_i64, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i64)], _c_int),
    "lcfir_apply_range": ([_ctxp, _vp, _c_i64, _vp, _c_i64, _c_i64, PROGRESS_FN, _vp], _c_int),
    "lcfir_staging_release": ([_c_int], _c_int),
    "lcfir_staging_count": ([_c_int, ctypes.POINTER(_c_int), ctypes.POINTER(_c_int)], _c_int),
    "lcfir_staging_set_mode": ([_c_int], _c_int),
    "lcfir_range_profile": ([_c_int], _c_int),
    "lcfir_range_stats_get": ([_vp, _c_int], _c_int),
    "lcfir_apply_range_dev": ([_ctxp, _vp, _c_i64, _vp, _c_i64, _c_i64, _vp], _c_int),
    "lcfir_filter_channels_dev": (
        [_ctxp, _vp, _c_i64, _c_i32, _c_i64, _vp, _c_i64, _vp, _vp], _c_int),
    "lcfir_filter_window_dev": (
        [_ctxp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i32, _vp, _c_i64, _c_i64, _c_i64, _c_i64,
         _vp, _c_i64, _vp], _c_int),
    "lcfir_filter_window_norm_dev": (
        [_ctxp, _vp, _c_i64, _c_i64, _c_i64, _c_i64, _c_i32, _vp, _c_i64, _c_i64, _c_i64, _c_i64,
         _vp, _c_i64, _vp, _c_i64, _vp, _c_i32, _c_int, _vp], _c_int),
    "lcfir_peak_reset_dev": ([_vp, _c_i32, _vp], _c_int),
    "lcfir_peak_dev": ([_vp, _c_i64, _c_i32, _c_i64, _vp, _vp], _c_int),
    "lcfir_normalize_dev": ([_vp, _c_i64, _c_i32, _c_i64, _vp, _c_i32, _c_int, _vp], _c_int),
    "lcfir_normalize_clear_dev": (
        [_vp, _c_i64, _c_i32, _c_i64, _vp, _c_i32, _c_int, _vp, _c_i32, _vp], _c_int),
    "lcfir_channel_peak": ([_c_int, _vp, _c_i64, ctypes.POINTER(ctypes.c_float)], _c_int),
    "lcfir_design_lowcut": ([ctypes.c_double, ctypes.c_double, ctypes.c_double, _vp, _c_i32,
                             ctypes.POINTER(_c_i32)], _c_int),
    "lcfir_pcm_bytes": ([_c_int], _c_int),
    "lcfir_decode_pcm_dev": ([_vp, _c_int, _c_i32, _c_i64, _vp, _c_i64, _vp], _c_int),
    "lcfir_encode_pcm_dev": ([_vp, _c_i64, _c_i32, _c_i64, _c_int, _vp, _vp], _c_int),
    "lcfir_encode_pcm_scaled_dev": ([_vp, _c_i64, _c_i32, _c_i64, _c_int, _vp, _c_i32, _c_int, _vp, _vp],
                                    _c_int),
    "lcfir_dev_malloc": ([_c_int, ctypes.c_size_t, ctypes.POINTER(_vp)], _c_int),
    "lcfir_dev_free": ([_vp], _c_int),
    "lcfir_memcpy_h2d": ([_vp, _vp, ctypes.c_size_t, _vp], _c_int),
    "lcfir_memcpy_d2h": ([_vp, _vp, ctypes.c_size_t, _vp], _c_int),
    "lcfir_memcpy_d2h_async": ([_vp, _vp, ctypes.c_size_t, _vp], _c_int),
    "lcfir_host_malloc": ([ctypes.c_size_t, ctypes.POINTER(_vp)], _c_int),
    "lcfir_host_free": ([_vp], _c_int),
    "lcfir_stream_create": ([_c_int, ctypes.POINTER(_vp)], _c_int),
    "lcfir_stream_destroy": ([_vp], _c_int),
    "lcfir_stream_sync": ([_vp], _c_int),
}

_lib = None
_lib_lock = threading.Lock()


def header_symbols(path: str = HEADER_PATH) -> list:
    """Every function the C header declares (used by the export test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(lcfir_\w+)\s*\(", text, re.M)))


def load(path: str = LIB_PATH):
    """Load liblcfir.so.  Raises LcfirError if it has not been built."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise LcfirError(EINTERNAL, f"{path} is missing: build it with "
                             "`python -c 'import __graft_entry__ as g; g.build()'`")
        # torch first (when installed): its libamdhip64.so.7 then serves both,
        # so device pointers from torch and from this library share one HIP
        # runtime whatever order the caller imports them in (hip_runtimes()).
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        lib = ctypes.CDLL(path)
        for name, (argtypes, restype) in _SIGNATURES.items():
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = restype
        if lib.lcfir_abi_version() != 1:
            raise LcfirError(EINTERNAL, "ABI version mismatch")
        _lib = lib
        return lib


def _check(rc: int):
    if rc != OK:
        msg = _lib.lcfir_last_error()
        raise LcfirError(rc, msg.decode() if msg else "")


def device_count() -> int:
    lib = load()
    c = ctypes.c_int(0)
    _check(lib.lcfir_device_count(ctypes.byref(c)))
    return c.value


def build_id() -> str:
    """lcfir_build_id: the loaded library's source hash (src_hash.sh)."""
    return load().lcfir_build_id().decode()


def _ptr(a) -> int:
    """Raw address of a numpy array or a torch tensor."""
    if isinstance(a, np.ndarray):
        return a.ctypes.data
    if hasattr(a, "data_ptr"):
        return a.data_ptr()
    if isinstance(a, int):
        return a
    raise TypeError(f"cannot take the address of {type(a)}")


class Filter:
    """One filter (tap set) resident on one device.

    Mirrors the reference's `WindowedSinc<float64_t>` as used by the hot path:
    it holds the M+1 taps and answers getMo2() (`half`).
    """

    def __init__(self, taps, device: int = 0, method: str = "auto"):
        lib = load()
        t = np.ascontiguousarray(np.asarray(taps, dtype=np.float64))
        self._taps = t
        self.device = device
        ctx = ctypes.c_void_p()
        _check(lib.lcfir_ctx_create(device, t.ctypes.data_as(_dp), int(t.size), ctypes.byref(ctx)))
        self._ctx = ctx
        try:
            self.set_method(method)
        except Exception:
            self.close()
            raise

    @property
    def ctx(self):
        return self._ctx

    def set_method(self, method: str):
        _check(load().lcfir_ctx_set_method(self._ctx, METHODS[method]))

    @property
    def method(self) -> str:
        m = ctypes.c_int()
        _check(load().lcfir_ctx_get_method(self._ctx, ctypes.byref(m)))
        return {v: k for k, v in METHODS.items()}[m.value]

    @property
    def half(self) -> int:
        h = ctypes.c_int32()
        _check(load().lcfir_ctx_half(self._ctx, ctypes.byref(h)))
        return h.value

    getMo2 = half

    @property
    def fft_info(self) -> dict:
        """The FFT plan this filter runs (lcfir_ctx_fft_info): segment length,
        tap partitions, zero-phase form (all 0 outside the FFT's range)."""
        L, P, Z = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _check(load().lcfir_ctx_fft_info(self._ctx, ctypes.byref(L), ctypes.byref(P), ctypes.byref(Z)))
        return {"seg_len": L.value, "parts": P.value, "zero_phase": bool(Z.value)}

    @property
    def fft_units(self) -> dict:
        """The plan's unit geometry (lcfir_ctx_fft_units): outputs per segment
        B, the kernel that runs a unit ("l16", "l32_park", "l32_reg"), and the
        most floats of a previous file's normalize one unit carries inside the
        filter launch (0: never fused)."""
        b, k, f = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_int32()
        _check(load().lcfir_ctx_fft_units(self._ctx, ctypes.byref(b), ctypes.byref(k), ctypes.byref(f)))
        return {"outputs": b.value, "kernel": FFT_KERNELS.get(k.value), "nrm_floats": f.value}

    @property
    def nrm_stats(self) -> dict:
        """lcfir_ctx_nrm_stats: previous-file normalizes carried inside the
        filter launch ("fused") and run as their own pass ("separate")."""
        f, sep = ctypes.c_int64(), ctypes.c_int64()
        _check(load().lcfir_ctx_nrm_stats(self._ctx, ctypes.byref(f), ctypes.byref(sep)))
        return {"fused": f.value, "separate": sep.value}

    def set_fft_tuning(self, seg_len: int = 0, zero_phase: bool = True, chunk: int = 0, max_units: int = 0):
        """lcfir_ctx_set_fft_tuning: explicit FFT-method choices (tests run
        every setting; the defaults are the product's)."""
        _check(load().lcfir_ctx_set_fft_tuning(self._ctx, int(seg_len), 1 if zero_phase else 0, int(chunk),
                                               int(max_units)))

    def set_fft_family(self, family: str = "default"):
        """lcfir_ctx_set_fft_family for zero-phase single-partition plans:
        "default" (fir_fft32r at L = 32 768, the LDS-column kernel at 16 384)
        or "lds" (the LDS-column kernels everywhere)."""
        _check(load().lcfir_ctx_set_fft_family(self._ctx, FFT_FAMILIES[family]))

    @property
    def ntaps(self) -> int:
        n = ctypes.c_int32()
        _check(load().lcfir_ctx_ntaps(self._ctx, ctypes.byref(n)))
        return n.value

    def window(self, n: int, start: int, end: int):
        """Input window (lo, hi) within [0, n) for which filter_window_dev's
        outputs [start, end) equal the whole-channel call's bit for bit
        (lcfir_ctx_window; the FFT method reads whole segments)."""
        lo, hi = ctypes.c_int64(), ctypes.c_int64()
        _check(load().lcfir_ctx_window(self._ctx, n, start, end, ctypes.byref(lo), ctypes.byref(hi)))
        return lo.value, hi.value

    @property
    def taps(self) -> np.ndarray:
        return self._taps

    def close(self):
        if self._ctx:
            load().lcfir_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- host-pointer hot path (FilterCore.h:20-79) ------------------------
    def apply_range(self, channel: np.ndarray, temp_output: np.ndarray, start: int, end: int,
                    progress: Optional[Callable[[int], None]] = None):
        if channel.dtype != np.float32 or temp_output.dtype != np.float32:
            raise TypeError("channel and temp_output must be float32")
        if not (channel.flags.c_contiguous and temp_output.flags.c_contiguous):
            raise ValueError("arrays must be contiguous")
        if temp_output.size < channel.size:
            raise ValueError("temp_output shorter than channel")
        cb = PROGRESS_FN(0) if progress is None else PROGRESS_FN(lambda _u, c: progress(int(c)))
        _check(load().lcfir_apply_range(self._ctx, channel.ctypes.data, channel.size,
                                        temp_output.ctypes.data, int(start), int(end), cb, None))

    # -- device-pointer variants ---------------------------------------------
    def apply_range_dev(self, d_x, n: int, d_y, start: int, end: int, stream=0):
        _check(load().lcfir_apply_range_dev(self._ctx, _ptr(d_x), n, _ptr(d_y), start, end,
                                            stream or None))

    def filter_channels_dev(self, d_x, x_stride: int, nch: int, n: int, d_y, y_stride: int,
                            d_peak=None, stream=0):
        _check(load().lcfir_filter_channels_dev(
            self._ctx, _ptr(d_x), x_stride, nch, n, _ptr(d_y), y_stride,
            _ptr(d_peak) if d_peak is not None else None, stream or None))


def _filter_window_dev(self, d_xw, x_lo: int, x_hi: int, x_stride: int, n: int, nch: int,
                       d_yw, y_lo: int, y_stride: int, start: int, end: int, d_peak=None,
                       stream=0, peak_stride: int = 1):
    """lcfir_filter_window_dev: outputs [start, end) of channels of length n
    from the sample window [x_lo, x_hi) (a file sharded by sample range)."""
    _check(load().lcfir_filter_window_dev(
        self._ctx, _ptr(d_xw), x_lo, x_hi, x_stride, n, nch, _ptr(d_yw), y_lo, y_stride,
        start, end, _ptr(d_peak) if d_peak is not None else None, peak_stride, stream or None))


def _filter_window_norm_dev(self, d_xw, x_lo: int, x_hi: int, x_stride: int, n: int, nch: int,
                            d_yw, y_lo: int, y_stride: int, start: int, end: int, d_peak,
                            peak_stride: int, d_ny, ncount: int, d_npeak, nnpeak: int, force: bool,
                            stream=0):
    """lcfir_filter_window_norm_dev: filter_window_dev plus a previous file's
    normalize of the ncount contiguous floats at d_ny (fused into the FFT
    launch where possible; bit-identical to normalize_dev either way)."""
    _check(load().lcfir_filter_window_norm_dev(
        self._ctx, _ptr(d_xw), x_lo, x_hi, x_stride, n, nch, _ptr(d_yw), y_lo, y_stride,
        start, end, _ptr(d_peak) if d_peak is not None else None, peak_stride, _ptr(d_ny), ncount,
        _ptr(d_npeak), nnpeak, 1 if force else 0, stream or None))


Filter.filter_window_dev = _filter_window_dev
Filter.filter_window_norm_dev = _filter_window_norm_dev


class ThreadSafeProgress:
    """Counterpart of the reference's ThreadSafeProgress (ProgressBar.h:57-82):
    an atomic counter fed by report(count) from several threads."""

    def __init__(self, total: int):
        self.total = total
        self.count = 0
        self._lock = threading.Lock()

    def report(self, count: int):
        with self._lock:
            self.count += count


def apply_filter_range(channel: np.ndarray, sinc: Filter, temp_output: np.ndarray,
                       startIdx: int, endIdx: int, progress: Optional[ThreadSafeProgress] = None):
    """Reference-signature mirror of apply_filter_range (FilterCore.h:20-27)."""
    sinc.apply_range(channel, temp_output, startIdx, endIdx,
                     None if progress is None else progress.report)


def filter_channel(channel: np.ndarray, sinc: Filter, num_threads: int,
                   progress: Optional[ThreadSafeProgress] = None) -> np.ndarray:
    """The per-channel chunk hand-off of ProcessFile.cp:57-87: chunk =
    N / num_threads, the last thread takes the remainder, every thread calls
    apply_filter_range on its disjoint range, then join."""
    n = channel.size
    out = np.zeros(n, dtype=np.float32)
    num_threads = max(1, int(num_threads))
    chunk = n // num_threads
    errors = []

    def run(s, e):
        try:
            apply_filter_range(channel, sinc, out, s, e, progress)
        except Exception as ex:  # surfaced after join
            errors.append(ex)

    threads = []
    for i in range(num_threads):
        s = i * chunk
        e = n if i == num_threads - 1 else s + chunk
        t = threading.Thread(target=run, args=(s, e))
        t.start()
        threads.append(t)
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return out


def staging_release(device: int = -1):
    """Free the idle staging slots of lcfir_apply_range (-1: every device)."""
    _check(load().lcfir_staging_release(device))


def staging_set_mode(mode: str):
    """lcfir_staging_set_mode: 'auto' (default: a fan-out's 2-32 MiB windows
    through the slot's page-locked buffers, the runtime's path otherwise),
    'pageable' (the runtime stages the caller's memory) or 'bounce' (the
    slot's page-locked buffers for every call)."""
    _check(load().lcfir_staging_set_mode({"bounce": STAGING_BOUNCE, "pageable": STAGING_PAGEABLE,
                                          "auto": STAGING_AUTO}[mode]))


def range_profile(enable: bool):
    _check(load().lcfir_range_profile(1 if enable else 0))


def range_stats(reset: bool = False) -> dict:
    st = RangeStats()
    _check(load().lcfir_range_stats_get(ctypes.byref(st), 1 if reset else 0))
    return st.as_dict()


def staging_count(device: int = 0):
    """(slots in existence, idle slots) of the lcfir_apply_range pool."""
    live, idle = ctypes.c_int(0), ctypes.c_int(0)
    _check(load().lcfir_staging_count(device, ctypes.byref(live), ctypes.byref(idle)))
    return live.value, idle.value


# -- device post-pass helpers (ProcessFile.cp:91-101) ---------------------------
def peak_reset_dev(d_peak, count: int, stream=0):
    _check(load().lcfir_peak_reset_dev(_ptr(d_peak), count, stream or None))


def peak_dev(d_y, stride: int, nch: int, n: int, d_peak, stream=0):
    _check(load().lcfir_peak_dev(_ptr(d_y), stride, nch, n, _ptr(d_peak), stream or None))


def normalize_dev(d_y, stride: int, nch: int, n: int, d_peak, npeak: int, force: bool, stream=0):
    _check(load().lcfir_normalize_dev(_ptr(d_y), stride, nch, n, _ptr(d_peak), npeak,
                                      1 if force else 0, stream or None))


def normalize_clear_dev(d_y, stride: int, nch: int, n: int, d_peak, npeak: int, force: bool,
                        d_clear, nclear: int, stream=0):
    """normalize_dev that also zeroes d_clear[0:nclear] in the same launch."""
    _check(load().lcfir_normalize_clear_dev(_ptr(d_y), stride, nch, n, _ptr(d_peak), npeak,
                                            1 if force else 0, _ptr(d_clear) if nclear else None,
                                            nclear, stream or None))


def channel_peak(y: np.ndarray, device: int = 0) -> float:
    p = ctypes.c_float()
    y = np.ascontiguousarray(y, dtype=np.float32)
    _check(load().lcfir_channel_peak(device, y.ctypes.data, y.size, ctypes.byref(p)))
    return p.value


# -- device memory through the C ABI (no torch needed) -------------------------
class DeviceBuffer:
    """A device allocation made through lcfir_dev_malloc (HBM of `device`)."""

    def __init__(self, nbytes: int, device: int = 0):
        p = ctypes.c_void_p()
        _check(load().lcfir_dev_malloc(device, int(nbytes), ctypes.byref(p)))
        self.ptr = p.value
        self.nbytes = int(nbytes)
        self.device = device

    @classmethod
    def from_array(cls, a: np.ndarray, device: int = 0) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes, device)
        b.upload(a)
        return b

    def upload(self, a: np.ndarray, stream=0):
        a = np.ascontiguousarray(a)
        assert a.nbytes <= self.nbytes
        _check(load().lcfir_memcpy_h2d(self.ptr, a.ctypes.data, a.nbytes, stream or None))
        if not stream:
            sync()

    def download(self, shape, dtype=np.float32, stream=0) -> np.ndarray:
        out = np.empty(shape, dtype=dtype)
        assert out.nbytes <= self.nbytes
        _check(load().lcfir_memcpy_d2h(out.ctypes.data, self.ptr, out.nbytes, stream or None))
        return out

    def data_ptr(self) -> int:
        return self.ptr

    def free(self):
        if self.ptr:
            load().lcfir_dev_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def sync(stream=0):
    """Wait for `stream` (0 = the legacy default stream)."""
    _check(load().lcfir_stream_sync(stream or None))


def hip_runtimes() -> list:
    """Paths of every libamdhip64 mapped into this process.  Device pointers
    from torch are only valid here if this is a single runtime (import torch
    before lcfir so the SONAME libamdhip64.so.7 resolves to torch's copy)."""
    paths = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                if "libamdhip64" in line:
                    paths.add(os.path.realpath(line.split()[-1]))
    except OSError:
        pass
    return sorted(paths)


# -- tap design (ProcessFile.cp:47-50) ------------------------------------------
def design_lowcut(freq_hz: float, slope_hz: float, fs: float) -> np.ndarray:
    """Low-cut taps as the reference builds them per file (host, long double)."""
    lib = load()
    n = ctypes.c_int32()
    _check(lib.lcfir_design_lowcut(freq_hz, slope_hz, fs, None, 0, ctypes.byref(n)))
    taps = np.zeros(n.value, np.float64)
    _check(lib.lcfir_design_lowcut(freq_hz, slope_hz, fs, taps.ctypes.data, n.value,
                                   ctypes.byref(n)))
    return taps


# -- sample codec (interleaved PCM <-> planar float32) --------------------------
PCM_FORMATS = {"s16le": 1, "s24le": 2, "s32le": 3, "f32le": 4,
               "s16be": 5, "s24be": 6, "s32be": 7, "f32be": 8}


def pcm_bytes(fmt: str) -> int:
    return load().lcfir_pcm_bytes(PCM_FORMATS[fmt])


def decode_pcm_dev(d_in, fmt: str, nch: int, frames: int, d_out, out_stride: int, stream=0):
    """Interleaved PCM bytes (device) -> planar float32 [nch][out_stride] (device)."""
    _check(load().lcfir_decode_pcm_dev(_ptr(d_in), PCM_FORMATS[fmt], nch, frames, _ptr(d_out),
                                       out_stride, stream or None))


def encode_pcm_dev(d_in, in_stride: int, nch: int, frames: int, fmt: str, d_out, stream=0):
    """Planar float32 (device) -> interleaved PCM bytes (device)."""
    _check(load().lcfir_encode_pcm_dev(_ptr(d_in), in_stride, nch, frames, PCM_FORMATS[fmt],
                                       _ptr(d_out), stream or None))


def encode_pcm_scaled_dev(d_in, in_stride: int, nch: int, frames: int, fmt: str, d_peak, npeak: int,
                          force: bool, d_out, stream=0):
    """normalize_dev + encode_pcm_dev in one pass (byte-identical; d_in is not rescaled)."""
    _check(load().lcfir_encode_pcm_scaled_dev(_ptr(d_in), in_stride, nch, frames, PCM_FORMATS[fmt],
                                              _ptr(d_peak), npeak, 1 if force else 0, _ptr(d_out),
                                              stream or None))

"""ctypes binding of libmsdsp.so (the C-ABI declared in include/msdsp.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C
meteor-scatter_amd/csrc``) and loaded from this directory.  There is no CPU
fallback: every compute entry point runs the HIP kernels, and a missing library
or a missing GPU raises ``MsdError`` / ``OSError`` loudly.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

LIB_PATH = Path(os.environ.get("MSD_LIB_PATH") or Path(__file__).with_name("libmsdsp.so"))

MSD_OK = 0
MSD_ERR_INVALID = -1
MSD_ERR_HIP = -2
MSD_ERR_UNSUPPORTED = -3
MSD_ERR_ASSERT = -4
MSD_ERR_CAPACITY = -5
MSD_ERR_INDEX = -6
MSD_ERR_RCCL = -7

MSD_U8, MSD_I16, MSD_I32, MSD_F32, MSD_F64 = 1, 2, 3, 4, 5
MSD_CI16, MSD_CF32 = 6, 7  # interleaved I/Q
DTYPE_CODES = {
    np.dtype(np.uint8): MSD_U8,
    np.dtype(np.int16): MSD_I16,
    np.dtype(np.int32): MSD_I32,
    np.dtype(np.float32): MSD_F32,
    np.dtype(np.float64): MSD_F64,
}

K_STFT, K_BLOCK, K_DSTAT, K_DSCAN, K_WELCH, K_LIVE, K_CSTFT = 0, 1, 2, 3, 4, 5, 6
K_IQDELTA, K_FRESH, K_SSCAN, K_REFINE, K_CSTFT_DC = 7, 8, 9, 10, 11
OPT_GENERIC_STFT = 1
OPT_FRESH_ALL = 2
OPT_REFINE_GOERTZEL = 3
OPT_CSTFT_RESERVE = 4
OPT_STREAM_CUS = 5
OPT_CSTFT_SCHED = 6
OPT_STFT_SCHED = 7
OPT_BLOCK_GOERTZEL = 8
OPT_WELCH_GOERTZEL = 9
COMM_ID_BYTES = 128


class MsdError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"libmsdsp error {code}: {msg}")
        self.code = code
        self.msg = msg


class MsdDet(C.Structure):
    _fields_ = [("start", C.c_int64), ("stop", C.c_int64), ("db", C.c_double)]


DET_DTYPE = np.dtype([("start", np.int64), ("stop", np.int64), ("db", np.float64)])


class MsdDetCfg(C.Structure):
    _fields_ = [
        ("adaptive", C.c_int32),
        ("reserved", C.c_int32),
        ("k_std", C.c_double),
        ("window_blocks", C.c_int64),
        ("freeze_before_blocks", C.c_int64),
        ("freeze_after_blocks", C.c_int64),
        ("fixed_init_blocks", C.c_int64),
    ]


class MsdHistCfg(C.Structure):
    _fields_ = [
        ("file_start_us", C.c_void_p),
        ("base_us", C.c_int64),
        ("bucket_us", C.c_int64),
        ("nbuckets", C.c_int32),
        ("reserved", C.c_int32),
        ("block_sec", C.c_double),
        ("counts", C.c_void_p),
    ]


WELCH_MAX_BANDS = 8


class MsdWelchCfg(C.Structure):
    _fields_ = [
        ("block_size", C.c_int32),
        ("nperseg", C.c_int32),
        ("noverlap", C.c_int32),
        ("nfft", C.c_int32),
        ("sample_scale", C.c_double),
        ("scale", C.c_double),
        ("nbands", C.c_int32),
        ("reserved", C.c_int32),
        ("band_lo", C.c_int32 * WELCH_MAX_BANDS),
        ("band_hi", C.c_int32 * WELCH_MAX_BANDS),
    ]


class MsdLiveCfg(C.Structure):
    _fields_ = [
        ("block_size", C.c_int32),
        ("avg_win_blocks", C.c_int32),
        ("fs", C.c_double),
        ("k_std", C.c_double),
        ("init_wait_sec", C.c_double),
        ("after_tracking_wait_sec", C.c_double),
        ("min_db_mean", C.c_double),
        ("min_dur_sec", C.c_double),
    ]


METEOR_DTYPE = np.dtype([("start_block", np.int64), ("stop_block", np.int64), ("time_start", np.float64),
                         ("time_stop", np.float64), ("duration", np.float64), ("db_min", np.float64),
                         ("db_max", np.float64), ("db_mean", np.float64), ("db_std", np.float64)])


class MsdStreamState(C.Structure):
    """msd_stream_state: the detector state entering a frame (main.py:455-493 variables), plus the
    frame whose fresh threshold ``thr`` is (-1: thr0) and its error bound (certification)."""
    _fields_ = [("freeze_until", C.c_int64), ("last_stop", C.c_int64), ("thr", C.c_double),
                ("src", C.c_int64), ("thr_err", C.c_double)]


class MsdWavInfo(C.Structure):
    _fields_ = [
        ("rate", C.c_int32),
        ("channels", C.c_int32),
        ("bits", C.c_int32),
        ("format", C.c_int32),
        ("dtype", C.c_int32),
        ("reserved", C.c_int32),
        ("frames", C.c_int64),
        ("data_offset", C.c_int64),
        ("data_bytes", C.c_int64),
    ]


# (name, restype, argtypes) — every symbol of include/msdsp.h
_P = C.c_void_p
_SIGS = [
    ("msd_abi_version", C.c_int, []),
    ("msd_last_error", C.c_char_p, []),
    ("msd_device_count", C.c_int, [C.POINTER(C.c_int)]),
    ("msd_create", C.c_int, [C.c_int, C.POINTER(_P)]),
    ("msd_destroy", None, [_P]),
    ("msd_synchronize", C.c_int, [_P]),
    ("msd_dev_alloc", C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    ("msd_dev_free", C.c_int, [_P, _P]),
    ("msd_memcpy_h2d", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("msd_memcpy_d2h", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("msd_memset_dev", C.c_int, [_P, _P, C.c_int, C.c_size_t]),
    ("msd_set_option", C.c_int, [_P, C.c_int, C.c_int]),
    ("msd_timing_enable", C.c_int, [_P, C.c_int]),
    ("msd_timing_select", C.c_int, [_P, C.c_uint32]),
    ("msd_timing_reset", C.c_int, [_P]),
    ("msd_timing_get", C.c_int, [_P, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int64)]),
    ("msd_stft_plan_create", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_double, C.POINTER(_P)]),
    ("msd_stft_plan_create_ex", C.c_int,
     [_P, C.c_int32, C.c_int32, C.c_int32, _P, C.c_double, C.c_int, C.POINTER(_P)]),
    ("msd_stft_plan_destroy", None, [_P]),
    ("msd_stft_bins", C.c_int32, [_P]),
    ("msd_stft_plan_set_detrend", C.c_int, [_P, C.c_int]),
    ("msd_stft_frames", C.c_int64, [_P, C.c_int64]),
    ("msd_stft_psd_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, C.c_int64]),
    ("msd_stft_psd", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, C.POINTER(C.c_int64)]),
    ("msd_stft_psd_f64_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, C.c_int64]),
    ("msd_stft_psd_f64", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, C.POINTER(C.c_int64)]),
    ("msd_block_plan_create", C.c_int,
     [_P, C.c_int64, C.c_int32, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.POINTER(_P)]),
    ("msd_block_plan_destroy", None, [_P]),
    ("msd_block_delta_dev", C.c_int,
     [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, _P, _P, C.c_int64]),
    ("msd_block_delta", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, _P, _P, C.POINTER(C.c_int64)]),
    ("msd_detect_dev", C.c_int,
     [_P, _P, _P, C.c_int64, C.c_int64, C.POINTER(MsdDetCfg), _P, C.c_int64, _P, _P, _P, _P,
      C.POINTER(MsdHistCfg)]),
    ("msd_detect", C.c_int,
     [_P, _P, C.c_int64, C.POINTER(MsdDetCfg), _P, C.c_int64, C.POINTER(C.c_int64), _P, _P]),
    ("msd_cstft_plan_create", C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_double, C.POINTER(_P)]),
    ("msd_cstft_plan_destroy", None, [_P]),
    ("msd_cstft_set_detrend", C.c_int, [_P, C.c_int]),
    ("msd_cstft_frames", C.c_int64, [_P, C.c_int64]),
    ("msd_cstft_psd_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P]),
    ("msd_cstft_psd", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, C.POINTER(C.c_int64)]),
    ("msd_cstft_psd_energy_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, _P]),
    ("msd_cstft_psd_fsums_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, _P, _P]),
    ("msd_cstft_energy_stride", C.c_int64, [C.c_int64, C.c_int64]),
    ("msd_spec_band_sum_dev", C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P]),
    ("msd_spec_band_sum_f64_dev", C.c_int,
     [_P, _P, C.c_int64, C.c_int32, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P]),
    ("msd_welch_plan_create", C.c_int, [_P, C.POINTER(MsdWelchCfg), _P, C.POINTER(_P)]),
    ("msd_welch_plan_destroy", None, [_P]),
    ("msd_welch_bands_dev", C.c_int, [_P, _P, C.c_int, _P, _P, C.c_int64, C.c_int64, _P, C.c_int64, _P]),
    ("msd_welch_bands", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, C.POINTER(C.c_int64)]),
    ("msd_welch_psd", C.c_int, [_P, _P, C.c_int, C.c_int64, _P, C.POINTER(C.c_int64)]),
    ("msd_live_detect_dev", C.c_int,
     [_P, _P, _P, C.c_int64, C.c_int64, C.POINTER(MsdLiveCfg), _P, C.c_int64, _P, _P, _P, _P]),
    ("msd_live_detect", C.c_int,
     [_P, _P, C.c_int64, C.POINTER(MsdLiveCfg), _P, C.c_int64, C.POINTER(C.c_int64), _P, _P]),
    ("msd_wav_probe", C.c_int, [C.c_char_p, C.POINTER(MsdWavInfo)]),
    ("msd_wav_read", C.c_int, [C.c_char_p, C.c_int32, C.c_int64, C.c_int64, _P, C.c_int64, C.POINTER(MsdWavInfo)]),
    ("msd_host_alloc", C.c_int, [_P, C.c_size_t, C.POINTER(_P)]),
    ("msd_host_free", C.c_int, [_P, _P]),
    ("msd_memcpy_h2d_async", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("msd_fence", C.c_int, [_P, C.c_int]),
    ("msd_copy_synchronize", C.c_int, [_P]),
    ("msd_stream_wait", C.c_int, [_P, _P]),
    ("msd_comm_get_unique_id", C.c_int, [_P]),
    ("msd_comm_init", C.c_int, [_P, C.c_int, _P, C.c_int, C.POINTER(_P)]),
    ("msd_comm_destroy", None, [_P]),
    ("msd_comm_allreduce_i64", C.c_int, [_P, _P, C.c_int64]),
    ("msd_comm_allgather", C.c_int, [_P, _P, _P, C.c_size_t]),
    ("msd_iq_band_delta_dev", C.c_int,
     [_P, _P, C.c_int64, C.c_int64, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P,
      C.c_int64]),
    ("msd_iq_band_delta_bound_dev", C.c_int,
     [_P, _P, _P, C.c_int64, C.c_int64, _P, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32, _P, _P, _P, _P,
      C.c_int64]),
    ("msd_iq_delta64_dev", C.c_int,
     [_P, _P, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_double, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
      _P, C.c_int64, _P, _P]),
    ("msd_iq_delta64_sums_dev", C.c_int,
     [_P, _P, C.c_int32, C.c_int64, C.c_int32, C.c_int64, C.c_double, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
      _P, C.c_int64, _P, _P, _P]),
    ("msd_iq_delta64_path", C.c_int,
     [C.c_int32, C.c_int64, C.c_double, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
    ("msd_stream_plan_create", C.c_int,
     [_P, C.POINTER(MsdDetCfg), C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.POINTER(_P)]),
    ("msd_stream_plan_destroy", None, [_P]),
    ("msd_stream_buffers", C.c_int,
     [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(C.c_int64), C.POINTER(_P), C.POINTER(C.c_int64),
      C.POINTER(_P)]),
    ("msd_stream_chunk_sums", C.c_int,
     [_P, C.c_int32, C.c_double, _P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    ("msd_stream_set_exact_thresholds", C.c_int, [_P, C.c_int32]),
    ("msd_stream_detect_local", C.c_int, [_P, C.c_int32, _P, C.c_int64, C.POINTER(C.c_int64),
                                          C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_int32),
                                          C.POINTER(C.c_int32)]),
    ("msd_stream_fresh", C.c_int, [_P]),
    ("msd_stream_predicted", C.c_int, [_P, _P, _P]),
    ("msd_stream_refine", C.c_int, [_P, C.POINTER(C.c_int32)]),
    ("msd_stream_scan", C.c_int,
     [_P, C.c_double, C.POINTER(MsdStreamState), C.c_int32, C.POINTER(MsdStreamState), C.POINTER(C.c_int32)]),
    ("msd_stream_runs", C.c_int, [_P, _P, C.c_int64, C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
    ("msd_stream_db", C.c_int, [_P, _P, C.c_int64]),
    ("msd_stream_set_certify", C.c_int, [_P, C.c_int32]),
    ("msd_stream_error_buffers", C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.POINTER(_P)]),
    ("msd_stream_ed_sums", C.c_int, [_P, C.POINTER(C.c_double), C.POINTER(C.c_double)]),
    ("msd_stream_set_terr0", C.c_int, [_P, C.c_double, C.c_double]),
    ("msd_stream_certificate", C.c_int,
     [_P, C.POINTER(C.c_int64), C.POINTER(C.c_double), C.POINTER(C.c_double), _P, _P, C.c_int64,
      C.POINTER(C.c_int64)]),
]
SYMBOLS = [s[0] for s in _SIGS]

_lib = None


def load() -> C.CDLL:
    """Load libmsdsp.so from the package directory (raises OSError if absent)."""
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise OSError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() or "
                f"`make -C meteor-scatter_amd/csrc` (there is no CPU fallback)")
        lib = C.CDLL(str(LIB_PATH), mode=os.RTLD_LOCAL | getattr(os, "RTLD_NOW", 2))
        for name, res, args in _SIGS:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int) -> None:
    if rc != MSD_OK:
        msg = load().msd_last_error()
        raise MsdError(rc, msg.decode() if msg else "")


def ptr(a: np.ndarray | None):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def dtype_code(dt) -> int:
    dt = np.dtype(dt)
    if dt.byteorder == ">":
        raise ValueError("big-endian samples are not supported")
    try:
        return DTYPE_CODES[dt.newbyteorder("=")]
    except KeyError:
        raise TypeError(f"unsupported sample dtype {dt}") from None


def device_count() -> int:
    n = C.c_int(0)
    check(load().msd_device_count(C.byref(n)))
    return n.value


class Context:
    """A device + HIP stream (msd_ctx).  Not thread-safe."""

    def __init__(self, device: int = 0):
        self.lib = load()
        h = C.c_void_p()
        check(self.lib.msd_create(int(device), C.byref(h)))
        self.h = h
        self.device = int(device)
        self.options: dict[int, int] = {}  # msd_set_option values set on this context
        self.timing_on = False

    def close(self):
        if getattr(self, "h", None):
            self.lib.msd_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def synchronize(self):
        check(self.lib.msd_synchronize(self.h))

    def wait_for(self, other: "Context"):
        """Work enqueued on this context from now on waits for ``other``'s work so far."""
        check(self.lib.msd_stream_wait(self.h, other.h))

    # ---- device memory
    def alloc(self, nbytes: int) -> "DeviceBuffer":
        return DeviceBuffer(self, nbytes)

    def set_option(self, option: int, value: int):
        check(self.lib.msd_set_option(self.h, int(option), int(value)))
        self.options[int(option)] = int(value)

    def timing(self, enable: bool = True):
        check(self.lib.msd_timing_enable(self.h, 1 if enable else 0))
        self.timing_on = bool(enable)

    def timing_select(self, kernels=None):
        """time only these kernel ids (K_*) while timing is on; None: all"""
        mask = 0xFFFFFFFF if kernels is None else sum(1 << int(k) for k in kernels)
        check(self.lib.msd_timing_select(self.h, mask))

    def sibling(self) -> "Context":
        """A new context (own HIP stream) on the same device with this one's options and timing
        switch, e.g. for a stage that runs beside this context's work."""
        c = Context(self.device)
        for k, v in self.options.items():
            c.set_option(k, v)
        if self.timing_on:
            c.timing(True)
        return c

    def timing_reset(self):
        check(self.lib.msd_timing_reset(self.h))

    def timing_get(self, kernel: int):
        ms = C.c_double(0)
        n = C.c_int64(0)
        check(self.lib.msd_timing_get(self.h, int(kernel), C.byref(ms), C.byref(n)))
        return ms.value, n.value


class DeviceBuffer:
    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = C.c_void_p()
        check(ctx.lib.msd_dev_alloc(ctx.h, C.c_size_t(self.nbytes), C.byref(p)))
        self.ptr = p

    def free(self):
        if self.ptr:
            check(self.ctx.lib.msd_dev_free(self.ctx.h, self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            if self.ptr and self.ctx.h:
                self.ctx.lib.msd_dev_free(self.ctx.h, self.ptr)
        except Exception:
            pass

    def at(self, byte_offset: int):
        return C.c_void_p(self.ptr.value + int(byte_offset))

    def upload(self, a: np.ndarray, byte_offset: int = 0):
        a = np.ascontiguousarray(a)
        if byte_offset + a.nbytes > self.nbytes:
            raise ValueError("upload overflows device buffer")
        check(self.ctx.lib.msd_memcpy_h2d(self.ctx.h, self.at(byte_offset), ptr(a), C.c_size_t(a.nbytes)))

    def download(self, out: np.ndarray, byte_offset: int = 0) -> np.ndarray:
        if not out.flags.c_contiguous:
            raise ValueError("download target must be contiguous")
        if byte_offset + out.nbytes > self.nbytes:
            raise ValueError("download overflows device buffer")
        check(self.ctx.lib.msd_memcpy_d2h(self.ctx.h, ptr(out), self.at(byte_offset), C.c_size_t(out.nbytes)))
        return out

    def memset(self, value: int = 0):
        check(self.ctx.lib.msd_memset_dev(self.ctx.h, self.ptr, int(value), C.c_size_t(self.nbytes)))


class StftPlan:
    """msd_stft_plan: nperseg-sample segments (hop apart) zero-padded to nfft (default nperseg),
    float32 (``precision=np.float32``) or float64 arithmetic and output [K = nfft/2 + 1][T]."""

    def __init__(self, ctx: Context, nperseg: int, hop: int, window: np.ndarray, scale: float, nfft: int | None = None,
                 precision=np.float32):
        self.ctx = ctx
        nfft = int(nperseg) if nfft is None else int(nfft)
        self.dtype = np.dtype(precision)
        if self.dtype not in (np.float32, np.float64):
            raise ValueError("precision must be float32 or float64")
        h = C.c_void_p()
        if nfft == nperseg and self.dtype == np.float32:
            w = np.ascontiguousarray(window, dtype=np.float32)
            if w.shape != (nperseg,):
                raise ValueError("window length must equal nperseg")
            check(ctx.lib.msd_stft_plan_create(ctx.h, int(nperseg), int(hop), ptr(w), float(scale), C.byref(h)))
        else:
            w = np.ascontiguousarray(window, dtype=np.float64)
            if w.shape != (nperseg,):
                raise ValueError("window length must equal nperseg")
            prec = MSD_F64 if self.dtype == np.float64 else MSD_F32
            check(ctx.lib.msd_stft_plan_create_ex(ctx.h, int(nperseg), nfft, int(hop), ptr(w), float(scale), prec,
                                                  C.byref(h)))
        self.h = h
        self.nperseg, self.hop, self.nfft = int(nperseg), int(hop), nfft
        self.nbins = int(ctx.lib.msd_stft_bins(h))

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:  # a plan outliving its context leaks, never crashes
            self.ctx.lib.msd_stft_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def frames(self, n: int) -> int:
        return int(self.ctx.lib.msd_stft_frames(self.h, int(n)))

    def set_detrend(self, detrend: bool):
        """True: scipy's 'constant' detrend (the default); False: none (matplotlib mlab)."""
        check(self.ctx.lib.msd_stft_plan_set_detrend(self.h, 1 if detrend else 0))

    def run(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x)
        T = self.frames(x.shape[0])
        out = np.empty((self.nbins, T), dtype=self.dtype)
        t = C.c_int64(0)
        fn = self.ctx.lib.msd_stft_psd_f64 if self.dtype == np.float64 else self.ctx.lib.msd_stft_psd
        check(fn(self.h, ptr(x), dtype_code(x.dtype), int(x.shape[0]), ptr(out), C.byref(t)))
        return out

    def run_dev(self, x: DeviceBuffer, dtype, off: DeviceBuffer, length: DeviceBuffer, nfiles: int,
                max_frames: int, out: DeviceBuffer, ld: int):
        fn = self.ctx.lib.msd_stft_psd_f64_dev if self.dtype == np.float64 else self.ctx.lib.msd_stft_psd_dev
        check(fn(self.h, x.ptr, dtype_code(dtype), off.ptr, length.ptr, int(nfiles), int(max_frames), out.ptr,
                 int(ld)))


class BlockPlan:
    def __init__(self, ctx: Context, block_size: int, nfft: int, window: np.ndarray, band: tuple[int, int],
                 noise: tuple[int, int]):
        self.ctx = ctx
        w = np.ascontiguousarray(window, dtype=np.float64)
        h = C.c_void_p()
        check(ctx.lib.msd_block_plan_create(ctx.h, int(block_size), int(nfft), ptr(w), int(band[0]), int(band[1]),
                                            int(noise[0]), int(noise[1]), C.byref(h)))
        self.h = h
        self.block_size = int(block_size)
        self.nfft = int(nfft)

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:  # a plan outliving its context leaks, never crashes
            self.ctx.lib.msd_block_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def run(self, x: np.ndarray):
        x = np.ascontiguousarray(x)
        nb = x.shape[0] // self.block_size
        band = np.empty(nb, np.float64)
        noise = np.empty(nb, np.float64)
        delta = np.empty(nb, np.float64)
        got = C.c_int64(0)
        check(self.ctx.lib.msd_block_delta(self.h, ptr(x), dtype_code(x.dtype), int(x.shape[0]), ptr(band),
                                           ptr(noise), ptr(delta), C.byref(got)))
        return band, noise, delta

    def run_dev(self, x: DeviceBuffer, dtype, off: DeviceBuffer, length: DeviceBuffer, nfiles: int,
                max_blocks: int, band, noise, delta: DeviceBuffer, ld: int):
        check(self.ctx.lib.msd_block_delta_dev(self.h, x.ptr, dtype_code(dtype), off.ptr, length.ptr, int(nfiles),
                                               int(max_blocks), band.ptr if band else None,
                                               noise.ptr if noise else None, delta.ptr, int(ld)))


def det_cfg(adaptive: bool, k_std: float, window_blocks: int = 0, freeze_before: int = 0, freeze_after: int = 0,
            fixed_init: int = 0) -> MsdDetCfg:
    return MsdDetCfg(1 if adaptive else 0, 0, float(k_std), int(window_blocks), int(freeze_before),
                     int(freeze_after), int(fixed_init))


def detect(ctx: Context, delta: np.ndarray, cfg: MsdDetCfg, cap: int | None = None):
    """Single-file detector on host delta: returns (dets[start, stop, db], thresholds, margin)."""
    d = np.ascontiguousarray(delta, dtype=np.float64)
    nb = d.shape[0]
    if cap is None:
        cap = nb // 2 + 2
    dets = np.zeros(cap, dtype=DET_DTYPE)
    thr = np.empty(max(nb, 1) if cfg.adaptive else 1, np.float64)
    count = C.c_int64(0)
    margin = C.c_double(0)
    check(ctx.lib.msd_detect(ctx.h, ptr(d), int(nb), C.byref(cfg), ptr(dets), int(cap), C.byref(count), ptr(thr),
                             C.byref(margin)))
    return dets[: count.value], thr[:nb] if cfg.adaptive else thr, margin.value


class WelchPlan:
    """Per-block Welch band powers (include/msdsp.h a8)."""

    def __init__(self, ctx: Context, cfg: MsdWelchCfg, window: np.ndarray):
        self.ctx = ctx
        w = np.ascontiguousarray(window, dtype=np.float64)
        if w.shape != (cfg.nperseg,):
            raise ValueError("window length must equal nperseg")
        h = C.c_void_p()
        check(ctx.lib.msd_welch_plan_create(ctx.h, C.byref(cfg), ptr(w), C.byref(h)))
        self.h = h
        self.cfg = cfg
        self.nbands = int(cfg.nbands)
        self.block_size = int(cfg.block_size)

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:  # a plan outliving its context leaks, never crashes
            self.ctx.lib.msd_welch_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def blocks(self, n: int) -> int:
        return (n - self.block_size) // self.block_size + 1 if n >= self.block_size else 0

    def run(self, x: np.ndarray) -> np.ndarray:
        """band dB [nbands][nb] of one signal (host buffers)."""
        x = np.ascontiguousarray(x)
        nb = self.blocks(x.shape[0])
        out = np.empty((self.nbands, nb), np.float64)
        got = C.c_int64(0)
        check(self.ctx.lib.msd_welch_bands(self.h, ptr(x), dtype_code(x.dtype), int(x.shape[0]), ptr(out),
                                           C.byref(got)))
        return out

    def psd(self, x: np.ndarray, nslots: int) -> np.ndarray:
        """[nb][nslots] per-block PSD of the band bins (host buffers)."""
        x = np.ascontiguousarray(x)
        nb = self.blocks(x.shape[0])
        out = np.empty((nb, nslots), np.float64)
        got = C.c_int64(0)
        check(self.ctx.lib.msd_welch_psd(self.h, ptr(x), dtype_code(x.dtype), int(x.shape[0]), ptr(out),
                                         C.byref(got)))
        return out

    def run_dev(self, x: DeviceBuffer, dtype, off: DeviceBuffer, length: DeviceBuffer, nfiles: int,
                max_blocks: int, band_db: DeviceBuffer, ld: int, psd: DeviceBuffer | None = None):
        check(self.ctx.lib.msd_welch_bands_dev(self.h, x.ptr, dtype_code(dtype), off.ptr, length.ptr, int(nfiles),
                                               int(max_blocks), band_db.ptr, int(ld), psd.ptr if psd else None))


def live_detect(ctx: Context, band_db: np.ndarray, cfg: MsdLiveCfg, cap: int | None = None):
    """Live-detector state machine on host band dB rows [3][nb]: (meteors, thresholds, over)."""
    b = np.ascontiguousarray(band_db, dtype=np.float64)
    if b.ndim != 2 or b.shape[0] != 3:
        raise ValueError("band_db must be [3][nb] (signal, noise 1, noise 2)")
    nb = b.shape[1]
    if cap is None:
        cap = nb // 2 + 2
    out = np.zeros(cap, dtype=METEOR_DTYPE)
    thr = np.empty(max(nb, 1), np.float64)
    over = np.empty(max(nb, 1), np.float64)
    count = C.c_int64(0)
    check(ctx.lib.msd_live_detect(ctx.h, ptr(b), int(nb), C.byref(cfg), ptr(out), int(cap), C.byref(count),
                                  ptr(thr), ptr(over)))
    return out[: count.value], thr[:nb], over[:nb]


class CStftPlan:
    """Two-sided power spectrogram of complex (I/Q) samples (include/msdsp.h, config C5)."""

    def __init__(self, ctx: Context, nperseg: int, hop: int, window: np.ndarray, scale: float):
        self.ctx = ctx
        w = np.ascontiguousarray(window, dtype=np.float32)
        if w.shape != (nperseg,):
            raise ValueError("window length must equal nperseg")
        h = C.c_void_p()
        check(ctx.lib.msd_cstft_plan_create(ctx.h, int(nperseg), int(hop), ptr(w), float(scale), C.byref(h)))
        self.h = h
        self.nperseg, self.hop = int(nperseg), int(hop)

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:  # a plan outliving its context leaks, never crashes
            self.ctx.lib.msd_cstft_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def frames(self, n: int) -> int:
        return int(self.ctx.lib.msd_cstft_frames(self.h, int(n)))

    def run(self, iq: np.ndarray, dtype_code_iq: int) -> np.ndarray:
        """iq: interleaved I/Q (int16 or float32), 2*n elements → float32 [T][nperseg] (frame-major)."""
        iq = np.ascontiguousarray(iq)
        n = iq.shape[0] // 2
        T = self.frames(n)
        out = np.empty((T, self.nperseg), np.float32)
        t = C.c_int64(0)
        check(self.ctx.lib.msd_cstft_psd(self.h, ptr(iq), int(dtype_code_iq), int(n), ptr(out), C.byref(t)))
        return out

    def run_dev(self, x: DeviceBuffer, dtype_code_iq: int, off: DeviceBuffer, length: DeviceBuffer, nstreams: int,
                max_frames: int, out: DeviceBuffer, etot: DeviceBuffer | None = None, fsums=None):
        """etot: also each frame's 16 total-power partials (msd_cstft_psd_energy_dev); fsums: each
        frame's (sum I, sum Q) float64 on the device (msd_cstft_psd_fsums_dev, e.g. from
        iq_delta64_dev(..., frame_sums=...))"""
        check(self.ctx.lib.msd_cstft_psd_fsums_dev(self.h, x.ptr, int(dtype_code_iq), off.ptr, length.ptr,
                                                   int(nstreams), int(max_frames), out.ptr,
                                                   None if etot is None else etot.ptr, _dp(fsums)))


class StreamPlan:
    """One rank's shard of a long stream's per-frame delta and the detector over it
    (include/msdsp.h, C5 stream detector); driven by meteorgpu.stream.StreamDetector."""

    def __init__(self, ctx: Context, cfg: MsdDetCfg, n_total: int, frame0: int, n_local: int,
                 seg_len: int = 8192, cap_per_seg: int = 256, head_frames: int = 8192):
        self.ctx = ctx
        self.cfg = cfg
        h = C.c_void_p()
        check(ctx.lib.msd_stream_plan_create(ctx.h, C.byref(cfg), int(n_total), int(frame0), int(n_local),
                                             int(seg_len), int(cap_per_seg), int(head_frames), C.byref(h)))
        self.h = h
        self.n_total, self.frame0, self.n_local = int(n_total), int(frame0), int(n_local)
        self.seg_len, self.cap_per_seg = int(seg_len), int(cap_per_seg)
        d, t, hd, thr = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        nt, nh = C.c_int64(0), C.c_int64(0)
        check(ctx.lib.msd_stream_buffers(h, C.byref(d), C.byref(t), C.byref(nt), C.byref(hd), C.byref(nh),
                                         C.byref(thr)))
        self.d_delta, self.d_tail, self.d_head, self.d_thr = d, t, hd, thr
        self.n_tail, self.n_head = nt.value, nh.value
        self.nseg = -(-self.n_local // self.seg_len) if self.n_local else 0
        e, et, eh = C.c_void_p(), C.c_void_p(), C.c_void_p()
        check(ctx.lib.msd_stream_error_buffers(h, C.byref(e), C.byref(et), C.byref(eh)))
        self.d_ed, self.d_ed_tail, self.d_ed_head = e, et, eh
        self.certify = False

    def close(self):
        if getattr(self, "h", None) and self.ctx.h:  # a plan outliving its context leaks, never crashes
            self.ctx.lib.msd_stream_plan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _put(self, dptr, a: np.ndarray):
        a = np.ascontiguousarray(a, dtype=np.float64)
        if a.size:
            check(self.ctx.lib.msd_memcpy_h2d(self.ctx.h, dptr, ptr(a), C.c_size_t(a.nbytes)))

    def _get(self, dptr, n: int) -> np.ndarray:
        out = np.empty(int(n), np.float64)
        if n:
            check(self.ctx.lib.msd_memcpy_d2h(self.ctx.h, ptr(out), dptr, C.c_size_t(out.nbytes)))
        return out

    def set_delta(self, delta: np.ndarray):
        if np.asarray(delta).shape != (self.n_local,):
            raise ValueError("delta must hold the shard's n_local frames")
        self._put(self.d_delta, delta)

    def delta(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        """the shard's delta [lo, hi) (local frame indices)"""
        hi = self.n_local if hi is None else hi
        return self._get(C.c_void_p(self.d_delta.value + 8 * lo), hi - lo) if hi > lo else np.zeros(0)

    def set_halos(self, tail: np.ndarray, head: np.ndarray):
        if np.asarray(tail).shape != (self.n_tail,) or np.asarray(head).shape != (self.n_head,):
            raise ValueError(f"halos must hold {self.n_tail} / {self.n_head} frames")
        self._put(self.d_tail, tail)
        self._put(self.d_head, head)

    # ---- certification against the float64 reference (include/msdsp.h msd_stream_set_certify)
    def set_certify(self, on: bool):
        check(self.ctx.lib.msd_stream_set_certify(self.h, 1 if on else 0))
        self.certify = bool(on)

    def set_ed(self, ed: np.ndarray):
        """the shard's delta error bounds (n_local; 0 = exact)"""
        if np.asarray(ed).shape != (self.n_local,):
            raise ValueError("ed must hold the shard's n_local frames")
        self._put(self.d_ed, ed)

    def ed(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.n_local if hi is None else hi
        return self._get(C.c_void_p(self.d_ed.value + 8 * lo), hi - lo) if hi > lo else np.zeros(0)

    def set_ed_halos(self, tail: np.ndarray, head: np.ndarray):
        if np.asarray(tail).shape != (self.n_tail,) or np.asarray(head).shape != (self.n_head,):
            raise ValueError(f"halos must hold {self.n_tail} / {self.n_head} frames")
        self._put(self.d_ed_tail, tail)
        self._put(self.d_ed_head, head)

    def ed_sums(self) -> tuple[float, float]:
        a, b = C.c_double(0), C.c_double(0)
        check(self.ctx.lib.msd_stream_ed_sums(self.h, C.byref(a), C.byref(b)))
        return a.value, b.value

    def set_terr0(self, s1: float, s2: float):
        check(self.ctx.lib.msd_stream_set_terr0(self.h, float(s1), float(s2)))

    def certificate(self, cap: int = 4096):
        """after the last scan: (uncertain decisions, min slack, max error zone, listed [(global frame,
        threshold source frame)])"""
        n, ms, mz, nl = C.c_int64(0), C.c_double(0), C.c_double(0), C.c_int64(0)
        fr = np.zeros(cap, np.int64)
        sr = np.zeros(cap, np.int64)
        check(self.ctx.lib.msd_stream_certificate(self.h, C.byref(n), C.byref(ms), C.byref(mz), ptr(fr), ptr(sr),
                                                  int(cap), C.byref(nl)))
        k = nl.value
        return n.value, ms.value, mz.value, np.stack([fr[:k], sr[:k]], 1)

    exact_thresholds = True

    def set_exact_thresholds(self, on: bool):
        """False: only the detections are numpy-exact (msd_stream_set_exact_thresholds)."""
        check(self.ctx.lib.msd_stream_set_exact_thresholds(self.h, 1 if on else 0))
        self.exact_thresholds = bool(on)

    def thresholds(self) -> np.ndarray:
        if not self.exact_thresholds:
            raise RuntimeError("StreamPlan.thresholds: the plan computes exact decisions only "
                               "(set_exact_thresholds(False))")
        return self._get(self.d_thr, self.n_local)

    def chunk_sums(self, mean: float | None = None) -> tuple[int, np.ndarray]:
        cap = self.n_local // 8192 + 2
        out = np.empty(cap, np.float64)
        n, c0 = C.c_int64(0), C.c_int64(0)
        check(self.ctx.lib.msd_stream_chunk_sums(self.h, 0 if mean is None else 1, 0.0 if mean is None else mean,
                                                 ptr(out), cap, C.byref(n), C.byref(c0)))
        return c0.value, out[: n.value].copy()

    def fresh(self):
        check(self.ctx.lib.msd_stream_fresh(self.h))

    def predicted(self) -> tuple[np.ndarray, np.ndarray]:
        """decisions-only mode, after fresh(): (predicted thresholds, error bounds)"""
        f = np.empty(self.n_local, np.float64)
        e = np.empty(self.n_local, np.float64)
        check(self.ctx.lib.msd_stream_predicted(self.h, ptr(f), ptr(e)))
        return f, e

    def refine(self) -> int:
        n = C.c_int32(0)
        check(self.ctx.lib.msd_stream_refine(self.h, C.byref(n)))
        return n.value

    def scan(self, thr0: float, entry: MsdStreamState, reset: int) -> tuple[MsdStreamState, int]:
        """reset 1: clean restart; 2: re-scan every segment (thresholds refined); 0: entry changed"""
        ex = MsdStreamState()
        rounds = C.c_int32(0)
        check(self.ctx.lib.msd_stream_scan(self.h, float(thr0), C.byref(entry), int(reset), C.byref(ex),
                                           C.byref(rounds)))
        return ex, rounds.value

    def runs(self) -> tuple[np.ndarray, float]:
        cap = max(1, self.nseg * self.cap_per_seg)
        out = np.zeros(cap, dtype=DET_DTYPE)
        n = C.c_int64(0)
        mg = C.c_double(0)
        check(self.ctx.lib.msd_stream_runs(self.h, ptr(out), cap, C.byref(n), C.byref(mg)))
        return out[: n.value].copy(), mg.value

    def detect_local(self, exact_thresholds: bool = True):
        """msd_stream_detect_local (the plan holds the whole stream): (detections, thr0, margin,
        rounds, refined)"""
        cap = max(1, self.nseg * self.cap_per_seg)
        out = np.zeros(cap, dtype=DET_DTYPE)
        n, thr0, mg = C.c_int64(0), C.c_double(0), C.c_double(0)
        rounds, refined = C.c_int32(0), C.c_int32(0)
        check(self.ctx.lib.msd_stream_detect_local(self.h, 1 if exact_thresholds else 0, ptr(out), cap, C.byref(n),
                                                   C.byref(thr0), C.byref(mg), C.byref(rounds), C.byref(refined)))
        self.exact_thresholds = bool(exact_thresholds)
        return out[: n.value].copy(), thr0.value, mg.value, rounds.value, refined.value

    def db(self, dets: np.ndarray) -> np.ndarray:
        d = np.ascontiguousarray(dets, dtype=DET_DTYPE).copy()
        check(self.ctx.lib.msd_stream_db(self.h, ptr(d), d.shape[0]))
        return d


def _dp(b):
    return b.ptr if isinstance(b, DeviceBuffer) else b


def iq_band_delta_dev(ctx: Context, spec: DeviceBuffer, nstreams: int, max_frames: int, frames: DeviceBuffer,
                      nperseg: int, band: tuple[int, int], noise: tuple[int, int], delta, ld: int,
                      band_db=None, noise_db=None, etot=None, ed=None):
    """delta (device pointer or DeviceBuffer) [s*ld + t] from the frame-major I/Q spectrogram; with
    etot (the spectrogram's energy partials) also the delta error bound ed [s*ld + t]."""
    check(ctx.lib.msd_iq_band_delta_bound_dev(ctx.h, spec.ptr, _dp(etot), int(nstreams), int(max_frames), frames.ptr,
                                              int(nperseg), int(band[0]), int(band[1]), int(noise[0]), int(noise[1]),
                                              _dp(band_db), _dp(noise_db), _dp(delta), _dp(ed), int(ld)))


REFINE_DIRECT, REFINE_GOERTZEL_ROWS, REFINE_INT8_MFMA = 1, 2, 3


def iq_delta64_path(nperseg: int, hop: int, fs: float, band: tuple[int, int], noise: tuple[int, int],
                    dtype_code_iq: int) -> int:
    """the block step msd_iq_delta64_dev takes (REFINE_*; host only)"""
    rc = load().msd_iq_delta64_path(int(nperseg), int(hop), float(fs), int(band[0]), int(band[1]), int(noise[0]),
                                    int(noise[1]), int(dtype_code_iq))
    check(min(rc, 0))
    return rc


def iq_delta64_dev(ctx: Context, x, dtype_code_iq: int, n_samples: int, nperseg: int, hop: int, fs: float,
                   band: tuple[int, int], noise: tuple[int, int], ranges: np.ndarray, delta, ed, frame_sums=None):
    """float64 delta of the frames in ranges ([n][2] frame [first, end), frame t at sample t*hop of
    x) and its error bound, into delta[t] / ed[t] (device pointers); frame_sums: also each frame's
    (sum I, sum Q) as float64 pairs at frame_sums[2 t] (MsdError UNSUPPORTED, nothing launched, on a
    block step without sums)"""
    r = np.ascontiguousarray(ranges, dtype=np.int64).reshape(-1, 2)
    check(ctx.lib.msd_iq_delta64_sums_dev(ctx.h, _dp(x), int(dtype_code_iq), int(n_samples), int(nperseg), int(hop),
                                          float(fs), int(band[0]), int(band[1]), int(noise[0]), int(noise[1]),
                                          ptr(r), r.shape[0], _dp(delta), _dp(ed), _dp(frame_sums)))

"""WAV files → HBM → detections, overlapped.

``read(path)`` is the native counterpart of ``scipy.io.wavfile.read`` (dsp/src/main.py:249):
libmsdsp parses the RIFF chunks and preads the samples.  ``WavDay`` runs a list of
equal-format recordings (a day of one-minute files) through ``BatchPipeline`` in batches,
double-buffered: while the GPU processes batch i, reader threads decode batch i+1 straight
into page-locked host memory (the C calls release the GIL), the upload runs on the context's
copy stream, and a stream fence orders the next compute after it.  File start times come from
the reference's file-name conventions (``wav.start_datetime_from_name``) or are given.
"""
from __future__ import annotations

import ctypes as C
import datetime
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from . import _lib
from .batch import BatchPipeline

_DT = {_lib.MSD_U8: np.uint8, _lib.MSD_I16: np.int16, _lib.MSD_I32: np.int32, _lib.MSD_F32: np.float32,
       _lib.MSD_F64: np.float64}
_EPOCH = datetime.datetime(1970, 1, 1)


def probe(path) -> _lib.MsdWavInfo:
    info = _lib.MsdWavInfo()
    _lib.check(_lib.load().msd_wav_probe(str(path).encode(), C.byref(info)))
    return info


def read(path, channel: int | None = None):
    """(rate, data) like scipy.io.wavfile.read: [n] for mono, [n, channels] for several
    (channel=None), or one channel's [n]."""
    info = probe(path)
    dt = np.dtype(_DT[info.dtype])
    ch = -1 if channel is None else int(channel)
    nch = info.channels if ch < 0 else 1
    out = np.empty(info.frames * nch, dt)
    _lib.check(_lib.load().msd_wav_read(str(path).encode(), ch, 0, info.frames, _lib.ptr(out), out.nbytes,
                                        C.byref(info)))
    if nch > 1:
        out = out.reshape(-1, nch)
    return info.rate, out


class PinnedBuffer:
    """Page-locked host memory (hipHostMalloc) with a numpy view."""

    def __init__(self, ctx: _lib.Context, nbytes: int):
        self.ctx = ctx
        p = C.c_void_p()
        _lib.check(ctx.lib.msd_host_alloc(ctx.h, C.c_size_t(int(nbytes)), C.byref(p)))
        self.ptr, self.nbytes = p, int(nbytes)

    def view(self, dtype, count: int, byte_offset: int = 0) -> np.ndarray:
        buf = (C.c_char * (count * np.dtype(dtype).itemsize)).from_address(self.ptr.value + byte_offset)
        return np.frombuffer(buf, dtype=dtype, count=count)

    def free(self):
        if self.ptr:
            self.ctx.lib.msd_host_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class WavDay:
    """Detections for many equal-format WAV files, batched and double-buffered (see module doc).

    ``run()`` returns (per-file detections [start, stop, db] rows, hour histogram, timings)."""

    def __init__(self, ctx: _lib.Context, paths, batch_files: int = 120, start_times=None, base_time=None,
                 readers: int = 8, **pipeline_kwargs):
        self.ctx, self.paths = ctx, [str(p) for p in paths]
        if not self.paths:
            raise ValueError("no files")
        info = probe(self.paths[0])
        self.info = info
        self.fs, self.n = info.rate, int(info.frames)
        self.dtype = np.dtype(_DT[info.dtype])
        self.B = min(int(batch_files), len(self.paths))
        if start_times is None:
            from .wav import start_datetime_from_name
            start_times = [start_datetime_from_name(p) for p in self.paths]
        self.start_us = np.array([(t - _EPOCH) // datetime.timedelta(microseconds=1) for t in start_times], np.int64)
        base = base_time if base_time is not None else min(start_times).replace(minute=0, second=0, microsecond=0)
        self.base_us = (base - _EPOCH) // datetime.timedelta(microseconds=1)
        self.bp = BatchPipeline(ctx, self.B, self.n, self.fs, dtype=self.dtype, **pipeline_kwargs)
        es = self.dtype.itemsize
        self.slot_bytes = self.B * self.bp.n_pad * es
        self.d_x = [self.bp.d_x, ctx.alloc(self.slot_bytes)]
        self.d_st = [self.bp.d_start_us, ctx.alloc(self.B * 8)]
        self.h_x = [PinnedBuffer(ctx, self.slot_bytes) for _ in range(2)]
        self.h_st = [PinnedBuffer(ctx, self.B * 8) for _ in range(2)]
        self.pool = ThreadPoolExecutor(max_workers=max(1, int(readers)))
        self.bp.hist.base_us = int(self.base_us)

    def _read_batch(self, b: int, slot: int) -> int:
        """Decode batch b's files into pinned slot `slot`; returns the number of files."""
        lo = b * self.B
        paths = self.paths[lo:lo + self.B]
        es = self.dtype.itemsize
        lib = self.ctx.lib
        base = self.h_x[slot].ptr.value

        def one(i):
            info = _lib.MsdWavInfo()
            dst = C.c_void_p(base + i * self.bp.n_pad * es)
            _lib.check(lib.msd_wav_read(paths[i].encode(), 0, 0, self.n, dst, self.n * es, C.byref(info)))
            if info.frames != self.n or info.rate != self.fs or info.dtype != self.info.dtype:
                raise ValueError(f"{paths[i]}: format differs from the batch's first file")

        list(self.pool.map(one, range(len(paths))))
        st = self.h_st[slot].view(np.int64, self.B)
        st[:] = 0
        st[: len(paths)] = self.start_us[lo:lo + len(paths)]
        return len(paths)

    def _upload(self, slot: int):
        # the slot's previous batch (b - 2) has finished: run() downloaded its results before
        # enqueuing the next batch, so the copy needs no fence behind the compute stream
        lib, h = self.ctx.lib, self.ctx.h
        _lib.check(lib.msd_memcpy_h2d_async(h, self.d_x[slot].ptr, self.h_x[slot].ptr, C.c_size_t(self.slot_bytes)))
        _lib.check(lib.msd_memcpy_h2d_async(h, self.d_st[slot].ptr, self.h_st[slot].ptr, C.c_size_t(self.B * 8)))
        _lib.check(lib.msd_fence(h, 0))  # compute enqueued next waits for the upload

    def run(self):
        import time
        nbatch = (len(self.paths) + self.B - 1) // self.B
        t0 = time.perf_counter()
        r0 = time.perf_counter()
        nfiles = self._read_batch(0, 0)
        t_read = time.perf_counter() - r0
        self._upload(0)
        out = []
        for b in range(nbatch):
            slot = b % 2
            if nfiles < self.B:  # a short last batch: the slot's tail files get no samples
                lens = np.full(self.B, self.n, np.int64)
                lens[nfiles:] = 0
                nbs = np.where(lens > 0, self.bp.nb, 0).astype(np.int64)
                self.bp.d_len.upload(lens)
                self.bp.d_nb.upload(nbs)
            self.bp.run(x=self.d_x[slot], start_us=self.d_st[slot], clear_hist=(b == 0))
            nxt = 0
            if b + 1 < nbatch:
                _lib.check(self.ctx.lib.msd_copy_synchronize(self.ctx.h))  # the other pinned slot is free
                r0 = time.perf_counter()
                nxt = self._read_batch(b + 1, 1 - slot)  # overlaps batch b on the GPU
                t_read += time.perf_counter() - r0
                self._upload(1 - slot)
            dets, counts, status, _ = self.bp.detections()  # waits for batch b
            out.extend(dets[:nfiles])
            nfiles = nxt
        hist = self.bp.hour_counts()
        wall = time.perf_counter() - t0
        return out, hist, {"wall_s": wall, "read_s": t_read, "files": len(self.paths)}

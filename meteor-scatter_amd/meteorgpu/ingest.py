"""WAV files → HBM → detections, overlapped.

``read(path)`` is the native counterpart of ``scipy.io.wavfile.read`` (dsp/src/main.py:249):
libmsdsp parses the RIFF chunks and preads the samples.  ``WavDay`` runs a list of
equal-format recordings (a day of one-minute files) through ``BatchPipeline`` in batches,
triple-buffered: while the GPU uploads and processes batch i, reader threads decode the next
batches straight into page-locked host memory (the C calls release the GIL), the uploads run
back to back on the context's copy stream, and a stream fence orders each batch's compute
after its own upload.  File start times come from
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
    """Detections for many equal-format WAV files, batched and triple-buffered (see module doc).

    ``run()`` returns (per-file detections [start, stop, db] rows, hour histogram, timings).
    The pipeline keeps the copy engine busy: a background thread decodes batch b + 1 (and b + 2)
    into free page-locked slots while batch b uploads and computes, and the upload of b + 1 is
    enqueued before the host waits for b's detections, so consecutive uploads run back to back
    and the whole run is bound by PCIe."""

    SLOTS = 3  # pinned host + device batch buffers: one uploading, one decoding, one computing

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
        nbatch = (len(self.paths) + self.B - 1) // self.B
        self.S = min(self.SLOTS, max(1, nbatch))
        self.d_x = [self.bp.d_x] + [ctx.alloc(self.slot_bytes) for _ in range(self.S - 1)]
        self.d_st = [self.bp.d_start_us] + [ctx.alloc(self.B * 8) for _ in range(self.S - 1)]
        self.h_x = [PinnedBuffer(ctx, self.slot_bytes) for _ in range(self.S)]
        self.h_st = [PinnedBuffer(ctx, self.B * 8) for _ in range(self.S)]
        self.pool = ThreadPoolExecutor(max_workers=max(1, int(readers)))
        self.decoder = ThreadPoolExecutor(max_workers=1)  # one batch at a time, its files on `pool`
        self.bp.hist.base_us = int(self.base_us)
        # max |x| per file for the near-tie bound (margin.py): the format's full scale for integer
        # samples (a conservative bound, no pass over the samples), measured per file for float
        self.full_scale = ({np.uint8: 255.0, np.int16: 32768.0, np.int32: 2.0 ** 31}.get(self.dtype.type)
                           if self.dtype.kind in "iu" else None)
        self.xmax = [np.full(self.B, self.full_scale or 0.0) for _ in range(self.S)]
        self._short = False  # d_len / d_nb hold a short last batch's lengths

    def _read_batch(self, b: int, slot: int):
        """Decode batch b's files into pinned slot `slot` (no HIP calls: runs on the decoder
        thread); returns (number of files, seconds)."""
        import time
        r0 = time.perf_counter()
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
            if self.full_scale is None:
                x = self.h_x[slot].view(self.dtype, self.n, i * self.bp.n_pad * es)
                self.xmax[slot][i] = float(np.max(np.abs(x))) if self.n else 0.0

        futs = [self.pool.submit(one, i) for i in range(len(paths))]
        errs = [f.exception() for f in futs]  # every reader has stopped writing into the slot
        err = next((e for e in errs if e is not None), None)
        if err is not None:
            raise err
        st = self.h_st[slot].view(np.int64, self.B)
        st[:] = 0
        st[: len(paths)] = self.start_us[lo:lo + len(paths)]
        return len(paths), time.perf_counter() - r0

    def _upload(self, slot: int):
        # the slot's previous batch (b - S) has finished: run() downloaded its results before
        # its slot was decoded into again, so the copy needs no fence behind the compute stream
        lib, h = self.ctx.lib, self.ctx.h
        _lib.check(lib.msd_memcpy_h2d_async(h, self.d_x[slot].ptr, self.h_x[slot].ptr, C.c_size_t(self.slot_bytes)))
        _lib.check(lib.msd_memcpy_h2d_async(h, self.d_st[slot].ptr, self.h_st[slot].ptr, C.c_size_t(self.B * 8)))
        # compute enqueued from now on waits for this upload; compute already enqueued (batch
        # b - 1) does not, so uploading b never delays b - 1
        _lib.check(lib.msd_fence(h, 0))

    def _set_lengths(self, nfiles: int):
        if nfiles == self.B and not self._short:
            return
        lens = np.full(self.B, self.n, np.int64)
        lens[nfiles:] = 0  # a short last batch: the slot's tail files get no samples
        self.bp.d_len.upload(lens)
        self.bp.d_nb.upload(np.where(lens > 0, self.bp.nb, 0).astype(np.int64))
        self._short = nfiles < self.B

    def run(self):
        import time
        nbatch = (len(self.paths) + self.B - 1) // self.B
        S = self.S
        t0 = time.perf_counter()
        # decode ahead: batch b into slot b % S as soon as that slot's batch b - S has computed
        reads, sub = {}, [0]

        def feed(last):  # submit the decodes of batches up to `last`
            while sub[0] <= last and sub[0] < nbatch:
                reads[sub[0]] = self.decoder.submit(self._read_batch, sub[0], sub[0] % S)
                sub[0] += 1

        t_read = 0.0
        out = []
        try:
            feed(max(0, S - 2))
            nfiles, dt = reads.pop(0).result()
            t_read += dt
            self._upload(0)
            for b in range(nbatch):
                slot = b % S
                feed(b + S - 1)  # batch b + S - 1's slot held b - 1, whose detections were downloaded
                self._set_lengths(nfiles)
                self.bp.run(x=self.d_x[slot], start_us=self.d_st[slot], clear_hist=(b == 0))
                nxt = 0
                if b + 1 < nbatch:  # enqueue the next upload now: it runs right behind this one
                    nxt, dt = reads.pop(b + 1).result()
                    t_read += dt
                    self._upload((b + 1) % S)
                self.bp.xmax[:] = self.xmax[slot]
                dets, counts, status, _ = self.bp.detections()  # waits for batch b
                out.extend(dets[:nfiles])
                nfiles = nxt
        except BaseException:
            # a failed file (or an interrupt) leaves decodes in flight that write into the pinned
            # slots: let them finish before the error propagates and the slots can be freed
            for f in reads.values():
                f.cancel()
            for f in reads.values():
                if not f.cancelled():
                    try:
                        f.result()
                    except BaseException:
                        pass
            self.ctx.synchronize()
            raise
        hist = self.bp.hour_counts()
        wall = time.perf_counter() - t0
        return out, hist, {"wall_s": wall, "read_s": t_read, "files": len(self.paths)}

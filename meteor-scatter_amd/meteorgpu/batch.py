"""Device-resident batch pipeline: many equal-length recordings (e.g. the 1440
one-minute files of a day) processed by one launch per stage:

    STFT power spectrogram (a7)  ─┐
    block band dB / delta (a2/a3) ─┴─► detector (a4/a5) ─► detections + per-hour counts (a11)

HBM layout:
    x      int16  [nfiles][n_pad]            samples, n_pad = n rounded up to 8 (16-B rows)
    spec   f32    [nfiles][K][ld_t]          K = nperseg/2+1, ld_t = T rounded up to 32
    delta  f64    [nfiles][ld_b]             ld_b = blocks per file
    thr    f64    [nfiles][ld_b]             thresholds used per block (adaptive)
    dets   {i64 start, i64 stop, f64 db} [nfiles][cap]
    counts i64 [nfiles], margin f64 [nfiles], status i32 [nfiles], hist i64 [nbuckets]
Multi-GPU: each rank owns a contiguous range of files; the per-hour histogram is
summed across ranks with one RCCL all-reduce (``Communicator``).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .dsp import band_bins, hann_periodic, hanning_sym


class BatchPipeline:
    def __init__(self, ctx: _lib.Context, nfiles: int, n_per_file: int, fs: float, *,
                 nperseg: int = 1024, noverlap: int | None = None, block_duration_sec: float = 0.2,
                 freq_band=(950.0, 1050.0), noise_band=(650.0, 750.0), n_fft: int = 512,
                 threshold_std_factor: float = 4.0, flag_adaptive_threshold: bool = True,
                 threshold_estimation_window_sec: float = 120, threshold_freeze_before_detection_sec: float = 3,
                 threshold_freeze_after_detection_sec: float = 20, threshold_fixed_init_duration_sec: float = 10,
                 with_spectrogram: bool = True, nbuckets: int = 24, bucket_us: int = 3600 * 10 ** 6,
                 dtype=np.int16, concurrent: bool = False):
        self.ctx = ctx
        # concurrent: block_delta -> detect run on a second context's stream beside the STFT
        # (they only share the read-only samples); run() forks from and joins back into ctx.
        # Off by default: on MI355X the step is no faster (7.19-7.21 ms either way)
        # -- the persistent VALU-bound STFT leaves no idle issue slots for them to fill
        # the side context inherits ctx's options (MSD_OPT_*) and timing switch; the options that
        # matter to block_delta / detect are the timing switch (MSD_OPT_GENERIC_STFT and
        # MSD_OPT_FRESH_ALL only change the STFT and the stream detector)
        self.side = ctx.sibling() if concurrent and with_spectrogram else None
        self.stage_ctx = self.side if self.side is not None else ctx
        self.nfiles, self.n, self.fs = int(nfiles), int(n_per_file), float(fs)
        self.dtype = np.dtype(dtype)
        self.with_spectrogram = with_spectrogram
        es = self.dtype.itemsize
        self.n_pad = (self.n + 7) // 8 * 8
        # --- plans
        if noverlap is None:
            noverlap = nperseg // 2
        self.hop = nperseg - noverlap
        w = hann_periodic(nperseg).astype(np.complex64)
        scale = float(np.real(1.0 / (fs * (w * w).sum())))
        self.stft = _lib.StftPlan(ctx, nperseg, self.hop, w.real.astype(np.float32), scale)
        self.K = nperseg // 2 + 1
        self.T = self.stft.frames(self.n)
        self.ld_t = max(32, (self.T + 31) // 32 * 32)
        nfft = 2 * n_fft
        self.block_size = int(fs * block_duration_sec)
        self.block_sec = block_duration_sec
        L = min(self.block_size, nfft)
        self.band_bins, self.noise_bins = band_bins(nfft, fs, freq_band), band_bins(nfft, fs, noise_band)
        self.blocks = _lib.BlockPlan(self.stage_ctx, self.block_size, nfft, hanning_sym(self.block_size)[:L],
                                     self.band_bins, self.noise_bins)
        self.nfft, self.L, self.k_std = nfft, L, float(threshold_std_factor)
        self.xmax = np.zeros(self.nfiles)  # max |x| per file (near-tie bound, margin.py)
        self.nb = self.n // self.block_size
        self.ld_b = max(1, self.nb)
        bs = block_duration_sec
        self.cfg = _lib.det_cfg(flag_adaptive_threshold, threshold_std_factor,
                                int(threshold_estimation_window_sec / bs),
                                int(threshold_freeze_before_detection_sec / bs),
                                int(threshold_freeze_after_detection_sec / bs),
                                int(threshold_fixed_init_duration_sec / bs))
        self.cap = self.nb // 2 + 2
        # --- device buffers
        F = self.nfiles
        self.d_x = ctx.alloc(F * self.n_pad * es)
        self.d_off = ctx.alloc(F * 8)
        self.d_len = ctx.alloc(F * 8)
        self.d_nb = ctx.alloc(F * 8)
        self.d_spec = ctx.alloc(F * self.K * self.ld_t * 4) if with_spectrogram else None
        self.d_delta = ctx.alloc(F * self.ld_b * 8)
        self.d_band = ctx.alloc(F * self.ld_b * 8)   # band / noise dB per block: the near-tie bound
        self.d_noise = ctx.alloc(F * self.ld_b * 8)
        self.d_thr = ctx.alloc(F * self.ld_b * 8)
        self.d_dets = ctx.alloc(F * self.cap * _lib.DET_DTYPE.itemsize)
        self.d_counts = ctx.alloc(F * 8)
        self.d_margin = ctx.alloc(F * 8)
        self.d_status = ctx.alloc(F * 4)
        self.d_start_us = ctx.alloc(F * 8)
        self.nbuckets = int(nbuckets)
        self.d_hist = ctx.alloc(max(1, self.nbuckets) * 8)
        self.d_off.upload(np.arange(F, dtype=np.int64) * self.n_pad)
        self.d_len.upload(np.full(F, self.n, dtype=np.int64))
        self.d_nb.upload(np.full(F, self.nb, dtype=np.int64))
        self.d_start_us.upload(np.zeros(F, dtype=np.int64))
        self.hist = _lib.MsdHistCfg(self.d_start_us.ptr, 0, int(bucket_us), self.nbuckets, 0, float(bs),
                                    self.d_hist.ptr)

    # ------------------------------------------------------------------ inputs
    def upload_file(self, i: int, x: np.ndarray):
        x = np.ascontiguousarray(x, dtype=self.dtype)
        if x.shape != (self.n,):
            raise ValueError(f"file {i}: expected {self.n} samples")
        self.d_x.upload(x, byte_offset=i * self.n_pad * self.dtype.itemsize)
        self.xmax[i] = float(np.max(np.abs(x.astype(np.float64)))) if x.size else 0.0

    def set_start_times(self, file_start_us: np.ndarray, base_us: int):
        self.d_start_us.upload(np.ascontiguousarray(file_start_us, dtype=np.int64))
        self.hist.base_us = int(base_us)

    # ------------------------------------------------------------------ the step
    def run(self, x: _lib.DeviceBuffer | None = None, start_us: _lib.DeviceBuffer | None = None,
            clear_hist: bool = True):
        """Enqueue one pass over the batch (no host synchronisation).  ``x`` / ``start_us``:
        alternative device buffers of the same layout as ``d_x`` / ``d_start_us`` (double-buffered
        ingest); ``clear_hist=False`` accumulates the hour histogram across batches."""
        lib, h = self.ctx.lib, self.stage_ctx.h
        x = self.d_x if x is None else x
        self.hist.file_start_us = (self.d_start_us if start_us is None else start_us).ptr
        if self.side is not None:
            self.side.wait_for(self.ctx)  # fork: uploads and earlier readers of the outputs first
        if clear_hist:
            _lib.check(lib.msd_memset_dev(h, self.d_hist.ptr, 0, self.d_hist.nbytes))
        if self.with_spectrogram:
            self.stft.run_dev(x, self.dtype, self.d_off, self.d_len, self.nfiles, self.T, self.d_spec, self.ld_t)
        self.blocks.run_dev(x, self.dtype, self.d_off, self.d_len, self.nfiles, self.nb, self.d_band, self.d_noise,
                            self.d_delta, self.ld_b)
        _lib.check(lib.msd_detect_dev(h, self.d_delta.ptr, self.d_nb.ptr, self.nfiles, self.ld_b, self.cfg,
                                      self.d_dets.ptr, self.cap, self.d_counts.ptr, self.d_thr.ptr,
                                      self.d_margin.ptr, self.d_status.ptr, self.hist))
        if self.side is not None:
            self.ctx.wait_for(self.side)  # join: everything after run() on ctx sees the detections

    @property
    def contexts(self):
        return [self.ctx] if self.side is None else [self.ctx, self.side]

    # ------------------------------------------------------------------ outputs
    def spectrogram(self, i: int) -> np.ndarray:
        out = np.empty((self.K, self.ld_t), np.float32)
        self.d_spec.download(out, byte_offset=i * self.K * self.ld_t * 4)
        return out[:, : self.T]

    def delta(self) -> np.ndarray:
        out = np.empty((self.nfiles, self.ld_b), np.float64)
        self.d_delta.download(out)
        return out[:, : self.nb]

    def thresholds(self) -> np.ndarray:
        out = np.empty((self.nfiles, self.ld_b), np.float64)
        self.d_thr.download(out)
        return out[:, : self.nb]

    def detections(self):
        counts = np.empty(self.nfiles, np.int64)
        self.d_counts.download(counts)
        dets = np.empty((self.nfiles, self.cap), _lib.DET_DTYPE)
        self.d_dets.download(dets)
        status = np.empty(self.nfiles, np.int32)
        self.d_status.download(status)
        margin = np.empty(self.nfiles, np.float64)
        self.d_margin.download(margin)
        self._near_ties(margin)
        return [dets[i, : min(counts[i], self.cap)] for i in range(self.nfiles)], counts, status, margin

    def _near_ties(self, margin: np.ndarray):
        """Per file: the decision bound (margin.py) and whether min |delta - thr| is within it
        (``self.decision_bounds``, ``self.near_tie``); one NearTieWarning names the files."""
        from . import margin as M
        band = np.empty((self.nfiles, self.ld_b), np.float64)
        noise = np.empty((self.nfiles, self.ld_b), np.float64)
        self.d_band.download(band)
        self.d_noise.download(noise)
        win = hanning_sym(self.block_size)[: self.L]
        err = M.delta_error_bounds(band[:, : self.nb], noise[:, : self.nb], nfft=self.nfft, L=self.L, window=win,
                                   xmax=np.asarray(self.xmax, np.float64)[: self.nfiles], band=self.band_bins,
                                   noise=self.noise_bins)
        self.decision_bounds = M.decision_bounds(err, self.k_std)
        self.near_tie = np.isfinite(margin) & (margin <= self.decision_bounds)
        if self.near_tie.any():
            idx = np.nonzero(self.near_tie)[0]
            M.check(float(margin[idx[0]]), float(self.decision_bounds[idx[0]]),
                    f"{idx.size} file(s) (first: {int(idx[0])}): ")

    def hour_counts(self) -> np.ndarray:
        out = np.empty(max(1, self.nbuckets), np.int64)
        self.d_hist.download(out)
        return out[: self.nbuckets]

    def close(self):
        """Frees the plans and the device buffers (after the context's stream has drained)."""
        self.ctx.synchronize()
        for pl in (self.stft, self.blocks):
            pl.close()
        for b in (self.d_x, self.d_off, self.d_len, self.d_nb, self.d_spec, self.d_delta, self.d_band, self.d_noise,
                  self.d_thr, self.d_dets, self.d_counts, self.d_margin, self.d_status, self.d_start_us, self.d_hist):
            if b is not None:
                b.free()


class Communicator:
    """RCCL communicator over the ranks of one job (one process per GPU).  The
    128-byte unique id is created by rank 0 and distributed by the caller
    (meteorgpu.launch.Group shares it through a rendezvous file)."""

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        buf = C.create_string_buffer(_lib.COMM_ID_BYTES)
        _lib.check(_lib.load().msd_comm_get_unique_id(buf))
        return buf.raw

    def __init__(self, ctx: _lib.Context, nranks: int, uid: bytes, rank: int):
        import ctypes as C
        self.ctx = ctx
        h = C.c_void_p()
        buf = C.create_string_buffer(bytes(uid), _lib.COMM_ID_BYTES)
        _lib.check(ctx.lib.msd_comm_init(ctx.h, int(nranks), buf, int(rank), C.byref(h)))
        self.h = h

    def allreduce_i64(self, buf: _lib.DeviceBuffer, n: int):
        _lib.check(self.ctx.lib.msd_comm_allreduce_i64(self.h, buf.ptr, int(n)))

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.msd_comm_destroy(self.h)
            self.h = None

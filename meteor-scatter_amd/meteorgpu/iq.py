"""Complex (I/Q) spectrogram — BASELINE config C5 (192 kHz I/Q, 4096-point frames, 75 %
overlap), the SDR-native form of the reference's spectrogram call (dsp/src/main.py:52-54 /
:132-133 with complex input, where scipy switches to the two-sided spectrum).

``spectrogram_iq(i, q, fs, nperseg=4096, noverlap=3072)`` returns scipy's ``(f, t, Sxx)``
with ``Sxx`` float32 [N][T] in FFT bin order; the device keeps the frame-major [T][N] layout
(``IQBatch``), of which scipy's is the transpose.  No CPU fallback.

The detector over the I/Q stream (``proc_iq_samples``, ``IQShardDetector``) is the reference's
block detector (dsp/src/main.py:380-527) with the STFT frame as the block (block_sec = hop/fs):
per frame the band and noise energies of the two-sided spectrum (fftfreq masks, main.py:382-388
semantics) give ``delta = band_dB - noise_dB``, and the global / adaptive detector runs over the
whole stream — time-sharded over ranks by ``meteorgpu.stream``.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from . import stream as _stream
from .dsp import OutputDetection, _blocks, _utc, context, hann_periodic, write_csv


def _plan(ctx, fs, nperseg, noverlap):
    w = hann_periodic(nperseg).astype(np.complex64)      # scipy casts the window to complex64
    scale = float(np.real(1.0 / (fs * (w * w).sum())))
    return _lib.CStftPlan(ctx, nperseg, nperseg - noverlap, w.real.astype(np.float32), scale)


def interleave(i: np.ndarray, q: np.ndarray) -> tuple[np.ndarray, int]:
    """(I, Q) → interleaved buffer + libmsdsp dtype code (int16 pairs or float32 pairs)."""
    i, q = np.asarray(i), np.asarray(q)
    if i.shape != q.shape or i.ndim != 1:
        raise ValueError("I and Q must be 1-D arrays of the same length")
    if i.dtype == np.int16 and q.dtype == np.int16:
        out = np.empty(2 * i.size, np.int16)
        code = _lib.MSD_CI16
    else:
        out = np.empty(2 * i.size, np.float32)
        code = _lib.MSD_CF32
    out[0::2], out[1::2] = i, q
    return out, code


def spectrogram_iq(i, q, fs, nperseg=4096, noverlap=None, device: int = 0):
    """scipy.signal.spectrogram(i + 1j*q, fs, 'hann', nperseg, noverlap) → (f, t, Sxx[N][T])."""
    if noverlap is None:
        noverlap = nperseg // 8  # scipy's default
    buf, code = interleave(i, q)
    plan = _plan(context(device), fs, nperseg, noverlap)
    try:
        S = plan.run(buf, code)
    finally:
        plan.close()
    n = buf.size // 2
    f = np.fft.fftfreq(nperseg, 1 / fs)
    t = np.arange(nperseg / 2, n - nperseg / 2 + 1, nperseg - noverlap) / float(fs)
    return f, t, S.T


class IQBatch:
    """Streams of interleaved I/Q resident in HBM: one launch for all frames.
    HBM: x [nstreams][2 n_pad] elements, out float32 [nstreams][T][N] (frame-major)."""

    def __init__(self, ctx: _lib.Context, nstreams: int, n_per_stream: int, fs, nperseg=4096, noverlap=3072,
                 dtype=np.int16):
        self.ctx, self.ns, self.n = ctx, int(nstreams), int(n_per_stream)
        self.dtype = np.dtype(dtype)
        self.code = _lib.MSD_CI16 if self.dtype == np.int16 else _lib.MSD_CF32
        self.plan = _plan(ctx, fs, nperseg, noverlap)
        self.N = int(nperseg)
        self.T = self.plan.frames(self.n)
        self.n_pad = (self.n + 3) // 4 * 4
        es = self.dtype.itemsize
        self.d_x = ctx.alloc(self.ns * 2 * self.n_pad * es)
        self.d_off = ctx.alloc(self.ns * 8)
        self.d_len = ctx.alloc(self.ns * 8)
        self.d_off.upload(np.arange(self.ns, dtype=np.int64) * self.n_pad)
        self.d_len.upload(np.full(self.ns, self.n, np.int64))
        self.d_out = ctx.alloc(self.ns * max(self.T, 1) * self.N * 4)

    def upload(self, s: int, iq: np.ndarray, sample_offset: int = 0):
        """interleaved I/Q elements for stream s starting at complex sample `sample_offset`."""
        iq = np.ascontiguousarray(iq, dtype=self.dtype)
        self.d_x.upload(iq, byte_offset=(s * 2 * self.n_pad + 2 * sample_offset) * self.dtype.itemsize)

    def run(self, etot: _lib.DeviceBuffer | None = None, fsums: _lib.DeviceBuffer | None = None):
        """etot: also each frame's 16 energy partials (float32 [ns][T][16], the error bound's input);
        fsums: each frame's (sum I, sum Q) float64 already on the device (from the exact delta), so
        the spectrogram's detrend needs no sums of its own (msd_cstft_psd_fsums_dev)"""
        self.plan.run_dev(self.d_x, self.code, self.d_off, self.d_len, self.ns, self.T, self.d_out, etot, fsums)

    def close(self):
        self.plan.close()
        for b in (self.d_x, self.d_off, self.d_len, self.d_out):
            b.free()

    def frames(self, s: int, t0: int, nt: int) -> np.ndarray:
        out = np.empty((nt, self.N), np.float32)
        self.d_out.download(out, byte_offset=((s * self.T + t0) * self.N) * 4)
        return out


# ----------------------------------------------------------------- detector over the I/Q stream
def iq_band_bins(nperseg: int, fs: float, band) -> tuple[int, int]:
    """Signed bin range [lo, hi] of fftfreq(nperseg, 1/fs) selected by (f >= band[0]) & (f <= band[1])
    (main.py:382 mask semantics on the two-sided spectrum); (0, -1) if no bin falls in the band."""
    f = np.fft.fftfreq(nperseg, d=1 / fs)
    b = np.fft.fftfreq(nperseg, d=1.0 / nperseg).round().astype(np.int64)  # signed bin index
    sel = (f >= band[0]) & (f <= band[1])
    if not sel.any():
        return 0, -1
    lo, hi = int(b[sel].min()), int(b[sel].max())
    assert sel.sum() == hi - lo + 1
    return lo, hi


def frame_shard(n_samples: int, nperseg: int, hop: int, rank: int, world: int):
    """Frames [f0, f1) of an n-sample stream owned by `rank`, and the samples [s0, s1) they read."""
    from .shard import shard_range
    T = (n_samples - nperseg) // hop + 1 if n_samples >= nperseg else 0
    f0, f1 = shard_range(T, rank, world)
    return T, f0, f1, f0 * hop, ((f1 - 1) * hop + nperseg) if f1 > f0 else f0 * hop


# the refinement's interval bookkeeping lives with the certify-then-refine loop (stream.py)
from .stream import _NO_IV, _as_iv, _iv_len, _merge, _merge_a, _subtract, _subtract_a  # noqa: E402,F401


class IQShardDetector(_stream.CertifyingShard):
    """One rank's time shard of an I/Q stream on the GPU: spectrogram (frame-major, kept in HBM) →
    per-frame band delta written straight into the stream plan → detector over the whole stream.

    Certification (``certify``, on by default, as in proc_iq_samples / proc_iq_wav_file; the
    uncertified fast path is ``certify=False``).  For int16 input at C5's geometry the detector's
    delta is then float64-grade for EVERY frame (``delta="auto"`` -> exact: msd_iq_delta64_dev's
    exact integer DFT of each 1024-sample block on the matrix cores, ~1e-13 dB bound), so one
    certified pass settles every decision and the dB means are float64 as they stand.  Otherwise
    (``delta="fp32"``, float32 input, other geometries) the delta comes from the fp32 spectrogram:
    the spectrogram kernel also writes each frame's energy,
    the band delta kernel a bound on |delta - delta_ref| against the float64 reference (scipy's
    spectrogram of complex128 input), and every decision of the detector is checked against its
    bounds (include/msdsp.h, msd_stream_set_certify).  ``detect(exact_decisions=True)`` then
    recomputes in float64 (msd_iq_delta64_dev, from the samples) the delta of every frame an
    uncertain decision depends on -- the frame itself and the window its threshold comes from -- and
    runs the detector again, until no decision is uncertain (or only float64-level near ties are
    left, flagged as ``near_tie``).  The detections are then the float64 reference's.  Last, the
    frames of every detection are made float64 too (the same refinement) and the dB means
    (main.py:501-502, np.mean over delta[start:stop]) recomputed over them, so the CSV's dB column
    is the float64 reference's within the refinement's ~1e-12 dB bound, not the fp32 path's."""

    def __init__(self, ctx: _lib.Context, n_samples_total: int, fs, nperseg, noverlap, freq_band, noise_band,
                 threshold_std_factor=4.0, flag_adaptive_threshold=True, threshold_estimation_window_sec=120,
                 threshold_freeze_before_detection_sec=3, threshold_freeze_after_detection_sec=20,
                 threshold_fixed_init_duration_sec=10, rank: int = 0, world: int = 1, dtype=np.int16,
                 seg_len: int = 8192, chunk_frames: int | None = None, certify: bool = True,
                 delta: str = "auto", overlap: int = 0):
        """chunk_frames: keep only that many frames of spectrogram in HBM and stream the shard through
        it (``process_host``); the detector still sees the whole shard's delta.  A 24 h 192 kHz
        stream (66 GB of int16 I/Q, 265 GB of spectrogram) then runs on one GPU.
        delta: where the detector's per-frame delta comes from -- "fp32": the band sums of the fp32
        spectrogram (iq_band_delta); "exact": every frame in float64 from the samples
        (msd_iq_delta64_dev), the spectrogram then only the product output; "auto": exact when
        certifying int16 input whose geometry the exact integer DFT on the matrix cores covers
        (REFINE_INT8_MFMA: blocks of 1024 samples, <= 10 bins, no band at 0 Hz -- C5), else fp32.
        With the exact delta every frame's error bound is ~1e-13 dB, so certification settles every
        decision in one pass (no energy partials, no refinement, no second detector pass).
        overlap: n > 0 runs the stream detector beside the spectrogram: the spectrogram on a sibling
        context whose persistent grid leaves n workgroup slots free (MSD_OPT_CSTFT_RESERVE; its
        workgroups then draw chunks of frames from a guided schedule, so one that starts late because
        a detector kernel held its slot does not end the launch late), the detector on another sibling.
        With the exact delta the detector does not need the spectrogram, so after the delta (the
        caller's context) the two run side by side: the detector's latency-bound kernels and host
        round trips under the spectrogram.  The caller's context is not changed.  0: one stream,
        in order."""
        self.ctx, self.fs, self.N = ctx, fs, int(nperseg)
        self.hop = self.N - int(noverlap)
        self.block_sec = self.hop / fs
        self.T, self.f0, self.f1, self.s0, self.s1 = frame_shard(int(n_samples_total), self.N, self.hop, rank, world)
        self.band = iq_band_bins(self.N, fs, freq_band)
        self.noise = iq_band_bins(self.N, fs, noise_band)
        bs = self.block_sec
        self.adaptive = bool(flag_adaptive_threshold)
        self.k = float(threshold_std_factor)
        self.W = _blocks(threshold_estimation_window_sec, bs) if self.adaptive else 0
        self.F0 = _blocks(threshold_fixed_init_duration_sec, bs) if self.adaptive else 0
        Fa = _blocks(threshold_freeze_after_detection_sec, bs) if self.adaptive else 0
        Fb = _blocks(threshold_freeze_before_detection_sec, bs) if self.adaptive else 0
        nloc = self.f1 - self.f0
        self.chunk = int(chunk_frames) if chunk_frames and 0 < int(chunk_frames) < nloc else None
        nb = (self.chunk - 1) * self.hop + self.N if self.chunk else max(self.s1 - self.s0, 1)
        self.overlap = int(overlap)
        if self.overlap < 0:
            raise ValueError("overlap must be >= 0 (workgroup slots left to the detector)")
        self.sctx = self.dctx = ctx  # the spectrogram's and the detector's contexts
        self.plan = None
        self.batch = None
        try:
            if self.overlap > 0:
                self.sctx, self.dctx = ctx.sibling(), ctx.sibling()
                self.sctx.set_option(_lib.OPT_CSTFT_RESERVE, self.overlap)
            self._init(ctx, fs, noverlap, freq_band, noise_band, threshold_std_factor, nb, dtype, delta,
                       seg_len, certify, Fa, Fb)
        except BaseException:
            self.close()
            raise

    def _init(self, ctx, fs, noverlap, freq_band, noise_band, threshold_std_factor, nb, dtype, delta, seg_len,
              certify, Fa, Fb):
        self.batch = IQBatch(self.sctx, 1, nb, fs, self.N, noverlap, dtype)
        if delta not in ("auto", "fp32", "exact"):
            raise ValueError(f"delta must be 'auto', 'fp32' or 'exact', not {delta!r}")
        try:
            self.delta_path = _lib.iq_delta64_path(self.N, self.hop, fs, self.band, self.noise, self.batch.code)
        except _lib.MsdError:  # a geometry the float64 refinement does not cover (nperseg > 65536)
            self.delta_path = 0
        if delta == "exact" and not self.delta_path:
            raise ValueError("delta='exact': msd_iq_delta64_dev does not cover this geometry")
        self._delta_mode = delta
        self.exact_delta = False
        self.d_frames = ctx.alloc(8)
        self.d_frames.upload(np.array([self.batch.T if self.s1 > self.s0 else 0], np.int64))
        cfg = _lib.det_cfg(self.adaptive, self.k, self.W, Fb, Fa, self.F0)
        self.plan = _lib.StreamPlan(self.dctx, cfg, self.T, self.f0, self.f1 - self.f0, seg_len=seg_len)
        self.ops = _stream.DeviceStreamOps(self.plan)
        self.d_etot = None
        self.d_fsum = None  # exact delta: the frames' sample sums, shared with the spectrogram's detrend
        self._fsums_ok = True
        self.certify = False
        self.set_certify(certify)
        self.fs_ = float(fs)
        self._read = None      # the shard's sample source when chunked (refinement re-reads samples)
        self._refined = _NO_IV  # global frame ranges whose delta is float64 already (merged, (n, 2))

    def set_delta(self, mode: str):
        """the delta source ("auto", "fp32", "exact"; class docstring), from the next
        spectrogram_and_delta on"""
        if mode not in ("auto", "fp32", "exact"):
            raise ValueError(f"delta must be 'auto', 'fp32' or 'exact', not {mode!r}")
        if mode == "exact" and not self.delta_path:
            raise ValueError("delta='exact': msd_iq_delta64_dev does not cover this geometry")
        self._delta_mode = mode
        self.exact_delta = mode == "exact" or (mode == "auto" and self.certify and
                                               self.delta_path == _lib.REFINE_INT8_MFMA)
        if self.certify and not self.exact_delta and self.d_etot is None:
            self.d_etot = self.ctx.alloc(16 * 4 * self.ctx.lib.msd_cstft_energy_stride(1, max(self.batch.T, 1)))
        if self.exact_delta and self.d_fsum is None:
            self.d_fsum = self.ctx.alloc(16 * max(self.batch.T, 1))

    def set_certify(self, on: bool):
        """certification on / off (takes effect at the next spectrogram_and_delta)"""
        self.certify = bool(on)
        self.plan.set_certify(self.certify)
        self.set_delta(self._delta_mode)  # "auto" follows certification

    def upload(self, iq: np.ndarray, sample_offset: int = 0):
        """interleaved I/Q of this shard's samples, starting at shard sample `sample_offset`"""
        self.batch.upload(0, iq, sample_offset)

    def spectrogram_and_delta(self):
        """async: spectrogram of the shard and its per-frame band delta (into the stream plan)"""
        self._refined = _NO_IV
        self._step_start()
        if self.f1 > self.f0:
            if self.exact_delta:
                # the exact delta first (full chip): the detector (dctx) then runs beside the spectrogram
                # (the delta on the spectrogram's own stream instead, in order behind the previous
                # step's spectrogram, measured 12.55-12.71 against 11.77-11.80 ms per step:
                # profiles/r5_c5_delta_stream_ab.txt)
                self._delta_exact(self.batch.n, self.f1 - self.f0, 0)
                self._after(self.dctx, self.ctx)
                self._after(self.sctx, self.ctx)
                self.batch.run(fsums=self._fsums())
            else:
                etot = self.d_etot if self.certify else None
                self._after(self.sctx, self.ctx)
                self.batch.run(etot)
                _lib.iq_band_delta_dev(self.sctx, self.batch.d_out, 1, self.batch.T, self.d_frames, self.N, self.band,
                                       self.noise, self.plan.d_delta, self.batch.T, etot=etot,
                                       ed=self.plan.d_ed if self.certify else None)
                self._after(self.dctx, self.sctx)
        if self.exact_delta:
            self._refined = np.array([[0, self.T]], np.int64)  # every rank's frames are float64 (the ranks agree on this list)

    @staticmethod
    def _after(a: _lib.Context, b: _lib.Context):
        """work enqueued on a from now on waits for b's so far (nothing when they share a stream)"""
        if a is not b:
            a.wait_for(b)

    def _step_start(self):
        """a new step on the caller's context (uploads, the delta) waits for the previous step's
        spectrogram (it reads the samples and the frame sums) and detector (it reads the delta)"""
        self._after(self.ctx, self.sctx)
        self._after(self.ctx, self.dctx)

    def _fsums(self):
        return self.d_fsum if self._fsums_ok else None

    def _delta_exact(self, n_samples: int, nframes: int, c0: int, ctx: _lib.Context | None = None):
        """float64 delta and bound of the local frames [c0, c0 + nframes), whose samples start at the
        batch buffer's first sample (frame c0 + j at sample j * hop); with them the frames' sample sums
        (batch-local frame j) for the spectrogram's detrend, where the block step carries them.  On
        ctx's stream (default: the caller's context)"""
        args = (ctx or self.ctx, self.batch.d_x, self.batch.code, n_samples, self.N, self.hop, self.fs_, self.band,
                self.noise, np.array([[0, nframes]], np.int64), _lib.C.c_void_p(self.plan.d_delta.value + 8 * c0),
                _lib.C.c_void_p(self.plan.d_ed.value + 8 * c0))
        if self._fsums_ok:
            try:
                _lib.iq_delta64_dev(*args, frame_sums=self.d_fsum)
                return
            except _lib.MsdError as e:
                if e.code != _lib.MSD_ERR_UNSUPPORTED:
                    raise
                self._fsums_ok = False  # no sums on this block step: the spectrogram sums itself
        _lib.iq_delta64_dev(*args)

    def process_host(self, iq_shard: np.ndarray):
        """interleaved I/Q of the shard's samples [s0, s1) on the host → the shard's delta in the
        stream plan, `chunk_frames` frames at a time (or all at once without chunking)"""
        iq_shard = np.ascontiguousarray(iq_shard)
        self.process_source(lambda a, b: iq_shard[2 * a: 2 * b])

    def process_source(self, read):
        """as process_host, with the samples pulled chunk by chunk: read(a, b) returns the
        interleaved I/Q of shard samples [a, b) (relative to s0), so a recording longer than host
        memory streams from its source (a file, an SDR ring) through HBM"""
        nloc = self.f1 - self.f0
        if not self.chunk:
            if nloc > 0:
                self.upload(np.ascontiguousarray(read(0, self.s1 - self.s0)))
            self.spectrogram_and_delta()
            return
        self._read = read
        self._refined = _NO_IV
        for c0 in range(0, nloc, self.chunk):
            nf = min(self.chunk, nloc - c0)
            a = c0 * self.hop
            b = a + (nf - 1) * self.hop + self.N
            self.sctx.synchronize()  # the previous chunk's spectrogram has read the batch buffer
            self.batch.upload(0, np.ascontiguousarray(read(a, b)))
            if self.exact_delta:
                self._after(self.ctx, self.sctx)
                self._delta_exact(b - a, nf, c0)
                # frames past nf read stale samples (and sums); the spectrogram is the product
                self._after(self.sctx, self.ctx)
                self.batch.run(fsums=self._fsums())
                continue
            self.d_frames.upload(np.array([nf], np.int64))
            etot = self.d_etot if self.certify else None
            self.batch.run(etot)  # frames past nf read stale samples; their powers are not used
            ed = _lib.C.c_void_p(self.plan.d_ed.value + 8 * c0) if self.certify else None
            _lib.iq_band_delta_dev(self.sctx, self.batch.d_out, 1, self.batch.T, self.d_frames, self.N, self.band,
                                   self.noise, _lib.C.c_void_p(self.plan.d_delta.value + 8 * c0), self.batch.T,
                                   etot=etot, ed=ed)
        self._after(self.dctx, self.ctx)
        self._after(self.dctx, self.sctx)
        if self.exact_delta:
            self._refined = np.array([[0, self.T]], np.int64)

    def _refine_local(self, ranges):
        """float64 delta (and its bound) of this rank's frames in the global ranges, from the samples"""
        r = _as_iv(ranges)
        r = np.stack([np.maximum(r[:, 0], self.f0), np.minimum(r[:, 1], self.f1)], 1) - self.f0
        loc = r[r[:, 1] > r[:, 0]]
        if not len(loc):
            return
        if not self.chunk:  # the shard's samples are resident: frame j at sample j * hop
            _lib.iq_delta64_dev(self.dctx, self.batch.d_x, self.batch.code, self.batch.n, self.N, self.hop, self.fs_,
                                self.band, self.noise, np.array(loc, np.int64), self.plan.d_delta, self.plan.d_ed)
            return
        # chunked: re-read each range's samples (<= chunk frames at a time) into the batch buffer
        for a, b in loc:
            for c in range(a, b, self.chunk):
                e = min(b, c + self.chunk)
                s0, s1 = c * self.hop, (e - 1) * self.hop + self.N
                self.synchronize()  # every kernel reading the batch buffer (both contexts) has finished
                self.batch.upload(0, np.ascontiguousarray(self._read(s0, s1)))
                _lib.iq_delta64_dev(self.dctx, self.batch.d_x, self.batch.code, s1 - s0, self.N, self.hop, self.fs_,
                                    self.band, self.noise, np.array([[0, e - c]], np.int64),
                                    _lib.C.c_void_p(self.plan.d_delta.value + 8 * c),
                                    _lib.C.c_void_p(self.plan.d_ed.value + 8 * c))

    def synchronize(self):
        """every context's work (delta, spectrogram and detector) finished"""
        self.ctx.synchronize()
        for c in (self.sctx, self.dctx):
            if c is not self.ctx:
                c.synchronize()

    def close(self):
        """frees the plans and buffers and the CU-split sibling contexts (the caller's context is
        left as it was); safe on a partly constructed detector"""
        self.synchronize()
        if self.plan is not None:
            self.plan.close()
            self.plan = None
        if self.batch is not None:
            self.batch.close()
            self.batch = None
        for name in ("d_etot", "d_fsum"):
            buf = getattr(self, name, None)
            if buf is not None:
                buf.free()
                setattr(self, name, None)
        for c in (self.sctx, self.dctx):
            if c is not self.ctx:
                c.close()
        self.sctx = self.dctx = self.ctx


def proc_iq_samples(i, q, fs, freq_band, noise_band, nperseg=4096, noverlap=3072, threshold_std_factor=4.0,
                    flag_adaptive_threshold=True, threshold_estimation_window_sec=120,
                    threshold_freeze_before_detection_sec=3, threshold_freeze_after_detection_sec=20,
                    threshold_fixed_init_duration_sec=10, wav_start_date_time=None, out_csv_file=None,
                    device: int = 0, chunk_sec: float | None = None, exact_decisions: bool = True,
                    certify: bool = True, delta: str = "auto"):
    """The batch detector of dsp/src/main.py (:380-527, :640-658) over an I/Q recording with the STFT
    frame as the block.  Returns (detections [OutputDetection], thresholds, delta, result).
    chunk_sec: stream the spectrogram through HBM in chunks of that many seconds (long recordings).
    certify / exact_decisions: every detector decision certified against the float64 reference, the
    uncertain ones recomputed in float64 (IQShardDetector); result.certified / near_tie /
    decision_bound / refined_delta_frames report it.  certify=False is the uncertified fast path.
    delta: IQShardDetector's delta source ("auto": the exact float64 delta of every frame for int16
    C5-like geometries, else the fp32 spectrogram's band sums with certification and refinement)."""
    buf, code = interleave(i, q)
    n = buf.size // 2
    det = IQShardDetector(context(device), n, fs, nperseg, noverlap, freq_band, noise_band, threshold_std_factor,
                          flag_adaptive_threshold, threshold_estimation_window_sec,
                          threshold_freeze_before_detection_sec, threshold_freeze_after_detection_sec,
                          threshold_fixed_init_duration_sec, dtype=buf.dtype,
                          chunk_frames=int(chunk_sec * fs / (nperseg - noverlap)) if chunk_sec else None,
                          certify=certify, delta=delta)
    try:
        det.process_host(buf[2 * det.s0: 2 * det.s1])
        res = det.detect(exact_decisions=exact_decisions)
        delta = det.plan.delta()
    finally:
        det.close()
    bs = det.block_sec
    out = []
    for d in res.detections:
        t_start, t_stop = int(d["start"]) * bs, int(d["stop"]) * bs
        out.append(OutputDetection(t_start=t_start, t_stop=t_stop, dur_s=t_stop - t_start, dB=np.float64(d["db"]),
                                   utc_start=_utc(wav_start_date_time, t_start),
                                   utc_stop=_utc(wav_start_date_time, t_stop)))
    if out_csv_file is not None:
        write_csv(out, out_csv_file)
    thr = [np.float64(v) for v in res.thresholds] if det.adaptive else np.float64(res.thr0)
    return out, thr, delta, res


def proc_iq_wav_file(file_path, freq_band, noise_band, nperseg=4096, noverlap=3072, threshold_std_factor=4.0,
                     flag_adaptive_threshold=True, threshold_estimation_window_sec=120,
                     threshold_freeze_before_detection_sec=3, threshold_freeze_after_detection_sec=20,
                     threshold_fixed_init_duration_sec=10, wav_start_date_time=None, out_csv_file=None,
                     device: int = 0, chunk_sec: float | None = None):
    """proc_iq_samples on a 2-channel (I, Q) WAV recording, read by the native reader (the SDR's
    I/Q recording; dsp/src/main.py:249-268 reads the demodulated mono audio instead).  Returns
    (detections, thresholds, delta, result) and writes the reference's CSV if asked."""
    import os
    from . import ingest
    assert os.path.isfile(file_path), f"File {file_path} does not exist"
    info = ingest.probe(file_path)
    assert info.channels == 2, "Only 2-channel (I, Q) WAV files are supported"
    fs, data = ingest.read(file_path)
    return proc_iq_samples(data[:, 0], data[:, 1], fs, freq_band, noise_band, nperseg, noverlap,
                           threshold_std_factor, flag_adaptive_threshold, threshold_estimation_window_sec,
                           threshold_freeze_before_detection_sec, threshold_freeze_after_detection_sec,
                           threshold_fixed_init_duration_sec, wav_start_date_time, out_csv_file, device, chunk_sec)

"""Complex (I/Q) spectrogram — BASELINE config C5 (192 kHz I/Q, 4096-point frames, 75 %
overlap), the SDR-native form of the reference's spectrogram call (dsp/src/main.py:52-54 /
:132-133 with complex input, where scipy switches to the two-sided spectrum).

``spectrogram_iq(i, q, fs, nperseg=4096, noverlap=3072)`` returns scipy's ``(f, t, Sxx)``
with ``Sxx`` float32 [N][T] in FFT bin order; the device keeps the frame-major [T][N] layout
(``IQBatch``), of which scipy's is the transpose.  No CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .dsp import context, hann_periodic


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

    def run(self):
        self.plan.run_dev(self.d_x, self.code, self.d_off, self.d_len, self.ns, self.T, self.d_out)

    def frames(self, s: int, t0: int, nt: int) -> np.ndarray:
        out = np.empty((nt, self.N), np.float32)
        self.d_out.download(out, byte_offset=((s * self.T + t0) * self.N) * 4)
        return out

"""Legacy pipeline pieces: the spectrogram and noise floor of
meteor_detect_class/prime_detection.py:65-91, on the GPU.

``specgram`` mirrors ``matplotlib.mlab.specgram`` (what ``plt.specgram`` computes) for a
real 1-D signal: symmetric Hann (``window_hanning``), no detrend, one-sided PSD with the
DC / Nyquist rows undoubled, ``/Fs/sum(w**2)``, zero padding to NFFT for a signal shorter than
NFFT — on libmsdsp's float64 STFT (``stft_any.hip``), the precision mlab computes in
(mlab.py:299-356); agreement with mlab is at the 1e-12 level (tested).
``noise_floor`` adds the band power over the noise band's rows and all frames
(``np.sum(Pxx[noise_band])``, a device reduction) and the reference's colour floor
``vmin = 10*log10(band_power/bandwidth) / (40/23) + C_MS_SPEC_CUT_FACTOR``.

Out of scope: the JPEG rendering and the ORB / DBSCAN burst clustering that follow in the
reference (image processing, not this data path).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .dsp import context, hanning_sym

C_MS_SPEC_CUT_FACTOR = 12  # prime_detection.py:22


def _freqs_times(n: int, NFFT: int, Fs: float, noverlap: int):
    """mlab._spectral_helper's frequency and time axes (onesided, even or odd pad_to = NFFT)."""
    num = NFFT // 2 + 1 if NFFT % 2 == 0 else (NFFT + 1) // 2
    freqs = np.fft.fftfreq(NFFT, 1 / Fs)[:num]
    if not NFFT % 2:
        freqs[-1] *= -1  # "get the last value correctly, it is negative otherwise"
    t = np.arange(NFFT / 2, n - NFFT / 2 + 1, NFFT - noverlap) / Fs
    return freqs, t


class SpecgramPlan:
    """mlab.specgram(x, NFFT, Fs, noverlap) for signals of one length, resident on the device."""

    def __init__(self, n: int, NFFT: int = 256, Fs: float = 2, noverlap: int = 128, dtype=np.int16,
                 device: int = 0):
        NFFT = int(NFFT)
        if NFFT < 16 or NFFT > 16384 or NFFT & (NFFT - 1):
            raise NotImplementedError("NFFT must be a power of two in [16, 16384]")
        if not 0 <= noverlap < NFFT:
            raise ValueError("noverlap must be less than NFFT")
        self.ctx = context(device)
        self.n, self.NFFT, self.Fs, self.noverlap = int(n), NFFT, float(Fs), int(noverlap)
        self.dtype = np.dtype(dtype)
        # mlab._spectral_helper: a signal shorter than NFFT is zero-padded to NFFT (one frame)
        self.n_dev = max(self.n, NFFT)
        w = hanning_sym(NFFT)                   # window_hanning(np.ones(NFFT)) = np.hanning(NFFT)
        scale = 1.0 / (Fs * (w ** 2).sum())     # result /= Fs; result /= (window**2).sum()
        self.plan = _lib.StftPlan(self.ctx, NFFT, NFFT - noverlap, w, scale, nfft=NFFT, precision=np.float64)
        self.plan.set_detrend(False)            # mlab default detrend_none
        self.K = NFFT // 2 + 1
        self.T = self.plan.frames(self.n_dev)
        self.ld = max(32, (self.T + 31) // 32 * 32)
        self.freqs, self.t = _freqs_times(self.n_dev, NFFT, Fs, noverlap)
        es = self.dtype.itemsize
        self.d_x = self.ctx.alloc((self.n_dev + 7) // 8 * 8 * es)
        self.d_x.memset(0)
        self.d_off = self.ctx.alloc(8)
        self.d_len = self.ctx.alloc(8)
        self.d_off.upload(np.zeros(1, np.int64))
        self.d_len.upload(np.array([self.n_dev], np.int64))
        self.d_spec = self.ctx.alloc(self.K * self.ld * 8)
        self.d_sum = self.ctx.alloc(8)

    def run(self, x: np.ndarray):
        x = np.ascontiguousarray(x, dtype=self.dtype)
        if x.shape != (self.n,):
            raise ValueError("signal length differs from the plan's")
        self.d_x.upload(x)  # the zero tail up to NFFT (short signals) was set at construction
        self.plan.run_dev(self.d_x, self.dtype, self.d_off, self.d_len, 1, self.T, self.d_spec, self.ld)

    def spectrogram(self) -> np.ndarray:
        out = np.empty((self.K, self.ld), np.float64)
        self.d_spec.download(out)
        return out[:, : self.T]

    def band_power(self, lo_hz: float, hi_hz: float) -> tuple[float, int]:
        """(np.sum(Pxx[(freqs >= lo) & (freqs <= hi)]), number of bins) on the device."""
        idx = np.nonzero((self.freqs >= lo_hz) & (self.freqs <= hi_hz))[0]
        if idx.size == 0:
            return 0.0, 0
        assert idx[-1] - idx[0] + 1 == idx.size
        _lib.check(self.ctx.lib.msd_spec_band_sum_f64_dev(self.ctx.h, self.d_spec.ptr, 1, self.K, self.T, self.ld,
                                                          int(idx[0]), int(idx[-1]), self.d_sum.ptr))
        s = np.empty(1, np.float64)
        self.d_sum.download(s)
        return float(s[0]), int(idx.size)


def specgram(x, NFFT=None, Fs=None, noverlap=None, device: int = 0):
    """matplotlib.mlab.specgram(x, NFFT, Fs, noverlap) defaults (window_hanning, detrend_none,
    one-sided psd, scale_by_freq): returns (spec float64 [NFFT//2+1, T], freqs, t)."""
    x = np.asarray(x)
    if x.ndim != 1:
        raise NotImplementedError("only 1-D real signals are implemented")
    NFFT = 256 if NFFT is None else int(NFFT)
    Fs = 2 if Fs is None else Fs
    noverlap = 128 if noverlap is None else int(noverlap)
    dt = x.dtype if x.dtype in (np.int16, np.int32, np.uint8, np.float32, np.float64) else np.float64
    p = SpecgramPlan(len(x), NFFT, Fs, noverlap, dtype=dt, device=device)
    p.run(x.astype(dt, copy=False))
    return p.spectrogram(), p.freqs, p.t


def noise_floor(x, fs, NFFT=2048, lower_freq=250, upper_freq=800, cut_factor=C_MS_SPEC_CUT_FACTOR, device: int = 0):
    """prime_detection.py:65-91 without the figure: returns (Pxx, freqs, bins, vmin,
    power_density_db_hz) for ``plt.specgram(x, Fs=fs, NFFT=NFFT, noverlap=NFFT // 2)``."""
    x = np.asarray(x)
    dt = x.dtype if x.dtype in (np.int16, np.int32, np.uint8, np.float32, np.float64) else np.float64
    p = SpecgramPlan(len(x), NFFT, fs, NFFT // 2, dtype=dt, device=device)
    p.run(x.astype(dt, copy=False))
    band_power, nbins = p.band_power(lower_freq, upper_freq)
    delta_f = fs / NFFT
    bandwidth = nbins * delta_f
    with np.errstate(divide="ignore", invalid="ignore"):
        pddb = 10 * np.log10(band_power / bandwidth)
    factor = 40 / 23
    vmin = pddb / factor + cut_factor
    return p.spectrogram(), p.freqs, p.t, float(vmin), float(pddb)


# ------------------------------------------------------------------ §8(f) legacy drop-in shim
def detect_and_cluster_bursts_audio(segment, fs, freq_band=(950.0, 1050.0), noise_band=(650.0, 750.0),
                                    n_fft=1024, block_duration_sec=0.1, threshold_std_factor=4.0,
                                    critical_min_dur_s=0.5, device: int = 0):
    """Audio-fed stand-in for ``detect_and_cluster_bursts(image_path, ...)``
    (meteor_detect_class/detector_and_classification.py:7-91) with its return shape
    ``(bursts, unique_labels, burst_positions, critical_bursts, non_critical_bursts)``, so the
    hourly loop of prime_detection.py:208-252 runs unchanged.  Bursts are the GPU block
    detector's detections on the segment (adaptive threshold, main.py:450-522); a burst is
    critical when it lasts >= 0.5 s, the duration rule of detector_and_classification.py:50
    (``duration >= 5`` pixels ≈ 0.5 s).  The counts are not those of the reference's ORB /
    DBSCAN image clustering (a different algorithm); only the interface and the hourly CSV
    format are compatible."""
    from .dsp import process_samples
    x = np.asarray(segment)
    if x.ndim == 2:
        x = x[:, 0]  # prime_detection.py:70 uses iq_segment[:, 0]
    res = process_samples(x, fs, block_duration_sec, freq_band, noise_band, n_fft, threshold_std_factor,
                          flag_adaptive_threshold=True, device=device)
    bursts = list(res.detections)
    labels = set(range(len(bursts)))
    positions = [(d.t_start, d.t_stop) for d in bursts]
    critical = [i for i, d in enumerate(bursts) if d.dur_s >= critical_min_dur_s]
    non_critical = [i for i, d in enumerate(bursts) if d.dur_s < critical_min_dur_s]
    return bursts, labels, positions, critical, non_critical


HOURLY_COLUMNS = ("Timestamp", "Anzahl", "Kritisch")  # prime_detection.py:138


def append_hourly_row(file_name, start_time, n_critical: int, n_non_critical: int) -> None:
    """prime_detection.py:229-245: append ``start_time;total;critical`` to the day's
    ``;``-separated CSV (header ``Timestamp;Anzahl;Kritisch``, created if missing — :139-146)."""
    import os
    new = not os.path.exists(file_name)
    with open(file_name, "a", newline="") as fh:
        if new:
            fh.write(";".join(HOURLY_COLUMNS) + "\n")
        fh.write(f"{start_time.strftime('%Y-%m-%d %H:%M:%S')};{n_critical + n_non_critical};{n_critical}\n")

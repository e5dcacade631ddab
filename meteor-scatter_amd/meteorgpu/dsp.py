"""Drop-in for the reference's batch detector, dsp/src/main.py.

``proc_wav_file`` keeps the reference's signature, argument meaning, prints,
assertion messages and outputs (detection CSV, Audacity labels); the numeric
work runs on the GPU through libmsdsp (no CPU fallback).  Lower-level pieces:

* ``block_powers``  — main.py:352-393  (block framing, Hann, rFFT crop, band dB, delta)
* ``get_detections`` / ``get_detections_adaptive`` — main.py:396-448 / 450-522
* ``spectrogram``   — scipy.signal.spectrogram as called at main.py:52-54, :132-133
* ``write_csv`` / ``write_audacity_labels`` — main.py:640-658 / 630-638
* ``count_per_hour`` — main.py:687-696 (Counter over utc_start hours)

The reference's figures are drawn from GPU arrays with matplotlib / plotly (``figures.py``):
the per-detection spectrogram + PSD export (``disable_show_and_write=False``,
main.py:721-806) and the debug figures ``debug_plot_whole`` (main.py:278-306),
``debug_plot_config`` (:324-350), ``debug_plot_output`` (:531-565, :660-716) and
``debug_plot_output_interactive`` (:567-624).  They are shown as in the reference; the
keyword-only ``figure_dir`` also saves them (headless runs).
"""
from __future__ import annotations

import csv
import datetime
import os
from collections import Counter
from dataclasses import dataclass, field

import numpy as np

from . import _lib, wav
from . import margin as margin_mod


@dataclass
class OutputDetection:
    """dsp/src/main.py:30-37."""
    t_start: float
    t_stop: float
    dur_s: float
    dB: float
    utc_start: datetime.datetime = None
    utc_stop: datetime.datetime = None


@dataclass
class ProcResult:
    """What proc_wav_file computed (the reference returns None; this is a superset)."""
    detections: list
    thresholds: object  # float (global) or list of float (adaptive)
    band_power: np.ndarray
    noise_power: np.ndarray
    delta_power: np.ndarray
    block_size: int
    num_blocks: int
    min_margin: float = field(default=float("nan"))
    # near-tie guard (margin.py): |delta - thr| at or below decision_bound can flip a decision
    # against the float64 numpy reference; near_tie says whether min_margin is that close
    decision_bound: float = field(default=float("nan"))
    near_tie: bool = False


_CTX: dict[int, _lib.Context] = {}


def context(device: int = 0) -> _lib.Context:
    """Process-wide context per device (created on first use)."""
    ctx = _CTX.get(device)
    if ctx is None:
        ctx = _CTX[device] = _lib.Context(device)
    return ctx


# --------------------------------------------------------------------------- windows / bins
def hanning_sym(m: int) -> np.ndarray:
    """np.hanning(m) (numpy/lib/_function_base_impl.py:3356-3364), float64."""
    if m < 1:
        return np.array([], dtype=np.float64)
    if m == 1:
        return np.ones(1, dtype=np.float64)
    n = np.arange(1 - m, m, 2)
    return 0.5 + 0.5 * np.cos(np.pi * n / (m - 1))


def hann_periodic(m: int) -> np.ndarray:
    """scipy.signal.get_window('hann', m) (fftbins=True): general_cosine(m+1, [.5,.5])[:-1]."""
    if m <= 1:
        return np.ones(max(m, 0), dtype=np.float64)
    fac = np.linspace(-np.pi, np.pi, m + 1)
    w = np.zeros(m + 1)
    for k, a in enumerate((0.5, 0.5)):
        w += a * np.cos(k * fac)
    return w[:-1]


def band_bins(n_fft: int, fs: float, band) -> tuple[int, int]:
    """Inclusive bin range selected by (freqs >= lo) & (freqs <= hi), freqs = rfftfreq(n_fft, 1/fs)
    (main.py:363, :382, :386).  Returns (0, -1) for an empty band."""
    freqs = np.fft.rfftfreq(n_fft, d=1 / fs)
    idx = np.nonzero((freqs >= band[0]) & (freqs <= band[1]))[0]
    if idx.size == 0:
        return 0, -1
    lo, hi = int(idx[0]), int(idx[-1])
    assert hi - lo + 1 == idx.size  # rfftfreq is monotone: the mask is one run
    return lo, hi


# --------------------------------------------------------------------------- a2/a3
def block_powers(wav_data: np.ndarray, fs: float, block_duration_sec: float, freq_band, noise_band, n_fft: int,
                 device: int = 0):
    """main.py:352-393 on the GPU.  ``n_fft`` is the reference's argument (doubled inside,
    main.py:353).  Returns (band_power, noise_power, delta_power, block_size) as float64."""
    nfft = int(n_fft) * 2
    block_size = int(fs * block_duration_sec)
    if block_size <= 0:
        raise ZeroDivisionError("integer division or modulo by zero")
    L = min(block_size, nfft)
    win = hanning_sym(block_size)[:L]
    plan = _lib.BlockPlan(context(device), block_size, nfft, win, band_bins(nfft, fs, freq_band),
                          band_bins(nfft, fs, noise_band))
    try:
        band, noise, delta = plan.run(np.ascontiguousarray(wav_data))
    finally:
        plan.close()
    return band, noise, delta, block_size


# --------------------------------------------------------------------------- a4/a5
def _blocks(sec: float, block_duration_sec: float) -> int:
    return int(sec / block_duration_sec)  # main.py:458-461


def _utc(wav_start_date_time, t):
    if wav_start_date_time is None:
        return None
    return wav_start_date_time + datetime.timedelta(seconds=t)


def get_detections(delta_power: np.ndarray, threshold_std_factor: float, block_duration_sec: float,
                   wav_start_date_time=None, device: int = 0, return_margin: bool = False):
    """main.py:396-448: global mean + k*std threshold; returns (detections, threshold)."""
    cfg = _lib.det_cfg(False, threshold_std_factor)
    try:
        dets, thr, margin = _lib.detect(context(device), delta_power, cfg)
    except _lib.MsdError as e:
        if e.code == _lib.MSD_ERR_INDEX:
            raise IndexError(e.msg) from None
        if e.code == _lib.MSD_ERR_ASSERT:
            # same ordering as the reference: the UTC assert (main.py:435) fires first
            if wav_start_date_time is not None:
                raise AssertionError("UTC start time must be before stop time") from None
            raise AssertionError(e.msg) from None
        raise
    out = []
    for d in dets:
        start, stop = np.int64(d["start"]), np.int64(d["stop"])
        t_start = start * block_duration_sec
        t_stop = stop * block_duration_sec
        out.append(OutputDetection(t_start=t_start, t_stop=t_stop, dB=np.float64(d["db"]), dur_s=t_stop - t_start,
                                   utc_start=_utc(wav_start_date_time, t_start),
                                   utc_stop=_utc(wav_start_date_time, t_stop)))
    threshold = np.float64(thr[0])
    return (out, threshold, margin) if return_margin else (out, threshold)


def get_detections_adaptive(delta_power: np.ndarray, threshold_std_factor: float, block_duration_sec: float,
                            threshold_estimation_window_sec=120, threshold_freeze_before_detection_sec=3,
                            threshold_freeze_after_detection_sec=20, fixed_threshold_duration_sec=10,
                            wav_start_date_time=None, device: int = 0, return_margin: bool = False):
    """main.py:450-522: adaptive threshold with freeze; returns (detections, thresholds list)."""
    cfg = _lib.det_cfg(True, threshold_std_factor,
                       _blocks(threshold_estimation_window_sec, block_duration_sec),
                       _blocks(threshold_freeze_before_detection_sec, block_duration_sec),
                       _blocks(threshold_freeze_after_detection_sec, block_duration_sec),
                       _blocks(fixed_threshold_duration_sec, block_duration_sec))
    dets, thr, margin = _lib.detect(context(device), delta_power, cfg)
    out = []
    for d in dets:
        start, stop = int(d["start"]), int(d["stop"])
        t_start = start * block_duration_sec
        t_stop = stop * block_duration_sec
        out.append(OutputDetection(t_start=t_start, t_stop=t_stop, dB=np.float64(d["db"]), dur_s=t_stop - t_start,
                                   utc_start=_utc(wav_start_date_time, t_start),
                                   utc_stop=_utc(wav_start_date_time, t_stop)))
    thresholds = [np.float64(v) for v in thr]
    return (out, thresholds, margin) if return_margin else (out, thresholds)


# --------------------------------------------------------------------------- a6 / a11
def write_csv(detections, out_csv_file) -> None:
    """main.py:640-658: csv.DictWriter, default dialect ('\\r\\n' rows), str() of each value."""
    with open(out_csv_file, "w", newline="") as csvfile:
        writer = csv.DictWriter(csvfile, fieldnames=["t_start", "t_stop", "dur_s", "dB", "utc_start", "utc_stop"])
        writer.writeheader()
        for det in detections:
            writer.writerow({
                "t_start": det.t_start,
                "t_stop": det.t_stop,
                "dur_s": det.dur_s,
                "dB": det.dB,
                "utc_start": det.utc_start.isoformat() if det.utc_start else None,
                "utc_stop": det.utc_stop.isoformat() if det.utc_stop else None,
            })


def write_audacity_labels(detections, path) -> None:
    """main.py:630-638."""
    with open(path, "w") as f:
        f.write("".join(f"{d.t_start:.2f}\t{d.t_stop:.2f}\tM\n" for d in detections))


def count_per_hour(detections) -> Counter:
    """main.py:690-696: Counter of utc_start truncated to the hour."""
    return Counter(d.utc_start.replace(minute=0, second=0, microsecond=0) for d in detections)


# --------------------------------------------------------------------------- a7
def spectrogram(x, fs=1.0, window="hann", nperseg=None, noverlap=None, nfft=None, detrend="constant",
                return_onesided=True, scaling="density", axis=-1, mode="psd", device: int = 0):
    """scipy.signal.spectrogram for the configuration the reference uses (main.py:52-54, :132-133):
    periodic Hann, constant detrend, one-sided density PSD of a real 1-D signal.
    As scipy: nperseg defaults to 256 and shrinks (with scipy's warning) to a shorter input;
    noverlap defaults to nperseg // 8; nfft >= nperseg zero-pads each segment.  nfft must be a
    power of two in [16, 16384].  Returns (f, t, Sxx) with Sxx [nfft//2+1, T] in scipy's output
    precision, np.result_type(x, np.complex64): float32 for u8 / i16 / u16 / f32 input, float64 for
    i32 / u32 / i64 / f64 (computed in float64 then)."""
    import warnings
    x = np.asarray(x)
    if isinstance(window, tuple):
        window = window[0] if len(window) == 1 else window
    if window not in ("hann", "hanning"):
        raise NotImplementedError("only window='hann' is implemented")
    if x.ndim != 1 or axis not in (-1, 0):
        raise NotImplementedError("only 1-D input is implemented")
    if detrend != "constant" or not return_onesided or scaling != "density" or mode != "psd":
        raise NotImplementedError("only detrend='constant', one-sided, density, mode='psd' are implemented")
    if np.iscomplexobj(x):
        raise NotImplementedError("complex (two-sided) input: use meteorgpu.iq")
    # scipy's output precision: np.result_type(x, np.complex64) (complex128 for i32 / u32 / i64 / u64 /
    # f64 input), decided on the caller's dtype before any conversion for the kernel
    double = np.result_type(x.dtype, np.complex64) == np.complex128
    if x.dtype == np.int64:
        x = x.astype(np.float64)  # same values up to 2^53; scipy computes these in float64 too
    n = x.shape[0]
    nperseg = 256 if nperseg is None else int(nperseg)
    if nperseg < 1:
        raise ValueError("nperseg must be a positive integer")
    if nperseg > n:  # scipy _triage_segments
        warnings.warn(f"nperseg = {nperseg:d} is greater than input length  = {n:d}, using nperseg = {n:d}",
                      stacklevel=2)
        nperseg = n
    noverlap = nperseg // 8 if noverlap is None else int(noverlap)
    if noverlap >= nperseg:
        raise ValueError("noverlap must be less than nperseg.")
    nfft = nperseg if nfft is None else int(nfft)
    if nfft < nperseg:
        raise ValueError("nfft must be greater than or equal to nperseg.")
    if nfft < 16 or nfft > 16384 or nfft & (nfft - 1):
        raise NotImplementedError("nfft must be a power of two in [16, 16384]")
    hop = nperseg - noverlap
    w64 = hann_periodic(nperseg)
    wc = w64.astype(np.complex128 if double else np.complex64)  # _spectral_helper casts the window
    scale = float(np.real(1.0 / (fs * (wc * wc).sum())))
    if x.dtype not in (np.uint8, np.int16, np.int32, np.float32, np.float64):
        x = x.astype(np.float64)
    plan = _lib.StftPlan(context(device), nperseg, hop, wc.real, scale, nfft=nfft,
                         precision=np.float64 if double else np.float32)
    try:
        sxx = plan.run(np.ascontiguousarray(x))
    finally:
        plan.close()
    freqs = np.fft.rfftfreq(nfft, 1 / fs)
    time = np.arange(nperseg / 2, n - nperseg / 2 + 1, nperseg - noverlap) / float(fs)
    return freqs, time, sxx


# --------------------------------------------------------------------------- main.py:207-806
def proc_wav_file(file_path,
                  block_duration_sec,
                  freq_band,
                  noise_band,
                  n_fft,
                  threshold_std_factor,
                  wav_start_sec=None,
                  wav_end_sec=None,
                  debug_plot_whole=False,
                  debug_plot_config=False,
                  debug_plot_output=False,
                  debug_plot_output_interactive=False,
                  outfile_path=None,
                  out_audacity_lbl_file=None,
                  out_csv_file=None,
                  wav_start_date_time=None,
                  disable_show_and_write=False,
                  flag_adaptive_threshold=True,
                  threshold_estimation_window_sec=120,
                  threshold_freeze_before_detection_sec=3,
                  threshold_freeze_after_detection_sec=20,
                  threshold_fixed_init_duration_sec=10,
                  *,
                  required_sample_rate=6000,
                  device=0,
                  verbose=True,
                  figure_dir=None):
    """GPU drop-in for dsp/src/main.py:207-806 (same arguments, asserts and outputs).

    ``required_sample_rate`` keeps the reference's ``assert fs == 6000`` (main.py:267);
    pass ``None`` to accept any rate (e.g. the 48 kHz configurations).  ``figure_dir``: also
    save every debug figure there (PNG; plotly figures as HTML instead of fig.show())."""
    say = print if verbose else (lambda *a, **k: None)
    assert os.path.exists(file_path), f"File does not exist: {file_path}"
    if outfile_path is not None:
        assert os.path.exists(os.path.dirname(outfile_path)), \
            f"Output directory does not exist: {os.path.dirname(outfile_path)}"
        now = datetime.datetime.now()  # main.py:235-237: a fresh timestamped export directory
        outfile_path = f"{outfile_path}/{now.strftime('%Y%m%d_%H%M%S')}/"
        os.makedirs(outfile_path, exist_ok=False)
    if out_audacity_lbl_file is not None:
        assert os.path.exists(os.path.dirname(out_audacity_lbl_file)), \
            f"Output directory does not exist: {os.path.dirname(out_audacity_lbl_file)}"
    if out_csv_file is not None:
        assert os.path.exists(os.path.dirname(out_csv_file)), \
            f"Output directory does not exist: {os.path.dirname(out_csv_file)}"
    wav_sample_rate, wav_data = wav.read(file_path)

    if wav_start_sec is not None or wav_end_sec is not None:
        if wav_start_sec is None:
            wav_start_sec = 0
        if wav_end_sec is None:
            wav_end_sec = len(wav_data) / wav_sample_rate
        start_sample = int(wav_start_sec * wav_sample_rate)
        end_sample = int(wav_end_sec * wav_sample_rate)
        assert start_sample < end_sample, "Start sample must be less than end sample"
        assert end_sample <= len(wav_data), "End sample exceeds length of audio data"
        wav_data = wav_data[start_sample:end_sample]

    if required_sample_rate is not None:
        assert wav_sample_rate == required_sample_rate, \
            f"Sample rate must be {required_sample_rate} Hz, but got {wav_sample_rate} Hz"
    assert len(wav_data.shape) == 1, f"Data must be mono or stereo, but got shape {wav_data.shape}"

    say("Wav duration [sec]:", len(wav_data) / wav_sample_rate)
    if debug_plot_whole or debug_plot_config or debug_plot_output or debug_plot_output_interactive:
        from . import figures
    if debug_plot_whole:  # main.py:278-306
        figures.debug_whole(wav_data, wav_sample_rate, freq_band, noise_band, figure_dir, device=device)
    if debug_plot_config:  # main.py:324-350
        figures.debug_config(wav_data, wav_sample_rate, freq_band, noise_band, figure_dir, device=device)
    res = process_samples(wav_data, wav_sample_rate, block_duration_sec, freq_band, noise_band, n_fft,
                          threshold_std_factor, wav_start_date_time=wav_start_date_time,
                          flag_adaptive_threshold=flag_adaptive_threshold,
                          threshold_estimation_window_sec=threshold_estimation_window_sec,
                          threshold_freeze_before_detection_sec=threshold_freeze_before_detection_sec,
                          threshold_freeze_after_detection_sec=threshold_freeze_after_detection_sec,
                          threshold_fixed_init_duration_sec=threshold_fixed_init_duration_sec,
                          device=device, verbose=verbose)

    times = np.arange(res.num_blocks) * block_duration_sec  # main.py:529
    if debug_plot_output:  # main.py:531-565
        figures.debug_output_delta(times, res.delta_power, res.thresholds, res.detections, flag_adaptive_threshold,
                                   figure_dir)
    if debug_plot_output_interactive:  # main.py:567-624
        figures.debug_output_interactive(times, res.band_power, res.noise_power, res.delta_power, res.thresholds,
                                         res.detections, freq_band, noise_band, figure_dir)
    for det in res.detections:
        say(f"Detection from {det.t_start:.2f} to {det.t_stop:.2f} seconds, dB: {det.dB:.2f} dB, "
            f"duration: {det.dur_s:.2f} seconds UTC_START: {det.utc_start}, UTC_STOP: {det.utc_stop}")
    if out_audacity_lbl_file is not None:
        write_audacity_labels(res.detections, out_audacity_lbl_file)
        say("Write Pre-Lbl File to:", out_audacity_lbl_file)
        say("Wrote Items", len(res.detections), "to Audacity LBL file")
    if out_csv_file is not None:
        write_csv(res.detections, out_csv_file)
        say("Wrote Items", len(res.detections), "to CSV file:", out_csv_file)
    if debug_plot_output:  # main.py:660-716: histograms, then the per-hour map
        figures.debug_output_hists(res.detections, figure_dir)
        figures.debug_time_map(res.detections, figure_dir)
    if not disable_show_and_write:  # main.py:721-806: per-detection spectrogram + PSD figures
        from .figures import export_detections
        export_detections(res.detections, wav_data, wav_sample_rate, freq_band, outfile_path, device=device)
    return res


def process_samples(wav_data, wav_sample_rate, block_duration_sec, freq_band, noise_band, n_fft,
                    threshold_std_factor, wav_start_date_time=None, flag_adaptive_threshold=True,
                    threshold_estimation_window_sec=120, threshold_freeze_before_detection_sec=3,
                    threshold_freeze_after_detection_sec=20, threshold_fixed_init_duration_sec=10,
                    device=0, verbose=False) -> ProcResult:
    """The numeric core of proc_wav_file (main.py:352-527) on an in-memory mono signal."""
    say = print if verbose else (lambda *a, **k: None)
    say("n_fft [real]:", n_fft)
    nfft = n_fft * 2
    block_size = int(wav_sample_rate * block_duration_sec)
    num_blocks = len(wav_data) // block_size
    say("Set n_fft to:", nfft, "samples")
    say("Wav block size in samples:", block_size)
    say("Number of wav blocks:", num_blocks)
    freqs = np.fft.rfftfreq(nfft, d=1 / wav_sample_rate)
    say("Num of freq bins:", len(freqs))
    say("Bandwidth per freq bin [Hz]:", freqs[1] - freqs[0])
    say("Min Frequency [Hz]:", freqs[0])
    say("Max Frequency [Hz]:", freqs[-1])
    say("Power Band bandwidth [Hz]:", freq_band[1] - freq_band[0])
    say("Noise Band bandwidth [Hz]:", noise_band[1] - noise_band[0])

    band, noise, delta, _ = block_powers(wav_data, wav_sample_rate, block_duration_sec, freq_band, noise_band,
                                         n_fft, device=device)
    L = min(block_size, nfft)
    xmax = float(np.max(np.abs(np.asarray(wav_data, dtype=np.float64)))) if len(wav_data) else 0.0
    err = margin_mod.delta_error_bound(band, noise, nfft=nfft, L=L, window=hanning_sym(block_size)[:L], xmax=xmax,
                                       band=band_bins(nfft, wav_sample_rate, freq_band),
                                       noise=band_bins(nfft, wav_sample_rate, noise_band))
    assert len(band) == num_blocks and len(noise) == num_blocks
    if not flag_adaptive_threshold:
        dets, thr, margin = get_detections(delta, threshold_std_factor, block_duration_sec, wav_start_date_time,
                                           device=device, return_margin=True)
        say("Threshold for delta power detection [dB]:", thr)
    else:
        dets, thr, margin = get_detections_adaptive(
            delta, threshold_std_factor, block_duration_sec, threshold_estimation_window_sec,
            threshold_freeze_before_detection_sec, threshold_freeze_after_detection_sec,
            threshold_fixed_init_duration_sec, wav_start_date_time, device=device, return_margin=True)
    bound = margin_mod.decision_bound(err, threshold_std_factor)
    near = margin_mod.check(margin, bound)
    return ProcResult(dets, thr, band, noise, delta, block_size, num_blocks, margin, bound, near)

"""CPU oracle for the complex (I/Q) spectrogram of BASELINE config C5 — TEST INFRASTRUCTURE ONLY.

Same rules as dsp_oracle.py.  The reference's spectrogram call (dsp/src/main.py:52-54 /
:132-133: scipy.signal.spectrogram(x, fs, window='hann', nperseg=N, noverlap=...)) applied to
SDR I/Q samples z = I + 1j*Q, where scipy switches to the two-sided spectrum in FFT bin order.
"""
from __future__ import annotations

import numpy as np


def spectrogram_iq_ref(i, q, fs, nperseg=4096, noverlap=3072):
    import warnings
    from scipy.signal import spectrogram
    z = np.asarray(i).astype(np.float64) + 1j * np.asarray(q).astype(np.float64)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")  # "Input data is complex, switching to return_onesided=False"
        return spectrogram(z, fs, window="hann", nperseg=nperseg, noverlap=noverlap)


def band_delta_iq_ref(Sxx, fs, nperseg, freq_band, noise_band):
    """dsp/src/main.py:380-393 per STFT frame of the two-sided spectrogram Sxx [N][T] (FFT bin order):
    masks (f >= lo) & (f <= hi) over fftfreq(N, 1/fs); E = np.sum(P[mask]) + 1e-12; dB = 10*log10(E)."""
    f = np.fft.fftfreq(nperseg, d=1 / fs)
    sb = (f >= freq_band[0]) & (f <= freq_band[1])
    sn = (f >= noise_band[0]) & (f <= noise_band[1])
    band = np.array([10 * np.log10(np.sum(Sxx[sb, t]) + 1e-12) for t in range(Sxx.shape[1])], np.float64)
    noise = np.array([10 * np.log10(np.sum(Sxx[sn, t]) + 1e-12) for t in range(Sxx.shape[1])], np.float64)
    return band, noise, band - noise


def proc_iq_ref(i, q, fs, freq_band, noise_band, nperseg=4096, noverlap=3072, threshold_std_factor=4.0,
                flag_adaptive_threshold=True, threshold_estimation_window_sec=120,
                threshold_freeze_before_detection_sec=3, threshold_freeze_after_detection_sec=20,
                threshold_fixed_init_duration_sec=10, wav_start_date_time=None):
    """The reference's block detector (main.py:380-527) with the STFT frame of the I/Q spectrogram as
    the block (block_sec = hop/fs): (detections, thresholds, band, noise, delta)."""
    from . import dsp_oracle as O
    _, _, S = spectrogram_iq_ref(i, q, fs, nperseg, noverlap)
    band, noise, delta = band_delta_iq_ref(S, fs, nperseg, freq_band, noise_band)
    bs = (nperseg - noverlap) / fs
    if flag_adaptive_threshold:
        dets, thr = O.get_detections_adaptive_ref(delta, threshold_std_factor, bs, threshold_estimation_window_sec,
                                                  threshold_freeze_before_detection_sec,
                                                  threshold_freeze_after_detection_sec,
                                                  threshold_fixed_init_duration_sec, wav_start_date_time)
    else:
        dets, thr = O.get_detections_ref(delta, threshold_std_factor, bs, wav_start_date_time)
    return dets, thr, band, noise, delta

"""CPU oracle for the legacy spectrogram noise floor — TEST INFRASTRUCTURE ONLY.

Same rules as dsp_oracle.py.  Restates meteor_detect_class/prime_detection.py:65-91 without
the figures: ``plt.specgram(iq_segment[:, 0], Fs=fs, NFFT=2048, noverlap=1024)`` (which is
matplotlib.mlab.specgram with its defaults), the noise-band power over bins and frames, and
the colour floor vmin.  The reference module imports pyaudio / twitchrealtimehandler / cv2
(absent) and opens a network stream at import, and running reference code is denied
(SURVEY §8c): pinned by restatement + matplotlib goldens ("partially pinned").
"""
from __future__ import annotations

import numpy as np

C_MS_SPEC_CUT_FACTOR = 12  # prime_detection.py:22


def specgram_ref(x, NFFT, Fs, noverlap):
    """matplotlib.mlab.specgram as plt.specgram calls it (prime_detection.py:70-71)."""
    from matplotlib import mlab
    return mlab.specgram(x, NFFT=NFFT, Fs=Fs, noverlap=noverlap)


def noise_floor_ref(x, fs, NFFT=2048, lower_freq=250, upper_freq=800, cut_factor=C_MS_SPEC_CUT_FACTOR):
    """prime_detection.py:65-91: (Pxx, freqs, bins, vmin, power_density_db_hz)."""
    delta_f = fs / NFFT                                               # :68
    Pxx, freqs, bins = specgram_ref(x, NFFT, fs, NFFT // 2)           # :70-71
    noise_band = (freqs >= lower_freq) & (freqs <= upper_freq)        # :75
    bandwidth = np.sum(noise_band) * delta_f                          # :77
    band_power = np.sum(Pxx[noise_band])                              # :83
    power_density_db_hz = 10 * np.log10(band_power / bandwidth)       # :84
    factor = 40 / 23                                                  # :85
    temp_vmin = power_density_db_hz / factor + cut_factor             # :91
    return Pxx, freqs, bins, temp_vmin, power_density_db_hz

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

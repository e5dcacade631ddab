"""GPU: scipy.signal.spectrogram shapes beyond the tiled kernels (csrc/stft_any.hip) and the
headline C1/C2 spectrogram at its full length.

* C1/C2: one 60 s 48 kHz recording, 1024 / 512 (2.88 M samples, 5624 frames), against scipy
  computed here, per frame (dsp/src/main.py:132-133);
* nperseg 4096 and 8192 (the whole-file debug spectrogram, main.py:127-133 with n_fft =
  1024*4, :278-300; the commented :753-759 sizes);
* nfft > nperseg (zero-padded segments) and inputs shorter than nperseg (scipy shrinks nperseg
  to the input length with a warning, _spectral_py.py _triage_segments);
* int32 / float64 input: scipy computes those in float64, and so does the device.

Bars: float32 results within SPEC_TOL relative per frame (the north-star tolerance); float64
results within 1e-10."""
import warnings

import numpy as np
import pytest
from scipy.signal import spectrogram as sp_spec

from meteorgpu import dsp, synth

pytestmark = pytest.mark.gpu

SPEC_TOL = 1e-5
F64_TOL = 1e-10


def _frame_err(S, ref):
    return (np.abs(S.astype(np.float64) - ref.astype(np.float64)).max(axis=0) /
            np.maximum(np.abs(ref).max(axis=0), 1e-300)).max()


def _signal(fs, n, dtype, seed):
    x, _ = synth.synth_real(seed=seed, fs=fs, duration_s=n / fs + 1, f0=1000.0, rate_per_min=30)
    x = x[:n]
    if np.dtype(dtype) == np.float32:
        return (x / 32768.0).astype(np.float32)
    if np.dtype(dtype) == np.float64:
        return x / 32768.0
    if np.dtype(dtype) == np.int32:
        return x.astype(np.int32) * 65536
    if np.dtype(dtype) == np.uint32:
        return (x.astype(np.int64) + 32768).astype(np.uint32) * 65536
    if np.dtype(dtype) == np.uint16:
        return (x.astype(np.int32) + 32768).astype(np.uint16)
    return x


def test_c1_full_minute_48k_vs_scipy():
    x, _ = synth.synth_real(seed=2001, fs=48000, duration_s=60.0, f0=1000.0)
    assert x.shape == (2_880_000,)
    fr, tr, Sr = sp_spec(x, fs=48000, window="hann", nperseg=1024, noverlap=512, nfft=1024, scaling="density",
                         mode="psd")
    f, t, S = dsp.spectrogram(x, fs=48000, window="hann", nperseg=1024, noverlap=512, nfft=1024)
    assert S.shape == Sr.shape == (513, 5624) and S.dtype == np.float32
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    assert _frame_err(S, Sr) <= SPEC_TOL


CASES = [
    # fs, nperseg, noverlap, nfft, dtype, n
    (6000, 4096, 2048, 4096, np.int16, 6000 * 60),    # debug_plot_whole at the reference rate
    (6000, 8192, 4096, 8192, np.int16, 6000 * 30),
    (48000, 16384, 8192, 16384, np.float32, 48000 * 4),
    (48000, 1024, 512, 4096, np.int16, 48000 * 3),     # zero padding
    (48000, 1000, 500, 1024, np.int16, 48000 * 3),     # zero padding, non-power-of-two segment
    (6000, 3000, 1000, 4096, np.float32, 6000 * 20),
    (48000, 1024, 512, 1024, np.int32, 48000 * 3),     # float64 path (scipy: complex128)
    (48000, 4096, 1024, 4096, np.float64, 48000 * 3),
    (48000, 2048, 0, 2048, np.uint8, 48000 * 2),
    (48000, 16384, 8192, 16384, np.float64, 48000 * 4),  # float64 nfft 16384: one in-place LDS buffer
    (48000, 8192, 2048, 16384, np.int32, 48000 * 2),     # float64, zero padding to 16384
    (48000, 1024, 512, 1024, np.uint32, 48000 * 2),      # scipy: complex128 (np.result_type), float64 out
    (48000, 1024, 512, 1024, np.uint16, 48000 * 2),      # scipy: complex64, float32 out
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[1]}-{c[2]}-{c[3]}-{np.dtype(c[4]).name}" for c in CASES])
def test_spectrogram_shapes_vs_scipy(case):
    fs, N, nov, nfft, dt, n = case
    x = _signal(fs, n, dt, seed=N + nfft + nov)
    if np.dtype(dt) == np.uint8:
        x = ((x.astype(np.int32) >> 8) + 128).astype(np.uint8) if x.dtype != np.uint8 else x
    fr, tr, Sr = sp_spec(x, fs=fs, window="hann", nperseg=N, noverlap=nov, nfft=nfft, scaling="density", mode="psd")
    f, t, S = dsp.spectrogram(x, fs=fs, window="hann", nperseg=N, noverlap=nov, nfft=nfft)
    assert S.shape == Sr.shape and S.dtype == Sr.dtype
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    assert _frame_err(S, Sr) <= (F64_TOL if S.dtype == np.float64 else SPEC_TOL)


@pytest.mark.parametrize("n", [900, 1023, 17])
def test_short_input_shrinks_nperseg(n):
    x = _signal(6000, n, np.int16, seed=n)
    with warnings.catch_warnings(record=True) as wr:
        warnings.simplefilter("always")
        fr, tr, Sr = sp_spec(x, fs=6000, window="hann", nperseg=1024, noverlap=n // 4, nfft=1024,
                             scaling="density", mode="psd")
    with warnings.catch_warnings(record=True) as wg:
        warnings.simplefilter("always")
        f, t, S = dsp.spectrogram(x, fs=6000, window="hann", nperseg=1024, noverlap=n // 4, nfft=1024)
    assert [str(w.message) for w in wg] == [str(w.message) for w in wr] != []
    assert S.shape == Sr.shape == (513, 1)
    np.testing.assert_array_equal(t, tr)
    assert _frame_err(S, Sr) <= SPEC_TOL


def test_dyn_lds_attribute_only_grows():
    """one stft_any instantiation serves plans of different nfft: a large plan, a small one, then
    the large one again must launch (the LDS attribute is never lowered under a later launch)"""
    x = _signal(6000, 6000 * 8, np.int16, seed=5)
    for nfft in (8192, 1024, 8192):
        fr, tr, Sr = sp_spec(x, fs=6000, window="hann", nperseg=1000, noverlap=500, nfft=nfft, scaling="density",
                             mode="psd")
        f, t, S = dsp.spectrogram(x, fs=6000, window="hann", nperseg=1000, noverlap=500, nfft=nfft)
        assert S.shape == Sr.shape and _frame_err(S, Sr) <= SPEC_TOL


def test_shape_errors_match_scipy():
    x = _signal(6000, 6000, np.int16, seed=1)
    with pytest.raises(ValueError, match="nfft must be greater than or equal to nperseg"):
        dsp.spectrogram(x, fs=6000, nperseg=1024, nfft=512)
    with pytest.raises(ValueError, match="noverlap must be less than nperseg"):
        dsp.spectrogram(x, fs=6000, nperseg=1024, noverlap=1024)
    with pytest.raises(NotImplementedError):
        dsp.spectrogram(x, fs=6000, nperseg=1000)  # nfft = 1000: not a power of two

"""Legacy spectrogram noise floor (prime_detection.py:65-91).

CPU: the oracle against the matplotlib golden (tests/golden/legacy_5k.npz).
GPU: meteorgpu.legacy (libmsdsp's float64 STFT with detrend off + device band sum) against the
golden and the oracle.  Bars: spectrogram within SPEC_TOL relative per frame (float64 on both
sides: mlab's pocketfft vs the device's radix-4 FFT), vmin within VMIN_TOL dB."""
import os

import numpy as np
import pytest

from oracle import legacy_oracle as LO

SPEC_TOL = 1e-12
VMIN_TOL = 1e-10


def _frame_rel(a, b):
    num = np.linalg.norm(a - b, axis=0)
    den = np.linalg.norm(b, axis=0)
    return float(np.max(num / np.maximum(den, 1e-300)))


def test_oracle_matches_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "legacy_5k.npz"))
    Pxx, freqs, t, vmin, pddb = LO.noise_floor_ref(g["x"], int(g["fs"]), int(g["NFFT"]))
    np.testing.assert_array_equal(Pxx, g["Pxx"])
    np.testing.assert_array_equal(freqs, g["freqs"])
    np.testing.assert_array_equal(t, g["t"])
    assert vmin == g["vmin"] and pddb == g["pddb"]


@pytest.mark.gpu
def test_noise_floor_golden(golden_dir):
    from meteorgpu import legacy
    g = np.load(os.path.join(golden_dir, "legacy_5k.npz"))
    Pxx, freqs, t, vmin, pddb = legacy.noise_floor(g["x"], int(g["fs"]), int(g["NFFT"]))
    assert Pxx.shape == g["Pxx"].shape
    np.testing.assert_array_equal(freqs, g["freqs"])
    np.testing.assert_array_equal(t, g["t"])
    assert _frame_rel(Pxx, g["Pxx"]) < SPEC_TOL
    assert abs(vmin - float(g["vmin"])) < VMIN_TOL
    assert abs(pddb - float(g["pddb"])) < VMIN_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("NFFT,fs,dtype,seconds", [
    (2048, 5000, np.int16, 8.0), (1024, 5000, np.int16, 8.0), (256, 6000, np.int16, 8.0),
    (512, 5000, np.float32, 8.0), (4096, 5000, np.int16, 8.0), (8192, 5000, np.float64, 8.0),
    (16384, 5000, np.int16, 12.0),  # float64 at nfft 16384: the in-place LDS passes (2 buffers = 256 KB)
    (2048, 5000, np.int16, 0.3)])  # the last: shorter than NFFT, zero-padded to one frame
def test_specgram_vs_mlab(NFFT, fs, dtype, seconds):
    from meteorgpu import legacy, synth
    x, _ = synth.synth_real(seed=NFFT + fs, fs=fs, duration_s=seconds, f0=1000.0, sigma=700.0, rate_per_min=15)
    if dtype == np.float32:
        x = (x / 32768.0).astype(np.float32)
    elif dtype == np.float64:
        x = x / 32768.0
    P, f, t = legacy.specgram(x, NFFT=NFFT, Fs=fs, noverlap=NFFT // 2)
    rP, rf, rt = LO.specgram_ref(x, NFFT, fs, NFFT // 2)
    assert P.shape == rP.shape
    np.testing.assert_array_equal(f, rf)
    np.testing.assert_array_equal(t, rt)
    assert _frame_rel(P, rP) < SPEC_TOL


@pytest.mark.gpu
def test_noise_floor_30s_reference_shape():
    """The reference's own configuration: 30 s at 5 kHz (C_SEG_LEN, C_SAMPLE_RATE), NFFT 2048."""
    from meteorgpu import legacy, synth
    x, _ = synth.synth_real(seed=31, fs=5000, duration_s=30.0, f0=1000.0, sigma=600.0, rate_per_min=10)
    P, f, t, vmin, pddb = legacy.noise_floor(x, 5000)
    rP, rf, rt, rvmin, rpddb = LO.noise_floor_ref(x, 5000)
    assert P.shape == rP.shape == (1025, 145)
    assert _frame_rel(P, rP) < SPEC_TOL
    assert abs(vmin - rvmin) < VMIN_TOL


def test_hourly_csv_matches_pandas_flow(tmp_path):
    """prime_detection.py:137-146 (create) and :229-245 (append) done with pandas as the
    reference does, against meteorgpu.legacy.append_hourly_row."""
    import datetime
    import pandas as pd
    from meteorgpu import legacy
    ref = tmp_path / "ref.csv"
    pd.DataFrame(columns=["Timestamp", "Anzahl", "Kritisch"]).to_csv(ref, sep=";", index=False)
    rows = [(datetime.datetime(2025, 6, 1, 10, 0, 3), 3, 4), (datetime.datetime(2025, 6, 1, 10, 59, 51), 0, 0)]
    for st, nc, nn in rows:
        df2 = pd.read_csv(ref, sep=";")
        df2 = pd.concat([df2, pd.DataFrame([{"Timestamp": st.strftime("%Y-%m-%d %H:%M:%S"),
                                             "Anzahl": nc + nn, "Kritisch": nc}])], ignore_index=True)
        df2.to_csv(ref, sep=";", index=False)
    ours = tmp_path / "ours.csv"
    for st, nc, nn in rows:
        legacy.append_hourly_row(ours, st, nc, nn)
    assert ours.read_bytes() == ref.read_bytes()


@pytest.mark.gpu
def test_burst_shim_classifies_by_duration():
    from meteorgpu import legacy, synth
    from oracle import dsp_oracle as O
    x, _ = synth.synth_real(seed=13, fs=5000, duration_s=30.0, f0=1000.0, sigma=500.0, rate_per_min=6,
                            band_hz=100.0, snr_db=(20, 35), dur_s=(0.2, 2.0))
    bursts, labels, pos, crit, noncrit = legacy.detect_and_cluster_bursts_audio(x, 5000)
    ref, *_ = O.proc_samples_ref(x, 5000, 0.1, (950.0, 1050.0), (650.0, 750.0), 1024, 4.0)
    assert [(d.t_start, d.t_stop) for d in bursts] == [(r[0], r[1]) for r in ref]
    assert len(bursts) > 0 and labels == set(range(len(bursts)))
    assert sorted(crit + noncrit) == list(range(len(bursts)))
    assert all(bursts[i].dur_s >= 0.5 for i in crit) and all(bursts[i].dur_s < 0.5 for i in noncrit)
    assert len(crit) >= 1 and len(noncrit) >= 1

"""Generate the golden vectors under tests/golden/ (committed; rerun to refresh).

The reference (th-nuernberg/meteor-scatter) ships no audio and no tests, and
running it was denied in this environment.  Its arithmetic is
entirely numpy/scipy, so the golden vectors are those third-party calls, made
exactly as the reference makes them, on seeded synthetic inputs:

  blocks_*.npz : np.fft.rfft(block * np.hanning(B), n=Nf) → |.|^2 band sums → dB
                 (dsp/src/main.py:376-393) for the 6 kHz reference configuration
                 (mb_files, main.py:825-899) and a 48 kHz configuration
  spec_*.npz   : scipy.signal.spectrogram(x, fs, 'hann', nperseg=N, noverlap=N//2,
                 nfft=N, scaling='density', mode='psd') (main.py:132-133), float32
  legacy_5k.npz: matplotlib.mlab.specgram(x, NFFT=2048, Fs=5000, noverlap=1024) as
                 plt.specgram computes it, the 250-800 Hz band power over bins and frames and
                 the colour floor vmin (meteor_detect_class/prime_detection.py:65-91)
  iq_192k_4096.npz: scipy.signal.spectrogram(I + 1j*Q, 192000, 'hann', 4096, noverlap 3072)
                 (two-sided, config C5 shape), stored as float32
  live_4k.npz  : per processing block, scipy.signal.welch(block, fs, nfft=n_fft) on the
                 soundfile float64 of PCM16 samples (x / 32768), the three inclusive band
                 masks and np.sum → dB (dsp/src/live/backend/processor.py:206, :349-369),
                 plus two blocks' full Welch PSD

Run:  python tests/golden/make_golden.py [name ...]   (default: all)
"""
import os
import sys

import numpy as np
from scipy.signal import spectrogram

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "..", "meteor-scatter_amd"))
from meteorgpu.synth import synth_real  # noqa: E402  (seeded generator, host-only)


def blocks(x, fs, bs, band, noise, n_fft):
    nfft = 2 * n_fft
    B = int(fs * bs)
    freqs = np.fft.rfftfreq(nfft, d=1 / fs)
    mb = (freqs >= band[0]) & (freqs <= band[1])
    mn = (freqs >= noise[0]) & (freqs <= noise[1])
    out = np.empty((len(x) // B, 3))
    for i in range(len(x) // B):
        blk = x[i * B:(i + 1) * B]
        p = np.abs(np.fft.rfft(blk * np.hanning(len(blk)), n=nfft)) ** 2
        out[i, 0] = 10 * np.log10(np.sum(p[mb]) + 1e-12)
        out[i, 1] = 10 * np.log10(np.sum(p[mn]) + 1e-12)
    out[:, 2] = out[:, 0] - out[:, 1]
    return out


def live_golden():
    from scipy.signal import welch
    fs, bs, n_fft, f0 = 4000, 0.2, 4096, 1000
    x, _ = synth_real(seed=4242, fs=fs, duration_s=40.0, f0=f0, sigma=300.0, rate_per_min=12, band_hz=100.0,
                      snr_db=(15, 30), dur_s=(0.4, 2.0))
    xf = x.astype(np.float64) / 32768.0                       # soundfile's PCM16 → float64
    B = int(bs * fs)
    bands = [(f0 - 50, f0 + 50), (f0 - 300 - 50, f0 - 300 + 50), (f0 + 300 - 50, f0 + 300 + 50)]
    rows, psd2 = [], []
    for k, i in enumerate(range(0, len(xf) - B + 1, B)):
        f, p = welch(xf[i:i + B], fs, nfft=n_fft)
        r = []
        for lo, hi in bands:
            P = np.sum(p[(f >= lo) & (f <= hi)])
            r.append(10 * np.log10(P) if P > 0 else -np.inf)
        rows.append(r)
        if k in (3, 77):
            psd2.append(p)
    np.savez_compressed(os.path.join(HERE, "live_4k.npz"), x=x, fs=fs, bs=bs, n_fft=n_fft, f0=f0,
                        bands=np.array(bands, dtype=np.float64), expected=np.array(rows).T,
                        psd_blocks=np.array([3, 77]), psd=np.array(psd2))


def legacy_golden():
    from matplotlib import mlab
    fs, NFFT = 5000, 2048
    x, _ = synth_real(seed=5151, fs=fs, duration_s=6.0, f0=1000.0, sigma=800.0, rate_per_min=20, band_hz=100.0,
                      snr_db=(10, 25))
    Pxx, freqs, t = mlab.specgram(x, NFFT=NFFT, Fs=fs, noverlap=NFFT // 2)    # prime_detection.py:70
    nb = (freqs >= 250) & (freqs <= 800)
    band_power = np.sum(Pxx[nb])
    pddb = 10 * np.log10(band_power / (np.sum(nb) * (fs / NFFT)))
    np.savez_compressed(os.path.join(HERE, "legacy_5k.npz"), x=x, fs=fs, NFFT=NFFT, Pxx=Pxx, freqs=freqs, t=t,
                        band_power=band_power, pddb=pddb, vmin=pddb / (40 / 23) + 12)


def iq_golden():
    from scipy.signal import spectrogram
    fs, N = 192000, 4096
    rng = np.random.default_rng(192)
    n = 8192
    t = np.arange(n) / fs
    z = 3000 * np.exp(2j * np.pi * 1000.0 * t) + 700 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    i = np.clip(np.round(z.real), -32768, 32767).astype(np.int16)
    q = np.clip(np.round(z.imag), -32768, 32767).astype(np.int16)
    f, tt, S = spectrogram(i.astype(np.float64) + 1j * q.astype(np.float64), fs, window="hann", nperseg=N,
                           noverlap=3 * N // 4)
    np.savez_compressed(os.path.join(HERE, "iq_192k_4096.npz"), i=i, q=q, fs=fs, nperseg=N, noverlap=3 * N // 4,
                        f=f, t=tt, S=S.astype(np.float32))


def main(names=()):
    if not names or "iq" in names:
        iq_golden()
    if not names or "live" in names:
        live_golden()
    if not names or "legacy" in names:
        legacy_golden()
    if names and "core" not in names:
        return
    # 6 kHz, the reference's own configuration (main.py:827-833, 865-899)
    x6, _ = synth_real(seed=1, fs=6000, duration_s=20.0, f0=1003.0, rate_per_min=12, band_hz=20.0)
    b6 = blocks(x6, 6000, 0.2, (993, 1013), (690, 710), 512)
    np.savez_compressed(os.path.join(HERE, "blocks_6k.npz"), x=x6, fs=6000, bs=0.2, band=(993, 1013),
                        noise=(690, 710), n_fft=512, expected=b6)
    # 48 kHz configuration with bands that hold FFT bins (SURVEY §0 degenerate-config warning)
    x48, _ = synth_real(seed=2001, fs=48000, duration_s=3.0, f0=1000.0, rate_per_min=30)
    b48 = blocks(x48, 48000, 0.2, (950, 1050), (650, 750), 512)
    np.savez_compressed(os.path.join(HERE, "blocks_48k.npz"), x=x48, fs=48000, bs=0.2, band=(950, 1050),
                        noise=(650, 750), n_fft=512, expected=b48)
    # STFT spectrogram, 48 kHz, N=1024 / hop 512 (C1 shape, shortened)
    xs = x48[:24000]
    f, t, S = spectrogram(xs, fs=48000, window="hann", nperseg=1024, noverlap=512, nfft=1024,
                          scaling="density", mode="psd")
    np.savez_compressed(os.path.join(HERE, "spec_48k_1024.npz"), x=xs, fs=48000, nperseg=1024, f=f, t=t, S=S)
    # STFT spectrogram, 6 kHz, N=256, float32 input
    xf = (x6[:6000].astype(np.float32) / 32768.0).astype(np.float32)
    f, t, S = spectrogram(xf, fs=6000, window="hann", nperseg=256, noverlap=128, nfft=256,
                          scaling="density", mode="psd")
    np.savez_compressed(os.path.join(HERE, "spec_6k_256_f32.npz"), x=xf, fs=6000, nperseg=256, f=f, t=t, S=S)
    for name in sorted(os.listdir(HERE)):
        if name.endswith(".npz"):
            print(name, os.path.getsize(os.path.join(HERE, name)))


if __name__ == "__main__":
    main(sys.argv[1:])

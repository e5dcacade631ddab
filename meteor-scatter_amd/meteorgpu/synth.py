"""Seeded synthetic SDR audio (SURVEY §8(d) generator): Gaussian noise plus
meteor pings (Poisson arrivals, fast rise / exponential decay tone bursts at the
band centre), quantised to int16 with clipping.  The reference ships no audio, so
every test and benchmark input is made here; seed = 1000*config + file_index.
"""
from __future__ import annotations

import numpy as np


def synth_real(seed: int, fs: float, duration_s: float, f0: float, sigma: float = 1000.0,
               rate_per_min: float = 5.0, band_hz: float = 100.0, snr_db=(3.0, 30.0),
               dur_s=(0.1, 3.0), dtype=np.int16):
    """Real mono signal; returns (samples, pings) with pings = [(t_start, duration, amplitude)]."""
    rng = np.random.default_rng(seed)
    n = int(round(fs * duration_s))
    x = rng.standard_normal(n) * sigma
    n_pings = rng.poisson(rate_per_min * duration_s / 60.0)
    noise_in_band = sigma ** 2 * band_hz / (fs / 2.0)
    pings = []
    for _ in range(n_pings):
        t0 = rng.uniform(0, duration_s)
        d = float(np.exp(rng.uniform(np.log(dur_s[0]), np.log(dur_s[1]))))
        snr = rng.uniform(*snr_db)
        amp = float(np.sqrt(2.0 * noise_in_band * 10 ** (snr / 10.0)))
        phi = rng.uniform(0, 2 * np.pi)
        i0 = int(t0 * fs)
        i1 = min(n, i0 + int(d * fs * 3))
        if i1 <= i0:
            continue
        t = np.arange(i1 - i0) / fs
        rise = 0.01
        env = np.where(t < rise, t / rise, np.exp(-(t - rise) / (d / 3.0)))
        x[i0:i1] += amp * env * np.sin(2 * np.pi * f0 * (t + t0) + phi)
        pings.append((t0, d, amp))
    if np.dtype(dtype) == np.int16:
        x = np.clip(np.rint(x), -32768, 32767).astype(np.int16)
    else:
        x = x.astype(dtype)
    return x, pings


def synth_iq(seed: int, fs: float, duration_s: float, f0: float, sigma: float = 1000.0,
             rate_per_min: float = 5.0, band_hz: float = 100.0, snr_db=(3.0, 30.0), dur_s=(0.1, 3.0)):
    """Complex baseband I/Q (BASELINE config C5):
    z = A*g(t)*exp(j*2*pi*f0*t) + (sigma/sqrt 2)(N + jN), int16 I and Q; returns (i, q, pings)."""
    rng = np.random.default_rng(seed)
    n = int(round(fs * duration_s))
    z = (rng.standard_normal(n) + 1j * rng.standard_normal(n)) * (sigma / np.sqrt(2.0))
    n_pings = rng.poisson(rate_per_min * duration_s / 60.0)
    noise_in_band = sigma ** 2 * band_hz / fs
    pings = []
    for _ in range(n_pings):
        t0 = rng.uniform(0, duration_s)
        d = float(np.exp(rng.uniform(np.log(dur_s[0]), np.log(dur_s[1]))))
        snr = rng.uniform(*snr_db)
        amp = float(np.sqrt(noise_in_band * 10 ** (snr / 10.0)))
        phi = rng.uniform(0, 2 * np.pi)
        i0 = int(t0 * fs)
        i1 = min(n, i0 + int(d * fs * 3))
        if i1 <= i0:
            continue
        t = np.arange(i1 - i0) / fs
        rise = 0.01
        env = np.where(t < rise, t / rise, np.exp(-(t - rise) / (d / 3.0)))
        z[i0:i1] += amp * env * np.exp(1j * (2 * np.pi * f0 * (t + t0) + phi))
        pings.append((t0, d, amp))
    i = np.clip(np.rint(z.real), -32768, 32767).astype(np.int16)
    q = np.clip(np.rint(z.imag), -32768, 32767).astype(np.int16)
    return i, q, pings

"""CPU oracle for the phase-2 live detector — TEST INFRASTRUCTURE ONLY.

Same rules as dsp_oracle.py: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg use it, as the checker / the timed CPU baseline.

Restates dsp/src/live/backend/processor.py:14-507 (wav_file_process) minus the plots
and the per-detection image export, with the arithmetic in scipy/numpy exactly as the
reference calls it: scipy.signal.welch(block, fs, nfft=n_fft) (processor.py:206), the
three inclusive band masks and np.sum (:349-369), the over-noise value and its history
statistics (:391-403), the locked thresholds (:405-412) and the state machine
(:448-507) with the states of dsp/src/live/backend/aggregates.py:4-24.  Parity pin:
the reference module needs `soundfile` (absent) and running reference code is denied
(SURVEY §8c), so this is pinned by restatement + scipy goldens + hand KATs ("partially
pinned").
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class ConfigDetectionRef:
    """aggregates.py:32-44 defaults."""
    proc_block_sec: float = 0.2
    n_fft: int = 4096
    signal_freq: int = 1000
    channel_width: int = 100
    noise_channel_offset: int = 300
    avg_win_sec: float = 8
    init_detection_wait_sec: float = 8 * 1.0
    after_tracking_wait_sec: float = 8 * 1.5
    threshold_std_factor: float = 4
    detection_db_over_noise_mean_min: float = -1
    detection_dur_min_sec: float = -1


@dataclass
class MeteorRef:
    """aggregates.py:66-74 DetectedMeteor."""
    time_start: float
    time_stop: float
    duration: float
    db_min: float
    db_max: float
    db_mean: float
    db_std: float


def band_edges(cfg: ConfigDetectionRef):
    """processor.py:32-45: (signal, noise 1, noise 2) [start, stop] in Hz."""
    ms = (cfg.signal_freq - cfg.channel_width / 2, cfg.signal_freq + cfg.channel_width / 2)
    n1 = ((cfg.signal_freq - cfg.noise_channel_offset) - cfg.channel_width / 2,
          (cfg.signal_freq - cfg.noise_channel_offset) + cfg.channel_width / 2)
    n2 = ((cfg.signal_freq + cfg.noise_channel_offset) - cfg.channel_width / 2,
          (cfg.signal_freq + cfg.noise_channel_offset) + cfg.channel_width / 2)
    return ms, n1, n2


def block_psd_ref(block, fs, n_fft):
    """processor.py:206: scipy.signal.welch(block_data, file_sample_rate, nfft=n_fft)."""
    from scipy.signal import welch
    return welch(block, fs, nfft=n_fft)


def band_db_ref(freqs, psd, lo, hi):
    """processor.py:349-353 (and :356-369 for the noise bands)."""
    mask = (freqs >= lo) & (freqs <= hi)
    p = np.sum(psd[mask])
    return 10 * np.log10(p) if p > 0 else -np.inf


def welch_band_db_ref(x, fs, cfg: ConfigDetectionRef):
    """Per block (processor.py:177-178 framing): (sig_dB, noise1_dB, noise2_dB) float64 [3][nb]."""
    bs = int(cfg.proc_block_sec * fs)
    ms, n1, n2 = band_edges(cfg)
    rows = []
    for i in range(0, len(x) - bs + 1, bs):
        f, p = block_psd_ref(x[i:i + bs], fs, cfg.n_fft)
        rows.append([band_db_ref(f, p, *ms), band_db_ref(f, p, *n1), band_db_ref(f, p, *n2)])
    return np.array(rows, dtype=np.float64).T.reshape(3, -1)


def live_detect_ref(band_db, fs, block_size, cfg: ConfigDetectionRef):
    """processor.py:391-507 over precomputed band dB rows.  Returns (meteors, thresholds,
    over_noise) with thresholds[b] the threshold used at block b (:395-412)."""
    W = int(cfg.avg_win_sec / cfg.proc_block_sec)  # processor.py:58
    over = []
    thresholds = []
    meteors = []
    state = ("init",)
    for b in range(band_db.shape[1]):
        start_idx = b * block_size
        t0 = start_idx / fs                       # :181
        t1 = (start_idx + block_size) / fs        # :182
        sig, n1, n2 = band_db[0, b], band_db[1, b], band_db[2, b]
        db2 = sig - np.mean([n1, n2])              # :391
        hist = over[-W:]                           # :392 (before the append)
        over.append(db2)
        with np.errstate(invalid="ignore", divide="ignore"):
            import warnings
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", RuntimeWarning)
                h_mean = np.mean(hist)             # :397
                h_std = np.std(hist)               # :398
        thr = h_mean + cfg.threshold_std_factor * h_std   # :402
        if state[0] == "tracking":                 # :404-406
            thr = state[1]
        elif state[0] == "detection":              # :407-410
            if state[2] > t1:
                thr = state[1]
        thresholds.append(thr)
        if state[0] == "init":                     # :448-460
            if t0 >= cfg.init_detection_wait_sec:
                state = ("detection", -1.0, -1.0)
        elif state[0] == "detection":              # :462-472
            if db2 > thr:
                state = ("tracking", thr + 0 * h_std, t0, [])
        elif state[0] == "tracking":               # :474-504
            lock, ts, h = state[1], state[2], state[3]
            h.append(db2)
            if db2 < thr:
                dur = t0 - ts
                m = np.mean(h)
                if m >= cfg.detection_db_over_noise_mean_min and dur >= cfg.detection_dur_min_sec:
                    meteors.append(MeteorRef(ts, t0, dur, min(h), max(h), np.mean(h), np.std(h)))
                state = ("detection", lock, t0 + cfg.after_tracking_wait_sec)
    return meteors, np.array(thresholds, dtype=np.float64), np.array(over, dtype=np.float64)


def wav_file_process_ref(x, fs, cfg: ConfigDetectionRef):
    """processor.py:14-507 on in-memory samples (float64 as soundfile returns them)."""
    bdb = welch_band_db_ref(x, fs, cfg)
    return live_detect_ref(bdb, fs, int(cfg.proc_block_sec * fs), cfg)

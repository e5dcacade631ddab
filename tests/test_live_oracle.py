"""CPU: the phase-2 live-detector oracle (oracle/live_oracle.py) against the scipy golden
(tests/golden/live_4k.npz) and hand-derived known answers for the state machine of
dsp/src/live/backend/processor.py:391-507 (SURVEY §8(a) a9 KAT list)."""
import math
import os

import numpy as np
import pytest

from oracle import live_oracle as L

FS, B = 4000, 800


def test_welch_band_db_matches_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "live_4k.npz"))
    cfg = L.ConfigDetectionRef(n_fft=int(g["n_fft"]), signal_freq=int(g["f0"]))
    got = L.welch_band_db_ref(g["x"].astype(np.float64) / 32768.0, int(g["fs"]), cfg)
    np.testing.assert_array_equal(got, g["expected"])


def test_band_edges_follow_processor():
    ms, n1, n2 = L.band_edges(L.ConfigDetectionRef(signal_freq=1020, channel_width=100, noise_channel_offset=300))
    assert ms == (970, 1070) and n1 == (670, 770) and n2 == (1270, 1370)


def _rows(over):
    """band dB rows whose over-noise value is exactly `over` (noise rows 0 dB)."""
    over = np.asarray(over, dtype=np.float64)
    return np.stack([over, np.zeros_like(over), np.zeros_like(over)])


def _cfg(**kw):
    base = dict(proc_block_sec=0.2, avg_win_sec=4.0, init_detection_wait_sec=1.0, after_tracking_wait_sec=1.0,
                threshold_std_factor=6.0)
    base.update(kw)
    return L.ConfigDetectionRef(**base)


def test_first_threshold_is_nan_and_flat_input_never_detects():
    m, thr, over = L.live_detect_ref(_rows(np.ones(60)), FS, B, _cfg())
    assert math.isnan(thr[0]) and thr[1] == 1.0     # mean 1, std 0
    assert m == []


def _noise(n, seed=3):
    return np.random.default_rng(seed).normal(0.0, 1.0, n)


def test_single_ping_times_and_history():
    o = _noise(80)
    o[30:34] = [20, 25, 18, 15]          # trigger at 30, blocks 31..33 above, 34 closes
    o[34] = -5
    m, thr, _ = L.live_detect_ref(_rows(o), FS, B, _cfg())
    assert len(m) == 1
    d = m[0]
    assert d.time_start == 30 * B / FS and d.time_stop == 34 * B / FS
    assert d.duration == 34 * B / FS - 30 * B / FS
    h = [25, 18, 15, -5]                  # trigger block excluded, closing block included
    assert d.db_min == -5 and d.db_max == 25
    assert d.db_mean == np.mean(h) and d.db_std == np.std(h)
    assert thr[31] == thr[30] and thr[34] == thr[30]      # locked while tracking


def test_init_phase_ignores_pings():
    o = _noise(60)
    o[2] = 50                             # t0 = 0.4 s < init wait 1 s
    m, _, _ = L.live_detect_ref(_rows(o), FS, B, _cfg())
    assert all(d.time_start != 2 * B / FS for d in m)


def test_locked_threshold_held_after_tracking_then_fresh():
    o = _noise(120)
    o[30:33] = [30, 10, -10]              # history [10, -10]: mean 0 >= min_db -1
    m, thr, _ = L.live_detect_ref(_rows(o), FS, B, _cfg(after_tracking_wait_sec=2.0))
    assert any(d.time_start == 30 * B / FS and d.time_stop == 32 * B / FS for d in m)
    lock = thr[30]
    stop_t0 = 32 * B / FS
    for b in range(33, 60):
        t1 = (b * B + B) / FS
        if stop_t0 + 2.0 > t1:
            assert thr[b] == lock
        else:
            assert thr[b] != lock or np.isnan(lock)
            break


def test_filters_min_db_and_min_duration():
    o = _noise(80)
    o[30:33] = [20, 3, -9]                # short, low-mean ping
    m, _, _ = L.live_detect_ref(_rows(o), FS, B, _cfg(detection_db_over_noise_mean_min=5))
    assert all(d.time_start != 30 * B / FS for d in m)
    m, _, _ = L.live_detect_ref(_rows(o), FS, B, _cfg(detection_dur_min_sec=1.0))
    assert all(d.time_start != 30 * B / FS for d in m)


def test_zero_window_uses_whole_history():
    o = _noise(50)
    _, thr, over = L.live_detect_ref(_rows(o), FS, B, _cfg(avg_win_sec=0.1))  # int(0.1/0.2) = 0 → [-0:]
    assert int(0.1 / 0.2) == 0
    _, thr_full, _ = L.live_detect_ref(_rows(o), FS, B, _cfg(avg_win_sec=100.0))
    np.testing.assert_array_equal(thr[:20], thr_full[:20])


def test_tracking_until_end_emits_nothing():
    o = _noise(40)
    o[30:] = 40                           # never falls below the lock
    m, _, _ = L.live_detect_ref(_rows(o), FS, B, _cfg())
    assert all(d.time_start < 30 * B / FS for d in m)


@pytest.mark.parametrize("n1,n2", [(-np.inf, -np.inf), (-np.inf, 3.0)])
def test_silent_noise_band_gives_ieee_values(n1, n2):
    rows = np.stack([np.full(30, 2.0), np.full(30, n1), np.full(30, n2)])
    m, thr, over = L.live_detect_ref(rows, FS, B, _cfg())
    assert np.isinf(over).all()

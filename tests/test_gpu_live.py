"""GPU parity of the phase-2 live detector: the HIP Welch band powers
and state machine, called through the C-ABI, against the scipy golden and the oracle.

Bars: band dB within DB_TOL of scipy (float64 Goertzel vs pocketfft rounding); the state
machine bit-exact on identical band rows; end to end, identical detection blocks and
times, dB statistics within STAT_TOL."""
import math
import os

import numpy as np
import pytest

from oracle import live_oracle as L

pytestmark = pytest.mark.gpu

DB_TOL = 1e-9
STAT_TOL = 1e-9


@pytest.fixture(scope="module")
def live():
    from meteorgpu import live as LV
    return LV


def _ref_cfg(c):
    return L.ConfigDetectionRef(**{k: getattr(c, k) for k in L.ConfigDetectionRef.__dataclass_fields__})


def test_welch_band_db_golden(live, golden_dir):
    g = np.load(os.path.join(golden_dir, "live_4k.npz"))
    cfg = live.ConfigDetection(n_fft=int(g["n_fft"]), signal_freq=int(g["f0"]))
    got = live.welch_band_db(g["x"], int(g["fs"]), cfg, sample_scale=1 / 32768)
    assert got.shape == g["expected"].shape
    np.testing.assert_allclose(got, g["expected"], rtol=0, atol=DB_TOL)


@pytest.mark.parametrize("fs,bs,nfft,f0,dtype,width", [
    (4000, 0.2, 4096, 1000, np.int16, 100),
    (4000, 0.5, 4096, 1020, np.int16, 100),
    (4000, 0.2, 2048, 1025, np.float64, 100),
    (8000, 0.1, 1024, 1500, np.int16, 100),
    (4000, 0.05, 512, 1000, np.int16, 100),     # 200-sample blocks: nperseg capped at the block
    (4000, 0.2, 4096, 1000, np.int16, 400),  # 400 Hz channels: 410 bins, numpy's full pairwise tree
    (8000, 0.2, 4096, 2000, np.int16, 300),  # 154 bins
])
def test_welch_band_db_vs_oracle(live, fs, bs, nfft, f0, dtype, width):
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=int(fs * bs) + nfft, fs=fs, duration_s=6.0, f0=f0, sigma=500, rate_per_min=20)
    if dtype == np.float64:
        xin, sc = x.astype(np.float64) / 32768.0, 1.0
    else:
        xin, sc = x, 1 / 32768
    cfg = live.ConfigDetection(proc_block_sec=bs, n_fft=nfft, signal_freq=f0, channel_width=width,
                               noise_channel_offset=max(300, width + 50))
    got = live.welch_band_db(xin, fs, cfg, sample_scale=sc)
    ref = L.welch_band_db_ref(x.astype(np.float64) / 32768.0, fs, _ref_cfg(cfg))
    np.testing.assert_allclose(got, ref, rtol=0, atol=DB_TOL)


def test_state_machine_bit_exact_on_oracle_rows(live, golden_dir):
    g = np.load(os.path.join(golden_dir, "live_4k.npz"))
    cfg = live.ConfigDetection(n_fft=int(g["n_fft"]), signal_freq=int(g["f0"]),
                               detection_db_over_noise_mean_min=1, detection_dur_min_sec=0.5)
    rows = g["expected"]
    m, thr, over = live.live_detect(rows, int(g["fs"]), cfg)
    rm, rthr, rover = L.live_detect_ref(rows, int(g["fs"]), int(cfg.proc_block_sec * g["fs"]), _ref_cfg(cfg))
    np.testing.assert_array_equal(over, rover)
    np.testing.assert_array_equal(thr, rthr)                      # NaN positions included
    assert len(m) == len(rm) == 2
    for a, b in zip(m, rm):
        assert (a.time_start, a.time_stop, a.duration, a.db_min, a.db_max, a.db_mean, a.db_std) == \
               (b.time_start, b.time_stop, b.duration, b.db_min, b.db_max, b.db_mean, b.db_std)


@pytest.mark.parametrize("seed", [1, 2, 3, 4])
@pytest.mark.parametrize("kw", [dict(), dict(avg_win_sec=0.1), dict(after_tracking_wait_sec=0.0),
                                dict(detection_db_over_noise_mean_min=4, detection_dur_min_sec=0.4)])
def test_state_machine_random_rows(live, seed, kw):
    rng = np.random.default_rng(seed)
    nb = 600
    sig = rng.normal(0, 1, nb)
    for s in rng.integers(50, nb - 10, 12):
        sig[s:s + rng.integers(1, 8)] += rng.uniform(5, 30)
    rows = np.stack([sig, rng.normal(0, 0.5, nb), rng.normal(0, 0.5, nb)])
    cfg = live.ConfigDetection(**kw)
    m, thr, over = live.live_detect(rows, 4000, cfg)
    rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
    np.testing.assert_array_equal(thr, rthr)
    assert [(a.time_start, a.time_stop, a.db_min, a.db_max, a.db_mean, a.db_std) for a in m] == \
           [(b.time_start, b.time_stop, b.db_min, b.db_max, b.db_mean, b.db_std) for b in rm]


def test_state_machine_edge_rows(live):
    cfg = live.ConfigDetection(init_detection_wait_sec=0.0)
    for rows in (np.zeros((3, 0)), np.ones((3, 1)), np.stack([np.full(40, 1.0), np.full(40, -np.inf),
                                                                 np.full(40, -np.inf)])):
        m, thr, over = live.live_detect(rows, 4000, cfg)
        rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
        np.testing.assert_array_equal(thr, rthr)
        np.testing.assert_array_equal(over, rover)
        assert len(m) == len(rm)


def test_wav_file_process_end_to_end(live, tmp_path):
    from meteorgpu import synth, wav
    x, _ = synth.synth_real(seed=77, fs=4000, duration_s=90.0, f0=1020.0, sigma=300.0, rate_per_min=10,
                            band_hz=100.0, snr_db=(15, 30), dur_s=(0.4, 2.0))
    p = tmp_path / "live.wav"
    wav.write(p, 4000, x)
    cfg = live.ConfigDetection(proc_block_sec=0.2, n_fft=4096, detection_db_over_noise_mean_min=1,
                               detection_dur_min_sec=0.5, signal_freq=1020)
    got = live.wav_file_process(str(p), cfg, live.ConfigVisualization(enable_ui_plots=False),
                                live.ConfigSpecExport(output_dir=""))
    ref, _, _ = L.wav_file_process_ref(x.astype(np.float64) / 32768.0, 4000, _ref_cfg(cfg))
    assert len(ref) > 0 and len(got) == len(ref)
    # the near-tie guard (margin.py, live part): no decision within the bound, which is tiny
    assert not got.near_tie and 0 < got.decision_bound < 1e-6 and got.min_margin > got.decision_bound
    for a, b in zip(got, ref):
        assert (a.time_start, a.time_stop, a.duration) == (b.time_start, b.time_stop, b.duration)
        for f in ("db_min", "db_max", "db_mean", "db_std"):
            assert math.isclose(getattr(a, f), getattr(b, f), rel_tol=STAT_TOL, abs_tol=STAT_TOL)


def test_wav_file_process_asserts(live, tmp_path):
    from meteorgpu import wav
    p = tmp_path / "a.wav"
    wav.write(p, 6000, np.zeros(6000, np.int16))
    with pytest.raises(AssertionError, match="Invalid Sample Rate: 6000"):
        live.wav_file_process(str(p), live.ConfigDetection(), live.ConfigVisualization(enable_ui_plots=False),
                              live.ConfigSpecExport())
    with pytest.raises(NotImplementedError):
        live.wav_file_process(str(p), live.ConfigDetection(), live.ConfigVisualization(),
                              live.ConfigSpecExport(), required_sample_rate=None)


def test_live_batch_matches_single(live):
    from meteorgpu import _lib, synth
    from meteorgpu.dsp import context
    cfg = live.ConfigDetection(detection_db_over_noise_mean_min=1, detection_dur_min_sec=0.4)
    xs = [synth.synth_real(seed=900 + i, fs=4000, duration_s=60.0, f0=1000.0, sigma=300.0, rate_per_min=12,
                           band_hz=100.0, snr_db=(15, 30), dur_s=(0.4, 2.0))[0] for i in range(5)]
    lb = live.LiveBatch(context(0), len(xs), len(xs[0]), 4000, cfg)
    for i, x in enumerate(xs):
        lb.upload_file(i, x)
    lb.run()
    bdb = lb.band_db()
    rows, counts = lb.meteors()
    for i, x in enumerate(xs):
        single = live.welch_band_db(x, 4000, cfg, sample_scale=1 / 32768)
        np.testing.assert_array_equal(bdb[i], single)
        m, _, _ = live.live_detect(single, 4000, cfg)
        assert counts[i] == len(m)
        assert [(r["time_start"], r["time_stop"], r["db_mean"]) for r in rows[i]] == \
               [(a.time_start, a.time_stop, a.db_mean) for a in m]
    assert counts.sum() > 0
    import warnings
    from meteorgpu import margin as M
    with warnings.catch_warnings():
        warnings.simplefilter("error", M.NearTieWarning)
        assert not lb.check_near_ties().any()
    assert (lb.decision_bounds > 0).all() and (lb.decision_bounds < 1e-6).all()
    assert (lb.min_margins > lb.decision_bounds).all()
    lb.span[1] = np.inf  # a bound too wide to separate anything: that file is flagged
    with pytest.warns(M.NearTieWarning, match="1 file"):
        lb.check_near_ties()
    assert lb.near_tie.tolist() == [False, True, False, False, False]


@pytest.mark.parametrize("fs,bs,nfft,f0", [(4000, 0.2, 4096, 1000), (8000, 0.1, 1024, 1500),
                                           (4000, 0.05, 512, 1000), (4000, 0.5, 4096, 1020)])
def test_over_noise_within_bound(live, fs, bs, nfft, f0):
    """the device's over-noise values (processor.py:391) against scipy's within the per-block
    bound of margin.live_over_error, on a stream with a DC-offset stretch and digital silence"""
    from meteorgpu import margin as M, synth
    x, _ = synth.synth_real(seed=int(fs * bs) + nfft + 5, fs=fs, duration_s=20.0, f0=f0, sigma=300, rate_per_min=20)
    x[: 3 * fs] = np.clip(x[: 3 * fs].astype(np.int32) + 20000, -32768, 32767)
    x[5 * fs: 7 * fs] = 0
    cfg = live.ConfigDetection(proc_block_sec=bs, n_fft=nfft, signal_freq=f0)
    bdb = live.welch_band_db(x, fs, cfg, sample_scale=1 / 32768)
    _, thr, over = live.live_detect(bdb, fs, cfg)
    ref = L.welch_band_db_ref(x.astype(np.float64) / 32768.0, fs, _ref_cfg(cfg))
    _, _, rover = L.live_detect_ref(ref, fs, int(bs * fs), _ref_cfg(cfg))
    c, win = live.welch_cfg(fs, cfg)
    span = M.block_span(x, int(c.block_size), 1 / 32768)[: bdb.shape[1]]
    err = M.live_over_error(bdb, block_size=int(c.block_size), nperseg=int(c.nperseg), noverlap=int(c.noverlap),
                            nfft=int(c.nfft), window=win, span=span,
                            bands=[(int(c.band_lo[j]), int(c.band_hi[j])) for j in range(3)], scale=float(c.scale))
    fin = np.isfinite(rover)
    assert np.array_equal(np.isfinite(over), fin) and (~fin).any()  # the silent blocks: NaN on both sides
    d = np.abs(over[fin] - rover[fin])
    # (the int8 path often matches scipy's float64 values exactly: d = 0 is a pass, not a vacuous test)
    assert (d <= err[fin]).all(), float(np.max(d / err[fin]))
    assert err[fin].max() < 1e-6  # not vacuous


@pytest.mark.parametrize("wait,dur", [(200.0, 60), (30.0, 400), (0.0, 1000)])
def test_state_machine_states_across_many_segments(live, wait, dur):
    """the whole-GPU state machine (128-block segments, rounds of scan / link): a lock held for
    1000 blocks after tracking, tracking runs of 400 and 1000 blocks -- a segment's entry then
    depends on states set 8+ segments earlier, so the rounds go past the first four and the
    convergence flag is read more than once; bit-exact against the oracle"""
    rng = np.random.default_rng(int(wait) + dur)
    nb = 9000
    sig = rng.normal(0, 1, nb)
    for s in (300, 2100, 5050, 7777):
        sig[s:s + dur] += 30
    rows = np.stack([sig, rng.normal(0, 0.5, nb), rng.normal(0, 0.5, nb)])
    cfg = live.ConfigDetection(after_tracking_wait_sec=wait)
    m, thr, over = live.live_detect(rows, 4000, cfg)
    rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
    np.testing.assert_array_equal(over, rover)
    np.testing.assert_array_equal(thr, rthr)
    got = [(a.time_start, a.time_stop, a.db_min, a.db_max, a.db_mean, a.db_std) for a in m]
    assert got == [(b.time_start, b.time_stop, b.db_min, b.db_max, b.db_mean, b.db_std) for b in rm]
    assert len(m) >= 1


def test_state_machine_long_rows_cross_chunks(live):
    """nb > the kernel's 2048-block LDS chunk: runs and histories straddling chunk edges."""
    rng = np.random.default_rng(11)
    nb = 5000
    sig = rng.normal(0, 1, nb)
    for s in (2040, 2046, 4093, 3000, 100, 4999 - 3):
        sig[s:s + 5] += 25
    rows = np.stack([sig, rng.normal(0, 0.5, nb), rng.normal(0, 0.5, nb)])
    cfg = live.ConfigDetection(after_tracking_wait_sec=0.4)
    m, thr, over = live.live_detect(rows, 4000, cfg)
    rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
    np.testing.assert_array_equal(thr, rthr)
    got = [(a.time_start, a.time_stop, a.db_min, a.db_max, a.db_mean, a.db_std) for a in m]
    assert got == [(b.time_start, b.time_stop, b.db_min, b.db_max, b.db_mean, b.db_std) for b in rm]
    assert any(2040 * 0.2 <= a.time_start <= 2050 * 0.2 for a in m)


@pytest.mark.parametrize("n,nperseg", [(48000, 4096), (3000, 4096), (20000, 256)])
def test_welch_psd_whole_signal_vs_scipy(live, n, nperseg):
    """live.welch_psd = scipy.signal.welch(x, fs, 'hann', nperseg, nperseg//2, nfft) over a whole
    float64 signal (the figure export's PSD panel, main.py:88-90); nperseg capped at len(x)."""
    import warnings
    from scipy.signal import welch
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n) * 0.1 + 0.5 * np.sin(2 * np.pi * 1000 * np.arange(n) / 6000)
    f, P = live.welch_psd(x, 6000, nperseg=nperseg, noverlap=nperseg // 2, nfft=nperseg)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        rf, rP = welch(x, 6000, window="hann", nperseg=nperseg, noverlap=nperseg // 2, nfft=nperseg)
    np.testing.assert_array_equal(f, rf)
    assert np.linalg.norm(P - rP) <= 1e-9 * np.linalg.norm(rP)


def test_proc_wav_file_exports_detection_figures(tmp_path):
    """disable_show_and_write=False (main.py:721-806): one spec_and_psd PNG per detection in a
    fresh timestamped directory under outfile_path."""
    from meteorgpu import dsp, synth, wav
    x, _ = synth.synth_real(seed=5, fs=6000, duration_s=60.0, f0=1003.0, rate_per_min=10, band_hz=20.0,
                            snr_db=(20, 35))
    p = tmp_path / "a.wav"
    wav.write(p, 6000, x)
    out = tmp_path / "spec_export"
    out.mkdir()
    res = dsp.proc_wav_file(str(p), 0.2, (993, 1013), (690, 710), 512, 4, outfile_path=str(out) + "/x",
                            disable_show_and_write=False, verbose=False)
    pngs = sorted(out.glob("x/*/spec_and_psd_*.png"))
    assert len(res.detections) > 0 and len(pngs) == len(res.detections)
    assert all(q.stat().st_size > 10000 for q in pngs)


@pytest.mark.parametrize("nb", [17, 100, 1601, 20000])
@pytest.mark.parametrize("kw", [dict(), dict(after_tracking_wait_sec=30.0), dict(init_detection_wait_sec=0.0),
                                dict(avg_win_sec=0.4, detection_dur_min_sec=0.2)])
def test_state_machine_segments(live, nb, kw):
    """the kernel splits each file into 16 time segments scanned in parallel to a fixed point:
    bursts and long plateaus on and across the segment edges (tracking and post-tracking locks
    carried over one or several edges), bit-exact with the oracle"""
    rng = np.random.default_rng(nb)
    sig = rng.normal(0, 1, nb)
    seg = -(-nb // 16)
    for e in range(seg, nb, seg):  # a burst straddling every edge, some long enough to span segments
        L_ = int(rng.choice([1, 3, seg // 2 + 1, 2 * seg + 1]))
        sig[max(0, e - 2): e - 2 + L_] += rng.uniform(8, 30)
    for s in rng.integers(0, nb, max(1, nb // 50)):
        sig[s: s + rng.integers(1, 10)] += rng.uniform(5, 30)
    rows = np.stack([sig, rng.normal(0, 0.5, nb), rng.normal(0, 0.5, nb)])
    cfg = live.ConfigDetection(**kw)
    m, thr, over = live.live_detect(rows, 4000, cfg)
    rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
    np.testing.assert_array_equal(thr, rthr)
    assert [(a.time_start, a.time_stop, a.db_min, a.db_max, a.db_mean, a.db_std) for a in m] == \
           [(b.time_start, b.time_stop, b.db_min, b.db_max, b.db_mean, b.db_std) for b in rm]

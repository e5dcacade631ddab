"""The near-tie guard (meteorgpu/margin.py): a bound on |delta_gpu - delta_numpy| and the flag
raised when a detector decision (main.py:406, :485 strict '>') lies within it.

CPU: the pocketfft half of the per-bin bound against an exact (long double) DFT on random and
adversarial blocks; the decision bound's flag on a constructed near-tie delta.
GPU: the device's delta against numpy's within the per-block bound on random files; the flag
in ProcResult and BatchPipeline.detections()."""
import warnings

import numpy as np
import pytest

from meteorgpu import margin as M
from oracle import dsp_oracle as O


def _exact_bins(xw, nfft, bins):
    """DFT of the windowed block at the given bins in long double (x86 80-bit)."""
    n = np.arange(len(xw), dtype=np.longdouble)
    out = []
    for k in bins:
        ang = -2 * np.pi * np.longdouble(k) * n / np.longdouble(nfft)
        out.append(np.sum(xw.astype(np.longdouble) * (np.cos(ang) + 1j * np.sin(ang))))
    return np.array(out)


@pytest.mark.parametrize("seed,offset,scale", [(0, 0, 1000), (1, 30000, 10), (2, -32768, 1), (3, 0, 32767)])
def test_pocketfft_within_bin_bound(seed, offset, scale):
    rng = np.random.default_rng(seed)
    B, nfft = 1200, 1024
    x = np.clip(offset + scale * rng.standard_normal(B), -32768, 32767).astype(np.int16)
    w = np.hanning(B)
    xw = (x * w)[:nfft]
    X = np.fft.rfft(x * w, n=nfft)
    bins = np.array([0, 1, 2, 170, 171, 172, 300, 511, 512])
    exact = _exact_bins(xw, nfft, bins)
    S = float(np.abs(x).max()) * float(w[:nfft].sum())
    bound = M._chain(nfft, nfft, bins, float(w[:nfft].sum())) * M.U * S
    err = np.abs(X[bins].astype(np.clongdouble) - exact).astype(np.float64)
    assert (err <= bound).all() and err.max() > 0


def test_band_db_error_monotone_and_infinite_for_empty_energy():
    e = np.array([-120.0, 0.0, 60.0, 100.0])
    b = M.band_db_error(e, 3, 1e-3)
    assert np.isinf(b[0]) and (np.diff(b[1:]) < 0).all()
    assert (M.band_db_error(e, 0, 1.0) == 0).all()  # empty band: E = 1e-12 on both sides


def test_flag_on_constructed_near_tie():
    """a block placed one ulp above its adaptive threshold (main.py:474-485) is a near tie for
    any positive bound; a block 1 dB away is not"""
    rng = np.random.default_rng(7)
    d = rng.normal(0, 1, 3000)
    dets, thr = O.get_detections_adaptive_ref(d, 4.0, 0.2)
    i = 2000
    d[i] = np.nextafter(thr[i], np.inf)  # thr[i] only depends on d[i-600:i]
    dets2, thr2 = O.get_detections_adaptive_ref(d, 4.0, 0.2)
    assert thr2[i] == thr[i] and any(t0 <= i * 0.2 < t1 for t0, t1, *_ in dets2)
    margin = abs(d[i] - thr2[i])
    with pytest.warns(M.NearTieWarning):
        assert M.check(margin, M.decision_bound(np.full(3000, 1e-12), 4.0))
    with warnings.catch_warnings():
        warnings.simplefilter("error")
        assert not M.check(1.0, M.decision_bound(np.full(3000, 1e-12), 4.0))


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
@pytest.mark.parametrize("fs,bs,n_fft,band,noise", [(6000, 0.2, 512, (993, 1013), (690, 710)),
                                                    (48000, 0.2, 512, (950, 1050), (2950, 3050)),
                                                    (6000, 0.1, 256, (980, 1020), (0, 40))])
def test_device_delta_within_bound(fs, bs, n_fft, band, noise):
    from meteorgpu import dsp, synth
    for seed in range(3):
        x, _ = synth.synth_real(seed=400 + seed, fs=fs, duration_s=60.0, f0=1000.0, rate_per_min=10)
        x[: fs * 5] = np.clip(x[: fs * 5].astype(np.int32) + 20000, -32768, 32767)  # a DC-offset stretch
        b, nz, d, B = dsp.block_powers(x, fs, bs, band, noise, n_fft)
        rb, rn, rd = O.block_powers_ref(x, fs, bs, band, noise, n_fft)
        nfft = 2 * n_fft
        L = min(B, nfft)
        err = M.delta_error_bound(b, nz, nfft=nfft, L=L, window=dsp.hanning_sym(B)[:L],
                                  xmax=float(np.abs(x.astype(np.float64)).max()),
                                  band=dsp.band_bins(nfft, fs, band), noise=dsp.band_bins(nfft, fs, noise))
        assert (np.abs(d - rd) <= err).all()
        assert err.max() < 1e-6  # the bound is useful: far below any real decision margin


@pytest.mark.gpu
def test_proc_result_and_batch_flags():
    from meteorgpu import dsp, synth
    from meteorgpu.batch import BatchPipeline
    x, _ = synth.synth_real(seed=9, fs=6000, duration_s=120.0, f0=1003.0, band_hz=20.0, rate_per_min=10)
    with warnings.catch_warnings():
        warnings.simplefilter("error", M.NearTieWarning)
        res = dsp.process_samples(x, 6000, 0.2, (993, 1013), (690, 710), 512, 4)
    assert 0 < res.decision_bound < 1e-6 and res.min_margin > res.decision_bound and not res.near_tie
    bp = BatchPipeline(dsp.context(0), 3, len(x), 6000, freq_band=(993, 1013), noise_band=(690, 710),
                       with_spectrogram=False)
    for i in range(3):
        bp.upload_file(i, x)
    bp.run()
    bp.detections()
    assert not bp.near_tie.any() and np.allclose(bp.decision_bounds, res.decision_bound, rtol=1e-12)
    bp.xmax[1] = np.inf  # a bound too wide to separate anything: that file is flagged
    with pytest.warns(M.NearTieWarning, match="1 file"):
        bp.detections()
    assert bp.near_tie.tolist() == [False, True, False]


# ------------------------------------------------------------------ live detector (margin.py, live part)
def test_welch_pocketfft_within_bin_bound():
    """scipy.signal.welch's segment transform (detrend, periodic Hann, rfft zero-padded to nfft)
    against an exact long-double DFT at the live bands' bins: within c_fft u S, S <= span sum w"""
    from scipy.signal import get_window
    rng = np.random.default_rng(21)
    nperseg, nfft = 256, 4096
    w = get_window("hann", nperseg)
    bins = np.r_[972:1075, 665:768, 1279:1382]  # 1000 Hz +- 50 and the two noise bands at fs 4 kHz
    for offset, scale in ((0.0, 0.3), (0.9, 0.05), (-0.5, 1e-4)):
        x = np.clip(offset + scale * rng.standard_normal(nperseg), -1, 1)
        d = x - np.mean(x)
        X = np.fft.rfft(w * d, n=nfft)
        exact = _exact_bins(w * d, nfft, bins)
        S = float(x.max() - x.min()) * float(w.sum())
        bound = (4.0 * np.log2(nfft) + 8.0) * M.U * S
        err = np.abs(X[bins].astype(np.clongdouble) - exact).astype(np.float64)
        assert (err <= bound).all() and err.max() > 0


def test_welch_band_db_error_edges():
    e = np.array([-np.inf, -120.0, -20.0])
    b = M.welch_band_db_error(e, 103, np.array([0.0, 1e-14, 1e-14]), 2.6e-6, 5)
    assert b[0] == 0.0 and np.isfinite(b[1]) and b[2] < b[1]  # silence: exact on both sides
    assert np.isinf(M.welch_band_db_error(np.array([-np.inf]), 103, 1e-14, 2.6e-6, 5))[0]
    assert (M.welch_band_db_error(e, 0, 1.0, 2.6e-6, 5) == 0).all()


def test_live_flag_on_constructed_near_tie():
    """a block in the Detection state placed one ulp above its history threshold (processor.py
    :397-402, :464) is a near tie for the live guard; the unmodified rows are not"""
    from meteorgpu import live as LV
    from oracle import live_oracle as L
    rng = np.random.default_rng(5)
    nb = 900
    rows = np.stack([rng.normal(-30, 1, nb), rng.normal(-40, 0.5, nb), rng.normal(-40, 0.5, nb)])
    cfg = LV.ConfigDetection()
    rcfg = L.ConfigDetectionRef()
    span = np.full(nb, 0.1)

    def check(r):
        _, thr, over = L.live_detect_ref(r, 4000, 800, rcfg)
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", M.NearTieWarning)
            return LV.near_tie_check(r, thr, over, span, 4000, cfg), thr, over

    (near, m, bound), thr, over = check(rows)
    assert not near and 0 < bound < 1e-8 and m > bound
    i = 600
    assert np.isfinite(thr[i]) and over[i] < thr[i]
    mean_n = np.mean([rows[1, i], rows[2, i]])
    s = thr[i] + mean_n
    while s - mean_n <= thr[i]:
        s = np.nextafter(s, np.inf)
    r2 = rows.copy()
    r2[0, i] = s  # db2 = sig - mean(n1, n2) a few ulp above the threshold: a trigger
    (near2, m2, bound2), thr2, over2 = check(r2)
    assert thr2[i] == thr[i] and over2[i] > thr2[i] and near2 and m2 <= bound2
    with pytest.warns(M.NearTieWarning):
        _, thr3, over3 = L.live_detect_ref(r2, 4000, 800, rcfg)
        LV.near_tie_check(r2, thr3, over3, span, 4000, cfg)


def test_batched_bounds_equal_per_file_loop():
    """delta_error_bounds / decision_bounds (BatchPipeline's one vectorised pass over a batch) equal
    delta_error_bound / decision_bound file by file, empty bands and zero-amplitude files included"""
    rng = np.random.default_rng(11)
    F, nb, L = 6, 40, 1024
    win = np.hanning(9600)[:L]
    band = rng.uniform(-40.0, 60.0, (F, nb))
    noise = rng.uniform(-40.0, 60.0, (F, nb))
    band[2, 5] = -120.0  # E = 1e-12
    xmax = np.array([4000.0, 32768.0, 1.0, 0.0, 123.0, 32767.0])
    for bb, nn in (((170, 172), (118, 121)), ((170, 172), (0, -1)), ((0, -1), (0, -1))):
        err = M.delta_error_bounds(band, noise, nfft=1024, L=L, window=win, xmax=xmax, band=bb, noise=nn)
        got = M.decision_bounds(err, 4.0)
        for i in range(F):
            e1 = M.delta_error_bound(band[i], noise[i], nfft=1024, L=L, window=win, xmax=xmax[i], band=bb, noise=nn)
            np.testing.assert_array_equal(err[i], e1)
            assert got[i] == M.decision_bound(e1, 4.0)

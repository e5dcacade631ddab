"""The live detector's Welch band powers for int16 audio on the exact integer path
(csrc/welch_i8.hip: the segment detrend folded into the coefficients c'_n = w_n e^{-i theta n} - W/L,
each quantised to 2^-53 in seven balanced base-256 digits, one int8 GEMM on the matrix cores) against
scipy (oracle/live_oracle.py, processor.py:206, :349-369) and against the float64 Goertzel path it
replaces by default (MSD_OPT_WELCH_GOERTZEL).

CPU: the path's arithmetic restated with Python integers (exact digit sums) stays within margin.py's
int8 term of the exact detrended DFT, the zero-sum rounding makes the offset term vanish, and the
digits reconstruct every coefficient.
GPU: band dB within 1e-9 of scipy and of the Goertzel path over the shapes the path takes (nperseg
64-512, 1-16 segments per block, several bands and widths), DC offsets, digital silence, full
scale, files at odd offsets and a ragged batch; the psd output; the over-noise bound."""
import numpy as np
import pytest

from meteorgpu import margin as M
from oracle import live_oracle as L

PI_LD = np.longdouble("3.14159265358979323846264338327950288")


def _coeffs(w, k, nfft):
    """c'_n = w_n e^{-2 pi i k n / nfft} - W_k / L in long double (re, im)"""
    L = len(w)
    a = 2 * PI_LD * ((int(k) * np.arange(L, dtype=np.int64)) % int(nfft)).astype(np.longdouble) / np.longdouble(nfft)
    wl = w.astype(np.longdouble)
    cr, ci = wl * np.cos(a), -wl * np.sin(a)
    return cr - cr.sum() / L, ci - ci.sum() / L


def _zero_sum_round(v):
    """welch_i8_build's rounding: T_n = floor(v_n 2^53), the largest remainders rounded up so that
    sum T_n = 0 exactly (the offset term 128 sum T_n of x = 256 h + l' + 128 vanishes)"""
    s = v * np.longdouble(2.0 ** 53)
    f = np.floor(s)
    T = [int(a) for a in f.astype(np.int64)]
    frac = s - f
    R = -sum(T)
    assert 0 <= R <= len(T)
    for n in sorted(range(len(T)), key=lambda n: -frac[n])[:R]:  # stable: ties in index order
        T[n] += 1
    return T


def _digits7(T):
    d = []
    for _ in range(7):
        r = T % 256
        if r >= 128:
            r -= 256
        d.append(r)
        T = (T - r) // 256
    assert T == 0
    return d[::-1]  # d_0 (most significant) .. d_6


@pytest.mark.parametrize("case", ["noise", "dc", "full_scale"])
def test_folded_detrend_quantisation_within_bound(case):
    rng = np.random.default_rng({"noise": 1, "dc": 2, "full_scale": 3}[case])
    L, nfft = 256, 4096
    if case == "noise":
        x = rng.normal(0, 300, L)
    elif case == "dc":
        x = 25000 + rng.normal(0, 5, L)
    else:
        x = rng.choice([-32768, 32767], L)
    x = np.clip(np.round(x), -32768, 32767).astype(np.int64)
    w = np.hanning(L + 1)[:-1]  # scipy get_window('hann', 256): periodic
    absx = float(np.abs(x).sum())
    for k in (0, 1, 100, 1024, 1025, 2048):
        cr, ci = _coeffs(w, k, nfft)
        Tr, Ti = _zero_sum_round(cr), _zero_sum_round(ci)
        assert sum(Tr) == 0 and sum(Ti) == 0
        two53 = np.longdouble(2.0 ** 53)
        assert max(abs(np.longdouble(t) - c * two53) for t, c in zip(Tr + Ti, list(cr) + list(ci))) < 1
        for T in Tr[:8] + Ti[:8]:
            d = _digits7(T)
            assert sum(di * 256 ** (6 - b) for b, di in enumerate(d)) == T
        re = sum(int(a) * b for a, b in zip(x, Tr))
        im = sum(int(a) * b for a, b in zip(x, Ti))
        # the kernel's accumulators hold the products with x - 128 (h and the offset-binary l'): the
        # same sums, since the T sum to zero
        assert re == sum((int(a) - 128) * b for a, b in zip(x, Tr))
        assert im == sum((int(a) - 128) * b for a, b in zip(x, Ti))
        # the exact detrended DFT: sum (x - mean) w e^{-i theta n}
        xm = x.astype(np.longdouble) - x.astype(np.longdouble).sum() / L
        a = 2 * PI_LD * ((k * np.arange(L, dtype=np.int64)) % nfft).astype(np.longdouble) / np.longdouble(nfft)
        er, ei = np.sum(xm * w * np.cos(a)), -np.sum(xm * w * np.sin(a))
        got_r = np.longdouble(re) / np.longdouble(2.0 ** 53)
        got_i = np.longdouble(im) / np.longdouble(2.0 ** 53)
        err = float(np.hypot(got_r - er, got_i - ei))
        assert err <= 1.5 * M.U * absx  # the quantisation: |T - c' 2^53| < 1, 2^-53 sum |x| per part
        assert err <= M.I8_WELCH * M.U * L * float(np.abs(x).max())


def _pair_bound(w, bins, nfft):
    """max over the plan's components and w = 0, 2, 4, 6 of (|a_w| + 256 |a_(w+1)|) / 2^31, the
    accumulators bounded by 128 (sum_n |d_(7-w)n| + sum_n |d_(6-w)n|) (welch_i8_build)"""
    worst = 0.0
    for k in bins:
        for comp in _coeffs(w, k, nfft):
            sad = np.abs(np.array([_digits7(t) for t in _zero_sum_round(comp)])).sum(axis=0)
            b = [128 * ((sad[7 - i] if i >= 1 else 0) + (sad[6 - i] if i <= 6 else 0)) for i in range(8)]
            worst = max(worst, max((b[i] + 256 * b[i + 1]) / 2 ** 31 for i in range(0, 8, 2)))
    return worst


def test_pair_bound_live_default():
    """the live default plan (nperseg 256, 309 band bins) combines its accumulators in int32 pairs:
    every pair's bound is below 2^31 (0.54 of it); at nperseg 512 the bound exceeds 2^31, so the
    GPU sweep's nperseg-512 case runs the eight-term digit sum"""
    w = np.hanning(257)[:-1]
    bins = list(range(870, 973)) + list(range(1175, 1278)) + list(range(460, 563))
    assert _pair_bound(w, bins[::8], 4096) < 0.75
    assert _pair_bound(np.hanning(513)[:-1], list(range(1850, 2160, 31)), 4096) > 1.0


# ----------------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def live():
    from meteorgpu import live as LV
    return LV


def _ref_cfg(c):
    return L.ConfigDetectionRef(**{k: getattr(c, k) for k in L.ConfigDetectionRef.__dataclass_fields__})


def _plan_cfg(live, fs, bs, nfft, f0, width, nperseg):
    """msd_welch_cfg + window for a given nperseg (noverlap nperseg // 2, scipy's default)"""
    from meteorgpu import dsp
    cfg = live.ConfigDetection(proc_block_sec=bs, n_fft=nfft, signal_freq=f0, channel_width=width,
                               noise_channel_offset=max(300, width + 50))
    c, _ = live.welch_cfg(fs, cfg, 1 / 32768)
    win = dsp.hann_periodic(nperseg)
    c.nperseg, c.noverlap = nperseg, nperseg // 2
    wc = win.astype(np.complex128)
    c.scale = float(np.real(1.0 / (fs * (wc * wc).sum())))
    return c, win


def _run(c, win, x, goertzel):
    from meteorgpu import _lib, dsp
    ctx = dsp.context(0)
    plan = _lib.WelchPlan(ctx, c, win)
    ctx.set_option(_lib.OPT_WELCH_GOERTZEL, int(goertzel))
    try:
        return plan.run(np.ascontiguousarray(x))
    finally:
        ctx.set_option(_lib.OPT_WELCH_GOERTZEL, 0)
        plan.close()


def _scipy_band_db(x, fs, c):
    """processor.py:206, :349-369 with scipy.signal.welch at the plan's nperseg, per block"""
    from scipy.signal import welch
    B = int(c.block_size)
    nb = (len(x) - B) // B + 1
    out = np.empty((3, nb))
    for b in range(nb):
        _, P = welch(x[b * B:(b + 1) * B].astype(np.float64) / 32768.0, fs, nperseg=int(c.nperseg),
                     noverlap=int(c.noverlap), nfft=int(c.nfft))
        for j in range(3):
            e = np.sum(P[int(c.band_lo[j]): int(c.band_hi[j]) + 1])
            out[j, b] = 10 * np.log10(e) if e > 0 else -np.inf
    return out


def _stress(x, fs):
    """a DC-offset stretch, digital silence, full-scale square, a near-full-scale offset"""
    x = x.copy()
    x[: 2 * fs] = np.clip(x[: 2 * fs].astype(np.int32) + 20000, -32768, 32767)
    x[3 * fs: 4 * fs] = 0
    x[5 * fs: 5 * fs + fs // 2] = np.where(np.arange(fs // 2) % 7 < 3, 32767, -32768)
    x[6 * fs: 7 * fs] = np.clip(x[6 * fs: 7 * fs].astype(np.int32) - 30000, -32768, 32767)
    return x


@pytest.mark.gpu
@pytest.mark.parametrize("fs,bs,nfft,f0,width,nperseg", [
    (4000, 0.2, 4096, 1000, 100, 256),   # the live default: 5 segments, 3 x 103 bins (39 column tiles)
    (4000, 0.5, 4096, 1020, 100, 256),   # 14 segments per block: one block per 16-row tile
    (8000, 0.1, 1024, 1500, 100, 256),   # 5 segments, 13-bin bands
    (4000, 0.2, 4096, 1000, 400, 256),   # 410-bin bands (> 128: numpy's full pairwise tree)
    (4000, 0.2, 2048, 900, 100, 128),    # nperseg 128 (2 K steps), 11 segments
    (4000, 0.2, 2048, 900, 100, 64),     # nperseg 64 (1 K step), 24 segments: > 16, the Goertzel
    (4000, 0.1, 2048, 900, 100, 64),     # nperseg 64, 11 segments
    (8000, 0.2, 4096, 2000, 300, 512),   # nperseg 512 (8 K steps), 5 segments, 154 bins
])
def test_welch_i8_vs_scipy_and_goertzel(live, fs, bs, nfft, f0, width, nperseg):
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=fs + nperseg + width, fs=fs, duration_s=9.0, f0=f0, sigma=400, rate_per_min=30)
    x = _stress(x, fs)
    c, win = _plan_cfg(live, fs, bs, nfft, f0, width, nperseg)
    got, gz = _run(c, win, x, False), _run(c, win, x, True)
    ref = _scipy_band_db(x, fs, c)
    assert got.shape == ref.shape == gz.shape
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin) and np.array_equal(np.isfinite(gz), fin)
    np.testing.assert_allclose(got[fin], ref[fin], rtol=0, atol=1e-9)
    np.testing.assert_allclose(got[fin], gz[fin], rtol=0, atol=1e-9)
    nseg = (int(c.block_size) - nperseg) // (nperseg - nperseg // 2) + 1
    # the int8 path ran where it applies (it rounds differently from the Goertzel), not elsewhere
    assert np.array_equal(got, gz) == (nseg > 16)


@pytest.mark.gpu
def test_welch_i8_ragged_batch_and_psd(live):
    """a batch of files of different lengths at odd offsets (the int8 kernel's row loads unaligned,
    tiles spanning files, blocks past a file's end untouched) through LiveBatch's plan, and the psd
    output against scipy's Welch PSD of each block"""
    from meteorgpu import _lib, dsp, synth
    fs = 4000
    cfg = live.ConfigDetection(proc_block_sec=0.2, n_fft=4096, signal_freq=1000)
    c, win = live.welch_cfg(fs, cfg, 1 / 32768)
    ctx = dsp.context(0)
    plan = _lib.WelchPlan(ctx, c, win)
    rng = np.random.default_rng(9)
    lens = [int(v) for v in (0, 799, 800, 801, 4000 * 3 + 13, 1601, 4000 * 2, 12345)]
    files = [synth.synth_real(seed=40 + i, fs=fs, duration_s=max(n, 1) / fs + 1, f0=1000.0, sigma=300,
                              rate_per_min=30)[0][:n] for i, n in enumerate(lens)]
    offs, pos = [], 3
    for n in lens:
        offs.append(pos)
        pos += n + int(rng.integers(1, 4))
    buf = np.zeros(pos + 16, np.int16)
    for o, f in zip(offs, files):
        buf[o: o + f.size] = f
    B = int(c.block_size)
    nbs = [(n - B) // B + 1 if n >= B else 0 for n in lens]
    max_blocks = max(nbs)
    ld = max_blocks + 2
    nf = len(lens)
    nslots = sum(int(c.band_hi[j]) - int(c.band_lo[j]) + 1 for j in range(3))
    d_x, d_off, d_len = ctx.alloc(2 * buf.size), ctx.alloc(8 * nf), ctx.alloc(8 * nf)
    d_db, d_psd = ctx.alloc(8 * nf * 3 * ld), ctx.alloc(8 * nf * ld * nslots)
    try:
        d_x.upload(buf)
        d_off.upload(np.array(offs, np.int64))
        d_len.upload(np.array(lens, np.int64))
        d_db.upload(np.full(nf * 3 * ld, -777.0))
        plan.run_dev(d_x, np.int16, d_off, d_len, nf, max_blocks, d_db, ld, psd=d_psd)
        ctx.synchronize()
        db = d_db.download(np.empty((nf, 3, ld), np.float64))
        psd = d_psd.download(np.empty((nf, ld, nslots), np.float64))
    finally:
        plan.close()
        for b in (d_x, d_off, d_len, d_db, d_psd):
            b.free()
    from scipy.signal import welch
    for i, f in enumerate(files):
        k = nbs[i]
        assert (db[i, :, k:] == -777.0).all()
        if k == 0:
            continue
        ref = L.welch_band_db_ref(f.astype(np.float64) / 32768.0, fs, _ref_cfg(cfg))
        np.testing.assert_allclose(db[i, :, :k], ref, rtol=0, atol=1e-9)
        sl = np.concatenate([np.arange(int(c.band_lo[j]), int(c.band_hi[j]) + 1) for j in range(3)])
        for b in (0, k - 1):
            _, P = welch(f[b * B:(b + 1) * B].astype(np.float64) / 32768.0, fs, nfft=int(c.nfft))
            np.testing.assert_allclose(psd[i, b], P[sl], rtol=1e-9, atol=0)


@pytest.mark.gpu
def test_welch_i8_pairs_bit_identical(live, monkeypatch):
    """the int32-pair digit combination (the default plan's) and the eight-term one give the same
    float64 values: both round the exact digit sum once; so do the live default's own instantiation
    (5 segments, folded scale) and the generic one"""
    from meteorgpu import synth
    fs = 4000
    x, _ = synth.synth_real(seed=77, fs=fs, duration_s=9.0, f0=1000, sigma=400, rate_per_min=30)
    x = _stress(x, fs)
    c, win = _plan_cfg(live, fs, 0.2, 4096, 1000, 100, 256)
    got = _run(c, win, x, False)
    monkeypatch.setenv("MSD_WELCH_I8_NOPAIRS", "1")
    ref = _run(c, win, x, False)
    assert np.array_equal(got, ref)
    # and the generic instantiation (runtime segment count) against the live default's own
    monkeypatch.setenv("MSD_WELCH_I8_GENERIC", "1")
    assert np.array_equal(_run(c, win, x, False), ref)
    np.testing.assert_allclose(got[np.isfinite(got)], _scipy_band_db(x, fs, c)[np.isfinite(got)], rtol=0, atol=1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [1 / 30000.0, 3.0e-5, 1.0])
def test_welch_i8_sample_scale_not_folded(live, scale):
    """a sample scale that is not a power of two (1/30000, 3e-5) leaves the digit units' scale out of
    the power's product (each component scaled first, as scipy scales the samples) and takes the
    generic instantiation; 1.0 folds.  Band dB within 1e-9 of scipy on x * scale either way"""
    from meteorgpu import synth
    from scipy.signal import welch
    fs = 4000
    x, _ = synth.synth_real(seed=91, fs=fs, duration_s=6.0, f0=1000, sigma=400, rate_per_min=40)
    x = _stress(x, fs)
    c, win = _plan_cfg(live, fs, 0.2, 4096, 1000, 100, 256)
    c.sample_scale = scale
    got = _run(c, win, x, False)
    B = int(c.block_size)
    nb = (len(x) - B) // B + 1
    ref = np.empty((3, nb))
    for b in range(nb):
        _, P = welch(x[b * B:(b + 1) * B].astype(np.float64) * scale, fs, nperseg=256, noverlap=128, nfft=4096)
        for j in range(3):
            e = np.sum(P[int(c.band_lo[j]): int(c.band_hi[j]) + 1])
            ref[j, b] = 10 * np.log10(e) if e > 0 else -np.inf
    fin = np.isfinite(ref)
    assert np.array_equal(np.isfinite(got), fin)
    np.testing.assert_allclose(got[fin], ref[fin], rtol=0, atol=1e-9)

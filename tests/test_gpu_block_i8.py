"""The block band energies of int16 blocks on the exact integer path (csrc/block_i8.hip: the windowed
DFT at the band bins as an int8 GEMM on the matrix cores) against the reference's numpy blocks
(dsp/src/main.py:352-393, oracle/dsp_oracle.block_powers_ref) and against the float64 Goertzel
path (MSD_OPT_BLOCK_GOERTZEL) it replaces by default.

CPU: the path's arithmetic restated with Python integers (coefficients rounded to 2^-54, exact
dot products) stays within margin.py's int8 chain of the exact long-double DFT.
GPU: dB within 1e-9 of numpy and of the Goertzel path, delta within the near-tie bound, over the
three block lengths the path takes (256, 512, 1024 samples; zero padding to nfft included),
1-8 bins (DC bin included), full-scale and constant blocks, misaligned file offsets (the per-row
fallback loads) and block counts that leave the last 16-block tile partial."""
import numpy as np
import pytest

from meteorgpu import margin as M
from oracle import dsp_oracle as O


PI_LD = np.longdouble("3.14159265358979323846264338327950288")  # np.pi is the float64 value


def _angles(k, L, nfft):
    """2 pi (k n mod nfft) / nfft in long double, the argument reduced exactly"""
    m = (int(k) * np.arange(L, dtype=np.int64)) % int(nfft)
    return 2 * PI_LD * m.astype(np.longdouble) / np.longdouble(nfft)


def _quantised_dft(x, w, nfft, k):
    """sum_n x_n round(w_n e^{-2 pi i k n / nfft} 2^54) / 2^54 with exact integer sums (the device's
    result before its float64 digit combination)"""
    a = _angles(k, len(x), nfft)
    scale = np.longdouble(2.0 ** 54)
    tr = np.rint(w.astype(np.longdouble) * np.cos(a) * scale).astype(np.int64)
    ti = np.rint(-w.astype(np.longdouble) * np.sin(a) * scale).astype(np.int64)
    xs = [int(v) for v in x]
    re = sum(a_ * int(b) for a_, b in zip(xs, tr))
    im = sum(a_ * int(b) for a_, b in zip(xs, ti))

    def ld(v):  # the exact integer to long double (64-bit mantissa) via two exact halves
        hi, lo = divmod(v, 1 << 32)
        return (np.longdouble(hi) * np.longdouble(2.0 ** 32) + np.longdouble(lo)) / scale

    return ld(re), ld(im)


@pytest.mark.parametrize("case", ["noise", "full_scale", "dc"])
def test_quantised_dft_within_i8_chain(case):
    rng = np.random.default_rng({"noise": 1, "full_scale": 2, "dc": 3}[case])
    B, nfft = 9600, 1024
    L = min(B, nfft)
    if case == "noise":
        x = rng.normal(0, 1000, L)
    elif case == "full_scale":
        x = rng.choice([-32768, 32767], L)
    else:
        x = 30000 + rng.normal(0, 3, L)
    x = np.clip(np.round(x), -32768, 32767).astype(np.int16)
    w = np.hanning(B)[:L]
    S = float(np.abs(x.astype(np.float64)).max()) * float(w.sum())
    chain = M._i8_chain(L, 5, float(w.sum()))
    for k in (0, 1, 21, 22, 63, 64, 65, 512):
        re, im = _quantised_dft(x, w, nfft, k)
        ang = _angles(k, L, nfft)
        xw = x.astype(np.longdouble) * w.astype(np.longdouble)
        ex_re, ex_im = np.sum(xw * np.cos(ang)), -np.sum(xw * np.sin(ang))
        err = float(np.hypot(re - ex_re, im - ex_im))
        assert err <= 0.26 * M.U * float(np.abs(x.astype(np.float64)).sum()) + 1e-18 * S
        assert err <= chain * M.U * S


# (fs, block_sec, n_fft, band, noise): L = min(B, 2 n_fft) and the bins
CONFIGS = [
    (48000, 0.2, 512, (950, 1050), (2950, 3050)),   # C3: L 1024, 2 + 3 bins
    (5120, 0.1, 256, (990, 1060), (3000, 2999)),    # L 512, 8 band bins, empty noise band
    (6000, 0.1, 128, (980, 1020), (0, 40)),         # L 256, noise band on the DC bin
    (10240, 0.1, 1024, (995, 1005), (300, 320)),    # B 1024 zero-padded to nfft 2048, 3 + 5 bins
]


def _signal(fs, seconds, seed, B):
    """noise + pings, then in blocks of B: 3-4 constant +full scale, 5-6 constant -full scale, 7-8
    alternating +-full scale, 9-10 silence, 11-19 a +25000 offset"""
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=seed, fs=fs, duration_s=seconds, f0=1000.0, rate_per_min=20)
    x = x.copy()
    x[3 * B: 5 * B] = 32767
    x[5 * B: 7 * B] = -32768
    x[7 * B: 9 * B] = np.where(np.arange(2 * B) % 2, 32767, -32768)
    x[9 * B: 11 * B] = 0
    x[11 * B: 20 * B] = np.clip(x[11 * B: 20 * B].astype(np.int32) + 25000, -32768, 32767)
    return x


ALT = [7, 8]  # the alternating blocks: band energy ~1e-9 of sum |x w|, so numpy's own float64
#               rounding (~(4 log2 nfft + 8) u sum |x w|) exceeds 1e-9 dB there; checked against the
#               exact (long double) DFT within each side's bound instead


def _exact_band_db(x, B, nfft, w, lo, hi):
    """10 log10(sum |X_k|^2 + 1e-12) over bins lo..hi of each block, X in long double"""
    L = min(B, nfft)
    pi = np.longdouble("3.14159265358979323846264338327950288")
    out = []
    for b in range(x.size // B):
        xw = x[b * B: b * B + L].astype(np.longdouble) * w[:L].astype(np.longdouble)
        e = np.longdouble(0)
        for k in range(lo, hi + 1):
            a = 2 * pi * ((k * np.arange(L, dtype=np.int64)) % nfft).astype(np.longdouble) / np.longdouble(nfft)
            e += np.sum(xw * np.cos(a)) ** 2 + np.sum(xw * np.sin(a)) ** 2
        out.append(10 * np.log10(float(e) + 1e-12))
    return np.array(out)


@pytest.mark.gpu
@pytest.mark.parametrize("fs,bs,n_fft,band,noise", CONFIGS)
def test_block_i8_matches_numpy_and_goertzel(fs, bs, n_fft, band, noise):
    from meteorgpu import _lib, dsp
    B = int(fs * bs)
    x = _signal(fs, 12.0, 500 + n_fft, B)
    nfft = 2 * n_fft
    L = min(B, nfft)
    bb, nb = dsp.band_bins(nfft, fs, band), dsp.band_bins(nfft, fs, noise)
    nbins = max(0, bb[1] - bb[0] + 1) + max(0, nb[1] - nb[0] + 1)
    assert L in (256, 512, 1024) and 1 <= nbins <= 8  # the int8 path's shapes
    ctx = dsp.context(0)
    w = dsp.hanning_sym(B)
    plan = _lib.BlockPlan(ctx, B, nfft, w[:L], bb, nb)
    try:
        b8, n8, d8 = plan.run(x)
        ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 1)
        bg, ng, dg = plan.run(x)
    finally:
        ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 0)
        plan.close()
    rb, rn, rd = O.block_powers_ref(x, fs, bs, band, noise, n_fft)
    keep = np.ones(rb.size, bool)
    keep[ALT] = False
    for got, ref in ((b8, rb), (n8, rn), (d8, rd), (b8, bg), (n8, ng), (d8, dg)):
        np.testing.assert_allclose(got[keep], ref[keep], rtol=0, atol=1e-9)
    xmax = float(np.abs(x.astype(np.float64)).max())
    err = M.delta_error_bound(b8, n8, nfft=nfft, L=L, window=w[:L], xmax=xmax, band=bb, noise=nb)
    assert (np.abs(d8 - rd) <= err).all()
    # the alternating blocks against the exact DFT: the int8 path within its own (quantisation) bound
    xs = x[: (ALT[-1] + 1) * B]
    wsum = float(w[:L].sum())
    dx8 = (M._i8_chain(L, nbins, wsum) + 8.0) * M.U * 32768.0 * wsum
    for (lo, hi), got in ((bb, b8), (nb, n8)):
        if hi < lo:
            continue
        ex = _exact_band_db(xs, B, nfft, w, lo, hi)[ALT]
        assert (np.abs(got[ALT] - ex) <= M.band_db_error(ex, hi - lo + 1, dx8)).all()


@pytest.mark.gpu
def test_block_i8_misaligned_files_and_partial_tile():
    """several files at odd sample offsets (rows whose start is not on 16 B take the per-row loads),
    lengths that are not whole blocks, and 3 x 23 blocks (the last 16-block tile partial)"""
    from meteorgpu import _lib, dsp
    fs, bs, n_fft, band, noise = 48000, 0.2, 512, (950, 1050), (2950, 3050)
    B, nfft = int(fs * bs), 2 * n_fft
    L = min(B, nfft)
    bb, nb = dsp.band_bins(nfft, fs, band), dsp.band_bins(nfft, fs, noise)
    files = [_signal(fs, 4.6 + 0.05 * i, 900 + i, B)[: int(fs * (4.6 + 0.05 * i))] for i in range(3)]
    offs = [3, 230405, 470021]  # odd: every block start misaligned
    n_tot = offs[-1] + files[-1].size + 16
    buf = np.zeros(n_tot, np.int16)
    for o, f in zip(offs, files):
        buf[o: o + f.size] = f
    lens = np.array([f.size for f in files], np.int64)
    max_blocks = int(lens.max() // B)
    ctx = dsp.context(0)
    plan = _lib.BlockPlan(ctx, B, nfft, dsp.hanning_sym(B)[:L], bb, nb)
    d_x, d_off, d_len = ctx.alloc(2 * n_tot), ctx.alloc(8 * 3), ctx.alloc(8 * 3)
    d_b, d_n, d_d = (ctx.alloc(8 * 3 * max_blocks) for _ in range(3))
    try:
        d_x.upload(buf)
        d_off.upload(np.array(offs, np.int64))
        d_len.upload(lens)
        out = {}
        for mode in (0, 1):
            ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, mode)
            plan.run_dev(d_x, np.int16, d_off, d_len, 3, max_blocks, d_b, d_n, d_d, max_blocks)
            ctx.synchronize()
            out[mode] = [b.download(np.empty((3, max_blocks), np.float64)) for b in (d_b, d_n, d_d)]
    finally:
        ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 0)
        plan.close()
        for b in (d_x, d_off, d_len, d_b, d_n, d_d):
            b.free()
    for i, f in enumerate(files):
        nbk = f.size // B
        keep = np.ones(nbk, bool)
        keep[ALT] = False
        rb, rn, rd = O.block_powers_ref(f, fs, bs, band, noise, n_fft)
        for j, ref in enumerate((rb, rn, rd)):
            np.testing.assert_allclose(out[0][j][i, :nbk][keep], ref[keep], rtol=0, atol=1e-9)
            np.testing.assert_allclose(out[0][j][i, :nbk][keep], out[1][j][i, :nbk][keep], rtol=0, atol=1e-9)
        # the alternating blocks: the same values as from an aligned single-file run (dsp.block_powers)
        b1, n1, d1, _ = dsp.block_powers(f, fs, bs, band, noise, n_fft)
        for j, one in enumerate((b1, n1, d1)):
            np.testing.assert_array_equal(out[0][j][i, :nbk], one)


@pytest.mark.gpu
@pytest.mark.parametrize("fs,bs,n_fft,band,noise", [(6000, 0.1, 128, (990, 1010), (2990, 3010)),
                                                     (48000, 0.2, 512, (950, 1050), (2950, 3050))])
def test_block_i8_ragged_batch(fs, bs, n_fft, band, noise):
    """a ragged batch as the file loader hands it over: 41 files of 0 to 37 blocks (shorter than one
    block, exactly one, one sample short of / past a whole count), odd and even offsets, so that a
    16-block tile spans up to 16 files and many rows of a tile do not exist; ld > max_blocks, with
    every entry the path must not write checked untouched"""
    from meteorgpu import _lib, dsp
    B, nfft = int(fs * bs), 2 * n_fft
    L = min(B, nfft)
    bb, nb = dsp.band_bins(nfft, fs, band), dsp.band_bins(nfft, fs, noise)
    assert L in (256, 512, 1024) and 1 <= max(0, bb[1] - bb[0] + 1) + max(0, nb[1] - nb[0] + 1) <= 8
    rng = np.random.default_rng(77 + n_fft)
    nblk = [0, 1, 1, 2, 0, 3, 37, 1, 5, 0, 16, 15, 17, 1, 2] + [int(v) for v in rng.integers(0, 12, 26)]
    lens = []
    for i, k in enumerate(nblk):
        extra = [0, B - 1, 1, int(rng.integers(0, B))][i % 4]
        lens.append(k * B + extra)  # k = 0: shorter than one block
    files, offs, pos = [], [], 5
    for i, n in enumerate(lens):
        t = np.arange(n) / fs
        f = 900.0 * rng.standard_normal(n) + 4000.0 * np.sin(2 * np.pi * 1000.0 * t + i) + float(rng.integers(-500, 500))
        files.append(np.clip(np.round(f), -32768, 32767).astype(np.int16))
        offs.append(pos)
        pos += n + int(rng.integers(0, 3))  # odd and even gaps
    nf = len(files)
    buf = np.zeros(pos + 8, np.int16)
    for o, f in zip(offs, files):
        buf[o: o + f.size] = f
    lens = np.array(lens, np.int64)
    max_blocks = int(lens.max() // B)
    ld = max_blocks + 3
    ctx = dsp.context(0)
    plan = _lib.BlockPlan(ctx, B, nfft, dsp.hanning_sym(B)[:L], bb, nb)
    d_x, d_off, d_len = ctx.alloc(2 * buf.size), ctx.alloc(8 * nf), ctx.alloc(8 * nf)
    d_out = [ctx.alloc(8 * nf * ld) for _ in range(3)]
    sentinel = np.full((nf, ld), -777.0)
    try:
        d_x.upload(buf)
        d_off.upload(np.array(offs, np.int64))
        d_len.upload(lens)
        for d in d_out:
            d.upload(sentinel)
        plan.run_dev(d_x, np.int16, d_off, d_len, nf, max_blocks, *d_out, ld)
        ctx.synchronize()
        got = [d.download(np.empty((nf, ld), np.float64)) for d in d_out]
    finally:
        plan.close()
        for d in (d_x, d_off, d_len, *d_out):
            d.free()
    for i, f in enumerate(files):
        k = f.size // B
        for j in range(3):
            assert (got[j][i, k:] == -777.0).all(), (i, j)  # past the file's blocks: untouched
        if k == 0:
            continue
        ref = O.block_powers_ref(f, fs, bs, band, noise, n_fft)
        for j in range(3):
            np.testing.assert_allclose(got[j][i, :k], ref[j], rtol=0, atol=1e-9)


@pytest.mark.gpu
def test_block_window_beyond_unit_takes_goertzel():
    """the int8 coefficients are round(w cos * 2^54) in seven balanced digits, which holds
    for |w_n| <= 1 only.  A plan whose window exceeds that (1.5 x Hann here) keeps the float64
    Goertzel kernel: the default launch is bit-identical to MSD_OPT_BLOCK_GOERTZEL, and both match
    numpy's rFFT band energies of the same window within 1e-9 dB"""
    from meteorgpu import _lib, dsp
    fs, bs, n_fft, band, noise = 48000, 0.2, 512, (950, 1050), (2950, 3050)
    B, nfft = int(fs * bs), 2 * n_fft
    L = min(B, nfft)
    bb, nb = dsp.band_bins(nfft, fs, band), dsp.band_bins(nfft, fs, noise)
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=31, fs=fs, duration_s=6.0, f0=1000.0, rate_per_min=20)
    w = 1.5 * dsp.hanning_sym(L)  # max 1.5 (the first L values of a B-point window stay below 0.12)
    assert w.max() > 1.0
    ctx = dsp.context(0)
    plan = _lib.BlockPlan(ctx, B, nfft, w, bb, nb)
    try:
        got = plan.run(x)
        ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 1)
        ref_g = plan.run(x)
    finally:
        ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 0)
        plan.close()
    for a, b in zip(got, ref_g):
        np.testing.assert_array_equal(a, b)
    nblk = x.size // B
    X = np.fft.rfft(x[: nblk * B].reshape(nblk, B)[:, :L].astype(np.float64) * w, n=nfft)
    P = np.abs(X) ** 2
    eb = 10 * np.log10(P[:, bb[0]: bb[1] + 1].sum(axis=1) + 1e-12)
    en = 10 * np.log10(P[:, nb[0]: nb[1] + 1].sum(axis=1) + 1e-12)
    np.testing.assert_allclose(got[0], eb, rtol=0, atol=1e-9)
    np.testing.assert_allclose(got[1], en, rtol=0, atol=1e-9)

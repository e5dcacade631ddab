"""Complex (I/Q) spectrogram, BASELINE config C5 shape (192 kHz, N = 4096, 75 % overlap).

CPU: the oracle against the scipy golden.  GPU: meteorgpu.iq (cstft4096_kernel through the
C-ABI) against the golden and the oracle, int16 and float32 I/Q, within SPEC_TOL relative per
frame (float32 kernel vs scipy's float64 for complex128 input)."""
import os

import numpy as np
import pytest

from oracle import iq_oracle as Q

SPEC_TOL = 1e-5


def _frame_rel(a, b):
    return float(np.max(np.linalg.norm(a - b, axis=0) / np.maximum(np.linalg.norm(b, axis=0), 1e-300)))


def test_oracle_matches_golden(golden_dir):
    g = np.load(os.path.join(golden_dir, "iq_192k_4096.npz"))
    f, t, S = Q.spectrogram_iq_ref(g["i"], g["q"], int(g["fs"]), int(g["nperseg"]), int(g["noverlap"]))
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    np.testing.assert_array_equal(S.astype(np.float32), g["S"])


@pytest.mark.gpu
def test_golden():
    from meteorgpu import iq
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "iq_192k_4096.npz"))
    f, t, S = iq.spectrogram_iq(g["i"], g["q"], int(g["fs"]), int(g["nperseg"]), int(g["noverlap"]))
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    assert S.shape == g["S"].shape
    assert _frame_rel(S, g["S"].astype(np.float64)) < SPEC_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int16", "float32"])
@pytest.mark.parametrize("n", [4096, 4096 + 1023, 65536 + 77])
def test_vs_scipy(kind, n):
    from meteorgpu import iq
    rng = np.random.default_rng(n)
    tt = np.arange(n) / 192000
    z = 5000 * np.exp(2j * np.pi * (-2500.0) * tt) + 900 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
    if kind == "int16":
        i, q = np.round(z.real).astype(np.int16), np.round(z.imag).astype(np.int16)
    else:
        i, q = (z.real / 32768).astype(np.float32), (z.imag / 32768).astype(np.float32)
    f, t, S = iq.spectrogram_iq(i, q, 192000, 4096, 3072)
    rf, rt, rS = Q.spectrogram_iq_ref(i, q, 192000, 4096, 3072)
    assert S.shape == rS.shape
    assert _frame_rel(S, rS) < SPEC_TOL


@pytest.mark.gpu
def test_batch_matches_single():
    from meteorgpu import iq
    from meteorgpu.dsp import context
    rng = np.random.default_rng(3)
    n = 40000
    streams = [rng.integers(-4000, 4000, 2 * n).astype(np.int16) for _ in range(3)]
    b = iq.IQBatch(context(0), 3, n, 192000)
    for s, x in enumerate(streams):
        b.upload(s, x)
    b.run()
    for s, x in enumerate(streams):
        _, _, S = iq.spectrogram_iq(x[0::2], x[1::2], 192000, 4096, 3072)
        np.testing.assert_array_equal(b.frames(s, 0, b.T), S.T)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int16", "float32"])
@pytest.mark.parametrize("noverlap", [3072, 2048, 3000])
def test_batch_ragged_persistent(kind, noverlap):
    """Enough frames that every workgroup runs several consecutive frames (the register shift
    for hops that are multiples of 256: 3072 → hop 1024, 2048 → hop 2048; 3000 → hop 1096
    reloads), streams of different lengths in one launch (frames past a stream's end are 0)."""
    from meteorgpu import iq
    from meteorgpu.dsp import context
    rng = np.random.default_rng(noverlap)
    n = 1_000_000
    lens = [n, n - 300_001, 4095]  # the last stream has no frame
    dt = np.int16 if kind == "int16" else np.float32
    b = iq.IQBatch(context(0), 3, n, 192000, 4096, noverlap, dtype=dt)
    streams = []
    for s in range(3):
        tt = np.arange(n) / 192000
        z = 4000 * np.exp(2j * np.pi * (1000.0 * (s + 1)) * tt) + 700 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))
        if kind == "int16":
            i, q = np.round(z.real).astype(np.int16), np.round(z.imag).astype(np.int16)
        else:
            i, q = (z.real / 32768).astype(np.float32), (z.imag / 32768).astype(np.float32)
        x = np.empty(2 * n, dt)
        x[0::2], x[1::2] = i, q
        b.upload(s, x)
        streams.append((i[: lens[s]], q[: lens[s]]))
    b.d_len.upload(np.array(lens, np.int64))
    b.run()
    hop = 4096 - noverlap
    for s, (i, q) in enumerate(streams):
        got = b.frames(s, 0, b.T)
        nf = (lens[s] - 4096) // hop + 1 if lens[s] >= 4096 else 0
        assert not got[nf:].any()
        if nf:
            _, _, rS = Q.spectrogram_iq_ref(i, q, 192000, 4096, noverlap)
            assert rS.shape[1] == nf
            assert _frame_rel(got[:nf].T.astype(np.float64), rS) < SPEC_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("dc", [0.0, 700.0])
@pytest.mark.parametrize("kind", ["int16", "float32"])
def test_detrend_from_given_frame_sums(dc, kind):
    """C5's post-FFT detrend (cstft4096_kernel PD): with the frames' sample sums computed by the
    spectrogram itself and with the exact sums the int8 delta step leaves (msd_iq_delta64_sums_dev
    -> msd_cstft_psd_fsums_dev) the spectrogram matches scipy within SPEC_TOL, also with a DC
    offset (the three corrected bins carry it), and the two agree to float32 rounding"""
    from meteorgpu import _lib, iq
    from meteorgpu.dsp import context
    rng = np.random.default_rng(11)
    fs, n = 192000, 60000
    tt = np.arange(n) / fs
    z = 3000 * np.exp(2j * np.pi * 1000.0 * tt) + 600 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) + dc * (1 + 1j)
    i, q = np.round(z.real).astype(np.int16), np.round(z.imag).astype(np.int16)
    dt = np.int16 if kind == "int16" else np.float32
    if kind == "float32":  # the same samples as float32 I/Q (the delta step's float64 Goertzel path)
        i, q = (i / 32768).astype(np.float32), (q / 32768).astype(np.float32)
    x = np.empty(2 * n, dt)
    x[0::2], x[1::2] = i, q
    ctx = context(0)
    b = iq.IQBatch(ctx, 1, n, fs, dtype=dt)
    b.upload(0, x)
    b.run()
    own = b.frames(0, 0, b.T)
    T = b.T
    fsum = ctx.alloc(16 * T)
    d = ctx.alloc(8 * T)
    e = ctx.alloc(8 * T)
    band, noise = iq.iq_band_bins(4096, fs, (950.0, 1050.0)), iq.iq_band_bins(4096, fs, (-3050.0, -2950.0))
    _lib.iq_delta64_dev(ctx, b.d_x, b.code, n, 4096, 1024, float(fs), band, noise,
                        np.array([[0, T]], np.int64), d, e, frame_sums=fsum)
    sums = np.empty(2 * T, np.float64)
    fsum.download(sums)
    if kind == "int16":
        w = np.lib.stride_tricks.sliding_window_view(x.astype(np.int64).reshape(-1, 2), 4096, axis=0)[::1024][:T]
        np.testing.assert_array_equal(sums.reshape(T, 2), w.sum(axis=2))  # exact integer sums
    else:
        w = np.lib.stride_tricks.sliding_window_view(x.astype(np.float64).reshape(-1, 2), 4096, axis=0)[::1024][:T]
        np.testing.assert_allclose(sums.reshape(T, 2), w.sum(axis=2), rtol=0, atol=1e-9)
    b.run(fsums=fsum)
    given = b.frames(0, 0, b.T)
    _, _, rS = Q.spectrogram_iq_ref(i, q, fs, 4096, 3072)
    assert _frame_rel(own.T.astype(np.float64), rS) < SPEC_TOL
    assert _frame_rel(given.T.astype(np.float64), rS) < SPEC_TOL
    if kind == "int16":  # exact sums either way: the same two-part mean, the same bits
        np.testing.assert_array_equal(given, own)
    else:
        assert _frame_rel(given.T.astype(np.float64), own.T.astype(np.float64)) < 1e-6
    for buf in (fsum, d, e):
        buf.free()
    b.close()


def _dc_bins_rel(S, R):
    """largest error of bins 0, 1, N-1 (the bins a DC offset lands in), each frame's error relative
    to that frame's mean power"""
    mean = R.mean(axis=0)
    return float(max(np.max(np.abs(S[k] - R[k]) / mean) for k in (0, 1, R.shape[0] - 1)))


@pytest.mark.gpu
@pytest.mark.parametrize("dc,sigma", [(700, 3.0), (4000, 30.0), (16000, 3.0), (30000, 3.0), (-32000, 30.0)])
@pytest.mark.parametrize("noverlap", [3072, 2048])
def test_large_dc_over_quiet_noise(dc, sigma, noverlap):
    """an SDR's DC offset far above the noise.  The detrend subtracts the frame mean before
    the window as an exact two-part float32 value (cstft.hip), so the result is scipy's within the
    float32 rounding of the detrended samples: per frame within SPEC_TOL, and bins 0, 1, N-1 -- where a
    mis-subtracted mean lands -- checked one by one against the frame's mean power.  With the exact
    frame sums given (the certified C5 path) and computed in the kernel alike; hop 1024 and 2048.
    (Round 4's post-FFT detrend gave 2.7e-5 per frame at (700, 3) and 9e-4 at (30000, 3); a
    single-float mean 1e-4 at (16000, 3): tools/dbg/dc_precision.py.)"""
    from meteorgpu import _lib, iq
    from meteorgpu.dsp import context
    rng = np.random.default_rng(abs(dc) + int(sigma))
    fs, n = 192000, 40000
    z = sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) + dc * (1 - 0.5j)
    i = np.clip(np.round(z.real), -32768, 32767).astype(np.int16)
    q = np.clip(np.round(z.imag), -32768, 32767).astype(np.int16)
    x = np.empty(2 * n, np.int16)
    x[0::2], x[1::2] = i, q
    ctx = context(0)
    b = iq.IQBatch(ctx, 1, n, fs, 4096, noverlap)
    b.upload(0, x)
    b.run()
    own = b.frames(0, 0, b.T).T.astype(np.float64)
    _, _, R = Q.spectrogram_iq_ref(i, q, fs, 4096, noverlap)
    assert _frame_rel(own, R) < SPEC_TOL
    assert _dc_bins_rel(own, R) < SPEC_TOL
    if noverlap == 3072:
        T = b.T
        fsum, d, e = ctx.alloc(16 * T), ctx.alloc(8 * T), ctx.alloc(8 * T)
        band, noise = iq.iq_band_bins(4096, fs, (950.0, 1050.0)), iq.iq_band_bins(4096, fs, (-3050.0, -2950.0))
        _lib.iq_delta64_dev(ctx, b.d_x, b.code, n, 4096, 1024, float(fs), band, noise,
                            np.array([[0, T]], np.int64), d, e, frame_sums=fsum)
        b.run(fsums=fsum)
        given = b.frames(0, 0, b.T).T.astype(np.float64)
        np.testing.assert_array_equal(given, own)
        for buf in (fsum, d, e):
            buf.free()
    b.close()


@pytest.mark.gpu
def test_large_dc_float32():
    """float32 I/Q with a DC offset 1e4 times the noise: the two-part mean from the float sums"""
    from meteorgpu import iq
    rng = np.random.default_rng(77)
    n = 30000
    z = 1e-4 * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) + (0.6 + 0.3j)
    i, q = z.real.astype(np.float32), z.imag.astype(np.float32)
    _, _, S = iq.spectrogram_iq(i, q, 192000, 4096, 3072)
    _, _, R = Q.spectrogram_iq_ref(i, q, 192000, 4096, 3072)
    assert _frame_rel(S, R) < SPEC_TOL
    assert _dc_bins_rel(S, R) < SPEC_TOL


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["int16", "float32"])
def test_chunked_schedule_matches_static(kind):
    """MSD_OPT_CSTFT_RESERVE > 0: the C5 kernel's workgroups draw chunks of frames from the guided
    schedule (cstft.hip DYN) -- the spectrogram, the energy partials and the given-sums variant are
    bit-identical to the fixed-range launch, over several streams of different lengths"""
    from meteorgpu import _lib, iq
    from meteorgpu.dsp import context
    rng = np.random.default_rng(5)
    n = 700_000
    dt = np.int16 if kind == "int16" else np.float32
    xs = []
    for s in range(3):
        z = rng.integers(-3000, 3000, 2 * n) + (500 if s == 1 else 0)
        xs.append(z.astype(np.int16) if kind == "int16" else (z / 32768).astype(np.float32))
    lens = [n, n - 123_457, 300_000]
    out = {}
    base = context(0)
    for reserve in (0, 8):
        ctx = base.sibling()
        try:
            if reserve:
                ctx.set_option(_lib.OPT_CSTFT_RESERVE, reserve)
            b = iq.IQBatch(ctx, 3, n, 192000, 4096, 3072, dtype=dt)
            for s in range(3):
                b.upload(s, xs[s])
            b.d_len.upload(np.array(lens, np.int64))
            T = b.T
            etot = ctx.alloc(16 * 4 * ctx.lib.msd_cstft_energy_stride(3, T))
            b.run(etot)
            spec = np.empty((3, T, 4096), np.float32)
            b.d_out.download(spec)
            e = np.empty(16 * ctx.lib.msd_cstft_energy_stride(3, T), np.float32)
            etot.download(e)
            out[reserve] = (spec, e)
            etot.free()
            b.close()
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[0][0], out[8][0])
    # the energy partials are written for each stream's frames (not for the zero frames past a shorter
    # stream's end): compare those
    T = out[0][0].shape[1]
    valid = np.zeros(out[0][1].size // 16, bool)
    for s_, ln in enumerate(lens):
        nf = (ln - 4096) // 1024 + 1 if ln >= 4096 else 0
        valid[s_ * T: s_ * T + nf] = True
    e0, e8 = out[0][1].reshape(16, -1), out[8][1].reshape(16, -1)
    np.testing.assert_array_equal(e0[:, valid], e8[:, valid])

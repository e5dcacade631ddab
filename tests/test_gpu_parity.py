"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle and the
golden vectors.  Bar:
  * detector: bit-exact thresholds, block indices and dB means for the same delta;
  * band/noise/delta dB (float64 direct DFT vs pocketfft): |diff| <= 1e-9 dB;
  * end to end: identical detection timestamps (CSV t/UTC columns), dB within 1e-9;
  * spectrogram vs scipy: per frame max|diff| <= 1e-5 * max|S| (float32 FFT).
"""
import datetime
import os

import numpy as np
import pytest

from meteorgpu import _lib, dsp, synth, wav
from meteorgpu.batch import BatchPipeline
from oracle import dsp_oracle as O
from tests.detector_kats import ADAPTIVE, GLOBAL

pytestmark = pytest.mark.gpu

DB_TOL = 1e-9
SPEC_TOL = 1e-5


def _golden(golden_dir, name):
    return np.load(os.path.join(golden_dir, name), allow_pickle=False)


def _frame_err(S, ref):
    return (np.abs(S.astype(np.float64) - ref.astype(np.float64)).max(axis=0) /
            np.maximum(np.abs(ref).max(axis=0), 1e-30)).max()


# ------------------------------------------------------------------ a2/a3 block powers
@pytest.mark.parametrize("name", ["blocks_6k.npz", "blocks_48k.npz"])
def test_block_powers_golden(golden_dir, name):
    g = _golden(golden_dir, name)
    band, noise, delta, _ = dsp.block_powers(g["x"], int(g["fs"]), float(g["bs"]), tuple(g["band"]),
                                             tuple(g["noise"]), int(g["n_fft"]))
    exp = g["expected"]
    assert np.abs(band - exp[:, 0]).max() <= DB_TOL
    assert np.abs(noise - exp[:, 1]).max() <= DB_TOL
    assert np.abs(delta - exp[:, 2]).max() <= DB_TOL


BLOCK_CASES = [
    # fs, block_sec, band, noise, n_fft, dtype, n
    (6000, 0.2, (993, 1013), (690, 710), 512, np.int16, 6000 * 30 + 777),      # reference config, ragged
    (48000, 0.2, (950, 1050), (650, 750), 512, np.int16, 48000 * 4),          # 48 kHz, crop 9600 → 1024
    (48000, 0.2, (990, 1010), (690, 710), 512, np.int16, 48000 * 2),          # zero-bin bands → -120 dB
    (6000, 0.05, (900, 1100), (500, 700), 512, np.float32, 6000 * 10 + 3),    # B=300 < Nf: zero padding
    (4000, 0.2, (950, 1050), (650, 750), 2048, np.float64, 4000 * 10),        # Nf=4096, L=800
    (6000, 0.2, (993, 1013), (690, 710), 512, np.uint8, 6000 * 5),
    (6000, 0.2, (993, 1013), (690, 710), 512, np.int32, 6000 * 5),
    (5000, 0.3, (0, 2500), (100, 200), 300, np.int16, 5000 * 6),              # Nf=600 (not 2^k), 301+21 bins
]


@pytest.mark.parametrize("case", BLOCK_CASES, ids=[f"{c[0]}Hz-{np.dtype(c[5]).name}-{i}" for i, c in
                                                    enumerate(BLOCK_CASES)])
def test_block_powers_vs_oracle(case):
    fs, bs, band_hz, noise_hz, n_fft, dt, n = case
    x, _ = synth.synth_real(seed=100 + n % 97, fs=fs, duration_s=n / fs, f0=sum(band_hz) / 2, rate_per_min=20)
    x = x[:n]
    if np.dtype(dt) == np.uint8:
        x = ((x.astype(np.int32) >> 8) + 128).astype(np.uint8)
    elif np.dtype(dt) == np.int32:
        x = x.astype(np.int32) << 8
    else:
        x = x.astype(dt)
    rb, rn, rd = O.block_powers_ref(x, fs, bs, band_hz, noise_hz, n_fft)
    b, nz, d, B = dsp.block_powers(x, fs, bs, band_hz, noise_hz, n_fft)
    assert B == int(fs * bs) and b.shape == rb.shape
    assert np.abs(b - rb).max() <= DB_TOL
    assert np.abs(nz - rn).max() <= DB_TOL
    assert np.abs(d - rd).max() <= DB_TOL


# ------------------------------------------------------------------ a4/a5 detector KATs
@pytest.mark.parametrize("case", GLOBAL, ids=[c[0] for c in GLOBAL])
def test_global_detector_kats(case):
    name, delta, k, exp, exp_thr, err = case
    d = np.array(delta, dtype=np.float64)
    if err is not None:
        with pytest.raises(err):
            dsp.get_detections(d, k, 1.0)
        return
    dets, thr = dsp.get_detections(d, k, 1.0)
    _, rthr = O.get_detections_ref(d, k, 1.0)
    assert thr == rthr
    assert [(int(x.t_start), int(x.t_stop)) for x in dets] == [(s, e) for s, e, _ in exp]
    assert [float(x.dB) for x in dets] == [db for *_, db in exp]


@pytest.mark.parametrize("case", ADAPTIVE, ids=[c[0] for c in ADAPTIVE])
def test_adaptive_detector_kats(case):
    name, delta, k, (w, fb, fa, f0), exp, exp_thr = case
    d = np.array(delta, dtype=np.float64)
    dets, thr = dsp.get_detections_adaptive(d, k, 1.0, w, fb, fa, f0)
    _, rthr = O.get_detections_adaptive_ref(d, k, 1.0, w, fb, fa, f0)
    assert [(int(x.t_start), int(x.t_stop)) for x in dets] == [(s, e) for s, e, _ in exp]
    assert [float(x.dB) for x in dets] == [db for *_, db in exp]
    np.testing.assert_array_equal(np.array(thr, float), np.array(rthr, float))


def _random_delta(seed, nb, bursts=20):
    rng = np.random.default_rng(seed)
    d = rng.standard_normal(nb) * 1.5 + rng.uniform(-3, 3)
    for _ in range(bursts):
        i = rng.integers(0, max(1, nb))
        d[i:i + rng.integers(1, 30)] += rng.uniform(3, 25)
    return d


@pytest.mark.parametrize("nb", [1, 2, 7, 300, 1000, 5000, 20000, 70000])
@pytest.mark.parametrize("bs", [0.2, 0.1])
def test_adaptive_detector_bit_exact(nb, bs):
    d = _random_delta(nb, nb, bursts=max(1, nb // 100))
    start = datetime.datetime(2025, 6, 25, 7, 51, 41)
    dets, thr = dsp.get_detections_adaptive(d, 4, bs, 120, 3, 20, 10, wav_start_date_time=start)
    rdets, rthr = O.get_detections_adaptive_ref(d, 4, bs, 120, 3, 20, 10, wav_start_date_time=start)
    np.testing.assert_array_equal(np.array(thr, float), np.array(rthr, float))
    assert len(dets) == len(rdets)
    for a, r in zip(dets, rdets):
        assert (a.t_start, a.t_stop, a.dur_s, a.utc_start, a.utc_stop) == (r[0], r[1], r[2], r[4], r[5])
        assert a.dB == r[3]


@pytest.mark.parametrize("nb,bs", [(6000, 0.05), (15000, 0.01)])
def test_adaptive_detector_long_windows_bit_exact(nb, bs):
    """windows past the four-level walk (120 s at 0.05 s: 2 400 blocks > 1 928) and past one numpy
    buffer chunk (120 s at 0.01 s: 12 000 blocks > 8 192: two chunks summed in turn), np_reduce.h"""
    d = _random_delta(nb + 7, nb, bursts=max(1, nb // 100))
    dets, thr = dsp.get_detections_adaptive(d, 4, bs, 120, 3, 20, 10)
    rdets, rthr = O.get_detections_adaptive_ref(d, 4, bs, 120, 3, 20, 10)
    np.testing.assert_array_equal(np.array(thr, float), np.array(rthr, float))
    assert [(a.t_start, a.t_stop, a.dB) for a in dets] == [(r[0], r[1], r[3]) for r in rdets]


@pytest.mark.parametrize("nb", [2, 300, 9000, 300000])
@pytest.mark.parametrize("k", [1.0, 3.5])
def test_global_detector_bit_exact(nb, k):
    d = _random_delta(nb + 1, nb, bursts=max(1, nb // 50))
    d[-1] = -10.0  # keep the last block below (the reference asserts otherwise)
    dets, thr = dsp.get_detections(d, k, 0.2)
    rdets, rthr = O.get_detections_ref(d, k, 0.2)
    assert thr == rthr
    assert [(x.t_start, x.t_stop, x.dur_s) for x in dets] == [tuple(r[:3]) for r in rdets]
    assert [x.dB for x in dets] == [r[3] for r in rdets]


def test_global_detector_zero_duration_asserts():
    d = np.zeros(50)
    d[-1] = 100.0
    with pytest.raises(AssertionError, match="Detection duration must be greater than 0"):
        dsp.get_detections(d, 1.0, 0.2)
    with pytest.raises(AssertionError, match="UTC start time must be before stop time"):
        dsp.get_detections(d, 1.0, 0.2, wav_start_date_time=datetime.datetime(2025, 1, 1))


# ------------------------------------------------------------------ end to end (a1-a6)
E2E = [
    # fs, seconds, band, noise, adaptive, k
    (6000, 600, (993, 1013), (690, 710), True, 4),      # mb_files configuration, 10 minutes
    (6000, 300, (996, 1016), (940, 960), True, 3.5),    # tl_files-like bands
    (6000, 300, (993, 1013), (690, 710), False, 4),     # global threshold
    (48000, 60, (950, 1050), (650, 750), True, 4),      # C1/C2: one 60 s 48 kHz file
]


@pytest.mark.parametrize("case", E2E, ids=[f"{c[0]}Hz-{c[1]}s-{'adaptive' if c[4] else 'global'}" for c in E2E])
def test_proc_wav_file_csv_matches_oracle(tmp_path, case):
    fs, secs, band, noise, adaptive, k = case
    x, pings = synth.synth_real(seed=1000 + secs + fs // 1000, fs=fs, duration_s=secs, f0=sum(band) / 2,
                                band_hz=band[1] - band[0], rate_per_min=6)
    x[-int(fs * 2):] = (x[-int(fs * 2):] // 4)  # quiet tail: keeps the global detector off the last block
    p = tmp_path / "expoFull_gqrx_20250625_075141_49969000.wav"
    wav.write(p, fs, x)
    start = wav.start_datetime_from_name(str(p))
    out_csv = tmp_path / "ours.csv"
    res = dsp.proc_wav_file(str(p), 0.2, band, noise, 512, k, out_csv_file=str(out_csv), wav_start_date_time=start,
                            disable_show_and_write=True, flag_adaptive_threshold=adaptive,
                            required_sample_rate=fs, out_audacity_lbl_file=str(tmp_path / "lbl.txt"))
    rdets, rthr, rb, rn, rd = O.proc_samples_ref(x, fs, 0.2, band, noise, 512, k, start, adaptive)
    assert np.abs(res.delta_power - rd).max() <= DB_TOL
    assert res.min_margin > 1e-7, "decision margin too small for a meaningful parity check"
    O.write_csv_ref(rdets, tmp_path / "ref.csv")
    ours = (out_csv).read_text().splitlines()
    ref = (tmp_path / "ref.csv").read_text().splitlines()
    assert len(ours) == len(ref) and len(ref) >= 2, "synthetic input should produce detections"
    for lo, lr in zip(ours[1:], ref[1:]):
        fo, fr = lo.split(","), lr.split(",")
        assert fo[0:3] == fr[0:3] and fo[4:] == fr[4:]       # t_start, t_stop, dur_s, utc_start, utc_stop
        assert abs(float(fo[3]) - float(fr[3])) <= DB_TOL   # dB
    assert (tmp_path / "lbl.txt").read_text() == O.audacity_ref(rdets)


# ------------------------------------------------------------------ a7 spectrogram
@pytest.mark.parametrize("name", ["spec_48k_1024.npz", "spec_6k_256_f32.npz"])
def test_spectrogram_golden(golden_dir, name):
    g = _golden(golden_dir, name)
    N = int(g["nperseg"])
    f, t, S = dsp.spectrogram(g["x"], fs=int(g["fs"]), window="hann", nperseg=N, noverlap=N // 2, nfft=N,
                              scaling="density", mode="psd")
    assert S.dtype == np.float32 and S.shape == g["S"].shape
    np.testing.assert_array_equal(f, g["f"])
    np.testing.assert_array_equal(t, g["t"])
    assert _frame_err(S, g["S"]) <= SPEC_TOL


SPEC_CASES = [
    # fs, nperseg, noverlap, dtype, n
    (48000, 1024, 512, np.int16, 48000 * 3 + 100),
    (48000, 1024, 768, np.int16, 48000),
    (48000, 1024, 0, np.int16, 48000),
    (6000, 256, 128, np.int16, 6000 * 5),
    (6000, 512, 256, np.float32, 6000 * 5),
    (6000, 2048, 1024, np.int16, 6000 * 10),
    (6000, 2048, 1024, np.uint8, 6000 * 10),
    (4000, 1024, 512, np.float32, 4000 * 3 + 1),
    (48000, 1024, 511, np.int16, 48000),   # odd hop: unaligned frame starts (scalar loads)
]


@pytest.mark.parametrize("case", SPEC_CASES, ids=[f"{c[1]}-{c[2]}-{np.dtype(c[3]).name}" for c in SPEC_CASES])
def test_spectrogram_vs_scipy(case):
    fs, N, nov, dt, n = case
    x, _ = synth.synth_real(seed=N + nov, fs=fs, duration_s=n / fs + 1, f0=1000.0, rate_per_min=30)
    x = x[:n]
    if np.dtype(dt) == np.float32:
        x = (x / 32768.0).astype(np.float32)
    elif np.dtype(dt) == np.uint8:
        x = ((x.astype(np.int32) >> 8) + 128).astype(np.uint8)
    from scipy.signal import spectrogram as sp_spec
    fr, tr, Sr = sp_spec(x, fs=fs, window="hann", nperseg=N, noverlap=nov, nfft=N, scaling="density", mode="psd")
    f, t, S = dsp.spectrogram(x, fs=fs, window="hann", nperseg=N, noverlap=nov, nfft=N)
    assert S.shape == Sr.shape and S.dtype == Sr.dtype == np.float32
    np.testing.assert_array_equal(f, fr)
    np.testing.assert_array_equal(t, tr)
    assert _frame_err(S, Sr) <= SPEC_TOL


@pytest.mark.parametrize("dc,sigma", [(700, 600.0), (700, 3.0), (12000, 3.0), (-16000, 30.0), (-30000, 30.0),
                                      (30000, 30.0), (-32000, 3.0), (32000, 3.0)])
@pytest.mark.parametrize("N,nov", [(1024, 512), (2048, 1024), (256, 128)])
def test_spectrogram_dc_offset(dc, sigma, N, nov):
    """a DC offset on the int16 audio (tests/test_iq.py's offset-700 case, and large offsets over quiet
    noise, up to +-32000 over sigma 3): scipy's spectrogram holds per frame and at bins 0, 1 -- where a
    residual of the mean lands -- against each frame's mean power.  stft1024_kernel (1024 / 512, C3)
    subtracts the mean's exact integer part before the FFT and its fractional part times the window's
    DFT from bins 0, 1 after it (round 6); the generic kernel (stft.hip) subtracts an
    exact two-part mean.  Both are exact at any offset."""
    rng = np.random.default_rng(abs(dc) + N)
    n = 48000 * 2
    t = np.arange(n) / 48000
    x = dc + sigma * rng.standard_normal(n) + 4 * sigma * np.sin(2 * np.pi * 1000.0 * t)
    x = np.clip(np.round(x), -32768, 32767).astype(np.int16)
    from scipy.signal import spectrogram as sp_spec
    _, _, Sr = sp_spec(x, fs=48000, window="hann", nperseg=N, noverlap=nov, nfft=N, scaling="density", mode="psd")
    _, _, S = dsp.spectrogram(x, fs=48000, window="hann", nperseg=N, noverlap=nov, nfft=N)
    assert _frame_err(S, Sr) <= SPEC_TOL
    R = Sr.astype(np.float64)
    mean = R.mean(axis=0)
    for k in (0, 1):
        assert np.max(np.abs(S[k].astype(np.float64) - R[k]) / mean) <= SPEC_TOL, k


@pytest.mark.parametrize("N,nov", [(1024, 512), (2048, 1024), (256, 128)])
def test_spectrogram_float32_dc_offset(N, nov):
    """float32 samples with a DC offset 6000 x the noise: the kernels' float sums run relative to each
    frame's first sample and the mean comes off as hi + lo, so the result is the float64 spectrogram
    of the same float32 samples within SPEC_TOL.  (scipy on the float32 array itself detrends in
    float32 with numpy's float32 pairwise mean and is 5e-4 away from that here -- shown below --
    so no float32 pipeline with another summation order can reproduce it to 1e-5.)"""
    rng = np.random.default_rng(N)
    x = (0.6 + 1e-4 * rng.standard_normal(48000)).astype(np.float32)
    from scipy.signal import spectrogram as sp_spec
    _, _, R64 = sp_spec(x.astype(np.float64), fs=48000, window="hann", nperseg=N, noverlap=nov, nfft=N,
                        scaling="density", mode="psd")
    _, _, R32 = sp_spec(x, fs=48000, window="hann", nperseg=N, noverlap=nov, nfft=N, scaling="density", mode="psd")
    _, _, S = dsp.spectrogram(x, fs=48000, window="hann", nperseg=N, noverlap=nov, nfft=N)
    assert _frame_err(S, R64) <= SPEC_TOL
    assert _frame_err(R32, R64) > 10 * SPEC_TOL  # scipy's own float32 detrend


def test_spectrogram_constant_input_is_zero():
    # constant detrend removes a DC-only signal entirely
    x = np.full(48000, 1234, np.int16)
    _, _, S = dsp.spectrogram(x, fs=48000, nperseg=1024, noverlap=512)
    assert np.abs(S).max() <= 1e-6


# ------------------------------------------------------------------ batch pipeline (C2/C3 shape)
def test_batch_pipeline_matches_single_file_path():
    ctx = dsp.context(0)
    fs, n, F = 48000, 48000 * 60, 6
    # noise band far from the ping: at 48 kHz the reference framing (hanning(9600)[:1024])
    # leaks a strong ping into neighbouring bands, so a nearby noise band would rise with it
    bp = BatchPipeline(ctx, F, n, fs, noise_band=(2950.0, 3050.0))
    xs = []
    for i in range(F):
        x, _ = synth.synth_real(seed=3000 + i, fs=fs, duration_s=60, f0=1000.0, rate_per_min=4,
                                snr_db=(25.0, 40.0))
        xs.append(x)
        bp.upload_file(i, x)
    base = datetime.datetime(2025, 6, 25, 0, 0, 0)
    starts = [base + datetime.timedelta(minutes=59 + i) for i in range(F)]  # straddles the 01:00 boundary
    epoch = datetime.datetime(1970, 1, 1)
    start_us = np.array([(s - epoch) // datetime.timedelta(microseconds=1) for s in starts], np.int64)
    bp.set_start_times(start_us, (base - epoch) // datetime.timedelta(microseconds=1))
    bp.run()
    ctx.synchronize()
    deltas = bp.delta()
    dets, counts, status, margin = bp.detections()
    assert (status == 0).all()
    total = 0
    from collections import Counter
    ref_hours = Counter()
    for i in range(F):
        _, _, S = dsp.spectrogram(xs[i], fs=fs, nperseg=1024, noverlap=512)
        np.testing.assert_array_equal(bp.spectrogram(i), S)
        _, _, d, _ = dsp.block_powers(xs[i], fs, 0.2, (950, 1050), (2950, 3050), 512)
        np.testing.assert_array_equal(deltas[i], d)
        rdets, _ = O.get_detections_adaptive_ref(d, 4.0, 0.2, wav_start_date_time=starts[i])
        assert [(int(a["start"]), int(a["stop"])) for a in dets[i]] == \
               [(int(round(r[0] / 0.2)), int(round(r[1] / 0.2))) for r in rdets]
        assert [a["db"] for a in dets[i]] == [r[3] for r in rdets]
        total += len(rdets)
        for h, c in O.count_per_hour_ref(rdets).items():
            ref_hours[(h - base) // datetime.timedelta(hours=1)] += c
    hist = bp.hour_counts()
    assert hist.sum() == total > 0
    for h in range(24):
        assert hist[h] == ref_hours.get(h, 0)


def test_batch_concurrent_stages_identical():
    """BatchPipeline(concurrent=True): block_delta -> detect on a second context's stream beside
    the STFT (msd_stream_wait fork/join) against the serial pipeline, bit for bit.  The concurrent
    pipeline alternates two DIFFERENT input buffers over back-to-back steps with no host
    synchronisation, so a dropped fork (side stream not waiting for ctx) or join (ctx not
    waiting for the side stream) leaves outputs of the wrong buffer or a half-written step;
    a last step runs straight after an upload into the buffer it reads."""
    ctx = dsp.context(0)
    fs, n, F = 48000, 48000 * 60, 8
    xa = [synth.synth_real(seed=3100 + i, fs=fs, duration_s=60, f0=1000.0, rate_per_min=6)[0] for i in range(F)]
    xb = [synth.synth_real(seed=3200 + i, fs=fs, duration_s=60, f0=1000.0, rate_per_min=9)[0] for i in range(F)]
    xc = [synth.synth_real(seed=3300 + i, fs=fs, duration_s=60, f0=1000.0, rate_per_min=12)[0] for i in range(F)]

    def outputs(bp):
        dets, counts, status, margin = bp.detections()
        assert (status == 0).all()
        return (bp.delta(), bp.thresholds(), counts, [d.tobytes() for d in dets], bp.hour_counts(),
                [bp.spectrogram(i) for i in (0, F - 1)])

    def same(a, b):
        for u, v in zip(a[:3] + (a[4],), b[:3] + (b[4],)):
            np.testing.assert_array_equal(u, v)
        assert a[3] == b[3]
        for u, v in zip(a[5], b[5]):
            np.testing.assert_array_equal(u, v)
        assert a[4].sum() == a[2].sum()

    def serial(xs):
        bp = BatchPipeline(ctx, F, n, fs, noise_band=(2950.0, 3050.0))
        for i, x in enumerate(xs):
            bp.upload_file(i, x)
        bp.set_start_times(np.arange(F, dtype=np.int64) * 60 * 10 ** 6, 0)
        bp.run()
        ctx.synchronize()
        return outputs(bp)

    want_b, want_c = serial(xb), serial(xc)
    assert want_b[2].tolist() != want_c[2].tolist()  # the inputs give different detections
    bp = BatchPipeline(ctx, F, n, fs, noise_band=(2950.0, 3050.0), concurrent=True)
    assert bp.side is not None
    d_b = ctx.alloc(bp.d_x.nbytes)
    for i in range(F):
        bp.upload_file(i, xa[i])
        d_b.upload(np.ascontiguousarray(xb[i], dtype=np.int16), byte_offset=i * bp.n_pad * 2)
    bp.set_start_times(np.arange(F, dtype=np.int64) * 60 * 10 ** 6, 0)
    for x in (None, d_b, None, d_b):  # A, B, A, B back to back
        bp.run(x=x)
    ctx.synchronize()
    same(outputs(bp), want_b)
    for i in range(F):  # upload C into the default buffer and run at once
        bp.upload_file(i, xc[i])
    bp.run()
    ctx.synchronize()
    same(outputs(bp), want_c)


def test_full_day_batch_properties():
    """C3 at full size (1440 x 60 s @ 48 kHz, 8.3 GB in, 16.6 GB spectrogram) through
    size-independent properties: replicated files give identical outputs at every offset
    (no 32-bit index overflow), per-frame Parseval on sampled frames, delta equal to the
    single-file path, histogram total equal to the detection count."""
    ctx = dsp.context(0)
    fs, n, F = 48000, 48000 * 60, 1440
    bp = BatchPipeline(ctx, F, n, fs)
    pool = [synth.synth_real(seed=4000 + j, fs=fs, duration_s=60, f0=1000.0)[0] for j in range(4)]
    for i in range(F):
        bp.upload_file(i, pool[i % 4])
    bp.run()
    ctx.synchronize()
    dets, counts, status, margin = bp.detections()
    assert (status == 0).all()
    assert bp.hour_counts().sum() == counts.sum()
    deltas = bp.delta()
    for j in range(4):
        np.testing.assert_array_equal(counts[j::4], counts[j])
        np.testing.assert_array_equal(deltas[j::4], np.broadcast_to(deltas[j], deltas[j::4].shape))
    for i in (0, 1, 717, 1438, 1439):
        S = bp.spectrogram(i)
        np.testing.assert_array_equal(S, bp.spectrogram(i % 4))
        x = pool[i % 4].astype(np.float64)
        w = dsp.hann_periodic(1024).astype(np.float32).astype(np.float64)
        scale = 1.0 / (fs * np.sum(w * w))
        for t in (0, 1, 2811, S.shape[1] - 1):
            v = x[t * 512:t * 512 + 1024]
            v = (v - v.mean()) * w
            want = scale * 1024 * np.sum(v * v)   # Parseval on the one-sided, doubled spectrum
            assert abs(S[:, t].astype(np.float64).sum() - want) <= 1e-5 * want
    _, _, d0, _ = dsp.block_powers(pool[1], fs, 0.2, (950, 1050), (650, 750), 512)
    np.testing.assert_array_equal(deltas[1437], d0)


@pytest.mark.gpu
def test_c4_day_sharded_over_eight_ranks():
    """C4 at full size: the 1440-file day cut into 8 contiguous file ranges (meteorgpu.shard.shard_range,
    as bench.py --shard-day), one BatchPipeline per rank-thread with its own context.  The hour
    histograms summed (the RCCL all-reduce's job) equal one pipeline over the whole day; every
    file's detections, counts and delta, and the spectrograms of each range's first and last file,
    equal the whole-day pipeline's bit for bit."""
    import threading
    from meteorgpu.shard import shard_range
    fs, n, F, W = 48000, 48000 * 60, 1440, 8
    pool = [synth.synth_real(seed=4100 + j, fs=fs, duration_s=60, f0=1000.0, rate_per_min=6)[0] for j in range(4)]
    epoch, day0 = datetime.datetime(1970, 1, 1), datetime.datetime(2025, 6, 1)
    us = lambda t: (t - epoch) // datetime.timedelta(microseconds=1)  # noqa: E731

    def make(ctx, lo, hi, spec_files):
        bp = BatchPipeline(ctx, hi - lo, n, fs, noise_band=(2950.0, 3050.0))  # the bench's bands
        for i in range(hi - lo):
            bp.upload_file(i, pool[(lo + i) % 4])
        bp.set_start_times(np.array([us(day0 + datetime.timedelta(minutes=lo + i)) for i in range(hi - lo)],
                                    np.int64), us(day0))
        bp.run()
        ctx.synchronize()
        dets, counts, status, _ = bp.detections()
        return dict(dets=dets, counts=counts, status=status, hist=bp.hour_counts(), delta=bp.delta(),
                    spec={lo + i: bp.spectrogram(i) for i in spec_files})

    whole = make(dsp.context(0), 0, F, range(4))  # files 0-3 = the 4 pool inputs
    assert (whole["status"] == 0).all() and whole["counts"].sum() > 1000 and whole["hist"].sum() == whole["counts"].sum()
    results, errs = [None] * W, []

    def body(r):
        try:
            ctx = _lib.Context(0)
            try:
                lo, hi = shard_range(F, r, W)
                results[r] = (lo, hi, make(ctx, lo, hi, (0, hi - lo - 1)))
            finally:
                ctx.close()
        except BaseException as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=body, args=(r,)) for r in range(W)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]
    assert np.array_equal(sum(res["hist"] for _, _, res in results), whole["hist"])
    assert [lo for lo, _, _ in results] == sorted(lo for lo, _, _ in results) and results[-1][1] == F
    for lo, hi, res in results:
        assert (res["status"] == 0).all()
        assert np.array_equal(res["counts"], whole["counts"][lo:hi])
        assert np.array_equal(res["delta"], whole["delta"][lo:hi])
        for i in range(hi - lo):
            assert np.array_equal(res["dets"][i], whole["dets"][lo + i])
        for f, sp in res["spec"].items():  # file f has pool input f % 4, as whole-day file f % 4
            assert np.array_equal(sp, whole["spec"][f % 4])


@pytest.mark.parametrize("dt", [np.int16, np.float32, np.uint8])
def test_stft_fast_path_matches_generic_kernel(dt):
    """The specialised N=1024 kernel and the generic Stockham kernel agree (A/B switch)."""
    x, _ = synth.synth_real(seed=77, fs=48000, duration_s=5.0, f0=1000.0, rate_per_min=60)
    if np.dtype(dt) == np.float32:
        x = (x / 32768.0).astype(np.float32)
    elif np.dtype(dt) == np.uint8:
        x = ((x.astype(np.int32) >> 8) + 128).astype(np.uint8)
    ctx = dsp.context(0)
    _, _, fast = dsp.spectrogram(x, fs=48000, nperseg=1024, noverlap=512)
    ctx.set_option(_lib.OPT_GENERIC_STFT, 1)
    try:
        _, _, gen = dsp.spectrogram(x, fs=48000, nperseg=1024, noverlap=512)
    finally:
        ctx.set_option(_lib.OPT_GENERIC_STFT, 0)
    assert _frame_err(fast, gen) <= 2e-6


def test_rccl_communicator_single_rank_allreduce():
    """The N>1 exchange step on the one-GPU box: an RCCL communicator of one rank sums a
    device histogram in place (identity), through msd_comm_* (dlopen'd librccl)."""
    from meteorgpu import _lib
    from meteorgpu.batch import Communicator
    from meteorgpu.dsp import context
    ctx = context(0)
    uid = Communicator.unique_id()
    assert len(uid) == _lib.COMM_ID_BYTES
    comm = Communicator(ctx, 1, uid, 0)
    try:
        h = np.arange(24, dtype=np.int64) * 7 - 3
        buf = ctx.alloc(h.nbytes)
        buf.upload(h)
        comm.allreduce_i64(buf, h.size)
        ctx.synchronize()
        out = np.empty_like(h)
        buf.download(out)
        np.testing.assert_array_equal(out, h)
    finally:
        comm.close()


@pytest.mark.parametrize("nperseg", [1024, 256])
def test_ragged_batch_through_the_c_abi(nperseg):
    """msd_stft_psd_dev / msd_block_delta_dev / msd_detect_dev on a ragged batch: files of
    different lengths, one shorter than a frame and a block, one empty, in one launch each —
    every file equals its single-file result (and the oracle); padding columns are zero."""
    ctx = dsp.context(0)
    fs = 48000
    lens = [fs * 7 + 313, 0, 700, fs * 3, fs * 11 + 5]
    xs = [synth.synth_real(seed=40 + i, fs=fs, duration_s=max(m, 1) / fs, f0=1000.0, rate_per_min=20,
                           snr_db=(25.0, 40.0))[0][:m] for i, m in enumerate(lens)]
    F = len(xs)
    offs = np.cumsum([0] + [(m + 7) // 8 * 8 for m in lens[:-1]]).astype(np.int64)
    total = int(offs[-1] + lens[-1] + 8)
    host = np.zeros(total, np.int16)
    for o, x in zip(offs, xs):
        host[o:o + len(x)] = x
    d_x = ctx.alloc(host.nbytes)
    d_x.upload(host)
    d_off, d_len = ctx.alloc(F * 8), ctx.alloc(F * 8)
    d_off.upload(offs)
    d_len.upload(np.array(lens, np.int64))
    w = dsp.hann_periodic(nperseg).astype(np.complex64)
    scale = float(np.real(1.0 / (fs * (w * w).sum())))
    plan = _lib.StftPlan(ctx, nperseg, nperseg // 2, w.real.astype(np.float32), scale)
    K = nperseg // 2 + 1
    T = [plan.frames(m) for m in lens]
    ld = max(32, (max(T) + 31) // 32 * 32)
    d_spec = ctx.alloc(F * K * ld * 4)
    plan.run_dev(d_x, np.int16, d_off, d_len, F, max(T), d_spec, ld)
    spec = np.empty((F, K, ld), np.float32)
    d_spec.download(spec)
    for i in range(F):
        if T[i]:
            _, _, S = dsp.spectrogram(xs[i], fs=fs, nperseg=nperseg, noverlap=nperseg // 2)
            np.testing.assert_array_equal(spec[i, :, :T[i]], S)
        assert not spec[i, :, T[i]:].any()
    # block delta + adaptive detector over the same ragged batch
    B = int(fs * 0.2)
    nb = [m // B for m in lens]
    ldb = max(1, max(nb))
    blk = _lib.BlockPlan(ctx, B, 1024, dsp.hanning_sym(B)[:1024], dsp.band_bins(1024, fs, (950, 1050)),
                         dsp.band_bins(1024, fs, (2950, 3050)))
    d_delta = ctx.alloc(F * ldb * 8)
    blk.run_dev(d_x, np.int16, d_off, d_len, F, ldb, None, None, d_delta, ldb)
    delta = np.empty((F, ldb), np.float64)
    d_delta.download(delta)
    cfg = _lib.det_cfg(True, 4.0, 600, 15, 100, 50)
    d_nb = ctx.alloc(F * 8)
    d_nb.upload(np.array(nb, np.int64))
    cap = ldb // 2 + 2
    d_dets, d_cnt, d_thr = ctx.alloc(F * cap * _lib.DET_DTYPE.itemsize), ctx.alloc(F * 8), ctx.alloc(F * ldb * 8)
    d_mg, d_st = ctx.alloc(F * 8), ctx.alloc(F * 4)
    _lib.check(ctx.lib.msd_detect_dev(ctx.h, d_delta.ptr, d_nb.ptr, F, ldb, cfg, d_dets.ptr, cap, d_cnt.ptr,
                                      d_thr.ptr, d_mg.ptr, d_st.ptr, None))
    cnt = np.empty(F, np.int64)
    d_cnt.download(cnt)
    dets = np.empty((F, cap), _lib.DET_DTYPE)
    d_dets.download(dets)
    for i in range(F):
        if nb[i] == 0:
            assert cnt[i] == 0
            continue
        _, _, d, _ = dsp.block_powers(xs[i], fs, 0.2, (950, 1050), (2950, 3050), 512)
        np.testing.assert_array_equal(delta[i, :nb[i]], d)
        rdets, _ = O.get_detections_adaptive_ref(d, 4.0, 0.2)
        assert [(int(a["start"]), int(a["stop"]), float(a["db"])) for a in dets[i, :cnt[i]]] == \
               [(int(round(r[0] / 0.2)), int(round(r[1] / 0.2)), r[3]) for r in rdets]


def test_stft_fast_path_wide_row_stride():
    """Rows of 2^21 frames and more (a > 6 h 48 kHz file): the N = 1024 kernel switches to 64-bit
    output offsets.  Exercised with a short signal and a padded row stride ld >= 2^21."""
    ctx = dsp.context(0)
    fs = 48000
    x, _ = synth.synth_real(seed=9, fs=fs, duration_s=3.0, f0=1000.0)
    w = dsp.hann_periodic(1024).astype(np.complex64)
    scale = float(np.real(1.0 / (fs * (w * w).sum())))
    plan = _lib.StftPlan(ctx, 1024, 512, w.real.astype(np.float32), scale)
    T = plan.frames(len(x))
    ld = (1 << 21) + 32
    d_x = ctx.alloc(x.nbytes)
    d_x.upload(x)
    d_off, d_len = ctx.alloc(8), ctx.alloc(8)
    d_off.upload(np.zeros(1, np.int64))
    d_len.upload(np.array([len(x)], np.int64))
    d_spec = ctx.alloc(513 * ld * 4)
    plan.run_dev(d_x, np.int16, d_off, d_len, 1, T, d_spec, ld)
    _, _, S = dsp.spectrogram(x, fs=fs, nperseg=1024, noverlap=512)
    row = np.empty(T + 32, np.float32)
    for k in (0, 1, 255, 511, 512):
        d_spec.download(row, byte_offset=k * ld * 4)
        np.testing.assert_array_equal(row[:T], S[k])
        assert not row[T:].any()
    tail = np.empty(64, np.float32)
    d_spec.download(tail, byte_offset=(512 * ld + ld - 64) * 4)
    assert not tail.any()


@pytest.mark.parametrize("hop_case", ["c3", "h768"])
def test_stft1024_chunked_schedule_identical(hop_case):
    """MSD_OPT_STFT_SCHED = 2: stft1024_kernel's workgroups draw chunks of consecutive tiles from a
    guided schedule (ticket) instead of one fixed range each -- the spectrogram is bit-identical over a
    batch of 40 files of different lengths, repeated launches (the ticket is reset per launch)"""
    from meteorgpu import _lib
    base = dsp.context(0)
    rng = np.random.default_rng(8)
    fs, n, F = 48000, 48000 * 20, 40
    hop = 512 if hop_case == "c3" else 768  # the shared-half pair (SH) and the plain one
    xs = [rng.integers(-6000, 6000, n).astype(np.int16) for _ in range(F)]
    lens = [n - (i * 7919) % 200_000 for i in range(F)]
    out = {}
    for sched in (1, 2):
        ctx = base.sibling()
        try:
            ctx.set_option(_lib.OPT_STFT_SCHED, sched)
            w = dsp.hann_periodic(1024).astype(np.float32)
            plan = _lib.StftPlan(ctx, 1024, hop, w, float(1.0 / (fs * (w.astype(np.float64) ** 2).sum())))
            T = (n - 1024) // hop + 1
            ld = (T + 31) // 32 * 32
            d_x, d_off, d_len = ctx.alloc(2 * F * n), ctx.alloc(8 * F), ctx.alloc(8 * F)
            d_x.upload(np.concatenate(xs))
            d_off.upload(np.arange(F, dtype=np.int64) * n)
            d_len.upload(np.array(lens, np.int64))
            d_out = ctx.alloc(4 * F * 513 * ld)
            res = []
            for _ in range(2):
                plan.run_dev(d_x, np.int16, d_off, d_len, F, T, d_out, ld)
                S = np.empty((F, 513, ld), np.float32)
                d_out.download(S)
                res.append(S)
            np.testing.assert_array_equal(res[0], res[1])
            out[sched] = res[0]
            for b in (d_x, d_off, d_len, d_out):
                b.free()
            plan.close()
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[1], out[2])


@pytest.mark.parametrize("frames", [1, 5, 32, 33])
def test_stft1024_chunked_schedule_single_tile(frames):
    """MSD_OPT_STFT_SCHED = 2 on one short file: one or two 32-frame tiles, so the guided schedule's only
    chunk holds a single tile (the first chunk's second ticket must be published before the
    first loop head reads it) -- identical to the static launch and to scipy"""
    from meteorgpu import _lib
    from scipy.signal import spectrogram as sp_spec
    base = dsp.context(0)
    rng = np.random.default_rng(frames)
    fs = 48000
    n = 1024 + 512 * (frames - 1)
    x = rng.integers(-9000, 9000, n).astype(np.int16)
    _, _, R = sp_spec(x, fs=fs, window="hann", nperseg=1024, noverlap=512, nfft=1024, scaling="density", mode="psd")
    out = {}
    for sched in (1, 2):
        ctx = base.sibling()
        try:
            ctx.set_option(_lib.OPT_STFT_SCHED, sched)
            w = dsp.hann_periodic(1024).astype(np.float32)
            plan = _lib.StftPlan(ctx, 1024, 512, w, float(1.0 / (fs * (w.astype(np.float64) ** 2).sum())))
            ld = (frames + 31) // 32 * 32
            d_x, d_off, d_len = ctx.alloc(2 * n), ctx.alloc(8), ctx.alloc(8)
            d_x.upload(x)
            d_off.upload(np.zeros(1, np.int64))
            d_len.upload(np.array([n], np.int64))
            d_out = ctx.alloc(4 * 513 * ld)
            for _ in range(3):
                plan.run_dev(d_x, np.int16, d_off, d_len, 1, frames, d_out, ld)
                S = np.empty((513, ld), np.float32)
                d_out.download(S)
                out.setdefault(sched, S)
                np.testing.assert_array_equal(S, out[sched])
            for b in (d_x, d_off, d_len, d_out):
                b.free()
            plan.close()
        finally:
            ctx.close()
    np.testing.assert_array_equal(out[1], out[2])
    assert not out[1][:, frames:].any()
    assert _frame_err(out[1][:, :frames], R) <= SPEC_TOL

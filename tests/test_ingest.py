"""WAV ingest.

CPU: libmsdsp's native parser (msd_wav_probe / msd_wav_read — host code, no GPU) against
scipy.io.wavfile.read on every format the reference's files use.  GPU: WavDay — files decoded
into pinned memory, uploaded on the copy stream, processed in double-buffered batches — gives
the same detections and hour histogram as the one-file-at-a-time drop-in."""
import datetime

import numpy as np
import pytest
import scipy.io.wavfile


@pytest.mark.parametrize("dtype", [np.int16, np.uint8, np.int32, np.float32, np.float64])
@pytest.mark.parametrize("channels", [1, 2, 3])
def test_native_reader_matches_scipy(tmp_path, dtype, channels):
    from meteorgpu import ingest
    rng = np.random.default_rng(1)
    n = 4099
    if np.dtype(dtype).kind == "f":
        x = rng.standard_normal((n, channels)).astype(dtype)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max, size=(n, channels), endpoint=True).astype(dtype)
    if channels == 1:
        x = x[:, 0]
    p = tmp_path / "a.wav"
    scipy.io.wavfile.write(p, 48000, x)
    fs, y = ingest.read(p)
    fs2, y2 = scipy.io.wavfile.read(p)
    assert fs == fs2 and y.dtype == y2.dtype and y.shape == y2.shape
    np.testing.assert_array_equal(y, y2)
    if channels > 1:
        fs3, y3 = ingest.read(p, channel=channels - 1)
        np.testing.assert_array_equal(y3, y2[:, channels - 1])


def _wav24(path, rate, ints, channels=1):
    """A 24-bit PCM file written byte by byte (scipy writes no 24-bit)."""
    import struct
    b = bytearray()
    for v in ints.reshape(-1):
        b += int(v).to_bytes(3, "little", signed=True)
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", 36 + len(b)) + b"WAVE")
        fh.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, channels, rate, rate * 3 * channels, 3 * channels, 24))
        fh.write(b"data" + struct.pack("<I", len(b)) + bytes(b))


def test_native_reader_24bit_and_extra_chunks(tmp_path):
    from meteorgpu import ingest
    rng = np.random.default_rng(2)
    v = rng.integers(-2 ** 23, 2 ** 23 - 1, size=(1001, 2))
    p = tmp_path / "b.wav"
    _wav24(p, 6000, v, channels=2)
    fs, y = ingest.read(p)
    fs2, y2 = scipy.io.wavfile.read(p)
    assert y.dtype == y2.dtype == np.int32
    np.testing.assert_array_equal(y, y2)
    # a LIST chunk before "data" and an odd-sized chunk are skipped
    x = rng.integers(-30000, 30000, 777).astype(np.int16)
    q = tmp_path / "c.wav"
    scipy.io.wavfile.write(q, 8000, x)
    raw = q.read_bytes()
    extra = b"LIST" + (5).to_bytes(4, "little") + b"abcde" + b"\x00"
    i = raw.index(b"data")
    (tmp_path / "d.wav").write_bytes(raw[:i] + extra + raw[i:])
    fs3, y3 = ingest.read(tmp_path / "d.wav")
    np.testing.assert_array_equal(y3, x)


def test_native_reader_errors(tmp_path):
    from meteorgpu import _lib, ingest
    p = tmp_path / "x.wav"
    p.write_bytes(b"RIFX" + b"\x00" * 40)
    with pytest.raises(_lib.MsdError, match="RIFX"):
        ingest.read(p)
    p.write_bytes(b"JUNK" + b"\x00" * 40)
    with pytest.raises(_lib.MsdError, match="Only 'RIFF'"):
        ingest.read(p)
    with pytest.raises(_lib.MsdError, match="cannot open"):
        ingest.read(tmp_path / "missing.wav")


@pytest.mark.gpu
def test_wav_day_matches_single_file_drop_in(tmp_path):
    from meteorgpu import dsp, ingest, synth, wav
    from meteorgpu.dsp import context
    day = datetime.datetime(2025, 6, 1, 3, 0)
    paths, xs = [], []
    for i in range(7):  # batches of 3: two full, one short
        x, _ = synth.synth_real(seed=70 + i, fs=6000, duration_s=60.0, f0=1003.0, rate_per_min=12, band_hz=20.0,
                                snr_db=(15, 30))
        t = day + datetime.timedelta(minutes=17 * i)
        p = tmp_path / f"SDR_gqrx_{t:%Y%m%d}_{t:%H%M%S}_49969000.wav"
        wav.write(p, 6000, x)
        paths.append(p)
        xs.append(x)
    refs = []
    for x in xs:
        res = dsp.process_samples(x, 6000, 0.2, (993, 1013), (690, 710), 512, 4.0)
        refs.append([(round(r.t_start / 0.2), round(r.t_stop / 0.2), r.dB) for r in res.detections])
    total = sum(len(r) for r in refs)
    assert total > 0
    # batches of 3 (three slots: two full batches and a short one), 4 (two slots, short second)
    # and 7 (one batch); each day run twice (the short batch's lengths must not leak into the
    # next run's first batch)
    for bf in (3, 4, 7):
        wd = ingest.WavDay(context(0), paths, batch_files=bf, freq_band=(993, 1013), noise_band=(690, 710),
                           n_fft=512)
        for _ in range(2):
            dets, hist, info = wd.run()
            assert len(dets) == 7 and info["files"] == 7
            for ref, d in zip(refs, dets):
                assert [(int(a["start"]), int(a["stop"]), float(a["db"])) for a in d] == ref
            assert int(hist.sum()) == total
            # the near-tie guard bounds with the int16 full scale (no pass over the samples)
            assert (wd.bp.decision_bounds > 0).all() and not wd.bp.near_tie.any()


@pytest.mark.gpu
def test_wav_day_bad_file_raises_after_readers_stop(tmp_path):
    """a file whose format differs from the first one fails the run with the file named; the
    decodes still in flight finish before the error leaves run(), and the day runs again once the
    file is fixed"""
    from meteorgpu import ingest, wav
    from meteorgpu.dsp import context
    day = datetime.datetime(2025, 6, 1, 3, 0)
    rng = np.random.default_rng(5)
    paths = []
    for i in range(7):
        t = day + datetime.timedelta(minutes=i)
        p = tmp_path / f"SDR_gqrx_{t:%Y%m%d}_{t:%H%M%S}_49969000.wav"
        wav.write(p, 6000, rng.integers(-3000, 3000, 6000 * 20, dtype=np.int16))
        paths.append(p)
    good = paths[5].read_bytes()
    wav.write(paths[5], 8000, rng.integers(-3000, 3000, 6000 * 20, dtype=np.int16))  # batch 2 of 3
    wd = ingest.WavDay(context(0), paths, batch_files=2, freq_band=(993, 1013), noise_band=(690, 710), n_fft=512)
    with pytest.raises(ValueError, match="format differs"):
        wd.run()
    paths[5].write_bytes(good)
    dets, hist, info = wd.run()
    assert len(dets) == 7 and info["files"] == 7

def test_iq_wav_file_rejects_mono(tmp_path):
    """the I/Q entry point asserts a 2-channel file before touching the GPU"""
    import pytest as _pt
    from meteorgpu import iq, wav
    p = tmp_path / "mono.wav"
    wav.write(p, 192000, np.zeros(4096, np.int16))
    with _pt.raises(AssertionError, match="2-channel"):
        iq.proc_iq_wav_file(str(p), (950, 1050), (-3050, -2950))
    with _pt.raises(AssertionError, match="does not exist"):
        iq.proc_iq_wav_file(str(tmp_path / "nope.wav"), (950, 1050), (-3050, -2950))

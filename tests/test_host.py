"""CPU: host-side logic of the drop-in (WAV ingest, windows, band bins, CSV / label
emitters, file-name → UTC, synthetic generator, argument asserts)."""
import csv
import datetime
import io
import os

import numpy as np
import pytest
import scipy.io.wavfile
from scipy.signal import get_window

from meteorgpu import dsp, synth, wav
from oracle import dsp_oracle as O


@pytest.mark.parametrize("dtype", [np.int16, np.uint8, np.int32, np.float32, np.float64])
@pytest.mark.parametrize("channels", [1, 2])
def test_wav_roundtrip_matches_scipy(tmp_path, dtype, channels):
    rng = np.random.default_rng(7)
    n = 1001
    if np.dtype(dtype).kind == "f":
        x = rng.standard_normal((n, channels)).astype(dtype)
    else:
        info = np.iinfo(dtype)
        x = rng.integers(info.min, info.max, size=(n, channels), endpoint=True).astype(dtype)
    if channels == 1:
        x = x[:, 0]
    p = tmp_path / "a.wav"
    scipy.io.wavfile.write(p, 6000, x)
    fs, y = wav.read(p)
    fs2, y2 = scipy.io.wavfile.read(p)
    assert fs == fs2 == 6000
    assert y.dtype == y2.dtype and y.shape == y2.shape
    np.testing.assert_array_equal(y, y2)
    q = tmp_path / "b.wav"
    wav.write(q, 6000, x)
    fs3, y3 = scipy.io.wavfile.read(q)
    assert fs3 == 6000
    np.testing.assert_array_equal(y3, x)


def test_wav_24bit_matches_scipy(tmp_path):
    # hand-built 24-bit PCM file
    import struct
    vals = np.array([0, 1, -1, 8388607, -8388608, 12345], dtype=np.int32)
    payload = b"".join(int(v).to_bytes(3, "little", signed=True) for v in vals)
    p = tmp_path / "c.wav"
    with open(p, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", 36 + len(payload)) + b"WAVE")
        fh.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, 6000, 18000, 3, 24))
        fh.write(b"data" + struct.pack("<I", len(payload)) + payload)
    fs, y = wav.read(p)
    fs2, y2 = scipy.io.wavfile.read(p)
    assert y.dtype == y2.dtype
    np.testing.assert_array_equal(y, y2)


@pytest.mark.parametrize("m", [1, 2, 5, 1200, 9600])
def test_hanning_is_numpy(m):
    np.testing.assert_array_equal(dsp.hanning_sym(m), np.hanning(m))


@pytest.mark.parametrize("m", [256, 1024, 4096])
def test_periodic_hann_is_scipy(m):
    np.testing.assert_array_equal(dsp.hann_periodic(m), get_window("hann", m))


@pytest.mark.parametrize("fs,nfft,band", [
    (6000, 1024, (993, 1013)), (6000, 1024, (690, 710)), (48000, 1024, (950, 1050)), (48000, 1024, (990, 1010)),
    (48000, 1024, (0, 0)), (4000, 4096, (970, 1070)), (6000, 1024, (3000, 3000)),
])
def test_band_bins_follow_reference_masks(fs, nfft, band):
    freqs = np.fft.rfftfreq(nfft, d=1 / fs)
    mask = (freqs >= band[0]) & (freqs <= band[1])
    lo, hi = dsp.band_bins(nfft, fs, band)
    sel = np.zeros_like(mask)
    if hi >= lo:
        sel[lo:hi + 1] = True
    np.testing.assert_array_equal(sel, mask)


def test_reference_config_bins():
    # signal (993,1013) → bins 170-172, noise (690,710) → 118-121; 48 kHz ±10 Hz → none
    assert dsp.band_bins(1024, 6000, (993, 1013)) == (170, 172)
    assert dsp.band_bins(1024, 6000, (690, 710)) == (118, 121)
    assert dsp.band_bins(1024, 48000, (993, 1013)) == (0, -1)


def _dets_from_oracle(dets):
    return [dsp.OutputDetection(t_start=a, t_stop=b, dur_s=c, dB=d, utc_start=e, utc_stop=f)
            for a, b, c, d, e, f in dets]


@pytest.mark.parametrize("with_utc", [False, True])
def test_csv_writer_byte_identical_to_reference_emitter(tmp_path, with_utc):
    d = np.zeros(300)
    d[[5, 6, 100, 101, 102, 250]] = 30.0
    start = datetime.datetime(2025, 6, 25, 7, 51, 41) if with_utc else None
    ref, _ = O.get_detections_adaptive_ref(d, 4, 0.2, wav_start_date_time=start)
    assert len(ref) == 3
    O.write_csv_ref(ref, tmp_path / "ref.csv")
    dsp.write_csv(_dets_from_oracle(ref), tmp_path / "ours.csv")
    a = (tmp_path / "ref.csv").read_bytes()
    b = (tmp_path / "ours.csv").read_bytes()
    assert a == b
    assert a.startswith(b"t_start,t_stop,dur_s,dB,utc_start,utc_stop\r\n")
    rows = list(csv.DictReader(io.StringIO(a.decode())))
    assert rows[0]["t_start"] == "1.0"
    dsp.write_audacity_labels(_dets_from_oracle(ref), tmp_path / "l.txt")
    assert (tmp_path / "l.txt").read_text() == O.audacity_ref(ref)


def test_count_per_hour():
    start = datetime.datetime(2025, 6, 25, 7, 59, 0)
    d = np.zeros(600)
    d[[10, 400]] = 40.0  # 2 s and 80 s after 07:59:00 → hours 07 and 08
    ref, _ = O.get_detections_adaptive_ref(d, 4, 0.2, wav_start_date_time=start)
    ours = dsp.count_per_hour(_dets_from_oracle(ref))
    assert ours == O.count_per_hour_ref(ref)
    assert sorted(ours.values()) == [1, 1]


def test_filename_to_utc():
    assert wav.start_datetime_from_name("/x/expoFull_gqrx_20250625_075141_49969000.wav") == \
        datetime.datetime(2025, 6, 25, 7, 51, 41)
    assert wav.start_datetime_from_name("/x/expoFull_Brams_250607_23MESZ.wav") == \
        datetime.datetime(2025, 6, 7, 21, 0, 0)


def test_synth_deterministic():
    a, pa = synth.synth_real(5, 48000, 2.0, 1000.0, rate_per_min=60)
    b, pb = synth.synth_real(5, 48000, 2.0, 1000.0, rate_per_min=60)
    np.testing.assert_array_equal(a, b)
    assert pa == pb and a.dtype == np.int16 and a.shape == (96000,)


def test_proc_wav_file_asserts_before_gpu(tmp_path):
    # the reference's argument asserts (main.py:230-268) fire before any device work
    with pytest.raises(AssertionError, match="File does not exist"):
        dsp.proc_wav_file(str(tmp_path / "missing.wav"), 0.2, (993, 1013), (690, 710), 512, 4,
                          disable_show_and_write=True)
    p = tmp_path / "f.wav"
    wav.write(p, 8000, np.zeros(8000, np.int16))
    with pytest.raises(AssertionError, match="Output directory does not exist"):
        dsp.proc_wav_file(str(p), 0.2, (993, 1013), (690, 710), 512, 4, out_csv_file="/nonexistent/dir/x.csv",
                          disable_show_and_write=True)
    with pytest.raises(AssertionError, match="Sample rate must be 6000 Hz, but got 8000 Hz"):
        dsp.proc_wav_file(str(p), 0.2, (993, 1013), (690, 710), 512, 4, disable_show_and_write=True)
    with pytest.raises(AssertionError, match="Start sample must be less than end sample"):
        dsp.proc_wav_file(str(p), 0.2, (993, 1013), (690, 710), 512, 4, wav_start_sec=0.5, wav_end_sec=0.5,
                          disable_show_and_write=True)
    with pytest.raises(AssertionError, match="End sample exceeds length of audio data"):
        dsp.proc_wav_file(str(p), 0.2, (993, 1013), (690, 710), 512, 4, wav_end_sec=2.0,
                          disable_show_and_write=True)



def test_refinement_path_query():
    """msd_iq_delta64_path (host only): which block step the float64 refinement takes -- the exact
    int8-MFMA DFT for int16 at C5's geometry, the float64 Goertzel rows for float32 input, other
    block sizes and bands at 0 Hz, one lane per block when D is not a multiple of 64"""
    from meteorgpu import _lib
    c5 = ((21, 22), (-65, -63))
    assert _lib.iq_delta64_path(4096, 1024, 192000, *c5, _lib.MSD_CI16) == _lib.REFINE_INT8_MFMA
    assert _lib.iq_delta64_path(4096, 1024, 192000, *c5, _lib.MSD_CF32) == _lib.REFINE_GOERTZEL_ROWS
    assert _lib.iq_delta64_path(4096, 2048, 192000, *c5, _lib.MSD_CI16) == _lib.REFINE_GOERTZEL_ROWS  # D 2048
    assert _lib.iq_delta64_path(4096, 1000, 192000, *c5, _lib.MSD_CI16) == _lib.REFINE_DIRECT        # D 8
    assert _lib.iq_delta64_path(4096, 1024, 192000, (-2, 2), (40, 42), _lib.MSD_CI16) == _lib.REFINE_GOERTZEL_ROWS
    assert _lib.iq_delta64_path(4096, 1024, 192000, (20, 27), (-66, -60), _lib.MSD_CI16) == _lib.REFINE_GOERTZEL_ROWS
    import pytest
    with pytest.raises(_lib.MsdError):
        _lib.iq_delta64_path(131072, 1024, 192000, *c5, _lib.MSD_CI16)


def test_interval_helpers_match_sets():
    """meteorgpu.iq's refinement bookkeeping (_merge, _subtract: vectorised) against plain sets of
    frames on random interval lists, touching and nested ones included"""
    import numpy as np
    from meteorgpu.iq import _merge, _subtract
    rng = np.random.default_rng(5)

    def frames(iv):
        return set().union(*[set(range(a, b)) for a, b in iv]) if iv else set()

    for _ in range(300):
        n, m = int(rng.integers(0, 12)), int(rng.integers(0, 6))
        iv = [(int(a), int(a + w)) for a, w in zip(rng.integers(0, 200, n), rng.integers(-3, 40, n))]
        dn = _merge([(int(a), int(a + w)) for a, w in zip(rng.integers(0, 200, m), rng.integers(0, 60, m))])
        mg = _merge(iv)
        assert frames(mg) == frames([(a, b) for a, b in iv if b > a])
        assert all(b > a for a, b in mg) and all(mg[i][1] < mg[i + 1][0] for i in range(len(mg) - 1))
        sub = _subtract(mg, dn)
        assert frames(sub) == frames(mg) - frames(dn)
        assert all(b > a for a, b in sub) and all(sub[i][1] < sub[i + 1][0] for i in range(len(sub) - 1))
    assert _subtract([[0, 10]], []) == [[0, 10]] and _subtract([], [[0, 5]]) == [] and _merge([]) == []

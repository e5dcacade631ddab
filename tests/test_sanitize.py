"""CPU sanitizer target: the host C++ that parses untrusted WAV
files or plans device work, built with g++ -fsanitize=address,undefined
(`make -C meteor-scatter_amd/csrc sanitize` -> build/host_check_san, csrc/host_check.cpp) and run on

* malformed WAV files next to scipy.io.wavfile.read (scipy/io/wavfile.py:568-733), the reader
  the reference uses (dsp/src/main.py:249): the two either both refuse a file or both return the
  same samples; libmsdsp's own reader (msd_wav_probe / msd_wav_read, the same wav_parse.h) agrees;
* a seeded fuzz of mutated / truncated WAV images decoded in memory (exact-size buffers: any read
  past the image is an AddressSanitizer report), numpy's np.sum leaf programs and the float64
  refinement planner.

A sanitizer report aborts the harness (-fno-sanitize-recover=all), which fails the test."""
import os
import shutil
import struct
import subprocess
import warnings

import numpy as np
import pytest
import scipy.io.wavfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "meteor-scatter_amd", "csrc")
EXE = os.path.join(CSRC, "build", "host_check_san")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="g++ needed for the sanitizer build")


@pytest.fixture(scope="module")
def harness():
    # one build at a time: pytest-xdist workers would otherwise exec a half-linked binary
    import fcntl
    os.makedirs(os.path.join(CSRC, "build"), exist_ok=True)
    with open(os.path.join(CSRC, "build", ".sanitize.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", CSRC, "sanitize"], check=True, capture_output=True)
    return EXE


def run(harness, *args):
    env = dict(os.environ, ASAN_OPTIONS="abort_on_error=1:detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([harness, *map(str, args)], capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode == 0, f"sanitizer / check failure:\n{r.stdout}\n{r.stderr[-4000:]}"
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    return r.stdout.strip()


def fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for x in b:
        h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def riff(chunks, riff_size=None):
    body = b"WAVE" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body) if riff_size is None else riff_size) + body


def chunk(cid, payload, size=None):
    pad = b"\x00" if len(payload) % 2 else b""
    return cid + struct.pack("<I", len(payload) if size is None else size) + payload + pad


def fmt(tag=1, ch=1, rate=48000, cont=2, bits=16, byte_rate=None, extra=b""):
    br = rate * cont * ch if byte_rate is None else byte_rate
    return chunk(b"fmt ", struct.pack("<HHIIHH", tag, ch, rate, br, cont * ch, bits) + extra)


EXT_TAIL = b"\x00\x00\x10\x00\x80\x00\x00\xAA\x00\x38\x9B\x71"
rng = np.random.default_rng(7)
S16 = rng.integers(-32768, 32767, 600).astype("<i2").tobytes()  # 300 stereo / 600 mono samples
S24 = rng.integers(0, 256, 3 * 301, dtype=np.uint8).tobytes()   # 301 mono 24-bit samples (odd size)

CASES = {
    "mono16": riff([fmt(), chunk(b"data", S16)]),
    "stereo16": riff([fmt(ch=2), chunk(b"data", S16)]),
    "u8": riff([fmt(cont=1, bits=8), chunk(b"data", S16[:301])]),
    "f32": riff([fmt(tag=3, cont=4, bits=32), chunk(b"data", np.linspace(-1, 1, 77, dtype="<f4").tobytes())]),
    "f64": riff([fmt(tag=3, cont=8, bits=64, ch=2), chunk(b"data", np.linspace(-1, 1, 64, dtype="<f8").tobytes())]),
    "pcm24_odd_frames": riff([fmt(cont=3, bits=24), chunk(b"data", S24)]),
    "extensible16": riff([fmt(tag=0xFFFE, extra=struct.pack("<HHI", 22, 16, 0) + struct.pack("<I", 1) + EXT_TAIL),
                          chunk(b"data", S16)]),
    "extensible_bad_guid": riff([fmt(tag=0xFFFE, extra=struct.pack("<HHI", 22, 16, 0) + struct.pack("<I", 1) +
                                     b"\x11" * 12), chunk(b"data", S16)]),
    "extensible_short_cb": riff([fmt(tag=0xFFFE, extra=struct.pack("<HHI", 20, 16, 0) + b"\x00" * 16),
                                 chunk(b"data", S16)]),
    "odd_list_padding": riff([fmt(), chunk(b"LIST", b"abcde"), chunk(b"data", S16)]),
    "odd_unknown_chunk": riff([chunk(b"junk", b"xyz"), fmt(ch=2), chunk(b"data", S16)]),
    "fmt_size_lt_16": riff([chunk(b"fmt ", struct.pack("<HHIIH", 1, 1, 48000, 96000, 2)), chunk(b"data", S16)]),
    "zero_channels": riff([fmt(ch=0, byte_rate=0), chunk(b"data", S16)]),
    "bad_byte_rate": riff([fmt(byte_rate=12345), chunk(b"data", S16)]),
    "no_fmt_before_data": riff([chunk(b"data", S16), fmt()]),
    "data_past_eof_mono": riff([fmt(), chunk(b"data", S16)[:-100]]),
    "data_past_eof_stereo_partial_frame": riff([fmt(ch=2), chunk(b"data", S16)[:-2]]),
    "data_size_ffffffff": riff([fmt(), b"data" + struct.pack("<I", 0xFFFFFFFF) + S16]),
    "data_size_ffffffff_stereo": riff([fmt(ch=2), b"data" + struct.pack("<I", 0xFFFFFFFF) + S16]),
    "chunk_size_ffffffff_before_data": riff([fmt(), chunk(b"LIST", b"ab", size=0xFFFFFFFF), chunk(b"data", S16)]),
    "truncated_chunk_header": riff([fmt(), b"LIS"]),
    "truncated_chunk_size": riff([fmt(), b"LIST\x05\x00"]),
    "truncated_fmt_body": riff([fmt()[:20]]),
    "riff_size_excludes_data": riff([fmt(), chunk(b"data", S16)], riff_size=4 + 24),
    "riff_size_small_but_covers_data": riff([fmt(), chunk(b"data", S16)], riff_size=4 + 24 + 8),
    "riff_size_ffffffff": riff([fmt(), chunk(b"data", S16)], riff_size=0xFFFFFFFF),
    "empty_data": riff([fmt(), chunk(b"data", b"")]),
    "not_riff": b"JUNK" + b"\x00" * 40,
    "short_file": b"RIFF\x00",
    "int64_pcm": riff([fmt(cont=8, bits=64), chunk(b"data", S16[:64])]),
}
# scipy reads these; libmsdsp refuses them (wav_parse.h "Differences"), so they are excluded from
# the both-agree check and asserted as refusals instead
OURS_REFUSE = {"int64_pcm"}


def scipy_read(path):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        try:
            fs, data = scipy.io.wavfile.read(path)
        except Exception as e:  # noqa: BLE001 -- any refusal (ValueError, struct.error, ZeroDivisionError, ...)
            return None, repr(e)
    return fs, np.ascontiguousarray(data)


@pytest.mark.parametrize("name", sorted(CASES))
def test_malformed_wav_matches_scipy(harness, tmp_path, name):
    p = tmp_path / f"{name}.wav"
    p.write_bytes(CASES[name])
    out = run(harness, "wav", p)
    fs, data = scipy_read(p)
    if name in OURS_REFUSE:
        assert out.startswith("err"), out
        return
    if fs is None:
        assert out.startswith("err"), f"scipy refuses ({data}) but the parser reads: {out}"
        return
    assert out.startswith("ok"), f"scipy reads {data.shape} {data.dtype} but the parser refuses: {out}"
    f = out.split()
    rate, channels, frames, digest = int(f[1]), int(f[2]), int(f[7]), int(f[10], 16)
    assert rate == fs and frames == data.shape[0] and channels == (1 if data.ndim == 1 else data.shape[1])
    assert digest == fnv1a(data.tobytes()), "decoded samples differ from scipy's"
    # libmsdsp's reader (the product path, same header) returns scipy's array
    from meteorgpu import ingest
    fs2, y = ingest.read(p)
    assert fs2 == fs and y.dtype == data.dtype and y.shape == data.shape
    np.testing.assert_array_equal(y, data)


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_fuzz_under_sanitizers(harness, seed):
    out = run(harness, "fuzz", seed, 4000)
    assert out.startswith("ok"), out
    parsed = int(out.split()[1])
    assert parsed > 1000  # most mutations still parse: the decode path is exercised


@pytest.mark.parametrize("n", [0, 1, 127, 128, 129, 8191, 8192, 8193, 22500, 3 * 8192 + 17])
def test_np_program_under_sanitizers(harness, n):
    assert run(harness, "program", n).startswith("ok")


def test_refine_plan_under_sanitizers(harness):
    # C5 (bins 21..22 and -65..-63: 9 needed bins, blocks of 1024, 4 per frame)
    assert run(harness, "refine", 4096, 1024, 21, 22, -65, -63, 10 ** 6, 0, 10, 40, 90).split()[1:4] == ["9", "1024", "4"]
    # a hop that is not a power of two (blocks of gcd(4096, 1000) = 8 samples)
    assert run(harness, "refine", 4096, 1000, 21, 22, -65, -63, 10 ** 6, 3, 9).split()[2:4] == ["8", "512"]
    # the 16-lane Goertzel rows only for D % 64 == 0: D = 1024 rows, D = 500 (N 1000,
    # hop 500) and D = 96 (N 192, hop 96) the one-lane direct path
    assert run(harness, "refine", 4096, 1024, 21, 22, -65, -63, 10 ** 6, 0, 10).split()[6] == "1"
    for n, hop, d in ((1000, 500, "500"), (192, 96, "96"), (4096, 2560, "512")):
        out = run(harness, "refine", n, hop, 3, 4, -9, -7, 10 ** 5, 0, 10).split()
        assert out[0] == "ok" and out[2] == d and out[6] == ("1" if int(d) % 64 == 0 else "0"), out
    # refused, not crashed: overlapping ranges, a band outside the spectrum, frames past the samples
    assert run(harness, "refine", 4096, 1024, 21, 22, -65, -63, 10 ** 6, 0, 10, 5, 20).startswith("err")
    assert run(harness, "refine", 4096, 1024, 21, 5000, -65, -63, 10 ** 6, 0, 10).startswith("err")
    assert run(harness, "refine", 4096, 1024, 21, 22, -65, -63, 8192, 0, 10).startswith("err")
    assert run(harness, "refine", 131072, 1024, 21, 22, -65, -63, 10 ** 7, 0, 10).startswith("err")  # > 65536

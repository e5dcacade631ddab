"""WAV ingest/egress: ``scipy.io.wavfile.read`` as the reference uses it
(dsp/src/main.py:249) and a writer.

``read(path) -> (rate, data)`` is libmsdsp's native reader (meteorgpu.ingest.read): the dtype scipy
returns for the format -- 8-bit PCM → uint8, 16-bit → int16, 24-bit → int32 (sample in the top 3
bytes, like scipy), 32-bit PCM → int32, IEEE float 32/64 → float32/float64; one channel → shape
(n,), several → (n, channels).  ``write`` emits PCM 8/16/32 or IEEE float 32/64.
``start_datetime_from_name`` restates the reference's file-name → UTC parsers
(dsp/src/main.py:858-863 gqrx names, :917-923 BRAMS MESZ names).
"""
from __future__ import annotations

import datetime
import os
import struct

import numpy as np

_PCM, _IEEE_FLOAT, _EXTENSIBLE = 0x0001, 0x0003, 0xFFFE


def read(path: str | os.PathLike, mmap: bool = False):
    """scipy.io.wavfile.read(path) through libmsdsp's native reader (msd_wav_probe / msd_wav_read:
    csrc/wav_parse.h, scipy's header rules, checked against scipy on well-formed and malformed files
    under AddressSanitizer in tests/test_sanitize.py).  Host code only, no GPU.  ``mmap`` is
    accepted for signature parity; the samples are always read into memory."""
    from . import ingest
    return ingest.read(path)


def write(path: str | os.PathLike, rate: int, data: np.ndarray) -> None:
    data = np.asarray(data)
    if data.dtype == np.int16:
        tag, bits = _PCM, 16
    elif data.dtype == np.uint8:
        tag, bits = _PCM, 8
    elif data.dtype == np.int32:
        tag, bits = _PCM, 32
    elif data.dtype == np.float32:
        tag, bits = _IEEE_FLOAT, 32
    elif data.dtype == np.float64:
        tag, bits = _IEEE_FLOAT, 64
    else:
        raise TypeError(f"unsupported dtype {data.dtype}")
    channels = 1 if data.ndim == 1 else data.shape[1]
    block_align = channels * bits // 8
    payload = np.ascontiguousarray(data).astype(data.dtype.newbyteorder("<"), copy=False).tobytes()
    with open(path, "wb") as fh:
        fh.write(b"RIFF" + struct.pack("<I", 36 + len(payload) + (len(payload) % 2)) + b"WAVE")
        fh.write(b"fmt " + struct.pack("<IHHIIHH", 16, tag, channels, int(rate), int(rate) * block_align,
                                       block_align, bits))
        fh.write(b"data" + struct.pack("<I", len(payload)))
        fh.write(payload)
        if len(payload) % 2:
            fh.write(b"\x00")


def start_datetime_from_name(file_path: str) -> datetime.datetime:
    """Recording start (UTC) from a file name, as the reference's drivers derive it.

    gqrx: ``*_gqrx_YYYYMMDD_HHMMSS_<freq>.wav`` (dsp/src/main.py:858-863);
    BRAMS: ``*_Brams_YYMMDD_HHMESZ.wav`` converted MESZ → UTC (:917-923).
    """
    parts = os.path.basename(file_path).split("_")
    if len(parts) == 5:
        return datetime.datetime.strptime(parts[2] + "-" + parts[3], "%Y%m%d-%H%M%S")
    if len(parts) == 4:
        stamp = (parts[2] + "-" + parts[3]).replace("MESZ.wav", "")
        return datetime.datetime.strptime(stamp, "%y%m%d-%H") - datetime.timedelta(hours=2)
    raise ValueError(f"cannot parse a start time from {file_path!r}")

"""WAV ingest/egress: the subset of ``scipy.io.wavfile.read`` the
reference relies on (dsp/src/main.py:249), restated on numpy.

``read(path) -> (rate, data)`` returns the dtype scipy returns for the format:
8-bit PCM → uint8, 16-bit → int16, 24-bit → int32 (sample in the top 3 bytes,
like scipy), 32-bit PCM → int32, IEEE float 32/64 → float32/float64; one
channel → shape (n,), several → (n, channels).  ``write`` emits PCM16 / float32.
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
    with open(path, "rb") as fh:
        head = fh.read(12)
        if len(head) < 12 or head[8:12] != b"WAVE" or head[:4] not in (b"RIFF", b"RIFX", b"RF64"):
            raise ValueError("File format {!r}... not understood. Only 'RIFF' WAV files are supported."
                             .format(head[:4]))
        if head[:4] == b"RIFX":
            raise ValueError("big-endian RIFX files are not supported")
        fmt = None
        while True:
            ch = fh.read(8)
            if len(ch) < 8:
                raise ValueError("Unexpected end of file: no data chunk")
            cid, size = ch[:4], struct.unpack("<I", ch[4:8])[0]
            if cid == b"fmt ":
                raw = fh.read(size)
                tag, channels, rate, _, block_align, bits = struct.unpack("<HHIIHH", raw[:16])
                if tag == _EXTENSIBLE and len(raw) >= 26:
                    tag = struct.unpack("<H", raw[24:26])[0]
                fmt = (tag, channels, rate, block_align, bits)
                if size % 2:
                    fh.read(1)
            elif cid == b"data":
                if fmt is None:
                    raise ValueError("No fmt chunk before data")
                tag, channels, rate, block_align, bits = fmt
                start = fh.tell()
                fsize = os.fstat(fh.fileno()).st_size
                size = min(size, fsize - start)
                break
            else:
                fh.seek(size + (size % 2), 1)
    tag, channels, rate, block_align, bits = fmt
    bytes_per = bits // 8
    if tag == _PCM:
        if bits == 8:
            dt = np.dtype(np.uint8)
        elif bits == 16:
            dt = np.dtype("<i2")
        elif bits == 32:
            dt = np.dtype("<i4")
        elif bits == 24:
            dt = None
        else:
            raise ValueError(f"Unsupported bit depth: the WAV file has {bits}-bit integer data.")
    elif tag == _IEEE_FLOAT:
        if bits == 32:
            dt = np.dtype("<f4")
        elif bits == 64:
            dt = np.dtype("<f8")
        else:
            raise ValueError(f"Unsupported bit depth: the WAV file has {bits}-bit floating-point data.")
    else:
        raise ValueError(f"Unknown wave file format: {tag:#06x}. Supported formats: PCM, IEEE_FLOAT")
    n_frames = size // (bytes_per * channels) if bytes_per and channels else 0
    if dt is None:  # 24-bit: pad each sample into the top 3 bytes of an int32
        raw = np.fromfile(path, dtype=np.uint8, count=n_frames * channels * 3, offset=start)
        a = np.zeros((n_frames * channels, 4), dtype=np.uint8)
        a[:, 1:] = raw.reshape(-1, 3)
        data = a.view("<i4").reshape(-1)
    elif mmap:
        data = np.memmap(path, dtype=dt, mode="c", offset=start, shape=(n_frames * channels,))
    else:
        data = np.fromfile(path, dtype=dt, count=n_frames * channels, offset=start)
    data = data.astype(data.dtype.newbyteorder("="), copy=False)
    if channels > 1:
        data = data.reshape(-1, channels)
    return rate, data


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

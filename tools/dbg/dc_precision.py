"""GPU: how the C5 spectrogram's detrend variants hold up against scipy when a large DC offset sits on
quiet noise (the post-FFT detrend subtracts two large float32 values at bins 0, 1, N-1).

For every (DC, noise sigma) the int16 I/Q stream is transformed by
  pd1   msd_cstft_psd_dev at hop 1024 (the kernel's own block sums, dc_fix_kernel),
  pd2   the same with the exact frame sums given (msd_cstft_psd_fsums_dev, the certified C5 path),
  pd0   hop 2048 (the pre-FFT detrend kernel; compared with scipy at the same hop),
and compared with scipy's float64 spectrogram: the per-frame normwise error (the tests' metric),
the relative error of bins 0, 1, N-1 one by one, and the largest error over the other bins
relative to each frame's mean power.  Usage (GPU box): python3 tools/dbg/dc_precision.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd")]

from meteorgpu import _lib, iq  # noqa: E402
from meteorgpu.dsp import context  # noqa: E402
from oracle import iq_oracle as Q  # noqa: E402


def run(i, q, noverlap, given):
    fs, n = 192000, i.size
    x = np.empty(2 * n, np.int16)
    x[0::2], x[1::2] = i, q
    ctx = context(0)
    b = iq.IQBatch(ctx, 1, n, fs, 4096, noverlap)
    b.upload(0, x)
    fsum = None
    if given:
        T = b.T
        fsum = ctx.alloc(16 * T)
        d, e = ctx.alloc(8 * T), ctx.alloc(8 * T)
        band, noise = iq.iq_band_bins(4096, fs, (950.0, 1050.0)), iq.iq_band_bins(4096, fs, (-3050.0, -2950.0))
        _lib.iq_delta64_dev(ctx, b.d_x, b.code, n, 4096, 1024, float(fs), band, noise,
                            np.array([[0, T]], np.int64), d, e, frame_sums=fsum)
    b.run(fsums=fsum)
    S = b.frames(0, 0, b.T).T.astype(np.float64)
    b.close()
    return S


def metrics(S, R):
    rel = np.linalg.norm(S - R, axis=0) / np.linalg.norm(R, axis=0)
    mean = R.mean(axis=0)
    out = {"frame": rel.max()}
    for k in (0, 1, 4095):
        out[f"b{k}"] = float(np.max(np.abs(S[k] - R[k]) / np.maximum(R[k], 1e-300)))
    other = np.abs(S[2:4095] - R[2:4095]) / mean
    out["other/mean"] = float(other.max())
    out["b0/mean"] = float(np.max(np.abs(S[0] - R[0]) / mean))
    return out


def main():
    rng = np.random.default_rng(5)
    n = 60000
    print(f"{'dc':>6} {'sigma':>6} {'var':>4} {'frame':>9} {'b0':>9} {'b1':>9} {'bN-1':>9} {'b0/mean':>9} {'oth/mean':>9}")
    for dc in (0, 700, 4000, 16000, 30000):
        for sigma in (3.0, 30.0, 600.0):
            z = sigma * (rng.standard_normal(n) + 1j * rng.standard_normal(n)) + dc * (1 - 0.5j)
            i = np.clip(np.round(z.real), -32768, 32767).astype(np.int16)
            q = np.clip(np.round(z.imag), -32768, 32767).astype(np.int16)
            for var, nov, given in (("pd1", 3072, False), ("pd2", 3072, True), ("pd0", 2048, False)):
                S = run(i, q, nov, given)
                _, _, R = Q.spectrogram_iq_ref(i, q, 192000, 4096, nov)
                m = metrics(S, R)
                print(f"{dc:>6} {sigma:>6g} {var:>4} {m['frame']:9.2e} {m['b0']:9.2e} {m['b1']:9.2e} "
                      f"{m['b4095']:9.2e} {m['b0/mean']:9.2e} {m['other/mean']:9.2e}", flush=True)


if __name__ == "__main__":
    main()

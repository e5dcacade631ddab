"""GPU: a randomised sweep of the int16 block energies on the int8 matrix-core path
(csrc/block_i8.hip) against the reference's numpy blocks (oracle/dsp_oracle.block_powers_ref) and
the float64 Goertzel path (MSD_OPT_BLOCK_GOERTZEL): random block lengths with L = 256, 512 or 1024,
random bands of 1-8 bins (DC and Nyquist included), random noise + tone + DC signals.  Prints the
largest |dB| difference per config; exits 1 if any exceeds 1e-9 dB.
Usage (GPU box): python3 tools/dbg/block_i8_sweep.py [CONFIGS]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd")]

from meteorgpu import _lib, dsp  # noqa: E402
from oracle import dsp_oracle as O  # noqa: E402


def main():
    nconf = int(sys.argv[1]) if len(sys.argv) > 1 else 120
    rng = np.random.default_rng(2025)
    ctx = dsp.context(0)
    worst = 0.0
    bad = 0
    for c in range(nconf):
        L = int(rng.choice([256, 512, 1024]))
        n_fft = int(rng.choice([L // 2, L, 2 * L])) if rng.random() < 0.5 else L // 2
        nfft = 2 * n_fft
        B = L if nfft > L else int(rng.integers(L, 4 * L))  # B > L crops, B = L < nfft zero-pads
        Lr = min(B, nfft)
        if Lr != L:
            continue
        fs = float(rng.choice([4000, 6000, 8000, 16000, 44100, 48000]))
        bs = B / fs
        df = fs / nfft
        nb = int(rng.integers(1, 5))
        nn = int(rng.integers(0, 9 - nb))
        kb = int(rng.integers(0, nfft // 2 + 1 - nb))
        kn = int(rng.integers(0, nfft // 2 + 1 - max(nn, 1)))
        band = ((kb - 0.25) * df, (kb + nb - 0.75) * df)
        noise = ((kn - 0.25) * df, (kn + nn - 0.75) * df) if nn else (fs, fs - 1)
        bb, nbb = dsp.band_bins(nfft, fs, band), dsp.band_bins(nfft, fs, noise)
        nbins = max(0, bb[1] - bb[0] + 1) + max(0, nbb[1] - nbb[0] + 1)
        if not 1 <= nbins <= 8:
            continue
        nblocks = int(rng.integers(1, 80))
        t = np.arange(nblocks * B + int(rng.integers(0, B))) / fs
        amp = float(rng.choice([3, 300, 3000, 20000]))
        x = amp * rng.standard_normal(t.size) + float(rng.integers(-3000, 3000))
        x += 5000 * np.sin(2 * np.pi * (kb + 0.3) * df * t)
        x = np.clip(np.round(x), -32768, 32767).astype(np.int16)
        B_ = int(fs * bs)
        if B_ != B:
            continue
        plan = _lib.BlockPlan(ctx, B, nfft, dsp.hanning_sym(B)[:L], bb, nbb)
        try:
            b8, n8, d8 = plan.run(x)
            ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 1)
            bg, ng, dg = plan.run(x)
        finally:
            ctx.set_option(_lib.OPT_BLOCK_GOERTZEL, 0)
            plan.close()
        rb, rn, rd = O.block_powers_ref(x, fs, bs, band, noise, n_fft)
        e = max(float(np.abs(b8 - rb).max()), float(np.abs(n8 - rn).max()), float(np.abs(d8 - rd).max()),
                float(np.abs(d8 - dg).max()))
        worst = max(worst, e)
        flag = e > 1e-9
        bad += flag
        print(f"{c:4d} L {L:5d} B {B:5d} nfft {nfft:5d} fs {fs:7.0f} bins {nbins} ({bb}, {nbb}) blocks {nblocks:3d} "
              f"amp {amp:6.0f}  max|dB diff| {e:.3e}{'  <-- over 1e-9' if flag else ''}", flush=True)
    print(f"worst {worst:.3e} dB, {bad} configs over 1e-9 dB")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()

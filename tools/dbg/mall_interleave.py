"""GPU: does a chunk-interleaved C5 step let the exact delta's sample reads come from the 256 MB
Infinity Cache (MALL) instead of HBM?  

The shard's samples stay resident.  For a chunk of F frames the spectrogram (cstft4096_kernel, own
frame sums) runs first and leaves the chunk's samples in the cache if they and the chunk's output
fit, then the exact delta step (block_i8_kernel + frame_kernel, msd_iq_delta64_sums_dev over the
same frames) reads them again.  Printed per chunk size: the delta step's device time summed over the
chunks against the same frames in one launch (HIP events, library timers), the spectrogram's likewise,
and the whole sequence's wall time.  A MALL hit shows as a delta faster per frame than in one launch,
and as less FETCH_SIZE for block_i8_kernel under rocprofv3 --pmc (one chunk size per run: argv).
Usage (GPU box): python3 tools/dbg/mall_interleave.py [FRAMES_PER_CHUNK ...]
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd")]

from meteorgpu import _lib, iq, synth  # noqa: E402

FS, N, HOP = 192000, 4096, 1024


def main():
    ctx = _lib.Context(0)
    nfr = 1 << 18  # 262 144 frames: 1/8 of the 3 h shard, 1.07 GB of int16 I/Q
    n = (nfr - 1) * HOP + N
    i_, q_, _ = synth.synth_iq(7, FS, 60.0, 1000.0, sigma=1000.0, rate_per_min=6)
    z = np.empty(2 * i_.size, np.int16)
    z[0::2], z[1::2] = i_, q_
    x = np.resize(z, 2 * n)
    batch = iq.IQBatch(ctx, 1, n, FS, N, N - HOP)
    batch.upload(0, x)
    band, noise = iq.iq_band_bins(N, FS, (950.0, 1050.0)), iq.iq_band_bins(N, FS, (-3050.0, -2950.0))
    d, e, fs = ctx.alloc(8 * nfr), ctx.alloc(8 * nfr), ctx.alloc(16 * nfr)
    off, ln = ctx.alloc(8), ctx.alloc(8)
    plan = batch.plan

    def chunked(F, reps=3):
        """every chunk: spectrogram of its frames, then the exact delta of the same frames"""
        best = None
        for _ in range(reps):
            ctx.timing(True)
            ctx.timing_reset()
            ctx.synchronize()
            t0 = time.perf_counter()
            for c0 in range(0, nfr, F):
                f = min(F, nfr - c0)
                off.upload(np.array([c0 * HOP], np.int64))
                ln.upload(np.array([(f - 1) * HOP + N], np.int64))
                plan.run_dev(batch.d_x, batch.code, off, ln, 1, f, batch.d_out)  # its own frame sums
                _lib.iq_delta64_dev(ctx, batch.d_x, batch.code, n, N, HOP, float(FS), band, noise,
                                    np.array([[c0, c0 + f]], np.int64), d, e, frame_sums=fs)
            ctx.synchronize()
            wall = time.perf_counter() - t0
            spec = ctx.timing_get(_lib.K_CSTFT)[0]
            dlt = ctx.timing_get(_lib.K_REFINE)[0]
            r = (wall * 1e3, spec, dlt)
            best = r if best is None or r[0] < best[0] else best
        ctx.timing(False)
        return best

    print(f"{nfr} frames ({n * 4 / 1e9:.2f} GB of samples, {nfr * N * 4 / 1e9:.2f} GB of spectrogram)")
    print(f"{'chunk frames':>12} {'samples MB':>10} {'out MB':>8} {'wall ms':>9} {'spec ms':>9} {'delta ms':>9} "
          f"{'delta/frame ns':>14}")
    sizes = [int(a) for a in sys.argv[1:]] or [nfr, 32768, 16384, 8192, 4096, 2048]
    for F in sizes:  # (one size and one repetition under rocprofv3 --pmc FETCH_SIZE: argv)
        wall, spec, dlt = chunked(F, reps=1 if len(sys.argv) > 1 else 3)
        print(f"{F:>12} {F * HOP * 4 / 1e6:>10.1f} {F * N * 4 / 1e6:>8.1f} {wall:>9.3f} {spec:>9.3f} {dlt:>9.3f} "
              f"{dlt * 1e6 / nfr:>14.2f}", flush=True)
    for b in (d, e, fs, off, ln):
        b.free()
    batch.close()


if __name__ == "__main__":
    main()

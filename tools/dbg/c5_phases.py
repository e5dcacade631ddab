"""Debug (GPU box): wall time of each phase of one C5 step (spectrogram + delta, then every
StreamDetector device call with a synchronize) on the 3 h bench shard."""
import os, sys, time
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "meteor-scatter_amd")]
import numpy as np
from meteorgpu import _lib, iq, stream, synth
ctx = _lib.Context(0)
FS, N, HOP = 192000, 4096, 1024
shard = FS * 3 * 3600
det = iq.IQShardDetector(ctx, shard + N - HOP, FS, N, N - HOP, (950.0, 1050.0), (-3050.0, -2950.0), 4.0, True)
chunk = FS * 60
pool = []
for j in range(4):
    i_, q_, _ = synth.synth_iq(5000 + j, FS, 60.0, 1000.0, sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))
    z = np.empty(2 * chunk, np.int16); z[0::2], z[1::2] = i_, q_
    pool.append(z)
n = det.s1 - det.s0; pos = k = 0
while pos < n:
    m = min(chunk, n - pos); det.upload(pool[k % 4][: 2 * m], sample_offset=pos); pos += m; k += 1
T = {}
def wrap(obj, name):
    f = getattr(obj, name)
    def g(*a, **kw):
        t = time.perf_counter(); r = f(*a, **kw); ctx.synchronize(); T[name] = T.get(name, 0) + time.perf_counter() - t; return r
    setattr(obj, name, g)
for nm in ("fresh", "refine", "chunk_sums", "scan", "runs", "db", "set_halos", "thresholds"):
    wrap(det.ops, nm)
for it in range(3):
    T.clear()
    t0 = time.perf_counter()
    det.spectrogram_and_delta(); ctx.synchronize(); t1 = time.perf_counter()
    res = det.detect(thresholds=False); ctx.synchronize(); t2 = time.perf_counter()
    print(f"spec {1e3*(t1-t0):.2f} detect {1e3*(t2-t1):.2f}", {k: round(v * 1e3, 2) for k, v in T.items()}, flush=True)

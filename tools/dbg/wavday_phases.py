"""Diagnostic (GPU): where WavDay.run's wall time goes (480 one-minute 48 kHz files, warm page
cache): host time inside read / upload-enqueue / pipeline-enqueue / detections().  Not a test."""
import collections
import datetime
import os
import shutil
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "meteor-scatter_amd"))
from meteorgpu import _lib, ingest, synth, wav  # noqa: E402

FS = 48000
ctx = _lib.Context(0)
pool = [synth.synth_real(seed=2000 + j, fs=FS, duration_s=60.0, f0=1000.0)[0] for j in range(16)]
d = tempfile.mkdtemp(prefix="msd_wavph_", dir=os.environ.get("TMPDIR", "/tmp"))
paths = []
for i in range(480):
    t = datetime.datetime(2025, 6, 1) + datetime.timedelta(minutes=i)
    p = os.path.join(d, f"SDR_gqrx_{t:%Y%m%d}_{t:%H%M%S}_49969000.wav")
    wav.write(p, FS, pool[i % 16])
    paths.append(p)
readers = int(sys.argv[1]) if len(sys.argv) > 1 else 8
bf = int(sys.argv[2]) if len(sys.argv) > 2 else 120
wd = ingest.WavDay(ctx, paths, batch_files=bf, readers=readers, freq_band=(950, 1050), noise_band=(2950, 3050),
                   n_fft=512, nperseg=1024, noverlap=512)
acc = collections.defaultdict(float)


def wrap(obj, name):
    f = getattr(obj, name)

    def g(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[name] += time.perf_counter() - t0
        return r
    setattr(obj, name, g)


for obj, name in ((wd, "_read_batch"), (wd, "_upload"), (wd.bp, "run"), (wd.bp, "detections"), (wd.bp, "hour_counts"), (wd.bp, "_near_ties")):
    wrap(obj, name)
wd.run()
for rep in range(4):
    acc.clear()
    t0 = time.perf_counter()
    wd.run()
    wall = time.perf_counter() - t0
    print(f"readers {readers} batch {bf} wall {wall * 1e3:.1f} ms: " + ", ".join(f"{k} {v * 1e3:.1f}" for k, v in acc.items()),
          flush=True)
shutil.rmtree(d, ignore_errors=True)

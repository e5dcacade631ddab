"""Debug (GPU box): the segment-boundary case of tests/test_gpu_live.py over many random streams
(argv[1] seeds, default 60; lengths and settings drawn per seed) against the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd"), os.path.join(ROOT, "tests")]
from meteorgpu import live  # noqa: E402
from oracle import live_oracle as L  # noqa: E402
from test_gpu_live import _ref_cfg  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 60
bad = 0
for seed in range(n):
    rng = np.random.default_rng(500 + seed)
    nb = int(rng.choice([16, 33, 250, 1000, 5000, 18000]))
    sig = rng.normal(0, 1, nb)
    for s in rng.integers(0, nb, max(1, nb // int(rng.choice([10, 40, 200])))):
        sig[s: s + rng.integers(1, 60)] += rng.uniform(3, 30)
    rows = np.stack([sig, rng.normal(0, 0.5, nb), rng.normal(0, 0.5, nb)])
    kw = dict(after_tracking_wait_sec=float(rng.choice([0.0, 2.0, 12.0, 60.0])),
              init_detection_wait_sec=float(rng.choice([0.0, 8.0, 100.0])),
              avg_win_sec=float(rng.choice([0.2, 8.0, 40.0])),
              detection_dur_min_sec=float(rng.choice([0.0, 0.4, 1.0])))
    cfg = live.ConfigDetection(**kw)
    m, thr, over = live.live_detect(rows, 4000, cfg)
    rm, rthr, rover = L.live_detect_ref(rows, 4000, 800, _ref_cfg(cfg))
    ok = np.array_equal(thr, rthr, equal_nan=True) and \
        [(a.time_start, a.time_stop, a.db_min, a.db_max, a.db_mean, a.db_std) for a in m] == \
        [(b.time_start, b.time_stop, b.db_min, b.db_max, b.db_mean, b.db_std) for b in rm]
    if not ok:
        bad += 1
        print("FAIL", seed, nb, kw, len(m), len(rm), flush=True)
print(f"{n} seeds, {bad} failures", flush=True)

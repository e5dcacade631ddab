"""Debug (GPU box): fraction of frames / 512-frame tiles where the adaptive detector recomputes
its threshold on the C5 bench stream (how much exact-threshold work the refine scheme needs)."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "meteor-scatter_amd")]
import numpy as np
from meteorgpu import synth, iq
chunks = [synth.synth_iq(5000 + j, 192000, 60.0, 1000.0, sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))[:2] for j in range(4)]
i = np.concatenate([c[0] for c in chunks] * 3); q = np.concatenate([c[1] for c in chunks] * 3)
dets, thr, delta, res = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950))
thr = np.asarray(thr)
ch = np.flatnonzero(thr[1:] != thr[:-1]) + 1
T = thr.size
print("frames", T, "dets", len(dets), "changing-thr frames", ch.size, "frac", ch.size / T)
tiles = np.unique(ch // 512)
print("tiles needed", tiles.size, "of", -(-T // 512))
print("first dets", [(round(d.t_start, 3), round(d.t_stop, 3)) for d in dets[:20]])

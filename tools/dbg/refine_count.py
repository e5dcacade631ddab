"""Debug (GPU box): tiles computed by each msd_stream_refine call on an N-minute bench-like I/Q
stream (argv[1] minutes), against the tiles where the thresholds actually change."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "..", "meteor-scatter_amd")]
import numpy as np
from meteorgpu import synth, iq, stream, _lib
from meteorgpu.dsp import context
minutes = int(sys.argv[1]) if len(sys.argv) > 1 else 12
chunks = [synth.synth_iq(5000 + j, 192000, 60.0, 1000.0, sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))[:2] for j in range(4)]
rep = minutes // 4
i = np.concatenate([c[0] for c in chunks] * rep); q = np.concatenate([c[1] for c in chunks] * rep)
orig = stream.DeviceStreamOps.refine
def refine(self):
    n = orig(self)
    print("refine computed", n, "of", self.plan.nseg * 0 + -(-self.n_local // 512), "tiles", flush=True)
    return n
stream.DeviceStreamOps.refine = refine
dets, thr, delta, res = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950))
thr = np.asarray(thr)
ch = np.flatnonzero(thr[1:] != thr[:-1]) + 1
print("frames", thr.size, "dets", len(dets), "tiles with thr changes", np.unique(ch // 512).size)

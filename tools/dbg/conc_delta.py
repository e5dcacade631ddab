"""GPU experiment: the certified C5 step with the exact delta running CONCURRENTLY with the
spectrogram instead of before it.

Today's step (iq.IQShardDetector.spectrogram_and_delta, exact delta, --c5-overlap n): the exact delta
(block_i8_kernel + frame_kernel, 1.87 ms, full chip) runs first, then the spectrogram (sibling context,
n workgroup slots reserved) beside the detector.  Here the spectrogram does not wait for the delta: it
takes its own frame sums (PD 0 instead of the delta's sums) and its guided chunk schedule lets
workgroups that the delta's kernels keep from dispatching join late.  The detector still waits for
the delta.  CONC_ORDER=delta_first (default) enqueues the delta before the spectrogram,
spec_first after it.

Usage (GPU box): python3 tools/dbg/conc_delta.py [bench.py args]   (CONC_ORDER=delta_first|spec_first)
"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd")]

import numpy as np  # noqa: E402

from meteorgpu import iq  # noqa: E402

ORDER = os.environ.get("CONC_ORDER", "delta_first")


def spectrogram_and_delta(self):
    self._refined = iq._NO_IV
    self._step_start()
    if self.f1 > self.f0:
        if not self.exact_delta or self.sctx is self.ctx:
            raise SystemExit("conc_delta: needs the exact delta and --c5-overlap > 0")
        self._after(self.sctx, self.ctx)  # what the caller enqueued before (uploads), not the delta
        if ORDER == "delta_first":
            self._delta_exact(self.batch.n, self.f1 - self.f0, 0)
            self.batch.run(fsums=None)
        else:
            self.batch.run(fsums=None)
            self._delta_exact(self.batch.n, self.f1 - self.f0, 0)
        self._after(self.dctx, self.ctx)
    self._refined = np.array([[0, self.T]], np.int64)


iq.IQShardDetector.spectrogram_and_delta = spectrogram_and_delta
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")

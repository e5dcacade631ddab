"""GPU: the ctypes stub INTEGRATION.md §2 shows a maintainer (the reference's main.py:352-393 and
:450-522 through the bare C-ABI, no meteorgpu) runs as printed and gives the oracle's detections."""
import os
import re

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_integration_ctypes_stub_runs():
    from meteorgpu import synth
    from oracle import dsp_oracle as O
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    code = re.search(r"## 2\. C-ABI level.*?```python\n(.*?)```", doc, re.S).group(1)
    samples, _ = synth.synth_real(seed=42, fs=6000, duration_s=120.0, f0=1003.0, band_hz=20.0, rate_per_min=10)
    env = {"samples": samples}
    cwd = os.getcwd()
    os.chdir(ROOT)  # the stub loads the library by its in-tree path
    try:
        exec(compile(code, "INTEGRATION.md", "exec"), env)
    finally:
        os.chdir(cwd)
    cnt, dets, bs = env["cnt"].value, env["dets"], env["bs"]
    got = [(dets[j].start * bs, dets[j].stop * bs) for j in range(cnt)]
    want, *_ = O.proc_samples_ref(samples, 6000, 0.2, (993, 1013), (690, 710), 512, 4.0)
    assert len(want) > 0
    assert got == [(w[0], w[1]) for w in want]

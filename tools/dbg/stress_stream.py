"""Debug (GPU box): run the randomised sharded-device parity case of tests/test_gpu_stream.py for
many more seeds (argv[1], default 80), with the thresholds output and in decisions-only mode,
and report failures."""
import os
import sys

ROOT = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd"), os.path.join(ROOT, "tests")]
import pytest  # noqa: E402

import test_gpu_stream as T  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 80
bad = []
for seed in range(100, 100 + n):
    for thresholds in (True, False):
        try:
            T._random_case(seed, thresholds)
        except pytest.skip.Exception:
            pass
        except Exception as e:  # noqa: BLE001
            bad.append((seed, thresholds, repr(e)[:200]))
            print("FAIL", seed, thresholds, repr(e)[:200], flush=True)
print(f"{n} seeds, {len(bad)} failures", flush=True)

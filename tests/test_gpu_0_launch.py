"""GPU: bench.py through the torch-free launcher (--spawn at --gpus 1: rendezvous file, RCCL
communicator, barrier / max / rank count through libmsdsp) for the three workloads the
multi-GPU configs use -- C3 (a day per GPU), C4 (--shard-day) and C5 (the I/Q stream with its
RCCL exchanges).  Named to run first in `-m gpu`, so the pytest process has not opened the
GPU when it starts the child."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "MSD_RDZV_KEY"):
        e.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--spawn", "--steps", "2",
                        "--warmup", "1", "--no-cpu-baseline", *args], capture_output=True, text=True,
                       timeout=timeout, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["value"] > 0
    return d


def test_spawn_c3():
    """the default line: C3 (weak), the C4 strong-scaling pass over the same ranks, C5 and live appended"""
    d = _bench("--files", "16", "--c5-seconds", "60")
    assert d["scaling"] == "weak" and d["config"]["files_per_gpu"] == 16 and d["roofline"]["frac"] > 0
    s = d["strong_scaling"]
    assert s["scaling"] == "strong" and s["files_total"] == 16 and s["ranks_seen"] == 1 and s["value"] > 0
    assert s["hour_total"] == s["detections_per_step"] == d["detections_per_step"]  # same day at N = 1
    c5 = d["c5"]
    assert c5["value"] > 0 and c5["roofline"]["frac"] > 0 and c5["detections_per_step"] > 0
    lv = d["live"]  # the live detector's day (round 6), through the same launched rank
    assert lv["value"] > 0 and lv["ranks_seen"] == 1 and lv["meteors_per_step"] > 0
    assert lv["near_tie"]["files"] == 24 and lv["near_tie"]["files_flagged"] == 0


def test_spawn_c4_shard_day():
    d = _bench("--files", "24", "--shard-day")
    assert d["scaling"] == "strong" and d["config"]["files_per_gpu"] == 24


def test_spawn_c5():
    d = _bench("--workload", "c5", "--c5-seconds", "300")
    assert d["config"]["samples_per_gpu"] == 192000 * 300 and d["detections_per_step"] > 0

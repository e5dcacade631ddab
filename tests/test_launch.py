"""The torch-free N-rank launcher (meteorgpu.launch, bench.py --gpus N) on the CPU: ranks are
started before any GPU call, share one RCCL-id-sized blob through the rendezvous file, and a
failing rank fails the job.  Covers both entries the driver uses: bench.py spawning its own
ranks, and `python -m torch.distributed.run ... bench.py --gpus N` setting WORLD_SIZE."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(cmd, env=None, timeout=120):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "MSD_RDZV_KEY"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e, cwd=ROOT)


@pytest.mark.parametrize("n", [2, 3, 8])
def test_bench_spawns_n_ranks(n, tmp_path):
    """N = 8 is the driver's full-node SCALE run: eight interpreters, one rendezvous"""
    r = _run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env={"MSD_RDZV_DIR": str(tmp_path)})
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    d = json.loads(lines[0])
    strong = d.pop("strong_scaling")
    c5 = d.pop("c5")
    live = d.pop("live")
    assert d == {"dry_run": True, "n_gpus": n, "ranks_seen": n, "id_agreed": True}
    assert c5 == {"ranks_seen": n}  # the C5 leg's own rank count (weak-scaled stream)
    assert live == {"ranks_seen": n}  # the live leg's (a day of 4 kHz audio per rank)
    # the C4 (strong scaling) pass the real N-rank line carries: one 1440-file day over the n ranks
    assert strong["scaling"] == "strong" and strong["files_total"] == 1440
    assert sum(strong["files_per_rank"]) == 1440 and max(strong["files_per_rank"]) == -(-1440 // n)
    assert not list(tmp_path.iterdir())  # rendezvous files cleaned up


def test_bench_under_torchrun(tmp_path):
    """the driver's N>1 command line: torchrun sets WORLD_SIZE, bench.py must not spawn again"""
    from meteorgpu import launch
    r = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
              "--master-addr", "127.0.0.1", "--master-port", str(launch.free_port()), BENCH, "--gpus", "2",
              "--dry-run"], env={"MSD_RDZV_DIR": str(tmp_path)}, timeout=180)
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and json.loads(lines[0])["ranks_seen"] == 2


def test_world_mismatch_is_an_error(tmp_path):
    r = _run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
             env={"WORLD_SIZE": "1", "RANK": "0", "MSD_RDZV_DIR": str(tmp_path)})
    assert r.returncode != 0 and "--gpus 4" in r.stderr


def test_failing_rank_fails_the_job(tmp_path):
    from meteorgpu import launch
    script = tmp_path / "w.py"
    script.write_text("import os, sys, time\n"
                      "r = int(os.environ['RANK'])\n"
                      "if r == 1: sys.exit(3)\n"
                      "time.sleep(60)\n")
    import time
    t0 = time.monotonic()
    rc = launch.spawn([str(script)], 3)
    assert rc == 3 and time.monotonic() - t0 < 30  # the sleeping ranks were terminated


def test_env_and_keys(monkeypatch, tmp_path):
    from meteorgpu import launch
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MSD_RDZV_KEY"):
        monkeypatch.delenv(k, raising=False)
    assert launch.env_world() == (0, 1, 0) and not launch.launched()
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "2")
    assert launch.env_world() == (2, 4, 2)
    monkeypatch.setenv("RANK", "4")
    with pytest.raises(ValueError):
        launch.env_world()
    monkeypatch.setenv("MASTER_PORT", "1234")
    k1 = launch.rdzv_key()
    monkeypatch.setenv("MASTER_PORT", "1235")
    assert launch.rdzv_key() != k1  # two launches on one node do not collide
    monkeypatch.setenv("MSD_RDZV_DIR", str(tmp_path))
    monkeypatch.setenv("MSD_RDZV_KEY", "t")
    with pytest.raises(TimeoutError):
        launch.share_bytes(1, lambda: b"", tag="never", timeout=0.2)
    assert launch.share_bytes(0, lambda: b"abc", tag="x") == b"abc"
    assert launch.share_bytes(1, lambda: b"", tag="x") == b"abc"
    launch.release(0, tag="x")
    assert not list(tmp_path.iterdir())


def test_rdzv_key_restart_and_single_node(monkeypatch):
    """an elastic restart gets a new key (a failed attempt's file is never read), and a multi-node
    launch is refused (the rendezvous file is node-local)"""
    from meteorgpu import launch
    monkeypatch.delenv("MSD_RDZV_KEY", raising=False)
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "2")
    monkeypatch.setenv("MASTER_PORT", "1234")
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "0")
    k0 = launch.rdzv_key()
    monkeypatch.setenv("TORCHELASTIC_RESTART_COUNT", "1")
    assert launch.rdzv_key() != k0
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "1")
    with pytest.raises(RuntimeError, match="single-node"):
        launch.rdzv_key()


def test_rank_dying_after_init_fails_the_job(tmp_path):
    """a rank that exits after the communicator rendezvous (the others blocked waiting for it, as
    in a collective) makes bench.py's parent exit with its code well within the rendezvous
    timeout, and every sibling rank is terminated and reaped (spawn starts children; nothing
    re-execs)"""
    import time
    pids = tmp_path / "pids"
    pids.mkdir()
    t0 = time.monotonic()
    r = _run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
             env={"MSD_RDZV_DIR": str(tmp_path), "MSD_DRYRUN_FAIL_RANK": "2", "MSD_DRYRUN_PID_DIR": str(pids)},
             timeout=100)
    assert r.returncode == 7, (r.returncode, r.stderr[-2000:])
    assert time.monotonic() - t0 < 60  # not the 120 s rendezvous timeout of the blocked ranks
    got = sorted(pids.iterdir())
    assert len(got) == 4
    for f in got:
        pid = int(f.read_text())
        assert pid != os.getpid()
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)  # gone (spawn waited for it: no zombie left either)
    assert not [p for p in tmp_path.iterdir() if p.name.startswith("msd_rdzv_")]  # rendezvous cleaned up


def test_rccl_init_failure_text_reaches_the_parent(tmp_path):
    """a rank whose communicator init fails: the parent's exit message names the rank and carries
    libmsdsp's own error text (msd_last_error through MsdError), not only an exit code"""
    r = _run([sys.executable, BENCH, "--gpus", "3", "--dry-run"],
             env={"MSD_RDZV_DIR": str(tmp_path), "MSD_DRYRUN_RCCL_FAIL_RANK": "1"}, timeout=100)
    assert r.returncode != 0
    line = [ln for ln in r.stderr.splitlines() if ln.startswith("meteorgpu.launch: rank 1 of 3")]
    assert line, r.stderr[-2000:]
    assert "RCCL communicator init failed" in line[0] and "ncclCommInitRank" in line[0], line[0]
    assert not [p for p in tmp_path.iterdir() if p.name.startswith("msd_rdzv_")]

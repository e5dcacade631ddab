"""One process per GPU without PyTorch: the launcher, the RCCL id rendezvous and the job group.

The reference is single-process (dsp/src/main.py:865-946 loops over files); the N-GPU form of
the path is N processes, one per GPU, over one RCCL communicator.  Nothing
here imports torch: the 128-byte RCCL unique id travels through a file that rank 0 writes
atomically into a directory every rank of the node sees, and the job's barrier, rank count
and max-over-ranks timing go through libmsdsp's RCCL wrappers (msd_comm_allreduce_i64 /
msd_comm_allgather, include/msdsp.h).

Two ways in:
  * ``spawn(argv, n)`` — a parent that has NOT touched the GPU starts ``n`` fresh interpreters
    with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT and a unique rendezvous
    key, waits for all of them, and returns the first failing exit code (the others are then
    terminated).  ``bench.py --gpus N`` uses it when WORLD_SIZE is unset.
  * an external launcher (``python -m torch.distributed.run ... bench.py``) sets the same
    variables; the rendezvous key is then derived from its run id and restart count, the shared
    parent PID and MASTER_PORT, which every worker of one launch attempt has in common.  Jobs
    must be single-node (LOCAL_WORLD_SIZE == WORLD_SIZE, checked).
"""
from __future__ import annotations

import hashlib
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np

RDZV_TIMEOUT_S = 120.0


def env_world() -> tuple[int, int, int]:
    """(rank, world, local_rank) from the launcher's environment; (0, 1, 0) without one."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world < 1 or not 0 <= rank < world or local < 0:
        raise ValueError(f"bad launcher environment: RANK={rank} WORLD_SIZE={world} LOCAL_RANK={local}")
    return rank, world, local


def launched() -> bool:
    return "WORLD_SIZE" in os.environ


def _rdzv_dir() -> str:
    return os.environ.get("MSD_RDZV_DIR") or tempfile.gettempdir()


def rdzv_key() -> str:
    """Key shared by the ranks of one launch and by nothing else: ``MSD_RDZV_KEY`` when spawn()
    started us, otherwise the external launcher's run id + parent PID + master port."""
    k = os.environ.get("MSD_RDZV_KEY")
    if k:
        return k
    check_single_node()
    # the restart count separates the attempts of an elastic job: a failed attempt may leave its
    # file behind (no release()), and the next attempt's ranks must not read the old RCCL id
    raw = "|".join((os.environ.get("TORCHELASTIC_RUN_ID", ""), os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"),
                    str(os.getppid()), os.environ.get("MASTER_ADDR", ""), os.environ.get("MASTER_PORT", "")))
    return hashlib.sha1(raw.encode()).hexdigest()[:16]


def check_single_node() -> None:
    """The file rendezvous needs every rank on one node (one shared directory, one parent PID):
    refuse a launch whose LOCAL_WORLD_SIZE differs from WORLD_SIZE."""
    world = os.environ.get("WORLD_SIZE")
    local = os.environ.get("LOCAL_WORLD_SIZE")
    if world is not None and local is not None and int(local) != int(world):
        raise RuntimeError(f"meteorgpu.launch: single-node jobs only (LOCAL_WORLD_SIZE={local}, "
                           f"WORLD_SIZE={world}); the RCCL id rendezvous goes through a node-local file")


def rdzv_path(tag: str = "rccl") -> str:
    return os.path.join(_rdzv_dir(), f"msd_rdzv_{rdzv_key()}_{tag}.bin")


def share_bytes(rank: int, make, tag: str = "rccl", timeout: float = RDZV_TIMEOUT_S) -> bytes:
    """Rank 0 calls ``make()`` and publishes the bytes (write to a temporary name, then an
    atomic rename); every other rank waits for the file and reads it.  Raises TimeoutError
    when rank 0 never publishes."""
    path = rdzv_path(tag)
    if rank == 0:
        data = bytes(make())
        tmp = f"{path}.{os.getpid()}.tmp"
        with open(tmp, "wb") as fh:
            fh.write(len(data).to_bytes(4, "little") + data)
            fh.flush()
            os.fsync(fh.fileno())
        os.replace(tmp, path)
        return data
    t_end = time.monotonic() + timeout
    while True:
        try:
            with open(path, "rb") as fh:
                blob = fh.read()
            if len(blob) >= 4 and len(blob) == 4 + int.from_bytes(blob[:4], "little"):
                return blob[4:]
        except FileNotFoundError:
            pass
        if time.monotonic() > t_end:
            raise TimeoutError(f"rank {rank}: no rendezvous file {path} after {timeout:.0f} s")
        time.sleep(0.01)


def release(rank: int, tag: str = "rccl") -> None:
    """Rank 0 removes the rendezvous file once every rank has read it (after a barrier)."""
    if rank == 0:
        try:
            os.unlink(rdzv_path(tag))
        except FileNotFoundError:
            pass


def report_failure(rank: int, text: str) -> None:
    """A rank's failure text for the parent: spawn() prints it beside the exit code (only under
    spawn, whose rendezvous key names the file and whose cleanup removes it)."""
    if not os.environ.get("MSD_RDZV_KEY"):
        return
    try:
        with open(rdzv_path(f"err{rank}"), "w") as fh:
            fh.write(text[-4000:])
    except OSError:
        pass


def _failure_text(key: str, rank: int) -> str:
    try:
        with open(os.path.join(_rdzv_dir(), f"msd_rdzv_{key}_err{rank}.bin")) as fh:
            return fh.read().strip()
    except OSError:
        return ""


def open_comm(make, rank: int):
    """``make()`` → the job's RCCL communicator.  A failure keeps libmsdsp's own message (the
    ``msd_last_error`` text MsdError carries: RCCL's error string, a missing librccl, a bad id)
    and names the rank, so the parent's exit message says why the job failed."""
    try:
        return make()
    except Exception as e:  # noqa: BLE001 -- re-raised with the rank and the library's text
        raise RuntimeError(f"rank {rank}: RCCL communicator init failed: {e}") from e


def free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn(argv: list[str], nprocs: int, env: dict | None = None, poll_s: float = 0.05) -> int:
    """Run ``[sys.executable, -u, *argv]`` as ``nprocs`` ranks and wait for them.  The caller
    must not have initialised the GPU (the children each open their own device).  Rank 0's
    stdout is this process's stdout; the other ranks' stdout goes to stderr so that only rank
    0's result line lands on stdout.  Returns 0, or the first non-zero exit code (after
    terminating the ranks still running)."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    base = dict(os.environ if env is None else env)
    base.update(WORLD_SIZE=str(nprocs), LOCAL_WORLD_SIZE=str(nprocs), MASTER_ADDR="127.0.0.1",
                MASTER_PORT=str(free_port()), MSD_RDZV_KEY=f"{os.getpid()}-{time.time_ns():x}")
    procs = []
    for r in range(nprocs):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        procs.append(subprocess.Popen([sys.executable, "-u", *argv], env=e,
                                      stdout=None if r == 0 else sys.stderr))
    rc = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                code = p.poll()
                if code is None:
                    continue
                live.remove(p)
                if code != 0 and rc == 0:
                    rc = code if code > 0 else 128 - code
                    r = procs.index(p)
                    why = _failure_text(base["MSD_RDZV_KEY"], r)
                    print(f"meteorgpu.launch: rank {r} of {nprocs} exited with code {code}"
                          + (f": {why}" if why else ""), file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        # every rendezvous file of this launch (the RCCL id and any other tag, or a rank's
        # half-written temporary): a failed job leaves none behind
        prefix = f"msd_rdzv_{base['MSD_RDZV_KEY']}_"
        for name in os.listdir(_rdzv_dir()):
            if name.startswith(prefix):
                try:
                    os.unlink(os.path.join(_rdzv_dir(), name))
                except FileNotFoundError:
                    pass
    return rc


class Group:
    """The job's RCCL communicator on this rank's context: barrier, rank count, max / sum over
    ranks, and the allgather the C5 stream protocol uses (``self.comm``, a stream.RcclComm)."""

    def __init__(self, ctx, rank: int, world: int):
        from . import _lib
        from .batch import Communicator
        from .stream import RcclComm
        self.ctx, self.rank, self.world = ctx, int(rank), int(world)
        uid = share_bytes(self.rank, Communicator.unique_id)
        self.rccl = open_comm(lambda: Communicator(ctx, self.world, uid, self.rank), self.rank)
        self.comm = RcclComm(self.rccl, self.rank, self.world)
        self._one = ctx.alloc(8)
        self._lib = _lib
        self.barrier()
        release(self.rank)

    def sum_i64(self, values) -> np.ndarray:
        a = np.ascontiguousarray(values, dtype=np.int64).reshape(-1)
        buf = self.ctx.alloc(max(8, a.nbytes))
        try:
            buf.upload(a)
            self.rccl.allreduce_i64(buf, a.size)
            out = np.empty_like(a)
            buf.download(out)  # download synchronises the context's stream
            return out
        finally:
            buf.free()

    def barrier(self) -> None:
        """All ranks have enqueued everything before this call and it has finished on each
        rank's stream: an all-reduce on the context stream, then a stream synchronise."""
        self.ctx.synchronize()
        self._one.upload(np.ones(1, np.int64))
        self.rccl.allreduce_i64(self._one, 1)
        self.ctx.synchronize()

    def ranks_seen(self) -> int:
        """How many ranks the communicator reduced over (an all-reduce of ones)."""
        return int(self.sum_i64(np.ones(1, np.int64))[0])

    def max_f64(self, v: float) -> float:
        got = self.comm.allgather_fixed(np.array([float(v)], np.float64))
        return float(max(g[0] for g in got))

    def close(self) -> None:
        if getattr(self, "rccl", None) is not None:
            self.ctx.synchronize()
            self.rccl.close()
            self.rccl = None

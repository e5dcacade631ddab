"""Test doubles for the C5 stream-detector protocol (meteorgpu/stream.py) — TEST INFRASTRUCTURE.

``NumpyStreamOps`` is a CPU stand-in for one rank's ``_lib.StreamPlan``: the same methods,
restated sequentially in numpy from dsp/src/main.py:450-522 (adaptive) / :396-448 (global), so
that the protocol's host logic (halos, chunk sums, the shard-edge state rounds, the run merge)
can be checked on the CPU at world size > 1 against the single-process oracle.
``ThreadComm`` is an in-process allgather for N ranks run as threads (CPU or GPU tests).
"""
from __future__ import annotations

import threading

import numpy as np

CHUNK = 8192


class NumpyStreamOps:
    def __init__(self, delta_local, n_total, frame0, adaptive, k, W, Fa, F0, head_frames=CHUNK):
        self.d = np.asarray(delta_local, np.float64)
        self.n_total, self.frame0, self.n_local = int(n_total), int(frame0), self.d.size
        self.adaptive, self.k, self.W, self.Fa, self.F0 = adaptive, float(k), int(W), int(Fa), int(F0)
        if not adaptive:
            self.W, self.F0 = 0, self.n_total
        self.n_tail = min(self.W, self.frame0)
        self.n_head = min(head_frames, self.n_total - self.frame0 - self.n_local)
        self.tail = self.head = None
        self.fr = np.full(self.n_local, np.nan)
        self.thr = np.full(self.n_local, np.nan)

    def _x(self):
        return np.concatenate([self.tail, self.d, self.head])

    def delta(self, lo=0, hi=None):
        return self.d[lo:hi].copy()

    def set_halos(self, tail, head):
        assert tail.shape == (self.n_tail,) and head.shape == (self.n_head,)
        self.tail, self.head = np.asarray(tail, np.float64), np.asarray(head, np.float64)

    def chunk_sums(self, mean=None):
        x, x0 = self._x(), self.frame0 - self.n_tail
        c0 = -(-self.frame0 // CHUNK)
        out = []
        c = c0
        while c * CHUNK < self.frame0 + self.n_local:
            g = c * CHUNK
            seg = x[g - x0: min(g + CHUNK, self.n_total) - x0]
            assert seg.size == min(CHUNK, self.n_total - g), "head halo too short"
            if mean is not None:
                seg = (seg - mean) * (seg - mean)
            out.append(np.add.reduce(seg))  # one pairwise tree (<= 8192 values)
            c += 1
        return c0, np.array(out, np.float64)

    def set_exact_thresholds(self, on):
        pass  # fresh() is exact everywhere

    def fresh(self):
        x, x0 = self._x(), self.frame0 - self.n_tail
        for j in range(self.n_local):
            i = self.frame0 + j
            if i < self.F0:
                continue
            win = x[max(0, i - self.W) - x0: i - x0]
            with np.errstate(all="ignore"):
                import warnings
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore")
                    self.fr[j] = np.mean(win) + self.k * np.std(win)

    def refine(self):
        return 0  # fresh() is exact already

    def scan(self, thr0, entry, reset):
        fz, last, thr, src = entry[:4]
        runs = []
        margin = np.inf
        for j in range(self.n_local):
            i = self.frame0 + j
            if i < self.F0:
                thr, src = thr0, -1
            elif i > fz:
                thr, src = self.fr[j], i
            self.thr[j] = thr
            v = self.d[j]
            margin = min(margin, abs(v - thr)) if not np.isnan(thr) else margin
            if v > thr:
                if i > last + 1:
                    runs.append([i, i])
                elif runs:
                    runs[-1][1] = i
                else:
                    runs.append([-1, i])  # continues the previous shard's run
                last = i
                fz = max(i + self.Fa, max(0, i))
        self._runs, self._margin = runs, margin
        return (fz, last, thr, src, 0.0), 1

    def runs(self):
        out = np.zeros(len(self._runs), [("start", np.int64), ("stop", np.int64), ("db", np.float64)])
        for n, (s, e) in enumerate(self._runs):
            out[n] = (s, e + 1, 0.0)
        return out, self._margin

    def db(self, dets):
        x, x0 = self._x(), self.frame0 - self.n_tail
        out = dets.copy()
        for n in range(len(out)):
            out["db"][n] = np.mean(x[out["start"][n] - x0: out["stop"][n] - x0])
        return out

    def thresholds(self):
        return self.thr.copy()


class ThreadComm:
    """allgather among `world` threads of one process (one instance per rank)."""

    class _Shared:
        def __init__(self, world):
            self.world = world
            self.barrier = threading.Barrier(world)
            self.slots = [None] * world

    def __init__(self, shared, rank):
        self.shared, self.rank, self.world = shared, rank, shared.world

    @classmethod
    def group(cls, world):
        sh = cls._Shared(world)
        return [cls(sh, r) for r in range(world)]

    def allgather_fixed(self, a):
        return self.allgather(a)

    def allgather(self, a):
        sh = self.shared
        sh.slots[self.rank] = np.array(a, copy=True)
        sh.barrier.wait()
        out = [np.array(s, copy=True) for s in sh.slots]
        sh.barrier.wait()
        return out


def run_threads(world, fn):
    """fn(rank, comm) on `world` threads; returns the per-rank results (re-raises failures)."""
    comms = ThreadComm.group(world)
    res, errs = [None] * world, [None] * world

    def body(r):
        try:
            res[r] = fn(r, comms[r])
        except BaseException as e:  # noqa: BLE001
            errs[r] = e
            comms[r].shared.barrier.abort()

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in errs:
        if e is not None and not isinstance(e, threading.BrokenBarrierError):
            raise e
    for e in errs:
        if e is not None:
            raise e
    return res


def shard_bounds(n_total, world, rank, cuts=None):
    if cuts is not None:
        b = [0] + list(cuts) + [n_total]
        return b[rank], b[rank + 1]
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)

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


class NumpyCertOps(NumpyStreamOps):
    """``NumpyStreamOps`` with the certification interface of a certifying ``_lib.StreamPlan``
    (msd_stream_set_certify): the rank's delta is an APPROXIMATION within ``ed`` per frame of the
    float64 one (the fp32 spectrogram's, on the device), and every decision is checked against its
    bounds -- |delta - thr| > ed[i] + terr(source) certifies it (NaN never does).  terr: a fresh
    threshold's window moves it by at most mean(ed) + |k| rms(ed) over the window (mean: 1-Lipschitz
    in the max norm, population std: in the rms norm); thr0 by stream.terr0_from over the whole
    stream's sums; a held threshold keeps its source's (stream.hip terr_kernel / scan_kernel,
    main.py:464-466, :475-480, :485)."""

    certify = True
    TERR_ROUND = 1e-12  # float64 rounding of the statistics, far below any ed used here

    def __init__(self, delta_local, ed_local, n_total, frame0, adaptive, k, W, Fa, F0, head_frames=CHUNK):
        super().__init__(delta_local, n_total, frame0, adaptive, k, W, Fa, F0, head_frames)
        self.e = np.asarray(ed_local, np.float64).copy()
        self.etail = self.ehead = None
        self.terr = np.full(self.n_local, np.nan)
        self.terr0 = 0.0
        self._unc, self._mslack, self._mzone = [], np.inf, 0.0

    def ed(self, lo=0, hi=None):
        return self.e[lo:hi].copy()

    def set_ed_halos(self, tail, head):
        assert tail.shape == (self.n_tail,) and head.shape == (self.n_head,)
        self.etail, self.ehead = np.asarray(tail, np.float64), np.asarray(head, np.float64)

    def ed_sums(self):
        return float(np.sum(self.e)), float(np.sum(self.e * self.e))

    def set_terr0(self, s1, s2):
        from meteorgpu.stream import terr0_from
        self.terr0 = terr0_from(s1, s2, self.n_total, self.k)

    def fresh(self):
        super().fresh()
        ex, x0 = np.concatenate([self.etail, self.e, self.ehead]), self.frame0 - self.n_tail
        for j in range(self.n_local):
            i = self.frame0 + j
            if i < self.F0:
                continue
            w = ex[max(0, i - self.W) - x0: i - x0]
            self.terr[j] = (np.mean(w) + abs(self.k) * np.sqrt(np.mean(w * w))) * (1 + 1e-9) + self.TERR_ROUND \
                if w.size else np.inf

    def scan(self, thr0, entry, reset):
        fz, last, thr, src, err = entry
        runs = []
        margin = np.inf
        unc, mslack, mzone = [], np.inf, 0.0
        for j in range(self.n_local):
            i = self.frame0 + j
            if i < self.F0:
                thr, src, err = thr0, -1, self.terr0
            elif i > fz:
                thr, src, err = self.fr[j], i, self.terr[j]
            self.thr[j] = thr
            v = self.d[j]
            margin = min(margin, abs(v - thr)) if not np.isnan(thr) else margin
            zone = self.e[j] + err
            slack = abs(v - thr) - zone
            mzone = max(mzone, zone) if np.isfinite(zone) else mzone
            if not slack > 0:  # NaN (a NaN threshold or bound) is uncertain too
                unc.append((i, src))
            elif slack < mslack:
                mslack = slack
            if v > thr:
                if i > last + 1:
                    runs.append([i, i])
                elif runs:
                    runs[-1][1] = i
                else:
                    runs.append([-1, i])
                last = i
                fz = max(i + self.Fa, max(0, i))
        self._runs, self._margin = runs, margin
        self._unc, self._mslack, self._mzone = unc, mslack, mzone
        return (fz, last, thr, src, err), 1

    def certificate(self):
        lst = np.array(self._unc, np.int64).reshape(-1, 2)
        return len(self._unc), self._mslack, self._mzone, lst


def make_cert_shard(exact, approx, ed, rank, world, adaptive, k, W, Fa, F0, cuts=None):
    """one rank's numpy certifying shard: the CertifyingShard loop of meteorgpu.stream over
    NumpyCertOps, whose _refine_local puts the float64 values (``exact``) and a float64-grade bound
    into the rank's own frames of the global ranges -- as IQShardDetector._refine_local recomputes
    them from the samples with msd_iq_delta64_dev"""
    from meteorgpu import stream

    n = exact.size
    lo, hi = shard_bounds(n, world, rank, cuts)

    class Shard(stream.CertifyingShard):
        certify = True

        def __init__(self):
            self.T, self.W, self.f0, self.f1 = n, (W if adaptive else 0), lo, hi
            self.adaptive, self.k, self.F0 = adaptive, k, (F0 if adaptive else 0)
            self.ops = NumpyCertOps(approx[lo:hi], ed[lo:hi], n, lo, adaptive, k, W, Fa, F0)
            self._refined = stream._NO_IV
            self.refined_local = 0  # frames this rank recomputed

        def _refine_local(self, ranges):
            for a, b in stream._as_iv(ranges):
                a, b = max(int(a), self.f0), min(int(b), self.f1)
                if b > a:
                    self.ops.d[a - self.f0: b - self.f0] = exact[a:b]
                    self.ops.e[a - self.f0: b - self.f0] = 1e-13
                    self.refined_local += b - a

    return Shard()


def cert_stream(n, seed, ed_scale=2e-3, plants=(), W=600, Fa=100, F0=50, k=4.0, rate=0.01):
    """(exact, approx, ed): a detector stream (test_stream_protocol.make_delta's shape: noise + bursts),
    its approximation within a per-frame bound ed, and near ties planted at the frames in ``plants``:
    each such frame's exact delta is moved to within 0.3 ed of the threshold the exact detector uses
    there (oracle), so the approximate delta (0.9 ed away, random sign) may decide it either way"""
    import sys, os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import dsp_oracle as O
    rng = np.random.default_rng(seed)
    d = rng.normal(0.0, 1.0, n)
    t = 0
    while True:
        t += int(rng.exponential(1 / rate))
        if t >= n:
            break
        L = int(rng.integers(1, 40))
        d[t: t + L] += rng.uniform(3.0, 9.0)
    ed = ed_scale * rng.uniform(0.5, 1.5, n)
    for i in sorted(plants):
        _, thr = O.get_detections_adaptive_ref(d, k, 1.0, W, 0, Fa, F0)
        if np.isfinite(thr[i]):
            d[i] = thr[i] + rng.choice([-0.3, 0.3]) * ed[i]
    approx = d + rng.choice([-0.9, 0.9], n) * ed
    return d, approx, ed

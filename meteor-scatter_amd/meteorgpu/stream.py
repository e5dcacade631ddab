"""The reference's detector over ONE long stream time-sharded over ranks (BASELINE config C5:
24 h of 192 kHz I/Q whose STFT frames are the detector's blocks, 8 GPUs).

get_detections_adaptive() (dsp/src/main.py:450-522) is a serial loop over the blocks of one
recording: its global threshold uses the mean/std of the WHOLE recording (:464-466), every
adaptive threshold looks back W blocks (:475-480), and the freeze / run state flows from one
block to the next (:485-493).  Sharding the frames over ranks therefore needs exactly three
exchanges, all small, done here on the host over a communicator's allgather:

1. halos: each rank sends its last W and first ``head_frames`` delta values; a rank keeps
   the W frames before its shard (the look-back) and the frames after it (chunk tails, runs
   that cross the edge);
2. the global threshold: numpy's add.reduce over n values is ``s = 0.0; s += pairwise(chunk)``
   over 8192-value chunks in order (np_reduce.h), so the ranks' chunk sums (the chunks that
   start in each shard), gathered in rank order and added in order, give numpy's sum bit for
   bit -- once for the mean, once for the squared deviations (np.std);
3. the state at the shard edges: every rank scans its shard from the clean state, then rank
   r re-scans from rank r-1's exit state until no entry state changes (at most world + 1
   rounds, normally 2).

The adaptive thresholds are only read where the detector is not frozen, so the first scan runs
on cheap predicted thresholds, marks what it read, the device computes those numpy-exactly
(``refine``), and the scan repeats until a scan read nothing that was not exact (normally 2).
Without the thresholds output (``run(thresholds=False)``) only decisions need exact values: the
predictor carries a rounding-error bound, and only frames whose delta lies within the bound of
their predicted threshold, or that trigger a detection (whose threshold is then held), are made
exact -- a few thousand frames a day instead of every unfrozen frame.

The device work per rank is ``_lib.StreamPlan`` (libmsdsp, stream.hip); ``ops`` may be any
object with the same methods (the CPU tests drive this protocol with a numpy stand-in over
gloo).  Results are identical on every rank: the merged detections of the whole stream.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from . import _lib

CHUNK = 8192  # numpy's reduction buffer


# ---------------------------------------------------------------- communicators
class LocalComm:
    """world size 1"""
    rank, world = 0, 1

    def allgather(self, a: np.ndarray) -> list[np.ndarray]:
        return [np.array(a, copy=True)]

    allgather_fixed = allgather  # every rank sends the same number of elements


class RcclComm:
    """RCCL over the GPUs of one job (msd_comm_allgather on device buffers)."""

    def __init__(self, comm, rank: int, world: int):
        self.comm, self.rank, self.world = comm, int(rank), int(world)
        self.ctx = comm.ctx
        self._cap, self._send, self._recv = 0, None, None  # grow-only device staging buffers

    def _gather_bytes(self, b: np.ndarray) -> np.ndarray:
        b = np.ascontiguousarray(b).view(np.uint8)
        n = b.size
        if n > self._cap or self._send is None:
            self._cap = max(n, 4096, 2 * self._cap)
            self._send = self.ctx.alloc(self._cap)
            self._recv = self.ctx.alloc(self._cap * self.world)
        send, recv = self._send, self._recv
        if n:
            send.upload(b)
        _lib.check(self.ctx.lib.msd_comm_allgather(self.comm.h, send.ptr, recv.ptr, n))
        out = np.empty(n * self.world, np.uint8)
        if n:
            recv.download(out)  # rank r's n bytes sit at r * n (ncclAllGather packs them)
        return out

    def allgather(self, a: np.ndarray) -> list[np.ndarray]:
        a = np.ascontiguousarray(a)
        ns = self._gather_bytes(np.array([a.size], np.int64)).view(np.int64)
        m = int(ns.max()) if ns.size else 0
        buf = np.zeros(max(m, 1), a.dtype)
        buf[: a.size] = a
        got = self._gather_bytes(buf).view(a.dtype).reshape(self.world, -1)
        return [got[r, : int(ns[r])].copy() for r in range(self.world)]

    def allgather_fixed(self, a: np.ndarray) -> list[np.ndarray]:
        a = np.ascontiguousarray(a)
        got = self._gather_bytes(a).view(a.dtype).reshape(self.world, -1)
        return [got[r].copy() for r in range(self.world)]


# ---------------------------------------------------------------- detector state
def clean_state(thr0: float, terr0: float = 0.0) -> tuple[int, int, float, int, float]:
    """(freeze_until_idx, last run's stop, threshold) before block 0 (main.py:454-468), plus the
    threshold's source frame (-1: thr0) and its error bound (certification)."""
    return (-1, -2, float(thr0), -1, float(terr0))


def same_state(x, y, a: int, F0: int) -> bool:
    """Do states x and y entering frame a lead to the same future (stream.hip same_state)?"""
    fx, fy = x[0] >= a, y[0] >= a
    if fx != fy:
        return False
    if fx:
        if x[0] != y[0]:
            return False
        if a >= F0 and (np.float64(x[2]).view(np.int64) != np.float64(y[2]).view(np.int64) or x[3] != y[3]):
            return False
    return (x[1] == a - 1) == (y[1] == a - 1)


NSTATE = 5  # int64 words of a packed state


def _pack(s) -> np.ndarray:
    return np.array([s[0], s[1], np.float64(s[2]).view(np.int64), s[3], np.float64(s[4]).view(np.int64)], np.int64)


def _unpack(a: np.ndarray):
    return (int(a[0]), int(a[1]), float(np.int64(a[2]).view(np.float64)), int(a[3]),
            float(np.int64(a[4]).view(np.float64)))


def terr0_from(s1: float, s2: float, n: int, k: float) -> float:
    """thr0's error bound from the whole stream's sum ed and sum ed^2 (stream.hip terr0_from)"""
    if n <= 0:
        return 0.0
    return (s1 / n + abs(k) * math.sqrt(s2 / n)) * (1.0 + 1e-9) + 1e-10


@dataclass
class StreamResult:
    detections: np.ndarray     # DET_DTYPE [start, stop) frame ranges + dB, the whole stream
    thr0: float                # mean + k*std of the whole stream (main.py:464-466 / :399-400)
    thresholds: np.ndarray     # this rank's thresholds actually used (adaptive) / [thr0] (global);
                               # None when run(thresholds=False)
    margin: float              # min |delta - threshold| over the stream
    rounds: int                # state-exchange rounds
    refined: int = 0           # this rank's exact-threshold work units (tiles; frames without the
                               # thresholds output)
    # certification against the float64 reference (plans with certify on; None / 0 otherwise):
    certified: bool | None = None   # every decision's |delta - thr| exceeds its error bounds
    uncertain: int = 0              # decisions the bounds cannot settle (the whole stream)
    min_slack: float = math.inf     # min over decisions of |delta - thr| - (ed + threshold bound)
    decision_bound: float = 0.0     # max over decisions of ed + threshold bound (dB)
    uncertain_frames: np.ndarray | None = None  # [(global frame, threshold source frame or -1)]
    refined_delta_frames: int = 0   # frames whose delta was recomputed in float64 (iq refinement)
    near_tie: bool = False          # uncertain decisions left after refinement (float64 near ties)
    uncertain_initial: int = 0      # uncertain decisions of the first pass (before any refinement)
    detector_passes: int = 1        # detector runs (1 + refinement rounds)
    db_refined_frames: int = 0      # detection frames made float64 for the dB means (exact decisions)
    refine_budget_exhausted: bool = False  # uncertain decisions left after MAX_REFINE refinements


class StreamDetector:
    """Runs the protocol above for one rank.  ``ops`` holds this rank's shard (delta already
    set) — a ``_lib.StreamPlan`` or a stand-in with the same methods."""

    def __init__(self, ops, comm, adaptive: bool, k_std: float, window_blocks: int = 0,
                 fixed_init_blocks: int = 0, head_frames: int = CHUNK):
        self.ops, self.comm = ops, comm
        self.adaptive, self.k = bool(adaptive), float(k_std)
        self.W, self.F0 = int(window_blocks), int(fixed_init_blocks)
        self.H = int(head_frames)

    @property
    def certify(self) -> bool:
        return bool(getattr(self.ops, "certify", False))

    # 1. halos (and, certifying, the same halos of the delta error bounds, in the same message)
    def exchange_halos(self):
        ops, r, n = self.ops, self.comm.rank, self.ops.n_local
        cf = self.certify
        if self.comm.world == 1:  # nothing before or after the only shard
            ops.set_halos(np.zeros(0), np.zeros(0))
            if cf:
                ops.set_ed_halos(np.zeros(0), np.zeros(0))
            return
        lo_t, hi_h = max(0, n - self.W) if self.W > 0 else n, min(self.H, n)
        tail, head = ops.delta(lo_t, n), ops.delta(0, hi_h)
        parts = [[float(tail.size)], tail, head]
        if cf:
            parts += [ops.ed(lo_t, n), ops.ed(0, hi_h)]
        got = self.comm.allgather(np.concatenate(parts))  # one exchange
        nts = [int(g[0]) for g in got]
        nhs = [(g.size - 1) // (2 if cf else 1) - nts[q] for q, g in enumerate(got)]

        def halos(off):  # off 0: delta, 1: ed
            tails = [g[1 + off * (nts[q] + nhs[q]): 1 + off * (nts[q] + nhs[q]) + nts[q]] for q, g in enumerate(got)]
            heads = [g[1 + off * (nts[q] + nhs[q]) + nts[q]: 1 + (off + 1) * (nts[q] + nhs[q])]
                     for q, g in enumerate(got)]
            before = np.concatenate([np.zeros(0)] + tails[:r])
            after = np.concatenate([np.zeros(0)] + heads[r + 1:])
            return (before[before.size - ops.n_tail:] if ops.n_tail else before[:0]), after[: ops.n_head]

        ops.set_halos(*halos(0))
        if cf:
            ops.set_ed_halos(*halos(1))

    # 2. numpy's sum over the whole stream from the ranks' chunk sums
    def _global_sum(self, mean=None) -> float:
        _, sums = self.ops.chunk_sums(mean)
        s = 0.0
        for part in self.comm.allgather(sums):
            for v in part:
                s += float(v)
        return s

    def global_threshold(self) -> float:
        n = self.ops.n_total
        mean = self._global_sum() / n
        std = math.sqrt(self._global_sum(mean) / n)
        return mean + self.k * std

    def global_threshold_error(self) -> float:
        """certifying: thr0's error bound from every rank's sum ed, sum ed^2 (set on the plan too)"""
        s1, s2 = self.ops.ed_sums()
        tot = np.sum(np.stack(self.comm.allgather_fixed(np.array([s1, s2], np.float64))), axis=0)
        self.ops.set_terr0(float(tot[0]), float(tot[1]))
        return terr0_from(float(tot[0]), float(tot[1]), self.ops.n_total, self.k)

    def certificate(self) -> tuple[int, float, float, np.ndarray]:
        """every rank's uncertain decisions after the last scan, merged (identical on every rank)"""
        n, ms, mz, lst = self.ops.certificate()
        msg = np.concatenate([[n, np.float64(ms).view(np.int64), np.float64(mz).view(np.int64)],
                              lst.reshape(-1)]).astype(np.int64)
        got = self.comm.allgather(msg)
        tot = sum(int(g[0]) for g in got)
        mslack = min(float(np.int64(g[1]).view(np.float64)) for g in got)
        mzone = max(float(np.int64(g[2]).view(np.float64)) for g in got)
        frames = np.concatenate([np.zeros((0, 2), np.int64)] + [g[3:].reshape(-1, 2) for g in got])
        return tot, mslack, mzone, frames

    def _certified(self, res: StreamResult) -> StreamResult:
        if not self.certify:
            return res
        tot, mslack, mzone, frames = self.certificate()
        res.certified, res.uncertain, res.min_slack = tot == 0, tot, mslack
        res.decision_bound, res.uncertain_frames, res.near_tie = mzone, frames, tot > 0
        return res

    # 3. the state at the shard edges
    def scan(self, thr0: float, refined: bool = False) -> int:
        """refined: thresholds changed since the last fixed point -- every segment re-scans from its
        converged entry state instead of a clean restart"""
        ops, comm, r = self.ops, self.comm, self.comm.rank
        F0 = self.F0 if self.adaptive else ops.n_total
        entry = self._entry if refined else clean_state(thr0, getattr(self, "terr0", 0.0))
        exit_, _ = ops.scan(thr0, entry, 2 if refined else 1)
        rounds = 1
        while True:
            # one exchange per round: every rank's exit and entry state and first frame, so each
            # rank decides every rank's "entry changed" alike
            got = comm.allgather_fixed(np.concatenate([_pack(exit_), _pack(entry), [ops.frame0]]))
            S = NSTATE
            exits = [_unpack(g[0:S]) for g in got]
            changed = [q > 0 and not same_state(exits[q - 1], _unpack(got[q][S:2 * S]), int(got[q][2 * S]), F0)
                       for q in range(comm.world)]
            if not any(changed):
                self._entry = entry
                return rounds
            rounds += 1
            if changed[r]:
                entry = exits[r - 1]
                exit_, _ = ops.scan(thr0, entry, 0)

    def db_means(self, dets: np.ndarray, refresh_halos: bool = False) -> np.ndarray:
        """np.mean dB of every detection (main.py:422-423, :501-502), computed by the rank whose
        shard holds the run's start (its head halo covers a run into the next shards) and
        allgathered.  refresh_halos: the delta of other ranks' frames changed since the halo
        exchange (float64 refinement): exchange them again first."""
        ops, comm = self.ops, self.comm
        if refresh_halos and comm.world > 1:
            self.exchange_halos()
        lo, hi = ops.frame0, ops.frame0 + ops.n_local
        mine = (dets["start"] >= lo) & (dets["start"] < hi)
        db_local = ops.db(dets[mine])["db"] if mine.any() else np.zeros(0)
        db_all = np.full(len(dets), np.nan)
        for g in comm.allgather(np.concatenate([np.flatnonzero(mine).astype(np.int64),
                                                np.asarray(db_local, np.float64).view(np.int64)])):
            m = g.size // 2  # the owner's detection indices, then their dB bits
            db_all[g[:m]] = g[m:].view(np.float64)
        return db_all

    def run(self, thresholds: bool = True) -> StreamResult:
        ops, comm = self.ops, self.comm
        if ops.n_total == 0:
            if not self.adaptive:  # above_thresh[0] on an empty array (main.py:412)
                raise IndexError("index 0 is out of bounds for axis 0 with size 0")
            return StreamResult(np.zeros(0, _lib.DET_DTYPE), float("nan"), np.zeros(0), math.inf, 0)
        if isinstance(comm, LocalComm) and hasattr(ops, "detect_local"):  # one native call, same results
            # (a one-rank RCCL or gloo group keeps the exchange protocol below)
            dets, thr0, margin, rounds, refined = ops.detect_local(thresholds if self.adaptive else True)
            thr = None if not thresholds else (ops.thresholds() if self.adaptive else np.array([thr0]))
            return self._certified(StreamResult(dets, thr0, thr, margin, rounds, refined))
        self.exchange_halos()
        if self.adaptive:  # state-free, independent of thr0: queued before the chunk-sum round trips
            # without the thresholds output only the decisions need exact thresholds: predicted
            # ones with an error bound elsewhere (same detections)
            ops.set_exact_thresholds(thresholds)
            ops.fresh()
        thr0 = self.global_threshold()
        self.terr0 = self.global_threshold_error() if self.certify else 0.0
        rounds = self.scan(thr0)
        refined = 0
        while self.adaptive:  # until the last scan read exact thresholds only, on every rank
            n = ops.refine()
            refined += n
            if not any(int(f[0]) for f in comm.allgather_fixed(np.array([n], np.int64))):
                break
            rounds += self.scan(thr0, refined=True)
        # runs of every shard, merged in stream order (a run continued across an edge has start -1)
        local, margin = ops.runs()
        got = comm.allgather(np.concatenate([np.array([margin], np.float64).view(np.int64),
                                             np.stack([local["start"], local["stop"]], 1).reshape(-1)]).astype(np.int64))
        margin = min(float(g[:1].view(np.float64)[0]) for g in got)
        parts = [g[1:] for g in got]
        allr = np.concatenate([np.zeros(0, np.int64)] + parts).reshape(-1, 2)
        if allr.size and allr[0, 0] < 0:
            raise RuntimeError("stream detector: the first shard's first run continues a previous shard")
        heads = np.flatnonzero(allr[:, 0] >= 0)  # a run continued over shard edges (start -1) joins its predecessor
        dets = np.zeros(heads.size, _lib.DET_DTYPE)
        if heads.size:
            dets["start"] = allr[heads, 0]
            dets["stop"] = np.maximum.reduceat(allr[:, 1], heads)
        if not self.adaptive and dets.size and dets["stop"][-1] == ops.n_total:
            dets["stop"][-1] = ops.n_total - 1  # burst_stops gets len-1 (main.py:414-415)
            if dets["stop"][-1] - dets["start"][-1] <= 0:
                raise AssertionError("Detection duration must be greater than 0")  # main.py:437
        dets["db"] = self.db_means(dets)
        thr = None if not thresholds else (ops.thresholds() if self.adaptive else np.array([thr0]))
        return self._certified(StreamResult(dets, thr0, thr, margin, rounds, refined))


# ------------------------------------------------------------ certified decisions (any plan / rank)
def _as_iv(iv) -> np.ndarray:
    if isinstance(iv, np.ndarray):
        return iv.astype(np.int64, copy=False).reshape(-1, 2)
    return np.asarray(list(iv), dtype=np.int64).reshape(-1, 2)


_NO_IV = np.zeros((0, 2), np.int64)


def _merge_a(iv) -> np.ndarray:
    """sorted, merged [a, b) intervals (touching ones joined), as an (n, 2) int64 array"""
    a = _as_iv(iv)
    a = a[a[:, 1] > a[:, 0]]
    if a.size == 0:
        return _NO_IV
    a = a[np.argsort(a[:, 0], kind="stable")]
    ends = np.maximum.accumulate(a[:, 1])
    new = np.ones(len(a), bool)
    new[1:] = a[1:, 0] > ends[:-1]  # a start past every earlier end opens a new interval
    heads = np.flatnonzero(new)
    tails = np.r_[heads[1:] - 1, len(a) - 1]
    return np.stack([a[heads, 0], ends[tails]], 1)


def _subtract_a(iv, done) -> np.ndarray:
    """the (merged) intervals iv minus the (merged) intervals done: the elementary segments between
    all their boundaries that iv covers and done does not, merged"""
    a, d = _as_iv(iv), _as_iv(done)
    if a.size == 0:
        return _NO_IV
    if d.size == 0:
        return a
    if len(d) == 1 and d[0, 0] <= a[0, 0] and a[-1, 1] <= d[0, 1]:  # all refined already (the exact delta)
        return _NO_IV
    pts = np.unique(np.concatenate([a.reshape(-1), d.reshape(-1)]))
    lo, hi = pts[:-1], pts[1:]

    def covered(x, seg):  # x inside one of the sorted disjoint [start, end)
        return np.searchsorted(seg[:, 0], x, "right") > np.searchsorted(seg[:, 1], x, "right")

    keep = covered(lo, a) & ~covered(lo, d)
    return _merge_a(np.stack([lo[keep], hi[keep]], 1))


def _merge(iv) -> list:
    """_merge_a as a list of [a, b]"""
    return _merge_a(iv).tolist()


def _subtract(iv, done) -> list:
    """_subtract_a as a list of [a, b]"""
    return _subtract_a(iv, done).tolist()


def _iv_len(iv) -> int:
    a = _as_iv(iv)
    return int((a[:, 1] - a[:, 0]).sum())


class CertifyingShard:
    """The certify-then-refine loop of one rank's shard (meteorgpu.iq.IQShardDetector; the CPU tests'
    numpy shard in tests/stream_np_ops.py): every pass runs the protocol above with certification on
    the plan, the uncertain decisions' dependencies (the frame and the window its threshold reads,
    main.py:475-480; the whole stream for thr0, main.py:464-466) are recomputed in float64 by
    ``_refine_local`` -- each rank its own part of the global ranges -- and the detector reruns until
    every decision is certified; then the detections' frames are made float64 for the dB means.
    Subclasses provide ``_refine_local(ranges)`` and the attributes ``ops`` (the rank's plan or a
    stand-in), ``adaptive``, ``k``, ``W`` (window), ``F0``, ``certify``, ``T`` (frames of the whole
    stream) and ``_refined`` (global frame ranges already float64, merged (n, 2)); ``_detector``
    builds the StreamDetector over ``ops``."""

    MAX_REFINE = 8  # refinement rounds before giving up (refine_budget_exhausted)

    def detect(self, comm=None, thresholds: bool = True, exact_decisions: bool = True) -> StreamResult:
        """The detector over the whole stream (every rank gets the same result).  Certifying, each
        decision is checked against its error bounds; exact_decisions refines the uncertain ones,
        then the detections' own frames (class docstring)."""
        comm = comm or LocalComm()
        refined, first, passes, exhausted, db_frames = 0, None, 0, False, 0
        while True:
            res = self._detector(comm).run(thresholds)
            passes += 1
            if first is None:
                first = res.uncertain
            if not self.certify or not exact_decisions:
                break
            if res.certified:
                # the detections' own frames in float64 (the CSV's dB column); with the thresholds
                # output one more pass, so that the thresholds, the delta and the dB means agree
                n = self._refine_detections(res)
                db_frames += n
                if n and thresholds and passes <= self.MAX_REFINE:
                    continue
                if n:
                    res.detections["db"] = self._detector(comm).db_means(res.detections, refresh_halos=True)
                break
            if passes > self.MAX_REFINE:  # refined MAX_REFINE times, still uncertain: reported, not a tie
                exhausted = True
                break
            need = self._dependencies(res.uncertain_frames)
            if not len(need):  # every uncertain decision already reads float64 values: a float64 near tie
                break
            self._refined = _merge_a(np.concatenate([self._refined, need]))
            refined += _iv_len(need)
        if self.certify:
            if exact_decisions and not res.certified:  # a near tie / exhausted budget: the dB still float64
                n = self._refine_detections(res)
                if n:
                    db_frames += n
                    res.detections["db"] = self._detector(comm).db_means(res.detections, refresh_halos=True)
            res.refined_delta_frames = refined + db_frames
            res.db_refined_frames = db_frames
            res.near_tie = not res.certified and not exhausted
            res.refine_budget_exhausted = exhausted
            res.uncertain_initial = first
            res.detector_passes = passes
        return res

    def _detector(self, comm) -> StreamDetector:
        return StreamDetector(self.ops, comm, self.adaptive, self.k, self.W, self.F0)

    def _refine_detections(self, res) -> int:
        """float64 delta for every frame of every detection not refined yet (main.py:501-502 takes
        np.mean(delta_power[start:stop]) over them); returns the frames refined.  Every rank holds
        the same detections and refined ranges and refines its own part."""
        dets = res.detections
        if dets is None or len(dets) == 0:
            return 0
        r = self._refined
        if len(r) == 1 and r[0, 0] <= dets["start"].min() and dets["stop"].max() <= r[0, 1]:
            return 0  # every frame float64 already (the exact delta): no interval work per step
        need = _subtract_a(_merge_a(np.stack([dets["start"], dets["stop"]], 1)), r)
        if not len(need):
            return 0
        self._refine_local(need)
        self._refined = _merge_a(np.concatenate([self._refined, need]))
        return _iv_len(need)

    def _dependencies(self, uncertain) -> np.ndarray:
        """global frame ranges the uncertain decisions (frame, threshold source) depend on, and
        refines this rank's part of them"""
        iv = []
        for f, src in np.asarray(uncertain, np.int64).reshape(-1, 2):
            if src < 0:  # thr0: the whole stream's mean and std
                iv.append((0, self.T))
            else:
                iv.append((max(0, int(src) - self.W), int(src)))  # the window delta[src - W : src]
            iv.append((int(f), int(f) + 1))
        need = _subtract_a(_merge_a(iv), self._refined)
        self._refine_local(need)
        return need

    def _refine_local(self, ranges):
        raise NotImplementedError


class DeviceStreamOps:
    """``_lib.StreamPlan`` with the protocol's method signatures."""

    def __init__(self, plan: _lib.StreamPlan):
        self.plan = plan
        self.n_total, self.frame0, self.n_local = plan.n_total, plan.frame0, plan.n_local
        self.n_tail, self.n_head = plan.n_tail, plan.n_head
        self.last_rounds = 0

    @property
    def certify(self) -> bool:
        return self.plan.certify

    def ed(self, lo=0, hi=None):
        return self.plan.ed(lo, hi)

    def set_ed_halos(self, tail, head):
        self.plan.set_ed_halos(tail, head)

    def ed_sums(self):
        return self.plan.ed_sums()

    def set_terr0(self, s1, s2):
        self.plan.set_terr0(s1, s2)

    def certificate(self):
        return self.plan.certificate()

    def delta(self, lo=0, hi=None):
        return self.plan.delta(lo, hi)

    def set_halos(self, tail, head):
        self.plan.set_halos(tail, head)

    def chunk_sums(self, mean=None):
        return self.plan.chunk_sums(mean)

    def set_exact_thresholds(self, on):
        self.plan.set_exact_thresholds(on)

    def detect_local(self, exact_thresholds=True):
        try:
            return self.plan.detect_local(exact_thresholds)
        except _lib.MsdError as e:  # the reference's exceptions, as the Python protocol raises them
            if e.code == _lib.MSD_ERR_INDEX:
                raise IndexError("index 0 is out of bounds for axis 0 with size 0") from None
            if e.code == _lib.MSD_ERR_ASSERT:
                raise AssertionError("Detection duration must be greater than 0") from None
            raise

    def fresh(self):
        self.plan.fresh()

    def refine(self):
        return self.plan.refine()

    def scan(self, thr0, entry, reset):
        ex, rounds = self.plan.scan(thr0, _lib.MsdStreamState(*entry), reset)
        self.last_rounds += rounds
        return (ex.freeze_until, ex.last_stop, ex.thr, ex.src, ex.thr_err), rounds

    def runs(self):
        return self.plan.runs()

    def db(self, dets):
        return self.plan.db(dets)

    def thresholds(self):
        return self.plan.thresholds()


def detect_stream(ctx: _lib.Context, delta_local: np.ndarray, n_total: int, frame0: int, comm=None,
                  adaptive: bool = True, k_std: float = 4.0, window_blocks: int = 0, freeze_after_blocks: int = 0,
                  freeze_before_blocks: int = 0, fixed_init_blocks: int = 0, seg_len: int = 8192,
                  cap_per_seg: int = 256, head_frames: int = CHUNK) -> StreamResult:
    """Host-buffer convenience: this rank's delta shard [frame0, frame0 + len) of an n_total-frame
    stream → the detections of the whole stream (identical on every rank)."""
    comm = comm or LocalComm()
    d = np.ascontiguousarray(delta_local, dtype=np.float64)
    cfg = _lib.det_cfg(adaptive, k_std, window_blocks, freeze_before_blocks, freeze_after_blocks, fixed_init_blocks)
    plan = _lib.StreamPlan(ctx, cfg, n_total, frame0, d.size, seg_len, cap_per_seg, head_frames)
    try:
        plan.set_delta(d)
        return StreamDetector(DeviceStreamOps(plan), comm, adaptive, k_std, window_blocks, fixed_init_blocks,
                              head_frames).run()
    finally:
        plan.close()

"""CPU: the host protocol of the C5 stream detector (meteorgpu/stream.py) — halos, the whole-stream
threshold from per-shard chunk sums, the shard-edge state rounds and the run merge — run at
world sizes 1-4 (threads) and 2 (gloo processes) with the numpy stand-in for the device plan
(tests/stream_np_ops.py), against the single-process oracle of dsp/src/main.py:396-522 over the
whole stream.  Bit-exact: run bounds, dB means, thresholds and the global threshold."""
import os
import socket
import sys

import numpy as np
import pytest

from stream_np_ops import NumpyStreamOps, run_threads, shard_bounds

from meteorgpu import stream
from oracle import dsp_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def make_delta(n, seed, rate=0.004, amp=(3.0, 9.0)):
    """noise + bursts (a few frames up to ~40) — per-frame band delta in dB"""
    rng = np.random.default_rng(seed)
    d = rng.normal(0.0, 1.0, n)
    t = 0
    while True:
        t += int(rng.exponential(1 / rate))
        if t >= n:
            break
        L = int(rng.integers(1, 40))
        d[t: t + L] += rng.uniform(*amp)
    return d


def oracle(d, adaptive, k, W, Fa, F0):
    if adaptive:
        dets, thr = O.get_detections_adaptive_ref(d, k, 1.0, W, 0, Fa, F0)
    else:
        dets, thr = O.get_detections_ref(d, k, 1.0)
    return [(int(a), int(b), db) for a, b, _, db, _, _ in dets], thr


def run_protocol(d, world, adaptive, k, W, Fa, F0, cuts=None):
    n = d.size

    def body(r, comm):
        lo, hi = shard_bounds(n, world, r, cuts)
        ops = NumpyStreamOps(d[lo:hi], n, lo, adaptive, k, W, Fa, F0)
        return stream.StreamDetector(ops, comm, adaptive, k, W, F0).run()

    return run_threads(world, body)


def check(res, d, adaptive, k, W, Fa, F0):
    want, thr = oracle(d, adaptive, k, W, Fa, F0)
    for r in res:  # every rank returns the whole stream's detections
        got = [(int(a), int(b), float(db)) for a, b, db in r.detections]
        assert [(a, b) for a, b, _ in got] == [(a, b) for a, b, _ in want]
        assert np.array_equal(np.array([g[2] for g in got]), np.array([w[2] for w in want]))
    if adaptive:
        allthr = np.concatenate([r.thresholds for r in res])
        assert np.array_equal(allthr, np.asarray(thr, np.float64), equal_nan=True)
    else:
        assert res[0].thr0 == thr
    return want


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_adaptive_shards(world):
    d = make_delta(30000, 11)
    want = check(run_protocol(d, world, True, 4.0, 600, 100, 50), d, True, 4.0, 600, 100, 50)
    assert len(want) > 20


def test_runs_and_freezes_across_edges():
    d = make_delta(30000, 12, rate=0.02)
    want, _ = oracle(d, True, 3.0, 600, 100, 50)
    # cut inside detections (continued runs) and inside freezes, plus an empty shard
    a = want[5][0] + 1
    b = want[12][0] + 30
    cuts = [a, a, b, b + 1]
    check(run_protocol(d, 5, True, 3.0, 600, 100, 50, cuts), d, True, 3.0, 600, 100, 50)


def test_long_window_two_chunks():
    # W > 8192: every window is two numpy reduction chunks; shards shorter than W
    d = make_delta(26000, 13)
    check(run_protocol(d, 3, True, 4.0, 9000, 300, 100, cuts=[5000, 9000]), d, True, 4.0, 9000, 300, 100)


def test_global_mode_and_end_quirk():
    d = make_delta(20000, 14)
    check(run_protocol(d, 3, False, 4.0, 0, 0, 0), d, False, 4.0, 0, 0, 0)
    e = d.copy()
    e[-5:] = 50.0  # a run reaching the end: stop = len-1 (main.py:414-415)
    check(run_protocol(e, 2, False, 4.0, 0, 0, 0), e, False, 4.0, 0, 0, 0)
    f = d.copy()
    f[-2] = -50.0
    f[-1] = 50.0  # one block at the end: t_dur == 0 → assert (main.py:437)
    with pytest.raises(AssertionError):
        run_protocol(f, 2, False, 4.0, 0, 0, 0)


def test_state_helpers():
    assert stream.same_state((-1, -2, 1.0, 3, 0.0), (5, -2, 2.0, 4, 0.0), 10, 0)       # both unfrozen
    assert not stream.same_state((12, -2, 1.0, 3, 0.0), (12, -2, 2.0, 3, 0.0), 10, 0)  # frozen, thresholds differ
    assert not stream.same_state((12, -2, 1.0, 3, 0.0), (12, -2, 1.0, 4, 0.0), 10, 0)  # same value, other window
    assert stream.same_state((12, -2, 1.0, 3, 0.0), (12, -2, 2.0, -1, 0.0), 10, 50)    # before F0 thr0 rules
    assert not stream.same_state((-1, 9, 1.0, 3, 0.0), (-1, -2, 1.0, 3, 0.0), 10, 0)   # adjacency of the last run
    s = (123, -2, float("nan"), 77, 1.5e-3)
    u = stream._unpack(stream._pack(s))
    assert u[:2] == s[:2] and u[3:] == s[3:]
    assert stream.clean_state(2.5, 1e-3) == (-1, -2, 2.5, -1, 1e-3)


def _gloo_rank(rank, world, port, out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from stream_np_ops import NumpyStreamOps as Ops
    from torch_comm import TorchComm
    from meteorgpu import stream as S
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        d = make_delta(25000, 15, rate=0.01)
        lo, hi = shard_bounds(d.size, world, rank)
        res = S.StreamDetector(Ops(d[lo:hi], d.size, lo, True, 4.0, 600, 100, 50), TorchComm(), True, 4.0,
                               600, 50).run()
        np.save(os.path.join(out, f"r{rank}.npy"), np.stack([res.detections["start"], res.detections["stop"]]))
        np.save(os.path.join(out, f"db{rank}.npy"), res.detections["db"])
        np.save(os.path.join(out, f"t{rank}.npy"), res.thresholds)
    finally:
        dist.destroy_process_group()


def test_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_gloo_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    d = make_delta(25000, 15, rate=0.01)
    want, thr = oracle(d, True, 4.0, 600, 100, 50)
    for r in range(2):
        se = np.load(tmp_path / f"r{r}.npy")
        assert [(int(a), int(b)) for a, b in se.T] == [(a, b) for a, b, _ in want]
        assert np.array_equal(np.load(tmp_path / f"db{r}.npy"), np.array([w[2] for w in want]))
    t = np.concatenate([np.load(tmp_path / f"t{r}.npy") for r in range(2)])
    assert np.array_equal(t, np.asarray(thr), equal_nan=True)


@pytest.mark.parametrize("seed", range(12))
def test_random_configs_and_cuts(seed):
    """seeded random detector settings and shard cuts (including empty shards and cuts inside
    runs): the protocol equals the one-process oracle"""
    rng = np.random.default_rng(9000 + seed)
    n = int(rng.integers(300, 4000))
    d = make_delta(n, 100 + seed, rate=float(rng.uniform(0.002, 0.05)))
    adaptive = bool(rng.integers(0, 4) > 0)
    k = float(rng.choice([1.5, 2.5, 4.0]))
    W, Fa, F0 = int(rng.integers(0, 400)), int(rng.integers(0, 300)), int(rng.integers(0, 200))
    world = int(rng.integers(1, 5))
    cuts = sorted(int(c) for c in rng.integers(0, n + 1, world - 1))
    try:
        want = oracle(d, adaptive, k, W, Fa, F0)
    except AssertionError:
        with pytest.raises(AssertionError):
            run_protocol(d, world, adaptive, k, W, Fa, F0, cuts)
        return
    res = run_protocol(d, world, adaptive, k, W, Fa, F0, cuts)
    check(res, d, adaptive, k, W, Fa, F0)
    assert want is not None


# ----------------------------------------------------------------------------------------------
# The certified C5 protocol (meteorgpu.stream.CertifyingShard, the loop IQShardDetector.detect runs)
# across ranks: an approximate delta within a per-frame bound, near ties planted at and beside shard
# edges so that uncertain decisions' threshold windows cross into other ranks' shards; each rank
# refines its own part of the merged dependencies, the halos (delta and bound) are exchanged again,
# and every rank ends certified with the float64 oracle's detections and dB means.
CERT_N, CERT_W, CERT_FA, CERT_F0, CERT_K = 12000, 600, 100, 50, 4.0


def _cert_plants(n, world):
    edges = [n * r // world for r in range(1, world)]
    return sorted({p for e in edges for p in (e - 7, e, e + 3, e + 250)} | {n // 2 + 11, n - 20})


def _cert_case(world, seed):
    from stream_np_ops import cert_stream
    return cert_stream(CERT_N, seed, plants=_cert_plants(CERT_N, world), W=CERT_W, Fa=CERT_FA, F0=CERT_F0,
                       k=CERT_K)


def _cert_body(exact, approx, ed, world, exact_decisions=True):
    from stream_np_ops import make_cert_shard

    def body(r, comm):
        sh = make_cert_shard(exact, approx, ed, r, world, True, CERT_K, CERT_W, CERT_FA, CERT_F0)
        res = sh.detect(comm, thresholds=False, exact_decisions=exact_decisions)
        return res, sh.refined_local
    return body


def _check_cert(results, exact):
    want, _ = oracle(exact, True, CERT_K, CERT_W, CERT_FA, CERT_F0)
    assert len(want) > 20
    for res, _ in results:
        assert res.certified and not res.near_tie and not res.refine_budget_exhausted
        assert res.uncertain_initial > 0 and res.detector_passes >= 2  # the planted ties were caught
        got = [(int(a), int(b)) for a, b, _ in res.detections]
        assert got == [(a, b) for a, b, _ in want]
        np.testing.assert_allclose(res.detections["db"], [w[2] for w in want], rtol=0, atol=1e-9)
    # every rank refined its own part of the merged ranges, and the same total
    assert len({int(res.refined_delta_frames) for res, _ in results}) == 1
    assert sum(n for _, n in results) == int(results[0][0].refined_delta_frames)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_certified_protocol_threads(world):
    exact, approx, ed = _cert_case(world, 40 + world)
    res = run_threads(world, _cert_body(exact, approx, ed, world))
    _check_cert(res, exact)
    if world > 1:  # the windows of the ties beside the edges reach into the previous shard
        assert all(n > 0 for _, n in res)


def test_certified_flag_only_reports_the_ties():
    """certification without refinement: the planted ties are listed, nothing is claimed certified"""
    exact, approx, ed = _cert_case(2, 42)
    res = run_threads(2, _cert_body(exact, approx, ed, 2, exact_decisions=False))
    for r, n in res:
        assert not r.certified and r.uncertain > 0 and n == 0
        frames = set(int(f) for f in r.uncertain_frames[:, 0])
        assert frames & set(_cert_plants(CERT_N, 2))
    assert np.array_equal(res[0][0].uncertain_frames, res[1][0].uncertain_frames)  # merged on every rank


def _gloo_cert_rank(rank, world, port, out):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from torch_comm import TorchComm
    import test_stream_protocol as T
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        exact, approx, ed = T._cert_case(world, 60 + world)
        res, n = T._cert_body(exact, approx, ed, world)(rank, TorchComm())
        np.savez(os.path.join(out, f"c{rank}.npz"), start=res.detections["start"], stop=res.detections["stop"],
                 db=res.detections["db"], info=np.array([res.certified, res.uncertain_initial, res.detector_passes,
                                                         res.refined_delta_frames, n, res.near_tie], np.int64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_certified_protocol_gloo(world, tmp_path):
    """the same across real processes (gloo allgathers): the certificate merge, the refinement of
    windows that cross shard edges by their owners, and the halo refresh before the dB means"""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_gloo_cert_rank, args=(world, port, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    exact, approx, _ = _cert_case(world, 60 + world)
    want, _ = oracle(exact, True, CERT_K, CERT_W, CERT_FA, CERT_F0)
    # the uncertified approximate delta would give other detections: the refinement is what fixes them
    assert [w[:2] for w in oracle(approx, True, CERT_K, CERT_W, CERT_FA, CERT_F0)[0]] != [w[:2] for w in want]
    tot = []
    for r in range(world):
        z = np.load(tmp_path / f"c{r}.npz")
        cert, unc0, passes, refined, n, tie = (int(v) for v in z["info"])
        assert cert == 1 and tie == 0 and unc0 > 0 and passes >= 2 and n > 0
        assert [(int(a), int(b)) for a, b in zip(z["start"], z["stop"])] == [(a, b) for a, b, _ in want]
        np.testing.assert_allclose(z["db"], [w[2] for w in want], rtol=0, atol=1e-9)
        tot.append((refined, n))
    assert len({t[0] for t in tot}) == 1 and sum(t[1] for t in tot) == tot[0][0]

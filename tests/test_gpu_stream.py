"""GPU: the C5 stream detector (stream.hip through the C-ABI, meteorgpu.stream / meteorgpu.iq)
against the oracle of dsp/src/main.py:396-522 over the whole stream.

Bars: run bounds, dB means, every threshold and the global threshold bit-exact on identical delta
(float64, numpy's pairwise order); the I/Q band delta within DELTA_TOL dB of the float64 scipy
spectrogram (the spectrogram is float32 on the device: <= 1e-5 relative per bin); end to end on
I/Q (proc_iq_samples: every decision certified against the float64 reference, tests/
test_gpu_certify.py) the same detections as the oracle, and the CSV's dB column within DB_TOL of
the oracle's (the detections' frames are recomputed in float64 before the means), the t / UTC
columns string-equal."""
import numpy as np
import pytest

from detector_kats import ADAPTIVE, GLOBAL
from stream_np_ops import run_threads, shard_bounds
from test_stream_protocol import make_delta, oracle

pytestmark = pytest.mark.gpu

DELTA_TOL = 1e-4  # dB, the fp32 spectrogram path's delta against scipy's float64 one
DB_TOL = 1e-9     # dB, the CSV's dB column (float64 detection frames) against the oracle's


def _ctx():
    from meteorgpu.dsp import context
    return context(0)


def _detect(d, adaptive, k, W, Fa, F0, seg_len=8192, cap=256):
    from meteorgpu import stream
    return stream.detect_stream(_ctx(), d, d.size, 0, adaptive=adaptive, k_std=k, window_blocks=W,
                                freeze_after_blocks=Fa, fixed_init_blocks=F0, seg_len=seg_len, cap_per_seg=cap)


def _check(res, d, adaptive, k, W, Fa, F0):
    want, thr = oracle(d, adaptive, k, W, Fa, F0)
    got = [(int(a), int(b)) for a, b, _ in res.detections]
    assert got == [(a, b) for a, b, _ in want]
    assert np.array_equal(res.detections["db"], np.array([w[2] for w in want], np.float64))
    if adaptive:
        assert np.array_equal(res.thresholds, np.asarray(thr, np.float64), equal_nan=True)
    else:
        assert res.thr0 == thr
    return want


def test_global_threshold_bit_exact():
    for n, seed in [(100, 1), (8192, 2), (8193, 3), (50000, 4)]:
        d = make_delta(n, seed)
        res = _detect(d, True, 4.0, 50, 10, 5)
        assert res.thr0 == np.mean(d) + 4.0 * np.std(d)


@pytest.mark.parametrize("seg_len", [64, 512, 8192])
def test_adaptive_segments(seg_len):
    d = make_delta(30000, 21, rate=0.01)
    want = _check(_detect(d, True, 4.0, 600, 100, 50, seg_len=seg_len), d, True, 4.0, 600, 100, 50)
    assert len(want) > 50


def test_adaptive_dense_freezes():
    # freeze longer than segments, detections every few hundred frames: chains across many segments
    d = make_delta(40000, 22, rate=0.02)
    _check(_detect(d, True, 2.5, 800, 700, 30, seg_len=128), d, True, 2.5, 800, 700, 30)


def test_long_window():
    # W = 9000 > 8192: every window is two numpy chunks, fresh_kernel's program has 2 chunk ends
    d = make_delta(36000, 23)
    _check(_detect(d, True, 4.0, 9000, 300, 100), d, True, 4.0, 9000, 300, 100)


def test_c5_window():
    # the C5 block counts: W = int(120 / (1024/192000)) = 22500, Fa = 3750, F0 = 1875
    d = make_delta(60000, 24, rate=0.001)
    _check(_detect(d, True, 4.0, 22500, 3750, 1875), d, True, 4.0, 22500, 3750, 1875)


def test_global_mode():
    d = make_delta(30000, 25)
    _check(_detect(d, False, 4.0, 0, 0, 0), d, False, 4.0, 0, 0, 0)
    e = d.copy()
    e[-3:] = 60.0
    _check(_detect(e, False, 4.0, 0, 0, 0), e, False, 4.0, 0, 0, 0)


@pytest.mark.parametrize("case", ADAPTIVE, ids=[c[0] for c in ADAPTIVE])
def test_adaptive_kats(case):
    name, delta, k, (wsec, fb, fa, f0), dets, thr = case
    d = np.asarray(delta, np.float64)
    res = _detect(d, True, k, int(wsec), int(fa), int(f0))
    assert [(int(a), int(b)) for a, b, _ in res.detections] == [(a, b) for a, b, _ in dets]
    assert np.allclose(res.detections["db"], [x[2] for x in dets])
    assert np.allclose(res.thresholds, thr, equal_nan=True, rtol=0, atol=1e-12)
    _check(res, d, True, k, int(wsec), int(fa), int(f0))


@pytest.mark.parametrize("case", GLOBAL, ids=[c[0] for c in GLOBAL])
def test_global_kats(case):
    name, delta, k, dets, thr, err = case
    d = np.asarray(delta, np.float64)
    if err is not None:
        with pytest.raises(err):
            _detect(d, False, k, 0, 0, 0)
        return
    res = _detect(d, False, k, 0, 0, 0)
    assert [(int(a), int(b), float(x)) for a, b, x in res.detections] == [(a, b, float(x)) for a, b, x in dets]
    assert res.thr0 == pytest.approx(thr)


def test_sharded_threads():
    """world 4 in one process (one context per rank-thread), shard edges inside runs and freezes,
    one empty shard: the rounds of the shard-edge state exchange, on the device kernels"""
    from meteorgpu import _lib, stream
    d = make_delta(40000, 26, rate=0.02)
    want, _ = oracle(d, True, 3.0, 600, 400, 50)
    a = want[10][0] + 1
    b = want[30][0] + 20
    cuts = [a, b, b]

    def body(r, comm):
        lo, hi = shard_bounds(d.size, 4, r, cuts)
        ctx = _lib.Context(0)
        try:
            cfg = _lib.det_cfg(True, 3.0, 600, 0, 400, 50)
            plan = _lib.StreamPlan(ctx, cfg, d.size, lo, hi - lo, seg_len=256)
            plan.set_delta(d[lo:hi])
            res = stream.StreamDetector(stream.DeviceStreamOps(plan), comm, True, 3.0, 600, 50).run()
            plan.close()
            return res
        finally:
            ctx.close()

    res = run_threads(4, body)
    for r in res:
        assert [(int(x), int(y)) for x, y, _ in r.detections] == [(p, q) for p, q, _ in want]
        assert np.array_equal(r.detections["db"], np.array([w[2] for w in want]))
    _, thr = oracle(d, True, 3.0, 600, 400, 50)
    assert np.array_equal(np.concatenate([r.thresholds for r in res]), np.asarray(thr), equal_nan=True)


def test_empty_and_tiny():
    from meteorgpu import stream
    r = _detect(np.zeros(0), True, 4.0, 10, 5, 2)
    assert len(r.detections) == 0
    with pytest.raises(IndexError):
        _detect(np.zeros(0), False, 4.0, 0, 0, 0)
    d = make_delta(37, 27)
    _check(_detect(d, True, 1.0, 10, 3, 2), d, True, 1.0, 10, 3, 2)
    assert stream is not None


@pytest.mark.parametrize("seed,adaptive", [(1, True), (2, True), (3, False)])
def test_iq_end_to_end(seed, adaptive):
    from meteorgpu import iq, synth
    from oracle import iq_oracle as Q
    i, q, _ = synth.synth_iq(seed, 192000, 40.0, 1000.0, rate_per_min=20)
    kw = dict(flag_adaptive_threshold=adaptive, threshold_estimation_window_sec=5,
              threshold_freeze_after_detection_sec=2, threshold_fixed_init_duration_sec=1)
    dets, thr, delta, res = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), **kw)
    rdets, rthr, _, _, rdelta = Q.proc_iq_ref(i, q, 192000, (950, 1050), (-3050, -2950), **kw)
    assert delta.shape == rdelta.shape
    assert np.max(np.abs(delta - rdelta)) < DELTA_TOL
    assert res.certified and not res.near_tie  # every decision proven to be the float64 reference's
    assert [(d.t_start, d.t_stop) for d in dets] == [(r[0], r[1]) for r in rdets]
    assert np.max(np.abs(np.array([d.dB for d in dets]) - [r[3] for r in rdets])) < DB_TOL
    inside = np.zeros(delta.size, bool)
    for r in rdets:  # the detections' frames are float64: within the refinement's bound of the oracle
        inside[int(round(r[0] * 192000 / 1024)): int(round(r[1] * 192000 / 1024))] = True
    assert np.max(np.abs(delta - rdelta)[inside]) < DB_TOL
    # int16 at C5's geometry: every frame's delta is the exact one already (none left to refine)
    assert res.refined_delta_frames == 0 and np.max(np.abs(delta - rdelta)) < DB_TOL
    # on the device's own delta the detector is bit-exact with the oracle's
    bs = 1024 / 192000
    from oracle import dsp_oracle as O
    if adaptive:
        odets, othr = O.get_detections_adaptive_ref(delta, 4.0, bs, 5, 3, 2, 1)
        assert np.array_equal(np.asarray(thr), np.asarray(othr), equal_nan=True)
    else:
        odets, othr = O.get_detections_ref(delta, 4.0, bs)
        assert thr == othr
    assert [(d.t_start, d.t_stop, d.dB) for d in dets] == [(r[0], r[1], r[3]) for r in odets]


def test_iq_sharded_threads():
    """an I/Q stream time-sharded over 3 rank-threads (each its own spectrogram of its samples):
    the same detections as one process"""
    from meteorgpu import _lib, iq, synth
    i, q, _ = synth.synth_iq(4, 192000, 30.0, 1000.0, rate_per_min=30)
    buf, _ = iq.interleave(i, q)
    kw = dict(threshold_estimation_window_sec=3, threshold_freeze_after_detection_sec=1,
              threshold_fixed_init_duration_sec=1)
    one, *_ = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), **kw)

    def body(r, comm):
        ctx = _lib.Context(0)
        try:
            det = iq.IQShardDetector(ctx, i.size, 192000, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                     3, 3, 1, 1, rank=r, world=3, seg_len=512)
            det.upload(buf[2 * det.s0: 2 * det.s1])
            det.spectrogram_and_delta()
            res = det.detect(comm)
            det.close()
            return res
        finally:
            ctx.close()

    res = run_threads(3, body)
    bs = 1024 / 192000
    for r in res:
        assert [(int(a) * bs, int(b) * bs) for a, b, _ in r.detections] == [(d.t_start, d.t_stop) for d in one]
        assert np.array_equal(r.detections["db"], np.array([d.dB for d in one]))


def test_iq_half_hour_sharded_matches_whole():
    """C5 at scale with the reference's defaults (window 120 s = 22 500 frames, freeze 20 s, fixed
    init 10 s): a 30-minute 192 kHz stream (337 k frames, tiled from seeded 1-minute chunks as the
    bench does) time-sharded over 4 rank-threads, each with its own context and spectrogram of its
    samples, gives the detections, dB values and thresholds of one process holding the whole
    stream, bit for bit (the oracle comparison lives at sizes the CPU finishes in seconds)"""
    from meteorgpu import _lib, iq, synth
    fs, minutes = 192000, 30
    chunk = fs * 60
    pool = []
    for j in range(4):
        i_, q_, _ = synth.synth_iq(700 + j, fs, 60.0, 1000.0, sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))
        z = np.empty(2 * chunk, np.int16)
        z[0::2], z[1::2] = i_, q_
        pool.append(z)
    n = chunk * minutes + 3072
    buf = np.empty(2 * n, np.int16)
    for k in range(minutes + 1):
        a, b = k * chunk, min((k + 1) * chunk, n)
        if a < b:
            buf[2 * a: 2 * b] = pool[k % 4][: 2 * (b - a)]

    def run(world, thresholds):
        def body(r, comm):
            ctx = _lib.Context(0)
            try:
                det = iq.IQShardDetector(ctx, n, fs, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                         rank=r, world=world, certify=False)
                det.upload(buf[2 * det.s0: 2 * det.s1])
                det.spectrogram_and_delta()
                res = det.detect(comm, thresholds=thresholds)
                det.close()
                return res
            finally:
                ctx.close()
        return run_threads(world, body)

    for thresholds in (False, True):
        one = run(1, thresholds)[0]
        assert len(one.detections) > 100
        four = run(4, thresholds)
        for r in four:
            assert np.array_equal(r.detections, one.detections)
            assert r.thr0 == one.thr0
        if thresholds:  # each rank holds the thresholds of its own frames
            got = np.concatenate([np.asarray(r.thresholds) for r in four])
            assert np.array_equal(got, np.asarray(one.thresholds), equal_nan=True)


def test_iq_day_eight_shards_chunked_matches_whole():
    """C5 as BASELINE configures it: 24 h of 192 kHz I/Q (16.2 M frames, 66 GB of int16 in, 265 GB
    of spectrogram), time-sharded over 8 rank-threads (the 8-GPU layout on one device, each with its
    own context), each streaming its 3 h through HBM in 2^19-frame chunks
    (IQShardDetector.process_source), the reference's default detector settings, decisions only
    (the bench's mode): the same detections, dB values and whole-stream threshold as one process
    streaming the whole day.  The stream is tiled from seeded 1-minute chunks, as in the bench."""
    from meteorgpu import _lib, iq, synth
    fs, chunk, period = 192000, 192000 * 60, 4
    pool = np.empty(2 * chunk * period, np.int16)  # 4 minutes, repeated
    for j in range(period):
        i_, q_, _ = synth.synth_iq(900 + j, fs, 60.0, 1000.0, sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))
        pool[2 * j * chunk: 2 * (j + 1) * chunk: 2], pool[2 * j * chunk + 1: 2 * (j + 1) * chunk: 2] = i_, q_
    P = chunk * period
    n = fs * 24 * 3600 + 3072

    def stream(a, b):  # interleaved samples [a, b) of the day
        parts = []
        while a < b:
            o = a % P
            m = min(b - a, P - o)
            parts.append(pool[2 * o: 2 * (o + m)])
            a += m
        return np.concatenate(parts) if len(parts) > 1 else parts[0]

    def run(world):
        def body(r, comm):
            ctx = _lib.Context(0)
            try:
                det = iq.IQShardDetector(ctx, n, fs, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                         rank=r, world=world, chunk_frames=1 << 19, certify=False)
                assert det.W == 22500
                det.process_source(lambda a, b: stream(det.s0 + a, det.s0 + b))
                res = det.detect(comm, thresholds=False)
                det.close()
                return res
            finally:
                ctx.close()
        return run_threads(world, body)

    one = run(1)[0]
    assert len(one.detections) > 5000
    for r in run(8):
        assert np.array_equal(r.detections, one.detections)
        assert r.thr0 == one.thr0


def test_stream_detector_over_rccl_single_rank():
    """The C5 exchange path through RCCL (msd_comm_allgather behind stream.RcclComm) at world
    size 1 on the one-GPU box: variable-length allgathers round-trip, and the detector run
    through them equals the oracle."""
    from meteorgpu import _lib, stream
    from meteorgpu.batch import Communicator
    ctx = _lib.Context(0)
    comm = Communicator(ctx, 1, Communicator.unique_id(), 0)
    try:
        rc = stream.RcclComm(comm, 0, 1)
        for a in (np.arange(5, dtype=np.int64), np.linspace(0, 1, 1000), np.zeros(0)):
            got = rc.allgather(a)
            assert len(got) == 1 and got[0].dtype == a.dtype and np.array_equal(got[0], a)
        d = make_delta(30000, 31, rate=0.01)
        cfg = _lib.det_cfg(True, 4.0, 600, 0, 100, 50)
        plan = _lib.StreamPlan(ctx, cfg, d.size, 0, d.size, seg_len=1024)
        plan.set_delta(d)
        res = stream.StreamDetector(stream.DeviceStreamOps(plan), rc, True, 4.0, 600, 50).run()
        plan.close()
        _check(res, d, True, 4.0, 600, 100, 50)
    finally:
        comm.close()
        ctx.close()


def test_iq_dc_band_float32_global():
    """a band straddling DC (its bins sit at both ends of the FFT-order row), float32 I/Q input,
    the global detector: band delta within DELTA_TOL of scipy, same detections"""
    from meteorgpu import iq, synth
    from oracle import iq_oracle as Q
    i, q, _ = synth.synth_iq(8, 192000, 20.0, 30.0, rate_per_min=6, snr_db=(25, 35))
    fi, fq = (i / 32768).astype(np.float32), (q / 32768).astype(np.float32)
    band, noise = (-80.0, 80.0), (2000.0, 2200.0)
    assert iq.iq_band_bins(4096, 192000, band)[0] < 0 <= iq.iq_band_bins(4096, 192000, band)[1]
    kw = dict(flag_adaptive_threshold=False)
    dets, thr, delta, _ = iq.proc_iq_samples(fi, fq, 192000, band, noise, **kw)
    rdets, rthr, _, _, rdelta = Q.proc_iq_ref(fi, fq, 192000, band, noise, **kw)
    assert np.max(np.abs(delta - rdelta)) < DELTA_TOL
    assert np.min(np.abs(rdelta - rthr)) > 10 * DELTA_TOL
    assert len(rdets) > 0
    assert [(d.t_start, d.t_stop) for d in dets] == [(r[0], r[1]) for r in rdets]


def test_iq_csv_matches_oracle(tmp_path):
    """proc_iq_samples writes the reference's detection CSV (main.py:640-658): against the CSV the
    oracle writes from its OWN detections and dB values, the header and the t_start / t_stop /
    dur_s / utc columns are string-equal row for row and the dB column is within DB_TOL"""
    import csv
    import datetime
    from meteorgpu import iq, synth
    from oracle import dsp_oracle as O
    from oracle import iq_oracle as Q
    i, q, _ = synth.synth_iq(1, 192000, 40.0, 1000.0, rate_per_min=20)
    t0 = datetime.datetime(2025, 6, 1, 13, 59, 50)
    kw = dict(threshold_estimation_window_sec=5, threshold_freeze_after_detection_sec=2,
              threshold_fixed_init_duration_sec=1, wav_start_date_time=t0)
    out = tmp_path / "gpu.csv"
    dets, *_ = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), out_csv_file=str(out), **kw)
    rdets, *_ = Q.proc_iq_ref(i, q, 192000, (950, 1050), (-3050, -2950), **kw)
    ref = tmp_path / "ref.csv"
    O.write_csv_ref(rdets, str(ref))
    assert len(dets) == len(rdets) > 0
    got, want = out.read_bytes().split(b"\r\n"), ref.read_bytes().split(b"\r\n")
    assert len(got) == len(want) and got[0] == want[0]  # rows and header
    rows = list(csv.DictReader(open(out, newline=""))), list(csv.DictReader(open(ref, newline="")))
    for g, w in zip(*rows):
        for col in ("t_start", "t_stop", "dur_s", "utc_start", "utc_stop"):
            assert g[col] == w[col], (col, g, w)
        assert abs(float(g["dB"]) - float(w["dB"])) < DB_TOL, (g["dB"], w["dB"])


def test_capacity_and_halo_errors_are_loud():
    """more runs in a segment than its capacity, or a shard whose last numpy chunk runs past its
    head halo, raise MsdError (never silently truncated results)"""
    from meteorgpu import _lib, stream
    d = make_delta(20000, 32, rate=0.05)
    with pytest.raises(_lib.MsdError) as e:
        _detect(d, True, 2.0, 300, 0, 10, seg_len=8192, cap=1)
    assert e.value.code == _lib.MSD_ERR_CAPACITY

    def body(r, comm):
        lo, hi = shard_bounds(d.size, 2, r)
        ctx = _lib.Context(0)
        try:
            cfg = _lib.det_cfg(True, 4.0, 300, 0, 50, 10)
            plan = _lib.StreamPlan(ctx, cfg, d.size, lo, hi - lo, seg_len=1024, head_frames=100)
            plan.set_delta(d[lo:hi])
            try:
                return stream.StreamDetector(stream.DeviceStreamOps(plan), comm, True, 4.0, 300, 10,
                                             head_frames=100).run()
            finally:
                plan.close()
        finally:
            ctx.close()

    with pytest.raises(_lib.MsdError) as e:
        run_threads(2, body)
    assert e.value.code == _lib.MSD_ERR_UNSUPPORTED


def test_iq_chunked_spectrogram_matches_whole():
    """streaming the spectrogram through HBM in chunks (long recordings on one GPU) gives the same
    delta, bit for bit, and the same detections as one pass"""
    from meteorgpu import iq, synth
    i, q, _ = synth.synth_iq(2, 192000, 40.0, 1000.0, rate_per_min=20)
    kw = dict(threshold_estimation_window_sec=5, threshold_freeze_after_detection_sec=2,
              threshold_fixed_init_duration_sec=1)
    d1, t1, delta1, _ = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), **kw)
    d2, t2, delta2, _ = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), chunk_sec=3.3, **kw)
    assert np.array_equal(delta1, delta2)
    assert [(d.t_start, d.t_stop, d.dB) for d in d1] == [(d.t_start, d.t_stop, d.dB) for d in d2]
    assert np.array_equal(np.asarray(t1), np.asarray(t2), equal_nan=True)


def _random_case(seed, thresholds=True):
    """seeded random settings, segment lengths and shard cuts through the device plans (one
    context per rank-thread): bit-exact with the one-process oracle"""
    from meteorgpu import _lib, stream
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(2000, 40000))
    d = make_delta(n, 200 + seed, rate=float(rng.uniform(0.002, 0.03)))
    adaptive = bool(rng.integers(0, 4) > 0)
    k = float(rng.choice([2.0, 3.0, 4.0]))
    W, Fa, F0 = int(rng.integers(0, 12000)), int(rng.integers(0, 3000)), int(rng.integers(0, 2000))
    world = int(rng.integers(1, 5))
    seg = int(rng.choice([64, 256, 1024, 8192]))
    cuts = sorted(int(c) for c in rng.integers(0, n + 1, world - 1))
    try:
        oracle(d, adaptive, k, W, Fa, F0)
    except AssertionError:
        pytest.skip("the reference asserts on this stream (zero-duration global run)")

    def body(r, comm):
        lo, hi = shard_bounds(n, world, r, cuts)
        ctx = _lib.Context(0)
        try:
            cfg = _lib.det_cfg(adaptive, k, W, 0, Fa, F0)
            plan = _lib.StreamPlan(ctx, cfg, n, lo, hi - lo, seg_len=seg, head_frames=16384)
            plan.set_delta(d[lo:hi])
            try:
                return stream.StreamDetector(stream.DeviceStreamOps(plan), comm, adaptive, k, W, F0,
                                             head_frames=16384).run(thresholds)
            finally:
                plan.close()
        finally:
            ctx.close()

    res = run_threads(world, body)
    want, thr = oracle(d, adaptive, k, W, Fa, F0)
    for r in res:
        assert [(int(a), int(b)) for a, b, _ in r.detections] == [(a, b) for a, b, _ in want]
        assert np.array_equal(r.detections["db"], np.array([w[2] for w in want], np.float64))
    if not thresholds:
        assert all(r.thresholds is None for r in res)
    elif adaptive:
        assert np.array_equal(np.concatenate([r.thresholds for r in res]), np.asarray(thr), equal_nan=True)
    else:
        assert res[0].thr0 == thr


@pytest.mark.parametrize("seed", range(8))
def test_random_sharded_device(seed):
    _random_case(seed)


@pytest.mark.parametrize("seed", range(8))
def test_random_sharded_decisions_only(seed):
    """run(thresholds=False): predicted thresholds with an error bound, exact only at near ties
    and triggers -- the same detections"""
    _random_case(seed, thresholds=False)


@pytest.mark.parametrize("seed", [1, 5])
def test_decisions_only_wide_bound(seed, monkeypatch):
    """the bound widened (MSD_STREAM_EPS_SCALE) until every unfrozen frame is a near tie: the
    per-frame exact path carries the whole detector"""
    monkeypatch.setenv("MSD_STREAM_EPS_SCALE", "1e30")
    _random_case(seed, thresholds=False)


def test_decisions_only_exact_ties():
    """frames whose delta is the numpy threshold itself, or one ulp either side: the prediction
    cannot decide them, the exact values must"""
    from meteorgpu import stream
    k, W, Fa, F0 = 3.0, 3000, 200, 100
    d = make_delta(30000, 77, rate=0.001)
    tied = []
    for n, i in enumerate(range(W + 500, d.size, 700)):
        win = d[i - W: i]
        t = np.mean(win) + k * np.std(win)
        d[i] = [t, np.nextafter(t, np.inf), np.nextafter(t, -np.inf)][n % 3]
        tied.append((i, t))
    want, thr = oracle(d, True, k, W, Fa, F0)
    used = [i for i, t in tied if thr[i] == t]  # the oracle was unfrozen there: a real tie
    assert len(used) >= 20  # 29 on this stream, a third of them detections (one ulp above)
    res = stream.detect_stream(_ctx(), d, d.size, 0, adaptive=True, k_std=k, window_blocks=W,
                               freeze_after_blocks=Fa, fixed_init_blocks=F0, seg_len=1024)
    _check(res, d, True, k, W, Fa, F0)
    ctxd = _ctx()
    from meteorgpu import _lib
    cfg = _lib.det_cfg(True, k, W, 0, Fa, F0)
    plan = _lib.StreamPlan(ctxd, cfg, d.size, 0, d.size, seg_len=1024)
    try:
        plan.set_delta(d)
        r = stream.StreamDetector(stream.DeviceStreamOps(plan), stream.LocalComm(), True, k, W, F0).run(False)
    finally:
        plan.close()
    assert [(int(a), int(b)) for a, b, _ in r.detections] == [(a, b) for a, b, _ in want]
    assert np.array_equal(r.detections["db"], np.array([w[2] for w in want], np.float64))


def test_iq_wav_file(tmp_path):
    """a 2-channel I/Q WAV through the native reader gives the same detections and CSV as the samples"""
    from meteorgpu import iq, synth, wav
    i, q, _ = synth.synth_iq(1, 192000, 40.0, 1000.0, rate_per_min=20)
    path = tmp_path / "iq.wav"
    wav.write(path, 192000, np.stack([i, q], 1))
    kw = dict(threshold_estimation_window_sec=5, threshold_freeze_after_detection_sec=2,
              threshold_fixed_init_duration_sec=1)
    a, *_ = iq.proc_iq_samples(i, q, 192000, (950, 1050), (-3050, -2950), out_csv_file=str(tmp_path / "a.csv"), **kw)
    b, *_ = iq.proc_iq_wav_file(str(path), (950, 1050), (-3050, -2950), out_csv_file=str(tmp_path / "b.csv"), **kw)
    assert len(a) > 0 and (tmp_path / "a.csv").read_bytes() == (tmp_path / "b.csv").read_bytes()


def test_fresh_all_option_agrees():
    """MSD_OPT_FRESH_ALL (every adaptive threshold exact up front) and the default scheme (only
    where a scan reads them) give identical results"""
    from meteorgpu import _lib, stream
    d = make_delta(30000, 41, rate=0.01)
    out = []
    for opt in (0, 1):
        ctx = _lib.Context(0)
        try:
            ctx.set_option(_lib.OPT_FRESH_ALL, opt)
            out.append(stream.detect_stream(ctx, d, d.size, 0, adaptive=True, k_std=4.0, window_blocks=2000,
                                            freeze_after_blocks=500, fixed_init_blocks=100, seg_len=1024))
        finally:
            ctx.close()
    a, b = out
    assert np.array_equal(a.detections, b.detections)
    assert np.array_equal(a.thresholds, b.thresholds, equal_nan=True)
    _check(a, d, True, 4.0, 2000, 500, 100)


def _bound_case(d, W, k, f0, nl):
    """predicted thresholds and bounds of the shard [f0, f0 + nl) vs numpy's thresholds"""
    from meteorgpu import _lib
    n = d.size
    ctx = _ctx()
    plan = _lib.StreamPlan(ctx, _lib.det_cfg(True, k, W, 0, 100, 0), n, f0, nl, seg_len=1024, head_frames=8192)
    try:
        plan.set_delta(d[f0: f0 + nl])
        plan.set_halos(d[f0 - plan.n_tail: f0], d[f0 + nl: f0 + nl + plan.n_head])
        plan.set_exact_thresholds(False)
        plan.fresh()
        pred, eps = plan.predicted()
    finally:
        plan.close()
    worst = 0.0
    for j in range(nl):
        i = f0 + j
        if i == 0:
            assert np.isnan(pred[j]) or np.isnan(eps[j])  # empty window: NaN, decided exactly
            continue
        win = d[max(0, i - W): i]
        t = np.mean(win) + k * np.std(win)
        err = abs(pred[j] - t)
        assert err <= eps[j], (i, pred[j], t, eps[j])
        worst = max(worst, err / eps[j] if eps[j] > 0 else 0.0)
    return worst


@pytest.mark.parametrize("kind", ["bursts", "dc_offset", "dynamic_range", "steps", "large"])
def test_prediction_error_bound(kind):
    """the decisions-only bound on |predicted - numpy| holds frame by frame (first shard with
    short windows, and a later shard over its halo), on streams chosen to stress it: a large DC
    offset over a tiny spread, values over 16 decades, constant stretches with jumps"""
    rng = np.random.default_rng({"bursts": 1, "dc_offset": 2, "dynamic_range": 3, "steps": 4, "large": 5}[kind])
    n, W = 20000, 3000
    if kind == "bursts":
        d = make_delta(n, 91)
    elif kind == "dc_offset":
        d = 1e4 + 1e-3 * rng.normal(size=n)
    elif kind == "dynamic_range":
        d = rng.normal(size=n) * 10.0 ** rng.uniform(-8, 8, n)
    elif kind == "steps":
        d = np.repeat(rng.choice([0.0, 1.0, 1e6, -3.5], n // 500), 500).astype(np.float64)
    else:
        d = 1e12 + rng.normal(size=n) * 1e3
    worst = max(_bound_case(d, W, 4.0, 0, 8000), _bound_case(d, W, 2.5, 9000, 6000))
    print(f"{kind}: max |predicted - numpy| / bound = {worst:.3g}")
    assert worst <= 1.0  # |error| <= eps (the bound carries a factor 4 of margin)


@pytest.mark.parametrize("adaptive,thresholds", [(True, True), (True, False), (False, True)])
def test_native_local_path_equals_protocol(adaptive, thresholds):
    """msd_stream_detect_local (one native call, taken with LocalComm) and the Python protocol
    over a one-rank group give identical results"""
    from meteorgpu import _lib, stream
    d = make_delta(30000, 61, rate=0.01)
    k, W, Fa, F0 = 3.0, 2000, 300, 100

    def one(comm):
        ctx = _lib.Context(0)
        try:
            plan = _lib.StreamPlan(ctx, _lib.det_cfg(adaptive, k, W, 0, Fa, F0), d.size, 0, d.size, seg_len=1024)
            try:
                plan.set_delta(d)
                return stream.StreamDetector(stream.DeviceStreamOps(plan), comm, adaptive, k, W, F0).run(thresholds)
            finally:
                plan.close()
        finally:
            ctx.close()

    a = one(stream.LocalComm())
    b = run_threads(1, lambda r, comm: one(comm))[0]
    assert np.array_equal(a.detections, b.detections) and len(a.detections) > 10
    assert a.thr0 == b.thr0 and a.margin == b.margin and a.refined == b.refined
    if thresholds:
        assert np.array_equal(a.thresholds, b.thresholds, equal_nan=True)
    _check(a, d, adaptive, k, W, Fa, F0) if thresholds else None


def test_native_local_path_errors():
    """the reference's exceptions through the native path: empty global input, zero-duration
    last global run"""
    from meteorgpu import _lib, stream
    ctx = _ctx()
    with pytest.raises(IndexError):
        stream.detect_stream(ctx, np.zeros(0), 0, 0, adaptive=False, k_std=4.0)
    d = make_delta(5000, 62)
    d[-2], d[-1] = -50.0, 50.0  # one block above at the end: t_dur == 0 (main.py:437)
    with pytest.raises(AssertionError):
        stream.detect_stream(ctx, d, d.size, 0, adaptive=False, k_std=4.0)


@pytest.mark.parametrize("chunk", [None, 1500])
def test_overlapped_detector_matches_in_order(chunk):
    """IQShardDetector(overlap=n): the exact delta first, then the spectrogram with n workgroup slots
    left free and the stream detector on a second context beside it -- the same detections, dB
    values and delta bit for bit as one in-order stream, and the same spectrogram (also when the
    shard streams through HBM in chunks)"""
    from meteorgpu import _lib, iq, synth
    i, q, _ = synth.synth_iq(12, 192000, 30.0, 1000.0, rate_per_min=20)
    buf, _ = iq.interleave(i, q)
    kw = dict(threshold_estimation_window_sec=5, threshold_freeze_after_detection_sec=2,
              threshold_fixed_init_duration_sec=1)
    out = []
    for ov in (0, 16):
        ctx = _lib.Context(0)
        try:
            det = iq.IQShardDetector(ctx, i.size, 192000, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                     5, 3, 2, 1, chunk_frames=chunk, overlap=ov)
            try:
                assert det.exact_delta
                det.process_host(buf[2 * det.s0: 2 * det.s1])
                res = det.detect()
                det.synchronize()
                spec = det.batch.frames(0, 0, 16) if chunk is None else None
                out.append((res, det.plan.delta(), spec))
            finally:
                det.close()
        finally:
            ctx.close()
    (a, da, sa), (b, db, sb) = out
    assert a.certified and b.certified and len(a.detections) > 5
    assert np.array_equal(a.detections, b.detections) and np.array_equal(da, db)
    if chunk is None:
        assert np.array_equal(sa, sb)


def test_overlap_leaves_the_callers_context():
    """the overlap's spectrogram reserve lives on a sibling context: the caller's context keeps its
    options (a context-wide option changed by the detector), also when the constructor fails"""
    from meteorgpu import _lib, iq
    ctx = _lib.Context(0)
    try:
        ctx.set_option(_lib.OPT_CSTFT_RESERVE, 3)
        before = dict(ctx.options)
        det = iq.IQShardDetector(ctx, 192000 * 5, 192000, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                 5, 3, 2, 1, overlap=16)
        assert det.sctx is not ctx and det.dctx is not ctx
        assert det.sctx.options[_lib.OPT_CSTFT_RESERVE] == 16
        det.close()
        assert ctx.options == before
        with pytest.raises(_lib.MsdError):  # the stream plan refuses seg_len 100 (not a multiple of 64)
            iq.IQShardDetector(ctx, 192000 * 5, 192000, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                               5, 3, 2, 1, overlap=16, seg_len=100)
        assert ctx.options == before
    finally:
        ctx.close()


def test_overlapped_certified_ranks_match_one_process():
    """the overlap at world > 1: 3 rank-threads, each with its detector beside its spectrogram (8
    workgroup slots reserved, the chunked spectrogram) and the exact delta, exchange halos, chunk sums,
    states, runs and the certificate through the thread allgather -- the detections, dB values and
    certificate of one in-order process over the whole stream"""
    from meteorgpu import _lib, iq, synth
    fs = 192000
    i, q, _ = synth.synth_iq(31, fs, 40.0, 1000.0, rate_per_min=20)
    buf, _ = iq.interleave(i, q)
    kw = dict(threshold_estimation_window_sec=5, threshold_freeze_after_detection_sec=2,
              threshold_fixed_init_duration_sec=1)

    def run(world, ov):
        def body(r, comm):
            ctx = _lib.Context(0)
            try:
                det = iq.IQShardDetector(ctx, i.size, fs, 4096, 3072, (950, 1050), (-3050, -2950), 4.0, True,
                                         rank=r, world=world, overlap=ov, **kw)
                try:
                    assert det.exact_delta
                    det.upload(buf[2 * det.s0: 2 * det.s1])
                    res = None
                    for _ in range(2):  # a second step on the same buffers (the step-to-step ordering)
                        det.spectrogram_and_delta()
                        res = det.detect(comm, thresholds=False)
                    return res
                finally:
                    det.close()
            finally:
                ctx.close()
        return run_threads(world, body)

    one = run(1, 0)[0]
    assert one.certified and len(one.detections) > 5
    for r in run(3, 8):
        assert r.certified
        assert np.array_equal(r.detections, one.detections)
        assert r.thr0 == one.thr0

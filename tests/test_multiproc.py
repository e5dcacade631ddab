"""CPU, world_size 2 over gloo: the N>1 path's host logic — contiguous file shards, the
per-hour histogram (host restatement of the device one in detect.hip), and the one
exchange step (sum of hour counts across ranks) — gives the same day totals as one
process, and those equal the reference's Counter of detection hours (main.py:690-696).
The per-file detections come from the oracle here (no GPU); on the GPU box the same
shard/reduce code runs around the HIP pipeline (bench.py, RCCL)."""
import datetime
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

FS = 6000
SECONDS = 60
NFILES = 7           # not a multiple of the world size: ragged shards
DAY0 = datetime.datetime(2025, 6, 1, 0, 0)
STEP = datetime.timedelta(minutes=37)  # files spread over ~4.3 h → several hour buckets
BAND, NOISE = (980.0, 1020.0), (690.0, 730.0)


def _file(i):
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=500 + i, fs=FS, duration_s=SECONDS, f0=1000.0, band_hz=40, rate_per_min=6,
                            snr_db=(20, 35))
    return x


def _dets(i):
    from oracle import dsp_oracle as O
    dets, *_ = O.proc_samples_ref(_file(i), FS, 0.2, BAND, NOISE, 512, 4.0, wav_start_date_time=DAY0 + i * STEP)
    return dets


def _rank_main(rank, world, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "meteor-scatter_amd"), os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from meteorgpu import shard
    from torch_comm import allreduce_counts
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        lo, hi = shard.shard_range(NFILES, rank, world)
        starts = [[round(d[0] / 0.2) for d in _dets(i)] for i in range(lo, hi)]
        file_us = [shard.to_us(DAY0 + i * STEP) for i in range(lo, hi)]
        local = shard.hour_histogram(starts, file_us, 0.2, shard.to_us(DAY0), 24)
        total = allreduce_counts(local)
        np.save(os.path.join(out_dir, f"r{rank}.npy"), np.stack([local, total]))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_covers_exactly():
    from meteorgpu import shard
    for n in (0, 1, 7, 1440):
        for w in (1, 2, 3, 8):
            rs = [shard.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [h - l for l, h in rs]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(4, 2, 2)


def test_hour_histogram_matches_reference_counter():
    from meteorgpu import shard
    from oracle import dsp_oracle as O
    starts, file_us, ref = [], [], {}
    for i in range(NFILES):
        d = _dets(i)
        starts.append([round(x[0] / 0.2) for x in d])
        file_us.append(shard.to_us(DAY0 + i * STEP))
        for k, v in O.count_per_hour_ref(d).items():
            ref[k] = ref.get(k, 0) + v
    h = shard.hour_histogram(starts, file_us, 0.2, shard.to_us(DAY0), 24)
    assert h.sum() == sum(ref.values()) > 0
    for k, v in ref.items():
        assert h[int((k - DAY0).total_seconds() // 3600)] == v


def test_two_rank_gloo_reduction_equals_single_process(tmp_path):
    import torch.multiprocessing as mp
    from meteorgpu import shard
    world = 2
    mp.start_processes(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    r = [np.load(tmp_path / f"r{k}.npy") for k in range(world)]
    single = shard.hour_histogram([[round(d[0] / 0.2) for d in _dets(i)] for i in range(NFILES)],
                                  [shard.to_us(DAY0 + i * STEP) for i in range(NFILES)], 0.2, shard.to_us(DAY0), 24)
    np.testing.assert_array_equal(r[0][1], single)        # all-reduced total on every rank
    np.testing.assert_array_equal(r[1][1], single)
    np.testing.assert_array_equal(r[0][0] + r[1][0], single)
    assert single.sum() > 0 and (r[0][0].sum() > 0 and r[1][0].sum() > 0)

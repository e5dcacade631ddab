"""Sharding of independent recordings over GPUs (one process per GPU) and the one
exchange step of the path: the per-hour detection counts summed across ranks.

The reference processes files one by one in a single process (main.py:865-935 loop,
per-hour aggregation main.py:687-716).  Files are independent: each file's global
threshold, adaptive window and freeze state are file-local (main.py:464-466, 450-522),
so a batch shards as contiguous file ranges with no data-path collective; only the
per-hour histogram (a few dozen int64) is all-reduced: one RCCL all-reduce on the device
histogram (``batch.Communicator``, set up by ``launch.Group``).  The CPU tests stand in
for it with a gloo all-reduce (tests/torch_comm.py).
"""
from __future__ import annotations

import datetime

import numpy as np

_EPOCH = datetime.datetime(1970, 1, 1)


def shard_range(n_items: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced [lo, hi) range of ``n_items`` for ``rank`` of ``world``
    (the first ``n_items % world`` ranks take one extra item)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    base, extra = divmod(int(n_items), int(world))
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def to_us(t: datetime.datetime) -> int:
    """Naive-UTC datetime → integer microseconds since the epoch (the device histogram's
    time base)."""
    if t.tzinfo is not None:
        t = t.astimezone(datetime.timezone.utc).replace(tzinfo=None)
    return (t - _EPOCH) // datetime.timedelta(microseconds=1)


def hour_histogram(start_blocks, file_start_us, block_sec: float, base_us: int, nbuckets: int,
                   bucket_us: int = 3600 * 10 ** 6) -> np.ndarray:
    """Host restatement of the device histogram (detect.hip): detection ``j`` of file ``f``
    starts at ``file_start_us[f] + round(start_blocks[f][j] * block_sec * 1e6)`` and falls in
    bucket ``floor((t - base_us) / bucket_us)``; out-of-range buckets are dropped.  With
    ``bucket_us`` = 1 h and ``base_us`` at a full hour this is main.py:690-696's
    ``utc_start.replace(minute=0, second=0, microsecond=0)`` key."""
    out = np.zeros(max(0, int(nbuckets)), np.int64)
    for f, starts in enumerate(start_blocks):
        for s in np.asarray(starts, dtype=np.int64):
            t = int(file_start_us[f]) + int(np.rint(float(s) * block_sec * 1e6))
            b = (t - int(base_us)) // int(bucket_us)
            if 0 <= b < nbuckets:
                out[b] += 1
    return out

"""Hand-derived known-answer cases for the reference detectors (SURVEY §8(a) KAT list).

Each case: delta, config, and the expected block-index detections [start, stop)
and thresholds, derived by hand from dsp/src/main.py:396-448 (global) and
:450-522 (adaptive) — see the comments — not by running any implementation.
block_sec = 1.0 keeps t = index exactly.
"""
import math

NAN = float("nan")

GLOBAL = [
    # name, delta, k, expected [(start, stop, dB)], expected threshold, error
    ("all_below", [0.0] * 10, 1.0, [], 0.0, None),
    # mean 1, std sqrt((9*1 + 81)/10) = 3 → thr 4; only block 3 above
    ("single_mid", [0, 0, 0, 10, 0, 0, 0, 0, 0, 0], 1.0, [(3, 4, 10.0)], 4.0, None),
    # above[0]: burst_starts gets 0 prepended (main.py:412-413)
    ("first_block", [10, 0, 0, 0, 0, 0, 0, 0, 0, 0], 1.0, [(0, 1, 10.0)], 4.0, None),
    # run reaching the end: stop = len-1 (main.py:414-415), so the last block is left out
    ("open_end", [0, 0, 0, 0, 0, 0, 0, 10, 10, 10], 0.5, [(7, 9, 10.0)], 3.0 + 0.5 * math.sqrt(21.0), None),
    # single block above at the very end: start = stop = 9 → t_dur == 0 → assert (main.py:437)
    ("last_block_assert", [0, 0, 0, 0, 0, 0, 0, 0, 0, 10], 1.0, None, 4.0, AssertionError),
    # two bursts
    ("two_bursts", [0, 10, 10, 0, 0, 10, 0, 0, 0, 0], 0.0, [(1, 3, 10.0), (5, 6, 10.0)], 3.0, None),
    # empty input: above_thresh[0] → IndexError (main.py:412)
    ("empty", [], 1.0, None, NAN, IndexError),
]

ADAPTIVE = [
    # name, delta, k, (window_sec, freeze_before_sec, freeze_after_sec, fixed_init_sec), expected dets,
    # expected thresholds
    # W=3, Fa=2, F0=0: i=0 empty window → NaN threshold; ties (1 > 1) are not detections; block 4 fires,
    # freeze until 6; i=7 window [9,1,1] → 11/3 + std; then back to 1.
    ("freeze_and_ties", [1, 1, 1, 1, 9, 1, 1, 1, 1, 1], 1.0, (3, 0, 2, 0), [(4, 5, 9.0)],
     [NAN, 1, 1, 1, 1, 1, 1, 11 / 3 + math.sqrt(((9 - 11 / 3) ** 2 + 2 * (1 - 11 / 3) ** 2) / 3), 1, 1]),
    # fixed threshold everywhere (F0=100 > nb): consecutive blocks merge, a one-block gap splits
    ("merge_and_split", [0, 10, 10, 0, 10, 0, 0, 10, 0, 0], 0.0, (120, 3, 20, 100),
     [(1, 3, 10.0), (4, 5, 10.0), (7, 8, 10.0)], [4.0] * 10),
    # detection inside the fixed-init phase (F0=3): the freeze (Fa=4 → until 6) holds thr0 past F0;
    # i=7,8 use fresh windows of zeros (thr 0): 5 > 0 fires at 8
    ("fixed_init_then_freeze", [0, 0, 10, 0, 0, 0, 0, 0, 5, 0], 0.0, (2, 0, 4, 3), [(2, 3, 10.0), (8, 9, 5.0)],
     [1.5] * 7 + [0.0, 0.0, 0.0]),
    # freeze-before is a no-op (max(i+Fa, i-Fb) = i+Fa): same answer with Fb = 5
    ("freeze_before_noop", [0, 0, 10, 0, 0, 0, 0, 0, 5, 0], 0.0, (2, 5, 4, 3), [(2, 3, 10.0), (8, 9, 5.0)],
     [1.5] * 7 + [0.0, 0.0, 0.0]),
    # constant delta (e.g. two zero-bin bands: both -120 dB): thresholds equal delta, nothing fires
    ("constant", [0.0] * 12, 4.0, (2, 0, 1, 0), [], [NAN] + [0.0] * 11),
    # empty input: no loop iterations, no detections, no error (main.py:470)
    ("empty", [], 4.0, (120, 3, 20, 10), [], []),
]

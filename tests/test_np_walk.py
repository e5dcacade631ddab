"""The iterative walk of numpy's pairwise-summation tree (csrc/np_reduce.h np_walk_iter, used by
np_sum / np_pairwise and the detector's fresh windows) restated step by step in Python: for every
length up to its depth limit it must produce numpy's association, i.e. the same expression tree
as numpy's recursion (DOUBLE_pairwise_sum, numpy/_core/src/umath/loops_utils.h.src: n <= 128 a
leaf, else n2 = n / 2 - (n / 2) % 8, left + right).  The device results themselves are checked
bit-exact against numpy in tests/test_gpu_parity.py (detector thresholds, dB means)."""
import numpy as np

NP_ITER_MAX = [128, 248, 488, 968, 1928, 3848, 7688, 8192]  # np_reduce.h


def _numpy_tree(b, n):
    if n <= 128:
        return ("leaf", b, n)
    n2 = n // 2
    n2 -= n2 % 8
    return ("+", _numpy_tree(b, n2), _numpy_tree(b + n2, n - n2))


def _walk(n, dmax, leaf=lambda b, m: ("leaf", b, m), add=lambda x, y: ("+", x, y)):
    """np_walk_iter: shifted register stacks of pending right subtrees and finished left sums"""
    pb, ps, pv = [0] * dmax, [0] * dmax, [None] * dmax
    b, s, d, right = 0, n, 0, 0
    while True:
        while s > 128:
            s2 = s // 2
            s2 -= s2 % 8
            pb[1:], ps[1:] = pb[:-1], ps[:-1]
            pb[0], ps[0] = b + s2, s - s2
            s = s2
            d += 1
            assert d <= dmax
            right &= ~(1 << d)
        v = leaf(b, s)
        while d > 0 and (right >> d) & 1:
            v = add(pv[0], v)
            pv[:-1] = pv[1:]
            d -= 1
        if d == 0:
            return v
        pv[1:] = pv[:-1]
        pv[0] = v
        b, s = pb[0], ps[0]
        pb[:-1], ps[:-1] = pb[1:], ps[1:]
        right |= 1 << d


def test_depth_limits():
    """NP_ITER_MAX[D] is the largest n whose tree is at most D splits deep"""
    from functools import lru_cache

    @lru_cache(maxsize=None)
    def depth(n):
        if n <= 128:
            return 0
        n2 = n // 2
        n2 -= n2 % 8
        return 1 + max(depth(n2), depth(n - n2))
    for dmax in range(7):
        first_deeper = next(n for n in range(1, 8193) if depth(n) > dmax)
        assert first_deeper == NP_ITER_MAX[dmax] + 1, dmax
    assert max(depth(n) for n in range(1, 8193)) == 7


def test_walk_is_numpys_association():
    for dmax in (4, 7):
        for n in range(0, NP_ITER_MAX[dmax] + 1, 1 if dmax == 4 else 3):
            assert _walk(n, dmax) == _numpy_tree(0, n), (dmax, n)


def test_walk_sum_matches_numpy_bits():
    rng = np.random.default_rng(5)
    for n in (129, 300, 1000, 1928, 5000, 8192):
        x = rng.standard_normal(n) * 10.0 ** rng.uniform(-3, 3, n)

        def leaf(b, m):  # numpy's leaf: 8 interleaved accumulators, then the tail
            if m < 8:
                r = -0.0
                for i in range(m):
                    r += x[b + i]
                return r
            r = [x[b + j] for j in range(8)]
            i = 8
            while i < m - m % 8:
                for j in range(8):
                    r[j] += x[b + i + j]
                i += 8
            res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))
            while i < m:
                res += x[b + i]
                i += 1
            return res
        got = 0.0 + _walk(n, 7, leaf=leaf, add=lambda a, c: a + c)
        assert got == float(np.sum(x)), n

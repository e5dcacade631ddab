"""Near-tie guard for the block detector: a bound on |delta_gpu - delta_numpy| and the decisions
it can flip.

The detector's decisions are strict comparisons ``delta[i] > thr[i]`` (dsp/src/main.py:406,
:485).  libmsdsp reproduces numpy's summation order for every threshold, so with IDENTICAL
delta values the decisions are identical bit for bit.  delta itself is not identical: the
reference takes it from pocketfft's float64 rFFT (main.py:379-393), the device from a float64
Goertzel over the band bins (csrc/block_delta.hip).  Both are accurate to a small multiple of
the unit roundoff; this module bounds the difference per block and flags a file whose smallest
decision margin ``min |delta - thr|`` (computed on the device) is not larger than the bound.
Such a file may differ from the reference in a detection boundary; every other file cannot.

The bound (standard floating-point error model, u = 2^-53):

* a computed bin differs from the exact DFT by at most ``c * u * S`` with
  ``S = sum_j |x_j w_j| <= max|x| * sum(w)`` over the L samples used and ``c`` the longest chain
  of roundings an input term passes through: pocketfft's real FFT ``4 log2(Nf) + 8``; the
  Goertzel segments ``3 L_seg G + 24`` (L_seg samples per lane, G = min(1/|sin theta|, L_seg)
  the recurrence's error gain at bin angle theta, 24 for the rotations and the 16-lane sum);
* a band energy E = sum |X_k|^2 + 1e-12 over n bins then moves by at most
  ``dE = 2 sqrt(n E) dX + n dX^2 + (n + 2) u E``;
* its dB value by at most ``10/ln 10 * r / (1 - r) + 2 u`` with r = dE / E (unbounded when
  r >= 1: a band with no energy is never trusted);
* delta by the sum of the band's and the noise band's;
* a threshold ``mean + k std`` over a window moves by at most (1 + k) max |d delta| (the mean
  and the population std are 1-Lipschitz in the max norm);
* so a decision can only flip where |delta - thr| <= (2 + k) max_i |d delta_i|.

``tests/test_near_tie.py`` checks the per-block bound against numpy on random and adversarial
blocks and the flag on a constructed near-tie stream.
"""
from __future__ import annotations

import math
import warnings

import numpy as np

U = 2.0 ** -53
DB = 10.0 / math.log(10.0)


class NearTieWarning(UserWarning):
    """A detection decision lies within the delta error bound of its threshold."""


def _chain(nfft: int, L: int, bins: np.ndarray) -> float:
    """c: longest rounding chain of a bin (pocketfft + the device's Goertzel segments)."""
    l_seg = max(1, -(-int(L) // 16))  # samples per lane: the block_delta kernel's 16 lanes
    theta = 2.0 * np.pi * np.asarray(bins, dtype=np.float64) / float(nfft)
    s = np.abs(np.sin(theta))
    gain = np.minimum(np.where(s > 0, 1.0 / np.maximum(s, 1e-300), np.inf), float(l_seg))
    g = float(gain.max()) if gain.size else 1.0
    return 4.0 * math.log2(nfft) + 8.0 + 3.0 * l_seg * g + 24.0


def band_db_error(e_db: np.ndarray, nbins: int, dx: float) -> np.ndarray:
    """Per-block bound on |10 log10 E_gpu - 10 log10 E_numpy| given the band's dB values."""
    e = np.power(10.0, np.asarray(e_db, dtype=np.float64) / 10.0)
    if nbins <= 0:  # empty band: E = 1e-12 exactly on both sides
        return np.zeros_like(e)
    de = 2.0 * np.sqrt(nbins * e) * dx + nbins * dx * dx + (nbins + 2) * U * e
    with np.errstate(divide="ignore", invalid="ignore"):
        r = de / e
        out = np.where(r < 1.0, DB * r / (1.0 - r) + 2.0 * U * DB, np.inf)
    return out


def delta_error_bound(band_db: np.ndarray, noise_db: np.ndarray, *, nfft: int, L: int, window: np.ndarray,
                      xmax: float, band: tuple[int, int], noise: tuple[int, int]) -> np.ndarray:
    """Per-block bound on |delta_gpu - delta_numpy| (dB).  ``band`` / ``noise``: inclusive bin
    ranges ((0, -1) when empty); ``window``: the L window values used; ``xmax``: max |x|."""
    s = float(xmax) * float(np.abs(np.asarray(window, dtype=np.float64)[:L]).sum())
    nb = max(0, band[1] - band[0] + 1)
    nn = max(0, noise[1] - noise[0] + 1)
    bins = np.concatenate([np.arange(band[0], band[1] + 1), np.arange(noise[0], noise[1] + 1)])
    dx = _chain(nfft, L, bins) * U * s
    return band_db_error(band_db, nb, dx) + band_db_error(noise_db, nn, dx)


def decision_bound(delta_err: np.ndarray, k_std: float) -> float:
    """|delta - thr| at or below this can flip a decision (module docstring)."""
    m = float(np.max(delta_err)) if np.size(delta_err) else 0.0
    return (2.0 + abs(float(k_std))) * m * (1.0 + 1e-6)


def check(min_margin: float, bound: float, what: str = "") -> bool:
    """True (and a NearTieWarning) when the smallest decision margin is within the bound."""
    near = bool(np.isfinite(min_margin)) and min_margin <= bound
    if near:
        warnings.warn(NearTieWarning(f"{what}decision margin {min_margin:.3e} dB is within the delta error "
                                     f"bound {bound:.3e} dB: a detection boundary may differ from the "
                                     f"float64 numpy reference"), stacklevel=3)
    return near

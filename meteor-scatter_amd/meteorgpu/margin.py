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
  the recurrence's error gain at bin angle theta, 24 for the rotations and the 16-lane sum), or,
  for int16 blocks on the exact integer path (csrc/block_i8.hip), ``10.25 L / sum(w)`` (its
  coefficients' 2^-55 quantisation is absolute, not relative to the window) -- the larger of
  the two;
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

The live detector (processor.py:206, :349-412) gets the same guard (``live_*`` below): its band
powers are scipy's Welch PSD (pocketfft over each detrended, windowed segment zero-padded to
nfft; segments averaged) against the device's float64 Goertzel over the segment
(csrc/live.hip welch_bands_kernel, one lane per bin over all nperseg samples).  The detrended
and windowed samples are bit-identical on both sides (numpy's pairwise mean is reproduced), so
only the transform differs:

* per segment and bin |dX| <= (c_fft + c_goertzel) u S, S = sum |w (x - mean)| <= span sum w with
  span = max x - min x over the block (a constant block is exactly 0 on both sides),
  c_fft = 4 log2(nfft) + 10 (the FFT, the detrend and the window), c_goertzel = 3 nperseg G + 24;
  int16 samples on the matrix cores (csrc/welch_i8.hip: the detrend folded into int8-digit
  coefficients) replace c_goertzel u S by 18 u nperseg max|x| -- the larger of the two is taken;
* a band energy E = scale / nseg * sum_s sum_k c_k |X_sk|^2 (c_k = 2 off DC / Nyquist) moves by
  at most dE = 2 dX sqrt(C scale E) + C scale dX^2 + (n + nseg + 10) u E, C = 2n (Cauchy-Schwarz
  over the n bins and nseg segments);
* the over-noise value sig_dB - mean(noise1_dB, noise2_dB) (processor.py:391) by
  e_sig + (e_n1 + e_n2) / 2 plus its own rounding;
* the history threshold mean + k std of the previous W values (:397-402), held while tracking or
  locked (:404-410), by (1 + k) max e plus rounding, so a decision (``db2 > thr`` :464,
  ``db2 < thr`` :478) can only flip where |db2 - thr| <= (2 + k) max e.
"""
from __future__ import annotations

import math
import warnings

import numpy as np

U = 2.0 ** -53
DB = 10.0 / math.log(10.0)


class NearTieWarning(UserWarning):
    """A detection decision lies within the delta error bound of its threshold."""


def _goertzel_chain(l_seg: int, bins, nfft: int) -> float:
    """3 L G + 24: a Goertzel recurrence over l_seg samples at the bins' angles (G = the error
    gain min(1/|sin theta|, l_seg)), its rotation and the lane sums."""
    theta = 2.0 * np.pi * np.asarray(bins, dtype=np.float64) / float(nfft)
    s = np.abs(np.sin(theta))
    gain = np.minimum(np.where(s > 0, 1.0 / np.maximum(s, 1e-300), np.inf), float(l_seg))
    g = float(gain.max()) if gain.size else 1.0
    return 3.0 * l_seg * g + 24.0


def _i8_chain(L: int, nbins: int, wsum: float) -> float:
    """The int16 blocks' exact integer DFT (csrc/block_i8.hip), where it applies (L = 256, 512 or
    1024, 1-8 bins): each coefficient w_n cos / sin is quantised to 2^-55 = u / 4 absolute and the
    float64 digit combination (7 digit terms) adds < 10 u of sum |x|, so |dX| <= 10.25 u sum|x| <=
    10.25 u L max|x| = (10.25 L / sum w) u S.  0 where the path does not apply."""
    if int(L) not in (256, 512, 1024) or not 1 <= int(nbins) <= 8:
        return 0.0
    return 10.25 * float(L) / wsum if wsum > 0 else 0.0  # sum w = 0: every coefficient is 0, X = 0


def _chain(nfft: int, L: int, bins: np.ndarray, wsum: float) -> float:
    """c: longest rounding chain of a bin (pocketfft + the device's transform: the Goertzel
    segments or, for int16 blocks of the int8 path's shapes, its quantisation -- the larger, so
    the bound holds whichever path ran)."""
    l_seg = max(1, -(-int(L) // 16))  # samples per lane: the block_delta kernel's 16 lanes
    dev = max(_goertzel_chain(l_seg, bins, nfft), _i8_chain(L, len(bins), wsum))
    return 4.0 * math.log2(nfft) + 8.0 + dev


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
    wsum = float(np.abs(np.asarray(window, dtype=np.float64)[:L]).sum())
    s = float(xmax) * wsum
    nb = max(0, band[1] - band[0] + 1)
    nn = max(0, noise[1] - noise[0] + 1)
    bins = np.concatenate([np.arange(band[0], band[1] + 1), np.arange(noise[0], noise[1] + 1)])
    dx = _chain(nfft, L, bins, wsum) * U * s
    return band_db_error(band_db, nb, dx) + band_db_error(noise_db, nn, dx)


def delta_error_bounds(band_db: np.ndarray, noise_db: np.ndarray, *, nfft: int, L: int, window: np.ndarray,
                       xmax: np.ndarray, band: tuple[int, int], noise: tuple[int, int]) -> np.ndarray:
    """delta_error_bound for many files at once: band_db / noise_db [files, blocks], xmax [files]
    (one vectorised pass instead of a Python loop over the files of a batch)."""
    wsum = float(np.abs(np.asarray(window, dtype=np.float64)[:L]).sum())
    nb = max(0, band[1] - band[0] + 1)
    nn = max(0, noise[1] - noise[0] + 1)
    bins = np.concatenate([np.arange(band[0], band[1] + 1), np.arange(noise[0], noise[1] + 1)])
    s = np.asarray(xmax, dtype=np.float64).reshape(-1, 1) * wsum
    dx = _chain(nfft, L, bins, wsum) * U * s
    return band_db_error(band_db, nb, dx) + band_db_error(noise_db, nn, dx)


def decision_bounds(delta_err: np.ndarray, k_std: float) -> np.ndarray:
    """decision_bound of each row of delta_err [files, blocks]."""
    e = np.asarray(delta_err, dtype=np.float64)
    m = e.max(axis=1) if e.shape[1] else np.zeros(e.shape[0])
    return (2.0 + abs(float(k_std))) * m * (1.0 + 1e-6)


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


# ------------------------------------------------------------------ live detector (module doc)
def welch_band_db_error(e_db: np.ndarray, nbins: int, dx, scale: float, nseg: int) -> np.ndarray:
    """Per-block bound on |10 log10 E_gpu - 10 log10 E_scipy| for a Welch band energy of nbins
    bins averaged over nseg segments (dx: the per-segment, per-bin transform bound, per block)."""
    e_db = np.asarray(e_db, dtype=np.float64)
    dx = np.broadcast_to(np.asarray(dx, dtype=np.float64), e_db.shape)
    if nbins <= 0:
        return np.zeros_like(e_db)
    e = np.power(10.0, e_db / 10.0)
    c = 2.0 * nbins
    de = 2.0 * dx * np.sqrt(c * scale * e) + c * scale * dx * dx + (nbins + nseg + 10) * U * e
    with np.errstate(divide="ignore", invalid="ignore", over="ignore"):
        r = de / e
        out = np.where(r < 1.0, DB * r / (1.0 - r) + 4.0 * U * (np.abs(e_db) + 1.0), np.inf)
    # a band with no power at all: exactly 0 on both sides when the samples are (dx == 0)
    return np.where(e > 0, out, np.where(dx == 0, 0.0, np.inf))


def block_span(x: np.ndarray, block_size: int, sample_scale: float = 1.0) -> np.ndarray:
    """max - min of each whole processing block's samples, times the sample scale."""
    x = np.asarray(x)
    nb = len(x) // block_size if block_size > 0 else 0
    if nb == 0:
        return np.zeros(0)
    v = x[: nb * block_size].reshape(nb, block_size)
    return (v.max(axis=1).astype(np.float64) - v.min(axis=1).astype(np.float64)) * abs(float(sample_scale))


def block_absmax(x: np.ndarray, block_size: int, sample_scale: float = 1.0) -> np.ndarray:
    """max |x| of each whole processing block's samples, times the sample scale."""
    x = np.asarray(x)
    nb = len(x) // block_size if block_size > 0 else 0
    if nb == 0:
        return np.zeros(0)
    v = np.abs(x[: nb * block_size].reshape(nb, block_size).astype(np.float64))
    return v.max(axis=1) * abs(float(sample_scale))


# the int16 Welch path on the matrix cores (csrc/welch_i8.hip): |dX| <= I8_WELCH u sum_n |x_n| per
# segment and bin.  Round 6's kernel needs about 5 u of it: the coefficients' zero-sum quantisation
# (|T - c' 2^53| < 1: u), the digit sum rounded once and the sample scale's product (u each of
# |X| <= 2 sum|x|); 18 is the bound of round 6's first form (rounded quantisation, a float64 Horner
# sum of 8 weights), kept
I8_WELCH = 18.0


def live_over_error(band_db: np.ndarray, *, block_size: int, nperseg: int, noverlap: int, nfft: int,
                    window: np.ndarray, span, bands, scale: float, absmax=None) -> np.ndarray:
    """Per-block bound on |db2_gpu - db2_scipy| (processor.py:391) from the device's band dB rows
    band_db [3][nb] (signal, noise 1, noise 2); ``bands``: their inclusive bin ranges, ``span``:
    max - min of each block's (scaled) samples (``block_span``), ``window``: the nperseg window.
    ``absmax`` (``block_absmax``, int16 input): the device may have taken the int8 path, whose error
    is relative to sum |x| rather than to the detrended samples; the bound then takes the larger of
    the two transforms' terms, so it holds whichever ran."""
    band_db = np.asarray(band_db, dtype=np.float64)
    step = nperseg - noverlap
    nseg = (block_size - nperseg) // step + 1
    s = np.asarray(span, dtype=np.float64) * float(np.abs(np.asarray(window, dtype=np.float64)).sum())
    bins = np.concatenate([np.arange(lo, hi + 1) for lo, hi in bands]) if bands else np.zeros(0)
    # scipy's side: pocketfft's chain plus the detrend and window roundings of its input
    dx = (4.0 * math.log2(nfft) + 10.0) * U * s
    dev = _goertzel_chain(nperseg, bins, nfft) * U * s
    if absmax is not None:
        dev = np.maximum(dev, I8_WELCH * U * float(nperseg) * np.asarray(absmax, dtype=np.float64))
    dx = dx + dev
    e = [welch_band_db_error(band_db[j], max(0, hi - lo + 1), dx, scale, nseg) for j, (lo, hi) in enumerate(bands)]
    with np.errstate(invalid="ignore"):
        rnd = 4.0 * U * (np.abs(band_db[0]) + np.abs(band_db[1]) + np.abs(band_db[2]))
        out = e[0] + 0.5 * (e[1] + e[2]) + np.where(np.isfinite(rnd), rnd, 0.0)
    return out


def live_decision_check(over: np.ndarray, thr: np.ndarray, over_err: np.ndarray, *, k_std: float, W: int,
                        first_block: int, what: str = "", warn: bool = True):
    """(near_tie, min_margin, bound) of one recording: the decisions are the blocks from
    ``first_block`` on (the first that can leave Init); min |db2 - thr| over those with finite
    values against (2 + k) max e plus the threshold's own rounding (W-element mean / std)."""
    over = np.asarray(over, dtype=np.float64)
    thr = np.asarray(thr, dtype=np.float64)
    sel = slice(max(0, int(first_block)), None)
    o, t = over[sel], thr[sel]
    ok = np.isfinite(o) & np.isfinite(t)
    m = float(np.min(np.abs(o[ok] - t[ok]))) if ok.any() else math.inf
    fin = over[np.isfinite(over)]
    big = float(np.max(np.abs(fin))) if fin.size else 0.0
    emax = float(np.max(over_err)) if np.size(over_err) else 0.0
    bound = (2.0 + abs(float(k_std))) * emax * (1.0 + 1e-6) + 8.0 * (W + 8) * U * big
    near = bool(np.isfinite(m)) and m <= bound
    if near and warn:
        warnings.warn(NearTieWarning(f"{what}decision margin {m:.3e} dB is within the over-noise error bound "
                                     f"{bound:.3e} dB: a meteor boundary may differ from the scipy reference"),
                      stacklevel=3)
    return near, m, bound

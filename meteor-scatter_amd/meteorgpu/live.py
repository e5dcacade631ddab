"""Drop-in for the reference's phase-2 live detector, dsp/src/live/backend/processor.py
(``wav_file_process``) with the dataclasses of dsp/src/live/backend/aggregates.py.

The per-block Welch PSD band powers (a8, processor.py:206 and :349-369) and the state
machine (a9, processor.py:391-507) run on the GPU through libmsdsp
(``msd_welch_bands*``, ``msd_live_detect*``); there is no CPU fallback.  The per-meteor
waterfall export (``ConfigSpecExport.output_dir``, processor.py:295-343) draws per-block Welch
PSD rows computed on the GPU (``msd_welch_psd``: only the rows the image shows, plus the
full rows of the initialisation blocks that set its colour range).  The live UI animation
(``enable_ui_plots``, an interactive matplotlib window) is not part of the drop-in: asking for
it raises ``NotImplementedError``.

Lower-level pieces: ``welch_band_db`` (band dB rows of one signal), ``live_detect`` (the
state machine over band dB rows), ``LiveBatch`` (many recordings resident in HBM).
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from . import _lib, margin, wav
from .dsp import context, hann_periodic


# ------------------------------------------------------------------ aggregates.py:4-74
@dataclass
class State:
    pass


@dataclass
class StateInitialization(State):
    history_channel_dB: list = field(default_factory=list)


@dataclass
class StateDetection(State):
    locked_threshold: float = -1.0
    use_locked_threshold_until_secs: float = -1.0


@dataclass
class StateTracking(State):
    locked_threshold: float
    time_start_detection: float
    history_over_noise_sig_dB: list


@dataclass
class Config:
    pass


@dataclass
class ConfigDetection(Config):
    proc_block_sec: float = 0.2
    n_fft: int = 4096
    signal_freq: int = 1000
    channel_width: int = 100
    noise_channel_offset: int = 300
    avg_win_sec: float = 8
    init_detection_wait_sec: float = 8 * 1.0
    after_tracking_wait_sec: float = 8 * 1.5
    threshold_std_factor: float = 4
    detection_db_over_noise_mean_min: float = -1
    detection_dur_min_sec: float = -1


@dataclass
class ConfigVisualization(Config):
    enable_ui_plots: bool = True
    realtime_factor: float = 16
    flag_realtime_animation: bool = True
    max_range_sec: int = 60
    limit_freq_offset_wf2_and_export: int = 100
    wf_offset_vmin: int = 20
    wf_offset_vmax: int = 20
    enable_debug_logs: bool = False


@dataclass
class ConfigSpecExport(Config):
    output_dir: str = ""
    time_before_meteor_sec: int = 3
    time_after_meteor_sec: int = 3


@dataclass
class DetectedMeteor:
    time_start: float
    time_stop: float
    duration: float
    db_min: float
    db_max: float
    db_mean: float
    db_std: float


class LiveMeteors(list):
    """``wav_file_process``'s meteors, with the near-tie guard's verdict (margin.py, live part):
    ``near_tie`` is True when a detector decision lies within the over-noise error bound of its
    threshold (a meteor boundary may then differ from the scipy reference; otherwise none can),
    ``min_margin`` = min |db2 - thr| over the decisions, ``decision_bound`` the bound."""
    near_tie: bool = False
    min_margin: float = float("inf")
    decision_bound: float = 0.0


# ------------------------------------------------------------------ configuration
def band_edges(cfg: ConfigDetection):
    """processor.py:32-45: [start, stop] in Hz of the signal band and the two noise bands."""
    half = cfg.channel_width / 2
    ms = (cfg.signal_freq - half, cfg.signal_freq + half)
    n1 = ((cfg.signal_freq - cfg.noise_channel_offset) - half, (cfg.signal_freq - cfg.noise_channel_offset) + half)
    n2 = ((cfg.signal_freq + cfg.noise_channel_offset) - half, (cfg.signal_freq + cfg.noise_channel_offset) + half)
    return ms, n1, n2


def _mask_bins(nfft: int, fs, lo: float, hi: float) -> tuple[int, int]:
    """Inclusive bin range of (freqs >= lo) & (freqs <= hi) over scipy's welch frequencies
    (sp_fft.rfftfreq(nfft, 1/fs)); (0, -1) when empty."""
    freqs = np.fft.rfftfreq(nfft, 1 / fs)
    idx = np.nonzero((freqs >= lo) & (freqs <= hi))[0]
    if idx.size == 0:
        return 0, -1
    assert idx[-1] - idx[0] + 1 == idx.size
    return int(idx[0]), int(idx[-1])


def welch_cfg(fs, cfg: ConfigDetection, sample_scale: float = 1.0):
    """scipy.signal.welch(block, fs, nfft=n_fft) defaults (window 'hann', nperseg 256 capped at
    the block length, noverlap nperseg//2) → (msd_welch_cfg, window)."""
    bs = int(cfg.proc_block_sec * fs)
    if bs < 1:
        raise ValueError("proc_block_sec * fs must give at least one sample per block")
    nperseg = 256 if bs >= 256 else bs
    noverlap = nperseg // 2
    nfft = int(cfg.n_fft)
    if nfft < nperseg:
        raise ValueError("nfft must be greater than or equal to nperseg.")  # scipy's message
    win = hann_periodic(nperseg)
    wc = win.astype(np.complex128)
    scale = np.real(1.0 / (fs * (wc * wc).sum()))  # scipy: win cast to the complex out dtype
    c = _lib.MsdWelchCfg()
    c.block_size, c.nperseg, c.noverlap, c.nfft = bs, nperseg, noverlap, nfft
    c.sample_scale = float(sample_scale)
    c.scale = float(scale)
    c.nbands = 3
    for j, (lo, hi) in enumerate(band_edges(cfg)):
        c.band_lo[j], c.band_hi[j] = _mask_bins(nfft, fs, lo, hi)
    return c, win


def live_cfg(fs, cfg: ConfigDetection) -> _lib.MsdLiveCfg:
    c = _lib.MsdLiveCfg()
    c.block_size = int(cfg.proc_block_sec * fs)
    c.avg_win_blocks = int(cfg.avg_win_sec / cfg.proc_block_sec)  # processor.py:58
    c.fs = float(fs)
    c.k_std = float(cfg.threshold_std_factor)
    c.init_wait_sec = float(cfg.init_detection_wait_sec)
    c.after_tracking_wait_sec = float(cfg.after_tracking_wait_sec)
    c.min_db_mean = float(cfg.detection_db_over_noise_mean_min)
    c.min_dur_sec = float(cfg.detection_dur_min_sec)
    return c


def _device_samples(data: np.ndarray):
    """Samples as the kernels take them + the factor that turns them into soundfile's float64
    (PCM16 / 32768, PCM32 and 24-bit-in-int32 / 2^31, 8-bit (x - 128) / 128)."""
    if data.dtype == np.int16:
        return data, 1.0 / 32768.0
    if data.dtype == np.int32:
        return data, 1.0 / 2147483648.0
    if data.dtype == np.uint8:
        return data.astype(np.int16) - 128, 1.0 / 128.0
    if data.dtype in (np.float32, np.float64):
        return data, 1.0
    raise TypeError(f"unsupported sample dtype {data.dtype}")


# ------------------------------------------------------------------ a8 / a9 entry points
def welch_band_db(x: np.ndarray, fs, config_detection: ConfigDetection, sample_scale: float = 1.0,
                  device: int = 0) -> np.ndarray:
    """Per-block (signal, noise 1, noise 2) dB, float64 [3][nb] (processor.py:206, :349-369)."""
    c, win = welch_cfg(fs, config_detection, sample_scale)
    plan = _lib.WelchPlan(context(device), c, win)
    try:
        return plan.run(np.ascontiguousarray(x))
    finally:
        plan.close()


def live_detect(band_db: np.ndarray, fs, config_detection: ConfigDetection, device: int = 0):
    """The state machine (processor.py:391-507): (list[DetectedMeteor], thresholds, over_noise)."""
    rows, thr, over = _lib.live_detect(context(device), band_db, live_cfg(fs, config_detection))
    mets = [DetectedMeteor(float(r["time_start"]), float(r["time_stop"]), float(r["duration"]), float(r["db_min"]),
                           float(r["db_max"]), float(r["db_mean"]), float(r["db_std"])) for r in rows]
    return mets, thr, over


def _first_decision_block(nb: int, fs, cfg: ConfigDetection) -> int:
    """the block at which Init ends (processor.py:452-455: block start >= the wait)"""
    bs = int(cfg.proc_block_sec * fs)
    for b in range(nb):
        if (b * bs) / fs >= cfg.init_detection_wait_sec:
            return b
    return nb


def near_tie_check(band_db: np.ndarray, thr: np.ndarray, over: np.ndarray, span: np.ndarray, fs,
                   cfg: ConfigDetection, what: str = "", warn: bool = True, absmax=None):
    """(near_tie, min_margin, bound) of one recording from the device's band dB rows, the
    thresholds used and the over-noise values (live_detect), and each block's sample span
    (margin.block_span); ``absmax`` (margin.block_absmax) for int16 samples, which may take the
    int8 path (csrc/welch_i8.hip); a NearTieWarning when near."""
    c, win = welch_cfg(fs, cfg)
    bands = [(int(c.band_lo[j]), int(c.band_hi[j])) for j in range(3)]
    err = margin.live_over_error(band_db, block_size=int(c.block_size), nperseg=int(c.nperseg),
                                 noverlap=int(c.noverlap), nfft=int(c.nfft), window=win, span=span, bands=bands,
                                 scale=float(c.scale), absmax=absmax)
    W = int(cfg.avg_win_sec / cfg.proc_block_sec)
    return margin.live_decision_check(over, thr, err, k_std=cfg.threshold_std_factor, W=W,
                                      first_block=_first_decision_block(len(over), fs, cfg), what=what, warn=warn)


def wav_file_process(wav_file_path: str,
                     config_detection: ConfigDetection,
                     config_visualization: ConfigVisualization,
                     config_spec_export: ConfigSpecExport,
                     wav_file_start_sec: float = 0,
                     wav_file_stop_sec: float = -1,
                     *,
                     required_sample_rate=4000,
                     device: int = 0):
    """GPU drop-in for processor.py:14-543 (same arguments, asserts and printed results).
    Returns the detected meteors as a ``LiveMeteors`` list (the reference returns None and only
    prints them) carrying the near-tie guard's verdict; a NearTieWarning when a decision lies
    within the error bound of the scipy reference."""
    assert os.path.exists(wav_file_path), f"File not found: {wav_file_path}"
    if config_spec_export.output_dir != "":
        assert os.path.exists(config_spec_export.output_dir), \
            f"Output Directory not found: {config_spec_export.output_dir}"
    if config_visualization.enable_ui_plots:
        raise NotImplementedError("the live UI animation (enable_ui_plots) is not part of the GPU drop-in; "
                                  "set enable_ui_plots=False (the spectrogram export, output_dir, is)")
    file_sample_rate, data = wav.read(wav_file_path)
    if required_sample_rate is not None:
        assert file_sample_rate == required_sample_rate, f"Invalid Sample Rate: {file_sample_rate}"
    start = int(wav_file_start_sec * file_sample_rate)
    if wav_file_stop_sec != -1:
        data = data[start:int(wav_file_stop_sec * file_sample_rate)]
    else:
        data = data[start:]
    if data.ndim > 1:
        print("WARNING: Multichannel file detected. Using first channel only.")
        data = data[:, 0]
    _print_config(config_detection, config_visualization)
    x, sample_scale = _device_samples(np.ascontiguousarray(data))
    block_size = int(config_detection.proc_block_sec * file_sample_rate)
    print()
    print("###############")
    print("Prepare Wav")
    print("###############")
    print("File Samplerate: ", file_sample_rate)
    print("File Blockgröße: ", block_size)
    print("File Dauer: ", len(x) / file_sample_rate)
    print()
    print("###############")
    print("Process Loop")
    print("###############")
    bdb = welch_band_db(x, file_sample_rate, config_detection, sample_scale, device)
    found, thr, over = live_detect(bdb, file_sample_rate, config_detection, device)
    meteors = LiveMeteors(found)
    span = margin.block_span(x, block_size, sample_scale)[: bdb.shape[1]]
    absmax = margin.block_absmax(x, block_size, sample_scale)[: bdb.shape[1]] if x.dtype == np.int16 else None
    meteors.near_tie, meteors.min_margin, meteors.decision_bound = near_tie_check(
        bdb, thr, over, span, file_sample_rate, config_detection, what=f"{wav_file_path}: ", absmax=absmax)
    for i, m in enumerate(meteors):
        print("Detected Meteor:", m, "Now Detected Meteors:", i + 1)
    not_exported = list(meteors)
    if config_spec_export.output_dir != "":
        _, not_exported = export_meteor_specs(x, sample_scale, file_sample_rate, bdb.shape[1], meteors,
                                              config_detection, config_visualization, config_spec_export, device)
    if len(not_exported) != 0:  # processor.py:539-543
        print("Detected Meteors not exported: ", len(not_exported))
        for t in not_exported:
            print(t)
    return meteors


def _print_config(cd: ConfigDetection, cv: ConfigVisualization):
    """processor.py:25-59: the band edges and window sizes it prints before processing."""
    (ms0, ms1), (n10, n11), (n20, n21) = band_edges(cd)
    print()
    print("###############")
    print("Init Config")
    print("###############")
    print("Freq MS Min: ", ms0)
    print("Freq MS Max: ", ms1)
    print("Freq Noise 1 Min: ", n10)
    print("Freq Noise 1 Max: ", n11)
    print("Freq Noise 2 Min: ", n20)
    print("Freq Noise 2 Max: ", n21)
    print("Waterfall Win Size: ", int(cv.max_range_sec / cd.proc_block_sec))
    print("Avg Win Size: ", int(cd.avg_win_sec / cd.proc_block_sec))


def block_psd_rows(x: np.ndarray, sample_scale: float, fs, cfg: ConfigDetection, b0: int, b1: int, k0: int, k1: int,
                   device: int = 0) -> np.ndarray:
    """Welch PSD of blocks [b0, b1), bins [k0, k1], float64 [b1-b0][k1-k0+1]: the rows of
    processor.py:206's ``welch(block, fs, nfft=n_fft)`` the waterfall image needs (GPU)."""
    c, win = welch_cfg(fs, cfg, sample_scale)
    c.nbands = 1
    c.band_lo[0], c.band_hi[0] = int(k0), int(k1)
    bs = int(c.block_size)
    plan = _lib.WelchPlan(context(device), c, win)
    try:
        return plan.psd(np.ascontiguousarray(x[b0 * bs: b1 * bs]), k1 - k0 + 1)
    finally:
        plan.close()


def export_meteor_specs(x: np.ndarray, sample_scale: float, fs, nb: int, meteors, cd: ConfigDetection,
                        cv: ConfigVisualization, ce: ConfigSpecExport, device: int = 0):
    """processor.py:295-343: each meteor is exported at the first block after the one that closed
    it whose waterfall window (the block-end times of the last max_range_sec / proc_block_sec
    blocks) contains [start - time_before, stop + time_after]; the image is that window's
    PSD rows in dB (imshow, colour range = the mean PSD dB of the initialisation blocks -
    wf_offset_vmin .. + wf_offset_vmax), cropped to those times and to signal_freq +-
    limit_freq_offset_wf2_and_export, saved as output_dir + spec_{start:.2f}_{stop:.2f}.jpg.
    Only the rows inside the crop (one more on each side) are computed: imshow with the
    matching sub-extent draws the same picture.  Returns (paths, meteors never exported)."""
    import matplotlib.pyplot as plt
    bs = int(cd.proc_block_sec * fs)
    W = int(cv.max_range_sec / cd.proc_block_sec)  # processor.py:57
    nfft = int(cd.n_fft)
    K = nfft // 2 + 1
    freqs = np.fft.rfftfreq(nfft, 1 / fs)
    end = lambda b: (b * bs + bs) / fs  # noqa: E731  block_end_elapsed_sec
    start_of = lambda b: (b * bs) / fs  # noqa: E731
    # the block that ends the initialisation (processor.py:452-455) and the colour range
    b_init = next((b for b in range(nb) if start_of(b) >= cd.init_detection_wait_sec), None)
    mean_init = None
    if b_init is not None:
        full = block_psd_rows(x, sample_scale, fs, cd, 0, b_init + 1, 0, K - 1, device)
        with np.errstate(divide="ignore"):
            mean_init = np.mean([np.mean(10 * np.log10(r)) for r in full])
    lo_f = cd.signal_freq - cv.limit_freq_offset_wf2_and_export
    hi_f = cd.signal_freq + cv.limit_freq_offset_wf2_and_export
    h = (freqs[-1] - freqs[0]) / K  # imshow row height of the full image
    k0 = max(0, int(np.floor((lo_f - freqs[0]) / h)) - 1)
    k1 = min(K - 1, int(np.ceil((hi_f - freqs[0]) / h)) + 1)
    ms0, ms1 = band_edges(cd)[0]
    paths, pending = [], []
    for m in meteors:
        c = int(round(m.time_stop * fs / bs))  # the block that closed the meteor
        t_sim0 = m.time_start - ce.time_before_meteor_sec
        t_sim1 = m.time_stop + ce.time_after_meteor_sec
        exp_b = None
        for b in range(c + 1, nb):
            w0 = end(max(0, b - W + 1))
            if w0 > t_sim0:
                break  # the window start only moves later
            if w0 <= t_sim0 <= end(b) and w0 <= t_sim1 <= end(b):
                exp_b = b
                break
        if exp_b is None:
            pending.append(m)
            continue
        b0 = max(0, exp_b - W + 1)
        with np.errstate(divide="ignore"):
            rows = 10 * np.log10(block_psd_rows(x, sample_scale, fs, cd, b0, exp_b + 1, k0, k1, device))
        vmin = vmax = None
        if mean_init is not None and b_init is not None and exp_b > b_init:
            vmin, vmax = mean_init - cv.wf_offset_vmin, mean_init + cv.wf_offset_vmax
        fig = plt.figure(figsize=(10, 5))
        plt.imshow(rows.T, aspect="auto", cmap="viridis", origin="lower",
                   extent=[end(b0), end(exp_b), freqs[0] + k0 * h, freqs[0] + (k1 + 1) * h], vmin=vmin, vmax=vmax)
        plt.xlim(t_sim0, t_sim1)
        plt.ylim(lo_f, hi_f)
        plt.xlabel("Time [s]")
        plt.ylabel("Frequency [Hz]")
        plt.title(f"Detection {m.time_start:.2f}-{m.time_stop:.2f}sec (d={m.duration:.2f}sec)\n"
                  + f"Min={m.db_min:.2f}dB, Max={m.db_max:.2f}dB, Mean={m.db_mean:.2f}dB, Std={m.db_std:.2f}dB")
        plt.axvline(m.time_start, color="grey", linestyle="--")
        plt.axvline(m.time_stop, color="grey", linestyle="--")
        plt.axhline(ms0, color="grey", linestyle="--")
        plt.axhline(ms1, color="grey", linestyle="--")
        path = ce.output_dir + f"spec_{m.time_start:.2f}_{m.time_stop:.2f}.jpg"
        plt.savefig(path, bbox_inches="tight", pad_inches=0)
        plt.close(fig)
        paths.append(path)
    return paths, pending


# ------------------------------------------------------------------ batch (device-resident)
class LiveBatch:
    """Many equal-format recordings resident in HBM: one Welch launch + one detector launch.

    HBM: x [nfiles][n_pad] samples, band_db [nfiles][3][ld], over / thr [nfiles][ld],
    meteors [nfiles][cap]."""

    def __init__(self, ctx: _lib.Context, nfiles: int, n_per_file: int, fs, cfg: ConfigDetection,
                 dtype=np.int16, sample_scale: float = 1.0 / 32768.0, cap: int = 1024):
        self.ctx, self.nfiles, self.n, self.fs = ctx, int(nfiles), int(n_per_file), fs
        self.dtype = np.dtype(dtype)
        wc, win = welch_cfg(fs, cfg, sample_scale)
        self.plan = _lib.WelchPlan(ctx, wc, win)
        self.lcfg = live_cfg(fs, cfg)
        self.nb = self.plan.blocks(self.n)
        self.ld = max(1, self.nb)
        self.cap = int(cap)
        es = self.dtype.itemsize
        self.n_pad = (self.n + 7) // 8 * 8
        F = self.nfiles
        self.d_x = ctx.alloc(F * self.n_pad * es)
        self.d_off = ctx.alloc(F * 8)
        self.d_len = ctx.alloc(F * 8)
        self.d_nb = ctx.alloc(F * 8)
        self.d_off.upload(np.arange(F, dtype=np.int64) * self.n_pad)
        self.d_len.upload(np.full(F, self.n, np.int64))
        self.d_nb.upload(np.full(F, self.nb, np.int64))
        self.d_band = ctx.alloc(F * 3 * self.ld * 8)
        self.d_over = ctx.alloc(F * self.ld * 8)
        self.d_thr = ctx.alloc(F * self.ld * 8)
        self.d_met = ctx.alloc(F * self.cap * _lib.METEOR_DTYPE.itemsize)
        self.d_counts = ctx.alloc(F * 8)
        self.d_status = ctx.alloc(F * 4)
        self.cfg = cfg
        self.sample_scale = float(sample_scale)
        self.span = np.zeros((F, self.nb))  # per-block sample span, for the near-tie guard
        # per-block max |x| of int16 recordings (the int8 path's error term, margin.live_over_error)
        self.absmax = np.zeros((F, self.nb)) if self.dtype == np.int16 else None
        self.near_tie = np.zeros(F, bool)
        self.min_margins = np.full(F, np.inf)
        self.decision_bounds = np.zeros(F)

    def close(self):
        """free the batch's device buffers and plan (the context stays)"""
        if getattr(self, "plan", None) is None:
            return
        self.ctx.synchronize()
        for b in (self.d_x, self.d_off, self.d_len, self.d_nb, self.d_band, self.d_over, self.d_thr, self.d_met,
                  self.d_counts, self.d_status):
            b.free()
        self.plan.close()
        self.plan = None

    def upload_file(self, i: int, x: np.ndarray):
        x = np.ascontiguousarray(x, dtype=self.dtype)
        if x.shape != (self.n,):
            raise ValueError("file length differs from the batch's")
        self.span[i] = margin.block_span(x, int(self.lcfg.block_size), self.sample_scale)[: self.nb]
        if self.absmax is not None:
            self.absmax[i] = margin.block_absmax(x, int(self.lcfg.block_size), self.sample_scale)[: self.nb]
        self.d_x.upload(x, byte_offset=i * self.n_pad * self.dtype.itemsize)

    def run(self):
        lib, h = self.ctx.lib, self.ctx.h
        self.plan.run_dev(self.d_x, self.dtype, self.d_off, self.d_len, self.nfiles, self.nb, self.d_band, self.ld)
        _lib.check(lib.msd_live_detect_dev(h, self.d_band.ptr, self.d_nb.ptr, self.nfiles, self.ld, self.lcfg,
                                           self.d_met.ptr, self.cap, self.d_counts.ptr, self.d_thr.ptr,
                                           self.d_over.ptr, self.d_status.ptr))

    def band_db(self) -> np.ndarray:
        out = np.empty((self.nfiles, 3, self.ld), np.float64)
        self.d_band.download(out)
        return out[:, :, : self.nb]

    def meteors(self):
        counts = np.empty(self.nfiles, np.int64)
        self.d_counts.download(counts)
        rows = np.empty((self.nfiles, self.cap), _lib.METEOR_DTYPE)
        self.d_met.download(rows)
        return [rows[i, : min(counts[i], self.cap)] for i in range(self.nfiles)], counts

    def thresholds(self) -> np.ndarray:
        out = np.empty((self.nfiles, self.ld), np.float64)
        self.d_thr.download(out)
        return out[:, : self.nb]

    def over_noise(self) -> np.ndarray:
        out = np.empty((self.nfiles, self.ld), np.float64)
        self.d_over.download(out)
        return out[:, : self.nb]

    def check_near_ties(self, warn: bool = True) -> np.ndarray:
        """The near-tie guard per recording (``near_tie_check``): sets ``near_tie``,
        ``min_margins`` and ``decision_bounds``; one NearTieWarning naming the flagged files."""
        bdb, thr, over = self.band_db(), self.thresholds(), self.over_noise()
        for i in range(self.nfiles):
            self.near_tie[i], self.min_margins[i], self.decision_bounds[i] = near_tie_check(
                bdb[i], thr[i], over[i], self.span[i], self.fs, self.cfg, warn=False,
                absmax=None if self.absmax is None else self.absmax[i])
        if warn and self.near_tie.any():
            import warnings
            idx = np.nonzero(self.near_tie)[0]
            warnings.warn(margin.NearTieWarning(
                f"{idx.size} file(s) {idx.tolist()[:10]} have a decision within the over-noise error bound of "
                f"their threshold: a meteor boundary may differ from the scipy reference"), stacklevel=2)
        return self.near_tie


def welch_psd(x, fs, nperseg=256, noverlap=None, nfft=None, sample_scale: float = 1.0, device: int = 0):
    """scipy.signal.welch(x, fs, window='hann', nperseg, noverlap, nfft, scaling='density') over a
    whole 1-D signal on the GPU (float64 arithmetic): returns (f, Pxx[nfft//2 + 1]).  As scipy
    does, nperseg is capped at len(x)."""
    x = np.ascontiguousarray(x)
    n = x.shape[0]
    if n == 0:
        return np.empty(0), np.empty(0)
    nperseg = min(int(nperseg), n)
    noverlap = nperseg // 2 if noverlap is None else int(noverlap)
    nfft = nperseg if nfft is None else int(nfft)
    if nfft < nperseg:
        raise ValueError("nfft must be greater than or equal to nperseg.")
    win = hann_periodic(nperseg)
    wc = win.astype(np.complex128)
    c = _lib.MsdWelchCfg()
    c.block_size, c.nperseg, c.noverlap, c.nfft = n, nperseg, noverlap, nfft
    c.sample_scale = float(sample_scale)
    c.scale = float(np.real(1.0 / (fs * (wc * wc).sum())))
    c.nbands = 1
    c.band_lo[0], c.band_hi[0] = 0, nfft // 2
    plan = _lib.WelchPlan(context(device), c, win)
    try:
        P = plan.psd(x if x.dtype != np.uint8 else x.astype(np.int16) - 128, nfft // 2 + 1)[0]
    finally:
        plan.close()
    return np.fft.rfftfreq(nfft, 1 / fs), P

"""GPU: the reference's own drivers run unchanged on the drop-in, figures included.

* ``mb_files`` (dsp/src/main.py:828-899): proc_wav_file with exactly its keyword arguments
  (debug_plot_output=True, adaptive threshold, gqrx file-name date);
* ``tl_files`` (main.py:905-946): debug_plot_config=True and debug_plot_output=True, k = 3.5,
  the BRAMS MESZ file-name date shifted to UTC;
* the remaining switches (debug_plot_whole: the 4096-point whole-file spectrogram,
  main.py:278-306; debug_plot_output_interactive: the plotly figures, :567-624);
* ``live/main.py:22-69``: wav_file_process with both of its configurations, exporting the
  per-meteor waterfall images (processor.py:295-343).

Synthetic WAVs under the Agg backend; the detections must equal the oracle's, the figures
must exist (``figure_dir``: the reference only shows its debug figures), and the waterfall
rows the export draws must equal scipy's Welch PSD per block."""
import datetime
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MB_NAME = "expoFull_gqrx_20250625_075141_49969000.wav"
TL_NAME = "expoFull_Brams_250607_23MESZ.wav"


@pytest.fixture(autouse=True)
def _agg():
    import matplotlib
    matplotlib.use("Agg")


def _wav6k(path, seed, f0, seconds=300.0):
    from meteorgpu import synth, wav
    x, _ = synth.synth_real(seed=seed, fs=6000, duration_s=seconds, f0=f0, band_hz=20.0, rate_per_min=6,
                            snr_db=(15, 35), dur_s=(0.4, 3.0))
    wav.write(path, 6000, x)
    return x


def _mb_date(file_path):  # main.py:858-863
    d = file_path.split("/")[-1].split("_")
    assert len(d) == 5
    return datetime.datetime.strptime(d[2] + "-" + d[3], "%Y%m%d-%H%M%S")


def _tl_date(file_path):  # main.py:917-923
    d = file_path.split("/")[-1].split("_")
    assert len(d) == 4
    d = (d[2] + "-" + d[3]).replace("MESZ.wav", "")
    return datetime.datetime.strptime(d, "%y%m%d-%H") - datetime.timedelta(hours=2)


def _same_as_oracle(res, x, fs, band, noise, n_fft, k, date):
    from oracle import dsp_oracle as O
    want, thr, *_ = O.proc_samples_ref(x, fs, 0.2, band, noise, n_fft, k, wav_start_date_time=date)
    assert len(want) > 0
    assert [(d.t_start, d.t_stop, d.utc_start, d.utc_stop) for d in res.detections] == \
           [(w[0], w[1], w[4], w[5]) for w in want]
    np.testing.assert_allclose([d.dB for d in res.detections], [w[3] for w in want], rtol=0, atol=1e-9)
    assert not res.near_tie


def test_mb_files_unchanged(tmp_path):
    from meteorgpu import dsp
    p = str(tmp_path / MB_NAME)
    x = _wav6k(p, 11, 1003.0)
    nf_freq, noise_freq, bandwidth = 1000 + 3, 700, 10
    figs = tmp_path / "figs"
    figs.mkdir()
    res = dsp.proc_wav_file(
        p, block_duration_sec=0.2, freq_band=(nf_freq - bandwidth, nf_freq + bandwidth),
        noise_band=(noise_freq - bandwidth, noise_freq + bandwidth), n_fft=512, debug_plot_whole=False,
        debug_plot_config=False, debug_plot_output=True, debug_plot_output_interactive=False, threshold_std_factor=4,
        wav_start_date_time=_mb_date(p), disable_show_and_write=True, flag_adaptive_threshold=True,
        threshold_estimation_window_sec=120, threshold_freeze_before_detection_sec=3,
        threshold_freeze_after_detection_sec=20, threshold_fixed_init_duration_sec=10, figure_dir=str(figs))
    _same_as_oracle(res, x, 6000, (993, 1013), (690, 710), 512, 4, _mb_date(p))
    for name in ("output_delta", "output_hist_duration", "output_hist_db", "output_time_map"):
        assert (figs / f"{name}.png").stat().st_size > 1000, name


def test_tl_files_unchanged(tmp_path):
    from meteorgpu import dsp
    p = str(tmp_path / TL_NAME)
    x = _wav6k(p, 12, 1006.0)
    nf_freq, noise_freq, bandwidth = 1000 + 6, 950, 10
    figs = tmp_path / "figs"
    figs.mkdir()
    res = dsp.proc_wav_file(
        p, block_duration_sec=0.2, freq_band=(nf_freq - bandwidth, nf_freq + bandwidth),
        noise_band=(noise_freq - bandwidth, noise_freq + bandwidth), n_fft=512, debug_plot_whole=False,
        debug_plot_config=True, debug_plot_output=True, debug_plot_output_interactive=False,
        threshold_std_factor=3.5, wav_start_date_time=_tl_date(p), disable_show_and_write=True,
        flag_adaptive_threshold=True, threshold_estimation_window_sec=120, threshold_freeze_before_detection_sec=3,
        threshold_freeze_after_detection_sec=20, threshold_fixed_init_duration_sec=10, figure_dir=str(figs))
    _same_as_oracle(res, x, 6000, (996, 1016), (940, 960), 512, 3.5, _tl_date(p))
    for name in ("config_psd_power_band", "config_psd_noise_band", "output_delta", "output_time_map"):
        assert (figs / f"{name}.png").stat().st_size > 1000, name


def test_whole_file_and_interactive_figures(tmp_path):
    pytest.importorskip("plotly")
    from meteorgpu import dsp
    p = str(tmp_path / MB_NAME)
    x = _wav6k(p, 13, 1003.0, seconds=180.0)
    figs = tmp_path / "figs"
    figs.mkdir()
    out = tmp_path / "exp"
    out.mkdir()
    res = dsp.proc_wav_file(p, 0.2, (993, 1013), (690, 710), 512, 4, debug_plot_whole=True,
                            debug_plot_output_interactive=True, wav_start_date_time=_mb_date(p),
                            disable_show_and_write=False, outfile_path=str(out) + "/", figure_dir=str(figs),
                            out_csv_file=str(tmp_path / "d.csv"))
    _same_as_oracle(res, x, 6000, (993, 1013), (690, 710), 512, 4, _mb_date(p))
    for name in ("whole_spec_power_band", "whole_spec_noise_band"):
        assert (figs / f"{name}.png").stat().st_size > 1000, name
    for name in ("interactive_band_power", "interactive_delta"):
        assert (figs / f"{name}.html").stat().st_size > 1000, name
    pngs = [f for d in out.iterdir() for f in d.iterdir()]  # outfile_path/<timestamp>/spec_and_psd_*.png
    assert len(pngs) == len(res.detections)
    import csv

    from oracle import dsp_oracle as O
    want, *_ = O.proc_samples_ref(x, 6000, 0.2, (993, 1013), (690, 710), 512, 4, wav_start_date_time=_mb_date(p))
    ref_csv = tmp_path / "ref.csv"
    O.write_csv_ref(want, str(ref_csv))
    rows = list(csv.reader(open(tmp_path / "d.csv", newline="")))
    rrows = list(csv.reader(open(ref_csv, newline="")))
    assert len(rows) == len(rrows) > 1 and rows[0] == rrows[0]
    for a, b in zip(rows[1:], rrows[1:]):  # t, dur and UTC columns string-equal; dB within 1e-9
        assert a[:3] + a[4:] == b[:3] + b[4:]
        assert abs(float(a[3]) - float(b[3])) <= 1e-9


# ------------------------------------------------------------------ live/main.py
LIVE_CONFIGS = [  # live/main.py:22-42 and :44-69
    dict(signal_freq=1020, wf_offset_vmin=0, wf_offset_vmax=25),
    dict(signal_freq=1025, wf_offset_vmin=-10, wf_offset_vmax=35),
]


def _export_blocks_ref(meteors, nb, bs, fs, W, before, after):
    """processor.py:295-343's bookkeeping, block by block: which meteors get exported (a meteor
    becomes a candidate after the block that closed it)."""
    pending, exported = [], []
    closing = {int(round(m.time_stop * fs / bs)): [] for m in meteors}
    for m in meteors:
        closing[int(round(m.time_stop * fs / bs))].append(m)
    ends = []
    for b in range(nb):
        ends.append((b * bs + bs) / fs)
        ends = ends[-W:]
        w0, w1 = ends[0], ends[-1]
        for m in list(pending):
            s0, s1 = m.time_start - before, m.time_stop + after
            if w0 <= s0 <= w1 and w0 <= s1 <= w1:
                exported.append(m)
                pending.remove(m)
        pending.extend(closing.get(b, []))
    return exported, pending


@pytest.mark.parametrize("cfg", LIVE_CONFIGS, ids=["test_my_file", "test_sonneberg"])
def test_live_main_unchanged(tmp_path, cfg, capsys):
    from meteorgpu import live as LV
    from meteorgpu import synth, wav
    from oracle import live_oracle as L
    x, _ = synth.synth_real(seed=31 + cfg["signal_freq"], fs=4000, duration_s=240.0, f0=float(cfg["signal_freq"]),
                            sigma=300.0, rate_per_min=8, band_hz=100.0, snr_db=(15, 30), dur_s=(0.5, 3.0))
    p = tmp_path / "gqrx_20241213_171350_49969000_sampled.wav"
    wav.write(p, 4000, x)
    out_dir = tmp_path / "spec_export" / "test_my_file"
    out_dir.mkdir(parents=True)
    cd = LV.ConfigDetection(proc_block_sec=0.20, n_fft=4096, detection_db_over_noise_mean_min=1,
                            detection_dur_min_sec=0.5, signal_freq=cfg["signal_freq"])
    cv = LV.ConfigVisualization(enable_ui_plots=False, wf_offset_vmin=cfg["wf_offset_vmin"],
                                wf_offset_vmax=cfg["wf_offset_vmax"], max_range_sec=60)
    ce = LV.ConfigSpecExport(output_dir=str(out_dir) + "/")
    got = LV.wav_file_process(wav_file_path=str(p), config_detection=cd, config_visualization=cv,
                              config_spec_export=ce)
    ref, _, _ = L.wav_file_process_ref(x.astype(np.float64) / 32768.0, 4000,
                                       L.ConfigDetectionRef(**{k: getattr(cd, k)
                                                               for k in L.ConfigDetectionRef.__dataclass_fields__}))
    assert len(ref) > 1 and [(m.time_start, m.time_stop) for m in got] == [(m.time_start, m.time_stop) for m in ref]
    nb = len(x) // 800
    exported, pending = _export_blocks_ref(got, nb, 800, 4000, 300, 3, 3)
    files = sorted(f.name for f in out_dir.iterdir())
    assert files == sorted(f"spec_{m.time_start:.2f}_{m.time_stop:.2f}.jpg" for m in exported)
    assert len(exported) > 0
    if pending:
        assert f"Detected Meteors not exported:  {len(pending)}" in capsys.readouterr().out


def test_waterfall_rows_match_scipy():
    """the PSD rows the export draws (GPU, only the bins inside the image) vs scipy's welch of
    each block (processor.py:206)"""
    from scipy.signal import welch

    from meteorgpu import live as LV
    from meteorgpu import synth
    x, _ = synth.synth_real(seed=5, fs=4000, duration_s=20.0, f0=1020.0, sigma=300.0, rate_per_min=20)
    cd = LV.ConfigDetection(signal_freq=1020)
    rows = LV.block_psd_rows(x, 1 / 32768, 4000, cd, 10, 40, 900, 1200)
    xf = x.astype(np.float64) / 32768
    for j, b in enumerate(range(10, 40)):
        _, P = welch(xf[b * 800:(b + 1) * 800], 4000, nfft=4096)
        np.testing.assert_allclose(10 * np.log10(rows[j]), 10 * np.log10(P[900:1201]), rtol=0, atol=1e-9)

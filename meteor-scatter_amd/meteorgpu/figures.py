"""The reference's figures, drawn from GPU arrays:

* the per-detection spectrogram + PSD export of proc_wav_file (``disable_show_and_write=False``,
  dsp/src/main.py:721-806, layout of internal_print_spec_and_psd_mod, main.py:40-116);
* the whole-file debug figures of proc_wav_file: ``debug_plot_whole`` (internal_print_spec,
  main.py:119-171, called at :278-306 with n_fft = 4096), ``debug_plot_config``
  (internal_print_psd, main.py:174-205, called at :324-350), ``debug_plot_output`` (the delta /
  threshold plot, :531-565, the duration and dB histograms, :660-685, the per-hour map,
  :687-716) and ``debug_plot_output_interactive`` (the plotly figures, :567-624);
* the live processor's per-meteor waterfall export (processor.py:295-343), in live.py.

The arrays come from the GPU (``dsp.spectrogram``, ``live.welch_psd``, the detector outputs);
matplotlib / plotly only draw them.  As in the reference a figure is shown with plt.show()
(a no-op under a non-interactive backend such as Agg); ``figure_dir`` additionally saves each
one (PNG, or HTML for plotly) for headless runs.  No parity is claimed beyond the arrays (the
figures themselves are not compared)."""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np


@dataclass
class Marker:
    """main.py's Marker (colour + optional frequency / time lines)."""
    color: str = "red"
    f_min: float | None = None
    f_max: float | None = None
    t_min: float | None = None
    t_max: float | None = None


def spec_and_psd(wav_data, fs, n_fft, eps=1e-10, freq_min=None, freq_max=None, markers=None, title=None,
                 filepath=None, device: int = 0):
    """Spectrogram (nperseg = n_fft, hop n_fft/2, dB) beside the 4096-point Welch PSD (dB),
    band-limited to [freq_min, freq_max]; saved to ``filepath`` (or shown)."""
    import matplotlib
    import matplotlib.pyplot as plt
    from matplotlib.gridspec import GridSpec

    from .dsp import spectrogram
    from .live import welch_psd

    x = np.asarray(wav_data)
    f, t, S = spectrogram(x, fs=fs, nperseg=n_fft, noverlap=n_fft // 2, nfft=n_fft, device=device)
    f_psd, P = welch_psd(x, fs, nperseg=4096, noverlap=2048, nfft=4096, device=device)
    if freq_min is not None and freq_max is not None:
        m = (f >= freq_min) & (f <= freq_max)
        f, S = f[m], S[m, :]
        mp = (f_psd >= freq_min) & (f_psd <= freq_max)
        f_psd, P = f_psd[mp], P[mp]
    fig = plt.figure(figsize=(14, 5))
    gs = GridSpec(1, 2, width_ratios=[7, 3], figure=fig)
    ax_s, ax_p = fig.add_subplot(gs[0, 0]), fig.add_subplot(gs[0, 1])
    if S.size:
        im = ax_s.pcolormesh(t, f, 10 * np.log10(S + eps), shading="gouraud")
        fig.colorbar(im, ax=ax_s, label="Leistungsdichte [dB/Hz]")
    ax_s.set(xlabel="Zeit (s)", ylabel="Frequenz (Hz)", title="Spektrogramm (Wasserfall)")
    ax_s.set_ylim(*((freq_min, freq_max) if freq_min is not None and freq_max is not None else (0, fs // 2)))
    ax_p.plot(f_psd, 10 * np.log10(P + eps))
    ax_p.set(xlabel="Frequenz (Hz)", ylabel="PSD [dB]", title="Power Spectral Density")
    ax_p.grid(True)
    for mk in markers or []:
        for v in (mk.f_min, mk.f_max):
            if v is not None:
                ax_s.axhline(y=v, color=mk.color, linestyle="--")
                ax_p.axvline(x=v, color=mk.color, linestyle="--")
        for v in (mk.t_min, mk.t_max):
            if v is not None:
                ax_s.axvline(x=v, color=mk.color, linestyle="--")
    if title:
        fig.suptitle(title)
    fig.tight_layout()
    if filepath is not None:
        fig.savefig(filepath)
    elif matplotlib.get_backend().lower() != "agg":
        plt.show()
    plt.close(fig)
    return f, t, S, f_psd, P


def _finish(fig, figure_dir=None, name=None, show=True):
    """Save ``fig`` as figure_dir/name.png when asked, show it as the reference does
    (plt.show(); skipped under a non-interactive backend), close it; returns the path or None."""
    import matplotlib
    import matplotlib.pyplot as plt
    path = None
    if figure_dir is not None and name is not None:
        import os
        path = os.path.join(figure_dir, f"{name}.png")
        fig.savefig(path)
    if show and matplotlib.get_backend().lower() not in ("agg", "pdf", "svg", "ps", "cairo", "template"):
        plt.show()
    plt.close(fig)
    return path


def print_spec(wav_data, fs, n_fft, eps=1e-10, freq_min=None, freq_max=None, markers=None, plt_title=None,
               plt_filepath=None, figure_dir=None, name=None, device: int = 0):
    """main.py:119-171 internal_print_spec: spectrogram (nperseg = nfft = n_fft, hop n_fft/2, dB)
    limited to [freq_min, freq_max]; saved to plt_filepath (the reference's argument) or shown."""
    import matplotlib.pyplot as plt

    from .dsp import spectrogram
    fig = plt.figure(figsize=(10, 5))
    f, t, S = spectrogram(wav_data, fs=fs, window="hann", nperseg=n_fft, noverlap=n_fft // 2, nfft=n_fft,
                          scaling="density", mode="psd", device=device)
    for mk in markers or []:
        if mk.f_min is not None:
            plt.axhline(y=mk.f_min, color=mk.color, linestyle="--", label=f"Marker {mk.f_min}-{mk.f_max} Hz")
        if mk.f_max is not None:
            plt.axhline(y=mk.f_max, color=mk.color, linestyle="--")
        if mk.t_min is not None:
            plt.axvline(x=mk.t_min, color=mk.color, linestyle="--", label=f"Marker {mk.t_min}-{mk.t_max} s")
        if mk.t_max is not None:
            plt.axvline(x=mk.t_max, color=mk.color, linestyle="--")
    if freq_min is not None and freq_max is not None:
        m = (f >= freq_min) & (f <= freq_max)
        f, S = f[m], S[m, :]
    plt.pcolormesh(t, f, 10 * np.log10(S + eps), shading="gouraud")
    plt.ylabel("Frequenz (Hz)")
    plt.xlabel("Zeit (s)")
    plt.title(plt_title if plt_title is not None else "Spektrogramm (Wasserfall)")
    plt.colorbar(label="Leistungsdichte [dB/Hz]")
    plt.ylim(*((freq_min, freq_max) if freq_min is not None and freq_max is not None else (0, fs // 2)))
    plt.tight_layout()
    if plt_filepath is not None:
        fig.savefig(plt_filepath)
        plt.close(fig)
        return plt_filepath
    return _finish(fig, figure_dir, name)


def print_psd(wav_data, fs, n_fft, eps=1e-10, freq_min=None, freq_max=None, markers=None, plt_title=None,
              figure_dir=None, name=None, device: int = 0):
    """main.py:174-205 internal_print_psd: Welch PSD (nperseg = nfft = n_fft, 50 % overlap, dB)
    limited to [freq_min, freq_max], shown."""
    import matplotlib.pyplot as plt

    from .live import welch_psd
    fig = plt.figure(figsize=(10, 5))
    x = np.asarray(wav_data)
    f_psd, P = welch_psd(x if x.dtype != np.uint8 else x, fs, nperseg=n_fft, noverlap=n_fft // 2, nfft=n_fft,
                         device=device)
    for mk in markers or []:
        if mk.f_min is not None:
            plt.axvline(x=mk.f_min, color=mk.color, linestyle="--", label=f"Marker {mk.f_min}-{mk.f_max} Hz")
        if mk.f_max is not None:
            plt.axvline(x=mk.f_max, color=mk.color, linestyle="--")
    if freq_min is not None and freq_max is not None:
        m = (f_psd >= freq_min) & (f_psd <= freq_max)
        f_psd, P = f_psd[m], P[m]
    with np.errstate(divide="ignore"):
        plt.plot(f_psd, 10 * np.log10(P + eps))
    plt.xlabel("Frequenz (Hz)")
    plt.ylabel("PSD [dB]")
    plt.title(plt_title if plt_title is not None else "Power Spectral Density (PSD) in dB")
    plt.grid(True)
    return _finish(fig, figure_dir, name)


def debug_whole(wav_data, fs, freq_band, noise_band, figure_dir=None, device: int = 0):
    """main.py:278-306 (debug_plot_whole): the 4096-point spectrogram around each band."""
    mk = [Marker(f_min=freq_band[0], f_max=freq_band[1], color="red"),
          Marker(f_min=noise_band[0], f_max=noise_band[1], color="blue")]
    return [print_spec(wav_data, fs, 1024 * 4, freq_min=freq_band[0] - 50, freq_max=freq_band[1] + 50, markers=mk,
                       plt_title="Spec Power Band", figure_dir=figure_dir, name="whole_spec_power_band", device=device),
            print_spec(wav_data, fs, 1024 * 4, freq_min=noise_band[0] - 50, freq_max=noise_band[1] + 50, markers=mk,
                       plt_title="Spec Noise Band", figure_dir=figure_dir, name="whole_spec_noise_band", device=device)]


def debug_config(wav_data, fs, freq_band, noise_band, figure_dir=None, device: int = 0):
    """main.py:324-350 (debug_plot_config): the 4096-point Welch PSD around each band."""
    return [print_psd(wav_data, fs, 1024 * 4, freq_min=freq_band[0] - 100, freq_max=freq_band[1] + 100,
                      markers=[Marker(f_min=freq_band[0], f_max=freq_band[1], color="red")],
                      plt_title="PSD Power Band", figure_dir=figure_dir, name="config_psd_power_band", device=device),
            print_psd(wav_data, fs, 1024 * 4, freq_min=noise_band[0] - 100, freq_max=noise_band[1] + 100,
                      markers=[Marker(f_min=noise_band[0], f_max=noise_band[1], color="blue")],
                      plt_title="PSD Noise Band", figure_dir=figure_dir, name="config_psd_noise_band", device=device)]


def debug_output_delta(times, delta_power, t_threshold, detections, adaptive: bool, figure_dir=None):
    """main.py:531-565 (debug_plot_output): delta over time, the global or adaptive threshold,
    the detections as orange spans."""
    import matplotlib.pyplot as plt
    fig = plt.figure(figsize=(10, 5))
    if not adaptive:
        plt.plot(times, delta_power, label="Delta Power")
        plt.axhline(y=t_threshold, color="red", linestyle="--", label="Threshold")
    else:
        plt.plot(times, delta_power, label="Delta Power")
        plt.plot(times, t_threshold, label="Adaptive Threshold", linestyle="--", color="red")
    for det in detections:
        plt.axvspan(det.t_start, det.t_stop, color="orange", alpha=0.5)
    plt.xlabel("Zeit (s)")
    plt.ylabel("Leistung (dB)")
    if not adaptive:
        plt.title("Delta (in dB) über Zeit")
    plt.legend()
    plt.grid()
    plt.tight_layout()
    return _finish(fig, figure_dir, "output_delta")


def debug_output_hists(detections, figure_dir=None):
    """main.py:660-685 (debug_plot_output): histograms of the detection durations and dB."""
    import matplotlib.pyplot as plt
    import matplotlib.ticker as ticker
    out = []
    fig = plt.figure(figsize=(10, 5))
    plt.hist([d.dur_s for d in detections], bins=30, color="blue", alpha=0.7)
    plt.xlabel("Duration (s)")
    plt.ylabel("Count")
    plt.title("Histogram of Detection Durations")
    plt.grid()
    plt.gca().xaxis.set_major_formatter(ticker.StrMethodFormatter("{x:.2f}"))
    plt.gca().yaxis.set_major_formatter(ticker.StrMethodFormatter("{x:.2f}"))
    plt.tight_layout()
    out.append(_finish(fig, figure_dir, "output_hist_duration"))
    fig = plt.figure(figsize=(10, 5))
    plt.hist([d.dB for d in detections], bins=30, color="green", alpha=0.7)
    plt.xlabel("dB")
    plt.ylabel("Count")
    plt.title("Histogram of Detection dB Values")
    plt.grid()
    plt.tight_layout()
    out.append(_finish(fig, figure_dir, "output_hist_db"))
    return out


def debug_time_map(detections, figure_dir=None):
    """main.py:687-716 show_time_map: detections per UTC hour as bars (utc_start must be set, as
    in the reference, which reads det.utc_start.replace)."""
    import matplotlib.pyplot as plt
    from collections import Counter
    hours = [det.utc_start.replace(minute=0, second=0, microsecond=0) for det in detections]
    count_per_hour = Counter(hours)
    keys = sorted(count_per_hour)
    x_labels = [dt.strftime("%Y-%m-%d %H:%M") for dt in keys]
    fig = plt.figure(figsize=(12, 6))
    plt.bar(x_labels, [count_per_hour[k] for k in keys], color="skyblue")
    plt.xlabel("UTC Zeit (Datum + Stunde)")
    plt.ylabel("Anzahl der Detektionen")
    plt.title("Detektionen pro Stunde")
    plt.xticks(rotation=45, ha="right")
    plt.grid(axis="y", linestyle="--", alpha=0.7)
    plt.tight_layout()
    return _finish(fig, figure_dir, "output_time_map")


def debug_output_interactive(times, band_power, noise_power, delta_power, t_threshold, detections, freq_band,
                             noise_band, figure_dir=None):
    """main.py:567-624 (debug_plot_output_interactive): the plotly band / noise power and delta
    figures, shown with fig.show() (and written as HTML under figure_dir).  Needs plotly, as the
    reference does (main.py:11)."""
    import os

    import plotly.graph_objects as go
    out = []
    fig = go.Figure()
    fig.add_trace(go.Scatter(x=times, y=band_power, mode="lines",
                             name=f"Signalband {freq_band[0]}-{freq_band[1]} Hz [dB]"))
    fig.add_trace(go.Scatter(x=times, y=noise_power, mode="lines",
                             name=f"Noiseband {noise_band[0]}-{noise_band[1]} Hz [dB]", line=dict(dash="dash")))
    fig.update_layout(title="Signal- und Noiseband-Leistung (in dB) über Zeit", xaxis_title="Zeit (s)",
                      yaxis_title="Leistung (dB)", legend=dict(x=0.01, y=0.99), template="simple_white")
    figs = [("interactive_band_power", fig)]
    fig = go.Figure()
    fig.add_trace(go.Scatter(x=times, y=delta_power, mode="lines", name="Delta [dB]"))
    # the reference repeats its threshold per time step (a list for the adaptive detector)
    fig.add_trace(go.Scatter(x=times, y=[t_threshold] * len(times), mode="lines", name="Threshold",
                             line=dict(color="red", dash="dash")))
    for det in detections:
        fig.add_shape(type="rect", x0=det.t_start, x1=det.t_stop, y0=min(delta_power), y1=max(delta_power),
                      fillcolor="orange", opacity=0.5, line_width=0)
    fig.update_layout(title="Delta (in dB) über Zeit", xaxis_title="Zeit (s)", yaxis_title="Leistung (dB)",
                      legend=dict(x=0.01, y=0.99), template="simple_white")
    figs.append(("interactive_delta", fig))
    for name, f in figs:
        if figure_dir is not None:
            path = os.path.join(figure_dir, f"{name}.html")
            f.write_html(path)
            out.append(path)
        else:
            f.show()
    return out


def export_detections(detections, wav_data, fs, freq_band, outfile_path=None, device: int = 0):
    """main.py:721-806: for each detection, the audio from 3 s before to 3 s after, n_fft 1024
    (2048 when that cut is longer than 8 s), the band +-50 Hz, the detection as red markers,
    spec_and_psd_{t_start:.2f}_{t_stop:.2f}.png under outfile_path; errors are printed."""
    written = []
    for det in detections:
        try:
            c_before = c_after = 3
            start = max(det.t_start - c_before, 0)
            stop = min(det.t_stop + c_after, len(wav_data) / fs)
            cut = wav_data[int(start * fs):int(stop * fs)]
            dur = len(cut) / fs
            n_fft = 2048 if dur > c_before + c_after + 2 else 1024
            title = (f"Detection from {det.t_start:.2f}s to {det.t_stop:.2f}s\n"
                     f"Wav duration: {dur:.2f}s, n_fft: {n_fft}\n"
                     f"Marker duration: {det.dur_s:.2f}s / dB: {det.dB:.2f}")
            path = f"{outfile_path}spec_and_psd_{det.t_start:.2f}_{det.t_stop:.2f}.png" if outfile_path else None
            spec_and_psd(cut, fs, n_fft, freq_min=freq_band[0] - 50, freq_max=freq_band[1] + 50,
                         markers=[Marker(color="red", t_min=det.t_start - start, t_max=det.t_stop - start)],
                         title=title, filepath=path, device=device)
            if path:
                written.append(path)
        except Exception as e:  # the reference prints and continues (main.py:805-806)
            print(f"Error processing detection: {e}")
    return written

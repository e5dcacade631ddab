"""Per-detection spectrogram + PSD figures: what proc_wav_file exports when
``disable_show_and_write`` is False (dsp/src/main.py:721-806 with the layout of
internal_print_spec_and_psd_mod, main.py:40-116).  The arrays come from the GPU
(``dsp.spectrogram``, ``live.welch_psd``); matplotlib only draws them.  No parity is claimed
beyond the arrays (the figures themselves are not compared)."""
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

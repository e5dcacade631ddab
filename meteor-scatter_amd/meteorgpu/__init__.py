"""meteorgpu — MI355X-native drop-in for the meteor-scatter DSP hot path.

Public surface (mirrors the reference's dsp/src/main.py):
    proc_wav_file, process_samples, OutputDetection, block_powers,
    get_detections, get_detections_adaptive, spectrogram, write_csv,
    write_audacity_labels, count_per_hour
Batch / multi-GPU: meteorgpu.batch.BatchPipeline.
All numerics run in libmsdsp.so (HIP, gfx950); there is no CPU fallback.
"""
from .dsp import (OutputDetection, ProcResult, block_powers, count_per_hour, get_detections,
                  get_detections_adaptive, proc_wav_file, process_samples, spectrogram, write_audacity_labels,
                  write_csv)

__all__ = ["OutputDetection", "ProcResult", "block_powers", "count_per_hour", "get_detections",
           "get_detections_adaptive", "proc_wav_file", "process_samples", "spectrogram", "write_audacity_labels",
           "write_csv"]

#!/usr/bin/env python3
"""Benchmark: one day of one-minute 48 kHz recordings per GPU (BASELINE.json configs[2];
configs[3] = the same sharded over 1/2/4/8 GPUs, one process per GPU).

A step = one pass of the hot path over the rank's batch, inputs resident in HBM:
  STFT power spectrogram (1024-pt, 50 % hop, float32 [K][T] per file)
  + block band dB / delta + adaptive threshold detector (reference framing)
  + per-hour detection counts, summed across ranks with one RCCL all-reduce.
Weak scaling: every rank owns `--files` files (default 1440 = one day).

Prints ONE JSON line on rank 0 with the roofline of the dominant kernel (the
STFT, timed live with HIP events on the stream it runs on) and the CPU baseline
(the numpy/scipy oracle of the reference path, 1 thread, on a bounded sample).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

With --gpus N > 1 and no launcher environment (WORLD_SIZE unset) bench.py starts the N ranks
itself (meteorgpu.launch.spawn) before anything touches a GPU.  No PyTorch anywhere: the ranks
share the RCCL unique id through a rendezvous file, and the barrier, the rank count and the
max-over-ranks time go through libmsdsp's RCCL wrappers (meteorgpu.launch.Group).
"""
import argparse
import datetime
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "meteor-scatter_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

FS = 48000
SECONDS = 60
BAND = (950.0, 1050.0)
NOISE = (2950.0, 3050.0)  # far from the ping: the 48 kHz crop leaks into near bands
NPERSEG, NOVERLAP = 1024, 512
C5_FS, C5_N, C5_HOP, C5_SECONDS = 192000, 4096, 1024, 3 * 3600
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, chip-level parameters (spec)
# C5 decision modes: (certify, delta source, exact decisions) -- meteorgpu.iq.IQShardDetector
C5_MODES = {"exact": (True, "auto", True), "off": (False, "fp32", False), "flag": (True, "fp32", False),
            "refine": (True, "fp32", True)}
SYNTH_PROCS = 16       # worker processes that make the synthetic inputs (the GPU box's CPU share)


# ------------------------------------------------------------------ synthetic inputs
# Every file / minute of every workload is distinct, seeded by SURVEY §8(d)'s rule (seed =
# 1000 * config + file index): C3 file i of day d is synth_real(3000 + 1440 d + i), C5 minute m of
# the stream synth_iq(5000 + m).  They are made by worker processes forked before any GPU call,
# straight into one shared anonymous mapping (no pickling of gigabytes), so the bench's full-size
# correctness guard (near_tie, certification) covers a day of distinct inputs.
_SYN = None


def _syn_real_row(i):
    from meteorgpu import synth
    mm, seeds, n, kw = _SYN
    np.frombuffer(mm, np.int16).reshape(len(seeds), n)[i] = synth.synth_real(seed=int(seeds[i]), **kw)[0][:n]
    return 0


def _syn_iq_row(i):
    from meteorgpu import synth
    mm, seeds, n, kw = _SYN
    i_, q_, _ = synth.synth_iq(int(seeds[i]), **kw)
    row = np.frombuffer(mm, np.int16).reshape(len(seeds), 2 * n)[i]
    row[0::2], row[1::2] = i_[:n], q_[:n]
    return 0


def synth_rows(kind, seeds, n, procs=SYNTH_PROCS, **kw):
    """[len(seeds)][n] int16 (kind "real") or [len(seeds)][2n] interleaved I/Q (kind "iq") in a
    shared anonymous mapping, one seeded recording per row, made on `procs` forked workers"""
    import mmap
    import multiprocessing as mp
    global _SYN
    width = n if kind == "real" else 2 * n
    mm = mmap.mmap(-1, max(1, len(seeds) * width * 2))  # MAP_SHARED | MAP_ANONYMOUS
    _SYN = (mm, list(seeds), n, kw)
    fn = _syn_real_row if kind == "real" else _syn_iq_row
    try:
        if procs > 1 and len(seeds) > 1:
            with mp.get_context("fork").Pool(min(procs, len(seeds))) as workers:
                workers.map(fn, range(len(seeds)), chunksize=max(1, len(seeds) // (8 * procs)))
        else:
            for i in range(len(seeds)):
                fn(i)
    finally:
        _SYN = None
    return np.frombuffer(mm, np.int16).reshape(len(seeds), width)


def day_seeds(day, lo, hi):
    """C3 seeds of files [lo, hi) of day `day`: 1000 * 3 + 1440 * day + file index"""
    return [3000 + 1440 * day + i for i in range(lo, hi)]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU); spawned here unless "
                    "an external launcher set WORLD_SIZE, which must then equal --gpus")
    ap.add_argument("--spawn", action="store_true", help="start the ranks through the launcher even at "
                    "--gpus 1 (the N>1 code path: rendezvous file + RCCL communicator on one GPU)")
    ap.add_argument("--dry-run", action="store_true", help="launcher self-test without a GPU: the ranks "
                    "rendezvous a random id and rank 0 prints what every rank saw")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10, help="untimed steps (the GPU clock ramps up over the first few)")
    ap.add_argument("--files", type=int, default=1440, help="one-minute files per GPU")
    ap.add_argument("--c5-seconds", type=float, default=C5_SECONDS, help="c5: seconds of the stream per GPU "
                    "(default 3 h: 24 h over 8 GPUs)")
    ap.add_argument("--cpu-files", type=int, default=150, help="files in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--concurrent-stages", action="store_true",
                    help="C3: run block_delta -> detect on a second stream beside the STFT (A/B; no gain measured)")
    ap.add_argument("--cpu-procs", type=int, default=16, help="processes of the multi-core CPU baseline "
                    "(the GPU box's CPU share is 16)")
    ap.add_argument("--no-spectrogram", action="store_true", help="detect-only mode (not the headline)")
    ap.add_argument("--no-c5", action="store_true", help="c3: skip the C5 run appended to the line (key \"c5\")")
    ap.add_argument("--no-live", action="store_true", help="c3: skip the live-detector run appended to the line "
                    "(key \"live\")")
    ap.add_argument("--c5-mode", choices=("all",) + tuple(C5_MODES), default="all",
                    help="C5 decisions: exact = the drop-in default (proc_iq_samples): every frame's delta in "
                         "float64 from the samples (exact integer DFT on the matrix cores), every decision "
                         "certified against the float64 reference; off = fp32 spectrogram band sums, uncertified; "
                         "flag = the same certified, uncertain decisions reported; refine = flag + the uncertain "
                         "ones and every detection's frames recomputed in float64 (round 3's certified path); "
                         "all = the line on 'exact', plus the other modes timed under \"modes\"")
    ap.add_argument("--c5-overlap", type=int, default=32,
                    help="C5: run the stream detector beside the spectrogram after the delta step, the "
                         "spectrogram leaving this many workgroup slots free (its workgroups then take chunks of "
                         "frames from a guided schedule; exact delta only: the detector does not read the "
                         "spectrogram; default 32 of ~1000); 0 = one stream, in order")
    ap.add_argument("--shard-day", action="store_true",
                    help="C4 as strong scaling: ONE day of --files files sharded over the ranks (contiguous "
                         "shard_range slices; the per-hour counts all-reduce into that day's 24 buckets) instead "
                         "of a day per GPU (the default, weak scaling)")
    ap.add_argument("--workload", choices=("c3", "live", "c5", "files"), default="c3",
                    help="c3: the headline day batch (default); live: the phase-2 live detector "
                         "(Welch band powers + state machine) over a day of 4 kHz audio; c5: 192 kHz I/Q, "
                         "4096-point two-sided spectrogram, 75 %% overlap, 3 h of the 24 h stream per GPU; files: "
                         "end to end from WAV files on disk (native reader, pinned triple-buffered uploads)")
    return ap.parse_args()


def cpu_baseline(pool, nfiles):
    """The reference path on the host: scipy.signal.spectrogram (main.py:132-133 call) + the
    block loop and adaptive detector of main.py:352-527, restated in oracle/, 1 thread."""
    from oracle import dsp_oracle as O
    t0 = time.perf_counter()
    for i in range(nfiles):
        x = pool[i % len(pool)]
        O.spectrogram_ref(x, FS, NPERSEG)
        O.proc_samples_ref(x, FS, 0.2, BAND, NOISE, 512, 4)
    dt = time.perf_counter() - t0
    return nfiles * FS * SECONDS / dt / 1e6, dt


_MP_POOL = None


def _mp_one(i):
    from oracle import dsp_oracle as O
    x = _MP_POOL[i % len(_MP_POOL)]
    O.spectrogram_ref(x, FS, NPERSEG)
    O.proc_samples_ref(x, FS, 0.2, BAND, NOISE, 512, 4)
    return 0


def cpu_baseline_mp(pool, nfiles, procs):
    """The same CPU path over `nfiles` files on `procs` worker processes.
    Forked before the GPU is touched (bench.py calls it first), one file per task."""
    import multiprocessing as mp
    global _MP_POOL
    _MP_POOL = pool
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as workers:
        workers.map(_mp_one, range(min(procs, nfiles)))  # warm the workers (imports)
        t0 = time.perf_counter()
        workers.map(_mp_one, range(nfiles), chunksize=1)
        dt = time.perf_counter() - t0
    return nfiles * FS * SECONDS / dt / 1e6, dt


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_pmc_traffic(name, **match):
    """HBM bytes per launch of the roofline kernel and where they come from: the committed
    rocprofv3 PMC summary profiles/<name>_pmc.json (FETCH_SIZE doubled per the gfx950 rule),
    if it was collected for this workload (the `match` keys agree).  The counters are NOT
    sampled in the run being reported (PMC passes cannot share a run with the timing): the
    figure is profile-derived, and "traffic_source" in the bench line names the profile round."""
    p = os.path.join(ROOT, "profiles", f"{name}_pmc.json")
    try:
        with open(p) as fh:
            d = json.load(fh)
        if all(d.get(k) == v for k, v in match.items()):
            return float(d["hbm_bytes_per_launch"]), f"profiles/{name}_pmc.json ({d.get('source', '?')})"
    except (OSError, ValueError, KeyError):
        pass
    return None, None


LIVE_FS, LIVE_FILE_S, LIVE_FILES = 4000, 3600, 24
FP64_PEAK_TFLOPS = 78.6  # MI355X FP64 vector, AMD spec sheet (not listed in MI355X_MICROARCH.md)


def cpu_baseline_live(pool, nfiles):
    """processor.py:177-507 restated (oracle/live_oracle.py): scipy welch per 0.2 s block, band
    sums, the state machine — 1 thread, on the first `nfiles` recordings of the day."""
    from oracle import live_oracle as L
    xs = [pool[i].astype(np.float64) / 32768.0 for i in range(nfiles)]
    t0 = time.perf_counter()
    for x in xs:
        L.wav_file_process_ref(x, LIVE_FS, L.ConfigDetectionRef(detection_db_over_noise_mean_min=1,
                                                                detection_dur_min_sec=0.5))
    dt = time.perf_counter() - t0
    return sum(len(x) for x in xs) / dt / 1e6, dt


def live_rows(rank):
    """the rank's day of live audio: 24 distinct seeded 1 h 4 kHz recordings (seed 6000 + 24 rank + j),
    made by forked workers before any GPU call"""
    return synth_rows("real", [6000 + LIVE_FILES * rank + j for j in range(LIVE_FILES)], LIVE_FS * LIVE_FILE_S,
                      fs=LIVE_FS, duration_s=LIVE_FILE_S, f0=1000.0, sigma=300.0, rate_per_min=5, band_hz=100.0,
                      snr_db=(10, 30), dur_s=(0.3, 2.0))


def main_live(a, world, rank, local, job_of):
    """--workload live: the live line alone."""
    from meteorgpu import _lib
    rows = live_rows(rank)
    ctx = _lib.Context(local)
    job = job_of(ctx)
    out = run_live(a, ctx, job, rank, world, rows)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if job is not None:
        job.close()


I8_PEAK_TOPS = 5000.0  # MI355X int8 MFMA, dense: 2x the BF16 rate (MI355X_MICROARCH.md, matrix cores)


def run_live(a, ctx, job, rank, world, rows):
    """Phase-2 live detector over a day of 4 kHz audio per GPU: 24 x 1 h int16 files.  Returns the
    line (cpu_baseline on rank 0 at N = 1 only)."""
    from meteorgpu import _lib
    from meteorgpu import live as LV
    cfg = LV.ConfigDetection(proc_block_sec=0.2, n_fft=4096, signal_freq=1000,
                             detection_db_over_noise_mean_min=1, detection_dur_min_sec=0.5)
    n = LIVE_FS * LIVE_FILE_S
    F = LIVE_FILES
    lb = LV.LiveBatch(ctx, F, n, LIVE_FS, cfg)
    for i in range(F):
        lb.upload_file(i, rows[i])

    def sync_all():
        ctx.synchronize()
        if job is not None:
            job.barrier()

    ctx.timing_select([_lib.K_WELCH])  # the roofline kernel only; the breakdown from one more step
    ctx.timing(True)
    for _ in range(a.warmup):
        lb.run()
    ctx.timing_reset()
    sync_all()  # no host work between the warm-up and the timed steps (the clock would drop)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        lb.run()
    sync_all()
    elapsed = time.perf_counter() - t0
    _, counts = lb.meteors()  # every step recomputes the same meteors
    if job is not None:
        elapsed = job.max_f64(elapsed)
    w_ms, w_n = ctx.timing_get(_lib.K_WELCH)
    ctx.timing_select(None)
    ctx.timing_reset()
    lb.run()
    sync_all()
    l_ms, l_n = ctx.timing_get(_lib.K_LIVE)
    ctx.timing(False)
    wc = lb.plan.cfg
    nseg = (wc.block_size - wc.nperseg) // (wc.nperseg - wc.noverlap) + 1
    nslots = sum(wc.band_hi[j] - wc.band_lo[j] + 1 for j in range(wc.nbands))
    blocks = F * lb.nb
    avg_s = w_ms / max(w_n, 1) / 1e3
    # int16 input takes the exact integer GEMM (csrc/welch_i8.hip): the dominant work is int8 MFMA,
    # per segment nperseg samples x 2 nslots components x (7 coefficient x 2 sample digits), 2 ops
    # per multiply-add, in 16-row tiles: the live default's 5-segment instantiation walks units of
    # 16 blocks = 5 full tiles, the generic one tiles of 16 // nseg whole blocks
    bpt = 16 // nseg
    tiles = 5 * -(-blocks // 16) if (nseg == 5 and wc.nperseg == 256) else -(-blocks // bpt)
    ncol = -(-2 * nslots // 16) * 16
    i8_ops = tiles * 16 * wc.nperseg * ncol * 14 * 2.0
    useful = blocks * nseg * wc.nperseg * 2 * nslots * 14 * 2.0
    live_traffic = load_pmc_traffic("welch", files=F, nperseg=int(wc.nperseg))
    out = {
        "metric": "Msamples/s processed (4 kHz live detector: Welch band powers + state machine)",
        "value": round(world * F * n * a.steps / elapsed / 1e6, 1),
        "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int8 MFMA (exact) / f64",
        "data": f"synthetic: {F} distinct seeded 1 h 4 kHz int16 noise+ping recordings per GPU "
                f"(seed 6000 + 24 rank + file index)",
        "config": {"workload": "phase-2 live detector day: 24 x 1 h 4 kHz int16 per GPU, 0.2 s blocks, "
                               "welch(nperseg 256, nfft 4096) on 3 x 100 Hz bands, 8 s history, k = 4",
                   "files_per_gpu": F, "samples_per_file": n, "blocks_per_file": lb.nb, "band_bins": nslots},
        "meteors_per_step": int(counts.sum()),
        "roofline": {"bound": "mfma", "achieved": round(i8_ops / avg_s / 1e12, 1), "peak": I8_PEAK_TOPS,
                     "unit": "TOPS (int8)", "frac": round(i8_ops / avg_s / 1e12 / I8_PEAK_TOPS, 4),
                     # HBM bytes of both kernels per launch (samples, the PSD written and read back):
                     # informational beside the MFMA bound, profile-derived like the C3 / C5 figures
                     "traffic": live_traffic[0], "traffic_source": live_traffic[1],
                     "kernel": "welch_i8_kernel<4> + welch_i8_bands_kernel", "kernel_ms": round(avg_s * 1e3, 4),
                     "int8_ops_per_launch": i8_ops, "useful_int8_ops_per_launch": useful},
        "kernel_ms_per_step": {"welch": round(avg_s * 1e3, 4), "live_detect": round(l_ms / max(l_n, 1), 4)},
    }
    # the near-tie guard of every recording (margin.py, live part; outside the timed region): a
    # decision within the proven over-noise error bound of its threshold would be flagged
    lb.check_near_ties(warn=False)
    out["near_tie"] = {"files_flagged": int(lb.near_tie.sum()), "files": F,
                       "max_decision_bound_db": float(np.max(lb.decision_bounds)),
                       "min_margin_db": float(np.min(lb.min_margins))}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_files > 0:
        nf = 6
        v, dt = cpu_baseline_live(rows, nf)
        out["cpu_baseline"] = {"value": round(v, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
                               "sample": f"{nf} of the 1 h 4 kHz files ({dt:.1f} s): scipy welch per block + "
                                         f"band sums + state machine (oracle/live_oracle.py), 1 thread"}
    out["ranks_seen"] = job.ranks_seen() if job is not None else 1
    lb.close()
    return out


C5_BAND, C5_NOISE = (950.0, 1050.0), (-3050.0, -2950.0)  # Hz from the SDR centre (two-sided spectrum)


def c5_geometry(a, rank, world):
    """(n_total, s0, s1): the stream of N shards and the samples rank's frames read"""
    from meteorgpu.iq import frame_shard
    shard = int(C5_FS * a.c5_seconds)
    n_total = shard * world + (C5_N - C5_HOP)  # the stream: N shards + the last frame's tail
    _, _, _, s0, s1 = frame_shard(n_total, C5_N, C5_HOP, rank, world)
    return n_total, s0, s1


def c5_rows(a, rank, world):
    """the distinct seeded minutes of the stream that rank's samples lie in (minute m: synth_iq(5000 + m),
    so the shards are pieces of one continuous stream), and the first one's sample offset"""
    _, s0, s1 = c5_geometry(a, rank, world)
    chunk = C5_FS * 60
    m0, m1 = s0 // chunk, -(-s1 // chunk)
    rows = synth_rows("iq", [5000 + m for m in range(m0, m1)], chunk, fs=C5_FS, duration_s=60.0, f0=1000.0,
                      sigma=1000.0, rate_per_min=6, snr_db=(10.0, 30.0))
    return rows, m0 * chunk


def main_c5(a, world, rank, local, job_of):
    """--workload c5: the C5 line alone."""
    from meteorgpu import _lib
    rows = c5_rows(a, rank, world)  # before any GPU call (forked workers)
    ctx = _lib.Context(local)
    job = job_of(ctx)
    out = run_c5(a, ctx, job, rank, world, rows)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if job is not None:
        job.close()


def run_c5(a, ctx, job, rank, world, rows):
    """BASELINE config C5: a 24 h 192 kHz I/Q stream time-sharded over the GPUs (3 h of it per
    GPU; weak scaling: the stream is 3 h x N long).  A step = the whole path on every rank:
    two-sided 4096-point power spectrogram at 75 % overlap (frame-major float32, kept in HBM),
    the per-frame band / noise dB delta, and the reference's adaptive detector over the WHOLE
    stream (meteorgpu.stream: halo, chunk-sum and shard-edge state exchanges over RCCL).
    Returns the bench line (identical on every rank but cpu_baseline, rank 0 only)."""
    from meteorgpu import _lib, iq, stream
    shard = int(C5_FS * a.c5_seconds)
    n_total = c5_geometry(a, rank, world)[0]
    head_mode = "exact" if a.c5_mode == "all" else a.c5_mode
    cert_on, delta_src, _ = C5_MODES[head_mode]
    det = iq.IQShardDetector(ctx, n_total, C5_FS, C5_N, C5_N - C5_HOP, C5_BAND, C5_NOISE, 4.0, True,
                             rank=rank, world=world, seg_len=int(os.environ.get("MSD_BENCH_SEG_LEN", "8192")),
                             certify=cert_on, delta=delta_src, overlap=a.c5_overlap)
    chunk = C5_FS * 60
    pool, first = rows  # distinct seeded minutes: noise + meteor pings at +1 kHz, int16 I/Q interleaved
    assert first <= det.s0 and first + pool.shape[0] * chunk >= det.s1
    n = det.s1 - det.s0
    pos = 0
    while pos < n:  # the rank's samples [s0, s1) minute by minute
        g = det.s0 + pos
        k, o = divmod(g - first, chunk)
        m = min(chunk - o, n - pos)
        det.upload(pool[k][2 * o: 2 * (o + m)], sample_offset=pos)
        pos += m
    comm = job.comm if job is not None else stream.LocalComm()

    mode = [head_mode]

    def step():
        det.spectrogram_and_delta()
        return det.detect(comm, thresholds=False, exact_decisions=C5_MODES[mode[0]][2])

    def sync_all():
        det.synchronize()
        if job is not None:
            job.barrier()

    res = None
    for _ in range(a.warmup):
        res = step()
    sync_all()
    # the timed region carries events only around the roofline kernel (on the spectrogram's context:
    # the caller's, or its CU-split sibling with --c5-overlap); the per-kernel breakdown
    # (kernel_ms_per_step) comes from one more step with every kernel timed, after it
    sctx = det.sctx
    ctxs = [ctx] + [c for c in {id(det.sctx): det.sctx, id(det.dctx): det.dctx}.values() if c is not ctx]
    sctx.timing_select([_lib.K_CSTFT])
    sctx.timing(True)
    sctx.timing_reset()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = step()
    sync_all()
    elapsed = time.perf_counter() - t0
    if job is not None:
        elapsed = job.max_f64(elapsed)
    k_ms, k_n = sctx.timing_get(_lib.K_CSTFT)
    sctx.timing_select(None)
    for c in ctxs:
        c.timing(True)
        c.timing_reset()
    step()
    sync_all()
    kms = {}
    for name, kid in (("cstft", _lib.K_CSTFT), ("band_delta", _lib.K_IQDELTA),
                      ("fresh_thresholds", _lib.K_FRESH), ("scan", _lib.K_SSCAN), ("delta64", _lib.K_REFINE)):
        kms[name] = round(sum(c.timing_get(kid)[0] for c in ctxs), 4)
    for c in ctxs:
        if c is not ctx:
            c.timing(False)
    kms["cstft"] = round(k_ms / max(k_n, 1), 4)  # the timed region's average

    def cert_info(r, m):
        if r.certified is None:
            return {"mode": m, "certified": None, "delta": "fp32"}
        return {"mode": m, "delta": "exact" if det.exact_delta else "fp32", "certified": bool(r.certified),
                "near_tie": bool(r.near_tie), "uncertain_before_refinement": int(r.uncertain_initial),
                "refined_delta_frames": int(r.refined_delta_frames), "db_refined_frames": int(r.db_refined_frames),
                "detector_passes": int(r.detector_passes), "refine_budget_exhausted": bool(r.refine_budget_exhausted),
                "decision_bound_db": float("%.6g" % r.decision_bound), "min_slack_db": float("%.6g" % r.min_slack)}

    cert = cert_info(res, head_mode)
    head_exact_delta = det.exact_delta
    others = {}
    if a.c5_mode == "all":
        # the other decision modes, each timed on its own after the headline (fewer steps): off = the
        # fp32 band sums uncertified, flag = certified with uncertain decisions reported, refine =
        # the uncertain ones and the detections' frames recomputed in float64 (round 3's path)
        for m in ("off", "flag", "refine"):
            mode[0] = m
            det.set_certify(C5_MODES[m][0])
            det.set_delta(C5_MODES[m][1])
            for _ in range(min(a.warmup, 3)):
                r = step()
            sync_all()
            ns = max(1, min(a.steps, 10))
            t1 = time.perf_counter()
            for _ in range(ns):
                r = step()
            sync_all()
            el = time.perf_counter() - t1
            if job is not None:
                el = job.max_f64(el)
            others[m] = cert_info(r, m)
            others[m].update(steps=ns, ms_per_step=round(el / ns * 1e3, 4),
                             value=round(world * int(C5_FS * a.c5_seconds) * ns / el / 1e6, 1),
                             same_detections=bool(np.array_equal(r.detections[["start", "stop"]],
                                                                 res.detections[["start", "stop"]])))
    avg_s = k_ms / max(k_n, 1) / 1e3
    T = det.f1 - det.f0
    samples = shard  # per rank: its 3 h (the 3072-sample frame tail is read, not counted)
    hrs = f"{a.c5_seconds / 3600:g} h"
    alg_bytes = (det.s1 - det.s0) * 4 + T * C5_N * 4
    c5_traffic = load_pmc_traffic("cstft", frames=T, nperseg=C5_N)
    out = {
        "metric": "Msamples/s processed (192 kHz I/Q: 4096-pt two-sided spectrogram, 75% overlap, band delta, "
                  "adaptive detector)",
        "value": round(world * samples * a.steps / elapsed / 1e6, 1),
        "unit": "Msamples/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
        "ms_per_step": round(elapsed / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32 spectrogram / f64 detector",
        "data": f"synthetic: {hrs} per GPU of one continuous 192 kHz int16 I/Q stream (noise + pings), every minute "
                f"distinct (minute m seeded 5000 + m, SURVEY §8(d))",
        "config": {"workload": f"C5: 192 kHz I/Q stream time-sharded {hrs} per GPU ({hrs} x N long), spectrogram "
                               "4096/1024 float32 [T][4096] frame-major + per-frame band dB (950..1050 Hz vs "
                               "-3050..-2950 Hz) + adaptive detector over the whole stream (k 4, window 120 s = "
                               f"{det.W} frames, freeze 20 s, fixed init 10 s)",
                   # the timed step: run(thresholds=False) -- the decisions and the detections' dB,
                   # not the per-frame thresholds list proc_iq_samples returns (the CSV, main.py:640-658,
                   # does not use it)
                   "detector": "decisions only (thresholds list not materialised)",
                   "samples_per_gpu": samples, "frames_per_gpu": T, "frames_total": det.T, "bins": C5_N,
                   "parallelism": f"time shards over {world} GPU(s), 1 process per GPU"},
        "detections_per_step": int(len(res.detections)),
        "state_rounds": int(res.rounds),
        "exact_threshold_frames": int(res.refined),
        # the headline's decision mode (C5_MODES): exact = the drop-in default, every frame's delta
        # float64 from the samples and every decision certified; "modes" times the others
        "decisions": head_mode,
        "detector_overlap": a.c5_overlap,
        "roofline": {"bound": "hbm", "achieved": round(alg_bytes / avg_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(alg_bytes / avg_s / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": c5_traffic[0], "traffic_source": c5_traffic[1],
                     "kernel": "cstft4096_kernel<int16>", "kernel_ms": round(avg_s * 1e3, 4),
                     "algorithmic_bytes_per_launch": alg_bytes},
        "kernel_ms_per_step": kms,
        "certification": cert,
        "modes": others or None,
    }
    if head_exact_delta:
        # the exact delta's block step (refine_i8.hip + refine.hip frame_kernel): it re-reads every
        # sample (4 B per complex sample) and writes / reads the 11-row block table (176 B per block)
        # and delta, ed (16 B per frame)
        nblk = (det.s1 - det.s0) // C5_HOP
        xb = (det.s1 - det.s0) * 4 + nblk * 176 * 2 + T * 16
        dms = kms["delta64"]
        out["exact_delta"] = {"kernel": "block_i8_kernel<7> + frame_kernel", "ms": dms, "bytes": xb,
                              "achieved_gbs": round(xb / (dms * 1e-3) / 1e9, 1) if dms > 0 else None,
                              "frac_of_hbm": round(xb / (dms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if dms > 0 else None}
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_files > 0:
        from oracle import iq_oracle as Q
        mins = 10
        m = C5_FS * 60 * mins  # the first 10 minutes of the rank's stream (~8 s on one core)
        z = pool[:mins].reshape(-1)  # consecutive minutes of the stream
        t1 = time.perf_counter()
        Q.proc_iq_ref(z[0:2 * m:2], z[1:2 * m:2], C5_FS, C5_BAND, C5_NOISE, C5_N, C5_N - C5_HOP, 4.0)
        dt = time.perf_counter() - t1
        out["cpu_baseline"] = {"value": round(m / dt / 1e6, 3), "unit": "Msamples/s", "cores": 1, "kind": "port",
                               "sample": f"{mins} min of the 192 kHz I/Q stream ({dt:.1f} s): scipy.signal.spectrogram "
                                         f"(complex input, 4096/3072) + per-frame band sums + adaptive detector "
                                         f"(oracle/iq_oracle.py), 1 thread"}
    out["ranks_seen"] = job.ranks_seen() if job is not None else 1
    det.close()
    return out


def main_files(a, world, rank, local, job_of):
    """End to end from disk: `--files` one-minute 48 kHz WAVs written to a temp dir, then
    meteorgpu.ingest.WavDay (native reader threads → pinned memory → copy stream → the C3
    pipeline, triple-buffered batches of 120).  The page cache is warm (files just written):
    this measures decode + PCIe + compute, not the disk."""
    import shutil
    import tempfile
    from meteorgpu import _lib, ingest, synth, wav
    ctx = _lib.Context(local)
    job = job_of(ctx)
    F = min(a.files, 480)
    pool = [synth.synth_real(seed=2000 + j, fs=FS, duration_s=SECONDS, f0=1000.0)[0] for j in range(POOL)]
    d = tempfile.mkdtemp(prefix=f"msd_wav_{rank}_", dir=os.environ.get("TMPDIR", "/tmp"))
    try:
        day0 = datetime.datetime(2025, 6, 1) + datetime.timedelta(days=rank)
        paths = []
        for i in range(F):
            t = day0 + datetime.timedelta(minutes=i)
            p = os.path.join(d, f"SDR_gqrx_{t:%Y%m%d}_{t:%H%M%S}_49969000.wav")
            wav.write(p, FS, pool[i % POOL])
            paths.append(p)
        wd = ingest.WavDay(ctx, paths, batch_files=120, freq_band=BAND, noise_band=NOISE, n_fft=512,
                           nperseg=NPERSEG, noverlap=NOVERLAP)
        wd.run()  # warm-up (kernels, page cache)
        best = None
        for _ in range(max(1, a.steps)):
            t0 = time.perf_counter()
            dets, hist, info = wd.run()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        if job is not None:
            best = job.max_f64(best)
        n = FS * SECONDS
        out = {
            "metric": "Msamples/s end to end from WAV files (48 kHz, C3 pipeline)",
            "value": round(world * F * n / best / 1e6, 1), "unit": "Msamples/s", "n_gpus": world,
            "steps": a.steps, "warmup": 1, "ms_per_step": round(best * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": f"synthetic: {F} one-minute 48 kHz int16 WAV files per GPU (page cache warm)",
            "config": {"workload": "files -> native WAV reader (8 threads) -> pinned host -> copy stream -> STFT + "
                                   "block delta + adaptive detector, batches of 120, triple-buffered",
                       "files_per_gpu": F, "read_s": round(info["read_s"], 3),
                       "detections": int(sum(len(x) for x in dets)), "hour_total": int(hist.sum())},
        }
        out["ranks_seen"] = job.ranks_seen() if job is not None else 1
        if rank == 0:
            print(json.dumps(out), flush=True)
    finally:
        shutil.rmtree(d, ignore_errors=True)
        if job is not None:
            job.close()


def dry_run(rank, world, files):
    """Launcher self-test without a GPU: the ranks share a random 128-byte id through the
    rendezvous file, each publishes the digest it saw, and rank 0 checks they all agree."""
    import hashlib
    from meteorgpu import launch
    if os.environ.get("MSD_DRYRUN_PID_DIR"):  # test hook: where the ranks' PIDs go (liveness checks)
        with open(os.path.join(os.environ["MSD_DRYRUN_PID_DIR"], f"rank{rank}.pid"), "w") as fh:
            fh.write(str(os.getpid()))
    uid = launch.share_bytes(rank, lambda: os.urandom(128))
    if os.environ.get("MSD_DRYRUN_FAIL_RANK") == str(rank):
        # test hook: this rank dies after the id rendezvous (where a real rank has its RCCL
        # communicator up) while the others block waiting for it -- once every rank is up
        pid_dir, t_end = os.environ.get("MSD_DRYRUN_PID_DIR"), time.monotonic() + 30
        while pid_dir and len(os.listdir(pid_dir)) < world and time.monotonic() < t_end:
            time.sleep(0.01)
        sys.exit(7)
    if os.environ.get("MSD_DRYRUN_RCCL_FAIL_RANK") == str(rank):
        # test hook: this rank's communicator init fails as libmsdsp reports it (MsdError with the
        # msd_last_error text), through the same wrapper launch.Group uses
        from meteorgpu import _lib
        launch.open_comm(lambda: (_ for _ in ()).throw(
            _lib.MsdError(-6, "msd_comm_init: ncclCommInitRank: unhandled system error (simulated)")), rank)
    launch.share_bytes(0, lambda: hashlib.sha1(uid).digest(), tag=f"seen{rank}")
    if rank != 0:
        return
    seen = [launch.share_bytes(1, lambda: b"", tag=f"seen{r}") for r in range(world)]
    for r in range(world):
        launch.release(0, tag=f"seen{r}")
    launch.release(0)
    ok = all(d == hashlib.sha1(uid).digest() for d in seen)
    from meteorgpu.shard import shard_range
    # the C4 strong-scaling pass the real run appends (key "strong_scaling"): one day of --files
    # files over the ranks, contiguous slices
    strong = {"files_total": files, "files_per_rank": [int(np.subtract(*shard_range(files, r, world)[::-1]))
                                                       for r in range(world)], "scaling": "strong"}
    # the real line carries ranks_seen for the C3 leg (top level), the C5 leg ("c5") and the live leg
    print(json.dumps({"dry_run": True, "n_gpus": world, "ranks_seen": len(seen), "id_agreed": ok,
                      "strong_scaling": strong, "c5": {"ranks_seen": len(seen)}, "live": {"ranks_seen": len(seen)}}),
          flush=True)
    if not ok:
        sys.exit(1)


def main():
    try:
        _main()
    except BaseException as e:  # noqa: BLE001 -- the parent (launch.spawn) prints this rank's reason
        if not (isinstance(e, SystemExit) and e.code in (0, None)):
            from meteorgpu import launch
            if launch.launched():
                launch.report_failure(int(os.environ.get("RANK", "0")), f"{type(e).__name__}: {e}")
        raise


def _main():
    a = parse()
    from meteorgpu import launch
    if not launch.launched() and (a.gpus > 1 or a.spawn):
        # start the ranks before anything here touches a GPU; each is this script again
        sys.exit(launch.spawn([os.path.abspath(__file__)] + sys.argv[1:], a.gpus))
    rank, world, local = launch.env_world()
    if world != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started {world} rank(s)")
    if a.dry_run:
        return dry_run(rank, world, a.files)
    from meteorgpu import _lib
    ndev = _lib.device_count()
    if local >= ndev:
        sys.exit(f"bench.py: rank {rank} wants device {local} but only {ndev} GPU(s) are visible")
    # the job's RCCL group: every launched rank (N > 1, or --spawn at N = 1) joins it
    job_of = (lambda ctx: launch.Group(ctx, rank, world)) if launch.launched() else (lambda ctx: None)
    if a.workload in ("live", "c5", "files"):
        {"live": main_live, "c5": main_c5, "files": main_files}[a.workload](a, world, rank, local, job_of)
        return

    from meteorgpu.shard import shard_range
    if a.shard_day:  # C4 strong scaling as the headline: files [lo, hi) of one day
        lo, hi = shard_range(a.files, rank, world)
    else:  # rank r holds day r (weak scaling)
        lo, hi = 0, a.files
    day = 0 if a.shard_day else rank
    pool = synth_rows("real", day_seeds(day, lo, hi), FS * SECONDS, fs=FS, duration_s=SECONDS, f0=1000.0)
    spool = None  # C4 after the weak-scaling line: this rank's share of day 0, made before any GPU call
    if not a.shard_day and (world > 1 or launch.launched()):
        slo, shi = shard_range(a.files, rank, world)
        spool = pool[slo:shi] if day == 0 else synth_rows("real", day_seeds(0, slo, shi), FS * SECONDS, fs=FS,
                                                          duration_s=SECONDS, f0=1000.0)
    # the C5 line's stream and the live line's day, made before any GPU call as well
    rows5 = c5_rows(a, rank, world) if not a.no_c5 and not a.shard_day else None
    rows_live = live_rows(rank) if not a.no_live and not a.shard_day else None
    mp_base = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_files > 0 and a.cpu_procs > 1:
        # before any GPU call: the workers are forked from this process
        mp_files = a.cpu_files * a.cpu_procs // 4
        v, dt = cpu_baseline_mp(pool, mp_files, a.cpu_procs)
        mp_base = {"value": round(v, 2), "unit": "Msamples/s", "cores": a.cpu_procs, "kind": "port",
                   "sample": f"{mp_files} of the 60 s 48 kHz files on {a.cpu_procs} processes ({dt:.1f} s), "
                             f"same path as cpu_baseline; CPU: {cpu_model()}"}
    ctx = _lib.Context(local)
    job = job_of(ctx)
    n = FS * SECONDS
    r = run_c3(a, ctx, job, rank, world, pool, lo, hi, a.shard_day, detail=True)
    F = hi - lo
    samples = (a.files if a.shard_day else world * F) * n
    out = {
        "metric": "Msamples/s processed (48 kHz SDR stream) + % HBM roofline, 1/2/4/8 MI355X",
        "value": round(samples * a.steps / r["elapsed"] / 1e6, 1),
        "unit": "Msamples/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(r["elapsed"] / a.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if a.shard_day else "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic: {F} distinct seeded 60 s 48 kHz int16 noise+ping recordings per GPU (seed 3000 + "
                f"1440 day + file index, SURVEY §8(d))",
        "config": {
            "workload": "C3 day batch: 1440 x 60 s 48 kHz mono int16 per GPU; STFT 1024/512 density PSD "
                        "(float32 [513][T]) + block band dB (0.2 s, n_fft 512 -> 1024-pt rFFT crop, bands 950-1050/2950-3050 Hz) + "
                        "adaptive detector + per-hour counts (RCCL all-reduce)" if not a.no_spectrogram else
                        "C3 day batch, detect-only",
            "files_per_gpu": F,
            "samples_per_file": n,
            "frames_per_file": r["T"],
            "bins": r["K"],
            "parallelism": (f"one day of {a.files} files sharded over {world} GPU(s) (C4, strong scaling)"
                            if a.shard_day else f"a day of files per GPU over {world} GPU(s) (weak scaling)")
                           + ", 1 process per GPU",
        },
        "detections_per_step": r["detections"],
    }
    if "roofline" in r:
        out["roofline"] = r["roofline"]
    out["kernel_ms_per_step"] = r["kernel_ms"]
    out["near_tie"] = r["near_tie"]  # margin.py's guard over this rank's files (C3 decisions vs numpy)
    if not a.shard_day:
        # BASELINE configs[3] (C4): the SAME 1440-file day sharded over the N ranks (strong scaling),
        # measured after the weak-scaling line so that the driver's 1/2/4/8 runs carry both curves
        if world > 1 or job is not None:
            slo, shi = shard_range(a.files, rank, world)
            rs = run_c3(a, ctx, job, rank, world, spool, slo, shi, True, detail=False)
            strong = {"value": round(a.files * n * a.steps / rs["elapsed"] / 1e6, 1),
                      "ms_per_step": round(rs["elapsed"] / a.steps * 1e3, 4), "files_total": a.files,
                      "files_per_gpu_max": -(-a.files // world), "detections_per_step": rs["detections"],
                      "hour_total": rs["hour_total"], "scaling": "strong", "steps": a.steps}
            if "roofline" in rs:
                strong["stft_kernel_ms"] = rs["roofline"]["kernel_ms"]
        else:  # one rank: the strong-scaling configuration is the run above
            strong = {"value": out["value"], "ms_per_step": out["ms_per_step"], "files_total": a.files,
                      "files_per_gpu_max": a.files, "detections_per_step": r["detections"],
                      "hour_total": r["hour_total"], "scaling": "strong", "steps": a.steps,
                      "note": "N = 1: the same run as the headline line"}
        strong["ranks_seen"] = job.ranks_seen() if job is not None else 1
        out["strong_scaling"] = strong
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.cpu_files > 0:
        v, dt = cpu_baseline(pool, a.cpu_files)
        out["cpu_baseline"] = {
            "value": round(v, 2),
            "unit": "Msamples/s",
            "cores": 1,
            "kind": "port",
            "sample": f"{a.cpu_files} of the 60 s 48 kHz files ({dt:.1f} s): scipy.signal.spectrogram "
                      f"1024/512 + main.py block loop + adaptive detector (oracle/), 1 thread",
        }
    if mp_base is not None:
        out["cpu_baseline_multicore"] = mp_base
    if not a.no_c5 and not a.shard_day:
        # BASELINE configs[4] (C5) in the same run, after the C3 timed region: the driver's record
        # then carries a C5 number of its own (the full line under "c5")
        try:
            c5 = run_c5(a, ctx, job, rank, world, rows5)
            out["c5"] = {k: c5[k] for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "scaling",
                                            "dtype", "roofline", "kernel_ms_per_step", "detections_per_step",
                                            "state_rounds", "exact_threshold_frames", "config", "cpu_baseline",
                                            "decisions", "certification", "modes", "exact_delta",
                                            "ranks_seen") if k in c5}
        except Exception as e:  # noqa: BLE001 -- one rank: the C3 line stands; several: fail as one job
            if world > 1:
                raise
            out["c5"] = {"error": f"{type(e).__name__}: {e}"}
    if rows_live is not None:
        # the phase-2 live detector in the same run, after C3 and C5 (key "live")
        try:
            out["live"] = run_live(a, ctx, job, rank, world, rows_live)
        except Exception as e:  # noqa: BLE001 -- one rank: the C3 line stands; several: fail as one job
            if world > 1:
                raise
            out["live"] = {"error": f"{type(e).__name__}: {e}"}
    out["ranks_seen"] = job.ranks_seen() if job is not None else 1
    if rank == 0:
        print(json.dumps(out), flush=True)
    if job is not None:
        job.close()


def run_c3(a, ctx, job, rank, world, pool, lo, hi, one_day, detail):
    """C3 / C4: files [lo, hi) of a day on this rank (one_day: of ONE day sharded over the ranks,
    else day `rank`); warm-up, then a.steps timed steps.  Returns the max-over-ranks time, the
    detections, the all-reduced hour total and (detail) the roofline and kernel breakdown.  The
    pipeline is freed before returning."""
    from meteorgpu import _lib
    from meteorgpu.batch import BatchPipeline
    n = FS * SECONDS
    F = hi - lo
    bp = BatchPipeline(ctx, F, n, FS, nperseg=NPERSEG, noverlap=NOVERLAP, freq_band=BAND, noise_band=NOISE,
                       with_spectrogram=not a.no_spectrogram, concurrent=a.concurrent_stages)
    for i in range(F):  # pool: this rank's files [lo, hi), one row each
        bp.upload_file(i, pool[i])
    # file i starts at minute lo + i of the day: 2025-06-01 (one day sharded) or 2025-06-(1+r) (a day per rank)
    epoch = datetime.datetime(1970, 1, 1)
    day0 = datetime.datetime(2025, 6, 1) + datetime.timedelta(days=0 if one_day else rank)
    us = lambda t: (t - epoch) // datetime.timedelta(microseconds=1)  # noqa: E731
    bp.set_start_times(np.array([us(day0 + datetime.timedelta(minutes=lo + i)) for i in range(F)], np.int64),
                       us(day0))

    def step():
        bp.run()
        if job is not None:
            job.rccl.allreduce_i64(bp.d_hist, bp.nbuckets)

    def sync_all():
        ctx.synchronize()
        if job is not None:
            job.barrier()

    # events only around the roofline kernel in the timed region; the breakdown of the other
    # kernels (kernel_ms_per_step) comes from one more step with every kernel timed, after it
    for c in bp.contexts:
        c.timing_select([_lib.K_STFT])
        c.timing(True)
        c.timing_reset()
    for _ in range(a.warmup):
        step()
    for c in bp.contexts:
        c.timing_reset()
    # the timed steps follow the warm-up with no host work in between: an idle gap lets the shader
    # clock drop, and the first timed launches then run slow while it ramps again (7.4 against
    # 5.9 ms, profiles/r3b_dispatches.txt)
    sync_all()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    sync_all()
    elapsed = time.perf_counter() - t0
    # correctness guard on the benchmarked data (after the timed region; every step recomputes the
    # same outputs): every file's detector finished cleanly and the (all-reduced) hour histogram
    # holds every detection of every rank
    import warnings
    with warnings.catch_warnings():  # the near-tie guard's verdict is reported in the line instead
        warnings.simplefilter("ignore")
        _, counts, status, margins = bp.detections()
    assert (status == 0).all(), "detector status"
    near = {"files_flagged": int(bp.near_tie.sum()), "files": F,
            "max_decision_bound_db": float(np.max(bp.decision_bounds)) if F else 0.0,
            "min_margin_db": float(np.min(margins)) if F else float("inf")}
    if job is not None:
        elapsed = job.max_f64(elapsed)
        total_dets = int(job.sum_i64([int(counts.sum())])[0])
    else:
        total_dets = int(counts.sum())
    hist = bp.hour_counts()
    assert int(hist.sum()) == total_dets, "hour histogram != detections"
    stft_ms, stft_launches = ctx.timing_get(_lib.K_STFT)
    res = {"elapsed": elapsed, "detections": total_dets, "hour_total": int(hist.sum()), "T": bp.T, "K": bp.K,
           "near_tie": near}
    if not a.no_spectrogram and stft_launches:
        avg_s = stft_ms / stft_launches / 1e3
        alg_bytes = F * (n * 2 + bp.K * bp.T * 4)  # samples read once + spectrogram written once
        traffic, traffic_src = load_pmc_traffic("stft", files=F, nperseg=NPERSEG)
        achieved = alg_bytes / avg_s / 1e9
        res["roofline"] = {
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "kernel": "stft1024_kernel<int16>",
            "kernel_ms": round(avg_s * 1e3, 4),
            "algorithmic_bytes_per_launch": alg_bytes,
        }
    for c in bp.contexts:
        c.timing_select(None)
        c.timing_reset()
    if detail:
        step()
        sync_all()
        blk_ms, blk_launches = bp.stage_ctx.timing_get(_lib.K_BLOCK)
        det_ms, det_launches = bp.stage_ctx.timing_get(_lib.K_DSCAN)
        res["kernel_ms"] = {
            "stft": round(stft_ms / max(stft_launches, 1), 4),
            "block_delta": round(blk_ms / max(blk_launches, 1), 4),
            "detect": round(det_ms / max(det_launches, 1), 4),
        }
    for c in bp.contexts:
        c.timing(False)
    bp.close()
    return res


if __name__ == "__main__":
    main()

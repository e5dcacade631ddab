/*
 * msdsp.h — C-ABI of libmsdsp.so, the MI355X (gfx950) implementation of the
 * meteor-scatter DSP hot path:
 *
 *   samples ──► STFT power spectrogram (scipy.signal.spectrogram semantics)
 *           └─► block framing → symmetric Hann → rFFT crop → band / noise dB → delta
 *               └─► global / adaptive threshold detector → detections (+ per-hour counts)
 *
 * The reference (th-nuernberg/meteor-scatter) is pure Python; its "FFI" for this
 * path is the numpy/scipy calls inside dsp/src/main.py.  Each entry point below
 * names the reference lines it replaces.  Conventions:
 *   - every function returns MSD_OK (0) or a negative MSD_ERR_* code; the message
 *     of the last failure on the calling thread is in msd_last_error();
 *   - "_dev" functions take device pointers and enqueue on the context's stream
 *     (no host synchronisation); the others take host pointers, borrow them for
 *     the duration of the call only, and return after the results are on the host;
 *   - a context is bound to one device and one HIP stream; it is not thread-safe.
 * No torch, numpy or HIP types appear in the signatures.
 */
#ifndef MSDSP_H
#define MSDSP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MSD_ABI_VERSION 1

#define MSD_OK 0
#define MSD_ERR_INVALID (-1)     /* bad argument (null pointer, size, ...)                 */
#define MSD_ERR_HIP (-2)         /* HIP runtime failure                                    */
#define MSD_ERR_UNSUPPORTED (-3) /* configuration outside what the kernels implement       */
#define MSD_ERR_ASSERT (-4)      /* a reference `assert` would fire (message says which)   */
#define MSD_ERR_CAPACITY (-5)    /* output capacity too small                              */
#define MSD_ERR_INDEX (-6)       /* reference would raise IndexError (empty global input)  */
#define MSD_ERR_RCCL (-7)        /* RCCL missing or failed                                 */

/* sample formats, as scipy.io.wavfile.read returns them (io/wavfile.py:568-733) */
#define MSD_U8 1
#define MSD_I16 2
#define MSD_I32 3
#define MSD_F32 4
#define MSD_F64 5
/* complex (I/Q) samples, interleaved I, Q: one complex sample = 2 elements */
#define MSD_CI16 6
#define MSD_CF32 7

typedef struct msd_ctx msd_ctx;
typedef struct msd_stft_plan msd_stft_plan;
typedef struct msd_block_plan msd_block_plan;
typedef struct msd_comm msd_comm;

/* ---------------------------------------------------------------- context */
int msd_abi_version(void);
const char *msd_last_error(void);
int msd_device_count(int *count);
int msd_create(int device, msd_ctx **out);
void msd_destroy(msd_ctx *ctx);
int msd_synchronize(msd_ctx *ctx);

/* device memory owned by the caller, allocated through the context's device */
int msd_dev_alloc(msd_ctx *ctx, size_t bytes, void **dptr);
int msd_dev_free(msd_ctx *ctx, void *dptr);
int msd_memcpy_h2d(msd_ctx *ctx, void *dst, const void *src, size_t bytes);
int msd_memcpy_d2h(msd_ctx *ctx, void *dst, const void *src, size_t bytes);
int msd_memset_dev(msd_ctx *ctx, void *dst, int value, size_t bytes);

/* Options: MSD_OPT_GENERIC_STFT = 1 → use the generic STFT kernel even where a
 * specialised one exists (A/B testing of the kernels; results must agree).
 * MSD_OPT_FRESH_ALL = 1 → the C5 stream detector computes every adaptive threshold exactly up
 * front instead of only where a scan reads it (A/B of that scheme; results must agree; also
 * set by MSD_FRESH_ALL=1 in the environment).
 * MSD_OPT_REFINE_GOERTZEL = 1 → msd_iq_delta64_dev computes int16 blocks with the float64
 * Goertzel kernel instead of the exact int8-MFMA one (A/B; both within their bounds).
 * MSD_OPT_CSTFT_RESERVE = n → the persistent C5 spectrogram kernel (msd_cstft_psd_dev) leaves n
 * of its resident workgroup slots free, so that small kernels on another context's stream (the
 * stream detector, when its delta does not come from the spectrogram) run beside it.
 * MSD_OPT_STREAM_CUS = n → the context's stream is re-created on a subset of the device's CUs
 * (hipExtStreamCreateWithCUMask): n > 0 the first n CUs, n < 0 all but those |n| -- two contexts
 * set to n and -n split the chip into disjoint parts --, 0 all CUs again; persistent grids are
 * sized for the CUs the stream may use.  Synchronises the context's stream first.
 * MSD_OPT_CSTFT_SCHED = 0 / 1 / 2 → how the persistent C5 spectrogram kernel (hop 1024) splits the
 * frames over its workgroups: 0 (default) and 2 chunks drawn from a guided schedule by an atomic
 * ticket; 1 one fixed range per workgroup (round-4 behaviour, A/B).  Same output either way.
 * (MSD_CSTFT_SCHED=static|chunked in the environment sets the default of new contexts, for A/B.)
 * MSD_OPT_STFT_SCHED = 0 / 1 / 2 → the same choice for stft1024_kernel's 32-frame tiles (the C3
 * spectrogram): 0 (default) and 1 fixed ranges, 2 chunks (MSD_STFT_SCHED=static|chunked).
 * MSD_OPT_BLOCK_GOERTZEL = 1 → msd_block_delta[_dev] computes int16 blocks with the float64
 * Goertzel kernel instead of the exact int8-MFMA one (plans with min(block_size, n_fft) = 256,
 * 512 or 1024 and at most 8 band + noise bins take the latter by default; A/B, both within the
 * near-tie bound of meteorgpu/margin.py; MSD_BLOCK_GOERTZEL=1 in the environment sets it for new
 * contexts).
 * MSD_OPT_WELCH_GOERTZEL = 1 → msd_welch_bands[_dev] / msd_welch_psd compute int16 samples with the
 * float64 Goertzel kernel instead of the exact int8-MFMA one (plans with nperseg a multiple of 64
 * up to 512, <= 16 segments per block and a window in [-1, 1] take the latter by default; A/B,
 * both within margin.py's live bound; MSD_WELCH_GOERTZEL=1 in the environment). */
#define MSD_OPT_GENERIC_STFT 1
#define MSD_OPT_FRESH_ALL 2
#define MSD_OPT_REFINE_GOERTZEL 3
#define MSD_OPT_CSTFT_RESERVE 4
#define MSD_OPT_STREAM_CUS 5
#define MSD_OPT_CSTFT_SCHED 6
#define MSD_OPT_STFT_SCHED 7
#define MSD_OPT_BLOCK_GOERTZEL 8
#define MSD_OPT_WELCH_GOERTZEL 9
int msd_set_option(msd_ctx *ctx, int option, int value);

/* Per-kernel device timing with HIP events on the context stream.
 * kernel id: 0 = STFT power, 1 = block delta, 2 = detector stats, 3 = detector scan,
 * 4 = Welch band powers, 5 = live detector, 6 = complex (I/Q) STFT, 7 = I/Q band delta,
 * 8 = stream fresh thresholds, 9 = stream scan, 10 = float64 delta (msd_iq_delta64_dev),
 * 11 = the I/Q STFT's post-FFT detrend of bins 0, +-1 (its separate fix-up kernels). */
int msd_timing_enable(msd_ctx *ctx, int enable);
/* which kernels get events while timing is on: bit k = kernel id k (default all); a timed
 * region that times only its roofline kernel carries no events around the others */
int msd_timing_select(msd_ctx *ctx, uint32_t kernel_mask);
int msd_timing_reset(msd_ctx *ctx);
int msd_timing_get(msd_ctx *ctx, int kernel, double *total_ms, int64_t *launches);

/* ------------------------------------------------- a7: STFT power spectrogram
 * Replaces scipy.signal.spectrogram(x, fs, window='hann', nperseg=N,
 * noverlap=N-hop, nfft=N, detrend='constant', scaling='density', mode='psd')
 * as called at dsp/src/main.py:52-54 and :132-133.
 * window: N float32 values of the periodic Hann (scipy get_window, cast to
 * complex64 by _spectral_helper, i.e. float32); scale = 1/(fs*sum(w^2)) as
 * scipy computes it.  Output: float32 [K = N/2+1][T], T = (n-N)/hop + 1, with
 * bins 1..N/2-1 doubled (one-sided, even N).  N: a power of two in [16, 16384]
 * (1024: stft1024.hip; 256..2048: stft.hip's tiled kernel; others: stft_any.hip). */
int msd_stft_plan_create(msd_ctx *ctx, int32_t nperseg, int32_t hop, const float *window, double scale,
                         msd_stft_plan **out);
/* The general form: segments of nperseg samples (any length >= 1) zero-padded to an nfft-point
 * transform (nfft a power of two in [16, 16384], nfft >= nperseg), K = nfft/2 + 1 bins, in
 * float32 (precision MSD_F32, output float) or float64 (MSD_F64, output double; the
 * msd_stft_psd_f64 entry points).  Covers scipy.signal.spectrogram(..., nfft=) and its
 * shrinking of nperseg to a short input (dsp/src/main.py:127-133 with n_fft = 1024*4,
 * :278-300; scipy _spectral_py.py _triage_segments) and matplotlib.mlab.specgram in float64
 * (prime_detection.py:70, window_hanning, detrend_none, pad_to = NFFT).  window: nperseg
 * float64 values (cast to float32 by a float32 plan). */
int msd_stft_plan_create_ex(msd_ctx *ctx, int32_t nperseg, int32_t nfft, int32_t hop, const double *window,
                            double scale, int precision, msd_stft_plan **out);
void msd_stft_plan_destroy(msd_stft_plan *plan);
/* K = nfft/2 + 1, the rows of the plan's spectrogram */
int32_t msd_stft_bins(const msd_stft_plan *plan);
/* detrend: 1 = 'constant' (scipy's default, the plan's initial setting), 0 = none
 * (matplotlib.mlab.specgram's detrend_none, prime_detection.py:70) */
int msd_stft_plan_set_detrend(msd_stft_plan *plan, int detrend);
/* frames of an n-sample signal (0 if n < nperseg) */
int64_t msd_stft_frames(const msd_stft_plan *plan, int64_t n);
/* batch, device-resident: file f occupies x[off[f] .. off[f]+len[f]) (elements of dtype);
 * its spectrogram is out[f*K*ld + k*ld + t] (ld >= max T, ld % 32 == 0; columns in
 * [T_f, ld) are written with zeros). off/len are DEVICE arrays of nfiles int64. */
int msd_stft_psd_dev(msd_stft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                     int64_t nfiles, int64_t max_frames, float *out, int64_t ld);
/* single signal, host buffers: out is dense float32 [K][T] */
int msd_stft_psd(msd_stft_plan *plan, const void *x, int dtype, int64_t n, float *out, int64_t *frames);
/* the same two for a float64 plan (msd_stft_plan_create_ex with MSD_F64): out is double */
int msd_stft_psd_f64_dev(msd_stft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                         int64_t nfiles, int64_t max_frames, double *out, int64_t ld);
int msd_stft_psd_f64(msd_stft_plan *plan, const void *x, int dtype, int64_t n, double *out, int64_t *frames);

/* --------------------------------------- a2/a3: block band energies → delta
 * Replaces the per-block loop of dsp/src/main.py:352-393:
 *   fft_block = np.fft.rfft(block * np.hanning(B), n=Nf); P = |fft_block|^2
 *   band_dB = 10*log10(sum(P[band]) + 1e-12); noise_dB likewise; delta = band_dB - noise_dB
 * block_size B = int(fs*block_duration_sec); nfft Nf (already doubled, main.py:353);
 * window: the first min(B, Nf) values of np.hanning(B) (float64);
 * band/noise: inclusive bin ranges [lo, hi] of rfftfreq(Nf, 1/fs) selected by the
 * reference masks (hi < lo means an empty band → energy 1e-12). Arithmetic is float64. */
int msd_block_plan_create(msd_ctx *ctx, int64_t block_size, int32_t nfft, const double *window, int32_t band_lo,
                          int32_t band_hi, int32_t noise_lo, int32_t noise_hi, msd_block_plan **out);
void msd_block_plan_destroy(msd_block_plan *plan);
/* batch, device-resident; block count of file f = len[f] / B; outputs [nfiles][ld]
 * (band_db / noise_db may be NULL) */
int msd_block_delta_dev(msd_block_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                        int64_t nfiles, int64_t max_blocks, double *band_db, double *noise_db, double *delta,
                        int64_t ld);
int msd_block_delta(msd_block_plan *plan, const void *x, int dtype, int64_t n, double *band_db, double *noise_db,
                    double *delta, int64_t *blocks);

/* ------------------------------------------------- a4/a5: threshold detector
 * adaptive = 0: get_detections()          dsp/src/main.py:396-448
 * adaptive = 1: get_detections_adaptive() dsp/src/main.py:450-522
 * Block counts are the host's int(x_sec / block_duration_sec) (main.py:458-461).
 * mean/std follow numpy (pairwise summation, population std) in float64 without
 * FMA contraction.  A detection is the block range [start, stop) and the mean of
 * delta over it (the reference's db_mean). */
typedef struct {
    int32_t adaptive;
    int32_t reserved;
    double k_std;                 /* threshold_std_factor              */
    int64_t window_blocks;        /* int(threshold_estimation_window_sec / bs)         */
    int64_t freeze_before_blocks; /* int(threshold_freeze_before_detection_sec / bs)   */
    int64_t freeze_after_blocks;  /* int(threshold_freeze_after_detection_sec / bs)    */
    int64_t fixed_init_blocks;    /* int(threshold_fixed_init_duration_sec / bs)       */
} msd_det_cfg;

typedef struct {
    int64_t start; /* first block                           */
    int64_t stop;  /* one past the last block (t_stop/bs)   */
    double db;     /* np.mean(delta[start:stop])            */
} msd_det;

/* optional per-hour histogram of detection starts (main.py:687-696 Counter of
 * utc_start.replace(minute=0, ...)): bucket = floor((file_start_us[f] +
 * round(start*block_sec*1e6) - base_us) / bucket_us); outside [0, nbuckets) → dropped */
typedef struct {
    const int64_t *file_start_us; /* device, nfiles  */
    int64_t base_us;
    int64_t bucket_us;
    int32_t nbuckets;
    int32_t reserved;
    double block_sec;
    int64_t *counts; /* device, nbuckets, accumulated (not cleared) */
} msd_hist_cfg;

/* status word per file (device int32): 0 ok, 1 zero-duration global detection (reference
 * assert at main.py:437), 2 empty global input (IndexError at main.py:412), 3 capacity */
int msd_detect_dev(msd_ctx *ctx, const double *delta, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                   const msd_det_cfg *cfg, msd_det *dets, int64_t cap, int64_t *counts, double *thresholds,
                   double *margin, int32_t *status, const msd_hist_cfg *hist);
/* single file, host buffers. thresholds (nb) and margin may be NULL.
 * global mode: *thresholds receives the single threshold in thresholds[0]. */
int msd_detect(msd_ctx *ctx, const double *delta, int64_t nb, const msd_det_cfg *cfg, msd_det *dets, int64_t cap,
               int64_t *count, double *thresholds, double *margin);

/* --------------------------------------- C5: two-sided STFT of complex (I/Q) input
 * scipy.signal.spectrogram(z, fs, 'hann', nperseg=N, noverlap=N-hop) for complex z (BASELINE
 * config C5: 192 kHz I/Q, N = 4096, 75 % overlap): two-sided, bins in FFT order (0..N/2-1,
 * -N/2..-1), |X|^2 * scale, constant detrend of the complex frame mean, complex64 arithmetic.
 * window: N float32 (periodic Hann); scale = 1/(fs*sum(w^2)).  nperseg must be 4096.
 * Output FRAME-major: out[(s*max_frames + t)*N + k] (scipy's Sxx[k][t] transposed; a
 * frequency-major tile of 4096 rows would not fit in LDS); frames past a stream's end are 0.
 * off/len: device int64 arrays in complex samples; dtype MSD_CI16 or MSD_CF32. */
typedef struct msd_cstft_plan msd_cstft_plan;
int msd_cstft_plan_create(msd_ctx *ctx, int32_t nperseg, int32_t hop, const float *window, double scale,
                          msd_cstft_plan **out);
void msd_cstft_plan_destroy(msd_cstft_plan *plan);
int msd_cstft_set_detrend(msd_cstft_plan *plan, int detrend);
int64_t msd_cstft_frames(const msd_cstft_plan *plan, int64_t n);
int msd_cstft_psd_dev(msd_cstft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                      int64_t nstreams, int64_t max_frames, float *out);
/* the same, plus (etot != NULL) an upper bound of each frame's total power sum_k out[k] as 16
 * float32 partials, etot[i*stride + s*max_frames + t] (device, stride =
 * msd_cstft_energy_stride(nstreams, max_frames)): Parseval's input norm for the fp32 FFT's
 * per-bin error bound (msd_iq_band_delta_bound_dev); each partial is the max over a group of up to
 * 4 consecutive frames */
int msd_cstft_psd_energy_dev(msd_cstft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                             int64_t nstreams, int64_t max_frames, float *out, float *etot);
/* the same, with each frame's complex sample sum given (frame_sums: device double [nstreams *
 * max_frames][2], (sum I, sum Q) of frame s*max_frames + t, e.g. from msd_iq_delta64_sums_dev):
 * at the C5 hop (1024) the kernel then takes each frame's detrend mean from these sums and computes
 * none itself; other hops ignore them.  Exact sums (int16 input) give output bit-identical to
 * msd_cstft_psd_energy_dev.  Either way the mean is subtracted before the window as an exact
 * two-part float32 value (hi + lo), so the result is scipy's within float32 rounding of the
 * detrended samples whatever the DC offset. */
int msd_cstft_psd_fsums_dev(msd_cstft_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                            int64_t nstreams, int64_t max_frames, float *out, float *etot, const double *frame_sums);
int64_t msd_cstft_energy_stride(int64_t nstreams, int64_t max_frames);
/* one stream, host buffers: n complex samples in, out float32 [T][N] */
int msd_cstft_psd(msd_cstft_plan *plan, const void *x, int dtype, int64_t n, float *out, int64_t *frames);

/* -------------------------------- C5: band / noise dB per frame of the I/Q spectrogram
 * The per-block band energies of dsp/src/main.py:380-393 taken per STFT frame of the two-sided
 * spectrogram (the frame is the detector's block, block_sec = hop/fs):
 *   E = sum(Sxx[mask, t]) + 1e-12;  dB = 10*log10(E);  delta = band_dB - noise_dB
 * with the masks of fftfreq(N, 1/fs) selected as (f >= lo) & (f <= hi).  Bands are inclusive
 * SIGNED bin ranges [lo, hi] in -N/2 .. N/2-1 (contiguous in frequency; bin b < 0 is column
 * b + N of the frame-major row); hi < lo = empty band (E = 1e-12).  spec: device float32
 * [s][max_frames][N] as msd_cstft_psd_dev writes it; frames: device int64 [nstreams];
 * outputs float64 [s*ld + t] (band_db / noise_db may be NULL).  Sums are float64. */
int msd_iq_band_delta_dev(msd_ctx *ctx, const float *spec, int64_t nstreams, int64_t max_frames,
                          const int64_t *frames, int32_t nperseg, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                          int32_t noise_hi, double *band_db, double *noise_db, double *delta, int64_t ld);
/* the same plus ed[s*ld + t] (device float64): a bound on |delta - delta_ref| against the float64
 * reference (scipy's spectrogram of complex128 input, its band sums and dB), from the standard
 * rounding-error model of the fp32 FFT and the frame energies etot of msd_cstft_psd_energy_dev
 * (stream.hip IQ_CHAIN); +inf where a band touches bins -1..1 (the detrend's DC term). */
int msd_iq_band_delta_bound_dev(msd_ctx *ctx, const float *spec, const float *etot, int64_t nstreams,
                                int64_t max_frames, const int64_t *frames, int32_t nperseg, int32_t band_lo,
                                int32_t band_hi, int32_t noise_lo, int32_t noise_hi, double *band_db, double *noise_db,
                                double *delta, double *ed, int64_t ld);

/* -------------------------- C5: the detector over one long stream, time-sharded over ranks
 * get_detections_adaptive() (dsp/src/main.py:450-522) and get_detections() (:396-448) over
 * the delta of ONE stream of n_total frames of which this rank holds [frame0, frame0+n_local).
 * Bit-exact with the reference's numpy arithmetic (pairwise sums in 8192-element chunks,
 * mean + k*std rounded as numpy, no FMA).  The whole-stream mean/std, the W-frame look-back
 * of the adaptive threshold and the freeze/run state at the shard edges are the only things
 * that cross ranks; the host moves them (meteorgpu/stream.py):
 *   1. halos: the tail halo holds the min(W, frame0) frames before frame0, the head halo
 *      the min(head_frames, n_total - frame0 - n_local) frames after the shard;
 *   2. msd_stream_chunk_sums: the pairwise sums of the 8192-frame chunks (of delta, or of
 *      (delta - mean)^2) that START in the shard; in chunk order, s = 0.0; s += c gives
 *      numpy's add.reduce over the whole stream;
 *   3. msd_stream_fresh + msd_stream_refine: every frame's mean + k*std(delta[max(0, i-W):i]) is
 *      state-free but only read where the detector is not frozen.  fresh() writes a cheap
 *      predictor (prefix sums; exact numpy order for windows shorter than W); each scan marks
 *      the 512-frame tiles whose fresh thresholds it read; refine() computes those tiles
 *      numpy-exactly and returns how many it computed.  Scan, refine, scan again until refine
 *      computes nothing: the last scan then read exact thresholds only;
 *   4. msd_stream_scan: the freeze/run scan of the shard from the state entering frame0,
 *      in parallel segments iterated to a fixed point; returns the state after the shard
 *      (rank r+1 enters with rank r's end state: repeat until no entry state changes);
 *   5. msd_stream_runs / msd_stream_db: the shard's runs [start, stop) (start = -1: a run
 *      continued from the previous shard) and their dB means.
 * cfg->adaptive = 0 gives the global detector (every frame uses thr0; the end quirk of
 * main.py:414-415 and the assert of :437 are the host's, on the last shard). */
typedef struct msd_stream_plan msd_stream_plan;
typedef struct {
    int64_t freeze_until; /* freeze_until_idx (main.py:455), -1 initially             */
    int64_t last_stop;    /* last frame of the last run, -2 if there is none           */
    double thr;           /* the `threshold` variable after the previous frame         */
    int64_t src;          /* the frame whose fresh threshold thr is; -1: thr0          */
    double thr_err;       /* certification: thr's error bound against the reference  */
} msd_stream_state;
int msd_stream_plan_create(msd_ctx *ctx, const msd_det_cfg *cfg, int64_t n_total, int64_t frame0, int64_t n_local,
                           int64_t seg_len, int64_t cap_per_seg, int64_t head_frames, msd_stream_plan **out);
void msd_stream_plan_destroy(msd_stream_plan *plan);
/* device pointers into the plan: the shard's delta (n_local, written by the caller, e.g. by
 * msd_iq_band_delta_dev), the tail halo (n_tail = min(W, frame0)), the head halo, and the
 * thresholds actually used per frame (after msd_stream_scan).  Any may be NULL. */
int msd_stream_buffers(msd_stream_plan *plan, double **delta, double **tail, int64_t *n_tail, double **head,
                       int64_t *n_head, double **thresholds);
/* use_mean = 0: sums of delta; 1: sums of (delta - mean)^2.  Synchronous; sums -> host
 * (cap >= chunks), *first_chunk = global index of the first chunk. */
int msd_stream_chunk_sums(msd_stream_plan *plan, int32_t use_mean, double mean, double *sums, int64_t cap,
                          int64_t *nchunks, int64_t *first_chunk);
/* on = 1 (default): every threshold the scan reads is numpy-exact, so the thresholds buffer holds
 * the reference's `thresholds` list.  on = 0 (decisions only): thresholds are predicted with a
 * rounding-error bound, and made exact only for the frames where a decision is within the bound
 * or where a detection holds the threshold; the detections are the same, the thresholds buffer
 * is not the reference's list.  Call before msd_stream_fresh. */
int msd_stream_set_exact_thresholds(msd_stream_plan *plan, int32_t on);
int msd_stream_fresh(msd_stream_plan *plan); /* async; needs the tail halo */
/* decisions-only mode, after msd_stream_fresh and before any refine: the predicted thresholds
 * and their error bounds (n_local each, host; either may be NULL) -- for checking the bound */
int msd_stream_predicted(msd_stream_plan *plan, double *fresh, double *eps);
/* synchronous; *computed = tiles (decisions only: frames) made exact now (0: the previous scan
 * read exact values only where they decide) */
int msd_stream_refine(msd_stream_plan *plan, int32_t *computed);
/* thr0 = mean + k*std of the whole stream.  reset = 1: every segment restarts from the clean
 * state (first call); 2: every segment re-scans from its last fixed-point entry state (after a
 * refine changed thresholds); 0: only the shard's entry state changed.  Synchronous; *rounds =
 * scan launches. */
int msd_stream_scan(msd_stream_plan *plan, double thr0, const msd_stream_state *entry, int32_t reset,
                    msd_stream_state *exit_state, int32_t *rounds);
/* the shard's runs in order, host out; stop is exclusive; margin = min |delta - thr| */
int msd_stream_runs(msd_stream_plan *plan, msd_det *runs, int64_t cap, int64_t *count, double *margin);
/* dets[j].db = np.mean(delta[start:stop]) for global [start, stop) inside the halos + shard */
int msd_stream_db(msd_stream_plan *plan, msd_det *dets, int64_t n);
/* One process holding the whole stream (frame0 = 0, n_local = n_total): the sequence above in
 * one call -- fresh, global threshold, scan / refine to the fixed point, runs (the global
 * mode's end quirk applied), dB means.  out: cap runs, *count of them; *thr0_out = mean +
 * k*std of the stream; *margin = min |delta - threshold read|; *rounds = scans; *refined =
 * exact-threshold work units (tiles, or frames with exact_thresholds = 0).  Errors as the
 * reference: MSD_ERR_INDEX (empty global input), MSD_ERR_ASSERT (zero-duration last run). */
int msd_stream_detect_local(msd_stream_plan *plan, int32_t exact_thresholds, msd_det *out, int64_t cap,
                            int64_t *count, double *thr0_out, double *margin, int32_t *rounds, int32_t *refined);

/* Certification against the float64 reference (C5: delta from the fp32 spectrogram).  With
 * msd_stream_set_certify(plan, 1) every scan also checks each decision delta > thr of the final
 * trajectory against error bounds: ed per frame (|delta - delta_ref|, written by
 * msd_iq_band_delta_bound_dev into msd_stream_error_buffers' local part; halos exchanged like
 * delta's; 0 = exact), the fresh thresholds' bound mean(ed) + |k| rms(ed) over their window
 * (computed by msd_stream_fresh), and thr0's over the whole stream (msd_stream_set_terr0 from the
 * ranks' msd_stream_ed_sums; msd_stream_detect_local computes it itself).  A decision with
 * |delta - thr| <= ed + threshold bound (+ the predictor's bound, decisions only) is uncertain;
 * msd_stream_certificate returns their count, the smallest slack, the largest error zone (ed +
 * threshold bound) of any decision and up to cap of them as
 * (global frame, frame whose window gave the threshold, -1 = thr0).  Zero uncertain decisions:
 * the detections are the reference's.  msd_stream_certificate fails (MSD_ERR_INVALID) unless the
 * plan's last full scan ran with certification on: msd_stream_set_certify invalidates the
 * certificate until the next msd_stream_scan with reset 1 or 2 (or msd_stream_detect_local).
 * msd_iq_delta64_dev: blocks of D = gcd(nperseg, hop) samples run as 16-lane Goertzel rows when D
 * is a multiple of 64, else one lane per block (any D). */
int msd_stream_set_certify(msd_stream_plan *plan, int32_t on);
int msd_stream_error_buffers(msd_stream_plan *plan, double **ed, double **tail, double **head);
int msd_stream_ed_sums(msd_stream_plan *plan, double *sum_ed, double *sum_ed2);
int msd_stream_set_terr0(msd_stream_plan *plan, double sum_ed, double sum_ed2);
int msd_stream_certificate(msd_stream_plan *plan, int64_t *uncertain, double *min_slack, double *max_zone,
                           int64_t *frames, int64_t *srcs, int64_t cap, int64_t *listed);
/* The refinement of uncertain decisions: delta of the frames in `ranges` ([nranges][2] host
 * int64, [first, end) frame indices, sorted and disjoint; frame t starts at complex sample t*hop
 * of x) recomputed in float64 from the samples -- the reference's quantity (scipy spectrogram of
 * complex128 input, periodic Hann, constant detrend, density; band sums in np.sum order;
 * 10*log10(E + 1e-12)) by a direct DFT of the band bins (blocks of gcd(nperseg, hop) samples, the
 * Hann window as three bin taps) -- into delta[t] and its error bound against the reference into
 * ed[t] (device float64).  x: device interleaved I/Q (MSD_CI16 or MSD_CF32), n_samples complex
 * samples.  Asynchronous on the context's stream (the ranges are copied before the call
 * returns; nperseg <= 65536). */
int msd_iq_delta64_dev(msd_ctx *ctx, const void *x, int32_t dtype, int64_t n_samples, int32_t nperseg, int64_t hop,
                       double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo, int32_t noise_hi,
                       const int64_t *ranges, int64_t nranges, double *delta, double *ed);
/* the same, plus each refined frame's complex sample sum (frame_sums[2 t], [2 t + 1]: sum I, sum Q
 * as float64 -- exact for int16 input) for msd_cstft_psd_fsums_dev.  MSD_ERR_UNSUPPORTED (nothing
 * launched) when the block step carries no sums: the int8 path with at most 8 needed bins. */
int msd_iq_delta64_sums_dev(msd_ctx *ctx, const void *x, int32_t dtype, int64_t n_samples, int32_t nperseg,
                            int64_t hop, double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                            int32_t noise_hi, const int64_t *ranges, int64_t nranges, double *delta, double *ed,
                            double *frame_sums);
/* Which block step msd_iq_delta64_dev takes for a geometry (host only, no GPU): int16 input with
 * blocks of D = gcd(nperseg, hop) = 1024 samples, no band touching bin 0 and at most 10 needed
 * bins (band and noise bins +- 1) runs the EXACT integer DFT on the matrix cores (int16 samples as
 * two int8 digits, the twiddles as six balanced base-256 digits, v_mfma_i32_16x16x64_i8, float64
 * combination; bound ~120 u instead of the Goertzel's ~3 L / |sin theta| u) unless
 * MSD_OPT_REFINE_GOERTZEL is set; other D % 64 == 0 the float64 Goertzel rows; any other D one
 * lane per block.  Returns the path (> 0) or an error code. */
#define MSD_REFINE_DIRECT 1
#define MSD_REFINE_GOERTZEL_ROWS 2
#define MSD_REFINE_INT8_MFMA 3
int msd_iq_delta64_path(int32_t nperseg, int64_t hop, double fs, int32_t band_lo, int32_t band_hi, int32_t noise_lo,
                        int32_t noise_hi, int32_t dtype);

/* ------------------------------------------- a10: legacy spectrogram noise floor
 * prime_detection.py:65-91: band_power = np.sum(Pxx[noise_band]) sums the spectrogram over
 * the band's bins AND all frames.  spec: device float32 [nfiles][K][ld] as msd_stft_psd_dev
 * writes it; out[f] (device) = sum over k in [lo, hi], t < frames of spec, float64. */
int msd_spec_band_sum_dev(msd_ctx *ctx, const float *spec, int64_t nfiles, int32_t K, int64_t frames, int64_t ld,
                          int32_t lo, int32_t hi, double *out);
/* the same over a float64 spectrogram (msd_stft_psd_f64_dev: the legacy specgram in mlab's
 * float64) */
int msd_spec_band_sum_f64_dev(msd_ctx *ctx, const double *spec, int64_t nfiles, int32_t K, int64_t frames,
                              int64_t ld, int32_t lo, int32_t hi, double *out);

/* ------------------------------------------------ a8: Welch band powers (phase 2)
 * Replaces, per processing block of dsp/src/live/backend/processor.py:177-206 and :349-369:
 *   f, psd = scipy.signal.welch(block, fs, nfft=n_fft)     (hann, nperseg 256, noverlap 128,
 *                                                           constant detrend, density, mean)
 *   P_band = np.sum(psd[(f >= lo) & (f <= hi)]);  dB = 10*log10(P_band) if P_band > 0 else -inf
 * Samples are converted to float64 and multiplied by sample_scale first (soundfile's float
 * conversion: 1/32768 for PCM16).  window: nperseg float64 (scipy get_window('hann', nperseg));
 * scale: 1/(fs*sum(win^2)) as scipy computes it.  Bands are inclusive bin ranges of
 * rfftfreq(nfft, 1/fs); hi < lo = empty band (P = 0 → -inf).  Arithmetic is float64. */
#define MSD_WELCH_MAX_BANDS 8
typedef struct {
    int32_t block_size; /* int(proc_block_sec * fs) */
    int32_t nperseg;    /* scipy default 256 (or block_size if shorter) */
    int32_t noverlap;   /* scipy default nperseg // 2 */
    int32_t nfft;       /* n_fft (>= nperseg) */
    double sample_scale;
    double scale;
    int32_t nbands;
    int32_t reserved;
    int32_t band_lo[MSD_WELCH_MAX_BANDS];
    int32_t band_hi[MSD_WELCH_MAX_BANDS];
} msd_welch_cfg;
typedef struct msd_welch_plan msd_welch_plan;
int msd_welch_plan_create(msd_ctx *ctx, const msd_welch_cfg *cfg, const double *window, msd_welch_plan **out);
void msd_welch_plan_destroy(msd_welch_plan *plan);
/* batch, device-resident (off/len device int64 arrays as for the STFT); blocks of file f:
 * (len[f] - block_size) / block_size + 1 (the reference's range(0, n - bs + 1, bs));
 * band_db[(f*nbands + j)*ld + b].  psd (may be NULL): the per-block Welch PSD of the band
 * bins, band after band, psd[(f*ld + b)*nslots + slot], nslots = sum of band widths. */
int msd_welch_bands_dev(msd_welch_plan *plan, const void *x, int dtype, const int64_t *off, const int64_t *len,
                        int64_t nfiles, int64_t max_blocks, double *band_db, int64_t ld, double *psd);
/* single signal, host buffers: band_db [nbands][nb] */
int msd_welch_bands(msd_welch_plan *plan, const void *x, int dtype, int64_t n, double *band_db, int64_t *blocks);
/* single signal, host buffers: the per-block PSD of the band bins, psd [nb][nslots] (one band
 * 0..nfft/2 and block_size = n gives scipy.signal.welch(x, fs, ...)'s whole PSD) */
int msd_welch_psd(msd_welch_plan *plan, const void *x, int dtype, int64_t n, double *psd, int64_t *blocks);

/* --------------------------------------------- a9: live detector state machine
 * Replaces processor.py:391-507 (states aggregates.py:4-24) over per-block band dB
 * rows (signal, noise 1, noise 2):
 *   over = sig - mean(n1, n2); hist = the previous min(W, b) values of over (W = 0: all);
 *   thr = mean(hist) + k*std(hist)  (NaN on the first block), replaced by the locked
 *   threshold while Tracking, and while Detection with until > block end;
 *   Init → Detection once block_start >= init_wait; Detection → Tracking when over > thr
 *   (lock = thr + 0*std, start = block start, trigger block not in the history);
 *   Tracking appends over and ends when over < thr: emit if mean >= min_db and
 *   duration >= min_dur, then Detection(lock, until = block start + after_wait).
 * Block b starts at (b*block_size)/fs seconds. */
typedef struct {
    int32_t block_size;
    int32_t avg_win_blocks; /* int(avg_win_sec / proc_block_sec), processor.py:58 */
    double fs;              /* the file's integer sample rate */
    double k_std;
    double init_wait_sec;
    double after_tracking_wait_sec;
    double min_db_mean;
    double min_dur_sec;
} msd_live_cfg;
typedef struct { /* aggregates.py:66-74 DetectedMeteor (+ the block indices) */
    int64_t start_block;
    int64_t stop_block;
    double time_start, time_stop, duration;
    double db_min, db_max, db_mean, db_std;
} msd_meteor;
/* band_db: [(f*3 + j)*ld + b] as msd_welch_bands_dev writes it (3 bands); thresholds / over
 * (may be NULL): [f*ld + b]; counts: meteors found per file (may exceed cap: only cap kept,
 * status 3). */
int msd_live_detect_dev(msd_ctx *ctx, const double *band_db, const int64_t *nblocks, int64_t nfiles, int64_t ld,
                        const msd_live_cfg *cfg, msd_meteor *out, int64_t cap, int64_t *counts, double *thresholds,
                        double *over, int32_t *status);
int msd_live_detect(msd_ctx *ctx, const double *band_db /* [3][nb] */, int64_t nb, const msd_live_cfg *cfg,
                    msd_meteor *out, int64_t cap, int64_t *count, double *thresholds, double *over);

/* ------------------------------------------- a1 / §8(f)1: WAV ingest and uploads
 * scipy.io.wavfile.read semantics for the reference's files (dsp/src/main.py:249; the rules in
 * csrc/wav_parse.h): RIFF little-endian; the sample container is nBlockAlign / nChannels; PCM
 * 1..8 bits → u8, 2-byte → i16, 3-byte → i32 (sample in the top 3 bytes), 4-byte → i32;
 * IEEE float 32 / 64; WAVE_FORMAT_EXTENSIBLE.  msd_wav_read decodes frames
 * [frame0, frame0+nframes) of one channel (channel >= 0) or all (channel = -1, interleaved)
 * with pread straight into dst (host memory; pinned memory from msd_host_alloc lets the
 * upload run asynchronously).  Thread-safe (no shared state). */
typedef struct {
    int32_t rate, channels, bits, format; /* format: 1 PCM, 3 IEEE float */
    int32_t dtype;                        /* MSD_* of the decoded samples */
    int32_t reserved;                     /* the file's bytes per sample (container) */
    int64_t frames;                       /* frames (samples per channel) */
    int64_t data_offset, data_bytes;
} msd_wav_info;
int msd_wav_probe(const char *path, msd_wav_info *info);
int msd_wav_read(const char *path, int32_t channel, int64_t frame0, int64_t nframes, void *dst, int64_t dst_bytes,
                 msd_wav_info *info);
int msd_host_alloc(msd_ctx *ctx, size_t bytes, void **ptr); /* pinned (page-locked) */
int msd_host_free(msd_ctx *ctx, void *ptr);
/* upload on the context's copy stream (overlaps the compute stream) */
int msd_memcpy_h2d_async(msd_ctx *ctx, void *dst, const void *src, size_t bytes);
/* direction 0: work enqueued on the compute stream from now on waits for the uploads enqueued
 * so far; 1: uploads enqueued from now on wait for the compute enqueued so far */
int msd_fence(msd_ctx *ctx, int direction);
int msd_copy_synchronize(msd_ctx *ctx);
/* work enqueued on waiter's stream from now on waits for the work enqueued on signaler's
 * stream so far (two contexts of one device: independent stages of a step run concurrently,
 * e.g. the STFT beside block_delta -> detect in BatchPipeline; no reference counterpart) */
int msd_stream_wait(msd_ctx *waiter, msd_ctx *signaler);

/* ------------------------------------------ multi-GPU: per-hour count reduction
 * RCCL (loaded at run time from librccl.so.1), one communicator per (process, GPU). */
#define MSD_COMM_ID_BYTES 128
int msd_comm_get_unique_id(char *id /* MSD_COMM_ID_BYTES */);
int msd_comm_init(msd_ctx *ctx, int nranks, const char *id, int rank, msd_comm **out);
void msd_comm_destroy(msd_comm *comm);
/* in-place sum of n int64 on the device, on the context stream */
int msd_comm_allreduce_i64(msd_comm *comm, int64_t *dbuf, int64_t n);
/* recv[r*bytes .. (r+1)*bytes) = rank r's send (device buffers, context stream) — the C5
 * stream detector's halo / chunk-sum / shard-state exchange */
int msd_comm_allgather(msd_comm *comm, const void *dsend, void *drecv, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* MSDSP_H */

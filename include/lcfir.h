/*
 * lcfir.h -- C ABI of the MI355X (gfx950) low-cut FIR hot path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (diskerror/audio-fir-filter, "lowcut"):
 *
 *   void apply_filter_range(const VectorMath<float32_t>& channel,
 *                           const WindowedSinc<float64_t>& sinc,
 *                           VectorMath<float32_t>& temp_output,
 *                           int_fast64_t startIdx, int_fast64_t endIdx,
 *                           ThreadSafeProgress* progress);      FilterCore.h:20-27
 *
 * called by N std::threads on disjoint [start,end) chunks of one channel
 * (ProcessFile.cp:60-83), plus the per-file peak/normalize post-pass
 * (ProcessFile.cp:91-101).  Every entry point below names the reference
 * interface it replaces.  Plain C: no exceptions cross this boundary, every
 * function returns an lcfir_status, and lcfir_last_error() holds a
 * thread-local message for the last failure on the calling thread.
 *
 * Semantics of a filtered sample (zero-padded, centred linear convolution,
 * output length = input length):
 *     y[n] = (float) sum_{k=0}^{T-1} h[k] * x[n - M/2 + k],   x[i] = 0 outside [0, N)
 * with T = M + 1 odd taps (WindowedSinc kernel length, getMo2() = M/2),
 * f32 samples, f64 taps, f64 accumulation, one round-to-nearest-even to f32.
 */
#ifndef LCFIR_H
#define LCFIR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LCFIR_ABI_VERSION 1

typedef struct lcfir_ctx lcfir_ctx;

typedef enum lcfir_status {
    LCFIR_OK = 0,
    LCFIR_EINVAL = 1,    /* bad argument (null pointer, even tap count, bad range) */
    LCFIR_EDEVICE = 2,   /* HIP runtime / device error */
    LCFIR_ENOMEM = 3,    /* device or host allocation failed */
    LCFIR_EINTERNAL = 4
} lcfir_status;

/* How the convolution is evaluated.  All methods meet the same parity bar. */
typedef enum lcfir_method {
    LCFIR_METHOD_AUTO = 0,   /* fastest method for the tap count: direct below 64 taps, else FFT */
    LCFIR_METHOD_DIRECT = 1, /* strict-order f64 FMA chain per output (bit-exact vs the
                                oracle's ORACLE_FMA restatement) */
    LCFIR_METHOD_FFT = 2     /* f64 overlap-save FFT convolution, any T up to 2^20 taps (longer
                                than ~10 900 taps: equal partitions summed in f64) */
} lcfir_method;

/* Progress callback: `count` more samples finished.  Replaces
 * ThreadSafeProgress::report(size_t) (ProgressBar.h:69-81). */
typedef void (*lcfir_progress_fn)(void *user, uint64_t count);

/* ---- library --------------------------------------------------------- */
int lcfir_abi_version(void);
const char *lcfir_last_error(void);
/* The library's build id: 16 hex digits of the SHA-256 of the sources it was
 * built from (audio-fir-filter_amd/src_hash.sh), "unknown" for a build outside
 * the Makefile.  bench.py matches PMC sidecars (profiles/traffic_*.json) to
 * the loaded library by it. */
const char *lcfir_build_id(void);
int lcfir_device_count(int *count);

/* ---- filter context ---------------------------------------------------- */
/* Uploads the taps to `device` once.  Replaces the per-file construction of
 * WindowedSinc<float64_t> (ProcessFile.cp:47-50) as seen by the hot path:
 * taps = the kernel, ntaps = M + 1 (must be odd), half = getMo2()
 * (FilterCore.h:29). */
int lcfir_ctx_create(int device, const double *taps, int32_t ntaps, lcfir_ctx **out);
/* Waits for the streams the ctx launched on (not the whole device) and frees
 * its device memory in stream order.  The caller must not destroy a stream
 * that still has work of this ctx queued before calling it. */
int lcfir_ctx_destroy(lcfir_ctx *ctx);
int lcfir_ctx_set_method(lcfir_ctx *ctx, int method);
int lcfir_ctx_get_method(const lcfir_ctx *ctx, int *method);
int lcfir_ctx_half(const lcfir_ctx *ctx, int32_t *half); /* getMo2() */
int lcfir_ctx_ntaps(const lcfir_ctx *ctx, int32_t *ntaps);
/* Diagnostic: the FFT plan this ctx runs (built if needed): overlap-save
 * segment length in real samples, the number of tap partitions, and whether
 * the filter runs in zero-phase form (linear-phase taps).  All 0 when the tap
 * count is outside the FFT method's range. */
int lcfir_ctx_fft_info(lcfir_ctx *ctx, int32_t *seg_len, int32_t *parts, int32_t *zero_phase);
/* Diagnostic: the unit geometry of the same plan.  *outputs: outputs per
 * overlap-save segment (B = seg_len - taps per partition + 1); *kernel: which
 * kernel runs a unit (LCFIR_FFT_KERNEL_*); *nrm_floats: the most floats of a
 * previous file's normalize (lcfir_filter_window_norm_dev) one unit carries
 * inside the filter launch, 0 when that kernel never carries one.  A call
 * fuses the normalize iff d_ny is 16-byte aligned and
 * ceil(ceil(ncount / U) / blk) x blk <= *nrm_floats, where
 * U = nseg x max(1, min(nch, max_units / nseg)) units share it,
 * nseg = ceil(outputs of the call's first launch chunk / B), max_units is
 * lcfir_ctx_set_fft_tuning's (2^31 - 1 by default) and blk = 2 048 floats on
 * the register kernel (LCFIR_FFT_KERNEL_L32_REG), 1 024 on the others.  All 0
 * when the tap count is outside the FFT method's range. */
#define LCFIR_FFT_KERNEL_L16 1      /* fir_fft_f64_kernel: L = 16 384, LDS columns */
#define LCFIR_FFT_KERNEL_L32_PARK 2 /* fir_fft32_f64_kernel: L = 32 768, two halves + park slab */
#define LCFIR_FFT_KERNEL_L32_REG 3  /* fir_fft32r_kernel: L = 32 768 held in registers (zero-phase) */
int lcfir_ctx_fft_units(lcfir_ctx *ctx, int32_t *outputs, int32_t *kernel, int32_t *nrm_floats);
/* Diagnostic: how many previous-file normalizes (lcfir_filter_window_norm_dev
 * with ncount > 0) this ctx carried inside its filter launch (*fused) and how
 * many it ran as their own pass (*separate) since it was created. */
int lcfir_ctx_nrm_stats(const lcfir_ctx *ctx, int64_t *fused, int64_t *separate);
/* Explicit FFT-method choices for this ctx (the library reads no environment
 * variables).  seg_len: 0 = automatic, or 16384 / 32768.  Automatic picks the
 * length with the lower estimated time per output for the taps alone: tap
 * partitions x the measured unit cost (a 32768-sample unit costs 2.2
 * 16384-sample ones on the register kernel, 2.9 on the park-slab kernel) /
 * outputs per segment.  It never depends on a call's
 * shape, so every call on a ctx (range, window, channels, fft_info; every
 * thread, rank or device stage) runs the same plan and the same bytes,
 * whichever call comes first.  zero_phase: 1 = linear-phase filters run in zero-phase form (the
 * default), 0 = always the general pair table; chunk: outputs per launch
 * chunk (0 = 2^28, else >= 4096); max_units: segments x channels per launch
 * (0 = 2^31 - 1).  Every setting gives outputs within 1 f32 ulp of every
 * other (the tests run each); the defaults are the fast ones.  Waits for the
 * ctx's queued launches and drops its plan; not to be called concurrently
 * with launches on the same ctx. */
int lcfir_ctx_set_fft_tuning(lcfir_ctx *ctx, int32_t seg_len, int32_t zero_phase, int64_t chunk,
                             int64_t max_units);
/* Which kernel family runs the ctx's zero-phase single-partition plans:
 * DEFAULT = the transform held in registers at L = 32 768 (fir_fft32r), the
 * LDS-column kernel at L = 16 384; LDS = the LDS-column kernels
 * (fir_fft_f64_kernel, fir_fft32_f64_kernel), which every other plan runs.
 * Outputs agree within 1 f32 ulp either way (tests run each); waits for the
 * ctx's queued launches and drops its plan, as lcfir_ctx_set_fft_tuning.
 * Any other value (2 named round 5's experimental register family, now
 * outside the library) fails with LCFIR_EINVAL. */
#define LCFIR_FFT_FAMILY_DEFAULT 0
#define LCFIR_FFT_FAMILY_LDS 1
int lcfir_ctx_set_fft_family(lcfir_ctx *ctx, int family);
/* Input window [*lo, *hi) (within [0, n)) of a channel of n samples that
 * makes a call for outputs [start, end) reproduce the whole-channel call's
 * outputs bit for bit, whatever the range: the partition invariance of
 * FilterCore.h's per-thread ranges (ProcessFile.cp:60-83).  The direct
 * method needs [start - half, end + half); the FFT method needs the samples
 * of the whole segments the range touches (its segment grid is anchored at
 * output 0), a few thousand more.  A narrower window that still covers
 * [start - half, end + half) gives outputs within 1 f32 ulp of those.
 * Builds the FFT plan if needed. */
int lcfir_ctx_window(lcfir_ctx *ctx, int64_t n, int64_t start, int64_t end, int64_t *lo, int64_t *hi);

/* ---- the hot path: host-pointer range call ----------------------------- */
/* Replaces apply_filter_range(channel, sinc, temp_output, startIdx, endIdx,
 * progress) (FilterCore.h:20-79).  x: the whole channel (n samples, host);
 * y: the caller's output buffer (n samples, host); only y[start, end) is
 * written; x is read over [start - half, end + half) intersected with [0, n).
 * Re-entrant: any number of host threads may call it concurrently on the
 * same ctx with disjoint ranges (the ProcessFile.cp:71-78 pattern).
 * progress may be NULL; otherwise it receives end - start once the range is
 * done (the reference batches reports every 2048 samples, FilterCore.h:38-54). */
int lcfir_apply_range(lcfir_ctx *ctx, const float *x, int64_t n, float *y, int64_t start,
                      int64_t end, lcfir_progress_fn progress, void *user);
/* lcfir_apply_range borrows a staging slot (a HIP stream + grow-only device
 * buffers) per call from a per-device pool of at most 16 slots; callers beyond
 * that wait for a free slot, so the reference's default of floor(0.7 cores)
 * threads per channel (main.cp:75) never creates a stream per thread.
 * lcfir_staging_release frees the idle slots of `device` (-1: every device),
 * and a device's two link queues (page-locked copies) once it has no slot left;
 * lcfir_staging_count reports the slots in existence and the idle ones. */
int lcfir_staging_release(int device);
int lcfir_staging_count(int device, int *live, int *idle);
/* How lcfir_apply_range moves the caller's (pageable) buffers over PCIe.
 * PAGEABLE: the caller's pointers go to hipMemcpyAsync as they are (the
 * runtime pins the pages itself: 35-56 GB/s each way for one thread's 115 MB
 * range on MI355X, but concurrent calls' copies run one at a time).  BOUNCE:
 * a call whose input window is 2-32 MiB (a multi-thread fan-out's share of a
 * channel) is copied whole by the calling thread into its staging slot's
 * page-locked buffers (grow-only, at most 32 MiB each, kept by the slot
 * until lcfir_staging_release; a slot that cannot page-lock them takes the
 * runtime's path) and moved over the
 * device's shared link queues, both ways at once; other calls through two
 * 4 MiB pinned chunks (slower than the runtime for one thread's whole
 * channel).  AUTO (the default): BOUNCE's whole-window path where it applies,
 * PAGEABLE otherwise (config 2's 16-thread fan-out: 0.31-0.45 of the
 * pinned-H2D bound against 0.19-0.22 pageable on one box, alternating).
 * Memory allocated page-locked (hipHostMalloc,
 * lcfir_host_malloc) is copied directly in every mode, on one H2D and one D2H
 * queue per device shared by all calls (the D2H by a kernel through the
 * buffer's device mapping when both ends are 16-byte aligned), so concurrent
 * calls use the link both ways at once.  hipHostRegister'd memory goes to
 * hipMemcpyAsync as it is (the runtime DMAs it directly, on the call's own
 * stream: ROCm 7.2 does not report a registration's extent, so the library
 * cannot prove a range lies in one).  Process-wide; takes effect at the next
 * call. */
typedef enum lcfir_staging_mode {
    LCFIR_STAGING_BOUNCE = 0,
    LCFIR_STAGING_PAGEABLE = 1,
    LCFIR_STAGING_AUTO = 2 /* the default */
} lcfir_staging_mode;
int lcfir_staging_set_mode(int mode);
/* Accounting of lcfir_apply_range calls since the last reset (process-wide).
 * Always: calls, outputs, bytes each way, bounce-staged calls, the calls'
 * host wall time (summed over calls, so concurrent calls add up).  With
 * lcfir_range_profile(1) each call also records HIP events (a few
 * microseconds per call), each on the queue that runs the step -- the
 * device's shared link queues for page-locked buffers of >= 2 MiB, else the
 * call's slot stream: H2D span (first DMA to last; bounce mode: first host
 * chunk copy to last DMA), kernel (samples landed to kernel end), D2H DMA
 * span, summed over the profiled calls.  The copy spans exclude any wait
 * behind other calls' copies on a shared link queue (round 6; round 5's
 * numbers included it). */
typedef struct lcfir_range_stats {
    uint64_t calls;
    uint64_t samples;
    uint64_t h2d_bytes;
    uint64_t d2h_bytes;
    uint64_t staged_calls;
    uint64_t profiled_calls;
    double wall_ms;
    double h2d_ms;
    double kernel_ms;
    double d2h_ms;
} lcfir_range_stats;
int lcfir_range_profile(int enable);
int lcfir_range_stats_get(lcfir_range_stats *out, int reset);

/* ---- device-resident variants (async on a hipStream_t passed as void*) -- */
/* Same as lcfir_apply_range with device pointers; no host synchronisation. */
int lcfir_apply_range_dev(lcfir_ctx *ctx, const float *d_x, int64_t n, float *d_y,
                          int64_t start, int64_t end, void *stream);

/* The whole per-channel loop of ProcessFile.cp:57-87 for nch deinterleaved
 * channels of n samples: channel c at d_x + c*x_stride, output at
 * d_y + c*y_stride (d_y must not alias d_x).  If d_peak is non-NULL it must
 * hold nch floats, zeroed by the caller (or by lcfir_peak_reset_dev); each
 * receives max|y| of its channel (fused into the filter kernel). */
int lcfir_filter_channels_dev(lcfir_ctx *ctx, const float *d_x, int64_t x_stride, int32_t nch,
                              int64_t n, float *d_y, int64_t y_stride, float *d_peak,
                              void *stream);

/* General windowed form, for a file sharded across processes/GPUs by sample
 * range: the caller holds only samples [x_lo, x_hi) of channels that are n
 * samples long (channel c's window at d_xw + c*x_stride, element 0 = sample
 * x_lo) and wants outputs [start, end) (channel c's at d_yw + c*y_stride,
 * element 0 = output y_lo).  The window must cover
 * [max(0, start - half), min(n, end + half)); lcfir_ctx_window's window
 * makes the outputs bit-identical to the whole-channel call's.  d_peak (nullable): channel c's
 * max|y| is max-ed into d_peak[c * peak_stride] (peak_stride 0 folds every
 * channel into one per-file slot, ProcessFile.cp:92-96). */
int lcfir_filter_window_dev(lcfir_ctx *ctx, const float *d_xw, int64_t x_lo, int64_t x_hi,
                            int64_t x_stride, int64_t n, int32_t nch, float *d_yw, int64_t y_lo,
                            int64_t y_stride, int64_t start, int64_t end, float *d_peak,
                            int64_t peak_stride, void *stream);

/* lcfir_filter_window_dev that also carries the PREVIOUS file's normalize
 * (ProcessFile.cp:98-101, applied per file by main.cp:132-147): the ncount
 * contiguous floats at d_ny are rescaled by 1/peak iff peak = max(d_npeak[0,
 * nnpeak)) > 1 or nforce -- exactly lcfir_normalize_dev(d_ny, ncount, 1,
 * ncount, d_npeak, nnpeak, nforce), bit for bit.  The peak slots must be
 * final when the call's work starts (written by earlier work on `stream`).
 * For single-partition FFT filters the rescale rides in the filter launch
 * (the workgroups' older waves do it while waiting at a barrier), so a batch
 * of files needs one normalize pass (the last file's) instead of one per
 * file; otherwise it runs as a separate pass after the filter.  d_ny must
 * not overlap the window or the outputs; ncount = 0 is a plain
 * lcfir_filter_window_dev call (d_ny, d_npeak may then be NULL). */
int lcfir_filter_window_norm_dev(lcfir_ctx *ctx, const float *d_xw, int64_t x_lo, int64_t x_hi,
                                 int64_t x_stride, int64_t n, int32_t nch, float *d_yw, int64_t y_lo,
                                 int64_t y_stride, int64_t start, int64_t end, float *d_peak,
                                 int64_t peak_stride, float *d_ny, int64_t ncount, const float *d_npeak,
                                 int32_t nnpeak, int nforce, void *stream);

/* ---- peak + normalize post-pass (ProcessFile.cp:91-101) ----------------- */
/* max_mag() over each channel (VectorMath::max_mag); d_peak[c] = max(d_peak[c], max|y_c|). */
int lcfir_peak_reset_dev(float *d_peak, int32_t count, void *stream);
int lcfir_peak_dev(const float *d_y, int64_t stride, int32_t nch, int64_t n, float *d_peak,
                   void *stream);
/* Per-file normalize decision and rescale, device-side (no host sync):
 * peak = max over d_peak[0..npeak); if (peak > 1 || force) every sample
 * becomes (float)((double)y * (1.0 / (double)peak)).  The scale rule of
 * c_lib's AudioSamples::normalize is unpinned. */
int lcfir_normalize_dev(float *d_y, int64_t stride, int32_t nch, int64_t n,
                        const float *d_peak, int32_t npeak, int force, void *stream);
/* lcfir_normalize_dev that also zeroes d_clear[0..nclear) in the same launch
 * (a batch driver's next-step peak slots: one launch per step fewer than a
 * separate lcfir_peak_reset_dev).  d_clear must not overlap d_peak[0..npeak)
 * (LCFIR_EINVAL).  nclear 0 = lcfir_normalize_dev. */
int lcfir_normalize_clear_dev(float *d_y, int64_t stride, int32_t nch, int64_t n,
                              const float *d_peak, int32_t npeak, int force, float *d_clear,
                              int32_t nclear, void *stream);
/* Host-pointer convenience: max|y| of one channel (VectorMath::max_mag). */
int lcfir_channel_peak(int device, const float *y, int64_t n, float *peak);

/* ---- tap design (host, long double) ---------------- */
/* Replaces `WindowedSinc<float64_t> sinc(freq / fs, slope / fs); sinc.makeLowCut();`
 * (ProcessFile.cp:47-50): dspguide ch.16 Blackman windowed-sinc low-pass with
 * unity DC gain, then spectral inversion to a high-pass (README.md:50,60-62).
 * Kernel length M + 1 with M = 4 / (slope / fs) rounded to the nearest even
 * integer (c_lib's exact rounding rule is unpinned).  Writes *ntaps; if taps
 * is non-NULL and cap >= *ntaps, also writes the taps.  -s 48 at 48 kHz
 * gives 4001 taps, -s 10 at 48 kHz 19 201. */
int lcfir_design_lowcut(double freq_hz, double slope_hz, double fs, double *taps, int32_t cap,
                        int32_t *ntaps);

/* ---- sample codec either side of the path -------- */
/* Interleaved PCM frames (WAV little-endian / AIFF big-endian) <-> the
 * deinterleaved float32 AudioBuffer the hot path works on.  Replaces, on the
 * device, c_lib's AudioSamples::readAll (ProcessFile.cp:40-41) and
 * AudioSamples::writeAll(buf, true) (:115-117), whose exact conventions are
 * unpinned; ours: int b-bit v <-> v / 2^(b-1), encode rounds half-to-even in
 * f64 and clamps to [-2^(b-1), 2^(b-1) - 1]; float32 is passed through. */
typedef enum lcfir_pcm_format {
    LCFIR_PCM_S16LE = 1,
    LCFIR_PCM_S24LE = 2, /* packed 3-byte */
    LCFIR_PCM_S32LE = 3,
    LCFIR_PCM_F32LE = 4,
    LCFIR_PCM_S16BE = 5,
    LCFIR_PCM_S24BE = 6,
    LCFIR_PCM_S32BE = 7,
    LCFIR_PCM_F32BE = 8
} lcfir_pcm_format;

int lcfir_pcm_bytes(int format); /* bytes per sample, 0 for an unknown format */
/* d_in: frames * nch interleaved samples; channel c goes to d_out + c*out_stride. */
int lcfir_decode_pcm_dev(const void *d_in, int format, int32_t nch, int64_t frames,
                         float *d_out, int64_t out_stride, void *stream);
int lcfir_encode_pcm_dev(const float *d_in, int64_t in_stride, int32_t nch, int64_t frames,
                         int format, void *d_out, void *stream);
/* lcfir_normalize_dev + lcfir_encode_pcm_dev in one pass (ProcessFile.cp:91-101
 * then :115-117): the normalize decision is taken from d_peak[0..npeak) on the
 * device and each sample is scaled exactly as lcfir_normalize_dev would scale
 * it before encoding -- byte-identical output, d_in is left unscaled. */
int lcfir_encode_pcm_scaled_dev(const float *d_in, int64_t in_stride, int32_t nch, int64_t frames,
                                int format, const float *d_peak, int32_t npeak, int force,
                                void *d_out, void *stream);

/* ---- device memory / stream helpers for hosts without a GPU runtime ----- */
int lcfir_dev_malloc(int device, size_t bytes, void **out);
int lcfir_dev_free(void *p);
int lcfir_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream);
int lcfir_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream); /* synchronous */
/* Pinned (page-locked) host memory: H2D/D2H from it run asynchronously at PCIe rate, so a
 * multi-file driver can overlap file i+1's upload and file i-1's download with file i's
 * filtering.  lcfir_memcpy_d2h_async returns once the copy is queued;
 * the caller syncs the stream before touching dst. */
int lcfir_host_malloc(size_t bytes, void **out);
int lcfir_host_free(void *p);
int lcfir_memcpy_d2h_async(void *dst, const void *src, size_t bytes, void *stream);
int lcfir_stream_create(int device, void **stream);
int lcfir_stream_destroy(void *stream);
int lcfir_stream_sync(void *stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* LCFIR_H */

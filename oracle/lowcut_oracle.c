/*
 * lowcut_oracle.c -- CPU restatement of the reference FIR hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (audio-fir-filter_amd/,
 * include/) links, loads or calls this file.  Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() use it, and only as the checker.
 *
 * PARITY STATUS: the convolution structure is pinned by the reference source
 * (FilterCore.h:28-76, ProcessFile.cp:57-101).  The tap dot product
 * `WindowedSinc<float64_t>::fms`, the tap design and `AudioSamples::normalize`
 * live in the un-vendored sibling project c_lib (no pinned version, absent
 * from /root/reference), and the reference ships no
 * tests, fixtures or golden vectors.  Those three pieces are therefore
 * "parity unpinned": they are restated here from their call sites and from the
 * published dspguide algorithm the README credits (README.md:50,60-62).
 * tests/test_oracle.py pins this restatement against an independent exact
 * rational-arithmetic restatement (Python fractions) of the same three loops.
 *
 * Conventions of fms() as implied by its three call sites:
 *   fms(p)          all T taps:      sum_{i<T}   h[i]         * p[i]
 *   fms(p, -c)      LAST c taps:     sum_{i<c}   h[T - c + i] * p[i]
 *   fms(p, +c)      FIRST c taps:    sum_{i<c}   h[i]         * p[i]
 * Summation runs i = 0, 1, ... in that order.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------- */
/* Tap design: dspguide ch.16 Blackman windowed-sinc low-pass, then spectral   */
/* inversion to a high-pass ("makeLowCut").  Reference call site:             */
/* ProcessFile.cp:47-50 `WindowedSinc<float64_t> sinc(freq/fs, slope/fs);     */
/* sinc.makeLowCut();`.  The M(slope) rounding rule of c_lib is unpinned;     */
/* we use dspguide's M = 4/BW rounded to the nearest even integer.            */
/* ------------------------------------------------------------------------- */

int oracle_lowcut_ntaps(double bw_norm) {
    if (!(bw_norm > 0.0)) return -1;
    long double half_m = 2.0L / (long double)bw_norm; /* M/2 */
    long long hm = llroundl(half_m);
    if (hm < 1) hm = 1;
    if (hm > (1LL << 28)) return -1;
    return (int)(2 * hm + 1);
}

/* fc_norm = cutoff / sample rate; ntaps = M + 1 (odd). */
int oracle_design_lowcut(double fc_norm, int ntaps, double *taps) {
    if (ntaps < 1 || (ntaps & 1) == 0) return -1;
    const int M = ntaps - 1;
    const int half = M / 2;
    const long double two_pi = 6.283185307179586476925286766559L;
    long double *h = (long double *)malloc(sizeof(long double) * (size_t)ntaps);
    if (!h) return -2;
    long double sum = 0.0L;
    for (int i = 0; i <= M; ++i) {
        long double v;
        int d = i - half;
        if (d == 0) v = two_pi * (long double)fc_norm;
        else v = sinl(two_pi * (long double)fc_norm * (long double)d) / (long double)d;
        long double w = 1.0L;
        if (M > 0)
            w = 0.42L - 0.5L * cosl(two_pi * (long double)i / (long double)M)
                + 0.08L * cosl(2.0L * two_pi * (long double)i / (long double)M);
        h[i] = v * w;
        sum += h[i];
    }
    for (int i = 0; i <= M; ++i) h[i] = -(h[i] / sum); /* unity DC gain, inverted */
    h[half] += 1.0L;                                   /* spectral inversion */
    for (int i = 0; i <= M; ++i) taps[i] = (double)h[i];
    free(h);
    return 0;
}

/* ------------------------------------------------------------------------- */
/* fms restatements.                                                          */
/* ------------------------------------------------------------------------- */

/* Sum of h[h0 + i] * p[i] for i in [0, cnt) in long double. */
static long double dot_ld(const double *h, const float *p, int64_t cnt) {
    long double acc = 0.0L;
    for (int64_t i = 0; i < cnt; ++i) acc += (long double)h[i] * (long double)p[i];
    return acc;
}

/* Same sum as a strict-order chain of IEEE double fused multiply-adds. */
static double dot_fma(const double *h, const float *p, int64_t cnt) {
    double acc = 0.0;
    for (int64_t i = 0; i < cnt; ++i) acc = fma(h[i], (double)p[i], acc);
    return acc;
}

/* Same sum, plain double multiply then add (what a non-FMA build does). */
static double dot_mul_add(const double *h, const float *p, int64_t cnt) {
    double acc = 0.0;
    for (int64_t i = 0; i < cnt; ++i) acc += h[i] * (double)p[i];
    return acc;
}

enum { ORACLE_LD = 0, ORACLE_FMA = 1, ORACLE_MULADD = 2 };

static long double dot_mode(int mode, const double *h, const float *p, int64_t cnt) {
    switch (mode) {
    case ORACLE_FMA: return (long double)dot_fma(h, p, cnt);
    case ORACLE_MULADD: return (long double)dot_mul_add(h, p, cnt);
    default: return dot_ld(h, p, cnt);
    }
}

/*
 * apply_filter_range restated: FilterCore.h:20-79.
 *   loop 1 (FilterCore.h:56-61): n in [start, min(end, half)):
 *       y[n] = fms(x, -(n + half + 1))   -- last n+half+1 taps
 *       The reference reads past x[N-1] here when N <= M (UB); we define
 *       those samples as zero (clip the count at N), i.e. zero padding.
 *   loop 2 (FilterCore.h:63-69): n in [.., min(end, N - half)):
 *       y[n] = fms(x + n - half)          -- all taps
 *   loop 3 (FilterCore.h:71-76): n in [.., end):
 *       y[n] = fms(x + n - half, N - n + half)  -- first taps
 *   Each output narrowed with static_cast<float32_t> (round to nearest even).
 * y64 (nullable) receives the un-narrowed accumulator, rounded to double.
 */
void oracle_apply_filter_range(const float *x, int64_t n_samples, const double *h, int ntaps,
                               float *y, double *y64, int64_t start, int64_t end, int mode) {
    const int64_t N = n_samples;
    const int64_t half = (int64_t)((ntaps - 1) / 2); /* getMo2() */
    const int64_t start_safe = half;
    const int64_t end_safe = N - half;
    int64_t n = start;
    for (; n < end && n < start_safe; ++n) {
        int64_t overlap = n + half + 1;
        int64_t cnt = overlap < N ? overlap : N; /* zero-pad instead of UB read */
        long double v = dot_mode(mode, h + (ntaps - overlap), x, cnt);
        y[n] = (float)(double)v;
        if (y64) y64[n] = (double)v;
    }
    int64_t safe_limit = end < end_safe ? end : end_safe;
    for (; n < safe_limit; ++n) {
        long double v = dot_mode(mode, h, x + n - half, ntaps);
        y[n] = (float)(double)v;
        if (y64) y64[n] = (double)v;
    }
    for (; n < end; ++n) {
        int64_t remaining = N - n + half;
        long double v = dot_mode(mode, h, x + n - half, remaining);
        y[n] = (float)(double)v;
        if (y64) y64[n] = (double)v;
    }
}

/*
 * Narrowing note: (float)(double)v double-rounds a long double.  For the
 * ORACLE_LD mode we want one rounding, long double -> float, so provide it.
 */
void oracle_apply_filter_range_ld1(const float *x, int64_t n_samples, const double *h, int ntaps,
                                   float *y, double *y64, int64_t start, int64_t end) {
    const int64_t N = n_samples;
    const int64_t half = (int64_t)((ntaps - 1) / 2);
    for (int64_t n = start; n < end; ++n) {
        long double v;
        if (n < half) {
            int64_t overlap = n + half + 1;
            int64_t cnt = overlap < N ? overlap : N;
            v = dot_ld(h + (ntaps - overlap), x, cnt);
        } else if (n < N - half) {
            v = dot_ld(h, x + n - half, ntaps);
        } else {
            v = dot_ld(h, x + n - half, N - n + half);
        }
        y[n] = (float)v;
        if (y64) y64[n] = (double)v;
    }
}

/* ------------------------------------------------------------------------- */
/* Chunk hand-off: ProcessFile.cp:57-87.  chunk = N / threads, the last      */
/* thread takes the remainder, every thread writes a disjoint [start,end).   */
/* ------------------------------------------------------------------------- */

typedef struct {
    const float *x;
    int64_t n;
    const double *h;
    int ntaps;
    float *y;
    int64_t start, end;
    int mode;
} range_job;

static void *range_worker(void *arg) {
    range_job *j = (range_job *)arg;
    if (j->mode == ORACLE_LD)
        oracle_apply_filter_range_ld1(j->x, j->n, j->h, j->ntaps, j->y, NULL, j->start, j->end);
    else
        oracle_apply_filter_range(j->x, j->n, j->h, j->ntaps, j->y, NULL, j->start, j->end, j->mode);
    return NULL;
}

int oracle_filter_channel_mt(const float *x, int64_t n, const double *h, int ntaps, float *y,
                             int nthreads, int mode) {
    if (nthreads < 1) nthreads = 1;
    pthread_t *tid = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
    range_job *jobs = (range_job *)calloc((size_t)nthreads, sizeof(range_job));
    if (!tid || !jobs) { free(tid); free(jobs); return -2; }
    const int64_t chunk = n / nthreads;
    for (int i = 0; i < nthreads; ++i) {
        jobs[i].x = x; jobs[i].n = n; jobs[i].h = h; jobs[i].ntaps = ntaps; jobs[i].y = y;
        jobs[i].start = (int64_t)i * chunk;
        jobs[i].end = (i == nthreads - 1) ? n : jobs[i].start + chunk;
        jobs[i].mode = mode;
    }
    int rc = 0;
    int spawned = 0;
    for (int i = 0; i < nthreads; ++i) {
        if (pthread_create(&tid[i], NULL, range_worker, &jobs[i]) != 0) { rc = -3; break; }
        ++spawned;
    }
    for (int i = 0; i < spawned; ++i) pthread_join(tid[i], NULL);
    free(tid);
    free(jobs);
    return rc;
}

/* ------------------------------------------------------------------------- */
/* Peak + normalize: ProcessFile.cp:91-101.  max_mag is max |y| over the     */
/* channel; AudioSamples::normalize's scale rule is unpinned (c_lib); we     */
/* scale every sample by 1/peak computed in double and round to float.      */
/* ------------------------------------------------------------------------- */

float oracle_max_mag(const float *y, int64_t n) {
    float m = 0.0f;
    for (int64_t i = 0; i < n; ++i) {
        float a = fabsf(y[i]);
        if (a > m) m = a;
    }
    return m;
}

void oracle_scale(float *y, int64_t n, double gain) {
    for (int64_t i = 0; i < n; ++i) y[i] = (float)((double)y[i] * gain);
}

/* Full per-file compute path (ProcessFile.cp:57-101) on deinterleaved
 * channels laid out [nch][n]; returns the pre-normalize peak. */
float oracle_process_buffer(float *buf, int nch, int64_t n, const double *h, int ntaps,
                            int nthreads, int normalize, int mode, float *tmp) {
    for (int c = 0; c < nch; ++c) {
        oracle_filter_channel_mt(buf + (int64_t)c * n, n, h, ntaps, tmp, nthreads, mode);
        memcpy(buf + (int64_t)c * n, tmp, sizeof(float) * (size_t)n);
    }
    float peak = 0.0f;
    for (int c = 0; c < nch; ++c) {
        float m = oracle_max_mag(buf + (int64_t)c * n, n);
        if (m > peak) peak = m;
    }
    if ((peak > 1.0f || normalize) && peak > 0.0f) {
        double gain = 1.0 / (double)peak;
        for (int c = 0; c < nch; ++c) oracle_scale(buf + (int64_t)c * n, n, gain);
    }
    return peak;
}

/* Outputs at an arbitrary list of positions (same arithmetic as
 * oracle_apply_filter_range / _ld1 at n): lets the tests check full-size
 * GPU runs at sampled positions without an O(N*T) CPU pass. */
void oracle_filter_points(const float *x, int64_t n_samples, const double *h, int ntaps,
                          const int64_t *idx, int64_t count, float *out, double *out64,
                          int mode) {
    float y1;
    double y64;
    for (int64_t i = 0; i < count; ++i) {
        const int64_t n = idx[i];
        /* the range functions index y by the global position: shift the base */
        if (mode == ORACLE_LD)
            oracle_apply_filter_range_ld1(x, n_samples, h, ntaps, &y1 - n, &y64 - n, n, n + 1);
        else
            oracle_apply_filter_range(x, n_samples, h, ntaps, &y1 - n, &y64 - n, n, n + 1, mode);
        out[i] = y1;
        if (out64) out64[i] = y64;
    }
}

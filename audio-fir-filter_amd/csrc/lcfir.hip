// lcfir.hip -- C ABI (include/lcfir.h) over the gfx950 FIR kernels.
//
// Host-side responsibilities:
//   * one lcfir_ctx per (device, filter): the taps live in HBM for the life
//     of the context (the reference builds its WindowedSinc once per file,
//     ProcessFile.cp:47-50);
//   * lcfir_apply_range: the reference's apply_filter_range call
//     (FilterCore.h:20-27) on host buffers, re-entrant for the concurrent
//     disjoint-range calls of ProcessFile.cp:71-78.  Each call borrows a
//     staging slot (stream + device buffers) from a per-device pool, copies
//     x[start-half, end+half) in, runs the kernel, copies y[start,end) out
//     (page-locked caller buffers through the device's two link queues, one
//     per direction, so concurrent calls move data both ways at once);
//   * device-pointer entry points that never synchronise the host.
// No CPU fallback exists: if the device or the kernels are unusable every
// call fails with LCFIR_EDEVICE and a message.
#include "lcfir.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <string>
#include <vector>

#include "codec.hpp"
#include "fir_direct.hpp"
#include "fir_fft.hpp"
#include "peak_scale.hpp"

struct lcfir_ctx {
    int device = 0;
    int32_t ntaps = 0;
    int32_t half = 0;
    int method = LCFIR_METHOD_AUTO;
    double *d_taps = nullptr;
    lcfir::FftPlan fft; // frequency-domain filter, built lazily
    lcfir::FftTuning tune; // lcfir_ctx_set_fft_tuning; the next plan build uses it
    std::mutex fft_mu;
    // The ctx's device memory is stream-ordered (hipMallocAsync on `own`), so
    // destroying a ctx frees it without hipFree's implicit device-wide
    // synchronisation: lcfir_ctx_destroy waits for the streams in `used` only.
    hipStream_t own = nullptr;
    std::mutex streams_mu;
    std::vector<hipStream_t> used; // every stream a launch of this ctx went to
    // partitioned FFT filters: f64 partial-sum scratch, one grow-only buffer
    // per stream (stream order keeps a stream's launches from racing on its own
    // buffer; different streams never share one)
    struct Scratch {
        hipStream_t stream;
        double *p;
        size_t cap;    // doubles
        bool captured; // a HIP graph captured on `stream` holds p: never freed before lcfir_ctx_destroy
    };
    std::vector<Scratch> scratch;
    std::vector<double *> retired; // outgrown scratch that a captured graph may still use
    // a HIP graph captured a launch of the current plan: its tables (kernel
    // arguments of that graph) are retired, not freed, when the tuning drops
    // the plan (lcfir_ctx_set_fft_tuning), and freed by lcfir_ctx_destroy
    bool plan_captured = false;
    std::vector<lcfir::FftPlan> retired_plans;
    // previous-file normalizes (lcfir_filter_window_norm_dev): carried inside
    // the filter launch / run as their own pass (lcfir_ctx_nrm_stats)
    std::atomic<int64_t> nrm_fused{0}, nrm_separate{0};
};

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define LCFIR_HIP(expr)                                                                          \
    do {                                                                                         \
        hipError_t e_ = (expr);                                                                  \
        if (e_ != hipSuccess)                                                                    \
            return fail(LCFIR_EDEVICE, "%s failed: %s", #expr, hipGetErrorString(e_));           \
    } while (0)

struct DeviceGuard {
    int prev = -1;
    bool ok = false;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

// ---- direct kernel configuration ---------------------------------------
constexpr int kDirR = 16;   // outputs per lane
constexpr int kDirNT = 256; // threads per workgroup (4 waves)
constexpr int kDirTC = 256; // taps per LDS stage -> 37 KB LDS per workgroup
// workgroups per CU the grid is capped at: the VGPR budget's waves per SIMD
// (each workgroup puts one wave on every SIMD)
constexpr int kDirWgPerCu = lcfir::kDirectWavesPerSimd;

// Compute units of the current device (cached per device id).
int device_cus() {
    static std::atomic<int> cache[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return c;
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0)
        c = 256;
    cache[dev].store(c, std::memory_order_relaxed);
    return c;
}

int launch_direct(lcfir::DirectParams p, int nch, hipStream_t s) {
    const int64_t count = p.end - p.start;
    if (count <= 0 || nch <= 0) return LCFIR_OK;
    constexpr int BO = kDirR * kDirNT;
    if (nch > 65535) return fail(LCFIR_EINVAL, "range too large for one launch");
    // tile-looping grid: what the chip holds at once (kDirWgPerCu per CU,
    // split over the channels), fir_direct.hpp
    const int64_t tiles = (count + BO - 1) / BO;
    const int64_t cap = std::max<int64_t>(1, (int64_t)device_cus() * kDirWgPerCu / nch);
    const int64_t gx = std::min(tiles, cap);
    constexpr size_t lds = lcfir::direct_lds_bytes<kDirR, kDirNT, kDirTC>();
    auto *kern = &lcfir::fir_direct_f64_kernel<kDirR, kDirNT, kDirTC>;
    static std::once_flag attr_once;
    std::call_once(attr_once, [&] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void *>(kern),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    });
    hipLaunchKernelGGL(kern, dim3((unsigned)gx, nch), dim3(kDirNT), lds, s, p);
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int resolve_method(lcfir_ctx *ctx) {
    if (ctx->method != LCFIR_METHOD_AUTO) return ctx->method;
    return lcfir::fft_preferred(ctx->ntaps) ? LCFIR_METHOD_FFT : LCFIR_METHOD_DIRECT;
}

// The FFT plan, built at the first use.  Its segment length (unless tuned) is
// a function of the taps alone (lcfir::fft_choose_seg_len), so every call on
// a ctx -- the reference's per-thread ranges, a rank's window of a split
// file, a multi-channel launch, fft_info -- runs the same segment grid and
// gives the same bytes, whichever comes first.
int ensure_fft(lcfir_ctx *ctx) {
    std::lock_guard<std::mutex> lk(ctx->fft_mu);
    if (ctx->fft.ready) return LCFIR_OK;
    std::string err;
    if (!lcfir::fft_plan_build(ctx->fft, ctx->d_taps, ctx->ntaps, ctx->tune, ctx->own, err))
        return fail(LCFIR_EDEVICE, "fft plan: %s", err.c_str());
    return LCFIR_OK;
}

// Remember stream s as one that launched on ctx (lcfir_ctx_destroy waits for it).
void note_stream(lcfir_ctx *ctx, hipStream_t s) {
    std::lock_guard<std::mutex> lk(ctx->streams_mu);
    for (hipStream_t u : ctx->used)
        if (u == s) return;
    ctx->used.push_back(s);
}

// The partial-sum scratch of stream s, at least `need` doubles, allocated and
// (when it grows) freed in s's own order: no device-wide synchronisation.
// Under HIP graph capture the scratch must already be large enough (an eager
// call of the same shape on s sizes it): a graph keeps the raw pointer, so an
// allocation made inside the capture, or a later growth that freed the
// captured buffer, would leave the graph writing freed memory.  A buffer a
// graph captured is retired on growth, not freed (lcfir_ctx_destroy frees it).
double *stream_scratch(lcfir_ctx *ctx, hipStream_t s, size_t need, bool &capture_error) {
    capture_error = false;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) != hipSuccess) cs = hipStreamCaptureStatusNone;
    const bool capturing = cs == hipStreamCaptureStatusActive;
    std::lock_guard<std::mutex> lk(ctx->streams_mu);
    lcfir_ctx::Scratch *slot = nullptr;
    for (auto &e : ctx->scratch)
        if (e.stream == s) slot = &e;
    if (!slot) {
        ctx->scratch.push_back({s, nullptr, 0, false});
        slot = &ctx->scratch.back();
    }
    if (slot->cap < need) {
        if (capturing) {
            capture_error = true;
            return nullptr;
        }
        if (slot->p) {
            if (slot->captured) ctx->retired.push_back(slot->p);
            else (void)hipFreeAsync(slot->p, s);
        }
        slot->p = nullptr;
        slot->cap = 0;
        slot->captured = false;
        if (hipMallocAsync(reinterpret_cast<void **>(&slot->p), need * sizeof(double), s) != hipSuccess)
            return nullptr;
        slot->cap = need;
    }
    if (capturing) slot->captured = true;
    return slot->p;
}

int launch_normalize(float *d_y, int64_t stride, int32_t nch, int64_t n, const unsigned *d_peak, int32_t npeak,
                     int force, unsigned *d_clear, int32_t nclear, hipStream_t s);

// Run the filter for outputs [start, end) of nch channels.  x/y geometry as
// in DirectParams.  nrm (nullable): a previous file's normalize, fused into
// the FFT launch where fft_nrm_fusable, else run as its own pass afterwards.
// track_stream: remember s for lcfir_ctx_destroy's wait (false for the
// staging streams of lcfir_apply_range, which synchronises its stream before
// returning and may destroy it later, lcfir_staging_release).
int run_filter(lcfir_ctx *ctx, lcfir::DirectParams p, int nch, hipStream_t s,
               const lcfir::FftNrm *nrm = nullptr, bool track_stream = true) {
    p.taps = ctx->d_taps;
    p.ntaps = ctx->ntaps;
    p.half = ctx->half;
    if (track_stream) note_stream(ctx, s);
    const int m = resolve_method(ctx);
    if (m == LCFIR_METHOD_FFT) {
        int rc = ensure_fft(ctx);
        if (rc) return rc;
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive) {
            std::lock_guard<std::mutex> lk(ctx->fft_mu);
            ctx->plan_captured = true;
        }
        std::string err;
        // per-stream scratch: the L = 32768 kernel's park slabs, then the
        // partitioned filters' f64 partial sums
        const size_t npark = lcfir::fft32_park_doubles(ctx->fft);
        const size_t need = npark + lcfir::fft_scratch_doubles(ctx->fft, p, nch);
        if (need > 0) {
            bool capture_error = false;
            double *base = stream_scratch(ctx, s, need, capture_error);
            if (capture_error)
                return fail(LCFIR_EINVAL, "FFT scratch of %zu doubles is not allocated on this stream: run "
                            "an eager call of this shape on it before HIP graph capture", need);
            if (!base) return fail(LCFIR_ENOMEM, "FFT scratch of %zu doubles", need);
            p.park = npark ? reinterpret_cast<double2 *>(base) : nullptr;
            p.y64 = ctx->fft.parts > 1 ? base + npark : nullptr;
        }
        const bool fuse = nrm && lcfir::fft_nrm_fusable(ctx->fft, *nrm, p, nch);
        if (!lcfir::fft_launch(ctx->fft, p, nch, s, err, fuse ? nrm : nullptr))
            return fail(LCFIR_EDEVICE, "fft launch: %s", err.c_str());
        if (fuse) ++ctx->nrm_fused;
        if (!nrm || fuse) return LCFIR_OK;
    } else {
        const int rc = launch_direct(p, nch, s);
        if (rc || !nrm) return rc;
    }
    ++ctx->nrm_separate;
    return launch_normalize(nrm->y, nrm->count, 1, nrm->count, nrm->peak, nrm->npeak, nrm->force, nullptr, 0, s);
}

bool ranges_overlap(const void *a, size_t an, const void *b, size_t bn) {
    auto pa = reinterpret_cast<uintptr_t>(a), pb = reinterpret_cast<uintptr_t>(b);
    return pa < pb + bn && pb < pa + an;
}

// ---- staging pool for the host-pointer entry point ------------------------
// The reference's buffers are pageable (std::vector inside VectorMath).
// LCFIR_STAGING_PAGEABLE: the caller's pointers go to hipMemcpyAsync as they
// are: ROCm 7.2 moves one thread's 115 MB range at 35-56 GB/s each way once
// its pages are known, but pins a fresh buffer's pages on the fly and runs
// concurrent calls' copies one at a time (a 16-thread fan-out: copy
// concurrency 1.00, the device idle 60-70 %, profiles/r06_dropin/).
// LCFIR_STAGING_BOUNCE: windows of kLinkMinBytes..kWinBounceMax (a fan-out's
// share of a channel) are copied whole by the calling thread into the slot's
// page-locked buffers, which the link queues then move both ways at once;
// other sizes through two 4 MiB bounce chunks (slower than the runtime's path
// for a whole channel from one thread).  LCFIR_STAGING_AUTO (the default):
// the window bounce where it applies, the runtime's pageable path otherwise --
// alternating on one box, the 16-thread fan-out of config 2's file moved at
// 0.31-0.45 of the pinned-H2D bound against 0.19-0.22 pageable, 4 threads
// 0.29-0.32 against 0.25-0.28 (profiles/r06_dropin/ab_pageable_bounce.log).
// Caller memory that is already pinned by hipHostMalloc is copied directly in
// every mode (host_pinned).
constexpr size_t kBounceBytes = (size_t)4 << 20;

struct Staging {
    int device = 0;
    hipStream_t stream = nullptr;
    float *d_x = nullptr;
    size_t x_cap = 0;
    float *d_y = nullptr;
    size_t y_cap = 0;
    void *h_bounce[2] = {nullptr, nullptr}; // pinned, kBounceBytes each (lazily)
    // BOUNCE mode, windows of kLinkMinBytes..kWinBounceMax: the whole input
    // window and output range in page-locked buffers of the slot (grow-only)
    void *h_win = nullptr, *h_out = nullptr;
    size_t win_cap = 0, out_cap = 0;
    hipEvent_t bev[2] = {nullptr, nullptr}; // the last DMA touching h_bounce[b] is done
    // lcfir_range_profile: H2D start / end, kernel end, D2H start / end, each
    // recorded on the queue that runs that step (the link queues on the link
    // path), so the copy spans exclude the wait behind other calls' copies
    hipEvent_t tev[5] = {};
    // link path (pinned caller buffers): slot stream ready / H2D landed /
    // kernel done, and the blocking-sync end of the call
    hipEvent_t ev_pre = nullptr, ev_in = nullptr, ev_k = nullptr, done = nullptr;
    bool linked = false; // this call queued copies on the device's link queues
};

// The host link's two directions, shared by every call on a device
// (page-locked caller buffers only).  ROCm 7.2 on MI355X moves 57 GB/s one
// way and 97 GB/s both ways at once when ONE stream carries each direction,
// but 52-63 GB/s in total when eight streams split the same bytes
// (tools/pcie_duplex.hip, profiles/r05_dropin/); the 16 concurrent calls of
// ProcessFile.cp:71-78 each on its own stream ran their copies one after the
// other (a rocprofv3 memory-copy trace of tests/cpp/dropin_bench).  So every
// call's H2D goes on the device's `in` queue and its D2H on the `out` queue, in
// call order, while its kernel runs on the call's own slot stream between
// them (stream events order the three).  The D2H is a kernel writing through
// the buffer's device mapping (pcie_copy) rather than a copy-engine transfer:
// with 16 calls in flight the runtime's D2H into page-locked memory now and
// then held its calling thread for ~8 ms and ran at 12.6 GB/s (HIP API +
// memory-copy trace, profiles/r05_dropin/), which the kernel path does not.
// Calls moving less than kLinkMinBytes one way keep their copies on their own
// slot stream: at the reference's default of 179 threads per channel a call is
// 0.6 MB, and 358 such copies a file one after another on a shared queue cost
// more in per-copy latency than the link's second direction gives back.
constexpr size_t kLinkMinBytes = (size_t)2 << 20;
struct Link {
    std::mutex in_mu, out_mu; // enqueue order = issue order on each queue
    hipStream_t in = nullptr, out = nullptr;
    int device = 0;
};
std::mutex g_link_mu; // taken after g_pool_mu where both are held
std::vector<Link *> g_links; // per device, created on first use; lcfir_staging_release frees them

Link *device_link(int device) {
    std::lock_guard<std::mutex> lk(g_link_mu);
    if ((int)g_links.size() <= device) g_links.resize((size_t)device + 1, nullptr);
    Link *&l = g_links[(size_t)device];
    if (!l) {
        auto *n = new Link;
        n->device = device;
        if (hipStreamCreateWithFlags(&n->in, hipStreamNonBlocking) != hipSuccess ||
            hipStreamCreateWithFlags(&n->out, hipStreamNonBlocking) != hipSuccess) {
            if (n->in) (void)hipStreamDestroy(n->in);
            delete n;
            return nullptr;
        }
        l = n;
    }
    return l;
}

int ensure_link_events(Staging *st) {
    for (hipEvent_t *e : {&st->ev_pre, &st->ev_in, &st->ev_k})
        if (!*e && hipEventCreateWithFlags(e, hipEventDisableTiming) != hipSuccess) {
            *e = nullptr;
            return fail(LCFIR_EDEVICE, "event creation failed");
        }
    if (!st->done && hipEventCreateWithFlags(&st->done, hipEventBlockingSync | hipEventDisableTiming) != hipSuccess) {
        st->done = nullptr;
        return fail(LCFIR_EDEVICE, "event creation failed");
    }
    return LCFIR_OK;
}

std::atomic<int> g_staging_mode{LCFIR_STAGING_AUTO};
// the runtime's pageable path for what the mode does not bounce
inline bool staging_runtime_path() {
    const int m = g_staging_mode.load(std::memory_order_relaxed);
    return m == LCFIR_STAGING_PAGEABLE || m == LCFIR_STAGING_AUTO;
}
std::atomic<int> g_range_profile{0};
std::mutex g_stats_mu;
lcfir_range_stats g_stats{};

// [p, p + bytes) lies in ONE page-locked host allocation (hipHostMalloc or
// hipHostRegister), which the DMA engine can read as a whole.  Checking only
// the two ends would accept a range that starts in one registration, ends in
// another and is pageable in between (hipMemcpyAsync resolves the allocation
// from the start pointer); such a range is treated as pageable.  ROCm 7.2's
// hipMemGetAddressRange reports a hipHostRegister'd range's size but a null
// base (tools/register_alias.hip, profiles/r06_dropin/register_probe.log), so
// registered memory is not recognised here either: it goes to hipMemcpyAsync
// as it is, and the runtime, which knows the registration, DMAs it directly
// on the call's own stream.
// dev (optional): the range's address in `device`'s mapping of that
// allocation -- null if it has none, or if the allocation was made or
// registered while another device was current (the caller then copies with
// hipMemcpyAsync, which resolves any host allocation, instead of writing
// through a mapping the device may not have)
bool host_pinned(const void *p, size_t bytes, void **dev = nullptr, int device = -1) {
    hipPointerAttribute_t a{};
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost) {
        (void)hipGetLastError();
        return false;
    }
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, const_cast<void *>(p)) != hipSuccess || !base) {
        (void)hipGetLastError();
        return false;
    }
    const auto b = reinterpret_cast<uintptr_t>(base), q = reinterpret_cast<uintptr_t>(p);
    if (!(q >= b && bytes <= size && q - b <= size - bytes)) return false;
    if (dev) {
        void *db = nullptr;
        if (a.device != device) {
            *dev = nullptr;
        } else if (hipHostGetDevicePointer(&db, reinterpret_cast<void *>(b), 0) != hipSuccess || !db) {
            (void)hipGetLastError();
            *dev = nullptr;
        } else {
            *dev = static_cast<char *>(db) + (q - b);
        }
    }
    return true;
}

// Device -> host-mapped copy of a call's outputs (see Link)
__global__ __launch_bounds__(256) void pcie_copy_kernel(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                        int64_t n4, float *__restrict__ dt, const float *__restrict__ st,
                                                        int tail) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += stride) dst[k] = src[k];
    if (blockIdx.x == 0 && (int)threadIdx.x < tail) dt[threadIdx.x] = st[threadIdx.x];
}
// 16-byte aligned ends and whole floats only (else the caller copies with
// hipMemcpyAsync): 256 workgroups stream the float4 body, a dword tail after
bool pcie_copy_fits(const void *dst, const void *src, size_t bytes) {
    const auto a = reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src);
    return (a & 15) == 0 && bytes % 4 == 0;
}
int pcie_copy(void *dst, const void *src, size_t bytes, hipStream_t s) {
    const int64_t n4 = (int64_t)(bytes / 16);
    const int tail = (int)((bytes % 16) / 4);
    hipLaunchKernelGGL(pcie_copy_kernel, dim3(256), dim3(256), 0, s, static_cast<float4 *>(dst),
                       static_cast<const float4 *>(src), n4, static_cast<float *>(dst) + 4 * n4,
                       static_cast<const float *>(src) + 4 * n4, tail);
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

// BOUNCE mode for a call whose window is kLinkMinBytes..kWinBounceMax (a
// multi-thread fan-out's share of a channel): the calling thread copies the
// whole window into the slot's page-locked h_win and the whole output out of
// h_out, and the DMAs between take the device's link queues as page-locked
// caller memory does.  The runtime's pageable path instead pins the caller's
// fresh pages on the fly and runs concurrent calls' copies one at a time
// (profiles/r06_dropin/: copy concurrency 1.00, the device idle 60-70 % of a
// 16-thread fan-out); the slot's buffers are pinned once and reused.  Larger
// windows (one thread per channel) keep the chunked bounce below: one thread's
// memcpy of a whole channel costs more than the runtime's copy.
constexpr size_t kWinBounceMax = (size_t)32 << 20;
// Grow-only page-locked buffer of a slot (at most kWinBounceMax: 16 slots
// hold at most 1 GiB, freed by lcfir_staging_release).  False when the host
// cannot page-lock more; the caller then takes the runtime's path.
bool grow_host(void *&buf, size_t &cap, size_t need) {
    if (cap >= need) return true;
    const size_t want = std::min(std::max(need, cap * 2), std::max(need, kWinBounceMax));
    if (buf) (void)hipHostFree(buf); // the slot's previous call has drained
    buf = nullptr;
    cap = 0;
    if (hipHostMalloc(&buf, want, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        buf = nullptr;
        return false;
    }
    cap = want;
    return true;
}

int ensure_bounce(Staging *st) {
    for (int b = 0; b < 2; ++b) {
        if (!st->h_bounce[b] && hipHostMalloc(&st->h_bounce[b], kBounceBytes, hipHostMallocDefault) != hipSuccess) {
            st->h_bounce[b] = nullptr;
            return fail(LCFIR_ENOMEM, "hipHostMalloc(%zu) for a staging bounce buffer failed", kBounceBytes);
        }
        if (!st->bev[b] && hipEventCreateWithFlags(&st->bev[b], hipEventDisableTiming) != hipSuccess) {
            st->bev[b] = nullptr;
            return fail(LCFIR_EDEVICE, "event creation failed");
        }
    }
    return LCFIR_OK;
}

// Host -> device on the slot's stream.  Pageable source in bounce mode: chunk
// i is copied into bounce i mod 2 once the DMA of chunk i - 2 has left it.
// Returns with the DMAs queued (the host copies done).  tev (optional): its
// [0] and [1] are recorded around the copies on the queue that runs them.
int h2d_staged(Staging *st, void *dst, const void *src, size_t bytes, bool &staged, hipEvent_t *tev = nullptr) {
    staged = false;
    st->linked = false;
    const bool pinned = host_pinned(src, bytes);
    if (pinned && bytes >= kLinkMinBytes) {
        Link *lk = device_link(st->device);
        if (!lk) return fail(LCFIR_EDEVICE, "stream creation failed");
        if (const int rc = ensure_link_events(st)) return rc;
        // the slot's buffers (stream-ordered allocations on st->stream) are
        // ready before the link queue writes them; the kernel waits for the copy
        LCFIR_HIP(hipEventRecord(st->ev_pre, st->stream));
        {
            std::lock_guard<std::mutex> g(lk->in_mu);
            LCFIR_HIP(hipStreamWaitEvent(lk->in, st->ev_pre, 0));
            if (tev) LCFIR_HIP(hipEventRecord(tev[0], lk->in));
            LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, lk->in));
            if (tev) LCFIR_HIP(hipEventRecord(tev[1], lk->in));
            LCFIR_HIP(hipEventRecord(st->ev_in, lk->in));
        }
        st->linked = true;
        LCFIR_HIP(hipStreamWaitEvent(st->stream, st->ev_in, 0));
        return LCFIR_OK;
    }
    if (tev) LCFIR_HIP(hipEventRecord(tev[0], st->stream));
    if (pinned || staging_runtime_path()) {
        LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st->stream));
        if (tev) LCFIR_HIP(hipEventRecord(tev[1], st->stream));
        return LCFIR_OK;
    }
    if (const int rc = ensure_bounce(st)) return rc;
    staged = true;
    auto *d = static_cast<char *>(dst);
    auto *s = static_cast<const char *>(src);
    for (size_t off = 0, i = 0; off < bytes; off += kBounceBytes, ++i) {
        const int b = (int)(i & 1);
        const size_t len = std::min(kBounceBytes, bytes - off);
        if (i >= 2) LCFIR_HIP(hipEventSynchronize(st->bev[b]));
        std::memcpy(st->h_bounce[b], s + off, len);
        LCFIR_HIP(hipMemcpyAsync(d + off, st->h_bounce[b], len, hipMemcpyHostToDevice, st->stream));
        LCFIR_HIP(hipEventRecord(st->bev[b], st->stream));
    }
    if (tev) LCFIR_HIP(hipEventRecord(tev[1], st->stream));
    return LCFIR_OK;
}

// Device -> host after the work queued on the slot's stream; returns once
// dst holds the bytes (stream order: the DMAs wait for the kernel).  tev
// (optional): its [3] and [4] are recorded around the copies on the queue
// that runs them.
int d2h_staged(Staging *st, void *dst, const void *src, size_t bytes, hipEvent_t *tev = nullptr) {
    void *dmap = nullptr;
    const bool pinned = host_pinned(dst, bytes, &dmap, st->device);
    if (pinned && bytes >= kLinkMinBytes) {
        Link *lk = device_link(st->device);
        if (!lk) return fail(LCFIR_EDEVICE, "stream creation failed");
        if (const int rc = ensure_link_events(st)) return rc;
        LCFIR_HIP(hipEventRecord(st->ev_k, st->stream));
        {
            std::lock_guard<std::mutex> g(lk->out_mu);
            LCFIR_HIP(hipStreamWaitEvent(lk->out, st->ev_k, 0));
            if (tev) LCFIR_HIP(hipEventRecord(tev[3], lk->out));
            if (dmap && pcie_copy_fits(dmap, src, bytes)) {
                if (const int rc = pcie_copy(dmap, src, bytes, lk->out)) return rc;
            } else {
                LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, lk->out));
            }
            if (tev) LCFIR_HIP(hipEventRecord(tev[4], lk->out));
            LCFIR_HIP(hipEventRecord(st->done, lk->out));
        }
        st->linked = true;
        // the thread sleeps until its copy lands (a polling wait from 16
        // threads takes the host cores the other calls need to issue theirs)
        LCFIR_HIP(hipEventSynchronize(st->done));
        return LCFIR_OK;
    }
    if (tev) LCFIR_HIP(hipEventRecord(tev[3], st->stream));
    if (pinned || staging_runtime_path()) {
        LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st->stream));
        if (tev) LCFIR_HIP(hipEventRecord(tev[4], st->stream));
        LCFIR_HIP(hipStreamSynchronize(st->stream));
        return LCFIR_OK;
    }
    if (const int rc = ensure_bounce(st)) return rc;
    auto *d = static_cast<char *>(dst);
    auto *s = static_cast<const char *>(src);
    const size_t n = (bytes + kBounceBytes - 1) / kBounceBytes;
    auto enqueue = [&](size_t i) -> int {
        const int b = (int)(i & 1);
        const size_t off = i * kBounceBytes, len = std::min(kBounceBytes, bytes - off);
        LCFIR_HIP(hipMemcpyAsync(st->h_bounce[b], s + off, len, hipMemcpyDeviceToHost, st->stream));
        LCFIR_HIP(hipEventRecord(st->bev[b], st->stream));
        if (tev && i + 1 == n) LCFIR_HIP(hipEventRecord(tev[4], st->stream));
        return LCFIR_OK;
    };
    for (size_t i = 0; i < n && i < 2; ++i)
        if (const int rc = enqueue(i)) return rc;
    for (size_t i = 0; i < n; ++i) {
        const int b = (int)(i & 1);
        const size_t off = i * kBounceBytes, len = std::min(kBounceBytes, bytes - off);
        LCFIR_HIP(hipEventSynchronize(st->bev[b]));
        std::memcpy(d + off, st->h_bounce[b], len);
        if (i + 2 < n)
            if (const int rc = enqueue(i + 2)) return rc;
    }
    return LCFIR_OK;
}

// Slots per device: enough streams to keep a GPU busy from host threads (each
// call is synchronous on its slot), few enough that the reference's default
// of floor(0.7 * cores) threads per channel (main.cp:75) on a large host does
// not create a stream per thread.  Callers beyond the cap wait for a slot.
constexpr int kStagingPerDevice = 16;

std::mutex g_pool_mu;
std::condition_variable g_pool_cv;
std::vector<Staging *> g_pool;   // idle slots
std::vector<int> g_pool_live;    // slots in existence, per device

void free_staging(Staging *s) {
    DeviceGuard g(s->device);
    if (s->d_x) (void)hipFreeAsync(s->d_x, s->stream);
    if (s->d_y) (void)hipFreeAsync(s->d_y, s->stream);
    (void)hipStreamSynchronize(s->stream);
    (void)hipStreamDestroy(s->stream);
    for (int b = 0; b < 2; ++b) {
        if (s->h_bounce[b]) (void)hipHostFree(s->h_bounce[b]);
        if (s->bev[b]) (void)hipEventDestroy(s->bev[b]);
    }
    if (s->h_win) (void)hipHostFree(s->h_win);
    if (s->h_out) (void)hipHostFree(s->h_out);
    for (hipEvent_t e : s->tev)
        if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : {s->ev_pre, s->ev_in, s->ev_k, s->done})
        if (e) (void)hipEventDestroy(e);
    delete s;
}

Staging *borrow_staging(int device) {
    std::unique_lock<std::mutex> lk(g_pool_mu);
    if ((int)g_pool_live.size() <= device) g_pool_live.resize((size_t)device + 1, 0);
    for (;;) {
        // the most recently returned slot first: a fan-out of T threads keeps
        // reusing T slots whose grow-only buffers (device, and the window
        // bounce's page-locked ones) already fit, instead of cycling through
        // every slot the pool has ever made
        for (size_t i = g_pool.size(); i-- > 0;) {
            if (g_pool[i]->device == device) {
                Staging *s = g_pool[i];
                g_pool.erase(g_pool.begin() + (long)i);
                return s;
            }
        }
        if (g_pool_live[(size_t)device] < kStagingPerDevice) break;
        g_pool_cv.wait(lk);
    }
    ++g_pool_live[(size_t)device];
    lk.unlock();
    Staging *s = new Staging;
    s->device = device;
    if (hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        std::lock_guard<std::mutex> lk2(g_pool_mu);
        --g_pool_live[(size_t)device];
        g_pool_cv.notify_one();
        return nullptr;
    }
    return s;
}

void return_staging(Staging *s) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        g_pool.push_back(s);
    }
    g_pool_cv.notify_one();
}

// grow-only staging buffer, stream-ordered on the slot's own stream
int grow(float *&buf, size_t &cap, size_t need, hipStream_t s) {
    if (cap >= need) return LCFIR_OK;
    const size_t want = std::max(need, cap * 2);
    if (buf) (void)hipFreeAsync(buf, s);
    buf = nullptr;
    cap = 0;
    if (hipMallocAsync(reinterpret_cast<void **>(&buf), want * sizeof(float), s) != hipSuccess)
        return fail(LCFIR_ENOMEM, "hipMallocAsync(%zu floats) failed", want);
    cap = want;
    return LCFIR_OK;
}

inline unsigned *peak_bits(float *p) { return reinterpret_cast<unsigned *>(p); }

int stream_blocks(int64_t n, int per_block_elems) {
    int64_t b = (n + per_block_elems - 1) / per_block_elems;
    return (int)std::max<int64_t>(1, std::min<int64_t>(b, 2048));
}

int launch_normalize(float *d_y, int64_t stride, int32_t nch, int64_t n, const unsigned *d_peak, int32_t npeak,
                     int force, unsigned *d_clear, int32_t nclear, hipStream_t s) {
    // grid-stride: 256 blocks per channel already saturate HBM when the pass
    // rescales, and keep the (common) no-op launch short
    const int blocks = std::min(stream_blocks(n, 256 * 16), 256);
    hipLaunchKernelGGL(lcfir::normalize_kernel, dim3(blocks, nch), dim3(256), 0, s, d_y, stride, n, d_peak, npeak,
                       force, d_clear, nclear);
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

// Change the ctx's FFT tuning: launches already queued may still read the
// old plan's tables, so wait for them, then free the plan (or retire it, if a
// captured graph holds it); the next launch builds one with the new tuning.
template <class F>
int retune(lcfir_ctx *ctx, F &&set) {
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    std::lock_guard<std::mutex> lk(ctx->fft_mu);
    {
        std::lock_guard<std::mutex> lk2(ctx->streams_mu);
        for (hipStream_t s : ctx->used) (void)hipStreamSynchronize(s);
    }
    if (ctx->plan_captured) {
        // a captured graph still passes these tables to its kernels
        ctx->retired_plans.push_back(ctx->fft);
        ctx->fft = lcfir::FftPlan{};
        ctx->plan_captured = false;
    } else {
        lcfir::fft_plan_free(ctx->fft, ctx->own);
    }
    LCFIR_HIP(hipStreamSynchronize(ctx->own));
    set(ctx->tune);
    return LCFIR_OK;
}

} // namespace

extern "C" {

int lcfir_abi_version(void) { return LCFIR_ABI_VERSION; }

const char *lcfir_last_error(void) { return g_err.c_str(); }

#ifndef LCFIR_BUILD_ID
#define LCFIR_BUILD_ID "unknown"
#endif
const char *lcfir_build_id(void) { return LCFIR_BUILD_ID; }

int lcfir_device_count(int *count) {
    if (!count) return fail(LCFIR_EINVAL, "count is null");
    int c = 0;
    LCFIR_HIP(hipGetDeviceCount(&c));
    *count = c;
    return LCFIR_OK;
}

int lcfir_ctx_create(int device, const double *taps, int32_t ntaps, lcfir_ctx **out) {
    if (!out) return fail(LCFIR_EINVAL, "out is null");
    *out = nullptr;
    if (!taps) return fail(LCFIR_EINVAL, "taps is null");
    if (ntaps < 1 || (ntaps & 1) == 0)
        return fail(LCFIR_EINVAL, "ntaps must be odd and >= 1 (kernel length M+1), got %d", ntaps);
    int ndev = 0;
    LCFIR_HIP(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev)
        return fail(LCFIR_EINVAL, "device %d out of range (%d devices)", device, ndev);
    DeviceGuard g(device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", device);
    auto *ctx = new lcfir_ctx;
    ctx->device = device;
    ctx->ntaps = ntaps;
    ctx->half = (ntaps - 1) / 2;
    if (hipStreamCreateWithFlags(&ctx->own, hipStreamNonBlocking) != hipSuccess) {
        delete ctx;
        return fail(LCFIR_EDEVICE, "stream creation failed");
    }
    int rc = LCFIR_OK;
    // zero-padded to a whole number of direct-kernel stages: the kernel reads
    // the taps of a stage rounded up to 2R without a bound check
    const size_t padded = (size_t)(ntaps + kDirTC - 1) / kDirTC * kDirTC;
    if (hipMallocAsync(reinterpret_cast<void **>(&ctx->d_taps), sizeof(double) * padded, ctx->own) != hipSuccess)
        rc = fail(LCFIR_ENOMEM, "hipMallocAsync for %d taps failed", ntaps);
    else if (hipMemsetAsync(ctx->d_taps, 0, sizeof(double) * padded, ctx->own) != hipSuccess ||
             hipMemcpyAsync(ctx->d_taps, taps, sizeof(double) * (size_t)ntaps, hipMemcpyHostToDevice,
                            ctx->own) != hipSuccess ||
             hipStreamSynchronize(ctx->own) != hipSuccess)
        rc = fail(LCFIR_EDEVICE, "tap upload failed");
    if (rc) {
        lcfir_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return LCFIR_OK;
}

int lcfir_ctx_destroy(lcfir_ctx *ctx) {
    if (!ctx) return LCFIR_OK;
    DeviceGuard g(ctx->device);
    // Wait for the streams this ctx launched on -- not the whole device (the
    // host-pointer calls have synchronised theirs already; a stream the caller
    // has destroyed since just reports an error here).  Then every buffer goes
    // back in `own`'s order, without hipFree's device-wide synchronisation.
    for (hipStream_t s : ctx->used) (void)hipStreamSynchronize(s);
    for (auto &e : ctx->scratch)
        if (e.p) (void)hipFreeAsync(e.p, ctx->own);
    for (double *p : ctx->retired) (void)hipFreeAsync(p, ctx->own);
    for (lcfir::FftPlan &rp : ctx->retired_plans) lcfir::fft_plan_free(rp, ctx->own);
    lcfir::fft_plan_free(ctx->fft, ctx->own);
    if (ctx->d_taps) (void)hipFreeAsync(ctx->d_taps, ctx->own);
    if (ctx->own) {
        (void)hipStreamSynchronize(ctx->own);
        (void)hipStreamDestroy(ctx->own);
    }
    delete ctx;
    return LCFIR_OK;
}

int lcfir_ctx_set_method(lcfir_ctx *ctx, int method) {
    if (!ctx) return fail(LCFIR_EINVAL, "ctx is null");
    if (method < LCFIR_METHOD_AUTO || method > LCFIR_METHOD_FFT)
        return fail(LCFIR_EINVAL, "unknown method %d", method);
    if (method == LCFIR_METHOD_FFT && !lcfir::fft_supported(ctx->ntaps))
        return fail(LCFIR_EINVAL, "FFT method supports at most %d taps (got %d)",
                    lcfir::kFftMaxTaps, ctx->ntaps);
    ctx->method = method;
    return LCFIR_OK;
}

int lcfir_ctx_get_method(const lcfir_ctx *ctx, int *method) {
    if (!ctx || !method) return fail(LCFIR_EINVAL, "null argument");
    *method = resolve_method(const_cast<lcfir_ctx *>(ctx));
    return LCFIR_OK;
}

int lcfir_ctx_half(const lcfir_ctx *ctx, int32_t *half) {
    if (!ctx || !half) return fail(LCFIR_EINVAL, "null argument");
    *half = ctx->half;
    return LCFIR_OK;
}

int lcfir_ctx_ntaps(const lcfir_ctx *ctx, int32_t *ntaps) {
    if (!ctx || !ntaps) return fail(LCFIR_EINVAL, "null argument");
    *ntaps = ctx->ntaps;
    return LCFIR_OK;
}

int lcfir_ctx_fft_info(lcfir_ctx *ctx, int32_t *seg_len, int32_t *parts, int32_t *zero_phase) {
    if (!ctx || !seg_len || !parts || !zero_phase) return fail(LCFIR_EINVAL, "null argument");
    *seg_len = *parts = *zero_phase = 0;
    if (!lcfir::fft_supported(ctx->ntaps)) return LCFIR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    const int rc = ensure_fft(ctx);
    if (rc != LCFIR_OK) return rc;
    *seg_len = ctx->fft.L;
    *parts = ctx->fft.parts;
    *zero_phase = ctx->fft.sym ? 1 : 0;
    return LCFIR_OK;
}

int lcfir_ctx_fft_units(lcfir_ctx *ctx, int32_t *outputs, int32_t *kernel, int32_t *nrm_floats) {
    if (!ctx || !outputs || !kernel || !nrm_floats) return fail(LCFIR_EINVAL, "null argument");
    *outputs = *kernel = *nrm_floats = 0;
    if (!lcfir::fft_supported(ctx->ntaps)) return LCFIR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    const int rc = ensure_fft(ctx);
    if (rc != LCFIR_OK) return rc;
    *outputs = ctx->fft.B;
    *kernel = ctx->fft.reg32 ? LCFIR_FFT_KERNEL_L32_REG
            : ctx->fft.L == lcfir::kFft32L ? LCFIR_FFT_KERNEL_L32_PARK : LCFIR_FFT_KERNEL_L16;
    *nrm_floats = (int32_t)lcfir::fft_nrm_unit_floats(ctx->fft);
    return LCFIR_OK;
}

int lcfir_ctx_nrm_stats(const lcfir_ctx *ctx, int64_t *fused, int64_t *separate) {
    if (!ctx || !fused || !separate) return fail(LCFIR_EINVAL, "null argument");
    *fused = ctx->nrm_fused.load();
    *separate = ctx->nrm_separate.load();
    return LCFIR_OK;
}

int lcfir_ctx_set_fft_tuning(lcfir_ctx *ctx, int32_t seg_len, int32_t zero_phase, int64_t chunk,
                             int64_t max_units) {
    if (!ctx) return fail(LCFIR_EINVAL, "ctx is null");
    if (seg_len != 0 && seg_len != lcfir::kFftL && seg_len != lcfir::kFft32L)
        return fail(LCFIR_EINVAL, "segment length %d not supported (0, %d or %d)", seg_len, lcfir::kFftL,
                    lcfir::kFft32L);
    if (zero_phase != 0 && zero_phase != 1) return fail(LCFIR_EINVAL, "zero_phase must be 0 or 1");
    if (chunk != 0 && chunk < 4096) return fail(LCFIR_EINVAL, "chunk must be 0 or >= 4096 outputs");
    if (max_units < 0 || max_units >= ((int64_t)1 << 31)) return fail(LCFIR_EINVAL, "max_units out of range");
    return retune(ctx, [&](lcfir::FftTuning &t) {
        t.seg_len = seg_len;
        t.zero_phase = zero_phase;
        t.chunk = chunk;
        t.max_units = max_units;
    });
}

int lcfir_ctx_set_fft_family(lcfir_ctx *ctx, int family) {
    if (!ctx) return fail(LCFIR_EINVAL, "ctx is null");
    static_assert(LCFIR_FFT_FAMILY_DEFAULT == lcfir::kFamilyDefault && LCFIR_FFT_FAMILY_LDS == lcfir::kFamilyLds);
    if (family != LCFIR_FFT_FAMILY_DEFAULT && family != LCFIR_FFT_FAMILY_LDS)
        return fail(LCFIR_EINVAL, "unknown FFT kernel family %d", family);
    return retune(ctx, [&](lcfir::FftTuning &t) { t.family = family; });
}

// [lo, hi) of lcfir_ctx_window, clipped to [0, n); start < end
static int range_window(lcfir_ctx *ctx, int64_t n, int64_t start, int64_t end, int64_t &lo, int64_t &hi) {
    lo = start - ctx->half;
    hi = end + ctx->half;
    if (resolve_method(ctx) == LCFIR_METHOD_FFT) {
        const int rc = ensure_fft(ctx);
        if (rc) return rc;
        lcfir::fft_window(ctx->fft, ctx->half, start, end, lo, hi);
    }
    lo = std::max<int64_t>(0, lo);
    hi = std::max(lo, std::min<int64_t>(n, hi));
    return LCFIR_OK;
}

int lcfir_ctx_window(lcfir_ctx *ctx, int64_t n, int64_t start, int64_t end, int64_t *lo, int64_t *hi) {
    if (!ctx || !lo || !hi) return fail(LCFIR_EINVAL, "null argument");
    if (n < 0 || start < 0 || end < start || end > n)
        return fail(LCFIR_EINVAL, "bad range [%lld, %lld) for n=%lld", (long long)start, (long long)end,
                    (long long)n);
    if (end == start) {
        *lo = *hi = start;
        return LCFIR_OK;
    }
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    int64_t l = 0, h = 0;
    const int rc = range_window(ctx, n, start, end, l, h);
    if (rc) return rc;
    *lo = l;
    *hi = h;
    return LCFIR_OK;
}

int lcfir_apply_range(lcfir_ctx *ctx, const float *x, int64_t n, float *y, int64_t start,
                      int64_t end, lcfir_progress_fn progress, void *user) {
    if (!ctx || !x || !y) return fail(LCFIR_EINVAL, "null argument");
    if (n < 0 || start < 0 || end < start || end > n)
        return fail(LCFIR_EINVAL, "bad range [%lld, %lld) for n=%lld", (long long)start,
                    (long long)end, (long long)n);
    if (end == start) return LCFIR_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    // the samples the range's units read: every thread's range gives the
    // whole-channel outputs bit for bit (ProcessFile.cp:60-83 at any -t)
    int64_t lo = 0, hi = 0;
    if (const int wrc = range_window(ctx, n, start, end, lo, hi)) return wrc;
    const auto t_call = std::chrono::steady_clock::now();
    Staging *st = borrow_staging(ctx->device);
    if (!st) return fail(LCFIR_EDEVICE, "stream creation failed");
    const bool prof = g_range_profile.load(std::memory_order_relaxed) != 0;
    int rc = grow(st->d_x, st->x_cap, (size_t)(hi - lo), st->stream);
    if (!rc) rc = grow(st->d_y, st->y_cap, (size_t)(end - start), st->stream);
    if (!rc && prof)
        for (hipEvent_t &e : st->tev)
            if (!e && hipEventCreate(&e) != hipSuccess) {
                e = nullptr;
                rc = fail(LCFIR_EDEVICE, "event creation failed");
                break;
            }
    bool staged = false;
    const size_t xbytes = sizeof(float) * (size_t)(hi - lo), ybytes = sizeof(float) * (size_t)(end - start);
    const int smode = g_staging_mode.load(std::memory_order_relaxed);
    const bool bounce = smode == LCFIR_STAGING_BOUNCE || smode == LCFIR_STAGING_AUTO;
    // (a slot that cannot page-lock its window buffers takes the runtime's path)
    const bool win_x = bounce && xbytes >= kLinkMinBytes && xbytes <= kWinBounceMax &&
                       !host_pinned(x + lo, xbytes) && grow_host(st->h_win, st->win_cap, xbytes);
    const bool win_y = bounce && ybytes >= kLinkMinBytes && ybytes <= kWinBounceMax &&
                       !host_pinned(y + start, ybytes) && grow_host(st->h_out, st->out_cap, ybytes);
    if (!rc && win_x) {
        // the window through the slot's page-locked h_win, then the link queue
        std::memcpy(st->h_win, x + lo, xbytes);
        rc = h2d_staged(st, st->d_x, st->h_win, xbytes, staged, prof ? st->tev : nullptr);
        staged = true;
    } else if (!rc) {
        rc = h2d_staged(st, st->d_x, x + lo, xbytes, staged, prof ? st->tev : nullptr);
    }
    if (!rc) {
        lcfir::DirectParams p{};
        p.x = st->d_x;
        p.x_lo = lo;
        p.x_hi = hi;
        p.x_stride = 0;
        p.y = st->d_y;
        p.y_lo = start;
        p.y_stride = 0;
        p.start = start;
        p.end = end;
        p.peak = nullptr;
        rc = run_filter(ctx, p, 1, st->stream, nullptr, /*track_stream=*/false);
    }
    if (!rc && prof && hipEventRecord(st->tev[2], st->stream) != hipSuccess)
        rc = fail(LCFIR_EDEVICE, "event record failed");
    if (!rc && win_y) {
        // the outputs into the slot's page-locked h_out over the link queue,
        // then out to the caller
        rc = d2h_staged(st, st->h_out, st->d_y, ybytes, prof ? st->tev : nullptr);
        if (!rc) std::memcpy(y + start, st->h_out, ybytes);
        staged = true;
    } else if (!rc) {
        rc = d2h_staged(st, y + start, st->d_y, ybytes, prof ? st->tev : nullptr);
    }
    if (!rc) {
        hipError_t e = hipStreamSynchronize(st->stream);
        if (e != hipSuccess) rc = fail(LCFIR_EDEVICE, "kernel failed: %s", hipGetErrorString(e));
    }
    if (!rc) {
        // H2D = [0, 1], kernel = [1, 2] (from the samples landing), D2H = [3, 4]
        float ms[3] = {0, 0, 0};
        if (prof) {
            (void)hipEventElapsedTime(&ms[0], st->tev[0], st->tev[1]);
            (void)hipEventElapsedTime(&ms[1], st->tev[1], st->tev[2]);
            (void)hipEventElapsedTime(&ms[2], st->tev[3], st->tev[4]);
        }
        const double wall =
            std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_call).count();
        std::lock_guard<std::mutex> lk(g_stats_mu);
        g_stats.calls += 1;
        g_stats.samples += (uint64_t)(end - start);
        g_stats.h2d_bytes += sizeof(float) * (uint64_t)(hi - lo);
        g_stats.d2h_bytes += sizeof(float) * (uint64_t)(end - start);
        g_stats.staged_calls += staged ? 1 : 0;
        g_stats.wall_ms += wall;
        if (prof) {
            g_stats.profiled_calls += 1;
            g_stats.h2d_ms += ms[0];
            g_stats.kernel_ms += ms[1];
            g_stats.d2h_ms += ms[2];
        }
    }
    if (rc) {
        // no DMA of this call may still touch the bounce buffers or the caller's
        Link *lk = st->linked ? device_link(st->device) : nullptr;
        if (lk) {
            (void)hipStreamSynchronize(lk->in);
            (void)hipStreamSynchronize(lk->out);
        }
        (void)hipStreamSynchronize(st->stream);
    }
    return_staging(st);
    if (!rc && progress) progress(user, (uint64_t)(end - start));
    return rc;
}

int lcfir_staging_set_mode(int mode) {
    if (mode != LCFIR_STAGING_BOUNCE && mode != LCFIR_STAGING_PAGEABLE && mode != LCFIR_STAGING_AUTO)
        return fail(LCFIR_EINVAL, "unknown staging mode %d", mode);
    g_staging_mode.store(mode);
    return LCFIR_OK;
}

int lcfir_range_profile(int enable) {
    g_range_profile.store(enable ? 1 : 0);
    return LCFIR_OK;
}

int lcfir_range_stats_get(lcfir_range_stats *out, int reset) {
    if (!out) return fail(LCFIR_EINVAL, "out is null");
    std::lock_guard<std::mutex> lk(g_stats_mu);
    *out = g_stats;
    if (reset) g_stats = lcfir_range_stats{};
    return LCFIR_OK;
}

int lcfir_staging_release(int device) {
    std::vector<Staging *> idle;
    std::vector<Link *> links;
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        for (size_t i = 0; i < g_pool.size();) {
            if (device < 0 || g_pool[i]->device == device) {
                idle.push_back(g_pool[i]);
                --g_pool_live[(size_t)g_pool[i]->device];
                g_pool.erase(g_pool.begin() + (long)i);
            } else {
                ++i;
            }
        }
        // a device left with no slot has no call in flight (a call holds its
        // slot throughout), and none can start while g_pool_mu is held: its
        // link queues go too (the next pinned call creates them again)
        std::lock_guard<std::mutex> lk2(g_link_mu);
        for (size_t d = 0; d < g_links.size(); ++d)
            if (g_links[d] && (device < 0 || (int)d == device) &&
                (d >= g_pool_live.size() || g_pool_live[d] == 0)) {
                links.push_back(g_links[d]);
                g_links[d] = nullptr;
            }
    }
    g_pool_cv.notify_all();
    for (Staging *st : idle) free_staging(st);
    for (Link *l : links) {
        DeviceGuard g(l->device);
        (void)hipStreamSynchronize(l->in);
        (void)hipStreamSynchronize(l->out);
        (void)hipStreamDestroy(l->in);
        (void)hipStreamDestroy(l->out);
        delete l;
    }
    return LCFIR_OK;
}

int lcfir_staging_count(int device, int *live, int *idle) {
    if (!live || !idle) return fail(LCFIR_EINVAL, "null argument");
    std::lock_guard<std::mutex> lk(g_pool_mu);
    *live = (device >= 0 && device < (int)g_pool_live.size()) ? g_pool_live[(size_t)device] : 0;
    int n = 0;
    for (Staging *st : g_pool) n += st->device == device;
    *idle = n;
    return LCFIR_OK;
}

int lcfir_apply_range_dev(lcfir_ctx *ctx, const float *d_x, int64_t n, float *d_y, int64_t start,
                          int64_t end, void *stream) {
    if (!ctx || !d_x || !d_y) return fail(LCFIR_EINVAL, "null argument");
    if (n < 0 || start < 0 || end < start || end > n)
        return fail(LCFIR_EINVAL, "bad range [%lld, %lld) for n=%lld", (long long)start,
                    (long long)end, (long long)n);
    if (end == start) return LCFIR_OK;
    if (ranges_overlap(d_x, sizeof(float) * (size_t)n, d_y + start,
                       sizeof(float) * (size_t)(end - start)))
        return fail(LCFIR_EINVAL, "output range aliases the input channel");
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    lcfir::DirectParams p{};
    p.x = d_x;
    p.x_lo = 0;
    p.x_hi = n;
    p.y = d_y;
    p.y_lo = 0;
    p.start = start;
    p.end = end;
    return run_filter(ctx, p, 1, reinterpret_cast<hipStream_t>(stream));
}

int lcfir_filter_channels_dev(lcfir_ctx *ctx, const float *d_x, int64_t x_stride, int32_t nch,
                              int64_t n, float *d_y, int64_t y_stride, float *d_peak,
                              void *stream) {
    if (!ctx || !d_x || !d_y) return fail(LCFIR_EINVAL, "null argument");
    if (nch < 0 || n < 0) return fail(LCFIR_EINVAL, "negative size");
    if (nch == 0 || n == 0) return LCFIR_OK;
    if (nch > 1 && (x_stride < n || y_stride < n))
        return fail(LCFIR_EINVAL, "channel stride smaller than channel length");
    const size_t xb = sizeof(float) * (size_t)(x_stride * (nch - 1) + n);
    const size_t yb = sizeof(float) * (size_t)(y_stride * (nch - 1) + n);
    if (ranges_overlap(d_x, xb, d_y, yb)) return fail(LCFIR_EINVAL, "d_y aliases d_x");
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    lcfir::DirectParams p{};
    p.x = d_x;
    p.x_lo = 0;
    p.x_hi = n;
    p.x_stride = x_stride;
    p.y = d_y;
    p.y_lo = 0;
    p.y_stride = y_stride;
    p.start = 0;
    p.end = n;
    p.peak = d_peak ? peak_bits(d_peak) : nullptr;
    p.peak_stride = 1;
    return run_filter(ctx, p, nch, reinterpret_cast<hipStream_t>(stream));
}

static int filter_window(lcfir_ctx *ctx, const float *d_xw, int64_t x_lo, int64_t x_hi, int64_t x_stride,
                         int64_t n, int32_t nch, float *d_yw, int64_t y_lo, int64_t y_stride, int64_t start,
                         int64_t end, float *d_peak, int64_t peak_stride, void *stream,
                         const lcfir::FftNrm *nrm) {
    if (!ctx || !d_xw || !d_yw) return fail(LCFIR_EINVAL, "null argument");
    if (nch < 0 || n < 0 || start < 0 || end < start || end > n)
        return fail(LCFIR_EINVAL, "bad range [%lld, %lld) for n=%lld", (long long)start,
                    (long long)end, (long long)n);
    if (nch == 0 || end == start) return LCFIR_OK;
    const int64_t need_lo = std::max<int64_t>(0, start - ctx->half);
    const int64_t need_hi = std::min<int64_t>(n, end + ctx->half);
    if (x_lo < 0 || x_hi > n || x_lo > need_lo || x_hi < need_hi)
        return fail(LCFIR_EINVAL,
                    "window [%lld, %lld) does not cover the samples [%lld, %lld) the outputs need",
                    (long long)x_lo, (long long)x_hi, (long long)need_lo, (long long)need_hi);
    if (y_lo > start) return fail(LCFIR_EINVAL, "y_lo after start");
    if (nch > 1 && (x_stride < x_hi - x_lo || y_stride < end - y_lo))
        return fail(LCFIR_EINVAL, "channel stride smaller than the window");
    const size_t xb = sizeof(float) * (size_t)(x_stride * (nch - 1) + (x_hi - x_lo));
    const size_t yb = sizeof(float) * (size_t)(y_stride * (nch - 1) + (end - y_lo));
    if (ranges_overlap(d_xw, xb, d_yw, yb)) return fail(LCFIR_EINVAL, "d_yw aliases d_xw");
    DeviceGuard g(ctx->device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
    lcfir::DirectParams p{};
    p.x = d_xw;
    p.x_lo = x_lo;
    p.x_hi = x_hi;
    p.x_stride = x_stride;
    p.y = d_yw;
    p.y_lo = y_lo;
    p.y_stride = y_stride;
    p.start = start;
    p.end = end;
    p.peak = d_peak ? peak_bits(d_peak) : nullptr;
    p.peak_stride = peak_stride;
    return run_filter(ctx, p, nch, reinterpret_cast<hipStream_t>(stream), nrm);
}

int lcfir_filter_window_dev(lcfir_ctx *ctx, const float *d_xw, int64_t x_lo, int64_t x_hi,
                            int64_t x_stride, int64_t n, int32_t nch, float *d_yw, int64_t y_lo,
                            int64_t y_stride, int64_t start, int64_t end, float *d_peak,
                            int64_t peak_stride, void *stream) {
    return filter_window(ctx, d_xw, x_lo, x_hi, x_stride, n, nch, d_yw, y_lo, y_stride, start, end, d_peak,
                         peak_stride, stream, nullptr);
}

int lcfir_filter_window_norm_dev(lcfir_ctx *ctx, const float *d_xw, int64_t x_lo, int64_t x_hi,
                                 int64_t x_stride, int64_t n, int32_t nch, float *d_yw, int64_t y_lo,
                                 int64_t y_stride, int64_t start, int64_t end, float *d_peak,
                                 int64_t peak_stride, float *d_ny, int64_t ncount, const float *d_npeak,
                                 int32_t nnpeak, int nforce, void *stream) {
    if (ncount == 0) // nothing to rescale (d_ny and the peak slots may be null)
        return lcfir_filter_window_dev(ctx, d_xw, x_lo, x_hi, x_stride, n, nch, d_yw, y_lo, y_stride, start, end,
                                       d_peak, peak_stride, stream);
    if (!d_ny || !d_npeak || ncount < 0 || nnpeak < 1) return fail(LCFIR_EINVAL, "bad normalize argument");
    if (!ctx || !d_xw || !d_yw) return fail(LCFIR_EINVAL, "null argument");
    if (nch > 0 && end > start) {
        const size_t xb = sizeof(float) * (size_t)(x_stride * (nch - 1) + (x_hi - x_lo));
        const size_t yb = sizeof(float) * (size_t)(y_stride * (nch - 1) + (end - y_lo));
        const size_t nb = sizeof(float) * (size_t)ncount;
        if (ranges_overlap(d_ny, nb, d_xw, xb) || ranges_overlap(d_ny, nb, d_yw, yb))
            return fail(LCFIR_EINVAL, "d_ny overlaps the window or the outputs");
    }
    lcfir::FftNrm nrm;
    nrm.y = d_ny;
    nrm.peak = reinterpret_cast<const unsigned *>(d_npeak);
    nrm.count = ncount;
    nrm.npeak = nnpeak;
    nrm.force = nforce ? 1 : 0;
    if (nch == 0 || end == start) {
        DeviceGuard g(ctx->device);
        if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", ctx->device);
        return launch_normalize(d_ny, ncount, 1, ncount, nrm.peak, nnpeak, nrm.force, nullptr, 0,
                                reinterpret_cast<hipStream_t>(stream));
    }
    return filter_window(ctx, d_xw, x_lo, x_hi, x_stride, n, nch, d_yw, y_lo, y_stride, start, end, d_peak,
                         peak_stride, stream, &nrm);
}

int lcfir_peak_reset_dev(float *d_peak, int32_t count, void *stream) {
    if (!d_peak || count < 0) return fail(LCFIR_EINVAL, "bad peak buffer");
    if (count == 0) return LCFIR_OK;
    // one small block (the runtime's fill kernel for a hipMemsetAsync of a few
    // bytes costs ~2x as long on the stream)
    hipLaunchKernelGGL(lcfir::peak_zero_kernel, dim3(1), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), peak_bits(d_peak), count);
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int lcfir_peak_dev(const float *d_y, int64_t stride, int32_t nch, int64_t n, float *d_peak,
                   void *stream) {
    if (!d_y || !d_peak || nch < 0 || n < 0) return fail(LCFIR_EINVAL, "bad argument");
    if (nch == 0 || n == 0) return LCFIR_OK;
    if (nch > 65535) return fail(LCFIR_EINVAL, "too many channels");
    const int blocks = stream_blocks(n, 256 * 16);
    hipLaunchKernelGGL(lcfir::peak_kernel, dim3(blocks, nch), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_y, stride, n, peak_bits(d_peak));
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int lcfir_normalize_clear_dev(float *d_y, int64_t stride, int32_t nch, int64_t n, const float *d_peak,
                              int32_t npeak, int force, float *d_clear, int32_t nclear, void *stream) {
    if (!d_y || !d_peak || nch < 0 || n < 0 || npeak < 1 || nclear < 0 || (nclear > 0 && !d_clear))
        return fail(LCFIR_EINVAL, "bad argument");
    if (nch > 65535) return fail(LCFIR_EINVAL, "too many channels");
    if (nclear > 0 && d_clear < d_peak + npeak && d_peak < d_clear + nclear)
        return fail(LCFIR_EINVAL, "the slots to clear overlap the peak slots read");
    if (nch == 0 || n == 0) return nclear > 0 ? lcfir_peak_reset_dev(d_clear, nclear, stream) : LCFIR_OK;
    return launch_normalize(d_y, stride, nch, n, reinterpret_cast<const unsigned *>(d_peak), npeak, force,
                            nclear > 0 ? peak_bits(d_clear) : nullptr, nclear,
                            reinterpret_cast<hipStream_t>(stream));
}

int lcfir_normalize_dev(float *d_y, int64_t stride, int32_t nch, int64_t n, const float *d_peak,
                        int32_t npeak, int force, void *stream) {
    return lcfir_normalize_clear_dev(d_y, stride, nch, n, d_peak, npeak, force, nullptr, 0, stream);
}

int lcfir_channel_peak(int device, const float *y, int64_t n, float *peak) {
    if (!y || !peak || n < 0) return fail(LCFIR_EINVAL, "bad argument");
    *peak = 0.0f;
    if (n == 0) return LCFIR_OK;
    DeviceGuard g(device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", device);
    Staging *st = borrow_staging(device);
    if (!st) return fail(LCFIR_EDEVICE, "stream creation failed");
    int rc = grow(st->d_x, st->x_cap, (size_t)n, st->stream);
    if (!rc) rc = grow(st->d_y, st->y_cap, 1, st->stream);
    if (!rc && hipMemcpyAsync(st->d_x, y, sizeof(float) * (size_t)n, hipMemcpyHostToDevice,
                              st->stream) != hipSuccess)
        rc = fail(LCFIR_EDEVICE, "H2D copy failed");
    if (!rc) rc = lcfir_peak_reset_dev(st->d_y, 1, st->stream);
    if (!rc) rc = lcfir_peak_dev(st->d_x, n, 1, n, st->d_y, st->stream);
    if (!rc && hipMemcpyAsync(peak, st->d_y, sizeof(float), hipMemcpyDeviceToHost, st->stream) !=
                   hipSuccess)
        rc = fail(LCFIR_EDEVICE, "D2H copy failed");
    if (!rc && hipStreamSynchronize(st->stream) != hipSuccess)
        rc = fail(LCFIR_EDEVICE, "peak kernel failed");
    return_staging(st);
    return rc;
}

int lcfir_design_lowcut(double freq_hz, double slope_hz, double fs, double *taps, int32_t cap,
                        int32_t *ntaps) {
    if (!ntaps) return fail(LCFIR_EINVAL, "ntaps is null");
    // freq 0 would make every low-pass tap 0 and the unity-gain normalisation
    // 0/0: NaN taps, an all-zero output file (the low-cut of nothing)
    if (!(fs > 0.0) || !(slope_hz > 0.0) || !(freq_hz > 0.0) || !(freq_hz < fs / 2))
        return fail(LCFIR_EINVAL, "need fs > 0, slope > 0, 0 < freq < fs/2");
    const long double bw = (long double)slope_hz / (long double)fs;
    const long double half_m = 2.0L / bw; // M / 2
    const long long hm = std::max<long long>(1, llroundl(half_m));
    if (hm > (1LL << 26)) return fail(LCFIR_EINVAL, "kernel too long (slope too small)");
    const int32_t T = (int32_t)(2 * hm + 1);
    *ntaps = T;
    if (!taps) return LCFIR_OK;
    if (cap < T) return fail(LCFIR_EINVAL, "cap %d < %d taps", cap, T);
    const int M = T - 1, half = M / 2;
    const long double fc = (long double)freq_hz / (long double)fs;
    const long double two_pi = 6.283185307179586476925286766559L;
    std::vector<long double> h((size_t)T);
    long double sum = 0.0L;
    for (int i = 0; i <= M; ++i) {
        const int d = i - half;
        const long double v = d == 0 ? two_pi * fc : sinl(two_pi * fc * (long double)d) / (long double)d;
        const long double w = 0.42L - 0.5L * cosl(two_pi * (long double)i / (long double)M) +
                              0.08L * cosl(2.0L * two_pi * (long double)i / (long double)M);
        h[(size_t)i] = v * w;
        sum += h[(size_t)i];
    }
    if (!(sum != 0.0L) || !std::isfinite((double)sum))
        return fail(LCFIR_EINVAL, "low-pass taps sum to %g: no unity-gain normalisation", (double)sum);
    for (int i = 0; i <= M; ++i) h[(size_t)i] = -(h[(size_t)i] / sum); // unity DC gain, inverted
    h[(size_t)half] += 1.0L;                                             // spectral inversion
    for (int i = 0; i <= M; ++i) taps[i] = (double)h[(size_t)i];
    return LCFIR_OK;
}

static bool pcm_format(int format, lcfir::PcmFormat &f) {
    switch (format) {
    case LCFIR_PCM_S16LE: f = {2, false, false}; return true;
    case LCFIR_PCM_S24LE: f = {3, false, false}; return true;
    case LCFIR_PCM_S32LE: f = {4, false, false}; return true;
    case LCFIR_PCM_F32LE: f = {4, true, false}; return true;
    case LCFIR_PCM_S16BE: f = {2, false, true}; return true;
    case LCFIR_PCM_S24BE: f = {3, false, true}; return true;
    case LCFIR_PCM_S32BE: f = {4, false, true}; return true;
    case LCFIR_PCM_F32BE: f = {4, true, true}; return true;
    default: return false;
    }
}

int lcfir_pcm_bytes(int format) {
    lcfir::PcmFormat f;
    return pcm_format(format, f) ? f.bytes : 0;
}

int lcfir_decode_pcm_dev(const void *d_in, int format, int32_t nch, int64_t frames,
                         float *d_out, int64_t out_stride, void *stream) {
    lcfir::PcmFormat f;
    if (!pcm_format(format, f)) return fail(LCFIR_EINVAL, "unknown PCM format %d", format);
    if (nch < 0 || frames < 0) return fail(LCFIR_EINVAL, "negative size");
    if (nch == 0 || frames == 0) return LCFIR_OK;
    if (!d_in || !d_out) return fail(LCFIR_EINVAL, "null argument");
    if (nch > 1 && out_stride < frames) return fail(LCFIR_EINVAL, "channel stride < frames");
    const int blocks = stream_blocks(frames * nch, 256 * 8);
    hipLaunchKernelGGL(lcfir::decode_pcm_kernel, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream),
                       reinterpret_cast<const uint8_t *>(d_in), f, (int)nch, frames, d_out,
                       out_stride);
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int lcfir_encode_pcm_dev(const float *d_in, int64_t in_stride, int32_t nch, int64_t frames,
                         int format, void *d_out, void *stream) {
    lcfir::PcmFormat f;
    if (!pcm_format(format, f)) return fail(LCFIR_EINVAL, "unknown PCM format %d", format);
    if (nch < 0 || frames < 0) return fail(LCFIR_EINVAL, "negative size");
    if (nch == 0 || frames == 0) return LCFIR_OK;
    if (!d_in || !d_out) return fail(LCFIR_EINVAL, "null argument");
    if (nch > 1 && in_stride < frames) return fail(LCFIR_EINVAL, "channel stride < frames");
    const int blocks = stream_blocks(frames * nch, 256 * 8);
    hipLaunchKernelGGL(lcfir::encode_pcm_kernel, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_in, in_stride, (int)nch, frames,
                       f, reinterpret_cast<uint8_t *>(d_out));
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int lcfir_encode_pcm_scaled_dev(const float *d_in, int64_t in_stride, int32_t nch, int64_t frames, int format,
                                const float *d_peak, int32_t npeak, int force, void *d_out, void *stream) {
    lcfir::PcmFormat f;
    if (!pcm_format(format, f)) return fail(LCFIR_EINVAL, "unknown PCM format %d", format);
    if (nch < 0 || frames < 0 || npeak < 0) return fail(LCFIR_EINVAL, "negative size");
    if (nch == 0 || frames == 0) return LCFIR_OK;
    if (!d_in || !d_out || (npeak > 0 && !d_peak)) return fail(LCFIR_EINVAL, "null argument");
    if (nch > 1 && in_stride < frames) return fail(LCFIR_EINVAL, "channel stride < frames");
    const int blocks = stream_blocks(frames * nch, 256 * 8);
    hipLaunchKernelGGL(lcfir::encode_pcm_scaled_kernel, dim3(blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), d_in, in_stride, (int)nch, frames, f,
                       reinterpret_cast<const unsigned *>(d_peak), (int)npeak, force ? 1 : 0,
                       reinterpret_cast<uint8_t *>(d_out));
    LCFIR_HIP(hipGetLastError());
    return LCFIR_OK;
}

int lcfir_dev_malloc(int device, size_t bytes, void **out) {
    if (!out) return fail(LCFIR_EINVAL, "out is null");
    *out = nullptr;
    DeviceGuard g(device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", device);
    if (hipMalloc(out, bytes ? bytes : 1) != hipSuccess)
        return fail(LCFIR_ENOMEM, "hipMalloc(%zu) failed", bytes);
    return LCFIR_OK;
}

int lcfir_dev_free(void *p) {
    if (p) LCFIR_HIP(hipFree(p));
    return LCFIR_OK;
}

int lcfir_memcpy_h2d(void *dst, const void *src, size_t bytes, void *stream) {
    if (!bytes) return LCFIR_OK;
    if (!dst || !src) return fail(LCFIR_EINVAL, "null argument");
    LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice,
                             reinterpret_cast<hipStream_t>(stream)));
    return LCFIR_OK;
}

int lcfir_memcpy_d2h(void *dst, const void *src, size_t bytes, void *stream) {
    if (!bytes) return LCFIR_OK;
    if (!dst || !src) return fail(LCFIR_EINVAL, "null argument");
    LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost,
                             reinterpret_cast<hipStream_t>(stream)));
    LCFIR_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return LCFIR_OK;
}

int lcfir_memcpy_d2h_async(void *dst, const void *src, size_t bytes, void *stream) {
    if (!bytes) return LCFIR_OK;
    if (!dst || !src) return fail(LCFIR_EINVAL, "null argument");
    LCFIR_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost,
                             reinterpret_cast<hipStream_t>(stream)));
    return LCFIR_OK;
}

int lcfir_host_malloc(size_t bytes, void **out) {
    if (!out) return fail(LCFIR_EINVAL, "out is null");
    *out = nullptr;
    if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
        return fail(LCFIR_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
    return LCFIR_OK;
}

int lcfir_host_free(void *p) {
    if (p) LCFIR_HIP(hipHostFree(p));
    return LCFIR_OK;
}

int lcfir_stream_create(int device, void **stream) {
    if (!stream) return fail(LCFIR_EINVAL, "stream is null");
    DeviceGuard g(device);
    if (!g.ok) return fail(LCFIR_EDEVICE, "hipSetDevice(%d) failed", device);
    hipStream_t s = nullptr;
    LCFIR_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    *stream = s;
    return LCFIR_OK;
}

int lcfir_stream_destroy(void *stream) {
    if (stream) LCFIR_HIP(hipStreamDestroy(reinterpret_cast<hipStream_t>(stream)));
    return LCFIR_OK;
}

int lcfir_stream_sync(void *stream) {
    LCFIR_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    return LCFIR_OK;
}

} // extern "C"

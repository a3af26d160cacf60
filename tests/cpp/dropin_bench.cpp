// Throughput of the drop-in path as the reference calls it: ProcessFile.cp:57-87's
// per-channel std::thread fan-out over include/lcfir/FilterCore.h's
// apply_filter_range (passed by name, FilterCore.h:20-27), on pageable host
// buffers (VectorMath's std::vector), for BASELINE config 2's file: 10 min
// stereo 48 kHz int24 samples (synthetic), 4001 taps (-f 20 -s 48).
//
// For each staging mode (lcfir_staging_set_mode) and thread count it times
// whole files -- both channels' fork/join, temp_output allocation and the move
// into buf[ch], as ProcessFile.cp does -- and reports Msamples/s, then one more
// file with lcfir_range_profile(1) for the per-call H2D / kernel / D2H split
// (lcfir_range_stats).  Every timed file's output must equal one device-side
// lcfir_filter_channels_dev call over the whole file bit for bit (partition
// invariance); the tool exits 3 otherwise.  This is the host-pointer rate,
// PCIe included: never bench.py's `value`.
//
// usage: dropin_bench [--seconds S] [--threads a,b,...] [--reps R] [--modes auto,pageable,bounce,pinned]
//   --threads: counts; "ref" = floor(0.7 x hardware_concurrency) (main.cp:75-76)
//   modes: the staging mode for pageable buffers, or "pinned": VectorMath's
//   samples in page-locked memory (lcfir_host_malloc; copied directly)
// Prints one JSON line per (mode, threads).
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "reference_types.hpp"

#define LCFIR_DROPIN_TYPES_DECLARED
#include "lcfir/FilterCore.h"

using namespace Diskerror;
using Clock = std::chrono::steady_clock;

static void die(const char *what) {
    std::fprintf(stderr, "dropin_bench: %s: %s\n", what, lcfir_last_error());
    std::exit(2);
}

static std::vector<std::string> split(const std::string &s) {
    std::vector<std::string> out;
    size_t a = 0;
    while (a <= s.size()) {
        size_t b = s.find(',', a);
        if (b == std::string::npos) b = s.size();
        if (b > a) out.push_back(s.substr(a, b - a));
        a = b + 1;
    }
    return out;
}

// one file through ProcessFile.cp:57-87 (call shape unchanged); returns
// seconds, and adds the span of temp_output's construction (ProcessFile.cp:58:
// a zero-filled VectorMath of numFrames, page faults included) and of the
// thread fan-out + join (:60-83, the drop-in calls) to *alloc_s / *fanout_s
static double process_file(std::vector<VectorMath<float>> &buf, const WindowedSinc<double> &sinc,
                           unsigned num_threads, ThreadSafeProgress &safe_progress, double *alloc_s,
                           double *fanout_s) {
    const auto t0 = Clock::now();
    for (size_t ch = 0; ch < buf.size(); ++ch) {
        const size_t numFrames = buf[ch].size();
        const auto ta = Clock::now();
        VectorMath<float> temp_output(numFrames);
        const auto tb = Clock::now();
        std::vector<std::thread> threads;
        threads.reserve(num_threads);
        const auto totalSamples = static_cast<int_fast64_t>(numFrames);
        const int_fast64_t chunkSize = totalSamples / num_threads;
        for (unsigned int i = 0; i < num_threads; ++i) {
            int_fast64_t start = i * chunkSize;
            int_fast64_t end = (i == num_threads - 1) ? totalSamples : (start + chunkSize);
            threads.emplace_back(apply_filter_range, std::cref(buf[ch]), std::cref(sinc), std::ref(temp_output),
                                 start, end, &safe_progress);
        }
        for (auto &t : threads) t.join();
        const auto tc = Clock::now();
        buf[ch] = std::move(temp_output);
        *alloc_s += std::chrono::duration<double>(tb - ta).count();
        *fanout_s += std::chrono::duration<double>(tc - tb).count();
    }
    return std::chrono::duration<double>(Clock::now() - t0).count();
}

int main(int argc, char **argv) {
    double seconds = 600.0;
    int reps = 3;
    std::string threads_arg = "1,16,ref", modes_arg = "auto,pageable,bounce,pinned";
    for (int i = 1; i < argc; ++i) {
        const std::string a = argv[i];
        auto next = [&]() -> const char * {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "%s needs a value\n", a.c_str());
                std::exit(2);
            }
            return argv[++i];
        };
        if (a == "--seconds") seconds = std::atof(next());
        else if (a == "--threads") threads_arg = next();
        else if (a == "--reps") reps = std::max(1, std::atoi(next()));
        else if (a == "--modes") modes_arg = next();
        else {
            std::fprintf(stderr, "usage: %s [--seconds S] [--threads a,b|ref] [--reps R] [--modes auto,pageable,bounce,pinned]\n",
                         argv[0]);
            return 2;
        }
    }
    const double fs = 48000.0;
    const size_t nch = 2, n = (size_t)std::llround(seconds * fs);
    // synthetic int24 samples (SURVEY.md s8d's form: DC + 997 Hz + noise)
    std::vector<std::vector<float>> x(nch, std::vector<float>(n));
    uint64_t s = 20260206;
    for (size_t c = 0; c < nch; ++c)
        for (size_t i = 0; i < n; ++i) {
            s = s * 6364136223846793005ULL + 1442695040888963407ULL;
            const double u = (double)(s >> 11) / 4503599627370496.0 - 1.0;
            const double v = 0.02 + 0.4 * std::sin(2.0 * M_PI * 997.0 * (double)i / fs + 0.3 * (double)c) + 0.1 * u;
            x[c][i] = (float)(std::nearbyint(std::clamp(v, -1.0, 1.0 - 0x1p-23) * 0x1p23) * 0x1p-23);
        }
    int32_t ntaps = 0;
    if (lcfir_design_lowcut(20.0, 48.0, fs, nullptr, 0, &ntaps)) die("design");
    std::vector<double> taps((size_t)ntaps);
    if (lcfir_design_lowcut(20.0, 48.0, fs, taps.data(), ntaps, &ntaps)) die("design");
    const WindowedSinc<double> sinc(taps);

    // the whole file on the device in one launch: what every partition must reproduce
    std::vector<float> want(nch * n);
    {
        lcfir_ctx *ctx = nullptr;
        if (lcfir_ctx_create(0, taps.data(), ntaps, &ctx)) die("ctx");
        void *dx = nullptr, *dy = nullptr;
        if (lcfir_dev_malloc(0, sizeof(float) * nch * n, &dx) || lcfir_dev_malloc(0, sizeof(float) * nch * n, &dy))
            die("malloc");
        for (size_t c = 0; c < nch; ++c)
            if (lcfir_memcpy_h2d(static_cast<float *>(dx) + c * n, x[c].data(), sizeof(float) * n, nullptr))
                die("h2d");
        if (lcfir_filter_channels_dev(ctx, static_cast<float *>(dx), (int64_t)n, (int32_t)nch, (int64_t)n,
                                      static_cast<float *>(dy), (int64_t)n, nullptr, nullptr))
            die("filter");
        if (lcfir_memcpy_d2h(want.data(), dy, sizeof(float) * nch * n, nullptr)) die("d2h");
        lcfir_dev_free(dx);
        lcfir_dev_free(dy);
        lcfir_ctx_destroy(ctx);
    }
    const unsigned hw = std::thread::hardware_concurrency();
    const unsigned ref_threads = std::max(1u, (unsigned)(0.7 * (double)hw)); // main.cp:75-76
    int bad = 0;
    for (const std::string &mode : split(modes_arg)) {
        if (mode != "bounce" && mode != "pageable" && mode != "pinned" && mode != "auto") {
            std::fprintf(stderr, "unknown mode %s\n", mode.c_str());
            return 2;
        }
        vectormath_pinned() = mode == "pinned";
        if (lcfir_staging_set_mode(mode == "bounce" ? LCFIR_STAGING_BOUNCE
                                   : mode == "auto" ? LCFIR_STAGING_AUTO
                                                    : LCFIR_STAGING_PAGEABLE))
            die("mode");
        for (const std::string &t : split(threads_arg)) {
            const unsigned nt = t == "ref" ? ref_threads : (unsigned)std::max(1, std::atoi(t.c_str()));
            auto fresh = [&]() {
                std::vector<VectorMath<float>> buf;
                for (size_t c = 0; c < nch; ++c) {
                    VectorMath<float> v(n);
                    std::memcpy(&v[0], x[c].data(), sizeof(float) * n);
                    buf.push_back(std::move(v));
                }
                return buf;
            };
            ThreadSafeProgress progress;
            double alloc_s = 0.0, fanout_s = 0.0;
            {
                auto buf = fresh();
                (void)process_file(buf, sinc, nt, progress, &alloc_s, &fanout_s); // warm-up: plan, slots, bounce buffers
            }
            alloc_s = fanout_s = 0.0;
            std::vector<double> times;
            bool identical = true;
            lcfir_range_stats st{};
            lcfir_range_stats_get(&st, 1);
            for (int r = 0; r < reps; ++r) {
                auto buf = fresh();
                times.push_back(process_file(buf, sinc, nt, progress, &alloc_s, &fanout_s));
                for (size_t c = 0; c < nch; ++c)
                    identical = identical && std::memcmp(&buf[c][0], want.data() + c * n, sizeof(float) * n) == 0;
            }
            lcfir_range_stats_get(&st, 1);
            // one profiled file: the per-call stage split
            lcfir_range_profile(1);
            double tprof, pa = 0.0, pf = 0.0;
            {
                auto buf = fresh();
                tprof = process_file(buf, sinc, nt, progress, &pa, &pf);
            }
            lcfir_range_profile(0);
            lcfir_range_stats sp{};
            lcfir_range_stats_get(&sp, 1);
            std::sort(times.begin(), times.end());
            const double med = times[times.size() / 2], best = times.front();
            const double samples = (double)(nch * n);
            const double calls = (double)std::max<uint64_t>(1, sp.profiled_calls);
            const double rate = samples / med / 1e6;
            std::printf(
                "{\"tool\": \"dropin_bench\", \"mode\": \"%s\", \"threads\": %u, \"hardware_concurrency\": %u, "
                "\"channels\": %zu, \"samples_per_channel\": %zu, \"ntaps\": %d, \"reps\": %d, "
                "\"msamples_per_s\": %.1f, \"msamples_per_s_best\": %.1f, \"ms_per_file\": %.3f, "
                "\"h2d_bound_frac\": %.4f, \"fanout_msamples_per_s\": %.1f, \"fanout_h2d_bound_frac\": %.4f, "
                "\"alloc_ms_per_file\": %.3f, \"fanout_ms_per_file\": %.3f, "
                "\"bit_identical\": %s, \"calls_per_file\": %.0f, "
                "\"staged_calls_frac\": %.3f, \"pcie_GBps_per_file\": %.2f, "
                "\"split_per_call_ms\": {\"wall\": %.4f, \"h2d\": %.4f, \"kernel\": %.4f, \"d2h\": %.4f}, "
                "\"split_sum_over_file_wall\": {\"h2d\": %.3f, \"kernel\": %.3f, \"d2h\": %.3f}, "
                "\"profiled_file_ms\": %.3f, "
                "\"note\": \"host-pointer drop-in (FilterCore.h through ProcessFile.cp:57-87's threads), "
                "pageable buffers, PCIe both ways; msamples_per_s = the whole ProcessFile.cp:57-87 loop "
                "(temp_output allocation included), fanout_* = the threads' spawn-to-join spans only (the "
                "drop-in calls); h2d_bound_frac = rate / (56 GB/s pinned H2D / 4 B); never bench.py value\"}\n",
                mode.c_str(), nt, hw, nch, n, ntaps, reps, rate, samples / best / 1e6, med * 1e3,
                rate / (56e9 / 4.0 / 1e6), samples / (fanout_s / reps) / 1e6,
                samples / (fanout_s / reps) / 1e6 / (56e9 / 4.0 / 1e6), alloc_s / reps * 1e3, fanout_s / reps * 1e3,
                identical ? "true" : "false", (double)st.calls / reps,
                st.calls ? (double)st.staged_calls / (double)st.calls : 0.0,
                (double)(st.h2d_bytes + st.d2h_bytes) / reps / med / 1e9, sp.wall_ms / calls, sp.h2d_ms / calls,
                sp.kernel_ms / calls, sp.d2h_ms / calls, sp.h2d_ms / (tprof * 1e3), sp.kernel_ms / (tprof * 1e3),
                sp.d2h_ms / (tprof * 1e3), tprof * 1e3);
            std::fflush(stdout);
            if (!identical) bad = 1;
        }
    }
    if (!lcfir::last_failure().empty()) {
        std::fprintf(stderr, "failure: %s\n", lcfir::last_failure().c_str());
        return 4;
    }
    return bad ? 3 : 0;
}

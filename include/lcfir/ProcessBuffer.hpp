// lcfir/ProcessBuffer.hpp -- the compute part of the reference's process_file
// (ProcessFile.cp:57-101) on an in-memory deinterleaved buffer, two ways:
//
//  * process_buffer(): the reference's structure kept verbatim -- channels in
//    series, each split into num_threads chunks (chunk = N / threads, the last
//    takes the remainder, ProcessFile.cp:64-69), one std::thread per chunk
//    calling apply_filter_range (ProcessFile.cp:71-78), join, move the result
//    into the buffer (:86), then the peak / normalize post-pass (:91-101).
//    With the GPU behind apply_filter_range the chunks are independent
//    device launches on separate HIP streams.
//
//  * process_buffer_device(): the same result with the buffer uploaded once,
//    all channels filtered in one launch with the peak fused into the kernel,
//    and the normalize decision taken on the device (no host round trip).
//
// Buffer = any sequence of channels (buf.size(), buf[ch]) whose channels are
// contiguous float containers with size()/data(), e.g.
// std::vector<std::vector<float>> or the reference's AudioBuffer of
// VectorMath<float32_t>.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <thread>
#include <utility>
#include <vector>

#include "lcfir/FilterCore.hpp"

namespace lcfir {

// ProcessFile.h:13-19
struct FilterOptions {
    double freq = 15.0;
    double slope = 10.0;
    bool normalize = false;
    bool verbose = false;
    unsigned num_threads = 0;
};

template <class Channel>
inline float max_mag(const Channel &c) { // VectorMath::max_mag
    float m = 0.0f;
    for (size_t i = 0; i < std::size(c); ++i) m = std::max(m, std::fabs(std::data(c)[i]));
    return m;
}

// AudioSamples::normalize: the scale rule of c_lib is unpinned; we scale by
// 1/peak in double and round to float (same rule as the device kernel).
template <class Buffer>
inline void normalize(Buffer &buf, float peak) {
    if (!(peak > 0.0f)) return;
    const double gain = 1.0 / (double)peak;
    for (size_t ch = 0; ch < std::size(buf); ++ch) {
        auto &c = buf[ch];
        for (size_t i = 0; i < std::size(c); ++i)
            std::data(c)[i] = (float)((double)std::data(c)[i] * gain);
    }
}

struct NullProgress {
    void report(size_t) {}
};

// Returns the pre-normalize peak over all channels.
template <class Buffer, class Sinc, class Progress = NullProgress>
float process_buffer(Buffer &buf, const Sinc &sinc, const FilterOptions &opts,
                     Progress *progress = nullptr) {
    const unsigned nthreads = opts.num_threads ? opts.num_threads : 1;
    for (size_t ch = 0; ch < std::size(buf); ++ch) {
        using Channel = std::decay_t<decltype(buf[ch])>;
        const int64_t total = (int64_t)std::size(buf[ch]);
        Channel temp_output(buf[ch]); // same size; every sample is overwritten
        std::vector<std::thread> threads;
        threads.reserve(nthreads);
        const int64_t chunk = total / (int64_t)nthreads;
        for (unsigned i = 0; i < nthreads; ++i) {
            const int64_t start = (int64_t)i * chunk;
            const int64_t end = (i == nthreads - 1) ? total : start + chunk;
            threads.emplace_back([&, start, end] {
                apply_filter_range(buf[ch], sinc, temp_output, start, end, progress);
            });
        }
        for (auto &t : threads) t.join();
        buf[ch] = std::move(temp_output);
    }
    float peak = 0.0f;
    for (size_t ch = 0; ch < std::size(buf); ++ch) peak = std::max(peak, max_mag(buf[ch]));
    if (peak > 1.0f || opts.normalize) normalize(buf, peak);
    return peak;
}

// Device-resident variant: one upload, one filter launch for all channels
// (fused peak), device-side normalize, one download.  Channels must have
// equal length.  Returns the pre-normalize peak.
template <class Buffer>
float process_buffer_device(Buffer &buf, const Filter &flt, const FilterOptions &opts) {
    const int32_t nch = (int32_t)std::size(buf);
    if (nch == 0) return 0.0f;
    const int64_t n = (int64_t)std::size(buf[0]);
    for (int32_t c = 1; c < nch; ++c)
        if ((int64_t)std::size(buf[c]) != n) throw Error(LCFIR_EINVAL, "channels differ in length");
    const size_t bytes = sizeof(float) * (size_t)n * (size_t)nch;
    void *stream = nullptr, *dx = nullptr, *dy = nullptr, *dpk = nullptr;
    struct Cleanup {
        void **p[3];
        void **s;
        ~Cleanup() {
            for (auto q : p) lcfir_dev_free(*q);
            if (*s) lcfir_stream_destroy(*s);
        }
    } cleanup{{&dx, &dy, &dpk}, &stream};
    check(lcfir_stream_create(flt.device(), &stream), "lcfir_stream_create");
    check(lcfir_dev_malloc(flt.device(), bytes, &dx), "lcfir_dev_malloc");
    check(lcfir_dev_malloc(flt.device(), bytes, &dy), "lcfir_dev_malloc");
    check(lcfir_dev_malloc(flt.device(), sizeof(float) * (size_t)nch, &dpk), "lcfir_dev_malloc");
    for (int32_t c = 0; c < nch; ++c)
        check(lcfir_memcpy_h2d((float *)dx + (size_t)c * (size_t)n, std::data(buf[c]),
                               sizeof(float) * (size_t)n, stream), "h2d");
    check(lcfir_peak_reset_dev((float *)dpk, nch, stream), "peak reset");
    check(lcfir_filter_channels_dev(flt.get(), (const float *)dx, n, nch, n, (float *)dy, n,
                                    (float *)dpk, stream), "filter");
    check(lcfir_normalize_dev((float *)dy, n, nch, n, (const float *)dpk, nch,
                              opts.normalize ? 1 : 0, stream), "normalize");
    std::vector<float> peaks((size_t)nch);
    check(lcfir_memcpy_d2h(peaks.data(), dpk, sizeof(float) * (size_t)nch, stream), "d2h");
    for (int32_t c = 0; c < nch; ++c)
        check(lcfir_memcpy_d2h(std::data(buf[c]), (float *)dy + (size_t)c * (size_t)n,
                               sizeof(float) * (size_t)n, stream), "d2h");
    return *std::max_element(peaks.begin(), peaks.end());
}

} // namespace lcfir

// The reference's per-channel chunk hand-off (ProcessFile.cp:57-87), restated
// against include/lcfir/FilterCore.h with the reference's exact call shape:
// apply_filter_range passed BY NAME to std::thread (ProcessFile.cp:71-78).
//
// VectorMath, WindowedSinc and ThreadSafeProgress come from the un-vendored
// c_lib / ProgressBar.h; reference_types.hpp has stand-ins exposing only what
// FilterCore.h and ProcessFile.cp use of them.
//
// usage: dropin_processfile in.f32 taps.f64 out.f32 nch n threads
// Prints "progress <count>" and "peak <max|y|>".
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <thread>
#include <vector>

#include "reference_types.hpp"

#define LCFIR_DROPIN_TYPES_DECLARED
#include "lcfir/FilterCore.h"

using namespace Diskerror;

template <class T>
static std::vector<T> read_all(const char *path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) {
        std::fprintf(stderr, "cannot open %s\n", path);
        std::exit(2);
    }
    const size_t bytes = (size_t)f.tellg();
    std::vector<T> v(bytes / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)bytes);
    return v;
}

int main(int argc, char **argv) {
    if (argc != 7) {
        std::fprintf(stderr, "usage: %s in.f32 taps.f64 out.f32 nch n threads\n", argv[0]);
        return 2;
    }
    const auto x = read_all<float>(argv[1]);
    const WindowedSinc<double> sinc(read_all<double>(argv[2]));
    const size_t numChannels = std::strtoul(argv[4], nullptr, 10);
    const size_t numFrames = std::strtoul(argv[5], nullptr, 10);
    const unsigned num_threads = (unsigned)std::strtoul(argv[6], nullptr, 10);
    if (x.size() != numChannels * numFrames || num_threads == 0) {
        std::fprintf(stderr, "bad arguments\n");
        return 2;
    }
    std::vector<VectorMath<float>> buf;
    for (size_t c = 0; c < numChannels; ++c) {
        VectorMath<float> ch(numFrames);
        for (size_t i = 0; i < numFrames; ++i) ch[i] = x[c * numFrames + i];
        buf.push_back(std::move(ch));
    }
    ThreadSafeProgress safe_progress;

    // ProcessFile.cp:57-87, call shape unchanged
    for (size_t ch = 0; ch < numChannels; ++ch) {
        VectorMath<float> temp_output(numFrames);
        std::vector<std::thread> threads;
        threads.reserve(num_threads);
        const auto totalSamples = static_cast<int_fast64_t>(numFrames);
        const int_fast64_t chunkSize = totalSamples / num_threads;
        for (unsigned int i = 0; i < num_threads; ++i) {
            int_fast64_t start = i * chunkSize;
            int_fast64_t end = (i == num_threads - 1) ? totalSamples : (start + chunkSize);
            threads.emplace_back(
                apply_filter_range,
                std::cref(buf[ch]),
                std::cref(sinc),
                std::ref(temp_output),
                start,
                end,
                &safe_progress);
        }
        for (auto &t : threads) t.join();
        buf[ch] = std::move(temp_output);
    }

    float maxMag = 0.0f;
    for (size_t ch = 0; ch < numChannels; ++ch) maxMag = std::max(maxMag, buf[ch].max_mag());
    std::ofstream o(argv[3], std::ios::binary);
    for (auto &c : buf)
        for (size_t i = 0; i < c.size(); ++i) o.write(reinterpret_cast<const char *>(&c[i]), sizeof(float));
    std::printf("progress %zu\npeak %.9g\n", safe_progress.count(), (double)maxMag);
    if (!lcfir::last_failure().empty()) {
        std::fprintf(stderr, "failure: %s\n", lcfir::last_failure().c_str());
        return 4;
    }
    return 0;
}

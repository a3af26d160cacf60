// Test driver for the C++ drop-in headers (include/lcfir/FilterCore.hpp,
// ProcessBuffer.hpp).  Reads a raw float32 [nch][n] buffer and float64 taps,
// runs the reference-structured process_buffer (threads calling
// apply_filter_range with the FilterCore.h signature) or the device-resident
// variant, writes the raw float32 result and prints "peak <value>".
//
// usage: filtercore_driver in.f32 taps.f64 out.f32 nch n threads mode normalize
//        mode 0 = process_buffer (threaded hand-off), 1 = process_buffer_device,
//        2 / 3 = process_buffer with a PaddedSinc / ReversedSinc,
//        4 / 5 = a WindowedSinc / PaddedSinc first used with other taps (half
//        of them), then rewritten in place (same object, same data() pointer):
//        the drop-in's per-object caches must miss on the second file
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <vector>

#include "lcfir/ProcessBuffer.hpp"

// Stand-in for c_lib's WindowedSinc<float64_t>: the drop-in only needs the taps.
struct WindowedSinc {
    std::vector<double> k;
    const double *data() const { return k.data(); }
    size_t size() const { return k.size(); }
};

// WindowedSinc stand-ins whose data()/size() are NOT the fms() kernel (c_lib's
// member layout is unpinned): the drop-in must notice (getMo2() / one fms()
// fingerprint) and recover the taps through fms() instead.  Padded: two extra
// zeros at the end; Reversed: the taps back to front.
struct SincFms {
    std::vector<double> h;
    int getMo2() const { return (int)(h.size() - 1) / 2; }
    template <class It>
    double fms(It p) const {
        double acc = 0;
        for (size_t k = 0; k < h.size(); ++k) acc += h[k] * (double)p[(long)k];
        return acc;
    }
};
struct PaddedSinc : SincFms {
    std::vector<double> padded;
    explicit PaddedSinc(std::vector<double> t) : SincFms{t}, padded(t) { padded.resize(t.size() + 2, 0.0); }
    const double *data() const { return padded.data(); }
    size_t size() const { return padded.size(); }
};
struct ReversedSinc : SincFms {
    std::vector<double> rev;
    explicit ReversedSinc(std::vector<double> t) : SincFms{t}, rev(t.rbegin(), t.rend()) {}
    const double *data() const { return rev.data(); }
    size_t size() const { return rev.size(); }
};

// Counterpart of ThreadSafeProgress (ProgressBar.h:57-82).
struct Progress {
    std::mutex mu;
    size_t count = 0;
    void report(size_t c) {
        std::lock_guard<std::mutex> lk(mu);
        count += c;
    }
};

template <class T>
static std::vector<T> read_all(const char *path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) { std::fprintf(stderr, "cannot open %s\n", path); std::exit(2); }
    const size_t bytes = (size_t)f.tellg();
    std::vector<T> v(bytes / sizeof(T));
    f.seekg(0);
    f.read(reinterpret_cast<char *>(v.data()), (std::streamsize)bytes);
    return v;
}

int main(int argc, char **argv) {
    if (argc != 9) {
        std::fprintf(stderr, "usage: %s in.f32 taps.f64 out.f32 nch n threads mode normalize\n", argv[0]);
        return 2;
    }
    const auto x = read_all<float>(argv[1]);
    WindowedSinc sinc{read_all<double>(argv[2])};
    const size_t nch = std::strtoul(argv[4], nullptr, 10), n = std::strtoul(argv[5], nullptr, 10);
    lcfir::FilterOptions opts;
    opts.num_threads = (unsigned)std::strtoul(argv[6], nullptr, 10);
    const int mode = std::atoi(argv[7]);
    opts.normalize = std::atoi(argv[8]) != 0;
    if (x.size() != nch * n) { std::fprintf(stderr, "size mismatch\n"); return 2; }
    std::vector<std::vector<float>> buf(nch);
    for (size_t c = 0; c < nch; ++c) buf[c].assign(x.begin() + (long)(c * n), x.begin() + (long)((c + 1) * n));
    float peak;
    Progress prog;
    try {
        if (mode == 0) {
            peak = lcfir::process_buffer(buf, sinc, opts, &prog);
            if (prog.count != nch * n) { std::fprintf(stderr, "progress %zu\n", prog.count); return 3; }
        } else if (mode == 1) {
            const std::vector<double> taps = lcfir::sinc_taps<std::vector<float>>(sinc);
            lcfir::Filter flt(taps.data(), (int32_t)taps.size());
            peak = lcfir::process_buffer_device(buf, flt, opts);
        } else if (mode == 4 || mode == 5) {
            std::vector<double> half(sinc.k);
            for (double &v : half) v *= 0.5;
            WindowedSinc ws{half};
            PaddedSinc ps(half);
            const double *before = mode == 4 ? ws.data() : ps.data();
            auto first = buf;  // the earlier file
            if (mode == 4) lcfir::process_buffer(first, ws, opts, &prog);
            else lcfir::process_buffer(first, ps, opts, &prog);
            for (double &v : ws.k) v *= 2.0;  // exact: the real taps, in place
            for (double &v : ps.h) v *= 2.0;
            for (double &v : ps.padded) v *= 2.0;
            if (before != (mode == 4 ? ws.data() : ps.data())) { std::fprintf(stderr, "moved\n"); return 3; }
            prog.count = 0;
            peak = mode == 4 ? lcfir::process_buffer(buf, ws, opts, &prog) : lcfir::process_buffer(buf, ps, opts, &prog);
            if (prog.count != nch * n) { std::fprintf(stderr, "progress %zu\n", prog.count); return 3; }
        } else if (mode == 2) {
            peak = lcfir::process_buffer(buf, PaddedSinc(sinc.k), opts, &prog);
        } else {
            peak = lcfir::process_buffer(buf, ReversedSinc(sinc.k), opts, &prog);
        }
    } catch (const lcfir::Error &e) {
        std::fprintf(stderr, "lcfir error %d: %s\n", e.code(), e.what());
        return 4;
    }
    std::ofstream o(argv[3], std::ios::binary);
    for (auto &c : buf) o.write(reinterpret_cast<const char *>(c.data()), (std::streamsize)(c.size() * sizeof(float)));
    std::printf("peak %.9g\n", (double)peak);
    return 0;
}

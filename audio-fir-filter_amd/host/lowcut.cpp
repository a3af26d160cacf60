// lowcut.cpp -- the reference's command-line tool (main.cp + process_file,
// ProcessFile.cp:27-120) with the hot path on an MI355X.
//
//   lowcut [options] <input_file> <output_file>
//   lowcut [options] <input_file1> [input_file2 ...] <output_directory>
//
// Options as main.cp:42-56: -f/--frequency (15), -s/--slope (10),
// -n/--normalize, -v/--verbose, -t/--threads (accepted; one device launch
// covers a channel), -O/--overwrite, -h/--help.  Extensions: --method
// auto|direct|fft, --device N, --info (print the parsed format, no GPU).
// Scenario checks and their errors follow main.cp:84-151; errors exit with
// EXIT_FAILURE after printing the message (main.cp:153-164).
//
// Per file (ProcessFile.cp): parse the container, design the low-cut for the
// file's sample rate (:47-50), upload the raw sample bytes, decode to
// deinterleaved f32 on the device, filter every channel in one launch with
// the peak fused, take the normalize decision on the device (:91-101),
// encode back to the file's own format, and write the input file's bytes
// with only the sample payload replaced (:103-117).
#include <cstdio>
#include <cstdlib>
#include <filesystem>
#include <functional>
#include <iostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "audio_file.hpp"
#include "lcfir.h"

namespace fs = std::filesystem;
using lcfir_host::AudioFile;

namespace {

struct UsageError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

struct Options {
    double freq = 15.0;
    double slope = 10.0;
    bool normalize = false;
    bool verbose = false;
    unsigned threads = 0;
    bool overwrite = false;
    bool info = false;
    int method = LCFIR_METHOD_AUTO;
    int device = 0;
    std::vector<std::string> paths;
};

const char *kHelp = R"(
Applies low-cut (high-pass) FIR filter to WAVE or AIFF file.
Usage:
  lowcut [options] <input_file> <output_file>
  lowcut [options] <input_file1> [input_file2 ...] <output_directory>
Options:
  -f [ --frequency ] arg (=15)  Filter cutoff frequency in Hz.
  -s [ --slope ] arg (=10)      Filter slope width in Hz.
  -n [ --normalize ]            Normalize output to maximum level.
  -v [ --verbose ]              Verbose output.
  -t [ --threads ] arg (=0)     Number of threads (accepted; the GPU filters a
                                whole channel per launch).
  -O [ --overwrite ]            Overwrite existing files.
  -h [ --help ]                 Display this help message.
  --method arg (=auto)          auto | direct | fft
  --device arg (=0)             GPU ordinal
  --info                        Print each input's format and exit.
)";

void check(int rc, const char *what) {
    if (rc != LCFIR_OK) throw std::runtime_error(std::string(what) + ": " + lcfir_last_error());
}

Options parse(int argc, char **argv) {
    Options o;
    auto value = [&](int &i, const std::string &name) -> std::string {
        if (i + 1 >= argc) throw UsageError("option " + name + " needs a value");
        return argv[++i];
    };
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        std::string v;
        const auto eq = a.find('=');
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            v = a.substr(eq + 1);
            a = a.substr(0, eq);
        }
        auto val = [&](const std::string &n) { return v.empty() ? value(i, n) : v; };
        if (a == "-f" || a == "--frequency") o.freq = std::stod(val(a));
        else if (a == "-s" || a == "--slope") o.slope = std::stod(val(a));
        else if (a == "-n" || a == "--normalize") o.normalize = true;
        else if (a == "-v" || a == "--verbose") o.verbose = true;
        else if (a == "-t" || a == "--threads") o.threads = (unsigned)std::stoul(val(a));
        else if (a == "-O" || a == "--overwrite") o.overwrite = true;
        else if (a == "-h" || a == "--help") {
            std::cout << kHelp << std::endl;
            std::exit(EXIT_SUCCESS);
        } else if (a == "--info") o.info = true;
        else if (a == "--device") o.device = std::stoi(val(a));
        else if (a == "--method") {
            const std::string m = val(a);
            if (m == "auto") o.method = LCFIR_METHOD_AUTO;
            else if (m == "direct") o.method = LCFIR_METHOD_DIRECT;
            else if (m == "fft") o.method = LCFIR_METHOD_FFT;
            else throw UsageError("unknown method " + m);
        } else if (!a.empty() && a[0] == '-' && a.size() > 1) throw UsageError("unknown option " + a);
        else o.paths.push_back(argv[i]);
    }
    return o;
}

struct DevBuf {
    void *p = nullptr;
    DevBuf(int dev, size_t bytes) { check(lcfir_dev_malloc(dev, bytes, &p), "lcfir_dev_malloc"); }
    ~DevBuf() { lcfir_dev_free(p); }
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
};

void process_file(const fs::path &in, const fs::path &out, const Options &o) {
    std::function<void(const std::string &)> status = [](const std::string &) {};
    if (o.verbose) status = [](const std::string &s) { std::cout << s << std::endl; };

    status("Opening input file.");
    AudioFile f = lcfir_host::read_audio_file(in.string());
    std::cout << "Processing file: " << in.filename().string() << std::endl;

    status("Creating sinc kernel for this file's sample rate.");
    int32_t ntaps = 0;
    check(lcfir_design_lowcut(o.freq, o.slope, f.sample_rate, nullptr, 0, &ntaps), "design");
    std::vector<double> taps((size_t)ntaps);
    check(lcfir_design_lowcut(o.freq, o.slope, f.sample_rate, taps.data(), ntaps, &ntaps), "design");
    lcfir_ctx *ctx = nullptr;
    check(lcfir_ctx_create(o.device, taps.data(), ntaps, &ctx), "lcfir_ctx_create");
    struct CtxGuard {
        lcfir_ctx *c;
        ~CtxGuard() { lcfir_ctx_destroy(c); }
    } guard{ctx};
    int method = o.method;
    if (method == LCFIR_METHOD_FFT && lcfir_ctx_set_method(ctx, method) != LCFIR_OK)
        method = LCFIR_METHOD_DIRECT; // tap count beyond the FFT segment
    check(lcfir_ctx_set_method(ctx, method), "lcfir_ctx_set_method");
    check(lcfir_ctx_get_method(ctx, &method), "lcfir_ctx_get_method");

    status("Reading samples.");
    const int nch = f.channels;
    const int64_t n = f.frames;
    void *stream = nullptr;
    check(lcfir_stream_create(o.device, &stream), "stream");
    struct StreamGuard {
        void *s;
        ~StreamGuard() { lcfir_stream_destroy(s); }
    } sguard{stream};
    const size_t nbytes = std::max<size_t>(1, f.data_bytes);
    const size_t plane = sizeof(float) * (size_t)std::max<int64_t>(1, n) * (size_t)nch;
    DevBuf d_raw(o.device, nbytes), d_x(o.device, plane), d_y(o.device, plane),
        d_peak(o.device, sizeof(float) * (size_t)nch);
    float peak_host = 0.0f;
    if (n > 0) {
        check(lcfir_memcpy_h2d(d_raw.p, f.bytes.data() + f.data_offset, f.data_bytes, stream), "h2d");
        check(lcfir_decode_pcm_dev(d_raw.p, f.pcm_format, nch, n, (float *)d_x.p, n, stream), "decode");
        status("Filtering.");
        check(lcfir_peak_reset_dev((float *)d_peak.p, nch, stream), "peak reset");
        check(lcfir_filter_channels_dev(ctx, (const float *)d_x.p, n, nch, n, (float *)d_y.p, n,
                                        (float *)d_peak.p, stream), "filter");
        std::vector<float> peaks((size_t)nch);
        check(lcfir_memcpy_d2h(peaks.data(), d_peak.p, sizeof(float) * (size_t)nch, stream), "d2h");
        for (float pk : peaks) peak_host = std::max(peak_host, pk);
        if (peak_host > 1.0f || o.normalize) status("Doing audio normalize.");
        check(lcfir_normalize_dev((float *)d_y.p, n, nch, n, (const float *)d_peak.p, nch,
                                  o.normalize ? 1 : 0, stream), "normalize");
        check(lcfir_encode_pcm_dev((const float *)d_y.p, n, nch, n, f.pcm_format, d_raw.p, stream),
              "encode");
        check(lcfir_memcpy_d2h(f.bytes.data() + f.data_offset, d_raw.p, f.data_bytes, stream), "d2h");
    }
    if (o.verbose)
        std::cout << "  " << nch << " ch x " << n << " frames, " << f.format_name() << ", "
                  << f.sample_rate << " Hz, " << ntaps << " taps ("
                  << (method == LCFIR_METHOD_FFT ? "fft" : "direct") << "), peak " << peak_host
                  << std::endl;
    status("Writing output file.");
    lcfir_host::write_bytes(out.string(), f.bytes);
    status("");
}

void print_info(const fs::path &in) {
    const AudioFile f = lcfir_host::read_audio_file(in.string());
    std::printf("%s: %s %s ch=%d frames=%lld rate=%.6g bits=%d data_offset=%zu data_bytes=%zu chunks=",
                in.string().c_str(), f.kind == AudioFile::Kind::Wave ? "WAVE" : "AIFF",
                f.format_name(), f.channels, (long long)f.frames, f.sample_rate, f.bits,
                f.data_offset, f.data_bytes);
    for (size_t i = 0; i < f.chunk_ids.size(); ++i)
        std::printf("%s%s", i ? "," : "", f.chunk_ids[i].c_str());
    std::printf("\n");
}

int run(int argc, char **argv) {
    Options o = parse(argc, argv);
    if (o.info) {
        for (const auto &p : o.paths) print_info(p);
        return EXIT_SUCCESS;
    }
    std::vector<fs::path> paths(o.paths.begin(), o.paths.end());
    if (paths.size() == 2) {
        // Scenario 1: input file -> output file (main.cp:84-109)
        const fs::path &in = paths[0], &out = paths[1];
        if (!fs::exists(in) || !fs::is_regular_file(in)) throw std::runtime_error("File not found: " + in.string());
        if (fs::exists(out) && fs::is_directory(out))
            throw UsageError("With two parameters the second parameter must be a file path, not a directory.");
        if (in.extension() != out.extension())
            throw UsageError("Input and output file types (WAVE or AIFF) must be the same (extensions must match).");
        if (fs::exists(out) && !o.overwrite) throw std::runtime_error("File exists: " + out.string());
        if (fs::exists(out)) fs::remove(out);
        process_file(in, out, o);
    } else if (paths.size() > 2) {
        // Scenario 2: input files -> output directory (main.cp:112-147)
        const fs::path &dest = paths.back();
        if (fs::exists(dest)) {
            if (!fs::is_directory(dest))
                throw UsageError("Destination exists but is not a directory: " + dest.string());
        } else {
            if (dest.has_extension())
                throw UsageError("Destination directory '" + dest.string() +
                                 "' does not exist and has a suffix. Undefined scenario.");
            if (o.verbose) std::cout << "Creating directory: " << dest.string() << std::endl;
            fs::create_directories(dest);
        }
        for (size_t i = 0; i + 1 < paths.size(); ++i) {
            const fs::path &in = paths[i];
            if (!fs::exists(in) || !fs::is_regular_file(in)) throw std::runtime_error("File not found: " + in.string());
            const fs::path out = dest / in.filename();
            if (fs::exists(out) && !o.overwrite) throw std::runtime_error("File exists: " + out.string());
            if (fs::exists(out)) fs::remove(out);
            process_file(in, out, o);
        }
    } else {
        throw UsageError("Invalid number of parameters. Need at least 2.");
    }
    return EXIT_SUCCESS;
}

} // namespace

int main(int argc, char **argv) {
    try {
        return run(argc, argv);
    } catch (const std::exception &e) {
        std::cerr << e.what() << std::endl;
        return EXIT_FAILURE;
    } catch (...) {
        std::cerr << "Caught an unknown exception." << std::endl;
        return EXIT_FAILURE;
    }
}

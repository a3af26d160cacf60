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
#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <exception>
#include <filesystem>
#include <functional>
#include <iostream>
#include <map>
#include <mutex>
#include <optional>
#include <set>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "audio_file.hpp"
#include "lcfir.h"

namespace fs = std::filesystem;
using lcfir_host::AudioFile;
using Clock = std::chrono::steady_clock;

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
    bool timing = false;
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
  --timing                      Print per-file read/GPU/write times and the
                                end-to-end rate.
)";

void check(int rc, const char *what) {
    if (rc != LCFIR_OK) throw std::runtime_error(std::string(what) + ": " + lcfir_last_error());
}

double seconds_since(Clock::time_point t0) {
    return std::chrono::duration<double>(Clock::now() - t0).count();
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
        else if (a == "--timing") o.timing = true;
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

// ---- pipeline plumbing ------------------------------------------------------

// Bounded blocking queue between the stages.
template <class T> class Channel {
public:
    explicit Channel(size_t cap) : cap_(cap) {}
    void push(T v) {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return q_.size() < cap_; });
        q_.push_back(std::move(v));
        cv_.notify_all();
    }
    std::optional<T> pop() {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return !q_.empty() || closed_; });
        if (q_.empty()) return std::nullopt;
        T v = std::move(q_.front());
        q_.pop_front();
        cv_.notify_all();
        return v;
    }
    void close() {
        std::lock_guard<std::mutex> lk(m_);
        closed_ = true;
        cv_.notify_all();
    }

private:
    std::mutex m_;
    std::condition_variable cv_;
    std::deque<T> q_;
    size_t cap_;
    bool closed_ = false;
};

// Pinned host buffers, recycled: page-locking a 1.4 GB file costs more than
// copying it, so buffers go back to the pool when the writer is done.
class PinnedPool {
public:
    ~PinnedPool() {
        for (auto &b : free_) lcfir_host_free(b.second);
    }
    std::shared_ptr<uint8_t> get(size_t n) {
        n = std::max<size_t>(n, 1);
        void *p = nullptr;
        size_t cap = 0;
        {
            std::lock_guard<std::mutex> lk(m_);
            auto it = free_.lower_bound(n);
            if (it != free_.end()) {
                cap = it->first;
                p = it->second;
                free_.erase(it);
            }
        }
        if (!p) {
            check(lcfir_host_malloc(n, &p), "lcfir_host_malloc");
            cap = n;
        }
        return std::shared_ptr<uint8_t>(static_cast<uint8_t *>(p), [this, cap](uint8_t *q) {
            std::lock_guard<std::mutex> lk(m_);
            free_.emplace(cap, q);
            while (free_.size() > kKeep) {
                lcfir_host_free(free_.begin()->second);
                free_.erase(free_.begin());
            }
        });
    }

private:
    static constexpr size_t kKeep = 4;
    std::mutex m_;
    std::multimap<size_t, void *> free_;
};

// Grow-only device allocation owned by one pipeline slot.
struct DevArena {
    void *p = nullptr;
    size_t cap = 0;
    void *get(int dev, size_t n) {
        if (n > cap) {
            lcfir_dev_free(p);
            p = nullptr;
            cap = 0;
            check(lcfir_dev_malloc(dev, n, &p), "lcfir_dev_malloc");
            cap = n;
        }
        return p;
    }
    ~DevArena() { lcfir_dev_free(p); }
};

struct Job {
    size_t index = 0;
    fs::path in, out;
    AudioFile f;
    std::exception_ptr error; // a scenario/read failure: stop the batch here
    int32_t ntaps = 0;
    int method = 0;
    float peak = 0.0f;
    double t_read = 0, t_gpu = 0, t_write = 0;
};

// One filter per sample rate (ProcessFile.cp:47-50 builds it per file; files
// of a batch usually share a rate, so the taps and FFT plan are reused).
struct FilterSet {
    const Options &o;
    struct Entry {
        lcfir_ctx *ctx;
        int method;
        int32_t ntaps;
    };
    std::map<double, Entry> by_rate;
    explicit FilterSet(const Options &opt) : o(opt) {}
    ~FilterSet() {
        for (auto &e : by_rate) lcfir_ctx_destroy(e.second.ctx);
    }
    const Entry &get(double fs) {
        auto it = by_rate.find(fs);
        if (it != by_rate.end()) return it->second;
        int32_t ntaps = 0;
        check(lcfir_design_lowcut(o.freq, o.slope, fs, nullptr, 0, &ntaps), "design");
        std::vector<double> taps((size_t)ntaps);
        check(lcfir_design_lowcut(o.freq, o.slope, fs, taps.data(), ntaps, &ntaps), "design");
        lcfir_ctx *ctx = nullptr;
        check(lcfir_ctx_create(o.device, taps.data(), ntaps, &ctx), "lcfir_ctx_create");
        int method = o.method;
        if (method == LCFIR_METHOD_FFT && lcfir_ctx_set_method(ctx, method) != LCFIR_OK)
            method = LCFIR_METHOD_DIRECT; // tap count beyond the FFT segment
        if (lcfir_ctx_set_method(ctx, method) != LCFIR_OK ||
            lcfir_ctx_get_method(ctx, &method) != LCFIR_OK) {
            lcfir_ctx_destroy(ctx);
            throw std::runtime_error(std::string("lcfir_ctx_set_method: ") + lcfir_last_error());
        }
        return by_rate.emplace(fs, Entry{ctx, method, ntaps}).first->second;
    }
};

// A GPU slot: its own stream and buffers, so two files are in flight at once
// (one's H2D/D2H under the other's kernels).
struct Slot {
    void *stream = nullptr;
    DevArena raw, x, y, peak;
    std::shared_ptr<uint8_t> peaks_host; // pinned, per-channel peaks
    size_t peaks_cap = 0;
    std::optional<Job> job;
    Clock::time_point t0;
};

// Enqueue the whole per-file compute of ProcessFile.cp:40-117 on the slot's
// stream: H2D raw bytes -> decode/deinterleave -> filter all channels with the
// peak fused -> encode with the device-side normalize decision and gain
// folded in (:91-101, :115-117) -> D2H into
// the same pinned buffer.  Nothing here waits on the device.
void enqueue_file(Slot &s, Job &j, FilterSet &filters, PinnedPool &pool, const Options &o) {
    const AudioFile &f = j.f;
    const auto &flt = filters.get(f.sample_rate);
    j.ntaps = flt.ntaps;
    j.method = flt.method;
    const int nch = f.channels;
    const int64_t n = f.frames;
    if (n <= 0) return;
    const size_t plane = sizeof(float) * (size_t)n * (size_t)nch;
    void *d_raw = s.raw.get(o.device, f.data_bytes);
    float *d_x = static_cast<float *>(s.x.get(o.device, plane));
    float *d_y = static_cast<float *>(s.y.get(o.device, plane));
    float *d_peak = static_cast<float *>(s.peak.get(o.device, sizeof(float) * (size_t)nch));
    if ((size_t)nch > s.peaks_cap) {
        s.peaks_host = pool.get(sizeof(float) * (size_t)nch);
        s.peaks_cap = (size_t)nch;
    }
    check(lcfir_memcpy_h2d(d_raw, f.data + f.data_offset, f.data_bytes, s.stream), "h2d");
    check(lcfir_decode_pcm_dev(d_raw, f.pcm_format, nch, n, d_x, n, s.stream), "decode");
    check(lcfir_peak_reset_dev(d_peak, nch, s.stream), "peak reset");
    check(lcfir_filter_channels_dev(flt.ctx, d_x, n, nch, n, d_y, n, d_peak, s.stream), "filter");
    // the normalize decision and gain ride in the encode pass, which reads every
    // sample anyway: no separate rescale pass over the f32 planes
    check(lcfir_encode_pcm_scaled_dev(d_y, n, nch, n, f.pcm_format, d_peak, nch, o.normalize ? 1 : 0, d_raw,
                                      s.stream),
          "encode");
    check(lcfir_memcpy_d2h_async(f.data + f.data_offset, d_raw, f.data_bytes, s.stream), "d2h");
    check(lcfir_memcpy_d2h_async(s.peaks_host.get(), d_peak, sizeof(float) * (size_t)nch, s.stream),
          "d2h");
}

void finish_file(Slot &s, const Options &o) {
    check(lcfir_stream_sync(s.stream), "stream sync");
    Job &j = *s.job;
    j.t_gpu = seconds_since(s.t0);
    if (j.f.frames > 0) {
        const float *pk = reinterpret_cast<const float *>(s.peaks_host.get());
        for (int c = 0; c < j.f.channels; ++c) j.peak = std::max(j.peak, pk[c]);
    }
    if (o.verbose) {
        if (j.peak > 1.0f || o.normalize) std::cout << "Doing audio normalize." << std::endl;
        std::cout << "  " << j.f.channels << " ch x " << j.f.frames << " frames, " << j.f.format_name()
                  << ", " << j.f.sample_rate << " Hz, " << j.ntaps << " taps ("
                  << (j.method == LCFIR_METHOD_FFT ? "fft" : "direct") << "), peak " << j.peak
                  << std::endl;
    }
}

// Reader -> GPU (2 slots) -> writer.  Files are read, filtered and written in
// order; a failure on file k (missing input, existing output without -O,
// unreadable container) ends the batch after files < k are written, as the
// reference's sequential loop does (main.cp:131-146).
void process_files(const std::vector<std::pair<fs::path, fs::path>> &todo, const Options &o) {
    const auto t_all = Clock::now();
    PinnedPool pool;
    Channel<Job> to_gpu(1), to_writer(2);
    std::thread reader([&] {
        // outputs scheduled by earlier jobs: the reference's sequential loop
        // (main.cp:131-146) has written them by the time it checks a later job,
        // so a repeated destination is "File exists" there too (without -O)
        std::set<fs::path> scheduled;
        for (size_t i = 0; i < todo.size(); ++i) {
            Job j;
            j.index = i;
            j.in = todo[i].first;
            j.out = todo[i].second;
            const auto t0 = Clock::now();
            try {
                if (!fs::exists(j.in) || !fs::is_regular_file(j.in))
                    throw std::runtime_error("File not found: " + j.in.string());
                const fs::path canon = fs::weakly_canonical(j.out);
                if ((fs::exists(j.out) || scheduled.count(canon)) && !o.overwrite)
                    throw std::runtime_error("File exists: " + j.out.string());
                scheduled.insert(canon);
                j.f = lcfir_host::read_audio_file(j.in.string(),
                                                  [&](size_t n) { return pool.get(n); });
            } catch (...) {
                j.error = std::current_exception();
            }
            j.t_read = seconds_since(t0);
            const bool stop = (bool)j.error;
            to_gpu.push(std::move(j));
            if (stop) break;
        }
        to_gpu.close();
    });
    std::exception_ptr write_error;
    std::thread writer([&] {
        while (auto j = to_writer.pop()) {
            if (write_error) continue;
            try {
                const auto t0 = Clock::now();
                if (fs::exists(j->out)) fs::remove(j->out);
                lcfir_host::write_bytes(j->out.string(), j->f.data, j->f.size);
                j->t_write = seconds_since(t0);
                if (o.timing)
                    std::printf("timing %s: read %.3f s, gpu %.3f s (h2d+filter+d2h), write %.3f s, "
                                "%lld frames x %d ch\n",
                                j->in.filename().string().c_str(), j->t_read, j->t_gpu, j->t_write,
                                (long long)j->f.frames, j->f.channels);
            } catch (...) {
                write_error = std::current_exception();
            }
            j->f = AudioFile{}; // the pinned buffer returns to the pool
        }
    });

    std::exception_ptr error;
    FilterSet filters(o);
    Slot slots[2];
    int64_t total_samples = 0;
    try {
        for (auto &s : slots) check(lcfir_stream_create(o.device, &s.stream), "stream");
        size_t k = 0;
        while (auto j = to_gpu.pop()) {
            Slot &s = slots[k++ % 2];
            if (s.job) { // this slot's previous file is done once its stream drains
                finish_file(s, o);
                to_writer.push(std::move(*s.job));
                s.job.reset();
            }
            if (j->error) {
                error = j->error;
                break;
            }
            std::cout << "Processing file: " << j->in.filename().string() << std::endl;
            total_samples += j->f.frames * j->f.channels;
            s.t0 = Clock::now();
            s.job.emplace(std::move(*j));
            enqueue_file(s, *s.job, filters, pool, o);
        }
        for (size_t i = 0; i < 2; ++i) {
            Slot &s = slots[k++ % 2];
            if (!s.job) continue;
            finish_file(s, o);
            to_writer.push(std::move(*s.job));
            s.job.reset();
        }
    } catch (...) {
        if (!error) error = std::current_exception();
    }
    to_writer.close();
    // drain the reader if the GPU stage stopped early
    while (to_gpu.pop()) {
    }
    reader.join();
    writer.join();
    for (auto &s : slots) {
        if (s.stream) {
            lcfir_stream_sync(s.stream);
            lcfir_stream_destroy(s.stream);
        }
    }
    if (error) std::rethrow_exception(error);
    if (write_error) std::rethrow_exception(write_error);
    if (o.timing) {
        const double t = seconds_since(t_all);
        std::printf("timing total: %zu file(s), %.3f s, %.1f Msamples/s end to end (disk + PCIe + GPU)\n",
                    todo.size(), t, (double)total_samples / t / 1e6);
    }
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
        process_files({{in, out}}, o);
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
        std::vector<std::pair<fs::path, fs::path>> todo;
        for (size_t i = 0; i + 1 < paths.size(); ++i) todo.emplace_back(paths[i], dest / paths[i].filename());
        process_files(todo, o); // per-file checks run in order inside the pipeline
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

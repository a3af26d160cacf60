// lowcut.cpp -- the reference's command-line tool (main.cp + process_file,
// ProcessFile.cp:27-120) with the hot path on an MI355X.
//
//   lowcut [options] <input_file> <output_file>
//   lowcut [options] <input_file1> [input_file2 ...] <output_directory>
//
// Options as main.cp:42-56: -f/--frequency (15), -s/--slope (10),
// -n/--normalize, -v/--verbose, -t/--threads (accepted; one device launch
// covers a channel), -O/--overwrite, -h/--help.  Extensions: --method
// auto|direct|fft, --devices LIST (default: every visible GPU) / --device N,
// --info (print the parsed format, no GPU), --plan (print the file-to-GPU
// dealing, no GPU).
//
// A batch (scenario 2, main.cp:132-147) is dealt round-robin over the
// devices, one file per GPU at a time (BASELINE.json north_star: "shard one
// file per GPU"): file i goes to GPU stage i mod D, each stage with its own
// filter contexts, streams and two pipeline slots.  Each file's normalize
// stays on its own GPU (the peak is per file, ProcessFile.cp:91-101), so no
// collective is needed; outputs are written in input order.
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
#include <atomic>
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
    std::vector<int> devices; // empty: every visible device
    int readers = 1;          // file-reader threads
    bool plan = false;
    std::vector<std::string> paths;
};

// "all" or a comma-separated list of device ordinals ("0,0" runs two GPU
// stages on one device)
std::vector<int> parse_devices(const std::string &v) {
    std::vector<int> out;
    if (v == "all") return out;
    size_t i = 0;
    while (i <= v.size()) {
        const size_t j = std::min(v.find(',', i), v.size());
        const std::string t = v.substr(i, j - i);
        if (t.empty() || t.find_first_not_of("0123456789") != std::string::npos)
            throw UsageError("bad --devices list: " + v);
        out.push_back(std::stoi(t));
        i = j + 1;
    }
    return out;
}

// GPU stage of file i in a batch dealt over `stages` stages: round-robin
size_t stage_of(size_t file_index, size_t stages) { return file_index % stages; }

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
  --devices arg (=all)          GPUs for a batch, e.g. 0,1,2,3 (files are dealt
                                round-robin, one file per GPU at a time)
  --device arg                  one GPU (= --devices arg)
  --readers arg (=1)            File-reader threads (files read in parallel;
                                more than one measured slower on one GPU).
  --plan                        Print which GPU stage each file goes to and exit.
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
        else if (a == "--device") o.devices = {std::stoi(val(a))};
        else if (a == "--devices") o.devices = parse_devices(val(a));
        else if (a == "--plan") o.plan = true;
        else if (a == "--readers") {
            const std::string v = val(a);
            if (v.empty() || v.find_first_not_of("0123456789") != std::string::npos || v.size() > 3)
                throw UsageError("bad --readers value: " + v);
            o.readers = std::stoi(v);
            if (o.readers < 1 || o.readers > 64) throw UsageError("--readers must be 1..64");
        }
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
    int device;
    struct Entry {
        lcfir_ctx *ctx;
        int method;
        int32_t ntaps;
    };
    std::map<double, Entry> by_rate;
    FilterSet(const Options &opt, int dev) : o(opt), device(dev) {}
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
        check(lcfir_ctx_create(device, taps.data(), ntaps, &ctx), "lcfir_ctx_create");
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
    const int dev = filters.device;
    const AudioFile &f = j.f;
    const auto &flt = filters.get(f.sample_rate);
    j.ntaps = flt.ntaps;
    j.method = flt.method;
    const int nch = f.channels;
    const int64_t n = f.frames;
    if (n <= 0) return;
    const size_t plane = sizeof(float) * (size_t)n * (size_t)nch;
    void *d_raw = s.raw.get(dev, f.data_bytes);
    float *d_x = static_cast<float *>(s.x.get(dev, plane));
    float *d_y = static_cast<float *>(s.y.get(dev, plane));
    float *d_peak = static_cast<float *>(s.peak.get(dev, sizeof(float) * (size_t)nch));
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

std::mutex g_print_mu; // the GPU stages print from their own threads

void finish_file(Slot &s, const Options &o) {
    check(lcfir_stream_sync(s.stream), "stream sync");
    Job &j = *s.job;
    j.t_gpu = seconds_since(s.t0);
    if (j.f.frames > 0) {
        const float *pk = reinterpret_cast<const float *>(s.peaks_host.get());
        for (int c = 0; c < j.f.channels; ++c) j.peak = std::max(j.peak, pk[c]);
    }
    if (o.verbose) {
        std::lock_guard<std::mutex> lk(g_print_mu);
        if (j.peak > 1.0f || o.normalize) std::cout << "Doing audio normalize." << std::endl;
        std::cout << "  " << j.f.channels << " ch x " << j.f.frames << " frames, " << j.f.format_name()
                  << ", " << j.f.sample_rate << " Hz, " << j.ntaps << " taps ("
                  << (j.method == LCFIR_METHOD_FFT ? "fft" : "direct") << "), peak " << j.peak
                  << std::endl;
    }
}

// One GPU stage: its device's filter contexts, two slots (streams + buffers),
// its own input queue; finished files go to the shared writer queue.
struct GpuStage {
    int device = 0;
    Channel<Job> in{1};
    std::exception_ptr error;
    std::thread th;
};

void run_stage(GpuStage &st, Channel<Job> &to_writer, PinnedPool &pool, const Options &o) {
    FilterSet filters(o, st.device);
    Slot slots[2];
    // the file being finished or enqueued when a step throws: the batch stops
    // there (main.cp:131-146), so files of this stage with a lower index --
    // at most the other slot's, enqueued earlier -- are still finished and
    // handed to the writer
    size_t at = (size_t)-1;
    try {
        for (auto &s : slots) check(lcfir_stream_create(st.device, &s.stream), "stream");
        size_t k = 0;
        while (auto j = st.in.pop()) {
            Slot &s = slots[k++ % 2];
            if (s.job) { // this slot's previous file is done once its stream drains
                at = s.job->index;
                finish_file(s, o);
                to_writer.push(std::move(*s.job));
                s.job.reset();
            }
            s.t0 = Clock::now();
            s.job.emplace(std::move(*j));
            at = s.job->index;
            enqueue_file(s, *s.job, filters, pool, o);
        }
        for (size_t i = 0; i < 2; ++i) {
            Slot &s = slots[k++ % 2];
            if (!s.job) continue;
            at = s.job->index;
            finish_file(s, o);
            to_writer.push(std::move(*s.job));
            s.job.reset();
        }
    } catch (...) {
        st.error = std::current_exception();
        for (auto &s : slots) {
            if (!s.job || s.job->index >= at) continue;
            try {
                finish_file(s, o);
                to_writer.push(std::move(*s.job));
            } catch (...) { // its stream failed too: the batch stops at the earlier file
            }
            s.job.reset();
        }
        while (st.in.pop()) { // keep the reader from blocking on this stage
        }
    }
    for (auto &s : slots) {
        if (s.stream) {
            lcfir_stream_sync(s.stream);
            lcfir_stream_destroy(s.stream);
        }
    }
}

// Readers -> GPU stages (file i on stage i mod D, 2 slots each) -> writer (in
// input order).  A failure on file k (missing input, existing output without
// -O, unreadable container, a GPU error) ends the batch after files < k are
// written, as the reference's sequential loop does (main.cp:131-146).
// The existence checks run first, in input order (they decide k for the
// reference's "File not found" / "File exists" cases before anything is
// read); then R reader threads (--readers, default 1) read files < k in
// index order from a shared counter.  One reader measured fastest on the
// one-GPU box (1 223 against 746 and 701 Msamples/s with 2 and 4 readers,
// 8 config-2 files: every reader in flight holds another pinned buffer);
// more may pay where several GPUs wait on fast storage.  Files finish out of order; the writer writes them in
// order and stops at the first failed one.
void process_files(const std::vector<std::pair<fs::path, fs::path>> &todo, const std::vector<int> &devices,
                   const Options &o) {
    const auto t_all = Clock::now();
    PinnedPool pool;
    std::vector<std::unique_ptr<GpuStage>> stages;
    for (int d : devices) {
        stages.push_back(std::make_unique<GpuStage>());
        stages.back()->device = d;
    }
    Channel<Job> to_writer(2 * stages.size());
    // the checks the reference makes before it processes file i, in order;
    // outputs scheduled by earlier jobs count as existing (the reference has
    // written them by the time it checks a later job)
    size_t limit = todo.size();
    std::exception_ptr check_error;
    {
        std::set<fs::path> scheduled;
        for (size_t i = 0; i < todo.size(); ++i) {
            try {
                const fs::path &in = todo[i].first, &out = todo[i].second;
                if (!fs::exists(in) || !fs::is_regular_file(in))
                    throw std::runtime_error("File not found: " + in.string());
                const fs::path canon = fs::weakly_canonical(out);
                if ((fs::exists(out) || scheduled.count(canon)) && !o.overwrite)
                    throw std::runtime_error("File exists: " + out.string());
                scheduled.insert(canon);
            } catch (...) {
                check_error = std::current_exception();
                limit = i;
                break;
            }
        }
    }
    std::mutex read_mu;
    std::exception_ptr read_error;
    size_t read_error_at = todo.size(); // index of the first file that failed to read
    std::atomic<size_t> next_file{0};
    std::atomic<int64_t> total_samples{0};
    std::atomic<size_t> readers_left;
    const size_t nreaders = (size_t)std::max(1, o.readers);
    readers_left = nreaders;
    std::vector<std::thread> readers;
    for (size_t r = 0; r < nreaders; ++r)
        readers.emplace_back([&] {
            for (;;) {
                const size_t i = next_file++;
                {
                    std::lock_guard<std::mutex> lk(read_mu);
                    if (i >= limit || i > read_error_at) break;
                }
                Job j;
                j.index = i;
                j.in = todo[i].first;
                j.out = todo[i].second;
                const auto t0 = Clock::now();
                try {
                    j.f = lcfir_host::read_audio_file(j.in.string(), [&](size_t n) { return pool.get(n); });
                } catch (...) {
                    std::lock_guard<std::mutex> lk(read_mu);
                    if (i < read_error_at) {
                        read_error_at = i;
                        read_error = std::current_exception();
                    }
                    continue;
                }
                j.t_read = seconds_since(t0);
                total_samples += j.f.frames * j.f.channels;
                stages[stage_of(i, stages.size())]->in.push(std::move(j));
            }
            if (--readers_left == 0)
                for (auto &st : stages) st->in.close();
        });
    for (auto &st : stages) st->th = std::thread([&, p = st.get()] { run_stage(*p, to_writer, pool, o); });
    std::exception_ptr write_error;
    std::thread writer([&] {
        std::map<size_t, Job> ready; // finished out of order across readers and stages
        size_t next = 0;
        while (auto j = to_writer.pop()) {
            const size_t idx = j->index;
            ready.emplace(idx, std::move(*j));
            for (auto it = ready.find(next); it != ready.end(); it = ready.find(next)) {
                Job &w = it->second;
                size_t stop;
                {
                    std::lock_guard<std::mutex> lk(read_mu);
                    stop = std::min(limit, read_error_at);
                }
                if (!write_error && w.index < stop) {
                    {
                        std::lock_guard<std::mutex> lk(g_print_mu);
                        std::cout << "Processing file: " << w.in.filename().string() << std::endl;
                    }
                    try {
                        const auto t0 = Clock::now();
                        if (fs::exists(w.out)) fs::remove(w.out);
                        lcfir_host::write_bytes(w.out.string(), w.f.data, w.f.size);
                        w.t_write = seconds_since(t0);
                        if (o.timing) {
                            std::lock_guard<std::mutex> lk(g_print_mu);
                            std::printf("timing %s: read %.3f s, gpu %.3f s (h2d+filter+d2h), write %.3f s, "
                                        "%lld frames x %d ch\n",
                                        w.in.filename().string().c_str(), w.t_read, w.t_gpu, w.t_write,
                                        (long long)w.f.frames, w.f.channels);
                        }
                    } catch (...) {
                        write_error = std::current_exception();
                    }
                }
                ready.erase(it); // the pinned buffer returns to the pool
                ++next;
            }
        }
    });
    for (auto &t : readers) t.join();
    for (auto &st : stages) st->th.join();
    to_writer.close();
    writer.join();
    // a GPU error stops its stage; a reader error at file k comes after every
    // file < k was dispatched (and, if no GPU error, written)
    for (auto &st : stages)
        if (st->error) std::rethrow_exception(st->error);
    // the first failure in input order: a check (its index is `limit`) or a read
    if (read_error && read_error_at < limit) std::rethrow_exception(read_error);
    if (check_error) std::rethrow_exception(check_error);
    if (write_error) std::rethrow_exception(write_error);
    if (o.timing) {
        const double t = seconds_since(t_all);
        std::printf("timing total: %zu file(s), %zu GPU stage(s), %zu reader(s), %.3f s, %.1f Msamples/s end to "
                    "end (disk + PCIe + GPU)\n",
                    todo.size(), stages.size(), nreaders, t, (double)total_samples.load() / t / 1e6);
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

// The GPU stages of this run: --devices/--device, else every visible device
// (asks the runtime only when no list was given).
std::vector<int> resolve_devices(const Options &o) {
    if (!o.devices.empty()) return o.devices;
    int n = 0;
    check(lcfir_device_count(&n), "lcfir_device_count");
    if (n < 1) throw std::runtime_error("no GPU visible");
    std::vector<int> d((size_t)n);
    for (int i = 0; i < n; ++i) d[(size_t)i] = i;
    return d;
}

void run_or_plan(const std::vector<std::pair<fs::path, fs::path>> &todo, const Options &o) {
    if (o.plan) {
        // the dealing only (no GPU touched): needs an explicit device list
        if (o.devices.empty()) throw UsageError("--plan needs --devices");
        for (size_t i = 0; i < todo.size(); ++i) {
            const size_t st = stage_of(i, o.devices.size());
            std::printf("plan %s -> %s stage %zu device %d\n", todo[i].first.string().c_str(),
                        todo[i].second.string().c_str(), st, o.devices[st]);
        }
        return;
    }
    process_files(todo, resolve_devices(o), o);
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
        run_or_plan({{in, out}}, o);
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
        run_or_plan(todo, o); // per-file checks run in order inside the pipeline
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

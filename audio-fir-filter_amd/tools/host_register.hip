// host_register.hip -- what pinning the caller's pageable channel would cost
// (development tool, not part of the product).
//
// The drop-in (lcfir_apply_range, ProcessFile.cp:57-87's threads) gets a
// pageable channel and a pageable temp_output from the reference.  The runtime
// then moves every call's window through its own staging (2.7-4.4 Gs/s for
// config 2's file, 0.19-0.31 of the pinned-H2D bound), while page-locked
// buffers reach the link directly.  The library could register the whole
// channel and output once per fan-out (hipHostRegister) and unregister them
// when the last range completes.  This tool prices that against the pageable
// copies it would replace, for config 2's channel (28.8 M floats = 115.2 MB):
//   * hipHostRegister + hipHostUnregister of a freshly touched pageable buffer
//     (each also for a second buffer, the output), cold and repeated;
//   * H2D of the channel and D2H of the outputs from / to pageable memory;
//   * the same copies once registered.
// Registration pays off only if register + unregister (both buffers) costs less
// than the pageable transfers minus the registered ones.  Then the pageable
// path's sensitivity to where a buffer starts (page-aligned or not).
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 host_register.hip -o host_register
//   ./host_register [floats] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) {
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

// a pageable buffer whose pages exist (the reference's VectorMath<float32_t>
// has been filled by the file reader before the threads start)
static float *pageable(size_t n) {
    auto *p = static_cast<float *>(std::aligned_alloc(4096, (n * sizeof(float) + 4095) / 4096 * 4096));
    if (!p) std::exit(1);
    for (size_t i = 0; i < n; ++i) p[i] = (float)(i & 1023) * 1e-3f;
    return p;
}

int main(int argc, char **argv) {
    const size_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (size_t)28800000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 5;
    const size_t bytes = n * sizeof(float);
    CK(hipSetDevice(0));
    float *d = nullptr;
    CK(hipMalloc(&d, bytes));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::printf("buffer: %zu floats = %.1f MB, %d reps\n", n, bytes / 1e6, reps);
    std::vector<double> reg, unreg, h2d_pg, d2h_pg, h2d_pin, d2h_pin;
    for (int r = 0; r < reps; ++r) {
        // fresh buffers each rep: a fan-out registers a channel it has never seen
        float *x = pageable(n), *y = pageable(n);
        auto t0 = clk::now();
        CK(hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        h2d_pg.push_back(ms_since(t0));
        t0 = clk::now();
        CK(hipMemcpyAsync(y, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        d2h_pg.push_back(ms_since(t0));
        t0 = clk::now();
        CK(hipHostRegister(x, bytes, hipHostRegisterDefault));
        CK(hipHostRegister(y, bytes, hipHostRegisterDefault));
        reg.push_back(ms_since(t0));
        t0 = clk::now();
        CK(hipMemcpyAsync(d, x, bytes, hipMemcpyHostToDevice, s));
        CK(hipStreamSynchronize(s));
        h2d_pin.push_back(ms_since(t0));
        t0 = clk::now();
        CK(hipMemcpyAsync(y, d, bytes, hipMemcpyDeviceToHost, s));
        CK(hipStreamSynchronize(s));
        d2h_pin.push_back(ms_since(t0));
        t0 = clk::now();
        CK(hipHostUnregister(x));
        CK(hipHostUnregister(y));
        unreg.push_back(ms_since(t0));
        std::free(x);
        std::free(y);
        std::printf("rep %d: pageable H2D %.2f D2H %.2f ms | register x+y %.2f | pinned H2D %.2f D2H %.2f | "
                    "unregister x+y %.2f ms\n",
                    r, h2d_pg.back(), d2h_pg.back(), reg.back(), h2d_pin.back(), d2h_pin.back(), unreg.back());
    }
    auto med = [](std::vector<double> v) {
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    const double pg = med(h2d_pg) + med(d2h_pg), pin = med(h2d_pin) + med(d2h_pin),
                 cost = med(reg) + med(unreg);
    std::printf("median: pageable H2D+D2H %.2f ms (%.1f / %.1f GB/s), pinned %.2f ms (%.1f / %.1f GB/s), "
                "register+unregister of both %.2f ms\n",
                pg, bytes / med(h2d_pg) / 1e6, bytes / med(d2h_pg) / 1e6, pin, bytes / med(h2d_pin) / 1e6,
                bytes / med(d2h_pin) / 1e6, cost);
    std::printf("verdict: registering %s (saves %.2f ms of transfer, costs %.2f ms)\n",
                cost < pg - pin ? "PAYS" : "does not pay", pg - pin, cost);

    // Does the pageable path care where the buffer starts?  The drop-in's
    // VectorMath storage comes from malloc (a 16-byte header in front of an
    // mmap'd block: not page aligned), this tool's from aligned_alloc.  Same
    // buffers every rep (warm, as a fan-out's channel is), three forms:
    // page-aligned, +16 B, and +16 B copied as head (to the next 4 KiB
    // boundary) + page-aligned body + tail.
    {
        const size_t pad = 8192;
        char *xa = reinterpret_cast<char *>(pageable(n + pad / 4));
        char *ya = reinterpret_cast<char *>(pageable(n + pad / 4));
        auto copy = [&](char *hx, char *hy, bool split) {
            double th = 0, td = 0;
            auto t0 = clk::now();
            if (!split) {
                CK(hipMemcpyAsync(d, hx, bytes, hipMemcpyHostToDevice, s));
            } else {
                const size_t head = (4096 - (reinterpret_cast<uintptr_t>(hx) & 4095)) & 4095;
                const size_t body = (bytes - head) / 4096 * 4096;
                if (head) CK(hipMemcpyAsync(d, hx, head, hipMemcpyHostToDevice, s));
                CK(hipMemcpyAsync(reinterpret_cast<char *>(d) + head, hx + head, body, hipMemcpyHostToDevice, s));
                if (head + body < bytes)
                    CK(hipMemcpyAsync(reinterpret_cast<char *>(d) + head + body, hx + head + body, bytes - head - body,
                                      hipMemcpyHostToDevice, s));
            }
            CK(hipStreamSynchronize(s));
            th = ms_since(t0);
            t0 = clk::now();
            if (!split) {
                CK(hipMemcpyAsync(hy, d, bytes, hipMemcpyDeviceToHost, s));
            } else {
                const size_t head = (4096 - (reinterpret_cast<uintptr_t>(hy) & 4095)) & 4095;
                const size_t body = (bytes - head) / 4096 * 4096;
                if (head) CK(hipMemcpyAsync(hy, d, head, hipMemcpyDeviceToHost, s));
                CK(hipMemcpyAsync(hy + head, reinterpret_cast<char *>(d) + head, body, hipMemcpyDeviceToHost, s));
                if (head + body < bytes)
                    CK(hipMemcpyAsync(hy + head + body, reinterpret_cast<char *>(d) + head + body, bytes - head - body,
                                      hipMemcpyDeviceToHost, s));
            }
            CK(hipStreamSynchronize(s));
            td = ms_since(t0);
            return std::make_pair(th, td);
        };
        const char *names[3] = {"page-aligned", "+16 B", "+16 B split at 4 KiB"};
        for (int form = 0; form < 3; ++form) {
            std::vector<double> h, dd;
            char *hx = form == 0 ? xa : xa + 16, *hy = form == 0 ? ya : ya + 16;
            for (int r = 0; r < reps + 1; ++r) {
                auto [th, td] = copy(hx, hy, form == 2);
                if (r) { // the first is a warm-up
                    h.push_back(th);
                    dd.push_back(td);
                }
            }
            std::printf("pageable %-22s H2D %.2f ms (%.1f GB/s)  D2H %.2f ms (%.1f GB/s)  [median of %d]\n",
                        names[form], med(h), bytes / med(h) / 1e6, med(dd), bytes / med(dd) / 1e6, reps);
        }
        // the fan-out's shape: T threads, each its own stream, each moving 1/T of
        // the +16 B buffer H2D then D2H (as T concurrent drop-in calls do)
        for (int T : {1, 4, 16}) {
            std::vector<hipStream_t> ss((size_t)T);
            for (auto &q : ss) CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
            std::vector<double> tot;
            for (int r = 0; r < reps + 1; ++r) {
                auto t0 = clk::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const size_t per = n / (size_t)T * 4, off = (size_t)t * per,
                                     len = t == T - 1 ? bytes - off : per;
                        CK(hipMemcpyAsync(reinterpret_cast<char *>(d) + off, xa + 16 + off, len,
                                          hipMemcpyHostToDevice, ss[(size_t)t]));
                        CK(hipMemcpyAsync(ya + 16 + off, reinterpret_cast<char *>(d) + off, len,
                                          hipMemcpyDeviceToHost, ss[(size_t)t]));
                        CK(hipStreamSynchronize(ss[(size_t)t]));
                    });
                for (auto &x : th) x.join();
                if (r) tot.push_back(ms_since(t0));
            }
            std::printf("pageable +16 B, %2d threads x (H2D then D2H of 1/%d): %.2f ms for both directions "
                        "(%.1f GB/s each way)\n", T, T, med(tot), bytes / med(tot) / 1e6);
            for (auto &q : ss) CK(hipStreamDestroy(q));
        }
        // the drop-in's device buffers come from the stream-ordered pool
        // (hipMallocAsync, lcfir.hip grow()): does a pageable copy to / from
        // pool memory take the same path as to hipMalloc'd memory?
        {
            void *dp = nullptr;
            CK(hipMallocAsync(&dp, bytes, s));
            CK(hipStreamSynchronize(s));
            std::vector<double> h, dd;
            for (int r = 0; r < reps + 1; ++r) {
                auto t0 = clk::now();
                CK(hipMemcpyAsync(dp, xa + 16, bytes, hipMemcpyHostToDevice, s));
                CK(hipStreamSynchronize(s));
                const double th = ms_since(t0);
                t0 = clk::now();
                CK(hipMemcpyAsync(ya + 16, dp, bytes, hipMemcpyDeviceToHost, s));
                CK(hipStreamSynchronize(s));
                if (r) {
                    h.push_back(th);
                    dd.push_back(ms_since(t0));
                }
            }
            std::printf("pageable +16 B <-> hipMallocAsync memory: H2D %.2f ms (%.1f GB/s)  D2H %.2f ms (%.1f GB/s)\n",
                        med(h), bytes / med(h) / 1e6, med(dd), bytes / med(dd) / 1e6);
            CK(hipFreeAsync(dp, s));
            CK(hipStreamSynchronize(s));
        }
        // per-call registration, the fan-out's shape: T threads each register
        // a disjoint page-aligned 1/T of the channel and of the output, copy
        // H2D and D2H from the registered slices, and unregister them
        for (int T : {1, 4, 16}) {
            std::vector<hipStream_t> ss((size_t)T);
            for (auto &q : ss) CK(hipStreamCreateWithFlags(&q, hipStreamNonBlocking));
            std::vector<double> tot, regw;
            for (int r = 0; r < reps + 1; ++r) {
                std::vector<double> treg((size_t)T);
                auto t0 = clk::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const size_t per = bytes / (size_t)T / 4096 * 4096, off = (size_t)t * per,
                                     len = t == T - 1 ? bytes - off : per;
                        auto a = clk::now();
                        CK(hipHostRegister(xa + off, len, hipHostRegisterDefault));
                        CK(hipHostRegister(ya + off, len, hipHostRegisterDefault));
                        treg[(size_t)t] = ms_since(a);
                        CK(hipMemcpyAsync(reinterpret_cast<char *>(d) + off, xa + off, len, hipMemcpyHostToDevice,
                                          ss[(size_t)t]));
                        CK(hipMemcpyAsync(ya + off, reinterpret_cast<char *>(d) + off, len, hipMemcpyDeviceToHost,
                                          ss[(size_t)t]));
                        CK(hipStreamSynchronize(ss[(size_t)t]));
                        CK(hipHostUnregister(xa + off));
                        CK(hipHostUnregister(ya + off));
                    });
                for (auto &x : th) x.join();
                if (r) {
                    tot.push_back(ms_since(t0));
                    regw.push_back(*std::max_element(treg.begin(), treg.end()));
                }
            }
            std::printf("per-call registration, %2d threads x 1/%d: register (slowest thread) %.2f ms, whole "
                        "register + H2D + D2H + unregister %.2f ms (%.1f GB/s each way)\n",
                        T, T, med(regw), med(tot), bytes / med(tot) / 1e6);
            for (auto &q : ss) CK(hipStreamDestroy(q));
        }
        // the bounce alternative, the fan-out's shape: T threads, each
        // memcpy's its 1/T of the pageable channel into its own pinned buffer
        // in C-byte chunks and has it DMA'd over ONE shared H2D stream, then
        // the D2H over ONE shared D2H stream into the pinned buffer and
        // memcpy's it out (the link both ways, the host copies in parallel)
        for (int T : {4, 16}) {
            const size_t per = bytes / (size_t)T;
            std::vector<void *> pin((size_t)T);
            for (auto &q : pin) CK(hipHostMalloc(&q, per + 4096, hipHostMallocDefault));
            hipStream_t hin, hout;
            CK(hipStreamCreateWithFlags(&hin, hipStreamNonBlocking));
            CK(hipStreamCreateWithFlags(&hout, hipStreamNonBlocking));
            std::mutex mu_in, mu_out;
            std::vector<double> tot, mcpy;
            for (int r = 0; r < reps + 1; ++r) {
                std::vector<double> tm((size_t)T);
                auto t0 = clk::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; ++t)
                    th.emplace_back([&, t] {
                        const size_t off = (size_t)t * per, len = t == T - 1 ? bytes - off : per;
                        char *pb = static_cast<char *>(pin[(size_t)t]);
                        hipEvent_t e;
                        CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                        auto a = clk::now();
                        std::memcpy(pb, xa + 16 + off, len);
                        double m = ms_since(a);
                        {
                            std::lock_guard<std::mutex> g(mu_in);
                            CK(hipMemcpyAsync(reinterpret_cast<char *>(d) + off, pb, len, hipMemcpyHostToDevice, hin));
                            CK(hipEventRecord(e, hin));
                        }
                        {
                            std::lock_guard<std::mutex> g(mu_out);
                            CK(hipStreamWaitEvent(hout, e, 0));
                            CK(hipMemcpyAsync(pb, reinterpret_cast<char *>(d) + off, len, hipMemcpyDeviceToHost, hout));
                            CK(hipEventRecord(e, hout));
                        }
                        CK(hipEventSynchronize(e));
                        a = clk::now();
                        std::memcpy(ya + 16 + off, pb, len);
                        m += ms_since(a);
                        tm[(size_t)t] = m;
                        CK(hipEventDestroy(e));
                    });
                for (auto &x : th) x.join();
                if (r) {
                    tot.push_back(ms_since(t0));
                    mcpy.push_back(*std::max_element(tm.begin(), tm.end()));
                }
            }
            std::printf("bounce over shared link streams, %2d threads x 1/%d: %.2f ms for both directions "
                        "(%.1f GB/s each way; slowest thread's two memcpys %.2f ms)\n",
                        T, T, med(tot), bytes / med(tot) / 1e6, med(mcpy));
            for (auto &q : pin) CK(hipHostFree(q));
            CK(hipStreamDestroy(hin));
            CK(hipStreamDestroy(hout));
        }
        std::free(xa);
        std::free(ya);
    }
    CK(hipFree(d));
    return 0;
}

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
// than the pageable transfers minus the registered ones.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 host_register.hip -o host_register
//   ./host_register [floats] [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
    CK(hipFree(d));
    return 0;
}

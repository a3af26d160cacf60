// fft_trace.hip -- phase timeline of fir_fft_f64_kernel (development tool, not
// part of the product).  Builds the kernel with LCFIR_FFT_TRACE, runs config 2
// (2 x 28.8 M samples, 4001 taps), and prints, per wave, the average cycles
// spent in each phase of a steady-state unit over 64 workgroups.
//   hipcc -O3 --offload-arch=gfx950 -I../csrc -DLCFIR_FFT_TRACE fft_trace.hip -o fft_trace
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir_fft.hpp"

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static const char *kNames[] = {"stage1 dft16+tw",    "B0 barrier",       "WG write",
                               "B1 barrier",         "A + x1 exchange",  "B + x2 exchange",
                               "C read+dft8",        "pair step",        "prefetch + A' + x3",
                               "B' + x4 exchange",   "C' + final write", "B2 barrier",
                               "final read+dft16",   "stores+peak"};
constexpr int kPhases = 14;

int main(int argc, char **argv) {
    const int64_t n = 28800000;
    const int nch = 2, T = 4001;
    std::vector<float> hx((size_t)n * nch);
    uint64_t s = 12345;
    for (auto &v : hx) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        v = (float)((double)(s >> 11) / 9007199254740992.0 - 0.5);
    }
    std::vector<double> taps(T);
    for (int i = 0; i < T; ++i) taps[i] = std::sin(0.001 * i) / (1.0 + i);
    float *dx, *dy;
    double *dt;
    CK(hipMalloc(&dx, sizeof(float) * hx.size()));
    CK(hipMalloc(&dy, sizeof(float) * hx.size()));
    CK(hipMalloc(&dt, sizeof(double) * T));
    CK(hipMemcpy(dx, hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, taps.data(), sizeof(double) * T, hipMemcpyHostToDevice));
    lcfir::FftPlan plan;
    std::string err;
    if (!lcfir::fft_plan_build(plan, dt, T, lcfir::FftTuning{}, nullptr, err)) {
        std::fprintf(stderr, "plan: %s\n", err.c_str());
        return 1;
    }
    lcfir::DirectParams p{};
    p.x = dx;
    p.x_lo = 0;
    p.x_hi = n;
    p.x_stride = n;
    p.y = dy;
    p.y_lo = 0;
    p.y_stride = n;
    p.taps = dt;
    p.ntaps = T;
    p.half = (T - 1) / 2;
    p.start = 0;
    p.end = n;
    // "peak": fused peak into one slot (as bench.py does, peak_stride 0);
    // "peakch": one slot per channel
    unsigned *dpeak = nullptr;
    CK(hipMalloc(&dpeak, 64));
    CK(hipMemset(dpeak, 0, 64));
    if (argc > 1 && std::string(argv[1]) == "peak") {
        p.peak = dpeak;
        p.peak_stride = 0;
    } else if (argc > 1 && std::string(argv[1]) == "peakch") {
        p.peak = dpeak;
        p.peak_stride = 1;
    }
    auto launch = [&]() { return lcfir::fft_launch(plan, p, nch, nullptr, err); };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 3; ++it)
        if (!launch()) return 1;
    // 5 rounds of 10 launches: min and median of the round means
    const int reps = 10, rounds = 5;
    std::vector<float> per;
    for (int r = 0; r < rounds; ++r) {
        CK(hipEventRecord(e0));
        for (int it = 0; it < reps; ++it)
            if (!launch()) return 1;
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        per.push_back(t);
    }
    std::sort(per.begin(), per.end());
    const float ms = per[rounds / 2], ms_min = per[0];
    const int64_t units = (int64_t)((n + plan.B - 1) / plan.B) * nch;
    std::printf("kernel %.4f ms (min %.4f)  (%.1f Gsamples/s), units %lld, units/WG %.2f\n", ms / reps, ms_min / reps,
                (double)n * nch / (ms / reps * 1e-3) / 1e9, (long long)units, (double)units / plan.cus);
#ifndef LCFIR_FFT_TRACE
    return 0;
#else
    static unsigned long long tr[64][8][24];
    CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_fft_trace), sizeof(tr)));
    // s_memtime counts at the constant 100 MHz "REFCLK" on some parts and the
    // shader clock on others: print raw ticks and the unit total.
    std::printf("%-26s", "phase \\ wave");
    for (int w = 0; w < 8; ++w) std::printf("%9d", w);
    std::printf("%9s\n", "avg");
    double total[8] = {0};
    for (int ph = 0; ph < kPhases; ++ph) {
        std::printf("%-26s", kNames[ph]);
        double sum = 0;
        for (int w = 0; w < 8; ++w) {
            double acc = 0;
            for (int g = 0; g < 64; ++g) acc += (double)(tr[g][w][ph + 1] - tr[g][w][ph]);
            acc /= 64;
            total[w] += acc;
            sum += acc;
            std::printf("%9.0f", acc);
        }
        std::printf("%9.0f\n", sum / 8);
    }
    std::printf("%-26s", "unit total");
    for (int w = 0; w < 8; ++w) std::printf("%9.0f", total[w]);
    std::printf("\n");
    return 0;
#endif
}

// launch_trace.hip -- per-unit timeline of whole fir_fft_f64_kernel launches
// (development tool, not part of the product).  Builds the kernel with
// LCFIR_FFT_UTRACE: thread 0 of every workgroup stamps s_memrealtime (100 MHz,
// one clock for the whole chip) at entry, at the top of every unit and at exit.
// For a channel length n (argv[1], default config 2's 28.8 M) it prints the
// launch time, the spread of workgroup starts and ends, and the mean duration
// of the first, the steady-state and the last unit of a workgroup.
//   hipcc -O3 --offload-arch=gfx950 -I../csrc -DLCFIR_FFT_UTRACE launch_trace.hip -o launch_trace
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

// one wave busy-waiting `ticks` of the 100 MHz clock: an almost idle GPU between launches
__global__ void spin_kernel(long long ticks) {
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

int main(int argc, char **argv) {
    const int64_t n = argc > 1 ? std::atoll(argv[1]) : 28800000;
    const int reps = argc > 2 ? std::atoi(argv[2]) : 10;
    const int sets = argc > 3 ? std::max(1, std::atoi(argv[3])) : 1; // buffer sets rotated over launches
    const int nch = argc > 5 ? std::atoi(argv[5]) : 2, T = 4001;
    std::vector<float> hx((size_t)n * nch);
    uint64_t s = 12345;
    for (auto &v : hx) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        v = (float)((double)(s >> 11) / 9007199254740992.0 - 0.5);
    }
    std::vector<double> taps(T);
    for (int i = 0; i < T; ++i) taps[i] = std::sin(0.001 * i) / (1.0 + i);
    std::vector<float *> dxs(sets), dys(sets);
    double *dt;
    for (int i = 0; i < sets; ++i) {
        CK(hipMalloc(&dxs[i], sizeof(float) * hx.size()));
        CK(hipMalloc(&dys[i], sizeof(float) * hx.size()));
        CK(hipMemcpy(dxs[i], hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice));
    }
    float *dx = dxs[0], *dy = dys[0];
    CK(hipMalloc(&dt, sizeof(double) * T));
    CK(hipMemcpy(dt, taps.data(), sizeof(double) * T, hipMemcpyHostToDevice));
    lcfir::FftPlan plan;
    std::string err;
    // the traced kernel is fir_fft_f64_kernel (L = 16 384); the L = 32 768 one
    // has no unit stamps and would also need DirectParams::park
    lcfir::FftTuning tune;
    tune.seg_len = lcfir::kFftL;
    if (!lcfir::fft_plan_build(plan, dt, T, tune, nullptr, err)) {
        std::fprintf(stderr, "plan: %s\n", err.c_str());
        return 1;
    }
    lcfir::DirectParams p{};
    p.x = dx;
    p.x_hi = n;
    p.x_stride = n;
    p.y = dy;
    p.y_stride = n;
    p.taps = dt;
    p.ntaps = T;
    p.half = (T - 1) / 2;
    p.end = n;
    unsigned *dpeak = nullptr;
    CK(hipMalloc(&dpeak, 64));
    CK(hipMemset(dpeak, 0, 64));
    p.peak = (argc > 4 && std::atoi(argv[4]) < 0) ? nullptr : dpeak; // argv[4]: peak stride, < 0 = no peak
    p.peak_stride = argc > 4 ? std::max(0, std::atoi(argv[4])) : 0;
    int which = 0;
    auto launch = [&]() {
        which = (which + 1) % sets;
        p.x = dxs[which];
        p.y = dys[which];
        if (!lcfir::fft_launch(plan, p, nch, nullptr, err)) {
            std::fprintf(stderr, "launch: %s\n", err.c_str());
            std::exit(1);
        }
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 3; ++it) launch();
    CK(hipEventRecord(e0));
    const int gap_us = argc > 6 ? std::atoi(argv[6]) : 0; // > 0: a spin kernel of ~gap_us between launches
    for (int it = 0; it < reps; ++it) {
        launch();
        if (gap_us > 0) hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, nullptr, (long long)gap_us * 100);
    }
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    const int64_t units = (int64_t)((n + plan.B - 1) / plan.B) * nch;
    const int grid = (int)std::min<int64_t>(units, plan.cus);
    std::printf("n %lld  units %lld  grid %d  units/WG %.2f  kernel %.4f ms (%.1f Gsamples/s)\n",
                (long long)n, (long long)units, grid, (double)units / grid, ms,
                (double)n * nch / (ms * 1e-3) / 1e9);

    // the last launch's stamps (10 ns ticks)
    static unsigned long long tr[1024][kUtraceSlots];
    CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_fft_utrace), sizeof(tr)));
    unsigned long long t0 = ~0ull, tmax_start = 0, tend_min = ~0ull, tend_max = 0;
    double first = 0, steady = 0, last = 0, entry = 0;
    int64_t nsteady = 0;
    std::vector<double> startd;
    for (int b = 0; b < grid; ++b) t0 = std::min(t0, tr[b][0]);
    for (int b = 0; b < grid; ++b) {
        int nu = 0;
        while (lcfir::fft_unit(nu, b, grid, units) < units) ++nu;
        if (nu + 1 >= kUtraceSlots) {
            std::fprintf(stderr, "too many units per workgroup for the trace\n");
            return 1;
        }
        const unsigned long long *r = tr[b];
        tmax_start = std::max(tmax_start, r[0]);
        tend_min = std::min(tend_min, r[nu + 1]);
        tend_max = std::max(tend_max, r[nu + 1]);
        startd.push_back((double)(r[0] - t0));
        entry += (double)(r[1] - r[0]);
        first += (double)(r[2] - r[1]);
        last += (double)(r[nu + 1] - r[nu]);
        for (int i = 2; i < nu; ++i) {
            steady += (double)(r[i + 1] - r[i]);
            ++nsteady;
        }
    }
    std::sort(startd.begin(), startd.end());
    const double us = 0.01; // 10 ns per tick
    std::printf("WG starts: spread %.2f us (median %.2f us after the first)\n",
                (double)(tmax_start - t0) * us, startd[startd.size() / 2] * us);
    std::printf("WG ends:   first %.2f us, last %.2f us after the first start\n",
                (double)(tend_min - t0) * us, (double)(tend_max - t0) * us);
    std::printf("per WG: entry->unit0 %.2f us, first unit %.2f us, steady unit %.2f us (%lld), last unit %.2f us\n",
                entry / grid * us, first / grid * us, nsteady ? steady / nsteady * us : 0.0,
                (long long)nsteady, last / grid * us);
    // shader clock: s_memtime ticks over s_memrealtime (100 MHz) from entry to exit
    static unsigned long long ck[1024][2];
    CK(hipMemcpyFromSymbol(ck, HIP_SYMBOL(g_fft_uclock), sizeof(ck)));
    double ghz = 0;
    for (int b = 0; b < grid; ++b) {
        int nu = 0;
        while (lcfir::fft_unit(nu, b, grid, units) < units) ++nu;
        ghz += (double)(ck[b][1] - ck[b][0]) / (double)(tr[b][nu + 1] - tr[b][0]) * 0.1;
    }
    std::printf("shader clock (s_memtime / s_memrealtime): %.3f GHz\n", ghz / grid);
    // mean unit duration by round (rounds every workgroup runs)
    const int nmin = (int)(units / grid);
    std::printf("by round (us):");
    for (int i = 1; i <= nmin; ++i) {
        double acc = 0;
        for (int b = 0; b < grid; ++b) acc += (double)(tr[b][i + 1] - tr[b][i]);
        if (i <= 24 || i > nmin - 4) std::printf(" %.2f", acc / grid * us);
        else if (i == 25) std::printf(" ...");
    }
    std::printf("\n");
    return 0;
}

// fft32r_trace.hip -- phase timeline of fir_fft32r_kernel (development tool,
// not part of the product): fft32_trace.hip for the register-resident
// L = 32 768 kernel.  Runs a config-3 shaped launch (8 x 5.76 M samples,
// 8001 symmetric taps) and prints, per wave, the average shader cycles of each
// phase of a steady-state unit over 64 workgroups.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 -I../csrc fft32r_trace.hip -o fft32r_trace
//   ./fft32r_trace [ntaps] [seg_len] [sym|asym] [nrm|-] [cus]
// "nrm": every launch also carries a previous file's normalize (FftNrm) of
// n x nch floats, as config 5's fused form does.  cus: persistent-grid size
// (default: every CU); fewer workgroups than CUs leaves the chip's memory
// system to fewer units in flight (is a phase's cost per CU or chip-wide?).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "fir_fft.hpp"

// lane 0 of every wave of workgroups < 64 records s_memtime at each phase
// boundary of its 3rd unit (the kernel's Probe hook)
__device__ unsigned long long g_fft32r_trace[64][8][24];
// residency: per workgroup its CU (HW_ID with the XCC id), the realtime of its
// first unit's start and of its last unit's end (100 MHz, chip-wide)
constexpr int kOccMax = 2048;
__device__ unsigned long long g_occ[kOccMax][3];
__device__ int g_last_stamp;
struct TraceProbe {
    __device__ static void stamp(int i, int rnd) {
        if (blockIdx.x < 64 && rnd == 2 && (threadIdx.x & 63) == 0)
            g_fft32r_trace[blockIdx.x][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime();
        if (threadIdx.x == 0 && blockIdx.x < kOccMax) {
            if (i == 0 && rnd == 0) {
                const unsigned hw = __builtin_amdgcn_s_getreg(0xF804); // hwreg(HW_REG_HW_ID)
                const unsigned xcc = __builtin_amdgcn_s_getreg(0xF814); // hwreg(HW_REG_XCC_ID)
                g_occ[blockIdx.x][0] = ((unsigned long long)xcc << 32) | hw;
                g_occ[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
            }
            if (i == g_last_stamp) g_occ[blockIdx.x][2] = __builtin_amdgcn_s_memrealtime();
        }
    }
};

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

static const char *kNames[] = {"stage1 (samples, dft32, tw)", "T1 w1", "BAR1", "peak + T1 r1", "BAR2",
                               "T1 w2", "BAR3 + T1 r2", "stage2 (dft32, tw)", "pair loads A", "T2",
                               "stage3 dft16", "pair step", "inv stage3", "T2 back", "inv stage2",
                               "T1' w1", "BAR4", "T1' r1", "BAR5", "T1' w2", "BAR6 + T1' r2",
                               "wait + DMA issue", "final + stores + peak"};
constexpr int kPhases = 23;

int main(int argc, char **argv) {
    const int T = argc > 1 ? std::atoi(argv[1]) : 8001;
    const int seg = argc > 2 ? std::atoi(argv[2]) : 32768;
    const int64_t n = 5760000;
    const int nch = 8;
    std::vector<float> hx((size_t)n * nch);
    uint64_t s = 12345;
    for (auto &v : hx) {
        s = s * 6364136223846793005ULL + 1442695040888963407ULL;
        v = (float)((double)(s >> 11) / 9007199254740992.0 - 0.5);
    }
    // a symmetric low-cut (Blackman windowed sinc, spectral inversion)
    std::vector<double> taps(T);
    const int M = T - 1, half = M / 2;
    double sum = 0;
    for (int i = 0; i < T; ++i) {
        const double d = i - half, fc = 20.0 / 96000.0;
        const double h = d == 0 ? 2 * M_PI * fc : std::sin(2 * M_PI * fc * d) / d;
        const double w = 0.42 - 0.5 * std::cos(2 * M_PI * i / M) + 0.08 * std::cos(4 * M_PI * i / M);
        taps[i] = h * w;
        sum += taps[i];
    }
    for (int i = 0; i < T; ++i) taps[i] = -taps[i] / sum;
    taps[half] += 1.0;
    for (int i = 0; i < half; ++i) taps[T - 1 - i] = taps[i];
    if (argc > 3 && std::string(argv[3]) == "asym")
        for (int i = 0; i < T; ++i) taps[i] += 1e-9 * (2.0 * i / M - 1.0);
    float *dx, *dy;
    double *dt;
    CK(hipMalloc(&dx, sizeof(float) * hx.size()));
    CK(hipMalloc(&dy, sizeof(float) * hx.size()));
    CK(hipMalloc(&dt, sizeof(double) * T));
    CK(hipMemcpy(dx, hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(dt, taps.data(), sizeof(double) * T, hipMemcpyHostToDevice));
    lcfir::FftPlan plan;
    lcfir::FftTuning tune;
    tune.seg_len = seg;
    std::string err;
    if (!lcfir::fft_plan_build(plan, dt, T, tune, nullptr, err)) {
        std::fprintf(stderr, "plan: %s\n", err.c_str());
        return 1;
    }
    if (argc > 5) plan.cus = std::atoi(argv[5]);
    {
        const int last = 23;
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_last_stamp), &last, sizeof(int)));
    }
    std::printf("plan: L %d, parts %d, zero-phase %d, B %d, grid %d\n", plan.L, plan.parts, (int)plan.sym, plan.B,
                plan.cus);
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
    p.half = half;
    p.start = 0;
    p.end = n;
    unsigned *dpeak = nullptr;
    CK(hipMalloc(&dpeak, 64));
    CK(hipMemset(dpeak, 0, 64));
    p.peak = dpeak;
    p.peak_stride = 1;
    const size_t npark = lcfir::fft32_park_doubles(plan);
    if (npark) CK(hipMalloc(reinterpret_cast<void **>(&p.park), npark * sizeof(double)));
    const size_t nscr = lcfir::fft_scratch_doubles(plan, p, nch);
    if (nscr) {
        CK(hipMalloc(reinterpret_cast<void **>(&p.y64), nscr * sizeof(double)));
        p.y64_stride = std::min<int64_t>(p.end - p.start, lcfir::fft_chunk_span(plan));
    }
    const bool with_nrm = argc > 4 && std::string(argv[4]) == "nrm";
    lcfir::FftNrm nrm{};
    if (with_nrm) {
        float *dprev;
        unsigned *dnpk;
        CK(hipMalloc(&dprev, sizeof(float) * hx.size()));
        CK(hipMemcpy(dprev, hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice));
        CK(hipMalloc(&dnpk, 4));
        const float two = 2.0f; // peak > 1: the rescale runs
        CK(hipMemcpy(dnpk, &two, 4, hipMemcpyHostToDevice));
        nrm.y = dprev;
        nrm.peak = dnpk;
        nrm.count = (int64_t)hx.size();
        nrm.npeak = 1;
        if (!lcfir::fft_nrm_fusable(plan, nrm, p, nch)) {
            std::fprintf(stderr, "normalize not fusable at this shape\n");
            return 1;
        }
        std::printf("fused normalize of %lld floats per launch\n", (long long)nrm.count);
    }
    if (!plan.reg32) {
        std::fprintf(stderr, "this plan runs no register kernel\n");
        return 1;
    }
    // one launch chunk covers the whole channel: fft_launch_group's q for it
    lcfir::DirectParams q = p;
    q.seg0 = 0;
    q.ntaps = plan.ntaps;
    auto launch = [&]() {
        return with_nrm ? lcfir::fft32r_launch_one<lcfir::kFftOutSym, true, TraceProbe>(plan, q, nch, nullptr, err, nrm)
                        : lcfir::fft32r_launch_one<lcfir::kFftOutSym, false, TraceProbe>(plan, q, nch, nullptr, err);
    };
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int it = 0; it < 20; ++it)
        if (!launch()) return 1;
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
    {
        // workgroups resident at once per CU (from the last timed launch)
        static unsigned long long occ[kOccMax][3];
        CK(hipMemcpyFromSymbol(occ, HIP_SYMBOL(g_occ), sizeof(occ)));
        const int nwg = (int)std::min<int64_t>((int64_t)units, (int64_t)plan.cus);
        std::vector<std::pair<unsigned long long, int>> ev; // (time, +1/-1) per CU key
        std::vector<unsigned long long> keys;
        for (int b = 0; b < std::min(nwg, kOccMax); ++b) {
            // CU identity: XCC, SE (bits 13..15), SH (12), CU (8..11)
            const unsigned long long key = (occ[b][0] >> 32) << 16 | ((occ[b][0] >> 8) & 0xFF);
            keys.push_back(key);
        }
        std::vector<unsigned long long> uk = keys;
        std::sort(uk.begin(), uk.end());
        uk.erase(std::unique(uk.begin(), uk.end()), uk.end());
        int maxc = 0;
        double sum_max = 0;
        for (unsigned long long k : uk) {
            std::vector<std::pair<unsigned long long, int>> e;
            for (int b = 0; b < (int)keys.size(); ++b)
                if (keys[b] == k) {
                    e.push_back({occ[b][1], 1});
                    e.push_back({occ[b][2], -1});
                }
            std::sort(e.begin(), e.end());
            int c = 0, m = 0;
            for (auto &x : e) m = std::max(m, c += x.second);
            maxc = std::max(maxc, m);
            sum_max += m;
        }
        std::printf("residency: %d workgroups on %zu CUs; max resident per CU %d, mean of per-CU max %.2f\n",
                    (int)keys.size(), uk.size(), maxc, uk.empty() ? 0.0 : sum_max / (double)uk.size());
        // the persistent grid's tail: each workgroup's busy span (its first
        // unit's start to its last unit's end, 100 MHz realtime) against the
        // launch's span; units are atomic and equal, so the launch lasts
        // ceil(units / grid) unit times and the last round keeps only
        // units mod grid CUs busy
        const int nk = std::min(nwg, kOccMax);
        unsigned long long t0 = ~0ull, t1 = 0;
        double busy = 0;
        std::vector<double> ends;
        for (int b = 0; b < nk; ++b) {
            t0 = std::min(t0, occ[b][1]);
            t1 = std::max(t1, occ[b][2]);
        }
        for (int b = 0; b < nk; ++b) {
            busy += (double)(occ[b][2] - occ[b][1]);
            ends.push_back((double)(occ[b][2] - t0));
        }
        std::sort(ends.begin(), ends.end());
        const double span = (double)(t1 - t0);
        const int64_t full = units / nk, rem = units % nk;
        std::printf("tail: %lld units on %d workgroups = %lld full rounds + %lld units; workgroups busy %.3f of "
                    "the launch span (ideal %.3f = units / (grid x ceil(units / grid))); first workgroup done at "
                    "%.3f of the span, median %.3f\n",
                    (long long)units, nk, (long long)full, (long long)rem, busy / (nk * span),
                    (double)units / ((double)nk * (double)(full + (rem ? 1 : 0))), ends.front() / span,
                    ends[ends.size() / 2] / span);
    }
    static unsigned long long tr[64][8][24];
    CK(hipMemcpyFromSymbol(tr, HIP_SYMBOL(g_fft32r_trace), sizeof(tr)));
    const int nw = 8, nph = kPhases;
    std::printf("%-32s", "phase \\ wave");
    for (int w = 0; w < nw; ++w) std::printf("%8d", w);
    std::printf("%8s\n", "avg");
    double total[8] = {0};
    for (int ph = 0; ph < nph; ++ph) {
        std::printf("%-32s", kNames[ph]);
        double sum2 = 0;
        for (int w = 0; w < nw; ++w) {
            double acc = 0;
            for (int g = 0; g < 64; ++g) acc += (double)(tr[g][w][ph + 1] - tr[g][w][ph]);
            acc /= 64;
            total[w] += acc;
            sum2 += acc;
            std::printf("%8.0f", acc);
        }
        std::printf("%8.0f\n", sum2 / nw);
    }
    std::printf("%-32s", "unit total");
    for (int w = 0; w < nw; ++w) std::printf("%8.0f", total[w]);
    std::printf("\n");
    return 0;
}

// cu_split.hip -- config 5's per-rank step with the previous file's normalize
// on CUs of its own (development tool, not part of the product).  Config 5
// (one 60-min stereo file per rank, 4 001 taps, the normalize deferred to the
// next step) runs the rescale fused into the filter launch today (the older
// waves' barrier waits, fir_fft32r_kernel's nrm_half); this tool measures the
// alternative: the rescale as a separate kernel on W CUs (one 1 024-thread
// workgroup per CU, pinned there by its LDS request) on a second stream,
// concurrently with the filter's persistent grid on the other 256 - W CUs.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 -I../csrc cu_split.hip -o cu_split
//   ./cu_split [W,W,...]
// Prints: the filter alone (all CUs, and 256 - W), the fused launch, the
// rescale alone on W CUs, and both at once (events around the pair).
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

constexpr int kNT = 1024;
constexpr int kPinLds = 96 * 1024; // > half the CU's LDS: one workgroup per CU

// y[i] = (float)((double)y[i] * gain), the product's normalize arithmetic
// (fft_nrm_store); float4 per thread, kDepth loads in flight per thread
template <int kDepth>
__global__ __launch_bounds__(kNT) void rescale_kernel(float *y, int64_t n4, const float *peak) {
    extern __shared__ float pin[];
    if (threadIdx.x == 0x7FFFFFFF) pin[0] = 0.0f; // keeps the LDS request
    const double gain = 1.0 / (double)peak[0];
    typedef float f4 __attribute__((ext_vector_type(4)));
    f4 *y4 = reinterpret_cast<f4 *>(y);
    const int64_t stride = (int64_t)gridDim.x * kNT;
    for (int64_t base = (int64_t)blockIdx.x * kNT * kDepth; base < n4; base += stride * kDepth) {
        f4 v[kDepth];
#pragma unroll
        for (int k = 0; k < kDepth; ++k) {
            const int64_t i = base + (int64_t)k * kNT + threadIdx.x;
            if (i < n4) v[k] = __builtin_nontemporal_load(y4 + i);
        }
#pragma unroll
        for (int k = 0; k < kDepth; ++k) {
            const int64_t i = base + (int64_t)k * kNT + threadIdx.x;
            if (i < n4) {
                f4 o;
                o.x = (float)((double)v[k].x * gain);
                o.y = (float)((double)v[k].y * gain);
                o.z = (float)((double)v[k].z * gain);
                o.w = (float)((double)v[k].w * gain);
                __builtin_nontemporal_store(o, y4 + i);
            }
        }
    }
}

int main(int argc, char **argv) {
    std::vector<int> ws = {16, 24, 32, 48};
    if (argc > 1) {
        ws.clear();
        for (const char *s = argv[1]; *s;) {
            ws.push_back(std::atoi(s));
            while (*s && *s != ',') ++s;
            if (*s) ++s;
        }
    }
    const int T = 4001, nch = 2;
    const int64_t n = 172800000; // 60 min at 48 kHz
    const size_t tot = (size_t)n * nch;
    std::vector<double> taps(T);
    const int M = T - 1, half = M / 2;
    double sum = 0;
    for (int i = 0; i < T; ++i) {
        const double d = i - half, fc = 20.0 / 48000.0;
        const double h = d == 0 ? 2 * M_PI * fc : std::sin(2 * M_PI * fc * d) / d;
        const double w = 0.42 - 0.5 * std::cos(2 * M_PI * i / M) + 0.08 * std::cos(4 * M_PI * i / M);
        taps[i] = h * w;
        sum += taps[i];
    }
    for (int i = 0; i < T; ++i) taps[i] = -taps[i] / sum;
    taps[half] += 1.0;
    for (int i = 0; i < half; ++i) taps[T - 1 - i] = taps[i];
    float *dx, *dy, *dprev, *dnpk;
    double *dt;
    unsigned *dpeak;
    CK(hipMalloc(&dx, sizeof(float) * tot));
    CK(hipMalloc(&dy, sizeof(float) * tot));
    CK(hipMalloc(&dprev, sizeof(float) * tot));
    CK(hipMalloc(&dt, sizeof(double) * T));
    CK(hipMalloc(&dpeak, 64));
    CK(hipMalloc(&dnpk, 4));
    {
        std::vector<float> hx(tot);
        uint64_t s = 12345;
        for (auto &v : hx) {
            s = s * 6364136223846793005ULL + 1442695040888963407ULL;
            v = (float)((double)(s >> 11) / 9007199254740992.0 - 0.5);
        }
        CK(hipMemcpy(dx, hx.data(), sizeof(float) * tot, hipMemcpyHostToDevice));
        CK(hipMemcpy(dprev, hx.data(), sizeof(float) * tot, hipMemcpyHostToDevice));
    }
    CK(hipMemcpy(dt, taps.data(), sizeof(double) * T, hipMemcpyHostToDevice));
    CK(hipMemset(dpeak, 0, 64));
    const float one = 1.0f; // gain 1: the buffer keeps its values over the repeats
    CK(hipMemcpy(dnpk, &one, 4, hipMemcpyHostToDevice));
    lcfir::FftPlan plan;
    lcfir::FftTuning tune;
    std::string err;
    if (!lcfir::fft_plan_build(plan, dt, T, tune, nullptr, err) || !plan.reg32) {
        std::fprintf(stderr, "plan: %s\n", err.c_str());
        return 1;
    }
    const int cus = plan.cus;
    lcfir::DirectParams p{};
    p.x = dx;
    p.x_lo = 0;
    p.x_hi = n;
    p.x_stride = n;
    p.y = dy;
    p.y_lo = 0;
    p.y_stride = n;
    p.taps = dt;
    p.ntaps = plan.ntaps;
    p.half = half;
    p.start = 0;
    p.end = n;
    p.peak = dpeak;
    p.peak_stride = 1;
    p.seg0 = 0;
    lcfir::FftNrm nrm{};
    nrm.y = dprev;
    nrm.peak = reinterpret_cast<unsigned *>(dnpk);
    nrm.count = (int64_t)tot;
    nrm.npeak = 1;
    nrm.force = 1;
    if (!lcfir::fft_nrm_fusable(plan, nrm, p, nch)) {
        std::fprintf(stderr, "normalize not fusable\n");
        return 1;
    }
    hipStream_t sa, sb;
    CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&rescale_kernel<4>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, kPinLds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&rescale_kernel<8>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, kPinLds));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&rescale_kernel<16>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, kPinLds));
    int depth = 4;
    hipEvent_t e0, e1, ea, eb;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventCreate(&ea));
    CK(hipEventCreate(&eb));
    auto filt = [&](int g, bool fused) {
        lcfir::FftPlan pl = plan;
        pl.cus = g;
        const bool ok = fused ? lcfir::fft32r_launch_one<lcfir::kFftOutSym, true>(pl, p, nch, sa, err, nrm)
                              : lcfir::fft32r_launch_one<lcfir::kFftOutSym, false>(pl, p, nch, sa, err);
        if (!ok) {
            std::fprintf(stderr, "launch: %s\n", err.c_str());
            std::exit(1);
        }
    };
    auto rescale = [&](int w, hipStream_t s) {
        if (depth == 16)
            hipLaunchKernelGGL(rescale_kernel<16>, dim3(w), dim3(kNT), kPinLds, s, dprev, (int64_t)(tot / 4), dnpk);
        else if (depth == 8)
            hipLaunchKernelGGL(rescale_kernel<8>, dim3(w), dim3(kNT), kPinLds, s, dprev, (int64_t)(tot / 4), dnpk);
        else
            hipLaunchKernelGGL(rescale_kernel<4>, dim3(w), dim3(kNT), kPinLds, s, dprev, (int64_t)(tot / 4), dnpk);
        CK(hipGetLastError());
    };
    // median of 7 timings of `reps` back-to-back issues of f on stream sa (f may fork to sb)
    auto timeit = [&](auto f) {
        const int reps = 5;
        std::vector<float> v;
        for (int r = 0; r < 8; ++r) {
            CK(hipEventRecord(e0, sa));
            for (int i = 0; i < reps; ++i) f();
            CK(hipEventRecord(e1, sa));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) v.push_back(t / reps); // the first: warm-up
        }
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    const double gb = 2.0 * 4.0 * (double)tot / 1e6; // MB: / ms = GB/s
    const float t_f = timeit([&] { filt(cus, false); });
    const float t_fused = timeit([&] { filt(cus, true); });
    const float t_full = timeit([&] { rescale(4 * cus, sa); });
    std::printf("filter alone, %d CUs: %.4f ms\n", cus, t_f);
    std::printf("filter + fused rescale (product, config 5 deferred): %.4f ms (+%.4f)\n", t_fused, t_fused - t_f);
    std::printf("rescale alone, %d workgroups: %.4f ms (%.0f GB/s)\n", 4 * cus, t_full, gb / t_full);
    for (int d : {4, 8, 16}) {
        depth = d;
        std::printf("rescale: %d float4 in flight per thread (%d KiB per CU)\n", d, d * kNT * 16 / 1024);
        for (int w : ws) {
            const int g = cus - w;
            const float t_g = timeit([&] { filt(g, false); });
            const float t_r = timeit([&] { rescale(w, sa); });
            // both: the rescale first on sb (it takes its W CUs), the filter on sa; sa waits for sb
            const float t_b = timeit([&] {
                CK(hipEventRecord(ea, sa));
                CK(hipStreamWaitEvent(sb, ea, 0));
                rescale(w, sb);
                CK(hipEventRecord(eb, sb));
                filt(g, false);
                CK(hipStreamWaitEvent(sa, eb, 0));
            });
            std::printf("  W %3d: filter on %d CUs %.4f ms; rescale on %d CUs %.4f ms (%.0f GB/s, %.1f GB/s per CU); "
                        "both at once %.4f ms (fused %.4f, filter alone %.4f)\n",
                        w, g, t_g, w, t_r, gb / t_r, gb / t_r / w, t_b, t_fused, t_f);
        }
    }
    return 0;
}

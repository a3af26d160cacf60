// rocfft_ols.hip -- the vendor-library baseline for the hot path: config 2's
// overlap-save convolution (2 channels x 28.8 M f32 samples, 4001 taps, the
// same segments as fir_fft.hpp: L = 16384, B = L - T + 1) built from rocFFT's
// batched f64 real transforms plus three small kernels, timed with HIP events
// next to liblcfir's fused kernel on the same data.
//
//   gather   x (f32) -> segments xs[s][0, L) in f64, zero padded at the edges
//   R2C      rocFFT, f64, batch = segments
//   multiply X[s][k] *= G[k]              (G = R2C of the zero-padded taps)
//   C2R      rocFFT, f64, batch = segments
//   scatter  y[n0 + m - (T-1)] = c[m] / L, m in [T-1, L), rounded to f32
//
// Reports each stage's time, the total, liblcfir's time for the same outputs
// and the largest |difference| between the two outputs.
//
// build (from audio-fir-filter_amd/):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../include -Icsrc -o tools/rocfft_ols \
//         tools/rocfft_ols.hip -L. -llcfir -lrocfft -Wl,-rpath,'$ORIGIN/..'
// usage: tools/rocfft_ols [reps]
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "lcfir.h"

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)
#define RK(x)                                                                  \
    do {                                                                       \
        rocfft_status s_ = (x);                                                \
        if (s_ != rocfft_status_success) {                                     \
            std::fprintf(stderr, "%s:%d rocfft status %d\n", __FILE__, __LINE__, (int)s_); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr int kL = 16384, kC = kL / 2 + 1;

__global__ void gather(const float *x, int64_t n, int nseg, int B, int half, double *xs) {
    const int s = blockIdx.y; // segment of the (channel, segment) grid
    const int ch = s / nseg, seg = s % nseg;
    const int64_t base = (int64_t)seg * B - half;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kL; i += gridDim.x * blockDim.x) {
        const int64_t g = base + i;
        xs[(size_t)s * kL + i] = g >= 0 && g < n ? (double)x[(size_t)ch * n + g] : 0.0;
    }
}

__global__ void multiply(double2 *X, const double2 *G, int nsegs) {
    const int s = blockIdx.y;
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < kC; k += gridDim.x * blockDim.x) {
        const double2 a = X[(size_t)s * kC + k], g = G[k];
        X[(size_t)s * kC + k] = make_double2(a.x * g.x - a.y * g.y, a.x * g.y + a.y * g.x);
    }
}

__global__ void scatter(const double *c, int64_t n, int nseg, int B, int T, float *y) {
    const int s = blockIdx.y;
    const int ch = s / nseg, seg = s % nseg;
    const int64_t n0 = (int64_t)seg * B;
    for (int m = T - 1 + blockIdx.x * blockDim.x + threadIdx.x; m < kL; m += gridDim.x * blockDim.x) {
        const int64_t o = n0 + m - (T - 1);
        if (o < n) y[(size_t)ch * n + o] = (float)(c[(size_t)s * kL + m] * (1.0 / kL));
    }
}

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const int nch = 2;
    const int64_t n = 28800000;
    // the bench's taps: -f 20 -s 48 at 48 kHz (4001)
    int32_t T = 0;
    if (lcfir_design_lowcut(20.0, 48.0, 48000.0, nullptr, 0, &T) != LCFIR_OK) return 1;
    std::vector<double> taps((size_t)T);
    if (lcfir_design_lowcut(20.0, 48.0, 48000.0, taps.data(), T, &T) != LCFIR_OK) return 1;
    const int half = (T - 1) / 2, B = kL - T + 1;
    const int nseg = (int)((n + B - 1) / B), S = nch * nseg;
    std::printf("taps %d  segments %d x %d  L %d  B %d\n", T, nch, nseg, kL, B);

    // synthetic int24-like samples
    std::vector<float> hx((size_t)nch * n);
    uint64_t st = 0x9E3779B97F4A7C15ULL;
    for (auto &v : hx) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        v = (float)((int32_t)(st >> 40) - (1 << 23)) / (float)(1 << 23) * 0.5f;
    }
    float *x, *y, *y_ref;
    double *xs, *c, *hz;
    double2 *X, *G;
    CK(hipMalloc(&x, sizeof(float) * hx.size()));
    CK(hipMalloc(&y, sizeof(float) * hx.size()));
    CK(hipMalloc(&y_ref, sizeof(float) * hx.size()));
    CK(hipMalloc(&xs, sizeof(double) * (size_t)S * kL));
    CK(hipMalloc(&c, sizeof(double) * (size_t)S * kL));
    CK(hipMalloc(&X, sizeof(double2) * (size_t)S * kC));
    CK(hipMalloc(&G, sizeof(double2) * kC));
    CK(hipMalloc(&hz, sizeof(double) * kL));
    CK(hipMemcpy(x, hx.data(), sizeof(float) * hx.size(), hipMemcpyHostToDevice));
    std::vector<double> hpad(kL, 0.0);
    for (int k = 0; k < T; ++k) hpad[(size_t)k] = taps[(size_t)k];
    CK(hipMemcpy(hz, hpad.data(), sizeof(double) * kL, hipMemcpyHostToDevice));

    RK(rocfft_setup());
    size_t len = kL;
    rocfft_plan fwd, inv, fwd1;
    RK(rocfft_plan_create(&fwd, rocfft_placement_notinplace, rocfft_transform_type_real_forward,
                          rocfft_precision_double, 1, &len, (size_t)S, nullptr));
    RK(rocfft_plan_create(&inv, rocfft_placement_notinplace, rocfft_transform_type_real_inverse,
                          rocfft_precision_double, 1, &len, (size_t)S, nullptr));
    RK(rocfft_plan_create(&fwd1, rocfft_placement_notinplace, rocfft_transform_type_real_forward,
                          rocfft_precision_double, 1, &len, 1, nullptr));
    size_t wf = 0, wi = 0, w1 = 0;
    RK(rocfft_plan_get_work_buffer_size(fwd, &wf));
    RK(rocfft_plan_get_work_buffer_size(inv, &wi));
    RK(rocfft_plan_get_work_buffer_size(fwd1, &w1));
    const size_t wbytes = std::max(std::max(wf, wi), w1);
    void *work = nullptr;
    if (wbytes) CK(hipMalloc(&work, wbytes));
    hipStream_t s;
    CK(hipStreamCreate(&s));
    rocfft_execution_info info;
    RK(rocfft_execution_info_create(&info));
    RK(rocfft_execution_info_set_stream(info, s));
    if (wbytes) RK(rocfft_execution_info_set_work_buffer(info, work, wbytes));
    {
        void *in[1] = {hz}, *out[1] = {G};
        RK(rocfft_execute(fwd1, in, out, info));
    }

    auto run = [&](hipEvent_t *ev) {
        CK(hipEventRecord(ev[0], s));
        hipLaunchKernelGGL(gather, dim3(16, S), dim3(256), 0, s, x, n, nseg, B, half, xs);
        CK(hipEventRecord(ev[1], s));
        void *in0[1] = {xs}, *out0[1] = {X};
        RK(rocfft_execute(fwd, in0, out0, info));
        CK(hipEventRecord(ev[2], s));
        hipLaunchKernelGGL(multiply, dim3(8, S), dim3(256), 0, s, X, G, S);
        CK(hipEventRecord(ev[3], s));
        void *in1[1] = {X}, *out1[1] = {c};
        RK(rocfft_execute(inv, in1, out1, info));
        CK(hipEventRecord(ev[4], s));
        hipLaunchKernelGGL(scatter, dim3(16, S), dim3(256), 0, s, c, n, nseg, B, T, y);
        CK(hipEventRecord(ev[5], s));
    };
    hipEvent_t ev[6];
    for (auto &e : ev) CK(hipEventCreate(&e));
    for (int i = 0; i < 3; ++i) run(ev); // warm-up (plans, clocks)
    CK(hipStreamSynchronize(s));
    double acc[5] = {0, 0, 0, 0, 0};
    for (int r = 0; r < reps; ++r) {
        run(ev);
        CK(hipEventSynchronize(ev[5]));
        for (int i = 0; i < 5; ++i) {
            float ms = 0;
            CK(hipEventElapsedTime(&ms, ev[i], ev[i + 1]));
            acc[i] += ms;
        }
    }
    const char *names[5] = {"gather", "R2C", "multiply", "C2R", "scatter"};
    double tot = 0;
    for (int i = 0; i < 5; ++i) {
        std::printf("%-9s %.4f ms\n", names[i], acc[i] / reps);
        tot += acc[i] / reps;
    }
    std::printf("rocFFT overlap-save total %.4f ms  (%.1f Gsamples/s)\n", tot, (double)nch * n / (tot * 1e-3) / 1e9);

    // liblcfir's fused kernel on the same data, same stream
    lcfir_ctx *ctx = nullptr;
    if (lcfir_ctx_create(0, taps.data(), T, &ctx) != LCFIR_OK) return 1;
    for (int i = 0; i < 3; ++i)
        if (lcfir_filter_channels_dev(ctx, x, n, nch, n, y_ref, n, nullptr, s) != LCFIR_OK) return 1;
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(ev[0], s));
    for (int r = 0; r < reps; ++r) lcfir_filter_channels_dev(ctx, x, n, nch, n, y_ref, n, nullptr, s);
    CK(hipEventRecord(ev[1], s));
    CK(hipEventSynchronize(ev[1]));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, ev[0], ev[1]));
    std::printf("liblcfir fused kernel    %.4f ms  (%.1f Gsamples/s)\n", ms / reps, (double)nch * n / (ms / reps * 1e-3) / 1e9);
    std::vector<float> a(hx.size()), b(hx.size());
    CK(hipMemcpy(a.data(), y, sizeof(float) * a.size(), hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), y_ref, sizeof(float) * b.size(), hipMemcpyDeviceToHost));
    double md = 0;
    size_t ndiff = 0;
    for (size_t i = 0; i < a.size(); ++i) {
        const double d = std::fabs((double)a[i] - (double)b[i]);
        md = std::max(md, d);
        ndiff += a[i] != b[i];
    }
    std::printf("max |rocFFT - liblcfir| %.3e  (%zu of %zu outputs differ)\n", md, ndiff, a.size());
    lcfir_ctx_destroy(ctx);
    rocfft_execution_info_destroy(info);
    rocfft_plan_destroy(fwd);
    rocfft_plan_destroy(inv);
    rocfft_plan_destroy(fwd1);
    rocfft_cleanup();
    return 0;
}

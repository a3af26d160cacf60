// overlap2wg.hip -- does splitting the register kernel's CU into two
// independent workgroups overlap LDS exchanges with f64 arithmetic?
// (development tool, not part of the product)
//
// fir_fft32r_kernel runs one 512-thread workgroup per CU; its six barriers
// keep every wave in the same phase, so the CU's LDS pipe and its f64 VALU
// take turns instead of overlapping.  This tool runs
// the kernel's per-unit sequence of phases -- the same DFT32 / DFT16 /
// twiddle-chain arithmetic (fir_fft32r.hpp) on 32 complex f64 per thread and
// the same LDS exchanges (two workgroup rounds with barriers, two wave-local
// rounds, back again) -- with no global memory at all, in two shapes that do
// the same work per CU:
//   * 512 threads per workgroup, one workgroup per CU (the product's shape);
//   * 256 threads per workgroup, two per CU (each with half the LDS), whose
//     phases are free to drift apart.
// Prints the time of each and their ratio.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 -I../csrc overlap2wg.hip -o overlap2wg
//   ./overlap2wg [units per workgroup] [cus]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "fir_fft.hpp"

using namespace lcfir;

constexpr int kRg = kR32Rg; // double2 per wave region (fir_fft32r.hpp)

__device__ __forceinline__ void bar() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

template <int NT>
__global__ __launch_bounds__(NT, 2) void mimic(double2 *out, int units, double2 w0) {
    constexpr int NW = NT / 64;
    extern __shared__ double2 lds[];
    double2 a[32], c[32];
    const double t = threadIdx.x * 1e-6 + blockIdx.x * 1e-9;
#pragma unroll
    for (int i = 0; i < 32; ++i) a[i] = make_double2(t + i, t - i);
    double2 wg = make_double2(w0.x - t * 1e-9, w0.y + t * 1e-9);
    double2 acc = make_double2(0.0, 0.0);
    for (int u = 0; u < units; ++u) {
        // laundered per unit (as the kernel does): no address hoisted out of the loop
        int j = threadIdx.x;
        asm volatile("" : "+v"(j));
        const int w = __builtin_amdgcn_readfirstlane(j >> 6), lane = j & 63;
        // stage 1
        dft32(a);
        r32_chain32acc(a, wg);
        // T1 round 1: own region, then gather from the others (barriers)
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 64 * i + lane] = a[i];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = lds[kRg * ((w + i) % NW) + 64 * ((i + 3) & 15) + lane];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * ((w + i + 1) % NW) + 64 * i + lane] = a[16 + i];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) c[16 + i] = lds[kRg * w + 64 * i + lane];
        // stage 2
        dft32(c);
        asm volatile("" : "+v"(wg.x), "+v"(wg.y));
        r32_chain32acc(c, wg);
        // T2: wave-local, two rounds
        double2 R1[16], R2[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 17 * (lane & 15) + 272 * (lane >> 4) + i] = c[i];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R1[i] = lds[kRg * w + 17 * i + 272 * (lane >> 4) + (lane & 15)];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 17 * (lane & 15) + 272 * (lane >> 4) + i] = c[16 + i];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) R2[i] = lds[kRg * w + 17 * i + 272 * (lane >> 4) + (lane & 15)];
        // stage 3, a pair step's worth of arithmetic, inverse stage 3
        dft16f(R1);
        dft16f(R2);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const double2 x = R1[i], y = R2[15 - i];
            R1[i] = make_double2(__builtin_fma(wg.x, x.x, y.y), __builtin_fma(wg.y, x.y, -y.x));
            R2[15 - i] = make_double2(__builtin_fma(wg.y, y.x, x.y), __builtin_fma(wg.x, y.y, x.x));
        }
        dft16f(R1);
        dft16f(R2);
        // T2 back
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 17 * i + 272 * (lane >> 4) + (lane & 15)] = R1[i];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] = lds[kRg * w + 17 * (lane & 15) + 272 * (lane >> 4) + i];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 17 * i + 272 * (lane >> 4) + (lane & 15)] = R2[i];
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) c[16 + i] = lds[kRg * w + 17 * (lane & 15) + 272 * (lane >> 4) + i];
        // inverse stage 2 (laundered base: the powers are rebuilt, not kept live
        // across the pair step, as in the kernel)
        asm volatile("" : "+v"(wg.x), "+v"(wg.y));
        r32_chain32acc(c, wg);
        dft32(c);
        // T1 back (barriers)
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * w + 64 * i + lane] = c[i];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) a[i] = lds[kRg * ((w + i) % NW) + 64 * ((i + 5) & 15) + lane];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) lds[kRg * ((w + i + 1) % NW) + 64 * i + lane] = c[16 + i];
        bar();
#pragma unroll
        for (int i = 0; i < 16; ++i) a[16 + i] = lds[kRg * w + 64 * i + lane];
        bar();
        // final
        asm volatile("" : "+v"(wg.x), "+v"(wg.y));
        r32_chain32acc(a, wg);
        dft32(a);
#pragma unroll
        for (int i = 0; i < 32; ++i) {
            acc = cadd(acc, a[i]);
            a[i] = make_double2(a[i].x * 1e-3 + t, a[i].y * 1e-3 - t); // keep magnitudes bounded
        }
    }
    out[(size_t)blockIdx.x * NT + threadIdx.x] = acc;
}

template <int NT>
float run(double2 *out, int grid, int units) {
    const size_t lds = sizeof(double2) * (size_t)(NT / 64) * kRg;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&mimic<NT>), hipFuncAttributeMaxDynamicSharedMemorySize,
                              (int)lds);
    const double2 w0 = make_double2(0.99998, -0.0063);
    hipLaunchKernelGGL(mimic<NT>, dim3(grid), dim3(NT), lds, 0, out, 2, w0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(mimic<NT>, dim3(grid), dim3(NT), lds, 0, out, units, w0);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        std::fprintf(stderr, "launch: %s\n", hipGetErrorString(e));
        std::exit(1);
    }
    return best;
}

int main(int argc, char **argv) {
    const int units = argc > 1 ? std::atoi(argv[1]) : 64;
    const int cus = argc > 2 ? std::atoi(argv[2]) : 256;
    double2 *out = nullptr;
    if (hipMalloc(&out, sizeof(double2) * 512 * 2 * (size_t)cus) != hipSuccess) return 1;
    const float t512 = run<512>(out, cus, units);
    const float t256 = run<256>(out, 2 * cus, units);
    const double ucyc = 2.4e6 / units; // cycles per ms at 2.4 GHz / units
    std::printf("one 512-thread workgroup per CU: %.3f ms (%.0f cycles per unit at 2.4 GHz)\n", t512, t512 * ucyc);
    std::printf("two 256-thread workgroups per CU: %.3f ms (%.0f cycles per pair of half units)\n", t256,
                t256 * ucyc);
    std::printf("ratio (512 / 256x2): %.3f\n", t512 / t256);
    return 0;
}

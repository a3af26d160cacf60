// valu_mix.hip -- f64 VALU rate of the FFT kernels' own instruction mix
// (development tool): the column stage's arithmetic (dft8 + twiddle8 with
// lane-varying twiddles, csrc/fir_fft.hpp) in registers only, no LDS, no
// barriers, one or two independent columns per wave, at 1, 2 and 4 waves per
// SIMD.  Reports ns per f64 wave-instruction per SIMD (f64 instructions per
// iteration counted from this file's own ISA by the caller) so the kernels'
// real-operand rate can be compared with tools/valu_rate.hip's single-operand
// v_fma_f64 chains.
//
// build: hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../csrc -o valu_mix valu_mix.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "fir_fft.hpp"

using namespace lcfir;

template <int COLS>
__global__ __launch_bounds__(1024) void mix(double2 *out, int n, double2 w1) {
    double2 x[COLS][8], tws[8];
    const double t = threadIdx.x * 1e-3;
    powers8(make_double2(w1.x + t * 1e-9, w1.y - t * 1e-9), tws);
#pragma unroll
    for (int c = 0; c < COLS; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) x[c][i] = make_double2(t + i + c, t - i);
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int c = 0; c < COLS; ++c) {
            dft8(x[c]);
            twiddle8(x[c], tws);
        }
    }
    double2 s = make_double2(0.0, 0.0);
#pragma unroll
    for (int c = 0; c < COLS; ++c)
#pragma unroll
        for (int i = 0; i < 8; ++i) s = cadd(s, x[c][i]);
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int COLS>
void run(double2 *out, int cus, int threads, int f64_per_col_iter) {
    const int n = 20000;
    const double2 w1 = make_double2(0.9999, -0.0001);
    hipLaunchKernelGGL(mix<COLS>, dim3(cus), dim3(threads), 0, 0, out, 200, w1);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL(mix<COLS>, dim3(cus), dim3(threads), 0, 0, out, n, w1);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double waves_per_simd = threads / 64.0 / 4.0;
    const double inst_per_simd = waves_per_simd * (double)n * COLS * f64_per_col_iter;
    std::printf("cols %d  %4d thr/CU (%.0f waves/SIMD): %.3f ms  %.2f ns per f64 wave-instr per SIMD\n", COLS,
                threads, waves_per_simd, ms, ms * 1e6 / inst_per_simd);
}

int main(int argc, char **argv) {
    const int f64 = argc > 1 ? std::atoi(argv[1]) : 84; // f64 instructions per dft8 + twiddle8
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double2 *out;
    (void)hipMalloc(&out, sizeof(double2) * cus * 1024);
    for (int thr : {256, 512, 1024}) {
        run<1>(out, cus, thr, f64);
        run<2>(out, cus, thr, f64);
    }
    return 0;
}

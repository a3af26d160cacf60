// lds_bench.hip -- LDS exchange throughput in the FFT kernel's shape
// (development tool): 512 threads, one workgroup per CU (137 KiB LDS), each
// lane writes 16 x 16 B then reads 16 x 16 B per iteration, contiguous
// conflict-free patterns.  Variants: store width (b128 / 2 x b64 / 4 x b32),
// and with or without a workgroup barrier between write and read.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <int MODE, bool BAR>
__global__ __launch_bounds__(512) void lds_kernel(double2 *out, int iters) {
    extern __shared__ double2 s[];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    double2 acc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = make_double2(r + j, r - j);
    for (int it = 0; it < iters; ++it) {
        double2 *blk = BAR ? s : s + 1024 * w; // WG-wide or wave-private region
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int idx = BAR ? 512 * r + j : 64 * r + lane;
            if constexpr (MODE == 0) blk[idx] = acc[r];
            else if constexpr (MODE == 1) {
                volatile double *d = reinterpret_cast<volatile double *>(blk);
                d[2 * idx] = acc[r].x;
                d[2 * idx + 1] = acc[r].y;
            } else {
                volatile float *f = reinterpret_cast<volatile float *>(blk);
                const int4 v = *reinterpret_cast<const int4 *>(&acc[r]);
                f[4 * idx] = __int_as_float(v.x);
                f[4 * idx + 1] = __int_as_float(v.y);
                f[4 * idx + 2] = __int_as_float(v.z);
                f[4 * idx + 3] = __int_as_float(v.w);
            }
        }
        if (BAR) __syncthreads();
        else __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int idx = BAR ? 512 * ((r + 1) & 15) + j : 64 * ((r + 1) & 15) + (lane ^ 1);
            const double2 v = blk[idx];
            acc[r] = make_double2(v.x + 1.0, v.y - 1.0);
        }
        if (BAR) __syncthreads();
        else __builtin_amdgcn_wave_barrier();
    }
    double t = 0;
#pragma unroll
    for (int r = 0; r < 16; ++r) t += acc[r].x + acc[r].y;
    out[blockIdx.x * 512 + j] = make_double2(t, 0);
}

template <int MODE, bool BAR>
void run(const char *name, double2 *out, int cus) {
    const size_t lds = 137 * 1024;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&lds_kernel<MODE, BAR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const int iters = 2000;
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    hipLaunchKernelGGL((lds_kernel<MODE, BAR>), dim3(cus), dim3(512), lds, 0, out, 10);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((lds_kernel<MODE, BAR>), dim3(cus), dim3(512), lds, 0, out, iters);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double bytes = 2.0 * 512 * 16 * 16 * (double)iters; // per CU: write + read
    const double per_exchange_us = ms * 1e3 / iters;
    std::printf("%-28s %.3f ms  %.2f us per 128 KiB exchange (write+read)  %.0f GB/s per CU\n", name, ms,
                per_exchange_us, bytes / (ms * 1e-3) / 1e9);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double2 *out;
    (void)hipMalloc(&out, sizeof(double2) * 512 * cus);
    run<0, true>("b128 + WG barrier", out, cus);
    run<1, true>("b64 + WG barrier", out, cus);
    run<2, true>("b32 + WG barrier", out, cus);
    run<0, false>("b128 wave-private", out, cus);
    run<1, false>("b64 wave-private", out, cus);
    run<2, false>("b32 wave-private", out, cus);
    return 0;
}

// overlap_bench.hip -- can f64 VALU work and LDS exchanges overlap on one CU?
// (development tool).  One 512-thread workgroup per CU, 137 KiB LDS.
// Roles per wave: F = dependent-free f64 FMA stream (8 independent chains),
// X = LDS exchange (16 ds_write_b128 + 16 ds_read_b128 into a wave-private
// region), I = idle.  Modes: all F; all X; F on waves 0-3 + X on 4-7; the
// same split but waves 4-7 also do F (both kinds interleaved per wave).
#include <hip/hip_runtime.h>

#include <cstdio>

__device__ __forceinline__ void fma_block(double (&a)[8], int n) {
    for (int i = 0; i < n; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) a[k] = __builtin_fma(a[k], 1.0000001, 0.5);
    }
}

template <int MODE, int NT = 512>
__global__ __launch_bounds__(NT) void ov_kernel(double2 *out, int iters, int fma_n) {
    extern __shared__ double2 s[];
    const int j = threadIdx.x, lane = j & 63, w = j >> 6;
    if (NT == 1024) iters /= 2; // same work per CU, spread over 16 waves
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] = k + j;
    double2 acc[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = make_double2(r + j, r - j);
    const bool doF = MODE == 0 || (MODE == 2 && w < 4) || MODE == 3;
    const bool doX = MODE == 1 || (MODE == 2 && w >= 4) || (MODE == 3);
    double2 *blk = s + (NT == 1024 ? 512 : 1024) * w; // 128 KiB of private blocks
    for (int it = 0; it < iters; ++it) {
        if (doF) fma_block(a, fma_n);
        if (doX) {
#pragma unroll
            for (int r = 0; r < 16; ++r) blk[64 * r + lane] = acc[r];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const double2 v = blk[64 * ((r + 1) & 15) + (lane ^ 1)];
                acc[r] = make_double2(v.x + 1.0, v.y - 1.0);
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    double t = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += a[k];
#pragma unroll
    for (int r = 0; r < 16; ++r) t += acc[r].x + acc[r].y;
    out[blockIdx.x * NT + j] = make_double2(t, 0);
}

template <int MODE, int NT = 512>
float run(double2 *out, int cus, int iters, int fma_n) {
    const size_t lds = 137 * 1024;
    (void)hipFuncSetAttribute(reinterpret_cast<const void *>(&ov_kernel<MODE, NT>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL((ov_kernel<MODE, NT>), dim3(cus), dim3(NT), lds, 0, out, 20, fma_n);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((ov_kernel<MODE, NT>), dim3(cus), dim3(NT), lds, 0, out, iters, fma_n);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms;
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    double2 *out;
    (void)hipMalloc(&out, sizeof(double2) * 1024 * cus);
    const int iters = 2000;
    for (int fma_n : {8, 16, 32}) {
        const float f = run<0>(out, cus, iters, fma_n), x = run<1>(out, cus, iters, fma_n),
                    split = run<2>(out, cus, iters, fma_n), both = run<3>(out, cus, iters, fma_n);
        std::printf("fma/iter %3d x8 chains: F-only %.3f ms  X-only %.3f ms  F(0-3)+X(4-7) %.3f ms  "
                    "F+X every wave %.3f ms   (sum F+X %.3f, max %.3f)\n",
                    fma_n * 8, f, x, split, both, f + x, f > x ? f : x);
        const float f16 = run<0, 1024>(out, cus, iters, fma_n), x16 = run<1, 1024>(out, cus, iters, fma_n),
                    both16 = run<3, 1024>(out, cus, iters, fma_n);
        std::printf("   16 waves/CU, same work: F-only %.3f ms  X-only %.3f ms  F+X every wave %.3f ms\n",
                    f16, x16, both16);
    }
    return 0;
}

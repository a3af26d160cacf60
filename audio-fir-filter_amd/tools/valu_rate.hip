// valu_rate.hip -- raw f64 VALU issue rates on this GPU (development tool):
// 8 independent chains per lane of v_fma_f64 / v_add_f64 / v_mul_f64.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int OP, int CH = 8>
__global__ void k(double *out, int n, double c) {
    double a[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) a[i] = threadIdx.x + i;
    for (int it = 0; it < n; ++it) {
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            if (OP == 0) a[i] = __builtin_fma(a[i], c, 0.5);
            else if (OP == 1) a[i] = a[i] + c;
            else a[i] = a[i] * c;
        }
    }
    double t = 0;
#pragma unroll
    for (int i = 0; i < CH; ++i) t += a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = t;
}

template <int OP, int CH = 8>
void run(const char *name, double *out, int cus, int threads) {
    const int n = 800000 / CH;
    hipLaunchKernelGGL((k<OP, CH>), dim3(cus), dim3(threads), 0, 0, out, 100, 1.0000001);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventRecord(a);
    hipLaunchKernelGGL((k<OP, CH>), dim3(cus), dim3(threads), 0, 0, out, n, 1.0000001);
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    const double inst = (double)cus * threads * n * CH; // lane-instructions
    const double waves = (double)cus * threads / 64;
    std::printf("%-8s %4d thr/CU: %.3f ms  %.1f T lane-op/s  %.2f ns per wave-instr per SIMD  (waves %.0f)\n",
                name, threads, ms, inst / (ms * 1e-3) / 1e12,
                (ms * 1e6) / ((double)n * CH * waves / (cus * 4.0)), waves);
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    int clk = 0;
    (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
    std::printf("CUs %d, max clock %d MHz\n", cus, clk / 1000);
    double *out;
    (void)hipMalloc(&out, sizeof(double) * cus * 1024);
    for (int thr : {256, 512}) {
        run<0, 8>("fma x8", out, cus, thr);
        run<0, 16>("fma x16", out, cus, thr);
        run<0, 32>("fma x32", out, cus, thr);
        run<1, 16>("add x16", out, cus, thr);
    }
    return 0;
}

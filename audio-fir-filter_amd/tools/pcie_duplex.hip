// pcie_duplex.hip -- host link throughput one way and both ways at once
// (development tool, not part of the product).  The drop-in's fan-out
// (tests/cpp/dropin_bench, ProcessFile.cp:57-87's threads) moves every sample
// H2D and every output D2H; its bound is 56 GB/s H2D only if the link carries
// the D2H stream at the same time.  This tool measures, for 256 MiB per
// direction: copy-engine transfers (hipMemcpyAsync) from hipHostMalloc and from
// hipHostRegister'd memory, and kernel transfers through the buffers' device
// mappings (the kcopy variant's path), each direction alone and both at once
// on two streams; then 4 streams per direction.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 pcie_duplex.hip -o pcie_duplex
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

__global__ __launch_bounds__(256) void copy_kernel(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                   int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * 256;
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n4; k += stride) dst[k] = src[k];
}

constexpr size_t kBytes = (size_t)256 << 20;

struct Bufs {
    char *h_in, *h_out;     // host (pinned one way or the other)
    char *m_in, *m_out;     // their device mappings
    char *d_in, *d_out;     // device
};

int main() {
    hipStream_t st[8];
    for (auto &s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    Bufs hm{}, hr{};
    CK(hipHostMalloc(reinterpret_cast<void **>(&hm.h_in), kBytes, hipHostMallocDefault));
    CK(hipHostMalloc(reinterpret_cast<void **>(&hm.h_out), kBytes, hipHostMallocDefault));
    hr.h_in = static_cast<char *>(std::aligned_alloc(4096, kBytes));
    hr.h_out = static_cast<char *>(std::aligned_alloc(4096, kBytes));
    std::memset(hr.h_in, 1, kBytes);
    std::memset(hr.h_out, 2, kBytes);
    std::memset(hm.h_in, 1, kBytes);
    CK(hipHostRegister(hr.h_in, kBytes, hipHostRegisterDefault));
    CK(hipHostRegister(hr.h_out, kBytes, hipHostRegisterDefault));
    for (Bufs *b : {&hm, &hr}) {
        CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&b->m_in), b->h_in, 0));
        CK(hipHostGetDevicePointer(reinterpret_cast<void **>(&b->m_out), b->h_out, 0));
    }
    char *d_in, *d_out;
    CK(hipMalloc(&d_in, kBytes));
    CK(hipMalloc(&d_out, kBytes));
    CK(hipMemset(d_out, 3, kBytes));
    // ms of f() (issues on the streams; e0 on st[0] first, every stream joined into st[0])
    auto timeit = [&](int nst, auto f) {
        std::vector<float> v;
        for (int r = 0; r < 5; ++r) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, st[0]));
            for (int i = 1; i < nst; ++i) CK(hipStreamWaitEvent(st[i], e0, 0));
            f();
            for (int i = 1; i < nst; ++i) {
                hipEvent_t ej;
                CK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
                CK(hipEventRecord(ej, st[i]));
                CK(hipStreamWaitEvent(st[0], ej, 0));
                CK(hipEventDestroy(ej));
            }
            CK(hipEventRecord(e1, st[0]));
            CK(hipEventSynchronize(e1));
            float t = 0;
            CK(hipEventElapsedTime(&t, e0, e1));
            if (r) v.push_back(t);
        }
        std::sort(v.begin(), v.end());
        return v[v.size() / 2];
    };
    const double mb = (double)kBytes / 1e6;
    auto report = [&](const char *name, float ms, double dirs) {
        std::printf("%-44s %8.3f ms  %7.1f GB/s total\n", name, ms, dirs * mb / ms);
    };
    auto kcopy = [&](void *dst, const void *src, size_t bytes, hipStream_t s, int blocks) {
        hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, s, static_cast<float4 *>(dst),
                           static_cast<const float4 *>(src), (int64_t)(bytes / 16));
        CK(hipGetLastError());
    };
    for (int which = 0; which < 2; ++which) {
        Bufs &b = which ? hr : hm;
        const char *tag = which ? "hipHostRegister" : "hipHostMalloc";
        std::printf("-- %s\n", tag);
        report("sdma H2D", timeit(1, [&] { CK(hipMemcpyAsync(d_in, b.h_in, kBytes, hipMemcpyHostToDevice, st[0])); }),
               1);
        report("sdma D2H", timeit(1, [&] { CK(hipMemcpyAsync(b.h_out, d_out, kBytes, hipMemcpyDeviceToHost, st[0])); }),
               1);
        report("sdma H2D + D2H (two streams)", timeit(2, [&] {
                   CK(hipMemcpyAsync(d_in, b.h_in, kBytes, hipMemcpyHostToDevice, st[0]));
                   CK(hipMemcpyAsync(b.h_out, d_out, kBytes, hipMemcpyDeviceToHost, st[1]));
               }),
               2);
        report("sdma H2D + D2H (4 + 4 streams, quarters)", timeit(8, [&] {
                   for (int q = 0; q < 4; ++q) {
                       const size_t o = q * (kBytes / 4);
                       CK(hipMemcpyAsync(d_in + o, b.h_in + o, kBytes / 4, hipMemcpyHostToDevice, st[q]));
                       CK(hipMemcpyAsync(b.h_out + o, d_out + o, kBytes / 4, hipMemcpyDeviceToHost, st[4 + q]));
                   }
               }),
               2);
        for (int blocks : {256, 1024}) {
            char name[96];
            std::snprintf(name, sizeof name, "kernel H2D (%d blocks)", blocks);
            report(name, timeit(1, [&] { kcopy(d_in, b.m_in, kBytes, st[0], blocks); }), 1);
            std::snprintf(name, sizeof name, "kernel D2H (%d blocks)", blocks);
            report(name, timeit(1, [&] { kcopy(b.m_out, d_out, kBytes, st[0], blocks); }), 1);
            std::snprintf(name, sizeof name, "kernel H2D + D2H (%d blocks each)", blocks);
            report(name, timeit(2, [&] {
                       kcopy(d_in, b.m_in, kBytes, st[0], blocks);
                       kcopy(b.m_out, d_out, kBytes, st[1], blocks);
                   }),
                   2);
        }
        report("sdma H2D + kernel D2H", timeit(2, [&] {
                   CK(hipMemcpyAsync(d_in, b.h_in, kBytes, hipMemcpyHostToDevice, st[0]));
                   kcopy(b.m_out, d_out, kBytes, st[1], 1024);
               }),
               2);
    }
    CK(hipHostUnregister(hr.h_in));
    CK(hipHostUnregister(hr.h_out));
    std::free(hr.h_in);
    std::free(hr.h_out);
    return 0;
}

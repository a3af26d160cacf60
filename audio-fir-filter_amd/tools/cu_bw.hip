// cu_bw.hip -- per-CU global-memory throughput (development tool, not part of
// the product).  The register kernels' memory phase (a unit's output stores
// and the next unit's sample loads) and config 5's fused
// rescale both run at a per-CU rate well below 8 TB/s / 256; this tool
// measures that rate by access kind: W workgroups of 1 024 threads, pinned one
// per CU by their LDS request, streaming 16-byte accesses over a 2 GiB buffer.
//   hipcc -O3 -std=c++2b --offload-arch=gfx950 cu_bw.hip -o cu_bw
//   ./cu_bw [W,W,...]
// kinds: read (b128 loads, summed), write (b128 stores), copy (load + store of
// the same float4: the rescale's pattern), each with the default cache policy
// and with the nontemporal bit the product's output stores carry.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            std::exit(1);                                                       \
        }                                                                       \
    } while (0)

constexpr int kNT = 1024, kDepth = 8;
constexpr int kPinLds = 96 * 1024;

// kind: 0 read, 1 write, 2 copy; aux: buffer instruction cache-policy bits
template <int kind, int aux>
__global__ __launch_bounds__(kNT) void bw_kernel(float *buf, int64_t n4, float *sink) {
    extern __shared__ float pin[];
    if (threadIdx.x == 0x7FFFFFFF) pin[0] = 0.0f;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(buf, (short)0, 0x7FFFFFFF, 0x00020000);
    using b128_t = decltype(__builtin_amdgcn_raw_buffer_load_b128(r, 0, 0, 0));
    // byte offsets stay below 2 GiB: n4 <= 2^27 float4
    const int stride = gridDim.x * kNT * kDepth;
    b128_t acc = {};
    for (int base = blockIdx.x * kNT * kDepth; base < n4; base += stride) {
        b128_t v[kDepth];
        if constexpr (kind != 1) {
#pragma unroll
            for (int k = 0; k < kDepth; ++k)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, 16 * (base + k * kNT + (int)threadIdx.x), 0, aux);
        }
#pragma unroll
        for (int k = 0; k < kDepth; ++k) {
            if constexpr (kind == 0) {
                acc ^= v[k];
            } else if constexpr (kind == 1) {
                const b128_t c = {(unsigned)base, (unsigned)k, 1u, 2u};
                __builtin_amdgcn_raw_buffer_store_b128(c, r, 16 * (base + k * kNT + (int)threadIdx.x), 0, aux);
            } else {
                __builtin_amdgcn_raw_buffer_store_b128(v[k], r, 16 * (base + k * kNT + (int)threadIdx.x), 0, aux);
            }
        }
    }
    if constexpr (kind == 0)
        if (acc[0] == 0x12345678u && acc[1] == 0x9ABCDEFu) sink[threadIdx.x] = 1.0f;
}

template <int kind, int aux>
static float run(float *buf, int64_t n4, float *sink, int w) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipFuncSetAttribute(reinterpret_cast<const void *>(&bw_kernel<kind, aux>),
                           hipFuncAttributeMaxDynamicSharedMemorySize, kPinLds));
    std::vector<float> v;
    for (int r = 0; r < 6; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((bw_kernel<kind, aux>), dim3(w), dim3(kNT), kPinLds, 0, buf, n4, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        if (r) v.push_back(t);
    }
    std::sort(v.begin(), v.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    std::vector<int> ws = {1, 8, 32, 128, 256};
    if (argc > 1) {
        ws.clear();
        for (const char *s = argv[1]; *s;) {
            ws.push_back(std::atoi(s));
            while (*s && *s != ',') ++s;
            if (*s) ++s;
        }
    }
    const int64_t full4 = (int64_t)1 << 27; // 2 GiB of float4
    float *buf, *sink;
    CK(hipMalloc(&buf, full4 * 16));
    CK(hipMalloc(&sink, kNT * 4));
    CK(hipMemset(buf, 0, full4 * 16));
    std::printf("%-18s %5s %10s %12s %14s\n", "kind", "CUs", "ms", "GB/s", "GB/s per CU");
    for (int w : ws) {
        // ~ 20 ms of traffic at 35 GB/s per CU, at most the whole buffer
        const int64_t n4 = std::min<int64_t>(full4, (int64_t)w * 40000000LL / 16);
        const double mb = (double)n4 * 16 / 1e6;
        auto line = [&](const char *name, float ms, double factor) {
            const double gbs = mb * factor / ms;
            std::printf("%-18s %5d %10.4f %12.1f %14.2f\n", name, w, ms, gbs, gbs / w);
        };
        line("read", run<0, 0>(buf, n4, sink, w), 1.0);
        line("read nt", run<0, 2>(buf, n4, sink, w), 1.0);
        line("write", run<1, 0>(buf, n4, sink, w), 1.0);
        line("write nt", run<1, 2>(buf, n4, sink, w), 1.0);
        line("copy (r+w bytes)", run<2, 0>(buf, n4, sink, w), 2.0);
        line("copy nt", run<2, 2>(buf, n4, sink, w), 2.0);
    }
    return 0;
}

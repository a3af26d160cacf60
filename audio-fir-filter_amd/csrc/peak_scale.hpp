// peak_scale.hpp -- the post-pass of ProcessFile.cp:91-101 on the device.
//
//   maxMag = max over channels of VectorMath::max_mag()     (ProcessFile.cp:92-96)
//   if (maxMag > 1.0f || opts.normalize) AudioSamples::normalize(buf)  (:98-101)
//
// Both are HBM-bound streaming passes: 16-B loads/stores per lane where the
// channel base is 16-B aligned, grid-stride, a handful of blocks per CU.
// The peak is kept as the bit pattern of a non-negative float so that an
// integer atomicMax orders it correctly.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lcfir {

__device__ __forceinline__ float wave_max(float m) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
    return m;
}

// grid: (blocks_per_channel, nch)
__global__ __launch_bounds__(256) void peak_kernel(const float *__restrict__ y, int64_t stride,
                                                   int64_t n, unsigned *__restrict__ peak) {
    const float *__restrict__ p = y + (int64_t)blockIdx.y * stride;
    float m = 0.0f;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        const int64_t n4 = n / 4;
        const float4 *__restrict__ p4 = reinterpret_cast<const float4 *>(p);
        for (int64_t i = tid; i < n4; i += nthreads) {
            const float4 v = p4[i];
            m = fmaxf(m, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
        }
        for (int64_t i = n4 * 4 + tid; i < n; i += nthreads) m = fmaxf(m, fabsf(p[i]));
    } else {
        for (int64_t i = tid; i < n; i += nthreads) m = fmaxf(m, fabsf(p[i]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) atomicMax(peak + blockIdx.y, __float_as_uint(m));
}

__global__ __launch_bounds__(256) void peak_zero_kernel(unsigned *__restrict__ peak, int count) {
    for (int i = threadIdx.x; i < count; i += blockDim.x) peak[i] = 0u;
}

__device__ __forceinline__ float scale_one(float v, double gain) {
    return (float)((double)v * gain);
}

// Normalize: the decision is taken on the device from d_peak, so no host
// round trip sits between the filter and the rescale.  Block (0, 0) also
// zeroes clear[0, nclear) -- the next step's peak slots (a separate buffer),
// which saves the batch driver one launch per step.
__global__ __launch_bounds__(256) void normalize_kernel(float *__restrict__ y, int64_t stride,
                                                        int64_t n, const unsigned *__restrict__ peak,
                                                        int npeak, int force, unsigned *__restrict__ clear,
                                                        int nclear) {
    if (blockIdx.x == 0 && blockIdx.y == 0)
        for (int i = threadIdx.x; i < nclear; i += blockDim.x) clear[i] = 0u;
    float pk = 0.0f;
    for (int i = 0; i < npeak; ++i) pk = fmaxf(pk, __uint_as_float(peak[i]));
    if (!(pk > 1.0f || force) || !(pk > 0.0f)) return;
    const double gain = 1.0 / (double)pk;
    float *__restrict__ p = y + (int64_t)blockIdx.y * stride;
    const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nthreads = (int64_t)gridDim.x * blockDim.x;
    if ((reinterpret_cast<uintptr_t>(p) & 15) == 0) {
        const int64_t n4 = n / 4;
        float4 *__restrict__ p4 = reinterpret_cast<float4 *>(p);
        int64_t i = tid;
        // four independent 16-byte loads in flight per thread: HBM latency x
        // bandwidth needs ~10 MB in flight chip-wide (2.76 GB per 60-min file
        // at 5.6 TB/s instead of 5.1 with one)
        for (; i + 3 * nthreads < n4; i += 4 * nthreads) {
            float4 v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = p4[i + u * nthreads];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                v[u].x = scale_one(v[u].x, gain);
                v[u].y = scale_one(v[u].y, gain);
                v[u].z = scale_one(v[u].z, gain);
                v[u].w = scale_one(v[u].w, gain);
                p4[i + u * nthreads] = v[u];
            }
        }
        for (; i < n4; i += nthreads) {
            float4 v = p4[i];
            v.x = scale_one(v.x, gain);
            v.y = scale_one(v.y, gain);
            v.z = scale_one(v.z, gain);
            v.w = scale_one(v.w, gain);
            p4[i] = v;
        }
        for (int64_t i = n4 * 4 + tid; i < n; i += nthreads) p[i] = scale_one(p[i], gain);
    } else {
        for (int64_t i = tid; i < n; i += nthreads) p[i] = scale_one(p[i], gain);
    }
}

} // namespace lcfir

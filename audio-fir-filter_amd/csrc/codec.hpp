// codec.hpp -- on-device sample codec either side of the hot path
// (SURVEY.md s8f row 1).
//
// The reference reads a whole file into a deinterleaved AudioBuffer of
// VectorMath<float32_t> (AudioSamples::readAll, ProcessFile.cp:40-41) and
// writes it back with AudioSamples::writeAll(buf, true) (:115-117); both live
// in the un-vendored c_lib, so the exact scaling/rounding is parity-unpinned.
// We use the standard conventions:
//   decode  int b-bit  v -> (float) v / 2^(b-1)        (exact in f32 for b <= 24)
//           float32    v -> v
//   encode  float f -> clamp(rint(f * 2^(b-1)), -2^(b-1), 2^(b-1) - 1)  (RNE, in f64)
//           float32    f -> f
// Interleaved frames (WAV: little-endian, AIFF: big-endian) <-> planar
// channels [nch][frames] with a channel stride.  Both kernels are HBM-bound
// byte shuffles: one thread per interleaved sample, byte-exact, no MFMA.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lcfir {

struct PcmFormat {
    int bytes;      // 2, 3, 4
    bool is_float;  // float32 (bytes == 4)
    bool big_endian;
};

__device__ __forceinline__ uint32_t load_bytes(const uint8_t *__restrict__ p, int nb, bool be) {
    uint32_t v = 0;
    if (be) {
        for (int b = 0; b < nb; ++b) v = (v << 8) | p[b];
    } else {
        for (int b = nb - 1; b >= 0; --b) v = (v << 8) | p[b];
    }
    return v;
}

__device__ __forceinline__ void store_bytes(uint8_t *__restrict__ p, uint32_t v, int nb, bool be) {
    if (be) {
        for (int b = nb - 1; b >= 0; --b) {
            p[b] = (uint8_t)(v & 0xff);
            v >>= 8;
        }
    } else {
        for (int b = 0; b < nb; ++b) {
            p[b] = (uint8_t)(v & 0xff);
            v >>= 8;
        }
    }
}

__device__ __forceinline__ float decode_one(uint32_t raw, const PcmFormat f) {
    if (f.is_float) return __uint_as_float(raw);
    const int bits = 8 * f.bytes;
    const int32_t s = (int32_t)(raw << (32 - bits)) >> (32 - bits); // sign-extend
    return (float)((double)s * (1.0 / (double)(1u << (bits - 1))));
}

__device__ __forceinline__ uint32_t encode_one(float v, const PcmFormat f) {
    if (f.is_float) return __float_as_uint(v);
    const int bits = 8 * f.bytes;
    const double scale = (double)(1ull << (bits - 1));
    double q = rint((double)v * scale);
    const double lo = -scale, hi = scale - 1.0;
    q = q < lo ? lo : (q > hi ? hi : q);
    if (q != q) q = 0.0; // NaN -> 0
    return (uint32_t)(int32_t)(int64_t)q;
}

// grid-stride over interleaved sample index i = frame * nch + ch
__global__ __launch_bounds__(256) void decode_pcm_kernel(const uint8_t *__restrict__ in, PcmFormat f,
                                                        int nch, int64_t frames,
                                                        float *__restrict__ out, int64_t stride) {
    const int64_t total = frames * nch;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t fr = i / nch;
        const int ch = (int)(i - fr * nch);
        const uint32_t raw = load_bytes(in + i * f.bytes, f.bytes, f.big_endian);
        out[(int64_t)ch * stride + fr] = decode_one(raw, f);
    }
}

__global__ __launch_bounds__(256) void encode_pcm_kernel(const float *__restrict__ in, int64_t stride,
                                                        int nch, int64_t frames, PcmFormat f,
                                                        uint8_t *__restrict__ out) {
    const int64_t total = frames * nch;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t fr = i / nch;
        const int ch = (int)(i - fr * nch);
        store_bytes(out + i * f.bytes, encode_one(in[(int64_t)ch * stride + fr], f), f.bytes,
                    f.big_endian);
    }
}

// encode_pcm_kernel with ProcessFile.cp:91-101's normalize folded in: the
// per-file decision (peak = max d_peak[0..npeak); rescale iff peak > 1 or
// force) is read from the device, and each sample is scaled exactly as
// normalize_kernel does ((float)((double)v * (1.0 / (double)peak))) before
// it is encoded -- byte-identical to normalize + encode, without the
// rescale pass's 8 B/sample of HBM traffic.
__global__ __launch_bounds__(256) void encode_pcm_scaled_kernel(const float *__restrict__ in, int64_t stride,
                                                               int nch, int64_t frames, PcmFormat f,
                                                               const unsigned *__restrict__ peak, int npeak,
                                                               int force, uint8_t *__restrict__ out) {
    float pk = 0.0f;
    for (int i = 0; i < npeak; ++i) pk = fmaxf(pk, __uint_as_float(peak[i]));
    const bool scale = (pk > 1.0f || force) && pk > 0.0f;
    const double gain = scale ? 1.0 / (double)pk : 1.0;
    const int64_t total = frames * nch;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (int64_t)gridDim.x * blockDim.x) {
        const int64_t fr = i / nch;
        const int ch = (int)(i - fr * nch);
        float v = in[(int64_t)ch * stride + fr];
        if (scale) v = (float)((double)v * gain);
        store_bytes(out + i * f.bytes, encode_one(v, f), f.bytes, f.big_endian);
    }
}

} // namespace lcfir

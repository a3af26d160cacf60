// fir_direct.hpp -- direct-form f64 FIR kernel for gfx950 (CDNA4).
//
// Replaces the per-output tap dot product of apply_filter_range
// (reference FilterCore.h:56-76, the three loops around
// WindowedSinc<float64_t>::fms).  One launch evaluates
//     y[n] = (float) sum_{k=0}^{T-1} h[k] * x[n - half + k]   (x = 0 outside [0,N))
// for n in [start, end) of every channel in the grid's y dimension.
//
// Mapping (output-stationary, no cross-lane reduction):
//   * a workgroup owns BO = NT*R consecutive outputs of one channel;
//   * lane `tid` owns the R consecutive outputs n0 + tid*R + [0, R);
//   * taps are processed in stages of <= tc taps: each stage stages the taps
//     h[c, c+kc) and the f64-converted sample window x[n0 - half + c, +BO+kc)
//     in LDS (f32 -> f64 conversion happens once per staged sample, not per
//     tap), then every lane slides a 2R-sample register window over its part
//     of the LDS window: per R taps it reads R samples (ds_read_b64) and R
//     wave-uniform taps (LDS broadcast) and issues R*R v_fma_f64.
//   * the LDS sample window is padded by one double every R doubles, so the
//     lane-strided ds_read_b64 of 32 lanes hit 64 distinct banks.
//   * accumulation order per output is k = 0, 1, ..., T-1, one fused
//     multiply-add per tap, starting from +0.0: the f64 result is bit-identical
//     to a strict-order C `fma()` chain (oracle ORACLE_FMA), and the zero
//     padding reproduces the reference's shortened prologue/epilogue sums.
//   * the narrowing is a plain (float) cast = RNE, as static_cast<float32_t>
//     at FilterCore.h:59,67,74.
//   * optional fused per-channel peak (max |y|) for ProcessFile.cp:91-96.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lcfir {

struct DirectParams {
    const float *x;    // channel 0, element 0 = global sample index x_lo
    int64_t x_lo;      // first global index present in x
    int64_t x_hi;      // one past the last present global index (<= channel length)
    int64_t x_stride;  // elements between channels of x
    float *y;          // channel 0, element 0 = global output index y_lo
    int64_t y_lo;
    int64_t y_stride;
    const double *taps;
    int32_t ntaps;
    int32_t half;
    int64_t start, end; // output range (global indices)
    int64_t seg0;       // FFT only: first output of the launch's first segment (<= start; fft_launch_group)
    int32_t tc;         // taps per LDS stage (multiple of 2R)
    unsigned *peak;     // max|y| as float bits (nullable): channel c -> peak[c * peak_stride]
    int64_t peak_stride;
    double *y64;        // partitioned FFT only: f64 partial sums, element 0 = output `start`
    int64_t y64_stride;
    double2 *park;      // L = 32768 FFT only: the workgroups' park slabs (fir_fft32.hpp)
};

template <int R>
__device__ __forceinline__ void fma_block(double (&acc)[R], const double (&wlo)[R],
                                          const double (&whi)[R], const double *__restrict__ t) {
#pragma unroll
    for (int u = 0; u < R; ++u) {
        const double h = t[u];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const double w = (r + u < R) ? wlo[r + u] : whi[r + u - R];
            acc[r] = __builtin_fma(h, w, acc[r]);
        }
    }
}

template <int R, int NT>
__global__ __launch_bounds__(NT) void fir_direct_f64_kernel(DirectParams p) {
    extern __shared__ double lds[];
    constexpr int BO = NT * R;
    const int ch = blockIdx.y;
    const int tid = threadIdx.x;
    const float *__restrict__ x = p.x + (int64_t)ch * p.x_stride;
    const int64_t n0 = p.start + (int64_t)blockIdx.x * BO;

    double *sh_t = lds;
    double *sh_x = lds + p.tc;

    double acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0.0;

    for (int c = 0; c < p.ntaps; c += p.tc) {
        // taps in this stage, rounded up to 2R (zero taps beyond T)
        int kc = p.ntaps - c;
        if (kc > p.tc) kc = p.tc;
        kc = (kc + 2 * R - 1) / (2 * R) * (2 * R);
        for (int i = tid; i < kc; i += NT) {
            const int k = c + i;
            sh_t[i] = (k < p.ntaps) ? p.taps[k] : 0.0;
        }
        const int win = BO + kc;
        const int64_t g0 = n0 - p.half + c;
        for (int i = tid; i < win; i += NT) {
            const int64_t g = g0 + i;
            const float v = (g >= p.x_lo && g < p.x_hi) ? x[g - p.x_lo] : 0.0f;
            sh_x[i + i / R] = (double)v;
        }
        __syncthreads();

        const double *__restrict__ wp = sh_x + tid * (R + 1);
        double wa[R], wb[R];
#pragma unroll
        for (int j = 0; j < R; ++j) wa[j] = wp[j];
        for (int k = 0; k < kc; k += 2 * R) {
            const int blk = k / R; // window block index (R samples per block, R+1 with pad)
#pragma unroll
            for (int j = 0; j < R; ++j) wb[j] = wp[(blk + 1) * (R + 1) + j];
            fma_block<R>(acc, wa, wb, sh_t + k);
#pragma unroll
            for (int j = 0; j < R; ++j) wa[j] = wp[(blk + 2) * (R + 1) + j];
            fma_block<R>(acc, wb, wa, sh_t + k + R);
        }
        __syncthreads();
    }

    float m = 0.0f;
    float *__restrict__ y = p.y + (int64_t)ch * p.y_stride;
    const int64_t gb = n0 + (int64_t)tid * R;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int64_t g = gb + r;
        if (g < p.end) {
            const float v = (float)acc[r];
            y[g - p.y_lo] = v;
            m = fmaxf(m, fabsf(v));
        }
    }
    if (p.peak) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
        if ((tid & 63) == 0) atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(m));
    }
}

// LDS bytes a launch of fir_direct_f64_kernel<R, NT> needs for stage size tc.
template <int R, int NT>
constexpr size_t direct_lds_bytes(int tc) {
    return sizeof(double) * ((size_t)tc + (size_t)(NT * R + tc) / R * (R + 1) + (R + 1));
}

} // namespace lcfir

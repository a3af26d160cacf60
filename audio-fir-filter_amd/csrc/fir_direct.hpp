// fir_direct.hpp -- direct-form f64 FIR kernel for gfx950 (CDNA4).
//
// Replaces the per-output tap dot product of apply_filter_range
// (reference FilterCore.h:56-76, the three loops around
// WindowedSinc<float64_t>::fms).  One launch evaluates
//     y[n] = (float) sum_{k=0}^{T-1} h[k] * x[n - half + k]   (x = 0 outside [0,N))
// for n in [start, end) of every channel in the grid's y dimension.
//
// Mapping (output-stationary, no cross-lane reduction):
//   * a tile is BO = NT*R consecutive outputs of one channel; a workgroup
//     walks its channel's tiles (the grid is capped, fir_direct_f64_kernel);
//   * lane `tid` owns the R consecutive outputs n0 + tid*R + [0, R);
//   * taps are processed in stages of <= TC taps (rounded up to R with zero
//     taps): each stage converts the sample window x[n0 - half + c, +BO+kc)
//     to f64 into LDS (once per staged sample, not per tap), then every lane
//     slides a 2R-sample register window over its part of the LDS window: per
//     R taps it reads R samples (ds_read_b64) and R wave-uniform taps (scalar
//     loads into SGPRs, h[c, c+kc) from the zero-padded device copy) and
//     issues R*R v_fma_f64;
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
    unsigned *peak;     // max|y| as float bits (nullable): channel c -> peak[c * peak_stride]
    int64_t peak_stride;
    double *y64;        // partitioned FFT only: f64 partial sums, element 0 = output `start`
    int64_t y64_stride;
    double2 *park;      // L = 32768 FFT only: the workgroups' park slabs (fir_fft32.hpp)
};

// Taps are read through the constant address space: wave-uniform scalar
// loads into SGPRs (v_fma_f64 takes one SGPR operand), which leaves the
// VGPRs to the accumulators and the sample window.
typedef const __attribute__((address_space(4))) double *ctap_ptr;

template <int R>
__device__ __forceinline__ void fma_block(double (&acc)[R], const double (&wlo)[R],
                                          const double (&whi)[R], ctap_ptr t) {
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

// The window of one stage: x[g0, g0 + win) of the channel into v, element
// i = ts + NT j in v[j].  Raw buffer loads through a resource over the part of
// the window that holds data, [lo, hi): element i >= lead reads offset
// 4 (i - lead), offsets past the resource read 0 (the zero padding of
// FilterCore.h's shortened edge sums), and elements before the data (i < lead)
// take an offset far past it -- a compare and a select per load, no reliance on
// negative offsets wrapping.  One offset register per load, all KW loads in
// flight at once, 32-bit offsets for any channel length.
template <int NT, int KW>
__device__ __forceinline__ void direct_load_window(const DirectParams &p, const float *x, int64_t g0, int win,
                                                   int ts, float (&v)[KW]) {
    const int64_t lo = g0 > p.x_lo ? g0 : p.x_lo;
    const int64_t hi = g0 + win < p.x_hi ? g0 + win : p.x_hi;
    const bool any = hi > lo;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float *>(x) + (any ? lo - p.x_lo : 0), (short)0, any ? (int)(4 * (hi - lo)) : 0, 0x00020000);
    const int lead = (int)(lo - g0 < win ? lo - g0 : win);
#pragma unroll
    for (int j = 0; j < KW; ++j) {
        const int i = ts + NT * j;
        const int o = i >= lead ? 4 * (i - lead) : 0x7ffffff0;
        v[j] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0));
    }
}

// taps in stage c, rounded up to R (zero taps beyond T): a 15-tap filter
// issues 16 fmas per output, not 32
template <int R, int TC>
__device__ __forceinline__ int direct_stage_taps(int ntaps, int c) {
    int kc = ntaps - c;
    if (kc > TC) kc = TC;
    return (kc + R - 1) / R * R;
}

// One tile = BO outputs of one channel.  The grid is capped at what the chip
// holds at once (launch_direct) and every workgroup walks its channel's tiles
// with stride gridDim.x, so the fused peak leaves a workgroup as ONE atomic
// per launch: one per wave per tile (57 600 same-address atomics for a
// 28.8 M-sample stereo launch) held a 15-tap filter at 0.67 ms, ~9x its HBM
// time.  Per stage (tile, c):
//   * the window's KW loads per lane were issued during the previous stage's
//     fmas (direct_load_window), so HBM latency overlaps the arithmetic; the
//     stage converts them into LDS;
//   * outputs leave through LDS: lane tid's R results go to a padded row, and
//     the wave then stores consecutive floats (one 256-B run per instruction
//     instead of 64 lanes 64 B apart).
// 3 waves per SIMD: 147 VGPRs hold the next stage's window beside the
// accumulators and the register window (4 spilled 25); the launch caps the
// grid at 3 workgroups per CU to match (lcfir.hip kDirWgPerCu)
constexpr int kDirectWavesPerSimd = 3;

template <int R, int NT, int TC>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(kDirectWavesPerSimd))) void fir_direct_f64_kernel(DirectParams p) {
    extern __shared__ double lds[];
    __shared__ float pk_lds[NT / 64];
    constexpr int BO = NT * R;
    constexpr int KW = (BO + TC + NT - 1) / NT; // window elements per lane, max
    const int ch = blockIdx.y;
    const float *__restrict__ x = p.x + (int64_t)ch * p.x_stride;
    float *__restrict__ y = p.y + (int64_t)ch * p.y_stride;
    const ctap_ptr taps = (ctap_ptr)p.taps; // zero-padded to a multiple of TC (lcfir_ctx_create)
    double *sh_x = lds;
    float *sh_y = reinterpret_cast<float *>(lds); // reused after the last stage
    const int64_t ntiles = (p.end - p.start + BO - 1) / BO;
    float m = 0.0f;

    float v[KW]; // the next stage's window, in flight
    if ((int64_t)blockIdx.x < ntiles)
        direct_load_window<NT, KW>(p, x, p.start + (int64_t)blockIdx.x * BO - p.half, BO + direct_stage_taps<R, TC>(p.ntaps, 0),
                                   (int)threadIdx.x, v);

    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t n0 = p.start + tile * BO;
        // laundered per tile: the per-element offsets below are recomputed,
        // not hoisted out of the tile loop into ~80 spilled registers
        unsigned tid = threadIdx.x;
        asm volatile("" : "+v"(tid));
        double acc[R];
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r] = 0.0;

        for (int c = 0; c < p.ntaps; c += TC) {
            const int kc = direct_stage_taps<R, TC>(p.ntaps, c);
            const int win = BO + kc;
            // window element i = tid + j NT sits at i + i / R (one pad double
            // per R): a per-lane base plus a constant per j, since NT % R == 0
            double *__restrict__ xs = sh_x + (tid + tid / R);
#pragma unroll
            for (int j = 0; j < BO / NT; ++j) xs[j * (NT + NT / R)] = (double)v[j];
#pragma unroll
            for (int j = BO / NT; j < KW; ++j)
                if (tid + j * NT < win) xs[j * (NT + NT / R)] = (double)v[j];
            __syncthreads();

            // the next stage's window: (tile, c + TC), else the next tile's first
            {
                int64_t nt = tile;
                int nc = c + TC;
                if (nc >= p.ntaps) {
                    nc = 0;
                    nt = tile + gridDim.x;
                }
                if (nt < ntiles) {
                    int ts = (int)tid; // laundered per stage: per-j offsets are not hoisted
                    asm volatile("" : "+v"(ts));
                    direct_load_window<NT, KW>(p, x, p.start + nt * BO - p.half + nc,
                                               BO + direct_stage_taps<R, TC>(p.ntaps, nc), ts, v);
                }
            }

            const double *__restrict__ wp = sh_x + tid * (R + 1);
            double wa[R], wb[R];
#pragma unroll
            for (int j = 0; j < R; ++j) wa[j] = wp[j];
            int k = 0;
#pragma unroll 1
            for (; k + 2 * R <= kc; k += 2 * R) {
                const int blk = k / R; // window block index (R samples per block, R+1 with pad)
#pragma unroll
                for (int j = 0; j < R; ++j) wb[j] = wp[(blk + 1) * (R + 1) + j];
                fma_block<R>(acc, wa, wb, taps + c + k);
#pragma unroll
                for (int j = 0; j < R; ++j) wa[j] = wp[(blk + 2) * (R + 1) + j];
                fma_block<R>(acc, wb, wa, taps + c + k + R);
            }
            if (k < kc) { // an odd number of R-tap blocks: the last one
                const int blk = k / R;
#pragma unroll
                for (int j = 0; j < R; ++j) wb[j] = wp[(blk + 1) * (R + 1) + j];
                fma_block<R>(acc, wa, wb, taps + c + k);
            }
            __syncthreads();
        }

        // lane tid's outputs -> LDS row tid (R + 1 floats, conflict-free), then
        // output i = tid + j*NT of the tile leaves from row i / R
#pragma unroll
        for (int r = 0; r < R; ++r) sh_y[tid * (R + 1) + r] = (float)acc[r];
        __syncthreads();
        const int64_t rem = p.end - n0; // outputs left in the range, > 0
        float *__restrict__ yt = y + (n0 - p.y_lo) + tid;
        // output i = tid + j NT is row i / R = tid / R + j NT / R, column tid % R
        const float *__restrict__ ys = sh_y + (tid / R) * (R + 1) + tid % R;
        // no select of min(rem, BO): hipcc (ROCm 7.2) compiled that one into an
        // s_cselect on a stale SCC, so a range's last, partial tile stored all
        // BO outputs (into the next channel)
        if (rem >= BO) {
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const float v = ys[j * (NT / R) * (R + 1)];
                yt[j * NT] = v;
                m = fmaxf(m, fabsf(v));
            }
        } else {
            const int cnt = (int)rem;
#pragma unroll
            for (int j = 0; j < R; ++j) {
                if ((int)tid + j * NT < cnt) {
                    const float v = ys[j * (NT / R) * (R + 1)];
                    yt[j * NT] = v;
                    m = fmaxf(m, fabsf(v));
                }
            }
        }
        __syncthreads(); // the next tile's staging overwrites sh_y
    }

    if (p.peak) {
        const int tid = threadIdx.x;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) m = fmaxf(m, __shfl_xor(m, off, 64));
        if ((tid & 63) == 0) pk_lds[tid >> 6] = m;
        __syncthreads();
        if (tid == 0) {
            float pk = pk_lds[0];
#pragma unroll
            for (int w = 1; w < NT / 64; ++w) pk = fmaxf(pk, pk_lds[w]);
            atomicMax(p.peak + ch * p.peak_stride, __float_as_uint(pk));
        }
    }
}

// LDS bytes a launch of fir_direct_f64_kernel<R, NT, TC> needs.
template <int R, int NT, int TC>
constexpr size_t direct_lds_bytes() {
    return sizeof(double) * ((size_t)(NT * R + TC) / R * (R + 1) + (R + 1));
}

} // namespace lcfir
